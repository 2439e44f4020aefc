"""CPU oracle for the wideband portrait-fit hot path (TEST INFRASTRUCTURE ONLY).

This package is a NumPy/SciPy restatement of the reference PulsePortraiture
algorithm for the per-sub-integration portrait fit.  It
is the CHECKER, never the product: only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` may import it.  The shipped path
(``pulseportraiture_amd``) never imports, calls or falls back to it.

Parity pinning: every function is checked against golden vectors produced by
running the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``,
``tests/test_oracle_golden.py``).

The Gaussian-template generator (gen_gaussian_portrait / gaussian_profile,
pplib.py:801-963) is restated here too, as the checker of the device
template kernel; it reproduces the reference's outputs bit for bit
(tests/golden/make_golden_gauss.py -> gauss.npz).

Third-party arithmetic restated / reused (as the reference uses it):
NumPy 2.2.6 ``numpy.fft`` (pocketfft), SciPy 1.15.3 ``optimize.minimize``
(trust-ncg, TNC) and ``optimize.brute`` + ``fmin``.
"""
from .ppfit_oracle import *  # noqa: F401,F403

"""Host (NumPy-only) synthetic sub-integrations for the full-shape golden
vectors (TEST INFRASTRUCTURE).

The full-shape fixtures (512 x 2048 fits, the example.py archive set, the
C4 ppalign set) would be tens of MB of float32 noise.  Instead the golden
generators (make_golden_full.py) build their inputs with this module from a
few stored parameters, hand them to the REFERENCE, and store only the
reference's outputs plus a SHA-256 of every input array; the tests rebuild
the same inputs with this module and check the hash before comparing (the
GPU box runs the same image, hence the same NumPy/pocketfft).

Mirrors make_fake_pulsar (pplib.py:3302-3499) minus PSRCHIVE: the template
is the reference's Gaussian portrait (oracle.gen_gaussian_portrait, which
reproduces pplib.gen_gaussian_portrait bit for bit, tests/golden/gauss.npz),
rounded to float32; each sub-integration is the template rotated by
(-phi, -DM[, -GM]) at nu0 (rfft -> phasor -> irfft, pplib.py:2427-2515),
optionally scattered (pplib.py:4212-4260, 3471-3477) and scintillated
(add_scintillation, pplib.py:1190-1218, with the example's nsin = 3,
amax = 1, wmax = 5 drawn from this module's own generator), plus white
noise, rounded to float32 as PSRCHIVE stores amplitudes.
"""
import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GMODEL = os.path.join(HERE, "example.gmodel")
P0 = 1.0 / 345.67890123456789          # examples/example.par F0
DM0 = 34.56789                          # examples/example.par DM
DCONST = 0.000241 ** -1                 # pplib.py:64-67


def read_gmodel(path=GMODEL):
    """(code, nu_ref, params [2 + 6 ngauss], alpha) of a .gmodel file, parsed
    as pplib.read_model does (pplib.py:2971-3057)."""
    code, nu_ref, dc, tau, alpha, comps = None, 0.0, 0.0, 0.0, 0.0, []
    for line in open(path):
        info = line.split()
        if not info:
            continue
        key = info[0]
        if key == "CODE":
            code = info[1]
        elif key == "FREQ":
            nu_ref = float(info[1])
        elif key == "DC":
            dc = float(info[1])
        elif key == "TAU":
            tau = float(info[1])
        elif key == "ALPHA":
            alpha = float(info[1])
        elif key[:4] == "COMP":
            comps.append([float(v) for v in info[1::2]])
    params = np.zeros(2 + 6 * len(comps))
    params[0], params[1] = dc, tau
    for i, c in enumerate(comps):
        params[2 + 6 * i:8 + 6 * i] = c
    return code, nu_ref, params, alpha


def write_gmodel(path, code, nu_ref, params, alpha, name="PSR_TEST"):
    """A .gmodel file in the layout of pplib.write_model (pplib.py:2931-2968)."""
    lines = ["MODEL   %s" % name, "CODE    %s" % code,
             "FREQ    %.5f" % nu_ref, "DC     % .8f 0" % params[0],
             "TAU    % .8f 0" % params[1], "ALPHA  % .3f      0" % alpha]
    for i in range((len(params) - 2) // 6):
        p = params[2 + 6 * i:8 + 6 * i]
        lines.append("COMP%02d  " % (i + 1) +
                     "  ".join("% .8f 0" % v for v in p))
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def channel_freqs(nchan, lo=1100.0, bw=800.0):
    cw = bw / nchan
    return np.linspace(lo + cw / 2, lo + bw - cw / 2, nchan)


def f32(x):
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def template(nchan, nbin, lo=1100.0, bw=800.0, gmodel=None):
    """(model [nchan, nbin] float32-rounded float64, freqs)."""
    import oracle as O
    code, nu_ref, params, alpha = read_gmodel(gmodel or GMODEL)
    freqs = channel_freqs(nchan, lo, bw)
    model = O.gen_gaussian_portrait(code, params, alpha,
                                    O.get_bin_centers(nbin), freqs, nu_ref)
    return f32(model), freqs


def rotate(port, phases):
    """rfft -> x exp(2 pi i k phase_row) -> irfft."""
    F = np.fft.rfft(port, axis=-1)
    k = np.arange(F.shape[-1])
    F = F * np.exp(2.0j * np.pi * np.outer(np.ravel(phases), k))
    return np.fft.irfft(F, n=port.shape[-1], axis=-1)


def scintillation(rng, nchan, nsin=3, amax=1.0, wmax=5.0):
    """add_scintillation's random pattern (pplib.py:1190-1218)."""
    pattern = np.zeros(nchan)
    for _ in range(nsin):
        a, w, p = rng.uniform(0, amax), rng.chisquare(wmax), rng.uniform(0, 1)
        pattern += a * np.sin(np.linspace(0, w * np.pi, nchan) + p * np.pi) ** 2
    return pattern


def subint(seed, model, freqs, phi, DM, P, nu0=1500.0, noise=1.5, GM=0.0,
           tau=0.0, alpha=-4.0, nu_tau=1500.0, scint=False):
    """One float32-rounded sub-integration [nchan, nbin] (see module doc)."""
    rng = np.random.default_rng(seed)
    nbin = model.shape[-1]
    ph = (-phi - DCONST * DM * (freqs ** -2 - nu0 ** -2) / P -
          DCONST ** 2 * GM * (freqs ** -4 - nu0 ** -4) / P)
    port = rotate(model, ph)
    if tau:
        taus = tau * (freqs / nu_tau) ** alpha
        k = np.arange(nbin // 2 + 1)
        B = 1.0 / (1.0 + 2j * np.pi * np.outer(taus, k))
        port = np.fft.irfft(B * np.fft.rfft(port, axis=-1), n=nbin, axis=-1)
    if scint:
        port = port * scintillation(rng, len(freqs))[:, None]
    port = port + rng.normal(0.0, noise, port.shape)
    return f32(port)


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()

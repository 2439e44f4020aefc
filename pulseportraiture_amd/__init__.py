"""pulseportraiture_amd -- MI355X-native wideband FFTFIT engine.

A drop-in accelerator for PulsePortraiture's per-sub-integration portrait fit
(SURVEY.md section 8): ``pplib`` / ``pptoaslib`` / ``pptoas`` mirror the
reference API; compute runs in hand-written gfx950 HIP kernels behind the C
ABI of ``lib/libppfit.so`` (include/ppfit.h), bound with ctypes in
``_lib``.  ``engine`` is the batched device API, ``dist`` the multi-GPU
sharding over RCCL, ``synth`` the synthetic-data generator.
"""
__version__ = "0.1.0"

from . import _lib  # noqa: F401

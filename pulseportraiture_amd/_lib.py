"""ctypes binding of libppfit.so (the C ABI in include/ppfit.h).

The shipped path has no CPU fallback: if the library cannot be loaded, or no
HIP device is visible when a compute entry point is first used, a
RuntimeError is raised.  Loading the library and querying its exports works
without a GPU (used by the CPU test-suite).
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PPFIT_LIB", os.path.join(_HERE, "lib", "libppfit.so"))

PPF_OK, PPF_EINVAL, PPF_EHIP, PPF_ENOMEM, PPF_EUNSUP = 0, -1, -2, -3, -4
PPF_F32, PPF_F64 = 0, 1
PPF_MODE_FULL, PPF_MODE_LEGACY2 = 0, 1
ST_SUCCESS, ST_MAXITER, ST_CONVERGED, ST_LINALG = 0, 1, 2, 3
ST_NO_ROOT, ST_SINGULAR, ST_NONFINITE, ST_NOFIT = 0x100, 0x200, 0x400, 0x800
ST_NOSPACE = 0x1000
OPT_NO_HCUT = 1           # ppf_fit_desc.options
OPT_NO_X = 2
OPT_SCIPY_TR = 4          # scattering fits follow scipy's trust-ncg path
OPT_MOM_X = 8             # phase/DM/GM fits: moments from the stored cross spectrum
OPT_FUSED_MOM = 16        # ... from the fused k_xmom_g pass (no X)
OPT_SPIN_WAIT = 32        # poll the iteration loop's read-backs (ppalign)
ABI_VERSION = 6

# ppf_result: 32 doubles (include/ppfit.h)
RESULT_FIELDS = (
    [("params", 5), ("param_errs", 5), ("nu_out", 3), ("nu_fit", 3)] +
    [(n, 1) for n in ("chi2", "red_chi2", "snr", "fun", "Sd", "phi_guess",
                      "nfeval", "status", "niter", "dof", "nchanx",
                      "x_fit_phi", "x_fit_tau", "npass")] +
    [("reserved", 2)])
RESULT_DOUBLES = sum(n for _, n in RESULT_FIELDS)
assert RESULT_DOUBLES == 32


def result_slices():
    out, o = {}, 0
    for name, n in RESULT_FIELDS:
        out[name] = slice(o, o + n) if n > 1 else o
        o += n
    return out


RESULT_INDEX = result_slices()

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32


class FitDesc(ctypes.Structure):
    """Mirror of ppf_fit_desc (include/ppfit.h)."""
    _fields_ = [
        ("nsub", _i32), ("nchan", _i32), ("nbin", _i32), ("data_dtype", _i32),
        ("data", _vp), ("model", _vp), ("nmodel", _i32), ("model_index", _vp),
        ("chan_mask", _vp), ("freqs", _vp), ("P", _vp), ("errs", _vp),
        ("init", _vp), ("fit_flags", _vp), ("nu_fits", _vp),
        ("nu_outs", _vp), ("log10_tau", _i32), ("option", _i32),
        ("is_toa", _i32), ("mode", _i32), ("max_iter", _i32), ("guess", _i32),
        ("guess_weights", _vp), ("guess_DM", _vp), ("guess_tau", _vp),
        ("guess_Ns", _i32),
        ("results", _vp), ("scales", _vp), ("scale_errs", _vp),
        ("channel_snrs", _vp), ("covariance", _vp), ("workspace", _vp),
        ("workspace_bytes", ctypes.c_size_t),
        ("x_subints", _i32), ("options", _i32), ("guess_ref", _i32),  # ABI 2
        ("bounds", _vp),                                               # ABI 3
    ]


# exported symbol -> (restype, argtypes)
SIGNATURES = {
    "ppf_abi_version": (ctypes.c_int, []),
    "ppf_sizeof_fit_desc": (ctypes.c_size_t, []),
    "ppf_sizeof_result": (ctypes.c_size_t, []),
    "ppf_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "ppf_destroy": (None, [_vp]),
    "ppf_last_error": (ctypes.c_char_p, [_vp]),
    "ppf_set_profiling": (ctypes.c_int, [_vp, ctypes.c_int]),
    "ppf_last_stage_ms": (ctypes.c_int, [_vp, _vp]),
    "ppf_stage_ms_history": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "ppf_kernel_ms_history": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "ppf_pass_ms_history": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "ppf_fit_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(FitDesc)]),
    "ppf_fit_batch": (ctypes.c_int, [_vp, ctypes.POINTER(FitDesc), _vp]),
    "ppf_fit2_batch": (ctypes.c_int, [_vp, ctypes.POINTER(FitDesc), _vp]),
    "ppf_rotate_batch": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _i32, _vp,
                                        _vp, _vp, _vp]),
    "ppf_rotate_batch_ref": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _i32,
                                            _vp, _vp, _vp, _vp]),
    "ppf_noise_batch": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _i32, _vp,
                                       _i32, _vp, _vp]),
    "ppf_rotate_long_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64,
                                                          ctypes.c_int64,
                                                          _i32]),
    "ppf_rotate_long": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int64,
                                       _i32, _vp, _vp, _vp, _i32, _vp,
                                       ctypes.c_size_t, _vp]),
    "ppf_noise_long_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64,
                                                         ctypes.c_int64]),
    "ppf_noise_long": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int64,
                                      _i32, _vp, _i32, _vp, _vp,
                                      ctypes.c_size_t, _vp]),
    "ppf_resid_chi2_batch": (ctypes.c_int, [_vp, ctypes.c_int64, _i32, _i32,
                                            _vp, _vp, _vp, _vp, _vp, _vp,
                                            ctypes.c_double, _vp, _vp]),
    "ppf_align_phases": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _vp, _vp,
                                        _vp, _vp, _vp, _vp, _vp]),
    "ppf_align_workspace_bytes": (ctypes.c_size_t, [_i32, _i32, _i32]),
    "ppf_align_accum": (ctypes.c_int, [_vp, _i32, _i32, _i32, _i32, _vp, _vp,
                                       _vp, _vp, _vp, _vp, ctypes.c_size_t,
                                       _vp]),
    "ppf_phase_shift_batch": (ctypes.c_int, [_vp, _i32, _i32, _i32, _vp, _vp,
                                             _vp, _vp, _i32, ctypes.c_double,
                                             ctypes.c_double, _vp, _vp]),
    "ppf_scales_batch": (ctypes.c_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp,
                                        _vp, _vp, _vp, _vp, _vp, _i32, _vp,
                                        _vp]),
    "ppf_gauss_portrait_batch": (ctypes.c_int, [_vp, _i32, _i32, _i32, _i32,
                                                ctypes.c_char_p, _vp, _vp, _vp,
                                                _vp, _vp, _vp]),
    "ppf_spline_portrait_batch": (ctypes.c_int, [_vp, _i32, _i32, _i32, _i32,
                                                 _i32, _i32, _i32, _vp, _vp,
                                                 _vp, _vp, _vp, _vp, _vp]),
    "ppf_synth_batch": (ctypes.c_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp,
                                       _vp, _vp, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_uint64,
                                       ctypes.c_int64, _i32, _vp, _vp]),
    "ppf_unpack_workspace_bytes": (ctypes.c_size_t, [_i32, _i32, _i32]),
    "ppf_unpack_psrfits_batch": (ctypes.c_int, [_vp, _i32, _i32, _i32, _i32,
                                                _i32, _vp, ctypes.c_int64,
                                                _vp, _vp, _vp, _i32, _i32,
                                                _vp, _vp, _vp, _vp, _vp,
                                                ctypes.c_size_t, _vp]),
    "ppf_copy_from_pinned": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64,
                                            _vp]),
    "ppf_read_rows": (ctypes.c_int, [_i32, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_int64, _vp,
                                     ctypes.c_int64, _i32]),
    "ppf_solver_ms_history": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "ppf_host_copy": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _i32]),
    "ppf_poly_real_roots_host": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "ppf_tr_subproblem_host": (ctypes.c_int, [_vp, _vp, ctypes.c_int,
                                              ctypes.c_double, _vp]),
}

_lib = None
_lock = threading.Lock()
_ctx = {}


def load():
    """Load libppfit.so (no GPU needed).  Raises RuntimeError if absent."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    "libppfit.so not found at %s: build it with `make` or "
                    "__graft_entry__.build(); there is no CPU fallback" %
                    LIB_PATH)
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.ppf_abi_version() != ABI_VERSION or \
                    lib.ppf_sizeof_fit_desc() != ctypes.sizeof(FitDesc) or \
                    lib.ppf_sizeof_result() != 8 * RESULT_DOUBLES:
                raise RuntimeError("libppfit ABI mismatch (rebuild with make)")
            _lib = lib
    return _lib


def context(device):
    """The ppf_ctx of a device (created lazily)."""
    lib = load()
    with _lock:
        if device not in _ctx:
            p = _vp()
            rc = lib.ppf_create(int(device), ctypes.byref(p))
            if rc != PPF_OK:
                raise RuntimeError(
                    "ppf_create(device=%d) failed (%d): no usable HIP device; "
                    "the wideband fit runs only on the GPU" % (device, rc))
            _ctx[device] = p
    return _ctx[device]


def check(rc, ctx):
    if rc != PPF_OK:
        msg = load().ppf_last_error(ctx)
        msg = msg.decode() if msg else ""
        exc = {PPF_EINVAL: ValueError, PPF_EUNSUP: NotImplementedError,
               PPF_ENOMEM: MemoryError}.get(rc, RuntimeError)
        raise exc("libppfit error %d: %s" % (rc, msg))


def poly_real_roots(coeffs):
    """Host (CPU) helper: real roots with np.roots semantics."""
    lib = load()
    c = np.ascontiguousarray(coeffs, dtype=np.float64)
    out = np.zeros(16)
    n = lib.ppf_poly_real_roots_host(c.ctypes.data, len(c) - 1,
                                     out.ctypes.data)
    if n < 0:
        raise RuntimeError("root finder failed")
    return out[:n]


def tr_subproblem(H, g, R):
    """Host (CPU) helper: the Newton solver's exact trust-region step
    (p, hits_boundary) for a symmetric H [n, n], g [n], radius R."""
    lib = load()
    H = np.ascontiguousarray(H, dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.float64)
    n = g.size
    p = np.zeros(n)
    rc = lib.ppf_tr_subproblem_host(H.ctypes.data, g.ctypes.data, n,
                                    float(R), p.ctypes.data)
    if rc < 0:
        raise ValueError("bad trust-region subproblem arguments")
    return p, bool(rc)

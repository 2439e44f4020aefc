"""Drop-in mirror of the parts of PulsePortraiture's ``pplib`` on the hot path.

Compute-bearing routines (FFT rotation, power-spectrum noise, 1-D FFTFIT and
the legacy 2-parameter portrait fit) run on the GPU through libppfit; the
rest is host bookkeeping (constants, reference-frequency algebra, Gaussian
model generation from .gmodel files, TOA text output) with the reference's
signatures.  There is no CPU fallback for the compute routines.

Reference: /root/reference/pplib.py (file:line cited per function).
"""
import os
import sys
import time

import pickle

import math

import numpy as np

from . import _lib, engine

# ---------------------------------------------------------------- settings --
Dconst_exact = 4.148808e3          # pplib.py:61
Dconst_trad = 0.000241 ** -1       # pplib.py:64
Dconst = Dconst_trad               # pplib.py:67
scattering_alpha = -4.0            # pplib.py:70
use_get_noise = True               # pplib.py:74
default_noise_method = "PS"        # pplib.py:78
F0_fact = 0                        # pplib.py:82
wid_max = 0.25                     # pplib.py:86
default_model = "000"              # pplib.py:95
binshift = 1.0                     # pplib.py:99

# scipy.optimize.fmin_tnc return codes (pplib.py:127-135)
RCSTRINGS = {"-1": "INFEASIBLE: Infeasible (low > up).",
             "0": "LOCALMINIMUM: Local minima reach (|pg| ~= 0).",
             "1": "FCONVERGED: Converged (|f_n-f_(n-1)| ~= 0.)",
             "2": "XCONVERGED: Converged (|x_n-x_(n-1)| ~= 0.)",
             "3": "MAXFUN: Max. number of function evaluations reach.",
             "4": "LSFAIL: Linear search failed.",
             "5": "CONSTANT: All lower bounds are equal to the upper bounds.",
             "6": "NOPROGRESS: Unable to progress.",
             "7": "USERABORT: User requested end of minimization."}


class DataBunch(dict):
    """dict with attribute access (pplib.py:142-152)."""

    def __init__(self, **kwds):
        dict.__init__(self, kwds)
        self.__dict__ = self


class MJD(object):
    """A PSRCHIVE-free MJD (psrchive.MJD's interface as get_TOAs and
    write_TOAs use it): integer day + fractional day, so a TOA keeps
    sub-nanosecond resolution.  MJD(days) or MJD(intday, fracday)."""

    def __init__(self, intday=0.0, fracday=None):
        # math.floor: the same integers as np.floor, without the NumPy
        # scalar round trip (GetTOAs makes two of these per TOA)
        if fracday is None:
            d = float(intday)
            i = math.floor(d)
            intday, fracday = i, d - i
        i, f = int(intday), float(fracday)
        k = math.floor(f)
        self._i, self._f = i + k, f - k

    @classmethod
    def _make(cls, i, f):
        """An MJD from an integer day and a fraction already in [0, 1)."""
        m = cls.__new__(cls)
        m._i, m._f = i, f
        return m

    def __add__(self, other):
        if isinstance(other, MJD):
            return MJD(self._i + other._i, self._f + other._f)
        return MJD(self._i, self._f + float(other) / 86400.0)   # seconds

    def intday(self):
        return self._i

    def fracday(self):
        return self._f

    def in_days(self):
        return self._i + self._f

    def __repr__(self):
        return "MJD(%d, %.15f)" % (self._i, self._f)


# ------------------------------------------------------------ host helpers --
def get_bin_centers(nbin, lo=0.0, hi=1.0):
    """pplib.py:694-707."""
    lo, hi = np.double(lo), np.double(hi)
    diff = hi - lo
    return np.double(np.linspace(lo + diff / (nbin * 2),
                                 hi - diff / (nbin * 2), nbin))


def weighted_mean(data, errs=1.0):
    """pplib.py:721-735."""
    if hasattr(errs, "is_integer"):
        errs = np.ones(len(data))
    iis = np.where(errs > 0.0)[0]
    w = errs[iis] ** -2.0
    return (data[iis] * w).sum() / w.sum(), w.sum() ** -0.5


def DM_delay(DM, freq, freq_ref=np.inf, P=None):
    """pplib.py:2672-2685."""
    delay = Dconst * DM * ((freq ** -2.0) - (freq_ref ** -2.0))
    return delay / P if P else delay


def phase_transform(phi, DM, nu_ref1=np.inf, nu_ref2=np.inf, P=None,
                    mod=False):
    """pplib.py:2688-2712."""
    if P is None:
        P, mod = 1.0, False
    phi_prime = phi + (Dconst * DM * P ** -1 *
                       (nu_ref2 ** -2.0 - nu_ref1 ** -2.0))
    if mod:
        phi_prime = np.where(abs(phi_prime) >= 0.5, phi_prime % 1, phi_prime)
        phi_prime = np.where(phi_prime >= 0.5, phi_prime - 1.0, phi_prime)
        if not phi_prime.shape:
            phi_prime = np.float64(phi_prime)
    return phi_prime


def guess_fit_freq(freqs, SNRs=None):
    """pplib.py:2715-2729: SNR * nu**-2 weighted centre frequency."""
    nu0 = (freqs.min() + freqs.max()) * 0.5
    if SNRs is None:
        SNRs = np.ones(len(freqs))
    w = SNRs * freqs ** -2
    return nu0 + np.sum((freqs - nu0) * w) / np.sum(w)


def scattering_times(tau, alpha, freqs, nu_tau):
    """pplib.py:4212-4216."""
    return tau * (freqs / nu_tau) ** alpha


def scattering_profile_FT(tau, nbin, binshift=binshift):
    """pplib.py:4219-4242 (host; model generation / flux only)."""
    nharm = nbin // 2 + 1
    if tau == 0.0:
        return np.ones(nharm)
    return (1.0 + 2 * np.pi * 1.0j * np.arange(nharm) * tau) ** -1


def scattering_portrait_FT(taus, nbin, binshift=binshift):
    """pplib.py:4245-4260 (host; complex128 on every NumPy)."""
    taus = np.asarray(taus, dtype=float)
    nharm = nbin // 2 + 1
    if not np.any(taus):
        return np.ones([len(taus), nharm])
    k = np.arange(nharm)
    out = 1.0 / (1.0 + 2j * np.pi * np.outer(taus, k))
    out[taus == 0.0] = 1.0
    return out


# ------------------------------------------ Gaussian models (device) --------
def gaussian_profile(nbin, loc, wid, norm=False, abs_wid=False, zeroout=True):
    """pplib.py:801-856 (unit peak, zeroout): one row of k_gauss_port with
    the linear evolution code at nu = nu_ref, which passes loc, wid and the
    unit amplitude through exactly."""
    if norm or not zeroout:
        raise NotImplementedError("gaussian_profile(norm=True / zeroout="
                                  "False) is outside the accelerated path")
    if abs_wid:
        wid = abs(wid)
    params = [0.0, 0.0, loc, 0.0, wid, 0.0, 1.0, 0.0]
    return gen_gaussian_portrait("111", params, 0.0, np.zeros(nbin), [1.0],
                                 1.0)[0]


def gen_gaussian_portrait(model_code, params, scattering_index, phases, freqs,
                          nu_ref, join_ichans=[], P=None):
    """pplib.py:886-963 for join_ichans == [], built on the device by
    ppf_gauss_portrait_batch (k_gauss_port)."""
    if len(join_ichans):
        raise NotImplementedError("join_ichans (ppgauss only) is out of scope")
    from . import engine
    params = np.asarray(params, dtype=float)
    out = engine.gauss_portraits(model_code, params[None, :],
                                 [scattering_index],
                                 np.asarray(freqs, dtype=float)[None, :],
                                 [nu_ref], len(phases))
    out = out[0].cpu().numpy()
    if len(phases) % 2 and params[1] != 0.0:
        # the reference's scattering irfft takes no length (pplib.py:957):
        # nbin - 1 bins at odd nbin
        out = out[:, :-1]
    return out


def read_model(modelfile, phases=None, freqs=None, P=None, quiet=False):
    """pplib.py:2971-3057: parse a .gmodel file; build the portrait if
    phases/freqs are given."""
    read_only = phases is None and freqs is None
    comps, fit_comps = [], []
    name = code = nu_ref = dc = tau = alpha = None
    fit_dc = fit_tau = fit_alpha = None
    with open(modelfile) as fh:      # a pickled spline model: UnicodeDecodeError
        lines = fh.readlines()
    for line in lines:
        info = line.split()
        if not info:
            continue
        key = info[0]
        try:
            if key == "MODEL":
                name = info[1]
            elif key == "CODE":
                code = info[1]
            elif key == "FREQ":
                nu_ref = np.float64(info[1])
            elif key == "DC":
                dc, fit_dc = np.float64(info[1]), int(info[2])
            elif key == "TAU":
                tau, fit_tau = np.float64(info[1]), int(info[2])
            elif key == "ALPHA":
                alpha, fit_alpha = np.float64(info[1]), int(info[2])
            elif key[:4] == "COMP":
                comps.append([np.float64(v) for v in info[1::2]])
                fit_comps.append([int(v) for v in info[2::2]])
        except IndexError:
            pass
    # a missing line leaves the reference's local unbound (pplib.py:3022-3026)
    for var, val in (("dc", dc), ("tau", tau), ("fit_dc", fit_dc),
                     ("fit_tau", fit_tau)):
        if val is None:
            raise UnboundLocalError("local variable '%s' referenced before "
                                    "assignment" % var)
    ngauss = len(comps)
    params = np.zeros(ngauss * 6 + 2)
    fit_flags = np.zeros(len(params))
    params[0], params[1] = dc, tau
    fit_flags[0], fit_flags[1] = fit_dc, fit_tau
    for ig in range(ngauss):
        params[2 + ig * 6:8 + ig * 6] = comps[ig]
        fit_flags[2 + ig * 6:8 + ig * 6] = fit_comps[ig]
    for var, val in (("modelname", name), ("model_code", code),
                     ("nu_ref", nu_ref), ("alpha", alpha)) + \
            ((("fit_alpha", fit_alpha),) if read_only else ()):
        if val is None:
            raise UnboundLocalError("local variable '%s' referenced before "
                                    "assignment" % var)
    if read_only:
        return (name, code, nu_ref, ngauss, params, fit_flags, alpha,
                fit_alpha)
    nbin = len(phases)
    if params[1] != 0:
        if P is None:
            print("Need period P for non-zero scattering value TAU.")
            return 0
        params[1] *= nbin / P
    model = gen_gaussian_portrait(code, params, alpha, phases, freqs, nu_ref)
    if not quiet:
        print("Model Name: %s" % name)
    return name, ngauss, model


def gen_spline_portrait(mean_prof, freqs, eigvec, tck, nbin=None):
    """pplib.py:966-990 on the device (ppf_spline_portrait_batch: splev of
    the B-spline curve per channel, eigenvector expansion, mean profile and,
    for nbin != len(mean_prof), scipy.signal.resample + the half-bin
    rotate_portrait)."""
    from . import engine
    out = engine.spline_portraits(mean_prof, eigvec, tck,
                                  np.asarray(freqs, dtype=float)[None, :],
                                  nbin)
    return out[0].cpu().numpy()


class _SplineUnpickler(pickle.Unpickler):
    """The reference reads spline models with a plain pickle.load
    (pplib.py:3083-3088), which runs whatever a crafted file names.  The
    6-tuple of strings, numpy arrays and splprep's tck needs only numpy's
    array reconstruction and a few builtins; any other global is refused."""
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"),
        ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"),
        ("numpy", "ndarray"), ("numpy", "dtype"),
        ("builtins", "list"), ("builtins", "tuple"), ("builtins", "int"),
        ("builtins", "float"), ("builtins", "str"), ("builtins", "bytes"),
        ("__builtin__", "list"), ("__builtin__", "tuple"),
        ("_codecs", "encode"), ("copy_reg", "_reconstructor"),
        ("copyreg", "_reconstructor"), ("__builtin__", "object"),
        ("builtins", "object"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError("spline model file names %s.%s, which "
                                     "a spline model never holds" %
                                     (module, name))


def read_spline_model(modelfile, freqs=None, nbin=None, quiet=False):
    """pplib.py:3060-3096: a make_spline_model(...) file -- the pickled
    (model name, source, datafile, mean profile, eigenvectors, tck) -- read
    as the reference reads it; with freqs, the portrait built on the device
    by gen_spline_portrait."""
    if not quiet:
        print("Reading model from %s..." % modelfile)
    try:
        with open(modelfile, "rb") as fh:
            modelname, source, datafile, mean_prof, eigvec, tck = \
                _SplineUnpickler(fh).load()
    except UnicodeDecodeError:       # python2 to python3 pickling issues
        with open(modelfile, "rb") as fh:
            modelname, source, datafile, mean_prof, eigvec, tck = \
                _SplineUnpickler(fh, encoding="bytes").load()
    if freqs is None:
        return (modelname, source, datafile, mean_prof, eigvec, tck)
    return (modelname, gen_spline_portrait(mean_prof, freqs, eigvec, tck,
                                           nbin))


# --------------------------------------------------------- device routines --
def get_noise(data, method=default_noise_method, **kwargs):
    """pplib.py:2290-2309."""
    if method == "PS":
        return get_noise_PS(data, **kwargs)
    if method == "fit":
        raise NotImplementedError("get_noise_fit is outside the accelerated "
                                  "path (SURVEY.md section 2, row 6)")
    print("Unknown get_noise method.")
    return 0


def get_noise_PS(data, frac=4, chans=False):
    """pplib.py:2312-2338 on the GPU (ppf_noise_batch)."""
    data = np.asarray(data)
    if chans:
        return engine.noise_rows(np.atleast_2d(data), frac).cpu().numpy()
    row = data.ravel()
    if not engine.noise_len_supported(row.size):
        # the flattened portrait (nchan nbin samples; pplib.py:2334-2338) is
        # longer than the LDS transforms of ppf_noise_batch (even <= 8192,
        # odd <= 4095 points): the long transforms of ppf_noise_long
        return engine.noise_long(row, frac)
    return float(engine.noise_rows(row[None, :], frac).cpu().numpy()[0])


def get_red_chi2(data, model, errs=None, dof=None):
    """pplib.py:754-779 (host: a single residual sum; the batched per-channel
    form used by get_channels_to_zap runs on the GPU, ppf_resid_chi2_batch)."""
    data = np.asarray(data, dtype=np.float64)
    resids = data - model
    if errs is None:
        if len(data.shape) == 1:
            errs = get_noise(data)
        elif len(data.shape) == 2:
            errs = get_noise(data, chans=True)
        else:
            print("Can only handle 1- or 2-D input.")
    if dof is None:
        dof = sum(data.shape)
    if len(data.shape) == 1:
        return np.sum((resids / errs) ** 2.0) / dof
    return np.array([(resids[ii] / errs[ii]) ** 2.0 for ii in
                     range(len(resids))]).sum() / dof


def rotate_data(data, phase=0.0, DM=0.0, Ps=None, freqs=None, nu_ref=np.inf):
    """pplib.py:2427-2515: per-row phases on the host, FFT rotation on the
    GPU (ppf_rotate_batch)."""
    data = np.asarray(data)
    shape, ndim = data.shape, data.ndim
    nbin = shape[-1]
    if DM == 0.0:
        nrows = int(np.prod(shape[:-1])) if ndim > 1 else 1
        out = engine.rotate_rows(data.reshape(nrows, nbin),
                                 np.full(nrows, float(phase)), ref_len=True)
        return engine.dev_to_host(out).reshape(shape[:-1] + (out.shape[-1],))
    d4 = data                       # only read: the result is a new array
    while d4.ndim != 4:
        d4 = d4[None]
    nsub, npol, nchan = d4.shape[:3]
    D = Dconst * DM / (np.ones(nsub) * Ps)
    if len(D) != nsub:
        print("Wrong shape for array of periods.")
        return 0
    try:
        float(nu_ref)
    except TypeError:
        print("Only one nu_ref permitted.")
        return 0
    if not hasattr(freqs, "ndim"):
        freqs = np.ones(nchan) * freqs
    if freqs.ndim == 0:
        freqs = np.ones(nchan) * float(freqs)
    if freqs.ndim == 1:
        if nchan != len(freqs):
            print("Wrong number of frequencies.")
            return 0
        fterm = np.tile(freqs, nsub).reshape(nsub, nchan) ** -2.0 - \
            nu_ref ** -2.0
    else:
        fterm = freqs ** -2.0 - nu_ref ** -2.0
    if fterm.shape[1] != nchan or fterm.shape[0] != nsub:
        print("Wrong shape for frequency array.")
        return 0
    if ndim not in (1, 2, 4):
        print("Wrong number of dimensions.")
        return 0
    ph = phase + D[:, None] * fterm
    ph = np.broadcast_to(ph[:, None, :], (nsub, npol, nchan))
    out = engine.rotate_rows(d4.reshape(-1, nbin), ph.reshape(-1),
                             ref_len=True)
    out = engine.dev_to_host(out).reshape(d4.shape[:3] + (out.shape[-1],))
    if ndim == 1:
        return out[0, 0, 0]
    if ndim == 2:
        return out[0, 0]
    return out


def rotate_portrait(port, phase=0.0, DM=None, P=None, freqs=None,
                    nu_ref=np.inf):
    """pplib.py:2518-2550."""
    port = np.asarray(port)
    nchan = len(port)
    if DM is None and freqs is None:
        ph = np.full(nchan, float(phase))
    else:
        D = Dconst * DM / P
        ph = phase + D * (np.asarray(freqs, dtype=float) ** -2.0 -
                          nu_ref ** -2.0)
    return engine.rotate_rows(port, ph, ref_len=True).cpu().numpy()


def rotate_profile(profile, phase=0.0):
    """pplib.py:2641-2652."""
    profile = np.asarray(profile)
    return engine.rotate_rows(profile[None, :], [phase],
                              ref_len=True).cpu().numpy()[0]


def fit_phase_shift(data, model, noise=None, bounds=[-0.5, 0.5], Ns=100):
    """pplib.py:2136-2182 on the GPU: brute grid of Ns points + scipy-fmin
    replica (Nelder-Mead) polish, then the reference's error formulas."""
    t0 = time.time()
    out = engine.phase_shift_batch(
        np.asarray(data)[None, :], np.asarray(model, dtype=float)[None, :],
        None if noise is None else np.array([noise], dtype=float), Ns,
        bounds).cpu().numpy()[0]
    return DataBunch(phase=out[0], phase_err=out[1], scale=out[2],
                     scale_err=out[3], snr=out[4], red_chi2=out[5],
                     duration=time.time() - t0)


def fit_portrait(data, model, init_params, P, freqs, nu_fit=None, nu_out=None,
                 errs=None, bounds=[(None, None), (None, None)], id=None,
                 quiet=True):
    """pplib.py:2185-2287: phase + DM FFTFIT on the GPU (ppf_fit2_batch).

    The reference minimises with scipy TNC; the device runs the trust-region
    Newton solver of fit_portrait_full on the same objective
    (pplib.py:1335-1447), which converges to the same stationary point
    (SURVEY.md Appendix A.5).  ``bounds`` on (phase, DM) hold as TNC's
    do: the device trust-region steps are projected onto the box
    (ppf_fit_desc.bounds)."""
    data = np.asarray(data)
    freqs = np.asarray(freqs, dtype=float)
    nchan, nbin = data.shape
    if nu_fit is None:
        nu_fit = freqs.mean()
    init = np.zeros((1, 5))
    init[0, :2] = np.asarray(init_params, dtype=float)[:2]
    t0 = time.time()
    res = engine.fit_batch(
        data[None], np.asarray(model, dtype=float)[None], freqs[None], [P],
        init, [1, 1, 0, 0, 0], nu_fits=np.full((1, 3), nu_fit),
        nu_outs=np.full((1, 3), np.nan if nu_out is None else nu_out),
        errs=None if errs is None else np.asarray(errs, dtype=float)[None],
        mode=_lib.PPF_MODE_LEGACY2, bounds=_box(bounds, 2))
    r = engine.results_numpy(res)
    duration = time.time() - t0
    R, I = r["results"][0], _lib.RESULT_INDEX
    status = int(R[I["status"]])
    _raise_status(status)
    rc = status & 0xff
    if not quiet and rc not in (1, 2, 4):
        sys.stderr.write("Fit failed with return code %d -- %s" %
                         (rc, RCSTRINGS.get(str(rc), "")))
    cov = r["covariance"][0]
    return DataBunch(phase=R[I["params"]][0], phase_err=R[I["param_errs"]][0],
                     DM=R[I["params"]][1], DM_err=R[I["param_errs"]][1],
                     scales=r["scales"][0], scale_errs=r["scale_errs"][0],
                     nu_ref=R[I["nu_out"]][0], covariance=cov[0, 1],
                     chi2=R[I["chi2"]], red_chi2=R[I["red_chi2"]],
                     snr=R[I["snr"]], duration=duration,
                     nfeval=int(R[I["nfeval"]]), return_code=rc)


def _box(bounds, n):
    """[5, 2] device bounds from the first n (lower, upper) pairs of a
    scipy bounds list (None: unbounded); None when nothing is bounded."""
    if bounds is None:
        return None
    b = np.full((5, 2), np.nan)
    for i, lu in enumerate(list(bounds)[:n]):
        if lu is None:
            continue
        for j in (0, 1):
            if lu[j] is not None:
                b[i, j] = float(lu[j])
    return None if np.isnan(b).all() else b


def _raise_status(status):
    """Map device status bits to the exceptions the reference raises."""
    if status & _lib.ST_NO_ROOT:
        raise ValueError("attempt to get argmin of an empty sequence "
                         "(no positive real zero-covariance frequency)")
    if status & _lib.ST_SINGULAR:
        raise np.linalg.LinAlgError("Singular matrix")
    if status & _lib.ST_NOFIT:
        raise ValueError("nothing to fit (no fit flag set or no channel)")
    if status & _lib.ST_NOSPACE:
        # the workspace had fewer cross-spectrum slots than fits that stream
        # it (the host's count disagreed with the device's k_classify): an
        # internal error, never a fit outcome
        raise RuntimeError("internal error: no cross-spectrum slot for a "
                           "scattering fit (PPF_ST_NOSPACE)")


# ------------------------------------------------------------- TOA output --
def filter_TOAs(TOAs, flag, cutoff, criterion=">=", pass_unflagged=False,
                return_culled=False):
    """pplib.py:3502-3548 (the >= / <= criteria used by write_TOAs)."""
    import operator
    ops = {">=": operator.ge, "<=": operator.le, ">": operator.gt,
           "<": operator.lt, "==": operator.eq}
    keep, culled = [], []
    for toa in TOAs:
        if flag in toa.flags:
            (keep if ops[criterion](toa.flags[flag], cutoff) else
             culled).append(toa)
        elif pass_unflagged:
            keep.append(toa)
        else:
            culled.append(toa)
    return (keep, culled) if return_culled else keep


def write_TOAs(TOAs, inf_is_zero=True, SNR_cutoff=0.0, outfile=None,
               append=True):
    """pplib.py:3588-3649: loosely IPTA-formatted TOA lines."""
    toas = TOAs if hasattr(TOAs, "__len__") else [TOAs]
    toas = filter_TOAs(toas, "snr", SNR_cutoff, ">=", pass_unflagged=False)
    of = open(outfile, "a" if append else "w") if outfile is not None \
        else None
    for toa in toas:
        freq = 0.0 if (toa.frequency == np.inf and inf_is_zero) else \
            toa.frequency
        line = "%s %.8f %d" % (toa.archive, freq, toa.MJD.intday()) + \
            ("%.15f   %.3f  %s" % (toa.MJD.fracday(), toa.TOA_error,
                                   toa.telescope_code))[1:]
        if toa.DM is not None:
            line += " -pp_dm %.7f" % toa.DM
        if toa.DM_error is not None:
            line += " -pp_dme %.7f" % toa.DM_error
        for flag, value in list(toa.flags.items()):
            if value is None:
                continue
            if hasattr(value, "lower"):
                line += " -%s %s" % (flag, value)
            elif "int" in str(type(value)):
                line += " -%s %d" % (flag, value)
            elif flag.find("_cov") >= 0:
                line += " -%s %.1e" % (flag, value)
            elif flag.find("phs") >= 0:
                line += " -%s %.8f" % (flag, value)
            elif flag.find("flux") >= 0:
                line += " -%s %.5f" % (flag, value)
            else:
                line += " -%s %.3f" % (flag, value)
        if of is not None:
            of.write(line + "\n")
        else:
            print(line)
    if of is not None:
        of.close()


# ------------------------------------------------------------ archive I/O --
def load_data(filename, **kwargs):
    """pplib.py:2749-2915.  Fold-mode PSRFITS files take the PSRCHIVE-free
    fast path (psrfits.load_data: raw DATA bytes to the device, unpacked,
    baseline-removed and pscrunched there); any other archive format needs
    PSRCHIVE, which is not installed in this image."""
    if file_is_type(filename, "FITS"):
        from . import psrfits
        return psrfits.load_data(filename, **kwargs)
    try:
        import psrchive  # noqa: F401
    except ImportError as exc:
        raise ImportError("load_data needs the PSRCHIVE Python bindings for "
                          "non-PSRFITS archives (archive I/O is host-side "
                          "and out of the accelerated path)") from exc
    raise NotImplementedError("PSRCHIVE-backed load_data is not provided in "
                              "this build; pass a DataBunch with the keys of "
                              "pplib.py:2904-2914")


def file_is_type(filename, filetype="ASCII"):
    """pplib.py:3126-3143 without the `file -L` subprocess: FITS files start
    with 'SIMPLE  =', ASCII metafiles decode as text."""
    with open(filename, "rb") as fh:
        head = fh.read(4096)
    if filetype == "FITS":
        return head.startswith(b"SIMPLE")
    if filetype == "ASCII":
        if b"\x00" in head or head.startswith(b"SIMPLE"):
            return False
        try:
            head.decode("ascii")
            return True
        except UnicodeDecodeError:
            return False
    return False

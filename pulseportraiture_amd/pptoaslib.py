"""Drop-in mirror of PulsePortraiture's ``pptoaslib`` hot path.

``fit_portrait_full`` keeps the reference signature and DataBunch, and runs
the whole per-sub-integration fit on the GPU (libppfit ``ppf_fit_batch``):
rfft + power-spectrum noise + cross spectrum, the scipy trust-ncg replica
over phi/DM/GM/tau/alpha, zero-covariance frequencies, output transform and
the O(nchan) Schur-complement covariance.  ``fit_portrait_full_batch`` is the
batched entry the GetTOAs driver uses.

Reference: /root/reference/pptoaslib.py (file:line cited per function).
"""
import sys
import time

import numpy as np

from . import _lib, engine
from .pplib import (DataBunch, Dconst, RCSTRINGS, _raise_status, _box,  # noqa: F401
                    scattering_times, scattering_portrait_FT, phase_transform,
                    get_bin_centers, guess_fit_freq, rotate_data)

METHODS = ("trust-ncg", "Newton-CG", "TNC")


def phase_shifts(phi, DM, GM, freqs, nu_DM=np.inf, nu_GM=np.inf, P=None,
                 mod=False):
    """pptoaslib.py:195-228 (host)."""
    if P is None:
        P, mod = 1.0, False
    delays = phi + Dconst * DM * (freqs ** -2 - nu_DM ** -2) / P + \
        Dconst ** 2 * GM * (freqs ** -4 - nu_GM ** -4) / P
    if mod:
        delays = np.where(abs(delays) >= 0.5, delays % 1, delays)
        delays = np.where(delays >= 0.5, delays - 1.0, delays)
        if not delays.shape:
            delays = np.float64(delays)
    return delays


def phase_shifts_deriv(freqs, nu_DM=np.inf, nu_GM=np.inf, P=None):
    """pptoaslib.py:231-242 (host)."""
    if P is None:
        P = 1.0
    one = np.ones(len(freqs)) if hasattr(freqs, "shape") else 1.0
    return np.array([one, Dconst * (freqs ** -2 - nu_DM ** -2) / P,
                     Dconst ** 2 * (freqs ** -4 - nu_GM ** -4) / P])


def GM_from_DMc(DMc, D, a_perp):
    """pptoaslib.py:93-105."""
    c = 3e10 / 3.1e21
    return DMc ** 2 * (c * D) / (2.0 * (a_perp * 4.8e-9) ** 2)


def DMc_from_GM(GM, D, a_perp):
    """pptoaslib.py:108-121."""
    c = 3e10 / 3.1e21
    return (GM * (2.0 * a_perp * (4.8e-9) ** 2) / (c * D)) ** 0.5


def rotate_portrait_full(port, phi, DM, GM, freqs, nu_DM=np.inf,
                         nu_GM=np.inf, P=None):
    """pptoaslib.py:61-90: per-channel phase on the host, rotation on the
    GPU."""
    if P is None:
        P = 1.0
    ph = phase_shifts(phi, DM, GM, np.asarray(freqs, dtype=float), nu_DM,
                      nu_GM, P, False)
    port = np.asarray(port)
    ph = np.broadcast_to(np.asarray(ph, dtype=float), (port.shape[0],))
    return engine.rotate_rows(port, ph, ref_len=True).cpu().numpy()


def _status_message(rc, sub_id):
    rcstring = RCSTRINGS.get(str(rc), "")
    if sub_id is not None:
        ii = sub_id[::-1].index("_")
        sys.stderr.write("Fit 'failed' with return code %d: %s -- %s subint "
                         "%s\n" % (rc, rcstring, sub_id[:-ii - 1],
                                   sub_id[-ii:]))
    else:
        sys.stderr.write("Fit 'failed' with return code %d -- %s" %
                         (rc, rcstring))


def _nu_zero_text(fit_flags):
    """The line get_nu_zeros prints for these fit flags when a reference
    frequency is not given (pptoaslib.py:941, 947-948), or None."""
    flags = [int(bool(f)) for f in fit_flags]
    known = ([1, 1, 0, 0, 0], [1, 0, 1, 0, 0], [0, 0, 0, 1, 1],
             [1, 1, 0, 1, 0], [1, 1, 1, 0, 0], [1, 1, 0, 1, 1],
             [1, 1, 1, 1, 0])
    if flags == [1, 1, 1, 1, 1]:
        return "Approximating zero-covariance frequencies..."
    if flags not in known and sum(flags) > 1:
        return "No zero-covariance frequencies found."
    return None


def _nu_zero_messages(fit_flags, nu_outs):
    """Reproduce get_nu_zeros' prints (pptoaslib.py:941, 947-948)."""
    if bool(np.all(nu_outs)):
        return
    text = _nu_zero_text(fit_flags)
    if text is not None:
        print(text)


def unpack_result(R, scales, scale_errs, channel_snrs, cov, fit_flags,
                  duration):
    """Build the fit_portrait_full DataBunch (pptoaslib.py:1134-1143) from one
    device result record."""
    I = _lib.RESULT_INDEX
    flags = [int(bool(f)) for f in fit_flags]
    nfit = int(sum(flags))
    params = list(np.asarray(R[I["params"]], dtype=float))
    param_errs = np.asarray(R[I["param_errs"]], dtype=float).copy()
    status = int(R[I["status"]])
    return DataBunch(
        params=params, param_errs=param_errs, phi=params[0],
        phi_err=param_errs[0], DM=params[1], DM_err=param_errs[1],
        GM=params[2], GM_err=param_errs[2], tau=params[3],
        tau_err=param_errs[3], alpha=params[4], alpha_err=param_errs[4],
        scales=scales, scale_errs=scale_errs, nu_DM=R[I["nu_out"]][0],
        nu_GM=R[I["nu_out"]][1], nu_tau=R[I["nu_out"]][2],
        covariance_matrix=np.asarray(cov)[:nfit, :nfit].copy(),
        chi2=R[I["chi2"]], red_chi2=R[I["red_chi2"]], snr=R[I["snr"]],
        channel_snrs=channel_snrs, duration=duration,
        nfeval=int(R[I["nfeval"]]), return_code=status & 0xff)


def fit_portrait_full(data_port, model_port, init_params, P, freqs,
                      nu_fits=[None, None, None], nu_outs=[None, None, None],
                      errs=None, fit_flags=[1, 1, 1, 1, 1],
                      bounds=[(None, None), (None, None), (None, None),
                              (None, None), (None, None)], log10_tau=True,
                      option=0, sub_id=None, method="trust-ncg", is_toa=True,
                      quiet=True):
    """pptoaslib.py:974-1144 on the GPU (single sub-integration).

    ``method`` 'trust-ncg' is the reference default: the device minimises
    the same objective to the same stationary point with a Newton trust
    region (scaled coordinates, exact subproblem; scipy's own path with
    engine.SOLVER = 'scipy'); 'Newton-CG' runs the same solver.  'TNC'
    applies ``bounds`` as the reference does
    (pptoaslib.py:1041-1046: only for TNC): the device trust-region steps
    are projected onto the box, so the fit ends at the bounded stationary
    point TNC converges to."""
    if method not in METHODS:
        print("Method '%s' is not implemented." % method)
        sys.exit()
    data_port = np.asarray(data_port)
    freqs = np.asarray(freqs, dtype=float)
    nchan, nbin = data_port.shape
    nu_f = np.array([np.nan if v is None else float(v) for v in nu_fits])
    nu_o = np.array([np.nan if v is None else float(v) for v in nu_outs])
    if not bool(np.all(nu_outs)):
        nu_o = np.where(np.array([v is None for v in nu_outs]), np.nan, nu_o)
    init = np.asarray(init_params, dtype=float).reshape(1, 5)
    t0 = time.time()
    res = engine.fit_batch(
        data_port[None], np.asarray(model_port, dtype=float)[None], freqs[None],
        [P], init, [int(bool(f)) for f in fit_flags], nu_fits=nu_f[None],
        nu_outs=nu_o[None],
        errs=None if errs is None else np.asarray(errs, dtype=float)[None],
        log10_tau=log10_tau, option=option, is_toa=is_toa,
        bounds=_box(bounds, 5) if method == "TNC" else None)
    r = engine.results_numpy(res)
    duration = time.time() - t0
    _nu_zero_messages(fit_flags, nu_outs)
    R = r["results"][0]
    status = int(R[_lib.RESULT_INDEX["status"]])
    _raise_status(status)
    rc = status & 0xff
    if rc not in (0, 1, 2, 4):
        _status_message(rc, sub_id)
    return unpack_result(R, r["scales"][0], r["scale_errs"][0],
                         r["channel_snrs"][0], r["covariance"][0], fit_flags,
                         duration)


def get_scales_full(params, data_portrait_FT, model_portrait_FT, errs_FT, P,
                    freqs, nu_DM, nu_GM, nu_tau, log10_tau):
    """pptoaslib.py:953-971: a_n = C_n / S_n at given params, from the given
    data and model spectra, on the GPU (ppf_scales_batch, k_scales: one wave
    per channel, the phasor with exact argument reduction)."""
    D = np.asarray(data_portrait_FT)
    out = engine.scales_batch(
        D, np.asarray(model_portrait_FT), np.asarray(params, dtype=float),
        float(P), np.asarray(freqs, dtype=float),
        [float(nu_DM), float(nu_GM), float(nu_tau)], log10_tau,
        errs_FT=None if errs_FT is None else np.asarray(errs_FT, dtype=float))
    return out[0].cpu().numpy()

"""NumPy/SciPy restatement of the reference wideband fit (oracle, tests only).

Every routine cites the reference file:line it restates.  Paths are relative
to the PulsePortraiture snapshot (pptoaslib.py, pplib.py, pptoas.py).  The
restatement keeps the reference's arithmetic (including its divide-by-C form
of the Hessian, pptoaslib.py:662-671) so that it can serve as a faithful
checker; the one deliberate change is the covariance, computed with the
O(nchan) Schur complement that is algebraically identical to the reference's
dense (5+n)x(5+n)xn block inversion (pptoaslib.py:731-766).
"""
import time
import warnings

import numpy as np
import scipy.optimize as opt

__all__ = [
    "DCONST", "F0_FACT", "get_bin_centers", "noise_ps", "phase_transform",
    "guess_fit_freq", "channel_terms", "objective", "gradient", "hessian",
    "fit_portrait_full", "fit_portrait", "rotate_rows", "rotate_data",
    "fit_phase_shift", "nu_zeros", "get_toas_archive", "align_archives",
    "channel_red_chi2s", "select_zap_channels", "gaussian_profile",
    "gen_gaussian_portrait", "get_scales_full",
]

DCONST = 0.000241 ** -1          # pplib.py:64-67 (Dconst = Dconst_trad)
F0_FACT = 0                      # pplib.py:82 (drop the k=0 harmonic)
LN10 = np.log(10.0)


# ---------------------------------------------------------------------------
# small host helpers
# ---------------------------------------------------------------------------
def get_bin_centers(nbin, lo=0.0, hi=1.0):
    """pplib.py:694-707."""
    diff = float(hi) - float(lo)
    return np.linspace(lo + diff / (nbin * 2), hi - diff / (nbin * 2), nbin)


def noise_ps(rows, frac=4):
    """get_noise_PS (pplib.py:2312-2338): sqrt(mean |rfft|^2/n over the top
    1/frac of harmonics), per row (last axis)."""
    rows = np.atleast_2d(rows)
    F = np.fft.rfft(rows, axis=-1)
    pows = (F.real ** 2 + F.imag ** 2) / rows.shape[-1]
    kc = int((1 - frac ** -1) * pows.shape[-1])
    return np.sqrt(pows[:, kc:].mean(axis=-1))


def phase_transform(phi, DM, nu_ref1=np.inf, nu_ref2=np.inf, P=None,
                    mod=False):
    """pplib.py:2688-2712."""
    if P is None:
        P, mod = 1.0, False
    out = phi + DCONST * DM / P * (nu_ref2 ** -2.0 - nu_ref1 ** -2.0)
    if mod:
        out = np.where(abs(out) >= 0.5, out % 1, out)
        out = np.where(out >= 0.5, out - 1.0, out)
        if not np.shape(out):
            out = np.float64(out)
    return out


def _wrap_half(x):
    """Wrap to [-0.5, 0.5) exactly as pptoaslib.py:1104-1105."""
    if abs(x) >= 0.5:
        x %= 1
    if x >= 0.5:
        x -= 1.0
    return x


def guess_fit_freq(freqs, SNRs=None):
    """pplib.py:2715-2729."""
    nu0 = (freqs.min() + freqs.max()) * 0.5
    if SNRs is None:
        SNRs = np.ones(len(freqs))
    w = SNRs * freqs ** -2
    return nu0 + np.sum((freqs - nu0) * w) / np.sum(w)


# ---------------------------------------------------------------------------
# likelihood pieces: pptoaslib.py:195-684 restated per channel
# ---------------------------------------------------------------------------
def _scat_B(taus, nharm):
    """scattering_portrait_FT (pplib.py:4219-4260): B = 1/(1+2 pi i k tau_n);
    all-ones (real) if every tau_n == 0; rows with tau_n == 0 are ones."""
    k = np.arange(nharm)
    if not np.any(taus):
        return np.ones((len(taus), nharm))
    B = 1.0 / (1.0 + 2j * np.pi * np.outer(taus, k))
    B[taus == 0.0] = 1.0
    return B


def channel_terms(theta, Dft, Mft, errs_FT, P, freqs, nu_DM, nu_GM, nu_tau,
                  log10_tau, need_hess=True):
    """C, dC, d2C, S, dS, d2S per channel (pptoaslib.py:195-561).

    Returns a dict with arrays shaped [nchan], [5, nchan], [5, 5, nchan]."""
    phi, DM, GM, tau, alpha = theta
    if log10_tau:
        tau = 10 ** tau
    nchan, nharm = Dft.shape
    k = np.arange(nharm)
    e2 = errs_FT ** 2
    # phase_shifts / _deriv (pptoaslib.py:195-242)
    dphi = np.array([np.ones(nchan),
                     DCONST * (freqs ** -2 - nu_DM ** -2) / P,
                     DCONST ** 2 * (freqs ** -4 - nu_GM ** -4) / P])
    phis = phi + DM * dphi[1] + GM * dphi[2]
    E = np.exp(2.0j * np.pi * np.outer(phis, k))
    # scattering times and their derivatives (pptoaslib.py:266-299)
    taus = tau * (freqs / nu_tau) ** alpha
    lnf = np.log(freqs / nu_tau)
    tsum = taus.sum()
    if log10_tau:
        dtau = LN10 * taus
        d2tau = LN10 * dtau
    else:
        dtau = taus / tau if tsum else np.zeros(nchan)
        d2tau = np.zeros(nchan)
    dalpha = lnf * taus
    if log10_tau:
        dtaudalpha = LN10 * dalpha
    else:
        dtaudalpha = dalpha / tau if tsum else np.zeros(nchan)
    d2alpha = lnf * dalpha
    B = _scat_B(taus, nharm)
    # scattering_portrait_FT_deriv / _2deriv (pptoaslib.py:344-383)
    if tsum:
        f1 = B * (B - 1.0) / taus[:, None]
        dB = np.array([f1 * dtau[:, None], f1 * dalpha[:, None]])
        H = B * (B - 1.0) / taus[:, None] ** 2
        H11 = H * (dtau ** 2)[:, None]
        if dtau.sum():
            H11 = H11 * (2 * (B - 1) + (d2tau * taus / dtau ** 2)[:, None])
        H22 = H * (dalpha ** 2)[:, None]
        if dalpha.sum():
            H22 = H22 * (2 * (B - 1) + (d2alpha * taus / dalpha ** 2)[:, None])
        H12 = H * (dtau * dalpha)[:, None]
        if dalpha.sum() and dtau.sum():
            H12 = H12 * (2 * (B - 1) +
                         (dtaudalpha * taus / (dtau * dalpha))[:, None])
        d2B = np.array([[H11, H12], [H12, H22]])
    else:
        dB = np.zeros((2, nchan, nharm))
        d2B = np.zeros((2, 2, nchan, nharm))
    M2 = np.abs(Mft) ** 2
    # Sbp / _deriv / _2deriv (pptoaslib.py:421-455)
    S = np.sum(np.abs(B) ** 2 * M2, axis=-1) / e2
    dabs = 2 * np.real(B * np.conj(dB))
    dS = np.zeros((5, nchan))
    dS[3:] = np.sum(dabs * M2, axis=-1) / e2
    d2S = np.zeros((5, 5, nchan))
    if need_hess:
        a11 = 2 * (np.abs(dB[0]) ** 2 + np.real(B * np.conj(d2B[0, 0])))
        a22 = 2 * (np.abs(dB[1]) ** 2 + np.real(B * np.conj(d2B[1, 1])))
        a12 = 2 * np.real(dB[0] * np.conj(dB[1]) + B * np.conj(d2B[0, 1]))
        d2S[3, 3] = np.sum(a11 * M2, axis=-1) / e2
        d2S[4, 4] = np.sum(a22 * M2, axis=-1) / e2
        d2S[3, 4] = d2S[4, 3] = np.sum(a12 * M2, axis=-1) / e2
    # Cdbp and derivatives (pptoaslib.py:458-561)
    base = Dft * np.conj(Mft) * E
    bB = base * np.conj(B)
    w1 = 2.0j * np.pi * k
    C = np.real(bB.sum(axis=-1)) / e2
    Cp = np.real((w1 * bB).sum(axis=-1))
    dC = np.zeros((5, nchan))
    dC[:3] = Cp * dphi / e2
    dC[3:] = np.real((base * np.conj(dB)).sum(axis=-1)) / e2
    d2C = np.zeros((5, 5, nchan))
    if need_hess:
        Cpp = np.real((w1 ** 2 * bB).sum(axis=-1))
        for i in range(3):
            for j in range(3):
                d2C[i, j] = Cpp * dphi[i] * dphi[j] / e2
        for i in range(2):
            for j in range(2):
                d2C[3 + i, 3 + j] = np.real(
                    (base * np.conj(d2B[i, j])).sum(axis=-1)) / e2
        cross = np.real((w1 * base * np.conj(dB)).sum(axis=-1))
        for i in range(3):
            for j in range(2):
                d2C[i, 3 + j] = d2C[3 + j, i] = dphi[i] * cross[j] / e2
    return dict(C=C, dC=dC, d2C=d2C, S=S, dS=dS, d2S=d2S, dphi=dphi,
                taus=taus, dtau=dtau, dalpha=dalpha, tau=tau)


def objective(t):
    """fit_portrait_full_function (pptoaslib.py:564-581)."""
    return -(t["C"] ** 2 / t["S"]).sum()


def gradient(t, flags):
    """fit_portrait_full_function_deriv (pptoaslib.py:584-614)."""
    C, S = t["C"], t["S"]
    g = -((C ** 2 / S) * (2 * t["dC"] / C - t["dS"] / S)).sum(axis=-1)
    return g * np.asarray(flags, dtype=float)


def hessian(t, flags, per_channel=False):
    """fit_portrait_full_function_2deriv (pptoaslib.py:617-684)."""
    C, S, dC, dS, d2C, d2S = (t[k] for k in ("C", "S", "dC", "dS", "d2C",
                                             "d2S"))
    f = np.asarray(flags, dtype=float)
    H = np.zeros((5, 5, len(C)))
    for i in range(5):
        for j in range(5):
            H[i, j] = -2 * ((C ** 2 / S) * (
                d2C[i, j] / C - 0.5 * d2S[i, j] / S + dC[i] * dC[j] / C ** 2 +
                dS[i] * dS[j] / S ** 2 -
                (dC[i] * dS[j] + dS[i] * dC[j]) / (C * S))) * f[i] * f[j]
    return H if per_channel else H.sum(axis=-1)


# ---------------------------------------------------------------------------
# zero-covariance frequencies: pptoaslib.py:776-950
# ---------------------------------------------------------------------------
def _real_pos_roots(coeffs):
    r = np.roots(coeffs)
    r = np.real(r[np.where(np.imag(r) == 0.0)[0]])
    return r[np.where(r > 0.0)[0]]


def nu_zeros(theta, Dft, Mft, errs_FT, P, freqs, nu_DM, nu_GM, nu_tau, flags,
             log10_tau, option=0, messages=None):
    flags = [int(bool(x)) for x in flags]
    t = channel_terms(theta, Dft, Mft, errs_FT, P, freqs, nu_DM, nu_GM,
                      nu_tau, log10_tau)
    Hn = hessian(t, flags, per_channel=True)
    dphi = t["dphi"]
    ta = t["dalpha"] / t["taus"] if np.all(t["taus"]) else None
    f2, f4 = freqs ** -2, freqs ** -4
    if flags == [1, 1, 0, 0, 0]:
        h = Hn[0, 1] / dphi[1]
        return [(np.sum(f2 * h) / h.sum()) ** -0.5, nu_GM, nu_tau]
    if flags == [1, 0, 1, 0, 0]:
        h = Hn[0, 2] / dphi[2]
        return [nu_DM, (np.sum(f4 * h) / h.sum()) ** -0.25, nu_tau]
    if flags == [0, 0, 0, 1, 1]:
        h = Hn[3, 4] / ta
        return [nu_DM, nu_GM, np.exp(np.sum(np.log(freqs) * h) / h.sum())]
    if flags == [1, 1, 0, 1, 0]:
        H21, H23 = Hn[1, 0] / dphi[1], Hn[1, 3] / dphi[1]
        Hs = Hn.sum(axis=-1)
        H13, H33 = Hs[3, 0], Hs[3, 3]
        num = H13 * np.sum(f2 * H23) - H33 * np.sum(f2 * H21)
        den = H13 * H23.sum() - H33 * H21.sum()
        return [(num / den) ** -0.5, nu_GM, nu_tau]
    if flags == [1, 1, 1, 0, 0]:
        if option not in (0, 1):
            return [nu_DM, nu_GM, nu_tau]
        if option == 0:
            H21, H23 = Hn[1, 0] / dphi[1], Hn[1, 2] / dphi[1]
            H31, H33 = Hn[2, 0] / dphi[2], Hn[2, 2] / dphi[2]
            A, B = (H31 * f4).sum(), H31.sum()
            C, D = (H23 * f2).sum(), H23.sum()
            E, F = (H33 * f4).sum(), H33.sum()
            G, H = (H21 * f2).sum(), H21.sum()
        else:
            H21, H22 = Hn[1, 0] / dphi[1], Hn[1, 1] / dphi[1]
            H31, H32 = Hn[2, 0] / dphi[2], Hn[2, 1] / dphi[2]
            A, B = (H21 * f4).sum(), H21.sum()
            C, D = (H32 * f2).sum(), H32.sum()
            E, F = (H22 * f4).sum(), H22.sum()
            G, H = (H31 * f2).sum(), H31.sum()
        roots = _real_pos_roots([A * C - E * G, 0.0, E * H - A * D, 0.0,
                                 F * G - B * C, 0.0, B * D - F * H])
        nz = roots[np.argmin(abs(freqs.mean() - roots))]
        return [nz, nz, nu_tau]
    if flags == [1, 1, 0, 1, 1]:
        # reduced ordering (phi, DM, tau, alpha)
        idx = [0, 1, 3, 4]
        Hr = Hn[np.ix_(idx, idx)]
        H21, H23, H24 = (Hr[1, j] / dphi[1] for j in (0, 2, 3))
        H41, H42, H43 = (Hr[3, j] / ta for j in (0, 1, 2))
        Hs = Hr.sum(axis=-1)
        H11, H22, H33, H44 = np.diag(Hs)
        H12, H13, H14 = Hs[0, 1:]
        H23s, H24s = Hs[1, 2:]
        H34 = Hs[2, 3]
        num = ((H34 * H34 - H33 * H44) * (f2 * H21).sum() +
               (H13 * H44 - H14 * H34) * (f2 * H23).sum() +
               (H14 * H33 - H13 * H34) * (f2 * H24).sum())
        den = ((H34 * H34 - H33 * H44) * H21.sum() +
               (H13 * H44 - H14 * H34) * H23.sum() +
               (H14 * H33 - H13 * H34) * H24.sum())
        nz_dm = (num / den) ** -0.5
        lf = np.log(freqs)
        num = ((H13 * H22 - H12 * H23s) * (lf * H41).sum() +
               (H11 * H23s - H12 * H13) * (lf * H42).sum() +
               (H12 * H12 - H11 * H22) * (lf * H43).sum())
        den = ((H13 * H22 - H12 * H23s) * H41.sum() +
               (H11 * H23s - H12 * H13) * H42.sum() +
               (H12 * H12 - H11 * H22) * H43.sum())
        return [nz_dm, nu_GM, np.exp(num / den)]
    if flags == [1, 1, 1, 1, 0]:
        if option not in (0, 1):
            return [nu_DM, nu_GM, nu_tau]
        Hr = Hn[:4, :4]
        Hs = Hr.sum(axis=-1)
        q2 = freqs ** -2 - nu_DM ** -2
        q4 = freqs ** -4 - nu_GM ** -4
        H14, H44 = Hs[3, 0], Hs[3, 3]
        if option == 0:
            H21, H23, H24 = (Hr[1, j] / q2 for j in (0, 2, 3))
            H31, H33, H34 = (Hr[2, j] / q4 for j in (0, 2, 3))
            A, a = (f4 * H34).sum(), H34.sum()
            B, b = (f2 * H21).sum(), H21.sum()
            C, c = (f4 * H31).sum(), H31.sum()
            D, d = (f2 * H23).sum(), H23.sum()
            E, e = (f4 * H33).sum(), H33.sum()
            F, f = (f2 * H24).sum(), H24.sum()
            P5 = A**2*B + H44*C*D + H14*E*F - H44*B*E - A*C*F - H14*A*D
            P4 = -A**2*b - H44*C*d - H14*E*f + H44*b*E + A*C*f + H14*A*d
            P3 = (-2*A*a*B - H44*c*D - H14*e*F + H44*B*e + (A*c + a*C)*F +
                  H14*a*D)
            P2 = (2*A*a*b + H44*c*d + H14*e*f - H44*b*e - (A*c + a*C)*f -
                  H14*a*d)
            P1 = a**2*B - a*c*F
            P0 = -a**2*b + a*c*f
            coeffs = [P5, P4, P3, P2, P1, P0]
        else:
            H21, H22, H24 = (Hr[1, j] / q2 for j in (0, 1, 3))
            H31, H32, H34 = (Hr[2, j] / q4 for j in (0, 1, 3))
            A, a = (f2 * H24).sum(), H24.sum()
            B, b = (f4 * H31).sum(), H31.sum()
            C, c = (f2 * H21).sum(), H21.sum()
            D, d = (f4 * H32).sum(), H32.sum()
            E, e = (f2 * H22).sum(), H22.sum()
            F, f = (f4 * H34).sum(), H34.sum()
            P4 = A**2*B + H44*C*D + H14*E*F - H44*B*E - A*C*F - H14*A*D
            P3 = (-2*A*a*B - H44*c*D - H14*e*F + H44*B*e + (A*c + a*C)*F +
                  H14*a*D)
            P2 = (-(A**2*b - a**2*B) - H44*C*d - H14*E*f + H44*b*E +
                  (A*C*f - a*c*F) + H14*A*d)
            P1 = (2*A*a*b + H44*c*d + H14*e*f - H44*b*e - (A*c + a*C)*f -
                  H14*a*d)
            P0 = -a**2*b + a*c*f
            coeffs = [P4, P3, P2, P1, P0]
        roots = _real_pos_roots(coeffs) ** 0.5
        nz = roots[np.argmin(abs(freqs.mean() - roots))]
        return [nz, nz, nu_tau]
    if flags == [1, 1, 1, 1, 1]:
        if messages is not None:
            messages.append("Approximating zero-covariance frequencies...")
        return nu_zeros(theta, Dft, Mft, errs_FT, P, freqs, nu_DM, nu_GM,
                        nu_tau, [1, 1, 0, 1, 1], log10_tau, option)
    if sum(flags) > 1 and messages is not None:
        messages.append("No zero-covariance frequencies found.")
    return [nu_DM, nu_GM, nu_tau]


# ---------------------------------------------------------------------------
# fit_portrait_full: pptoaslib.py:974-1144
# ---------------------------------------------------------------------------
def _spectra(data_port, model_port):
    Dft = np.fft.rfft(data_port, axis=-1)
    Dft[:, 0] *= F0_FACT
    Mft = np.fft.rfft(model_port, axis=-1)
    Mft[:, 0] *= F0_FACT
    return Dft, Mft


def fit_portrait_full(data_port, model_port, init_params, P, freqs,
                      nu_fits=(None, None, None), nu_outs=(None, None, None),
                      errs=None, fit_flags=(1, 1, 1, 1, 1), log10_tau=True,
                      option=0, is_toa=True, messages=None,
                      method="trust-ncg", bounds=None, x_fit=None):
    """pptoaslib.py:974-1144 (Schur covariance instead of the dense cube).
    method 'TNC' minimises with scipy TNC under `bounds` exactly as
    pptoaslib.py:1041-1060 does (minfev = dof - Sd, xtol 1e-10; maxiter is
    not a TNC option and scipy ignores it); x_fit (test infrastructure)
    skips the minimiser and reports the post-fit quantities at x_fit."""
    data_port = np.asarray(data_port, dtype=np.float64)
    model_port = np.asarray(model_port, dtype=np.float64)
    freqs = np.asarray(freqs, dtype=np.float64)
    flags = [int(bool(x)) for x in fit_flags]
    ifit = np.where(flags)[0]
    nfit = len(ifit)
    nchan, nbin = data_port.shape
    dof = data_port.size - (nfit + nchan)
    Dft, Mft = _spectra(data_port, model_port)
    if errs is None:
        errs_FT = noise_ps(data_port) * np.sqrt(nbin / 2.0)
    else:
        errs_FT = np.asarray(errs, dtype=np.float64) * np.sqrt(nbin / 2.0)
    Sd = ((np.abs(Dft) ** 2).T / errs_FT ** 2.0).T.sum()
    nu_fit = [freqs.mean() if v is None else v for v in nu_fits]
    args = (Dft, Mft, errs_FT, P, freqs, nu_fit[0], nu_fit[1], nu_fit[2],
            log10_tau)
    cache = {}

    def terms(x):
        key = tuple(np.asarray(x, dtype=float))
        if key not in cache:
            cache.clear()
            cache[key] = channel_terms(np.asarray(x, dtype=float), *args)
        return cache[key]

    t0 = time.time()
    if x_fit is not None:
        x = np.asarray(x_fit, dtype=float)
        res = opt.OptimizeResult(x=x, fun=objective(terms(x)), nfev=0,
                                 status=0)
    elif method == "TNC":
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", opt.OptimizeWarning)
            res = opt.minimize(
                lambda x: objective(terms(x)), np.asarray(init_params,
                                                          dtype=float),
                method="TNC", jac=lambda x: gradient(terms(x), flags),
                bounds=bounds, options={"maxiter": 2000, "disp": False,
                                        "xtol": 1e-10,
                                        "minfev": dof - Sd})
    else:
        res = opt.minimize(lambda x: objective(terms(x)), np.asarray(
            init_params, dtype=float), method="trust-ncg",
            jac=lambda x: gradient(terms(x), flags),
            hess=lambda x: hessian(terms(x), flags), options={"gtol": -1})
    duration = time.time() - t0
    phi_fit, DM_fit, GM_fit, tau_fit, alpha_fit = res.x
    nu_out = list(nu_outs)
    if not bool(np.all(nu_outs)):
        nz = nu_zeros(res.x, Dft, Mft, errs_FT, P, freqs, nu_fit[0],
                      nu_fit[1], nu_fit[2], flags, log10_tau, option,
                      messages)
        nu_out = [nz[i] if nu_out[i] is None else nu_out[i] for i in range(3)]
    if is_toa:
        if flags[1]:
            nu_out[1] = nu_out[0]
        elif flags[2]:
            nu_out[0] = nu_out[1]
    phi_inf = phi_fit - DCONST * DM_fit * nu_fit[0] ** -2 / P - \
        DCONST ** 2 * GM_fit * nu_fit[1] ** -4 / P
    phi_out = phi_inf + DCONST / P * DM_fit * nu_out[0] ** -2 + \
        DCONST ** 2 / P * GM_fit * nu_out[1] ** -4
    phi_out = _wrap_half(phi_out)
    tau_lin = 10 ** tau_fit if log10_tau else tau_fit
    tau_out = tau_lin * (nu_out[2] / nu_fit[2]) ** alpha_fit
    if log10_tau:
        tau_out = np.log10(tau_out)
    params = [phi_out, DM_fit, GM_fit, tau_out, alpha_fit]
    t = channel_terms(np.array(params), Dft, Mft, errs_FT, P, freqs,
                      nu_out[0], nu_out[1], nu_out[2], log10_tau)
    cov_full, scale_errs, scales = _schur_covariance(t, flags)
    param_errs = np.zeros(5)
    param_errs[ifit] = np.sqrt(np.diag(cov_full))
    S = t["S"]
    channel_snrs = scales * np.sqrt(S)
    snr = np.sqrt(np.sum(channel_snrs ** 2))
    chi2 = Sd + res.fun
    return dict(params=params, param_errs=param_errs, phi=phi_out,
                phi_err=param_errs[0], DM=DM_fit, DM_err=param_errs[1],
                GM=GM_fit, GM_err=param_errs[2], tau=tau_out,
                tau_err=param_errs[3], alpha=alpha_fit,
                alpha_err=param_errs[4], scales=scales, scale_errs=scale_errs,
                nu_DM=nu_out[0], nu_GM=nu_out[1], nu_tau=nu_out[2],
                covariance_matrix=cov_full, chi2=chi2, red_chi2=chi2 / dof,
                snr=snr, channel_snrs=channel_snrs, duration=duration,
                nfeval=res.nfev, return_code=res.status, Sd=Sd,
                fun=res.fun, x_fit=res.x)


def get_scales_full(params, Dft, Mft, errs_FT, P, freqs, nu_DM, nu_GM,
                    nu_tau, log10_tau):
    """pptoaslib.py:953-971: a_n = C_n / S_n (Cdbp / Sbp, pptoaslib.py:421-469)
    at given parameters from given spectra."""
    phi, DM, GM, tau, alpha = params
    if log10_tau:
        tau = 10 ** tau
    nharm = Dft.shape[-1]
    phis = (phi + DCONST * DM * (freqs ** -2 - nu_DM ** -2) / P +
            DCONST ** 2 * GM * (freqs ** -4 - nu_GM ** -4) / P)
    E = np.exp(2.0j * np.pi * np.outer(phis, np.arange(nharm)))
    B = _scat_B(tau * (freqs / nu_tau) ** alpha, nharm)
    S = np.sum(np.abs(B) ** 2 * np.abs(Mft) ** 2, axis=-1) / errs_FT ** 2
    C = np.real(np.sum(Dft * np.conj(Mft) * np.conj(B) * E, axis=-1)) / \
        errs_FT ** 2
    return C / S


def _schur_covariance(t, flags):
    """Covariance of (theta, a_n) from the full Hessian of
    fit_portrait_full_function_2deriv_with_scales (pptoaslib.py:687-773),
    evaluated with the Schur complement instead of the dense cube."""
    C, S, dC, dS, d2C, d2S = (t[k] for k in ("C", "S", "dC", "dS", "d2C",
                                             "d2S"))
    f = np.asarray(flags, dtype=float)
    ifit = np.where(flags)[0]
    scales = C / S
    A = np.zeros((5, 5))
    for i in range(5):
        for j in range(5):
            A[i, j] = np.sum(-2 * ((C ** 2 / S) * (d2C[i, j] / C -
                                                   0.5 * d2S[i, j] / S))
                             ) * f[i] * f[j]
    U = (-2 * (dC - scales * dS)) * f[:, None]
    A, U = A[np.ix_(ifit, ifit)], U[ifit]
    cinv = 1.0 / (2 * S)
    X = A - (U * cinv) @ U.T
    Xinv = np.linalg.inv(X)
    cov_theta = 2.0 * Xinv
    var_a = 2.0 * (cinv + np.einsum("in,ij,jn->n", U, Xinv, U) * cinv ** 2)
    return cov_theta, np.sqrt(var_a), scales


# ---------------------------------------------------------------------------
# pplib.fit_portrait (legacy 2-parameter FFTFIT): pplib.py:1335-1447, 2185-2287
# ---------------------------------------------------------------------------
def _fp_terms(params, mFFT, p_n, dFFT, errs, P, freqs, nu_ref):
    phase, DM = params
    D = DCONST * DM / P
    k = np.arange(mFFT.shape[1])
    ph = phase + D * (freqs ** -2.0 - nu_ref ** -2.0)
    E = np.exp(2.0j * np.pi * np.outer(ph, k))
    prod = dFFT * np.conj(mFFT) * E
    Cdp = np.real(prod).sum(axis=1)
    d1 = np.real(2.0j * np.pi * k * prod).sum(axis=1)
    d2 = np.real((2.0j * np.pi * k) ** 2 * prod).sum(axis=1)
    dDM = (freqs ** -2.0 - nu_ref ** -2.0) * (DCONST / P)
    return Cdp, d1, d2, dDM


def fit_portrait(data, model, init_params, P, freqs, nu_fit=None, nu_out=None,
                 errs=None, bounds=((None, None), (None, None))):
    data = np.asarray(data, dtype=np.float64)
    model = np.asarray(model, dtype=np.float64)
    dFFT, mFFT = _spectra(data, model)
    nbin = data.shape[1]
    if errs is None:
        errs = noise_ps(data) * np.sqrt(nbin / 2.0)
    else:
        errs = np.copy(errs) * np.sqrt(nbin / 2.0)
    d = np.real(np.sum((errs ** -2.0)[:, None] * (dFFT * np.conj(dFFT))))
    p_n = np.real(np.sum(mFFT * np.conj(mFFT), axis=1))
    if nu_fit is None:
        nu_fit = freqs.mean()
    a = (mFFT, p_n, dFFT, errs, P, freqs, nu_fit)

    def fun(x):
        Cdp, _, _, _ = _fp_terms(x, *a)
        return -np.sum(Cdp ** 2.0 / (errs ** 2.0 * p_n))

    def jac(x):
        Cdp, d1, _, dDM = _fp_terms(x, *a)
        w = -2 * Cdp * d1 / (errs ** 2.0 * p_n)
        return np.array([w.sum(), (w * dDM).sum()])

    t0 = time.time()
    res = opt.minimize(fun, init_params, method="TNC", jac=jac,
                       bounds=list(bounds),
                       options={"disp": False, "xtol": 1e-10})
    duration = time.time() - t0
    phi, DM = res.x

    def hess_nz(x, nu_ref):
        Cdp, d1, d2, dDM = _fp_terms(x, mFFT, p_n, dFFT, errs, P, freqs,
                                     nu_ref)
        W = (d1 ** 2.0 + Cdp * d2) / (errs ** 2.0 * p_n)
        H = np.array([(-2.0 * W).sum(), (-2.0 * W * dDM ** 2.0).sum(),
                      (-2.0 * W * dDM).sum()])
        return H, (W.sum() / np.sum(W * freqs ** -2)) ** 0.5

    nu_zero = hess_nz(np.array([phi, DM]), nu_fit)[1]
    if nu_out is None:
        nu_out = nu_zero
    phi_out = phase_transform(phi, DM, nu_fit, nu_out, P, mod=True)
    h = hess_nz(np.array([phi_out, DM]), nu_out)[0]
    cov = np.linalg.inv(0.5 * np.array([[h[0], h[2]], [h[2], h[1]]]))
    param_errs = np.diag(cov) ** 0.5
    dof = data.size - (len(freqs) + 2)
    chi2 = d + res.fun
    Cdp, _, _, _ = _fp_terms(np.array([phi, DM]), *a)
    scales = Cdp / p_n
    scale_errs = (p_n / errs ** 2.0) ** -0.5
    snr = np.sum(scales ** 2.0 * p_n / errs ** 2.0) ** 0.5
    return dict(phase=phi_out, phase_err=param_errs[0], DM=DM,
                DM_err=param_errs[1], scales=scales, scale_errs=scale_errs,
                nu_ref=nu_out, covariance=cov[0, 1], chi2=chi2,
                red_chi2=chi2 / dof, snr=snr, duration=duration,
                nfeval=res.nfev, return_code=res.status)


# ---------------------------------------------------------------------------
# rotation: pplib.py:2427-2550, pptoaslib.py:61-90
# ---------------------------------------------------------------------------
def rotate_rows(rows, phases):
    """rfft -> x exp(2 pi i k phase_row) -> irfft, one phase per row."""
    rows = np.atleast_2d(rows)
    F = np.fft.rfft(rows, axis=-1)
    k = np.arange(F.shape[-1])
    F *= np.exp(2.0j * np.pi * np.outer(np.ravel(phases), k))
    return np.fft.irfft(F, n=rows.shape[-1], axis=-1)


def rotate_data(data, phase=0.0, DM=0.0, Ps=None, freqs=None, nu_ref=np.inf):
    """pplib.rotate_data (pplib.py:2427-2515) for the well-formed branches."""
    data = np.asarray(data, dtype=np.float64)
    nbin = data.shape[-1]
    if DM == 0.0:
        rows = data.reshape(-1, nbin)
        out = rotate_rows(rows, np.full(len(rows), phase))
        return out.reshape(data.shape)
    d4 = data
    while d4.ndim != 4:
        d4 = d4[None]
    nsub, npol, nchan, _ = d4.shape
    D = DCONST * DM / (np.ones(nsub) * Ps)
    freqs = np.asarray(freqs, dtype=float)
    if freqs.ndim == 0:
        freqs = np.ones(nchan) * float(freqs)
    if freqs.ndim == 1:
        fterm = np.tile(freqs, nsub).reshape(nsub, nchan) ** -2.0 - \
            nu_ref ** -2.0
    else:
        fterm = freqs ** -2.0 - nu_ref ** -2.0
    ph = phase + D[:, None] * fterm                     # [nsub, nchan]
    ph = np.broadcast_to(ph[:, None, :], (nsub, npol, nchan))
    out = rotate_rows(d4.reshape(-1, nbin), ph.reshape(-1)).reshape(d4.shape)
    if data.ndim == 1:
        return out[0, 0, 0]
    if data.ndim == 2:
        return out[0, 0]
    return out


# ---------------------------------------------------------------------------
# fit_phase_shift: pplib.py:1294-1332, 2136-2182
# ---------------------------------------------------------------------------
def fit_phase_shift(data, model, noise=None, bounds=(-0.5, 0.5), Ns=100):
    dFFT = np.fft.rfft(data)
    dFFT[0] *= F0_FACT
    mFFT = np.fft.rfft(model)
    mFFT[0] *= F0_FACT
    if noise is None:
        err = noise_ps(data)[0] * np.sqrt(len(data) / 2.0)
    else:
        err = noise * np.sqrt(len(data) / 2.0)
    d = np.real(np.sum(dFFT * np.conj(dFFT))) / err ** 2.0
    p = np.real(np.sum(mFFT * np.conj(mFFT))) / err ** 2.0
    k = np.arange(len(mFFT))
    xm = dFFT * np.conj(mFFT)

    def f(phase):
        return -np.real((xm * np.exp(k * 2.0j * np.pi * phase)).sum()) / \
            err ** 2.0

    res = opt.brute(f, [tuple(bounds)], Ns=Ns, full_output=True)
    phase = res[0][0]
    fmin = res[1]
    scale = -fmin / p
    d2 = -np.real((-4.0 * np.pi ** 2 * k ** 2 * xm *
                   np.exp(k * 2.0j * np.pi * phase)).sum()) / err ** 2.0
    return dict(phase=phase, phase_err=(scale * d2) ** -0.5, scale=scale,
                scale_err=p ** -0.5, snr=(scale ** 2 * p) ** 0.5,
                red_chi2=(d - fmin ** 2 / p) / (len(data) - 2))


# ---------------------------------------------------------------------------
# GetTOAs.get_TOAs inner loop for one archive (pptoas.py:384-729), host-only
# bookkeeping that needs no PSRCHIVE: guess -> fit -> Doppler -> DeltaDM.
# ---------------------------------------------------------------------------
def get_toas_archive(subints, models, freqs, weights, SNRs, Ps, DM_stored,
                     doppler_factors, ok_isubs=None, noise_stds=None,
                     fit_flags=(1, 1, 0, 0, 0), bary=True, DM0=None,
                     tau_guess=0.0, alpha_guess=-4.0, log10_tau=True,
                     scat_guess=None):
    """subints [nsub, nchan, nbin]; models [nsub, nchan, nbin] (or one
    [nchan, nbin] shared); weights / SNRs [nsub, nchan].  With a scattering
    fit (fit_flags[3] or [4]) the guesses follow pptoas.py:467-492: tau_guess
    [rot] at nu_fit scatters the mean model profile of the phase guess, and
    with log10_tau a zero tau_guess becomes log10(1 / nbin); scat_guess =
    (tau [s], its reference frequency [MHz], alpha) overrides them per
    sub-int as pptoas.py:469-472 does."""
    nsub, nchan, nbin = subints.shape
    if ok_isubs is None:
        ok_isubs = np.arange(nsub)
    out = {k: np.zeros(nsub) for k in ("phis", "phi_errs", "DMs", "DM_errs",
                                       "red_chi2s", "snrs", "GMs", "taus",
                                       "alphas")}
    out["param_errs"] = np.zeros((nsub, 5))
    out["nu_refs"] = np.zeros((nsub, 3))
    out["nu_fits"] = np.zeros((nsub, 3))
    out["scales"] = np.zeros((nsub, nchan))
    nfit = int(np.sum(fit_flags))
    out["covariances"] = np.zeros((nsub, nfit, nfit))
    for isub in ok_isubs:
        ok = np.where(weights[isub] != 0.0)[0]
        freqsx = freqs[isub, ok]
        portx = subints[isub][ok]
        model = models if models.ndim == 2 else models[isub]
        modelx = model[ok]
        P = Ps[isub]
        errs = noise_ps(portx) if noise_stds is None else noise_stds[isub, ok]
        nu_mean = freqsx.mean()
        nu_fit = guess_fit_freq(freqsx, SNRs[isub, ok])
        rot = rotate_data(portx, 0.0, DM_stored, P, freqsx, nu_mean)
        rot_prof = np.average(rot, axis=0, weights=weights[isub, ok])
        scat = bool(fit_flags[3] or fit_flags[4])
        mprof = modelx.mean(axis=0)
        tg, ag = 0.0, 0.0
        if scat:
            tg, ag = float(tau_guess), float(alpha_guess)
            if scat_guess is not None:
                ag = float(scat_guess[2])
                tg = (scat_guess[0] / P) * (nu_fit / scat_guess[1]) ** ag
            B = _scat_B(np.array([tg]), nbin // 2 + 1)[0]
            mprof = np.fft.irfft(B * np.fft.rfft(mprof), n=nbin)
        phi_guess = fit_phase_shift(rot_prof, mprof, Ns=100)["phase"]
        phi_guess = phase_transform(phi_guess, DM_stored, nu_mean, nu_fit, P,
                                    mod=True)
        lt = bool(log10_tau) and scat
        if lt:
            tg = np.log10(tg if tg != 0.0 else 1.0 / nbin)
        flags = list(fit_flags)
        if len(freqsx) == 1:
            flags = [1, 0, 0, 0, 0]
        r = fit_portrait_full(portx, modelx, [phi_guess, DM_stored, 0.0, tg,
                                              ag], P, freqsx,
                              [nu_fit] * 3, [None] * 3, errs, flags,
                              log10_tau=lt)
        df = doppler_factors[isub] if bary else 1.0
        DM = r["DM"] * df if flags[1] else r["DM"]
        out["phis"][isub] = r["phi"]
        out["phi_errs"][isub] = r["phi_err"]
        out["DMs"][isub] = DM
        out["DM_errs"][isub] = r["DM_err"]
        out["GMs"][isub] = r["GM"] * df ** 3 if flags[2] else r["GM"]
        out["taus"][isub] = r["tau"]
        out["alphas"][isub] = r["alpha"]
        out["param_errs"][isub] = r["param_errs"]
        out["red_chi2s"][isub] = r["red_chi2"]
        out["snrs"][isub] = r["snr"]
        out["nu_refs"][isub] = [r["nu_DM"], r["nu_GM"], r["nu_tau"]]
        out["nu_fits"][isub] = [nu_fit] * 3
        out["scales"][isub, ok] = r["scales"]
        cm = r["covariance_matrix"]
        if cm.shape == out["covariances"][isub].shape:
            out["covariances"][isub] = cm
    DM0 = DM_stored if DM0 is None else DM0
    dDMs = out["DMs"] - DM0
    errs = out["DM_errs"][ok_isubs]
    w = errs ** -2 if np.all(errs) else np.ones(len(errs))
    mean, wsum = np.average(dDMs[ok_isubs], weights=w, returned=True)
    var = wsum ** -1
    if len(ok_isubs) > 1:
        var *= np.sum((dDMs[ok_isubs] - mean) ** 2 * w) / (len(ok_isubs) - 1)
    out["DeltaDM_mean"] = mean
    out["DeltaDM_err"] = var ** 0.5
    return out


# ---------------------------------------------------------------------------
# ppalign.align_archives (ppalign.py:65-257), the iteration only: archives
# come in as DataBunch-like objects (the keys of pplib.py:2904-2914), no
# archive I/O, no output archive.
# ---------------------------------------------------------------------------
def align_archives(archives, model_data, fit_dm=True, niter=1, npol=1):
    """archives: list of objects with .subints [nsub, npol, nchan, nbin],
    .weights, .freqs, .Ps, .SNRs, .noise_stds, .ok_isubs, .ok_ichans, .DM,
    .dmc, .nbin; model_data likewise (one sub-int).  Returns (aligned_port
    [npol, nchan, nbin], total_weights [nchan, nbin])."""
    model_port = (model_data.masks * model_data.subints)[0, 0]
    nchan, nbin = model_port.shape
    for _ in range(niter):
        aligned_port = np.zeros((npol, nchan, nbin))
        total_weights = np.zeros((nchan, nbin))
        for data in archives:
            try:
                fd = data.freqs - model_data.freqs
                same_freqs = fd.min() == fd.max() == 0.0
            except Exception:
                same_freqs = False
            DM_guess = data.DM * np.logical_not(data.dmc)
            for isub in data.ok_isubs:
                if same_freqs:
                    ichans = np.intersect1d(data.ok_ichans[isub],
                                            model_data.ok_ichans[0])
                    model_ichans = ichans
                else:
                    ichans = data.ok_ichans[isub]
                    mok = model_data.ok_ichans[0]
                    model_ichans = np.array([
                        mok[np.argmin(abs(model_data.freqs[0][mok] -
                                          data.freqs[isub, ic]))]
                        for ic in ichans])
                port = data.subints[isub, 0, ichans]
                freqs = data.freqs[isub, ichans]
                model = model_port[model_ichans]
                P = data.Ps[isub]
                SNRs = data.SNRs[isub, 0, ichans]
                errs = data.noise_stds[isub, 0, ichans]
                nu_fit = guess_fit_freq(freqs, SNRs)
                rot_port = rotate_data(port, 0.0, DM_guess, P, freqs, nu_fit)
                phase_guess = fit_phase_shift(
                    np.average(rot_port, axis=0,
                               weights=data.weights[isub, ichans]),
                    model.mean(axis=0), Ns=nbin)["phase"]
                if len(freqs) > 1:
                    flags = [1, int(bool(fit_dm)), 0, 0, 0]
                    r = fit_portrait_full(port, model,
                                          [phase_guess, DM_guess, 0.0, 0.0,
                                           0.0], P, freqs, [nu_fit] * 3,
                                          [None] * 3, errs, flags,
                                          log10_tau=False)
                    phase, DM, nu_ref = r["phi"], r["DM"], r["nu_DM"]
                    scales = r["scales"]
                else:
                    r = fit_phase_shift(port[0], model[0], errs[0], Ns=nbin)
                    phase, DM, nu_ref = r["phase"], data.DM, freqs[0]
                    scales = np.array([r["scale"]])
                weights = np.outer(scales / errs ** 2, np.ones(nbin))
                for ipol in range(npol):
                    aligned_port[ipol, model_ichans] += weights * rotate_data(
                        data.subints[isub, ipol, ichans], phase, DM, P, freqs,
                        nu_ref)
                total_weights[model_ichans] += weights
        good = np.where(total_weights > 0)[0]
        for ipol in range(npol):
            aligned_port[ipol, good] /= total_weights[good]
        model_port = aligned_port[0]
    return aligned_port, total_weights


# ---------------------------------------------------------------------------
# GetTOAs.get_channels_to_zap (pptoas.py:1266-1343): per-channel reduced chi^2
# of the rotated data against the scaled model (show_fit, pptoas.py:1375-1480;
# get_red_chi2, pplib.py:754-779), then the S/N / chi^2 selection.
# ---------------------------------------------------------------------------
def channel_red_chi2s(rows, phases, model_rows, scales, errs, dof):
    """rows / model_rows [n, nbin]; phases, scales, errs [n].  Row r:
    sum((rotate(rows[r], phases[r]) - scales[r] model_rows[r]) / errs[r])^2
    / dof, with the rotation of rotate_portrait_full (pptoaslib.py:61-90)."""
    rot = rotate_rows(np.asarray(rows, dtype=np.float64), phases)
    res = rot - np.asarray(scales)[:, None] * np.asarray(model_rows)
    return np.sum((res / np.asarray(errs)[:, None]) ** 2, axis=-1) / dof


def select_zap_channels(red_chi2s, ok_ichans, channel_snrs, SNR_threshold,
                        rchi2_threshold, iterate):
    """pptoas.py:1296-1333 for one sub-integration: red_chi2s per ok channel
    (same order as ok_ichans); channel_snrs indexed by absolute channel.
    Returns the bad channel list in the reference's append order."""
    nchx = len(ok_ichans)
    thr = (SNR_threshold ** 2.0 / nchx) ** 0.5
    bad = []
    for ichan, c in zip(ok_ichans, red_chi2s):
        if c > rchi2_threshold or np.isnan(c):
            bad.append(ichan)
        elif SNR_threshold and channel_snrs[ichan] < thr:
            bad.append(ichan)
    if iterate and SNR_threshold and len(bad):
        old = len(bad)
        added = True
        while added and (nchx - len(bad)):
            thr = (SNR_threshold ** 2.0 / (nchx - len(bad))) ** 0.5
            for ichan in ok_ichans:
                if ichan in bad:
                    continue
                if channel_snrs[ichan] < thr:
                    bad.append(ichan)
            added = bool(len(bad) - old)
            old = len(bad)
    return bad


# ---------------------------------------------------------------------------
# Gaussian-component model portraits (the checker of ppf_gauss_portrait_batch)
# ---------------------------------------------------------------------------
def _evolve(freqs, nu_ref, value, evol, code):
    """evolve_parameter (pplib.py:1032-1084): '0' power_law_evolution
    (pplib.py:1000-1014), '1' linear_evolution (pplib.py:1017-1029)."""
    nchan = len(freqs)
    if code == "0":
        return np.exp(np.outer(np.log(freqs) - np.log(nu_ref), evol) +
                      np.outer(np.ones(nchan), np.log(value)))
    if code == "1":
        return np.outer(freqs - nu_ref, evol) + \
            np.outer(np.ones(nchan), value)
    raise KeyError(code)


def gaussian_profile(nbin, loc, wid):
    """gaussian_profile(norm=False, abs_wid=False, zeroout=True)
    (pplib.py:801-856): unit-peak wrapped Gaussian, truncated at |z| >= 20;
    the peak factor uses the wrapped bin centre at the first argmax and the
    unwrapped loc (pplib.py:847-849)."""
    if not wid > 0.0:
        return np.zeros(nbin, "d")
    sigma = wid / (2 * np.sqrt(2 * np.log(2)))
    mean = loc % 1.0
    x = get_bin_centers(nbin)
    if mean < 0.5:
        x = np.where(np.greater(x, mean + 0.5), x - 1.0, x)
    else:
        x = np.where(np.less(x, mean - 0.5), x + 1.0, x)
    zs = (x - mean) / sigma
    ok = np.compress(np.fabs(zs) < 20.0, np.arange(nbin))
    prof = np.zeros(nbin, "d")
    np.put(prof, ok, np.exp(-0.5 * np.take(zs, ok) ** 2.0) /
           (sigma * np.sqrt(2 * np.pi)))
    if np.max(abs(prof)) == 0.0:
        return prof
    imax = prof.argmax()
    z = (x[imax] - loc) / sigma
    return np.exp(-0.5 * z ** 2.0) / prof[imax] * prof


def gen_gaussian_portrait(model_code, params, scattering_index, phases, freqs,
                          nu_ref):
    """gen_gaussian_portrait (pplib.py:886-963) with join_ichans = []: per
    channel gen_gaussian_profile (pplib.py:859-883, DC then components in
    order), then the scattering convolution by scattering_portrait_FT
    (pplib.py:951-957, 4245-4260; complex128 where the reference's
    'complex_' alias no longer exists)."""
    params = np.asarray(params, dtype=float)
    tau = params[1]
    nbin, nchan = len(phases), len(freqs)
    freqs = np.asarray(freqs, dtype=float)
    L = _evolve(freqs, nu_ref, params[2::6], params[3::6], model_code[0])
    W = _evolve(freqs, nu_ref, params[4::6], params[5::6], model_code[1])
    A = _evolve(freqs, nu_ref, params[6::6], params[7::6], model_code[2])
    port = np.empty([nchan, nbin])
    for ichan in range(nchan):
        prof = np.zeros(nbin, dtype="d") + params[0]
        for ig in range(L.shape[1]):
            prof += A[ichan, ig] * gaussian_profile(nbin, L[ichan, ig],
                                                    W[ichan, ig])
        port[ichan] = prof
    if tau != 0.0:
        taus = float(tau) / nbin * (freqs / nu_ref) ** scattering_index
        nharm = nbin // 2 + 1
        B = np.ones([nchan, nharm], dtype=np.complex128)
        k = np.arange(nharm)
        for ichan in range(nchan):
            if taus[ichan] != 0.0:
                B[ichan] = (1.0 + 2 * np.pi * 1.0j * k * taus[ichan]) ** -1
        port = np.fft.irfft(B * np.fft.rfft(port, axis=-1), axis=-1)
    return port

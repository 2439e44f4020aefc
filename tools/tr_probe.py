"""CPU probe: evaluations per scattering fit of scipy's trust-ncg (the
reference's minimiser, pptoaslib.py:1055-1060, run through the oracle's
objective) against the Newton trust region of the device solver
(ppf_solve.hip tr_update_newton, restated here in NumPy), and how far apart
their end points are in units of the fit's own uncertainties.

    python tools/tr_probe.py c3s 8      # 128 x 1024, phi+DM+GM+tau+alpha
    python tools/tr_probe.py c3 3       # 512 x 2048 (configs[2] shape)
    python tools/tr_probe.py c5 4       # 1024 x 1024, 400-800 MHz, phi+DM+tau+alpha
    python tools/tr_probe.py c5big 3    # 4096 x 1024, same band
    python tools/tr_probe.py c3n 6      # 128 x 1024 at low S/N

Test infrastructure (imports the oracle); nothing here is on the product
path.  Round-3 numbers: DESIGN.md section 4.
"""
import os
import sys

import numpy as np
import scipy.optimize as opt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import synth_np as SN  # noqa: E402
import oracle.ppfit_oracle as O  # noqa: E402

DCONST = 1.0 / 0.000241
R0, TOL = 10.0, float(os.environ.get("TR_TOL", "1e-12"))   # kNewtonR0, kNewtonTol (ppf_internal.hpp)


def make(nchan, nbin, tau, nu_tau, lo, bw, seed, noise=1.5, alpha=-4.0):
    """A scattered sub-int of the example template and the GetTOAs-style
    start (phase near the truth, stored DM, log10 tau = log10(1/nbin),
    alpha = -4; pptoas.py:467-492)."""
    model, freqs = SN.template(nchan, nbin, lo, bw)
    P = 1 / 345.67890123456789
    rng = np.random.default_rng(seed)
    k = np.arange(nbin // 2 + 1)
    B = 1 / (1 + 2j * np.pi * np.outer(tau * (freqs / nu_tau) ** alpha, k))
    phi0, dm0 = rng.uniform(-0.5, 0.5), 34.56789 + rng.normal(3e-4, 2e-4)
    ph = phi0 + DCONST * dm0 * (freqs ** -2 - 1500.0 ** -2) / P
    data = np.fft.irfft(np.fft.rfft(model, axis=-1) * B *
                        np.exp(-2j * np.pi * np.outer(ph, k)), n=nbin, axis=-1)
    data = (data + rng.normal(0, noise, data.shape)).astype(np.float32)
    data = data.astype(float)
    nu_fit = O.guess_fit_freq(freqs)
    phs = phi0 + DCONST * dm0 * (nu_fit ** -2 - 1500.0 ** -2) / P
    x0 = np.array([((phs + 0.5) % 1) - 0.5 + rng.normal(0, 2e-3), 34.56789,
                   0.0, np.log10(1.0 / nbin), -4.0])
    Dft, Mft = O._spectra(data, model)
    eFT = O.noise_ps(data) * np.sqrt(nbin / 2.0)
    return (Dft, Mft, eFT, P, freqs, nu_fit, nu_fit, nu_fit, True), x0


def tr_exact(g, H, R):
    """min g.p + p.H p / 2, |p| <= R (eigendecomposition + secular equation;
    the device's tr_exact)."""
    lam, Q = np.linalg.eigh(H)
    gp = Q.T @ g
    if lam[0] > 0 and np.linalg.norm(gp / lam) <= R:
        return Q @ (-gp / lam), False
    lo = max(0.0, -lam[0])
    sh = lam + lo
    if lam[0] <= 0:
        sh[0] = 0.0
    if lam[0] <= 0 and abs(gp[0]) <= 1e-10 * np.linalg.norm(gp):
        q = np.where(sh > 0, gp / np.where(sh > 0, sh, 1), 0.0)
        q[0] = 0.0
        if q @ q < R * R:
            q[0] = -np.sqrt(R * R - q @ q)
            return -(Q @ q), True
    e = max(abs(gp[0]) / R, np.linalg.norm(g) / R - lam[-1] - lo, 1e-300)
    for _ in range(100):
        q = gp / (sh + e)
        n2, w = q @ q, np.sum(q * q / (sh + e))
        nq = np.sqrt(n2)
        if abs(nq - R) <= 1e-13 * R or not w > 0:
            break
        en = e + (n2 / w) * (nq - R) / R
        en = en if en > 0 else 0.5 * e
        if en == e:
            break
        e = en
    q = gp / (sh + e)
    if q @ q > R * R:
        q *= R / np.sqrt(q @ q)
    return -(Q @ q), True


def newton_tr(fgh, x0, flags, maxit=1000):
    idx = np.where(flags)[0]
    x = x0.copy()
    f, g, H = fgh(x)
    nfev, r = 1, R0
    for _ in range(maxit):
        d = np.sqrt(np.maximum(np.abs(np.diag(H[np.ix_(idx, idx)])), 1e-300))
        gs, Hs = g[idx] / d, H[np.ix_(idx, idx)] / np.outer(d, d)
        p, hb = tr_exact(gs, Hs, r)
        pred = -(gs @ p + 0.5 * p @ Hs @ p)
        if not pred > TOL:
            break
        xn = x.copy()
        xn[idx] += p / d
        fn, gn, Hn = fgh(xn)
        nfev += 1
        rho = (f - fn) / pred
        if rho < 0.25:
            r = 0.25 * np.linalg.norm(p)
        elif rho > 0.75 and hb:
            r = min(4 * r, 1e6)
        if rho > 0.15:
            x, f, g, H = xn, fn, gn, Hn
    return x, f, nfev


def subset_newton(args, x0, flags, stride, switch=1.0, maxit=1000):
    """newton_tr with the device's channel-subset warm start (every
    stride-th group of 64 channels until an interior step predicts less than
    `switch`, then every channel from the accepted point); returns (x, f,
    cost in full-evaluation equivalents)."""
    Dft, Mft, eFT, P, fr, n1, n2, n3, lt = args
    nchan = Dft.shape[0]
    sel = np.where((np.arange(nchan) // 64) % stride == 0)[0]
    frac = len(sel) / nchan
    sub_args = (Dft[sel], Mft[sel], eFT[sel], P, fr[sel], n1, n2, n3, lt)

    def fgh_of(a):
        def fgh(x):
            t = O.channel_terms(np.asarray(x, float), *a)
            return O.objective(t), O.gradient(t, flags), O.hessian(t, flags)
        return fgh
    full, part = fgh_of(args), fgh_of(sub_args)
    idx = np.where(flags)[0]
    insub = stride > 1
    cur = part if insub else full
    x = x0.copy()
    f, g, H = cur(x)
    cost, r = (frac if insub else 1.0), R0
    for _ in range(maxit):
        d = np.sqrt(np.maximum(np.abs(np.diag(H[np.ix_(idx, idx)])), 1e-300))
        gs, Hs = g[idx] / d, H[np.ix_(idx, idx)] / np.outer(d, d)
        p, hb = tr_exact(gs, Hs, r)
        pred = -(gs @ p + 0.5 * p @ Hs @ p)
        if insub and ((not hb and pred < switch) or not pred > TOL):
            insub, cur = False, full
            f, g, H = cur(x)
            cost += 1.0
            continue
        if not pred > TOL:
            break
        xn = x.copy()
        xn[idx] += p / d
        fn, gn, Hn = cur(xn)
        cost += frac if insub else 1.0
        rho = (f - fn) / pred
        if rho < 0.25:
            r = 0.25 * np.linalg.norm(p)
        elif rho > 0.75 and hb:
            r = min(4 * r, 1e6)
        if rho > 0.15:
            x, f, g, H = xn, fn, gn, Hn
    return x, f, cost


def compare(args, x0, flags):
    def fgh(x):
        t = O.channel_terms(np.asarray(x, float), *args)
        return O.objective(t), O.gradient(t, flags), O.hessian(t, flags)
    ref = opt.minimize(lambda x: fgh(x)[0], x0, method="trust-ncg",
                       jac=lambda x: fgh(x)[1], hess=lambda x: fgh(x)[2],
                       options={"gtol": -1})
    idx = np.where(flags)[0]
    H = fgh(ref.x)[2][np.ix_(idx, idx)]
    sig = np.sqrt(np.diag(np.linalg.inv(0.5 * H)))
    x, f, n = newton_tr(fgh, x0, flags)
    ng = (args[0].shape[0] + 63) // 64
    stride = 1
    while stride * 2 <= 16 and stride * 2 <= ng // 2:
        stride *= 2
    xs, fs, cost = subset_newton(args, x0, flags, stride)
    return (ref.nfev, n, np.max(np.abs((x - ref.x)[idx] / sig)), f - ref.fun,
            cost, np.max(np.abs((xs - ref.x)[idx] / sig)))


CASES = {
    "c3s": (dict(nchan=128, nbin=1024, tau=2e-3, nu_tau=1500., lo=1100.,
                 bw=800.), [1, 1, 1, 1, 1]),
    "c3": (dict(nchan=512, nbin=2048, tau=2e-3, nu_tau=1500., lo=1100.,
                bw=800.), [1, 1, 1, 1, 1]),
    "c3n": (dict(nchan=128, nbin=1024, tau=2e-3, nu_tau=1500., lo=1100.,
                 bw=800., noise=15.0), [1, 1, 1, 1, 1]),
    "c5": (dict(nchan=1024, nbin=1024, tau=5e-3, nu_tau=600., lo=400.,
                bw=400.), [1, 1, 0, 1, 1]),
    "c5big": (dict(nchan=4096, nbin=1024, tau=5e-3, nu_tau=600., lo=400.,
                   bw=400.), [1, 1, 0, 1, 1]),
}

if __name__ == "__main__":
    kw, flags = CASES[sys.argv[1]]
    with np.errstate(all="ignore"):
        for seed in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
            a, x0 = make(seed=seed, **kw)
            nr, nn, dev, df, cost, dev_s = compare(a, x0, flags)
            print("seed %d: scipy trust-ncg %3d evaluations, Newton TR %3d; "
                  "end points %.1e sigma apart, objective %+.1e; with the "
                  "channel-subset warm start %.2f full-evaluation "
                  "equivalents, %.1e sigma from scipy's" %
                  (seed, nr, nn, dev, df, cost, dev_s), flush=True)

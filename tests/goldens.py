"""Loaders for the golden vectors in tests/golden/ (produced by make_golden.py
from the reference itself; see that script's header)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Parity bar (BASELINE.json north_star): fitted parameters within 0.01 sigma of
# the reference's own reported uncertainty, chi2_red within 1e-8 relative.
SIGMA_TOL = 0.01
RCHI2_RTOL = 1e-8

PARAM_NAMES = ("phi", "DM", "GM", "tau", "alpha")


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def case_names(fname):
    z = _load(fname)
    return sorted(set(k.split("/")[0] for k in z.files))


class Case(dict):
    __getattr__ = dict.__getitem__


def load_case(fname, name):
    z = _load(fname)
    out = Case()
    for k in z.files:
        if k.startswith(name + "/"):
            v = z[k]
            out[k[len(name) + 1:]] = v[()] if v.shape == () else v
    return out


def full_case(name):
    return load_case("fit_portrait_full.npz", name)


def fp_case(name):
    return load_case("fit_portrait.npz", name)


def misc():
    z = _load("misc.npz")
    return Case({k: z[k] for k in z.files})


def gettoas():
    z = _load("get_toas.npz")
    return Case({k: z[k] for k in z.files})


def full_case_args(c):
    """Positional/keyword arguments of fit_portrait_full for a golden case."""
    errs = None if np.all(np.isnan(c["errs"])) else c["errs"]
    nu_outs = [None if np.isnan(v) else float(v) for v in c["nu_outs"]]
    return dict(data_port=c["data"].astype(np.float64),
                model_port=c["model"].astype(np.float64),
                init_params=list(c["init"]), P=float(c["P"]),
                freqs=c["freqs"], nu_fits=list(c["nu_fits"]),
                nu_outs=nu_outs, errs=errs,
                fit_flags=[int(x) for x in c["flags"]],
                log10_tau=bool(c["log10_tau"]), option=int(c["option"]))


def phase_diff(a, b):
    """Difference of two phases modulo 1, in [-0.5, 0.5)."""
    d = (np.asarray(a) - np.asarray(b) + 0.5) % 1.0 - 0.5
    return d


DCONST = 0.000241 ** -1


def to_reference_frequencies(got, ref, P, log10_tau):
    """Re-express ``got``'s phase and scattering time at ``ref``'s output
    reference frequencies: phi moves with the fitted
    DM/GM (phase_transform semantics, pplib.py:2688-2712, plus the nu**-4
    term), tau with the fitted alpha (pptoaslib.py:1107-1113)."""
    phi, DM, GM, tau, alpha = (float(v) for v in got["params"])
    phi = (phi + DCONST * DM / P * (ref["nu_DM"] ** -2 - got["nu_DM"] ** -2) +
           DCONST ** 2 * GM / P * (ref["nu_GM"] ** -4 - got["nu_GM"] ** -4))
    if log10_tau:
        tau = tau + alpha * np.log10(ref["nu_tau"] / got["nu_tau"])
    else:
        tau = tau * (ref["nu_tau"] / got["nu_tau"]) ** alpha
    return [phi, DM, GM, tau, alpha]


def param_deviation_sigma(got, ref, P=None, log10_tau=False):
    """|got - ref| / ref_err per parameter (phase mod 1), after moving got to
    ref's reference frequencies when both carry nu_DM/nu_GM/nu_tau.

    Returns an array of 5 deviations (0 where the parameter is not fit)."""
    if P is not None and "nu_DM" in got and "nu_DM" in ref:
        gp = np.asarray(to_reference_frequencies(got, ref, P, log10_tau))
    else:
        gp = np.asarray(got["params"], float)
    rp = np.asarray(ref["params"], float)
    re = np.asarray(ref["param_errs"], float)
    dev = np.zeros(5)
    for i in range(5):
        if re[i] == 0:
            continue
        d = phase_diff(gp[i], rp[i]) if i == 0 else gp[i] - rp[i]
        dev[i] = abs(d) / re[i]
    return dev


def ref_bunch(c):
    """The reference's DataBunch fields of a golden fit_portrait_full case."""
    return dict(params=c["out_params"], param_errs=c["out_param_errs"],
                nu_DM=float(c["out_nu_DM"]), nu_GM=float(c["out_nu_GM"]),
                nu_tau=float(c["out_nu_tau"]))


class Bunch(dict):
    """DataBunch stand-in (attribute access), as pplib.DataBunch."""
    __getattr__ = dict.__getitem__


def align():
    z = _load("align.npz")
    return Case({k: z[k] for k in z.files})


def align_inputs(c=None):
    """(archives, model_data) of the ppalign golden case, rebuilt exactly as
    tests/golden/make_golden_align.py handed them to the reference."""
    c = align() if c is None else c
    nfile, nsub = int(c["nfile"]), int(c["nsub"])
    nchan, nbin = int(c["nchan"]), int(c["nbin"])
    freqs = c["freqs"]
    P, DM0 = float(c["P"]), float(c["DM0"])
    archives = []
    for i in range(nfile):
        sub = c["f%d_subints" % i].astype(np.float64)[:, None]
        w = c["f%d_weights" % i]
        wnorm = np.where(w == 0.0, 0.0, 1.0)
        archives.append(Bunch(
            DM=DM0, dmc=0, freqs=np.tile(freqs, (nsub, 1)),
            masks=np.einsum("ij,k", wnorm, np.ones(nbin))[:, None],
            nbin=nbin, nchan=nchan,
            noise_stds=c["f%d_noise" % i][:, None], npol=1, nsub=nsub,
            ok_ichans=[np.compress(wnorm[j], list(range(nchan)))
                       for j in range(nsub)],
            ok_isubs=np.arange(nsub), prof_SNR=100.0,
            Ps=np.ones(nsub) * P, SNRs=c["f%d_snrs" % i][:, None],
            subints=sub, weights=w, state="Intensity"))
    model_data = Bunch(
        DM=0.0, dmc=1, freqs=freqs[None, :], masks=np.ones([1, 1, nchan, nbin]),
        nbin=nbin, nchan=nchan, noise_stds=np.ones([1, 1, nchan]), npol=1,
        nsub=1, ok_ichans=[np.arange(nchan)], ok_isubs=np.arange(1),
        prof_SNR=100.0, Ps=np.ones(1) * P, SNRs=np.ones([1, 1, nchan]),
        subints=c["guess"][None, None], weights=np.ones([1, nchan]),
        arch=None, state="Intensity")
    return archives, model_data


def narrowband():
    z = _load("narrowband.npz")
    return Case({k: z[k] for k in z.files})


def narrowband_opts():
    """tests/golden/narrowband_opts.npz (make_golden_nb_opts.py)."""
    z = _load("narrowband_opts.npz")
    return Case({k: z[k] for k in z.files})


def zap():
    """tests/golden/zap.npz (make_golden_zap.py) plus the reference's ragged
    get_channels_to_zap outputs unflattened to [call][file][sub] lists."""
    z = _load("zap.npz")
    c = Case({k: z[k] for k in z.files})
    nfile, nsub = int(c["nfile"]), int(c["nsub"])
    ncall = len(c["calls"])
    chi, zp = [], []
    ic = iz = j = 0
    for _ in range(ncall):
        cc, zz = [], []
        for _ in range(nfile):
            cs, zs = [], []
            for _ in range(nsub):
                n, m = int(c["out_chi2_n"][j]), int(c["out_zap_n"][j])
                cs.append(c["out_chi2"][ic:ic + n])
                zs.append([int(v) for v in c["out_zap"][iz:iz + m]])
                ic, iz, j = ic + n, iz + m, j + 1
            cc.append(cs)
            zz.append(zs)
        chi.append(cc)
        zp.append(zz)
    c["chi2"], c["zap"] = chi, zp
    return c


def gauss():
    """tests/golden/gauss.npz (make_golden_gauss.py): the reference's
    gen_gaussian_portrait / gaussian_profile / read_model outputs."""
    z = _load("gauss.npz")
    return Case({k: z[k] for k in z.files})


def gauss_case(g, name):
    return dict(code=str(g[name + "__code"]), params=g[name + "__params"],
                alpha=float(g[name + "__alpha"]),
                nu_ref=float(g[name + "__nu_ref"]),
                freqs=g[name + "__freqs"], out=g[name + "__out"])

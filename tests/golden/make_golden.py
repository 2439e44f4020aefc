#!/usr/bin/env python
"""Generate golden input/output vectors by running the REFERENCE implementation.

Runs ONLY in the build container, where /root/reference (PulsePortraiture,
read-only) is importable through three small import shims kept in
tests/golden/refshim/ (``past.utils.old_div``, a PSRCHIVE ``MJD`` stand-in) plus
a NumPy-2 compatible rebinding of ``scattering_portrait_FT`` (the reference
uses the removed ``'complex_'`` dtype alias at pplib.py:4253; the replacement
below is numerically identical and only used when some tau_n != 0).

Nothing here travels to the GPU box: tests read only the .npz files written
next to this script.  Inputs (data and model portraits) are rounded to float32
BEFORE the reference sees them, so the device path (which stores float32
amplitudes, as PSRCHIVE does) and the reference consume bit-identical inputs.

Usage:  python tests/golden/make_golden.py [--quick]
"""
import io
import json
import os
import sys
import time
import contextlib

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, "refshim"), REF]
os.environ.setdefault("MPLBACKEND", "Agg")

import numpy as np  # noqa: E402

with contextlib.redirect_stdout(io.StringIO()):
    import pplib  # noqa: E402
    import pptoaslib  # noqa: E402
    import pptoas  # noqa: E402


def _scattering_portrait_FT(taus, nbin, binshift=1.0):
    # NumPy>=2 stand-in for pplib.scattering_portrait_FT (pplib.py:4245-4260):
    # identical arithmetic, dtype complex128 instead of the removed 'complex_'.
    nchan = len(taus)
    nharm = nbin // 2 + 1
    if not np.any(taus):
        return np.ones([nchan, nharm])
    out = np.zeros([nchan, nharm], dtype=np.complex128)
    for ichan in range(nchan):
        out[ichan] = pplib.scattering_profile_FT(taus[ichan], nbin, binshift)
    return out


for _mod in (pplib, pptoaslib, pptoas):
    _mod.scattering_portrait_FT = _scattering_portrait_FT

GMODEL = os.path.join(REF, "examples", "example.gmodel")
P0 = 1.0 / 345.67890123456789          # examples/example.par F0
DM0 = 34.56789                          # examples/example.par DM


def channel_freqs(nchan, lo=1100.0, bw=800.0):
    cw = bw / nchan
    return np.linspace(lo + cw / 2, lo + bw - cw / 2, nchan)


def f32(x):
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def make_portrait(rng, nchan, nbin, phi, DM, P, nu0=1500.0, lo=1100.0,
                  bw=800.0, noise=1.5, tau_ref=0.0, alpha=-4.0, nu_tau=1500.0,
                  GM=0.0):
    """Synthetic sub-integration: model rotated by (-phi, -DM[, -GM]), optional
    scattering, white noise.  Returns fp32-rounded (data, model, freqs)."""
    freqs = channel_freqs(nchan, lo, bw)
    phases = pplib.get_bin_centers(nbin)
    with contextlib.redirect_stdout(io.StringIO()):
        _, _, model = pplib.read_model(GMODEL, phases, freqs, P, quiet=True)
    model = f32(model)
    port = pptoaslib.rotate_portrait_full(model, -phi, -DM, -GM, freqs, nu0,
                                          nu0, P)
    if tau_ref:
        taus = pplib.scattering_times(tau_ref, alpha, freqs, nu_tau)
        port = np.fft.irfft(_scattering_portrait_FT(taus, nbin) *
                            np.fft.rfft(port, axis=-1), axis=-1)
    port = port + rng.normal(0.0, noise, port.shape)
    return f32(port), model, freqs


def databunch_to_dict(res, prefix=""):
    out = {}
    for k, v in res.items():
        if v is None:
            continue
        out[prefix + k] = np.asarray(v, dtype=np.float64)
    return out


# ---------------------------------------------------------------------------
# fit_portrait_full cases
# ---------------------------------------------------------------------------
FULL_CASES = [
    # name, nchan, nbin, fit_flags, log10_tau, extra
    dict(name="pd_64x512", nchan=64, nbin=512, flags=[1, 1, 0, 0, 0], seed=1,
         errs_none=True),
    dict(name="pd_128x1024", nchan=128, nbin=1024, flags=[1, 1, 0, 0, 0],
         seed=2),
    dict(name="pd_512x2048", nchan=512, nbin=2048, flags=[1, 1, 0, 0, 0],
         seed=3, big=True),
    dict(name="pd_nuout_64x512", nchan=64, nbin=512, flags=[1, 1, 0, 0, 0],
         seed=4, nu_outs=[1400.0, 1400.0, 1400.0]),
    dict(name="p_1chan", nchan=1, nbin=512, flags=[1, 0, 0, 0, 0], seed=5),
    dict(name="pd_2chan", nchan=2, nbin=512, flags=[1, 1, 0, 0, 0], seed=6),
    dict(name="pdg_64x512", nchan=64, nbin=512, flags=[1, 1, 1, 0, 0], seed=7),
    dict(name="pdg_opt1_64x512", nchan=64, nbin=512, flags=[1, 1, 1, 0, 0],
         seed=8, option=1),
    dict(name="pg_64x512", nchan=64, nbin=512, flags=[1, 0, 1, 0, 0], seed=9),
    dict(name="pdta_64x512", nchan=64, nbin=512, flags=[1, 1, 0, 1, 1],
         seed=10, scat=True),
    dict(name="pdt_64x512", nchan=64, nbin=512, flags=[1, 1, 0, 1, 0],
         seed=11, scat=True),
    dict(name="all_64x512", nchan=64, nbin=512, flags=[1, 1, 1, 1, 1],
         seed=12, scat=True),
    dict(name="pdgt_64x512", nchan=64, nbin=512, flags=[1, 1, 1, 1, 0],
         seed=13, scat=True),
    dict(name="pdgt_opt1_64x512", nchan=64, nbin=512, flags=[1, 1, 1, 1, 0],
         seed=14, scat=True, option=1),
    dict(name="ta_64x512", nchan=64, nbin=512, flags=[0, 0, 0, 1, 1],
         seed=15, scat=True),
    dict(name="pdta_lin_64x512", nchan=64, nbin=512, flags=[1, 1, 0, 1, 1],
         seed=16, scat=True, log10_tau=False),
    dict(name="pdta_128x1024", nchan=128, nbin=1024, flags=[1, 1, 0, 1, 1],
         seed=17, scat=True),
    dict(name="pd_fixedtau_64x512", nchan=64, nbin=512, flags=[1, 1, 0, 0, 0],
         seed=18, scat=True, fixed_tau=True),
]


def run_full_case(c):
    rng = np.random.default_rng(20250217 + c["seed"])
    nchan, nbin = c["nchan"], c["nbin"]
    phi_true = rng.uniform(-0.5, 0.5)
    dDM = rng.normal(3e-4, 2e-4)
    P = P0 * (1.0 + 1e-6 * rng.normal())
    scat = c.get("scat", False)
    tau_ref = 2e-3 if scat else 0.0        # [rot] at 1500 MHz
    data, model, freqs = make_portrait(rng, nchan, nbin, phi_true,
                                       DM0 + dDM, P, tau_ref=tau_ref)
    nu_fit = float(pplib.guess_fit_freq(freqs))
    # initial guesses as GetTOAs would form them (pptoas.py:461-502), but with
    # the guess phase perturbed from truth instead of the brute-force FFTFIT
    phi_guess = pplib.phase_transform(phi_true + rng.normal(0, 2e-3), DM0,
                                      1500.0, nu_fit, P, mod=True)
    log10_tau = c.get("log10_tau", True)
    flags = list(c["flags"])
    if scat:
        tau_g = 1.0 / nbin if not c.get("fixed_tau") else \
            tau_ref * (nu_fit / 1500.0) ** -4.0
        tau_g_par = np.log10(tau_g) if log10_tau else tau_g
        alpha_g = -4.0
    else:
        tau_g_par, alpha_g = 0.0, 0.0
        log10_tau = c.get("log10_tau", False)
    if c.get("fixed_tau"):
        log10_tau = True
        tau_g_par = np.log10(tau_ref * (nu_fit / 1500.0) ** -4.0)
    init = [float(phi_guess), DM0, 0.0, float(tau_g_par), alpha_g]
    errs = None if c.get("errs_none") else pplib.get_noise(data, chans=True)
    nu_fits = [nu_fit, nu_fit, nu_fit]
    nu_outs = c.get("nu_outs", [None, None, None])
    t0 = time.time()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        res = pptoaslib.fit_portrait_full(
            data, model, init, P, freqs, nu_fits, nu_outs, errs, flags,
            log10_tau=log10_tau, option=c.get("option", 0), is_toa=True,
            quiet=True)
    dt = time.time() - t0
    out = dict(data=data.astype(np.float32), model=model.astype(np.float32),
               freqs=freqs, P=np.float64(P), init=np.array(init),
               flags=np.array(flags), nu_fits=np.array(nu_fits),
               nu_outs=np.array([np.nan if v is None else v for v in nu_outs]),
               log10_tau=np.int64(log10_tau),
               option=np.int64(c.get("option", 0)),
               errs=(np.full(nchan, np.nan) if errs is None else errs),
               truth=np.array([phi_true, DM0 + dDM, 0.0, tau_ref, -4.0]),
               ref_seconds=np.float64(dt),
               stdout=np.array(buf.getvalue()))
    out.update(databunch_to_dict(res, "out_"))
    return out


# ---------------------------------------------------------------------------
# pplib.fit_portrait (legacy, TNC) cases
# ---------------------------------------------------------------------------
FP_CASES = [dict(name="fp_64x512", nchan=64, nbin=512, seed=31),
            dict(name="fp_256x1024", nchan=256, nbin=1024, seed=32,
                 errs_given=True)]


def run_fp_case(c):
    rng = np.random.default_rng(20250217 + c["seed"])
    nchan, nbin = c["nchan"], c["nbin"]
    phi_true = rng.uniform(-0.5, 0.5)
    dDM = rng.normal(3e-4, 2e-4)
    P = P0
    data, model, freqs = make_portrait(rng, nchan, nbin, phi_true, DM0 + dDM, P)
    nu_fit = float(freqs.mean())
    phi_guess = pplib.phase_transform(phi_true + rng.normal(0, 2e-3), DM0,
                                      1500.0, nu_fit, P, mod=True)
    errs = pplib.get_noise(data, chans=True) if c.get("errs_given") else None
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        res = pplib.fit_portrait(data, model, np.array([phi_guess, DM0]), P,
                                 freqs, None, None, errs)
    dt = time.time() - t0
    out = dict(data=data.astype(np.float32), model=model.astype(np.float32),
               freqs=freqs, P=np.float64(P), init=np.array([phi_guess, DM0]),
               errs=(np.full(nchan, np.nan) if errs is None else errs),
               ref_seconds=np.float64(dt))
    out.update(databunch_to_dict(res, "out_"))
    return out


# ---------------------------------------------------------------------------
# rotate_data / rotate_portrait / get_noise / fit_phase_shift
# ---------------------------------------------------------------------------
def run_misc():
    rng = np.random.default_rng(777)
    out = {}
    nbin = 512
    prof = f32(rng.normal(size=nbin))
    port = f32(rng.normal(size=(16, nbin)))
    cube = f32(rng.normal(size=(3, 2, 16, nbin)))
    freqs = channel_freqs(16)
    freqs2 = np.tile(freqs, (3, 1)) * (1 + 1e-4 * np.arange(3))[:, None]
    Ps = P0 * (1 + 1e-3 * np.arange(3))
    out["rot_prof"] = prof
    out["rot_port"] = port
    out["rot_cube"] = cube
    out["rot_freqs"] = freqs
    out["rot_freqs2"] = freqs2
    out["rot_Ps"] = Ps
    out["rot1_dm0"] = pplib.rotate_data(prof, 0.123)
    out["rot2_dm0"] = pplib.rotate_data(port, -0.377)
    out["rot4_dm0"] = pplib.rotate_data(cube, 0.05)
    out["rot1_dm"] = pplib.rotate_data(prof, 0.1, 10.0, P0, 1300.0, 1500.0)
    out["rot2_dm"] = pplib.rotate_data(port, 0.2, 34.5, P0, freqs, 1500.0)
    out["rot4_dm"] = pplib.rotate_data(cube, -0.3, 12.5, Ps, freqs, 1400.0)
    out["rot4_dm_f2"] = pplib.rotate_data(cube, 0.01, 5.0, Ps, freqs2,
                                          np.inf)
    out["rotp_dm"] = pplib.rotate_portrait(port, 0.25, 20.0, P0, freqs, 1450.0)
    out["rotp_nodm"] = pplib.rotate_portrait(port, -0.125)
    out["rotf_dmgm"] = pptoaslib.rotate_portrait_full(port, 0.1, 3.0, 2.0,
                                                      freqs, 1500., 1600., P0)
    # noise
    out["noise_port"] = pplib.get_noise(port, chans=True)
    out["noise_prof"] = pplib.get_noise(prof)
    for nb in (256, 1000, 2048):
        x = f32(rng.normal(size=(4, nb)) * 2.0)
        out["noise_in_%d" % nb] = x
        out["noise_out_%d" % nb] = pplib.get_noise(x, chans=True)
    # fit_phase_shift
    with contextlib.redirect_stdout(io.StringIO()):
        _, _, model = pplib.read_model(GMODEL, pplib.get_bin_centers(1024),
                                       channel_freqs(8), P0, quiet=True)
    mprof = f32(model.mean(axis=0))
    fps = []
    for i in range(6):
        shift = rng.uniform(-0.5, 0.5)
        d = f32(pplib.rotate_data(mprof, -shift) * rng.uniform(0.5, 3.0) +
                rng.normal(0, 0.3 + 0.5 * i, 1024))
        ns = [100, 100, 50, 1024, 100, 100][i]
        noise = None if i % 2 == 0 else 0.4
        r = pplib.fit_phase_shift(d, mprof, noise=noise, Ns=ns)
        fps.append(np.concatenate([d, [shift, ns, np.nan if noise is None
                                       else noise, r.phase, r.phase_err,
                                       r.scale, r.scale_err, r.snr,
                                       r.red_chi2]]))
    out["fps_model"] = mprof
    out["fps_rows"] = np.array(fps)
    # misc host helpers
    out["gff_freqs"] = freqs
    out["gff_snrs"] = np.abs(rng.normal(size=16)) * 10
    out["gff_out"] = np.array([pplib.guess_fit_freq(freqs, out["gff_snrs"]),
                               pplib.guess_fit_freq(freqs)])
    return out


# ---------------------------------------------------------------------------
# GetTOAs.get_TOAs end to end (load_data replaced by a synthetic loader)
# ---------------------------------------------------------------------------
def run_gettoas(nfile=2, nsub=6, nchan=64, nbin=512):
    from pplib import DataBunch
    import psrchive as pr
    rng = np.random.default_rng(4242)
    freqs1 = channel_freqs(nchan)
    phases = pplib.get_bin_centers(nbin)
    files = {}
    inputs = {}
    for ifile in range(nfile):
        subints = np.zeros([nsub, 1, nchan, nbin])
        truth = []
        for isub in range(nsub):
            phi = rng.uniform(-0.5, 0.5)
            ddm = rng.normal(3e-4, 2e-4)
            d, model, _ = make_portrait(rng, nchan, nbin, phi, DM0 + ddm, P0)
            subints[isub, 0] = d
            truth.append([phi, DM0 + ddm])
        weights = np.ones([nsub, nchan])
        if ifile == 1:     # zap a few channels, differently per sub-int
            for isub in range(nsub):
                weights[isub, rng.choice(nchan, 5 + isub, replace=False)] = 0
        noise = np.array([[pplib.get_noise(subints[i, 0], chans=True)]
                          for i in range(nsub)])
        snrs = np.abs(subints.max(axis=-1)) / noise * 3.0
        wnorm = np.where(weights == 0.0, 0.0, 1.0)
        ok_ichans = [np.compress(wnorm[i], list(range(nchan)))
                     for i in range(nsub)]
        dfs = 1.0 + 1e-4 * rng.normal(size=nsub)
        epochs = 57000.0 + np.arange(nsub) * 60.0 / 86400.0 + ifile
        name = "fake%d.fits" % ifile
        files[name] = DataBunch(
            arch=None, backend="fake_be", backend_delay=0.0, bw=800.0,
            doppler_factors=dfs, DM=DM0, dmc=0,
            epochs=[pr.MJD(e) for e in epochs], filename=name,
            flux_prof=np.array([]), freqs=np.tile(freqs1, (nsub, 1)),
            frontend="fake_rx", integration_length=60.0 * nsub,
            masks=np.einsum("ij,k", wnorm, np.ones(nbin))[:, None],
            nbin=nbin, nchan=nchan, noise_stds=noise, npol=1, nsub=nsub,
            nu0=1500.0, ok_ichans=ok_ichans, ok_isubs=np.arange(nsub),
            parallactic_angles=np.zeros(nsub), phases=phases, prof=None,
            prof_noise=1.0, prof_SNR=100.0, Ps=np.ones(nsub) * P0,
            SNRs=snrs, source="J1234-5678", state="Intensity",
            subints=subints, subtimes=[60.0] * nsub, telescope="GBT",
            telescope_code="1", weights=weights)
        inputs["f%d_subints" % ifile] = subints[:, 0].astype(np.float32)
        inputs["f%d_weights" % ifile] = weights
        inputs["f%d_snrs" % ifile] = snrs[:, 0]
        inputs["f%d_dfs" % ifile] = dfs
        inputs["f%d_epochs" % ifile] = epochs
        inputs["f%d_truth" % ifile] = np.array(truth)
    pptoas.load_data = lambda filename, **kw: files[filename]
    gt = pptoas.GetTOAs.__new__(pptoas.GetTOAs)
    # replicate __init__ without the `file -L` probe (pptoas.py:92-159)
    gt.datafiles = list(files.keys())
    gt.is_FITS_model = False
    gt.modelfile = GMODEL
    for attr in ["obs", "doppler_fs", "nu0s", "nu_fits", "nu_refs",
                 "ok_idatafiles", "ok_isubs", "epochs", "MJDs", "Ps", "phis",
                 "phi_errs", "TOAs", "TOA_errs", "DM0s", "DMs", "DM_errs",
                 "DeltaDM_means", "DeltaDM_errs", "GMs", "GM_errs", "taus",
                 "tau_errs", "alphas", "alpha_errs", "scales", "scale_errs",
                 "snrs", "channel_snrs", "profile_fluxes",
                 "profile_flux_errs", "fluxes", "flux_errs", "flux_freqs",
                 "red_chi2s", "channel_red_chi2s", "covariances", "nfevals",
                 "rcs", "fit_durations", "order", "TOA_list", "zap_channels"]:
        setattr(gt, attr, [])
    gt.instrumental_response_dict = gt.ird = {"DM": 0.0, "wids": [],
                                              "irf_types": []}
    gt.quiet = True
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        gt.get_TOAs(quiet=True)
    dt = time.time() - t0
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        pplib.write_TOAs(gt.TOA_list)
    out = dict(inputs)
    out.update(nfile=np.int64(nfile), nsub=np.int64(nsub),
               nchan=np.int64(nchan), nbin=np.int64(nbin), P=np.float64(P0),
               DM0=np.float64(DM0), freqs=freqs1, ref_seconds=np.float64(dt))
    for key in ["phis", "phi_errs", "DMs", "DM_errs", "red_chi2s", "snrs",
                "scales", "scale_errs", "channel_snrs", "covariances",
                "nfevals", "rcs", "DeltaDM_means", "DeltaDM_errs", "GMs",
                "taus", "alphas"]:
        out["out_" + key] = np.array(getattr(gt, key), dtype=np.float64)
    out["out_nu_refs"] = np.array(gt.nu_refs, dtype=np.float64)
    out["out_nu_fits"] = np.array(gt.nu_fits, dtype=np.float64)
    out["out_TOA_days"] = np.array([t.MJD.in_days() for t in gt.TOA_list])
    out["out_tim_lines"] = np.array(buf.getvalue().splitlines())
    return out


def main():
    quick = "--quick" in sys.argv
    manifest = {}
    full = {}
    for c in FULL_CASES:
        if quick and c.get("big"):
            continue
        t0 = time.time()
        r = run_full_case(c)
        for k, v in r.items():
            full[c["name"] + "/" + k] = v
        manifest[c["name"]] = dict(c, seconds=time.time() - t0)
        print("full", c["name"], "%.2fs" % (time.time() - t0),
              "nfev", r.get("out_nfeval"), "rc", r.get("out_return_code"))
    np.savez_compressed(os.path.join(HERE, "fit_portrait_full.npz"), **full)
    fp = {}
    for c in FP_CASES:
        r = run_fp_case(c)
        for k, v in r.items():
            fp[c["name"] + "/" + k] = v
        manifest[c["name"]] = c
        print("fp", c["name"])
    np.savez_compressed(os.path.join(HERE, "fit_portrait.npz"), **fp)
    np.savez_compressed(os.path.join(HERE, "misc.npz"), **run_misc())
    print("misc done")
    g = run_gettoas()
    np.savez_compressed(os.path.join(HERE, "get_toas.npz"), **g)
    print("get_toas done", g["ref_seconds"])
    manifest["_env"] = dict(numpy=np.__version__,
                            scipy=__import__("scipy").__version__,
                            reference="/root/reference @ 2025-02-17")
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, default=str)


if __name__ == "__main__":
    main()

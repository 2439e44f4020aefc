#!/usr/bin/env python
"""Full-shape golden vectors, produced by running the REFERENCE in this
container (never on the GPU box): the BASELINE.json configs at (or at the
per-sub-integration shape of) their named sizes.

  fits (pptoaslib.fit_portrait_full, pptoaslib.py:974-1144)
    c3_all_512x2048_{a,b}   configs[2] fit: phi, DM, GM, tau, alpha (log10 tau)
                            at 512 x 2048, injected scattering
    c3_pdta_512x2048        phi, DM, tau, alpha at 512 x 2048
    narrow_pd_512x2048      phase + DM with a narrow-component template whose
                            power reaches Nyquist (the harmonic cutoff must
                            switch itself off)
    pd_64x4096, pdta_64x128 the block-FFT fallback shapes (nbin outside the
                            wave-FFT range 256..2048)
  get_TOAs (pptoas.py:161-792, load_data replaced by synthetic DataBunches)
    c1   examples/example.py shape: 5 archives x 10 sub-ints x 64 x 512,
         scintillation, per-archive injected dDM, get_TOAs(DM0=DM0)
    c2   one archive x 8 sub-ints x 512 x 2048 (configs[1] sub-int shape)
    narrow  one archive x 4 sub-ints x 512 x 2048 with the narrow template
  align_archives (ppalign.py:65-280)
    c4   16 tscrunched archives x 256 x 1024, niter = 3, initial template =
         archive 0's mean profile tiled (configs[3])
    dup  archives whose 32 channels map two-to-one onto a 16-channel template
         (duplicate model channels)
  get_scales_full (pptoaslib.py:953-971) on a scattering golden case

Inputs are NOT stored: they are rebuilt from the stored parameters by
tests/golden/synth_np.py and checked against the stored SHA-256.

Usage:  python tests/golden/make_golden_full.py [--only NAME,...]
"""
import contextlib
import io
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))   # repo (oracle)
import make_golden as mg  # noqa: E402  (imports the reference with the shims)
import make_golden_align as mga  # noqa: E402
import numpy as np  # noqa: E402
import synth_np as S  # noqa: E402
from full_inputs import (FITS, TOAS, ALIGNS, fit_inputs,  # noqa: E402
                         toa_inputs, align_inputs, write_narrow, SPLINES,
                         SPLINE_MODEL, write_spline, write_scat, toa_gmodel,
                         archive_fields)

OUT = os.path.join(HERE, "full.npz")


def run_fit(c):
    data, model, freqs, P, truth, init, nu_fit = fit_inputs(c)
    scat = c["flags"][3] == 1
    errs = mg.pplib.get_noise(data, chans=True)
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        res = mg.pptoaslib.fit_portrait_full(
            data, model, init, P, freqs, [nu_fit] * 3, [None] * 3, errs,
            c["flags"], log10_tau=scat, option=0, is_toa=True, quiet=True)
    dt = time.time() - t0
    out = dict(sha=np.array(S.sha(data.astype(np.float32),
                                  model.astype(np.float32))),
               nchan=np.int64(c["nchan"]), nbin=np.int64(c["nbin"]),
               seed=np.int64(c["seed"]), flags=np.array(c["flags"]),
               narrow=np.int64(bool(c.get("narrow"))),
               tau=np.float64(c.get("tau", 0.0)), P=np.float64(P),
               init=np.array(init, dtype=float), nu_fit=np.float64(nu_fit),
               errs=errs, truth=truth, log10_tau=np.int64(scat),
               ref_seconds=np.float64(dt))
    out.update(mg.databunch_to_dict(res, "out_"))
    return out


# ---------------------------------------------------------------------------
# get_TOAs on synthetic archives
# ---------------------------------------------------------------------------
def run_toas(c):
    from pplib import DataBunch
    import psrchive as pr
    files_in, freqs = toa_inputs(c)
    nbin = c["nbin"]
    files = {}
    out = {}
    hashes = []
    for f, fi in enumerate(files_in):
        subints = fi["subints"][:, None]
        nsub_f = subints.shape[0]
        noise = np.array([mg.pplib.get_noise(subints[i, 0], chans=True)
                          for i in range(nsub_f)])
        snrs = np.abs(subints[:, 0].max(axis=-1)) / noise * 3.0
        name = "%s_%d.fits" % (c["name"], f)
        files[name] = DataBunch(
            epochs=[pr.MJD(e) for e in fi["epochs"]], filename=name,
            phases=mg.pplib.get_bin_centers(nbin),
            **archive_fields(c, fi, freqs, noise, snrs))
        hashes.append(S.sha(fi["subints"].astype(np.float32)))
        out["f%d_noise" % f] = noise
        out["f%d_snrs" % f] = snrs

    def loader(filename, **kw):
        # load_data must be asked for the tscrunched archive exactly when
        # get_TOAs was (pptoas.py:262-266)
        assert bool(kw.get("tscrunch")) == bool(c.get("tscrunch")), kw
        return files[filename]
    mg.pptoas.load_data = loader
    gt = mg.pptoas.GetTOAs.__new__(mg.pptoas.GetTOAs)
    gt.datafiles = list(files.keys())
    gt.is_FITS_model = False
    gt.modelfile = mg.GMODEL if toa_gmodel(c) == S.GMODEL else toa_gmodel(c)
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
        gt.get_TOAs(quiet=True, DM0=S.DM0 if c.get("DM0") else None,
                    **c.get("kw", {}))
    dt = time.time() - t0
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        mg.pplib.write_TOAs(gt.TOA_list)
    out.update(nfile=np.int64(c["nfile"]),
               nsub=np.int64(files_in[0]["subints"].shape[0]),
               nchan=np.int64(c["nchan"]), nbin=np.int64(nbin),
               seed=np.int64(c["seed"]), scint=np.int64(bool(c.get("scint"))),
               narrow=np.int64(bool(c.get("narrow"))),
               DM0_given=np.int64(bool(c.get("DM0"))), P=np.float64(S.P0),
               DM0=np.float64(S.DM0), freqs=freqs, sha=np.array(hashes),
               ref_seconds=np.float64(dt))
    for f, fi in enumerate(files_in):
        out["f%d_weights" % f] = fi["weights"]
        out["f%d_dfs" % f] = fi["dfs"]
        out["f%d_epochs" % f] = fi["epochs"]
    for key in ["phis", "phi_errs", "DMs", "DM_errs", "red_chi2s", "snrs",
                "scales", "scale_errs", "channel_snrs", "covariances",
                "DeltaDM_means", "DeltaDM_errs", "GMs", "GM_errs", "taus",
                "tau_errs", "alphas", "alpha_errs", "fluxes", "flux_errs",
                "flux_freqs", "profile_fluxes", "profile_flux_errs",
                "nu_fits", "rcs", "nfevals"]:
        out["out_" + key] = np.array(getattr(gt, key), dtype=np.float64)
    out["out_nu_refs"] = np.array(gt.nu_refs, dtype=np.float64)
    out["out_tim_lines"] = np.array(buf.getvalue().splitlines())
    return out


# ---------------------------------------------------------------------------
# align_archives
# ---------------------------------------------------------------------------
def run_align(c):
    from pplib import DataBunch
    arch_in, guess, freqs, tfreqs = align_inputs(c)
    nchan, nbin, nsub = c["nchan"], c["nbin"], c["nsub"]
    files, out = {}, {}
    for f, a in enumerate(arch_in):
        subints = a["subints"][:, None]
        noise = np.array([[mg.pplib.get_noise(subints[i, 0], chans=True)]
                          for i in range(nsub)])
        snrs = np.abs(subints.max(axis=-1)) / noise * 3.0
        wnorm = np.where(a["weights"] == 0.0, 0.0, 1.0)
        files["arch%d.fits" % f] = DataBunch(
            arch=None, DM=S.DM0, dmc=0, freqs=np.tile(freqs, (nsub, 1)),
            masks=np.einsum("ij,k", wnorm, np.ones(nbin))[:, None],
            nbin=nbin, nchan=nchan, noise_stds=noise, npol=1, nsub=nsub,
            ok_ichans=[np.compress(wnorm[i], list(range(nchan)))
                       for i in range(nsub)], ok_isubs=np.arange(nsub),
            phases=mg.pplib.get_bin_centers(nbin), prof_SNR=100.0,
            Ps=np.ones(nsub) * S.P0, SNRs=snrs, subints=subints,
            weights=a["weights"])
        out["f%d_weights" % f] = a["weights"]
        out["f%d_noise" % f] = noise[:, 0]
        out["f%d_snrs" % f] = snrs[:, 0]
    tn = len(tfreqs)
    rec = mga.FakeArch(1, tn, nbin)
    files["guess.fits"] = DataBunch(
        arch=rec, DM=0.0, dmc=1, freqs=tfreqs[None, :],
        masks=np.ones([1, 1, tn, nbin]), nbin=nbin, nchan=tn,
        noise_stds=np.ones([1, 1, tn]), npol=1, nsub=1,
        ok_ichans=[np.arange(tn)], ok_isubs=np.arange(1),
        phases=mg.pplib.get_bin_centers(nbin), prof_SNR=100.0,
        Ps=np.ones(1) * S.P0, SNRs=np.ones([1, 1, tn]),
        subints=guess[None, None], weights=np.ones([1, tn]))
    mga.ppalign.load_data = lambda filename, **kw: files[filename]
    mga.ppalign.sub.Popen = lambda *a, **kw: mga._VapPopen(tn, nbin)
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        mga.ppalign.align_archives(["arch%d.fits" % i for i in
                                    range(c["nfile"])], "guess.fits",
                                   fit_dm=True, niter=c["niter"],
                                   outfile="aligned.fits", quiet=True)
    dt = time.time() - t0
    out.update(nfile=np.int64(c["nfile"]),
               nsub=np.int64(files_in[0]["subints"].shape[0]),
               nchan=np.int64(c["nchan"]), nbin=np.int64(nbin),
               niter=np.int64(c["niter"]), seed=np.int64(c["seed"]),
               tmpl_nchan=np.int64(tn), P=np.float64(S.P0),
               DM0=np.float64(S.DM0), freqs=freqs, tfreqs=tfreqs,
               sha=np.array(S.sha(np.stack([a["subints"] for a in arch_in])
                                  .astype(np.float32), guess)),
               ref_seconds=np.float64(dt), out_aligned=rec.amps[0].copy(),
               out_weights=rec.weights.copy())
    return out


def run_scales():
    """pptoaslib.get_scales_full on the spectra of the all_64x512 golden
    case at its fitted parameters and output reference frequencies."""
    z = np.load(os.path.join(HERE, "fit_portrait_full.npz"))
    c = {k.split("/", 1)[1]: z[k] for k in z.files
         if k.startswith("all_64x512/")}
    data = c["data"].astype(np.float64)
    model = c["model"].astype(np.float64)
    nbin = data.shape[1]
    dFT = np.fft.rfft(data, axis=1)
    dFT[:, 0] *= 0
    mFT = np.fft.rfft(model, axis=1)
    mFT[:, 0] *= 0
    errs_FT = c["errs"] * np.sqrt(nbin / 2.0)
    out = {}
    for i, (params, nus, lt) in enumerate([
            (c["out_params"], (c["out_nu_DM"], c["out_nu_GM"],
                               c["out_nu_tau"]), True),
            (np.array([0.1, 34.5, 0.0, -2.5, -4.0]), (1300.0, 1300.0, 1400.0),
             True),
            (np.array([0.1, 34.5, 0.0, 2e-3, -3.5]), (1300.0, 1300.0, 1400.0),
             False),
            (np.array([-0.2, 34.6, 1e-5, 0.0, -4.0]), (1500.0, 1400.0,
                                                       1400.0), False)]):
        sc = mg.pptoaslib.get_scales_full(list(params), dFT, mFT, errs_FT,
                                          float(c["P"]), c["freqs"],
                                          float(nus[0]), float(nus[1]),
                                          float(nus[2]), lt)
        out["s%d_params" % i] = np.asarray(params, dtype=float)
        out["s%d_nus" % i] = np.asarray(nus, dtype=float)
        out["s%d_log10_tau" % i] = np.int64(lt)
        out["s%d_out" % i] = np.asarray(sc)
    out["case"] = np.array("all_64x512")
    return out


def run_splines():
    """pplib.gen_spline_portrait (pplib.py:966-990) through
    read_spline_model (pplib.py:3060-3096) on tests/golden/spline.spl: same,
    up- and down-sampled nbin, other frequency grids; plus the ncomp = 0
    (mean profile only) branch."""
    out = {}
    for name, nchan, lo, bw, nbin in SPLINES:
        freqs = S.channel_freqs(nchan, lo, bw)
        with contextlib.redirect_stdout(io.StringIO()):
            _, port = mg.pplib.read_spline_model(SPLINE_MODEL, freqs, nbin,
                                                 quiet=True)
        out[name + "_freqs"] = freqs
        out[name + "_nbin"] = np.int64(-1 if nbin is None else nbin)
        out[name + "_out"] = port
    _, _, _, mean_prof, eigvec, tck = mg.pplib.read_spline_model(
        SPLINE_MODEL, quiet=True)
    freqs = S.channel_freqs(16, 1100.0, 800.0)
    out["mean_freqs"] = freqs
    out["mean_out"] = mg.pplib.gen_spline_portrait(
        mean_prof, freqs, np.zeros((len(mean_prof), 0)), tck, 1024)
    return out


def main():
    only = None
    if "--only" in sys.argv:
        only = set(sys.argv[sys.argv.index("--only") + 1].split(","))
    write_narrow()
    write_spline()
    write_scat()
    old = {}
    if os.path.exists(OUT):
        z = np.load(OUT)
        old = {k: z[k] for k in z.files}
    store = dict(old)
    manifest = {}
    jobs = ([("fit", c, run_fit) for c in FITS] +
            [("toas", c, run_toas) for c in TOAS] +
            [("align", c, run_align) for c in ALIGNS] +
            [("scales", dict(name="scales"), lambda c: run_scales())] +
            [("spline", dict(name="gen"), lambda c: run_splines())])
    for kind, c, fn in jobs:
        key = "%s_%s" % (kind, c["name"])
        if only is not None and key not in only and c["name"] not in only:
            continue
        t0 = time.time()
        r = fn(c)
        for k in [k for k in store if k.startswith(key + "/")]:
            del store[k]
        for k, v in r.items():
            store[key + "/" + k] = v
        manifest[key] = dict(c, seconds=round(time.time() - t0, 2))
        print(key, "%.1fs" % (time.time() - t0), flush=True)
    np.savez_compressed(OUT, **store)
    mpath = os.path.join(HERE, "MANIFEST_full.json")
    m = json.load(open(mpath)) if os.path.exists(mpath) else {}
    m.update(manifest)
    m["_env"] = dict(numpy=np.__version__,
                     scipy=__import__("scipy").__version__,
                     reference="/root/reference @ 2025-02-17")
    json.dump(m, open(mpath, "w"), indent=1, default=str)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Golden vectors for GetTOAs.get_narrowband_TOAs (pptoas.py:794-1189),
produced by running the REFERENCE in this container (never on the GPU box),
with the import shims and the synthetic-archive ``load_data`` of
make_golden.py (same archives as its get_TOAs case, smaller).

Usage:  python tests/golden/make_golden_nb.py
"""
import contextlib
import io
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (imports the reference with the shims)
import numpy as np  # noqa: E402


def make_files(nfile=2, nsub=3, nchan=16, nbin=256, seed=99):
    from pplib import DataBunch
    import psrchive as pr
    rng = np.random.default_rng(seed)
    freqs1 = mg.channel_freqs(nchan)
    phases = mg.pplib.get_bin_centers(nbin)
    files, inputs = {}, {}
    for ifile in range(nfile):
        subints = np.zeros([nsub, 1, nchan, nbin])
        for isub in range(nsub):
            phi = rng.uniform(-0.5, 0.5)
            ddm = rng.normal(3e-4, 2e-4)
            d, _, _ = mg.make_portrait(rng, nchan, nbin, phi, mg.DM0 + ddm,
                                       mg.P0, noise=0.5)
            subints[isub, 0] = d
        weights = np.ones([nsub, nchan])
        if ifile == 1:
            for isub in range(nsub):
                weights[isub, rng.choice(nchan, 2 + isub, replace=False)] = 0
        noise = np.array([[mg.pplib.get_noise(subints[i, 0], chans=True)]
                          for i in range(nsub)])
        snrs = np.abs(subints.max(axis=-1)) / noise * 3.0
        wnorm = np.where(weights == 0.0, 0.0, 1.0)
        ok_ichans = [np.compress(wnorm[i], list(range(nchan)))
                     for i in range(nsub)]
        epochs = 57000.0 + np.arange(nsub) * 60.0 / 86400.0 + ifile
        name = "nb%d.fits" % ifile
        files[name] = DataBunch(
            arch=None, backend="fake_be", backend_delay=1e-5, bw=800.0,
            doppler_factors=np.ones(nsub), DM=mg.DM0, dmc=0,
            epochs=[pr.MJD(e) for e in epochs], filename=name,
            flux_prof=np.array([]), freqs=np.tile(freqs1, (nsub, 1)),
            frontend="fake_rx", integration_length=60.0 * nsub,
            masks=np.einsum("ij,k", wnorm, np.ones(nbin))[:, None],
            nbin=nbin, nchan=nchan, noise_stds=noise, npol=1, nsub=nsub,
            nu0=1500.0, ok_ichans=ok_ichans, ok_isubs=np.arange(nsub),
            parallactic_angles=np.zeros(nsub), phases=phases, prof=None,
            prof_noise=1.0, prof_SNR=100.0, Ps=np.ones(nsub) * mg.P0,
            SNRs=snrs, source="J1234-5678", state="Intensity",
            subints=subints, subtimes=[60.0] * nsub, telescope="GBT",
            telescope_code="1", weights=weights)
        inputs["f%d_subints" % ifile] = subints[:, 0].astype(np.float32)
        inputs["f%d_weights" % ifile] = weights
        inputs["f%d_snrs" % ifile] = snrs[:, 0]
        inputs["f%d_noise" % ifile] = noise[:, 0]
        inputs["f%d_epochs" % ifile] = epochs
    return files, inputs, freqs1


def run_nb():
    files, inputs, freqs = make_files()
    mg.pptoas.load_data = lambda filename, **kw: files[filename]
    gt = mg.pptoas.GetTOAs.__new__(mg.pptoas.GetTOAs)
    gt.datafiles = list(files.keys())
    gt.is_FITS_model = False
    gt.modelfile = mg.GMODEL
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
        gt.get_narrowband_TOAs(quiet=True)
    dt = time.time() - t0
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        mg.pplib.write_TOAs(gt.TOA_list)
    out = dict(inputs)
    f0 = files["nb0.fits"]
    out.update(nfile=np.int64(len(files)), nsub=np.int64(f0.nsub),
               nchan=np.int64(f0.nchan), nbin=np.int64(f0.nbin),
               P=np.float64(mg.P0), DM0=np.float64(mg.DM0), freqs=freqs,
               ref_seconds=np.float64(dt))
    for key in ["phis", "phi_errs", "scales", "scale_errs", "channel_snrs",
                "channel_red_chi2s"]:
        out["out_" + key] = np.array(getattr(gt, key), dtype=np.float64)
    out["out_TOA_days"] = np.array([t.MJD.in_days() for t in gt.TOA_list])
    out["out_TOA_errs"] = np.array([t.TOA_error for t in gt.TOA_list])
    out["out_tim_lines"] = np.array(buf.getvalue().splitlines())
    return out


def main():
    out = run_nb()
    path = os.path.join(HERE, "narrowband.npz")
    np.savez_compressed(path, **out)
    print("wrote %s (%d TOAs, %.1f s of reference time)" % (
        path, len(out["out_TOA_days"]), float(out["ref_seconds"])))


if __name__ == "__main__":
    main()

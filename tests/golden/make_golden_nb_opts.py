#!/usr/bin/env python
"""Golden vectors for GetTOAs.get_narrowband_TOAs' options (pptoas.py:
794-1189), produced by running the REFERENCE in this container (never on the
GPU box) with make_golden.py's import shims and make_golden_nb.py's
synthetic archives:

  * print_phase=True and print_flux=True: the exception the reference raises
    (it reads results.phi / fluxes, which that path never defines,
    pptoas.py:1131-1137), as "Type: message";
  * tscrunch=True with print_parangle=True and extra TOA flags: the loader
    hands over the archives tscrunched (one integration: the weight-weighted
    mean profile per channel, summed weights -- PSRCHIVE's weighted Profile
    average, emulated here because PSRCHIVE is absent), and the outputs and
    .tim lines of the run.

Usage:  python tests/golden/make_golden_nb_opts.py
"""
import contextlib
import io
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (imports the reference with the shims)
import make_golden_nb as nb  # noqa: E402
import numpy as np  # noqa: E402


def tscrunched(d):
    """The archive d as load_data(tscrunch=True) would hand it over."""
    from pplib import DataBunch
    import psrchive as pr
    w = d.weights
    wsum = w.sum(axis=0)
    x = (w[:, :, None] * d.subints[:, 0]).sum(axis=0) / \
        np.where(wsum > 0, wsum, 1.0)[:, None]
    noise = mg.pplib.get_noise(x, chans=True)
    snrs = np.abs(x.max(axis=-1)) / noise * 3.0
    wn = np.where(wsum == 0.0, 0.0, 1.0)
    mjd = np.mean([e.in_days() for e in d.epochs])
    return DataBunch(
        arch=None, backend=d.backend, backend_delay=d.backend_delay,
        bw=d.bw, doppler_factors=np.ones(1), DM=d.DM, dmc=0,
        epochs=[pr.MJD(mjd)], filename=d.filename, flux_prof=np.array([]),
        freqs=d.freqs[:1], frontend=d.frontend,
        integration_length=d.integration_length,
        masks=np.einsum("ij,k", wn[None], np.ones(d.nbin))[:, None],
        nbin=d.nbin, nchan=d.nchan, noise_stds=noise[None, None], npol=1,
        nsub=1, nu0=d.nu0, ok_ichans=[np.compress(wn, list(range(d.nchan)))],
        ok_isubs=np.arange(1), parallactic_angles=np.array([0.25]),
        phases=d.phases, prof=None, prof_noise=1.0, prof_SNR=100.0,
        Ps=d.Ps[:1], SNRs=snrs[None, None], source=d.source,
        state="Intensity", subints=x[None, None],
        subtimes=[float(np.sum(d.subtimes))], telescope=d.telescope,
        telescope_code=d.telescope_code, weights=wsum[None])


def _gettoas(files):
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
    return gt


def main():
    files, inputs, freqs = nb.make_files()
    ts = {k: tscrunched(v) for k, v in files.items()}
    out = dict(nfile=np.int64(len(files)), nchan=np.int64(16),
               nbin=np.int64(256), P=np.float64(mg.P0),
               DM0=np.float64(mg.DM0), freqs=freqs)
    out.update(inputs)
    # the options the reference's narrowband path cannot print
    for opt in ("print_phase", "print_flux"):
        mg.pptoas.load_data = lambda filename, **kw: files[filename]
        gt = _gettoas(files)
        msg = "no exception"
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                gt.get_narrowband_TOAs(quiet=True, **{opt: True})
        except Exception as exc:          # the reference's own failure
            msg = "%s: %s" % (type(exc).__name__, exc)
        out["exc_" + opt] = np.array(msg)
    # tscrunch (+ print_parangle and extra flags)
    seen = []

    def load(filename, **kw):
        seen.append(bool(kw.get("tscrunch")))
        return ts[filename] if kw.get("tscrunch") else files[filename]
    mg.pptoas.load_data = load
    gt = _gettoas(files)
    with contextlib.redirect_stdout(io.StringIO()):
        gt.get_narrowband_TOAs(quiet=True, tscrunch=True, print_parangle=True,
                               addtnl_toa_flags={"pta": "TEST"})
    assert seen and all(seen), seen
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        mg.pplib.write_TOAs(gt.TOA_list)
    for i, name in enumerate(files):
        d = ts[name]
        out["ts_f%d_subints" % i] = d.subints[:, 0]
        out["ts_f%d_weights" % i] = d.weights
        out["ts_f%d_noise" % i] = d.noise_stds[:, 0]
        out["ts_f%d_snrs" % i] = d.SNRs[:, 0]
        out["ts_f%d_epoch" % i] = np.float64(d.epochs[0].in_days())
    for key in ["phis", "phi_errs", "scales", "scale_errs", "channel_snrs",
                "channel_red_chi2s"]:
        out["ts_out_" + key] = np.array(getattr(gt, key), dtype=np.float64)
    out["ts_out_tim_lines"] = np.array(buf.getvalue().splitlines())
    path = os.path.join(HERE, "narrowband_opts.npz")
    np.savez_compressed(path, **out)
    print("wrote %s: %s | %s | %d tscrunched TOAs" % (
        path, out["exc_print_phase"], out["exc_print_flux"],
        len(out["ts_out_tim_lines"])))


if __name__ == "__main__":
    main()

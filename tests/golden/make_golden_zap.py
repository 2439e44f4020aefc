#!/usr/bin/env python
"""Golden vectors for GetTOAs.get_channels_to_zap (pptoas.py:1266-1343, which
goes through show_fit pptoas.py:1375-1480 and get_red_chi2 pplib.py:754-779),
produced by running the REFERENCE in this container (never on the GPU box)
with the import shims and synthetic-archive ``load_data`` of make_golden.py.

The archives carry what the zapper is meant to catch: a low-harmonic
sinusoid (RFI that get_noise_PS does not see, so its reduced chi^2 is high)
in a few channels, a per-channel signal gain ramp (weak channels below the
S/N cut, so the iterated threshold matters), masked channels and Doppler
factors != 1 (show_fit divides DM by them).  The reference's own get_TOAs
outputs are stored too, so the oracle can be checked on exactly the
parameters the reference zapped with.

Usage:  python tests/golden/make_golden_zap.py
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

ATTRS = ["obs", "doppler_fs", "nu0s", "nu_fits", "nu_refs", "ok_idatafiles",
         "ok_isubs", "epochs", "MJDs", "Ps", "phis", "phi_errs", "TOAs",
         "TOA_errs", "DM0s", "DMs", "DM_errs", "DeltaDM_means",
         "DeltaDM_errs", "GMs", "GM_errs", "taus", "tau_errs", "alphas",
         "alpha_errs", "scales", "scale_errs", "snrs", "channel_snrs",
         "profile_fluxes", "profile_flux_errs", "fluxes", "flux_errs",
         "flux_freqs", "red_chi2s", "channel_red_chi2s", "covariances",
         "nfevals", "rcs", "fit_durations", "order", "TOA_list",
         "zap_channels"]

# (SNR_threshold, rchi2_threshold, iterate) per get_channels_to_zap call
CALLS = [(8.0, 1.3, True), (30.0, 2.0, True), (30.0, 2.0, False),
         (0.0, 1.1, True)]


def make_files(nfile=2, nsub=3, nchan=32, nbin=256, seed=777):
    from pplib import DataBunch
    import psrchive as pr
    rng = np.random.default_rng(seed)
    freqs1 = mg.channel_freqs(nchan)
    phases = mg.pplib.get_bin_centers(nbin)
    files, inputs = {}, {}
    gain = np.linspace(0.02, 1.0, nchan)[rng.permutation(nchan)]
    for ifile in range(nfile):
        subints = np.zeros([nsub, 1, nchan, nbin])
        for isub in range(nsub):
            phi = rng.uniform(-0.5, 0.5)
            ddm = rng.normal(3e-4, 2e-4)
            clean, _, _ = mg.make_portrait(rng, nchan, nbin, phi,
                                           mg.DM0 + ddm, mg.P0, noise=0.0)
            port = clean * gain[:, None] + rng.normal(0.0, 1.5, clean.shape)
            for ich in rng.choice(nchan, 2, replace=False):   # slow RFI
                port[ich] += 2.0 * np.sin(2 * np.pi * (2 + isub) * phases
                                          + rng.uniform(0, 2 * np.pi))
            subints[isub, 0] = mg.f32(port)
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
        dfs = 1.0 + 1e-4 * rng.normal(size=nsub)
        epochs = 57000.0 + np.arange(nsub) * 60.0 / 86400.0 + ifile
        name = "zap%d.fits" % ifile
        files[name] = DataBunch(
            arch=None, backend="fake_be", backend_delay=0.0, bw=800.0,
            doppler_factors=dfs, DM=mg.DM0, dmc=0,
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
        inputs["f%d_dfs" % ifile] = dfs
        inputs["f%d_epochs" % ifile] = epochs
    return files, inputs, freqs1


def run_zap():
    files, inputs, freqs = make_files()
    mg.pptoas.load_data = lambda filename, **kw: files[filename]
    gt = mg.pptoas.GetTOAs.__new__(mg.pptoas.GetTOAs)
    gt.datafiles = list(files.keys())
    gt.is_FITS_model = False
    gt.modelfile = mg.GMODEL
    for attr in ATTRS:
        setattr(gt, attr, [])
    gt.instrumental_response_dict = gt.ird = {"DM": 0.0, "wids": [],
                                              "irf_types": []}
    gt.quiet = True
    with contextlib.redirect_stdout(io.StringIO()):
        gt.get_TOAs(quiet=True)
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        for snr_t, rchi2_t, it in CALLS:
            gt.get_channels_to_zap(SNR_threshold=snr_t,
                                   rchi2_threshold=rchi2_t, iterate=it)
    dt = time.time() - t0
    out = dict(inputs)
    f0 = files["zap0.fits"]
    out.update(nfile=np.int64(len(files)), nsub=np.int64(f0.nsub),
               nchan=np.int64(f0.nchan), nbin=np.int64(f0.nbin),
               P=np.float64(mg.P0), DM0=np.float64(mg.DM0), freqs=freqs,
               calls=np.array(CALLS, dtype=np.float64),
               ref_seconds=np.float64(dt))
    for key in ["phis", "phi_errs", "DMs", "DM_errs", "GMs", "taus",
                "alphas", "scales", "channel_snrs", "doppler_fs",
                "nu_refs"]:
        out["out_" + key] = np.array(getattr(gt, key), dtype=np.float64)
    # [ncall * nfile][nsub][nchx]: ragged -> flat values + per-(entry, sub)
    # lengths; zap lists keep the reference's append order
    chi, chi_n, zap, zap_n = [], [], [], []
    for entry_c, entry_z in zip(gt.channel_red_chi2s, gt.zap_channels):
        for c, z in zip(entry_c, entry_z):
            chi.extend(c)
            chi_n.append(len(c))
            zap.extend(int(v) for v in z)
            zap_n.append(len(z))
    out["out_chi2"] = np.array(chi, dtype=np.float64)
    out["out_chi2_n"] = np.array(chi_n, dtype=np.int64)
    out["out_zap"] = np.array(zap, dtype=np.int64)
    out["out_zap_n"] = np.array(zap_n, dtype=np.int64)
    out.update(run_ppzap(files, gt))
    return out


def run_ppzap(files, gt):
    """ppzap.py: the noise-median zapper (get_zap_channels, ppzap.py:23-53)
    over each archive, and print_paz_cmds (ppzap.py:56-106) for the
    model-based zap lists and the noise-based ones, all flag combinations."""
    with contextlib.redirect_stdout(io.StringIO()):
        import ppzap
    out = {}
    zl = []
    for nstd in (1.0, 3.0):
        for name in sorted(files):
            zl.append(ppzap.get_zap_channels(files[name], nstd=nstd))
    flat, nz = [], []
    for a in zl:
        for s in a:
            flat.extend(int(v) for v in s)
            nz.append(len(s))
    out["ppzap_noise_zap"] = np.array(flat, dtype=np.int64)
    out["ppzap_noise_zap_n"] = np.array(nz, dtype=np.int64)
    ok_files = list(np.array(gt.datafiles)[gt.ok_idatafiles])
    lines = []
    for zap_list in (gt.zap_channels[:2], zl[:2]):
        for all_subs in (False, True):
            for modify in (False, True):
                buf = io.StringIO()
                with contextlib.redirect_stdout(buf):
                    ppzap.print_paz_cmds(ok_files, zap_list,
                                         all_subs=all_subs, modify=modify)
                lines.append(buf.getvalue())
    out["ppzap_paz_out"] = np.array(lines)
    return out


def main():
    out = run_zap()
    path = os.path.join(HERE, "zap.npz")
    np.savez_compressed(path, **out)
    print("wrote %s (%d channel chi2s, %d zapped, %.2f s of reference time)"
          % (path, len(out["out_chi2"]), len(out["out_zap"]),
             float(out["ref_seconds"])))
    print("zap counts per (call, file, sub):", list(out["out_zap_n"]))


if __name__ == "__main__":
    main()

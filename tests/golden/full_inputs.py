"""Inputs of the full-shape golden cases (tests/golden/full.npz), rebuilt
from a few stored parameters (TEST INFRASTRUCTURE; no reference import).

make_golden_full.py builds the inputs here, hands them to the REFERENCE and
stores only its outputs plus a SHA-256 of the inputs; the tests rebuild the
inputs here and check the hash (see synth_np.py).
"""
import os

import numpy as np

import synth_np as S

HERE = os.path.dirname(os.path.abspath(__file__))

NARROW_GMODEL = os.path.join(HERE, "narrow.gmodel")
# example.gmodel plus a narrow (FWHM 0.002 rot) component: its power at
# 2048 bins stays above 1e-28 of the peak up to Nyquist
NARROW_PARAMS = np.concatenate([S.read_gmodel()[2],
                                [0.62, 0.0, 0.002, 0.0, 3.0, -1.0]])


SPLINE_MODEL = os.path.join(HERE, "spline.spl")
SPLINE_NBIN, SPLINE_NCOMP = 512, 3


def spline_parts():
    """A make_spline_model-type model (ppspline.py's PCA + B-spline, built
    here with numpy/scipy from the example.gmodel portrait at 64 channels,
    512 bins): (modelname, source, datafile, mean_prof, eigvec [512, 3],
    tck = splprep(projections, u=freqs, k=3))."""
    import scipy.interpolate as si
    model, freqs = S.template(64, SPLINE_NBIN)
    mean_prof = model.mean(axis=0)
    delta = model - mean_prof
    _, _, vt = np.linalg.svd(delta, full_matrices=False)
    eigvec = np.ascontiguousarray(vt[:SPLINE_NCOMP].T)
    proj = delta @ eigvec
    tck, _ = si.splprep(list(proj.T), u=freqs, k=3,
                        s=1e-4 * float((proj ** 2).sum()))
    tck = [np.asarray(tck[0]), [np.asarray(c) for c in tck[1]], int(tck[2])]
    return ("synthetic_spline", "J1234-5678", "synthetic.fits", mean_prof,
            eigvec, tck)


def write_spline(path=SPLINE_MODEL):
    """tests/golden/spline.spl (committed; rewritten only if missing): the
    pickle read_spline_model reads (pplib.py:3083-3088)."""
    import pickle
    if os.path.exists(path):
        return
    with open(path, "wb") as fh:
        pickle.dump(spline_parts(), fh, protocol=4)


def write_narrow(path=NARROW_GMODEL):
    """tests/golden/narrow.gmodel (committed; rewritten only if missing)."""
    if os.path.exists(path):
        return
    code, nu_ref, _, alpha = S.read_gmodel()
    S.write_gmodel(path, code, nu_ref, NARROW_PARAMS, alpha,
                   name="PSR_NARROW")


FITS = [
    dict(name="c3_all_512x2048_a", nchan=512, nbin=2048, flags=[1, 1, 1, 1, 1],
         seed=101, tau=2e-3),
    dict(name="c3_all_512x2048_b", nchan=512, nbin=2048, flags=[1, 1, 1, 1, 1],
         seed=102, tau=2e-3),
    dict(name="c3_pdta_512x2048", nchan=512, nbin=2048, flags=[1, 1, 0, 1, 1],
         seed=103, tau=2e-3),
    dict(name="narrow_pd_512x2048", nchan=512, nbin=2048,
         flags=[1, 1, 0, 0, 0], seed=104, narrow=True),
    dict(name="pd_64x4096", nchan=64, nbin=4096, flags=[1, 1, 0, 0, 0],
         seed=105),
    dict(name="pdta_64x128", nchan=64, nbin=128, flags=[1, 1, 0, 1, 1],
         seed=106, tau=2e-3),
    # low S/N (round 3): |C_n| far below sum_k |Y_k|, where
    # the moment expansion's truncation bound (relative to sum |Y|) is
    # loosest, and the initial DM several bins off at the band edges
    dict(name="lowsnr_pd_512x2048", nchan=512, nbin=2048, flags=[1, 1, 0, 0, 0],
         seed=107, noise=40.0, dm_off=4e-3),
    dict(name="lowsnr_pd_64x512", nchan=64, nbin=512, flags=[1, 1, 0, 0, 0],
         seed=108, noise=12.0, dm_off=1.5e-2),
    dict(name="lowsnr_all_512x2048", nchan=512, nbin=2048,
         flags=[1, 1, 1, 1, 1], seed=109, tau=2e-3, noise=12.0),
    # round 4: nbin not a power of two (numpy's rfft takes any length,
    # pptoaslib.py:1022-1025): the mixed-radix LDS FFT (2^2 5^3, 2^8 3)
    dict(name="pd_128x1000", nchan=128, nbin=1000, flags=[1, 1, 0, 0, 0],
         seed=110),
    dict(name="pdta_128x1536", nchan=128, nbin=1536, flags=[1, 1, 0, 1, 1],
         seed=111, tau=2e-3),
    # round 5: nbin / 2 with a prime factor above 7 (the generic-radix
    # stage): 1022 = 2 * 7 * 73 (wave-per-row spectrum pass), 2006 =
    # 2 * 17 * 59 (block FFT, nbin / 2 > 1024)
    dict(name="pd_128x1022", nchan=128, nbin=1022, flags=[1, 1, 0, 0, 0],
         seed=112),
    dict(name="pdta_64x2006", nchan=64, nbin=2006, flags=[1, 1, 0, 1, 1],
         seed=113, tau=2e-3),
    # odd nbin (the row transformed as nbin complex points): 1023 = 3 * 11 *
    # 31 (radix 3 + generic stages), 1001 = 7 * 11 * 13 with scattering
    dict(name="pd_128x1023", nchan=128, nbin=1023, flags=[1, 1, 0, 0, 0],
         seed=114),
    dict(name="pdta_64x1001", nchan=64, nbin=1001, flags=[1, 1, 0, 1, 1],
         seed=115, tau=2e-3),
    # round 6: rows past the LDS transforms (even nbin > 8192, odd > 4095):
    # the rFFTs on the long (four-step / chirp z) transforms, fits on X
    dict(name="pd_16x16384", nchan=16, nbin=16384, flags=[1, 1, 0, 0, 0],
         seed=116),
    dict(name="pdta_16x10002", nchan=16, nbin=10002, flags=[1, 1, 0, 1, 1],
         seed=117, tau=2e-3),
    dict(name="pd_16x8193", nchan=16, nbin=8193, flags=[1, 1, 0, 0, 0],
         seed=118),
]


def fit_inputs(c):
    """(data, model, freqs, P, truth, init, nu_fit) of a fit case, rebuilt
    identically by the tests (tests/test_gpu_fullshape.py)."""
    rng = np.random.default_rng(20251016 + c["seed"])
    nchan, nbin = c["nchan"], c["nbin"]
    phi = rng.uniform(-0.5, 0.5)
    dDM = rng.normal(3e-4, 2e-4)
    P = S.P0 * (1.0 + 1e-6 * rng.normal())
    phi_guess_off = rng.normal(0, 2e-3)
    model, freqs = S.template(nchan, nbin, gmodel=NARROW_GMODEL if
                              c.get("narrow") else None)
    tau = c.get("tau", 0.0)
    data = S.subint(c["seed"], model, freqs, phi, S.DM0 + dDM, P, tau=tau,
                    noise=c.get("noise", 1.5))
    nu_fit = float(_guess_fit_freq(freqs))
    phi_g = _phase_transform(phi + phi_guess_off, S.DM0, 1500.0, nu_fit, P)
    scat = c["flags"][3] == 1
    init = [phi_g, S.DM0 + c.get("dm_off", 0.0), 0.0,
            np.log10(1.0 / nbin) if scat else 0.0, -4.0 if scat else 0.0]
    return data, model, freqs, P, np.array([phi, S.DM0 + dDM, 0.0, tau,
                                            -4.0]), init, nu_fit


def _guess_fit_freq(freqs, SNRs=None):
    nu0 = (freqs.min() + freqs.max()) * 0.5
    w = (np.ones(len(freqs)) if SNRs is None else SNRs) * freqs ** -2
    return nu0 + np.sum((freqs - nu0) * w) / np.sum(w)


def _phase_transform(phi, DM, nu1, nu2, P):
    x = phi + S.DCONST * DM / P * (nu2 ** -2 - nu1 ** -2)
    x = x % 1.0
    return x - 1.0 if x >= 0.5 else x


SCAT_GMODEL = os.path.join(HERE, "scat.gmodel")
# example.gmodel with a nonzero TAU [s] at its FREQ (1300 MHz): GetTOAs'
# scattering branch takes its tau guess from it (pptoas.py:478-480) and
# phase-fits the mean model scattered by that guess (pptoas.py:484-489)
SCAT_TAU_S = 1.5e-3 * S.P0 * (1300.0 / 1500.0) ** -4


def write_scat(path=SCAT_GMODEL):
    """tests/golden/scat.gmodel (committed; rewritten only if missing)."""
    if os.path.exists(path):
        return
    code, nu_ref, params, alpha = S.read_gmodel()
    params = params.copy()
    params[1] = SCAT_TAU_S
    S.write_gmodel(path, code, nu_ref, params, alpha, name="PSR_SCAT")


TOAS = [
    dict(name="c1", nfile=5, nsub=10, nchan=64, nbin=512, scint=True,
         seed=201, DM0=True),
    dict(name="c2", nfile=1, nsub=8, nchan=512, nbin=2048, seed=202),
    dict(name="narrow", nfile=1, nsub=4, nchan=512, nbin=2048, seed=203,
         narrow=True),
    # get_TOAs with a spline template (pptoas.py:416-419), 512 -> 1024 bins
    dict(name="spline", nfile=2, nsub=4, nchan=64, nbin=1024, seed=204,
         spline=True),
    # round 6: rows past the LDS transforms (the guess profile's rFFT and
    # every row's on the long transforms)
    dict(name="long16384", nfile=1, nsub=3, nchan=16, nbin=16384, seed=208),
    # and with the scattered .gmodel (its convolution on the long
    # transforms), fitting scattering
    dict(name="scatlong", nfile=1, nsub=2, nchan=16, nbin=16384, seed=210,
         gmodel="scat", tau=2e-3, kw=dict(fit_scat=True)),
    # ---- the non-default branches of get_TOAs (round 3) ----------------
    # (a) configs[2]'s drop-in entry: fit_GM + fit_scat at 512 x 2048 with a
    # .gmodel whose TAU != 0 (tau guess from gparams, phase guess against
    # the scattered mean model, pptoas.py:467-492; gm / scat_time /
    # log10_scat_time / scat_ind flags, pptoas.py:659-677)
    dict(name="scatgm", nfile=1, nsub=3, nchan=512, nbin=2048, seed=205,
         gmodel="scat", tau=2e-3, kw=dict(fit_GM=True, fit_scat=True)),
    # (b) configs[4]'s band (400-800 MHz): fit_scat with scat_guess and
    # fix_alpha (pptoas.py:469-472, 236), flux of the scattered model
    # (print_flux, pptoas.py:598-624)
    dict(name="scatfix", nfile=1, nsub=4, nchan=128, nbin=1024, seed=206,
         lo=400.0, bw=400.0, nu0=600.0, tau=5e-3, nu_tau=600.0,
         kw=dict(fit_scat=True, fix_alpha=True, print_flux=True,
                 scat_guess=[4e-3 * S.P0, 600.0, -4.0])),
    # (c) user nu_refs and nu_fits (pptoas.py:440-456, 691-693),
    # print_phase / print_flux / print_parangle and extra flags
    dict(name="opts", nfile=2, nsub=4, nchan=64, nbin=512, seed=207,
         parangle=True,
         kw=dict(nu_refs=(1400.0, 1450.0), nu_fits=(1350.0, 1380.0),
                 print_phase=True, print_flux=True, print_parangle=True,
                 addtnl_toa_flags={"pta": "TEST", "ver": 0.1})),
    # (d) 1- and 2-channel sub-ints under fit_GM (pptoas.py:519-529): the
    # fit_flags list carries over from one sub-int (and archive) to the next
    dict(name="chan12", nfile=2, nsub=5, nchan=64, nbin=512, seed=208,
         chans={0: [None, 2, 1, 2, None], 1: [2, None, 1, None, 2]},
         kw=dict(fit_GM=True)),
    # (e) tscrunch=True (forwarded to load_data) and bary=False, with a
    # linear-tau scattering fit (scat_time_err, pptoas.py:669-673)
    dict(name="tscr", nfile=2, nsub=3, nchan=128, nbin=512, seed=209,
         gmodel="scat", tau=3e-3, same_phi=True, tscrunch=True,
         kw=dict(tscrunch=True, bary=False, fit_scat=True, log10_tau=False)),
    # (f) method='TNC' (bounded, pptoas.py:503-513; pptoaslib.py:1041-1053):
    # phase + DM (default bounds); a scattering fit with user bounds whose
    # alpha bound is active at the solution
    dict(name="tnc", nfile=1, nsub=4, nchan=64, nbin=512, seed=210,
         kw=dict(method="TNC")),
    dict(name="tncscat", nfile=1, nsub=4, nchan=128, nbin=512, seed=211,
         gmodel="scat", tau=3e-3,
         kw=dict(method="TNC", fit_scat=True,
                 bounds=[(None, None), (None, None), (None, None),
                         (-3.5, None), (-10.0, -4.4)])),
    # (g) method='Newton-CG' (pptoaslib.py:1049-1050)
    dict(name="ncg", nfile=1, nsub=2, nchan=64, nbin=512, seed=212,
         kw=dict(method="Newton-CG")),
    # (h) round 4: nbin = 1000 through the whole get_TOAs loop (guess
    # profile, its FFTFIT, the fit) on the mixed-radix FFT
    dict(name="nb1000", nfile=1, nsub=3, nchan=64, nbin=1000, seed=213),
    # (i) round 5: nbin = 1022 (2 * 7 * 73), the generic-radix FFT stage
    dict(name="nb1022", nfile=1, nsub=3, nchan=64, nbin=1022, seed=214),
    # (j) odd nbin = 1023 = 3 * 11 * 31 through the whole get_TOAs loop
    dict(name="nb1023", nfile=1, nsub=3, nchan=64, nbin=1023, seed=215),
]


def toa_gmodel(c):
    """The template file of a get_TOAs case."""
    if c.get("narrow"):
        write_narrow()
        return NARROW_GMODEL
    if c.get("spline"):
        write_spline()
        return SPLINE_MODEL
    if c.get("gmodel") == "scat":
        write_scat()
        return SCAT_GMODEL
    return S.GMODEL

# gen_spline_portrait cases: (name, nchan, lo, bw, nbin [None = model's])
SPLINES = [("same", 64, 1100.0, 800.0, None), ("n512", 48, 1150.0, 700.0, 512),
           ("up1024", 64, 1100.0, 800.0, 1024), ("up4096", 32, 1200.0, 600.0,
                                                   4096),
           ("down256", 64, 1100.0, 800.0, 256), ("down64", 100, 1120.0, 760.0,
                                                 64),
           # round 6: resampled to lengths that are not powers of two (the
           # mixed-radix LDS transforms)
           ("n1000", 64, 1100.0, 800.0, 1000), ("n1536", 48, 1150.0, 700.0,
                                                1536),
           ("down300", 64, 1100.0, 800.0, 300)]


def toa_inputs(c):
    """Per archive: subints [nsub, nchan, nbin] f32-rounded, weights, SNRs,
    doppler factors, epochs; plus freqs.  Rebuilt identically by the tests."""
    rng = np.random.default_rng(20251016 + c["seed"])
    nchan, nbin, nsub = c["nchan"], c["nbin"], c["nsub"]
    model, freqs = S.template(nchan, nbin, lo=c.get("lo", 1100.0),
                              bw=c.get("bw", 800.0),
                              gmodel=NARROW_GMODEL if c.get("narrow")
                              else None)
    files = []
    for f in range(c["nfile"]):
        dDM = rng.normal(3e-4, 2e-4)            # example.py: one per archive
        subs = np.zeros((nsub, nchan, nbin))
        if c.get("same_phi"):
            phi0 = rng.uniform(-0.5, 0.5)
        for s in range(nsub):
            phi = phi0 if c.get("same_phi") else rng.uniform(-0.5, 0.5)
            subs[s] = S.subint(c["seed"] * 1000 + f * 100 + s, model, freqs,
                               phi, S.DM0 + dDM, S.P0,
                               nu0=c.get("nu0", 1500.0),
                               tau=c.get("tau", 0.0),
                               nu_tau=c.get("nu_tau", 1500.0),
                               scint=c.get("scint", False))
        weights = np.ones((nsub, nchan))
        if f == 1 or c["nfile"] == 1:           # zap a few channels
            for s in range(nsub):
                weights[s, rng.choice(nchan, 3 + s % 4, replace=False)] = 0.0
        for s, nk in enumerate(c.get("chans", {}).get(f, [])):
            if nk is not None:                  # keep only nk channels
                weights[s] = 0.0
                weights[s, rng.choice(nchan, nk, replace=False)] = 1.0
        dfs = 1.0 + 1e-4 * rng.normal(size=nsub)
        epochs = 57202.0 + 20.0 * f + np.arange(nsub) * 60.0 / 86400.0
        pa = (np.linspace(-40.0, 40.0, nsub) + 7.0 * f if c.get("parangle")
              else np.zeros(nsub))
        if c.get("tscrunch"):
            # what load_data(tscrunch=True) hands over: one sub-int, the
            # mean of the sub-ints (same phase), channels usable in all
            subs = S.f32(subs.mean(axis=0))[None]
            weights = weights.min(axis=0)[None]
            dfs, epochs, pa = dfs[:1], epochs.mean()[None], pa[:1]
        files.append(dict(subints=subs, weights=weights, dfs=dfs,
                          epochs=epochs, dDM=dDM, parangles=pa))
    return files, freqs


def archive_fields(c, fi, freqs, noise, snrs):
    """The load_data DataBunch fields (pplib.py:2904-2914) of one synthetic
    archive, apart from `epochs` (PSRCHIVE MJD objects, built by the
    caller); noise [nsub, nchan], snrs [nsub, nchan]."""
    subints = np.asarray(fi["subints"], dtype=np.float64)[:, None]
    nsub = subints.shape[0]
    nbin = int(c["nbin"])
    nchan = len(freqs)
    wn = np.where(fi["weights"] == 0.0, 0.0, 1.0)
    return dict(
        arch=None, backend="fake_be", backend_delay=0.0,
        bw=float(c.get("bw", 800.0)), doppler_factors=fi["dfs"], DM=S.DM0,
        dmc=0, flux_prof=np.array([]), freqs=np.tile(freqs, (nsub, 1)),
        frontend="fake_rx", integration_length=60.0 * nsub,
        masks=np.einsum("ij,k", wn, np.ones(nbin))[:, None], nbin=nbin,
        nchan=nchan, noise_stds=np.asarray(noise)[:, None], npol=1,
        nsub=nsub, nu0=float(c.get("lo", 1100.0) + c.get("bw", 800.0) / 2),
        ok_ichans=[np.compress(wn[i], list(range(nchan)))
                   for i in range(nsub)],
        ok_isubs=np.arange(nsub), parallactic_angles=fi["parangles"],
        prof=None, prof_noise=1.0, prof_SNR=100.0,
        Ps=np.ones(nsub) * S.P0, SNRs=np.asarray(snrs)[:, None],
        source="J1234-5678", state="Intensity", subints=subints,
        subtimes=[60.0] * nsub, telescope="GBT", telescope_code="1",
        weights=fi["weights"])


ALIGNS = [
    dict(name="c4", nfile=16, nsub=1, nchan=256, nbin=1024, niter=3,
         seed=301),
    dict(name="dup", nfile=4, nsub=2, nchan=32, nbin=256, niter=2, seed=302,
         tmpl_nchan=16),
]


def align_inputs(c):
    """(archives, guess template [tmpl_nchan, nbin], data freqs, template
    freqs) rebuilt identically by the tests."""
    rng = np.random.default_rng(20251016 + c["seed"])
    nchan, nbin, nsub = c["nchan"], c["nbin"], c["nsub"]
    model, freqs = S.template(nchan, nbin)
    arch = []
    for f in range(c["nfile"]):
        subs = np.zeros((nsub, nchan, nbin))
        for s in range(nsub):
            phi = rng.uniform(-0.5, 0.5)
            dDM = rng.normal(3e-4, 2e-4)
            subs[s] = S.subint(c["seed"] * 1000 + f * 10 + s, model, freqs,
                               phi, S.DM0 + dDM, S.P0,
                               noise=c.get("noise", 0.5))
        weights = np.ones((nsub, nchan))
        if f == 2:
            weights[:, rng.choice(nchan, 4, replace=False)] = 0.0
        arch.append(dict(subints=subs, weights=weights))
    tn = c.get("tmpl_nchan", nchan)
    tfreqs = S.channel_freqs(tn)
    # initial template as in the reference's notebook (make_constant_portrait
    # with DataPortrait.prof): archive 0's mean profile, dedispersed at DM0
    # to the band centre, tiled over the template's channels
    ded = S.rotate(arch[0]["subints"].reshape(-1, nbin),
                   np.tile(S.DCONST * S.DM0 * (freqs ** -2 - 1500.0 ** -2) /
                           S.P0, nsub))
    prof = S.f32(ded.mean(axis=0))
    guess = np.tile(prof, (tn, 1))
    return arch, guess, freqs, tfreqs


# configs[4] (16384 x 1024, CHIME-like 400-800 MHz, phi + DM + tau + alpha):
# the reference cannot run this width (its dense covariance cube,
# pptoaslib.py:731, needs 3.5e13 B), so these outputs come from the ORACLE
# (make_golden_oracle.py), itself pinned to the reference at <= 512 channels
C5 = [dict(name="c5_a", nchan=16384, nbin=1024, flags=[1, 1, 0, 1, 1],
           seed=401, tau=5e-3, nu_tau=600.0),
      dict(name="c5_b", nchan=16384, nbin=1024, flags=[1, 1, 0, 1, 1],
           seed=402, tau=5e-3, nu_tau=600.0)]


def c5_inputs(c):
    """(data, model, freqs, P, truth, init, nu_fit) of a configs[4] case."""
    rng = np.random.default_rng(20251016 + c["seed"])
    nchan, nbin = c["nchan"], c["nbin"]
    phi = rng.uniform(-0.5, 0.5)
    dDM = rng.normal(3e-4, 2e-4)
    P = S.P0
    model, freqs = S.template(nchan, nbin, lo=400.0, bw=400.0)
    data = S.subint(c["seed"], model, freqs, phi, S.DM0 + dDM, P,
                    tau=c["tau"], nu_tau=c["nu_tau"])
    nu_fit = float(_guess_fit_freq(freqs))
    # GetTOAs guesses (pptoas.py:467-502): log10 tau = log10(1/nbin),
    # alpha = -4; the phase guess starts within 1e-3 rot of the truth
    phi_g = _phase_transform(phi + rng.normal(0, 1e-3), S.DM0, 1500.0,
                             nu_fit, P)
    init = [phi_g, S.DM0, 0.0, np.log10(1.0 / nbin), -4.0]
    return data, model, freqs, P, np.array([phi, S.DM0 + dDM, 0.0, c["tau"],
                                            -4.0]), init, nu_fit

"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the oracle.  Bar (BASELINE.json north_star): fitted parameters
within 0.01 sigma of the reference's reported uncertainty, compared at the
reference's output reference frequencies, chi2_red
within 1e-8 relative."""
import numpy as np
import pytest

import goldens as G

pytestmark = pytest.mark.gpu

SIG = G.SIGMA_TOL
RCHI2 = G.RCHI2_RTOL


@pytest.fixture(scope="module")
def ppt():
    from pulseportraiture_amd import pptoaslib
    return pptoaslib


@pytest.fixture(scope="module")
def ppl():
    from pulseportraiture_amd import pplib
    return pplib


# ----------------------------------------------------------- FFT building ---
def test_noise_matches_reference(ppl):
    m = G.misc()
    np.testing.assert_allclose(ppl.get_noise(m["rot_port"], chans=True),
                               m["noise_port"], rtol=1e-12)
    assert abs(ppl.get_noise(m["rot_prof"]) / m["noise_prof"] - 1) < 1e-12
    # nbin 1000: nbin/2 = 2^2 5^3 on the mixed-radix LDS FFT
    for nb in (256, 1000, 2048):
        np.testing.assert_allclose(
            ppl.get_noise(m["noise_in_%d" % nb], chans=True),
            m["noise_out_%d" % nb], rtol=1e-12)
    # nbin/2 with a prime factor above 7 (the generic-radix stage): 1002 =
    # 2 x 3 x 167, 1022 = 2 x 7 x 73, 4094 = 2 x 23 x 89; the reference's
    # arithmetic (pplib.py:2312-2338) restated in NumPy
    for shape in ((2, 1002), (3, 1022), (2, 4094)):
        x = np.random.default_rng(6).normal(size=shape)
        F = np.fft.rfft(x, axis=-1)
        p = np.real(F * np.conj(F)) / shape[-1]
        want = np.sqrt(np.mean(p[:, int((1 - 4 ** -1) * p.shape[-1]):],
                               axis=-1))
        np.testing.assert_allclose(ppl.get_noise(x, chans=True), want,
                                   rtol=1e-12, err_msg=str(shape))
    # odd nbin (the row as nbin complex points): 1001 = 7 x 11 x 13,
    # 1023 = 3 x 11 x 31, 4093 prime (one generic-radix stage)
    for shape in ((2, 1001), (3, 1023), (2, 4093), (2, 33)):
        x = np.random.default_rng(7).normal(size=shape)
        F = np.fft.rfft(x, axis=-1)
        p = np.real(F * np.conj(F)) / shape[-1]
        want = np.sqrt(np.mean(p[:, int((1 - 4 ** -1) * p.shape[-1]):],
                               axis=-1))
        np.testing.assert_allclose(ppl.get_noise(x, chans=True), want,
                                   rtol=1e-12, err_msg=str(shape))
    # rows past the LDS transforms (odd > 4095, even > 8192): ppf_noise_long
    # per row -- 4097 and 16382 = 2 x 8191 on the chirp z-transform, 16384
    # on the four-step
    for shape in ((2, 4097), (2, 16382), (3, 16384)):
        x = np.random.default_rng(8).normal(size=shape)
        F = np.fft.rfft(x, axis=-1)
        p = np.real(F * np.conj(F)) / shape[-1]
        want = np.sqrt(np.mean(p[:, int((1 - 4 ** -1) * p.shape[-1]):],
                               axis=-1))
        np.testing.assert_allclose(ppl.get_noise(x, chans=True), want,
                                   rtol=1e-11, err_msg=str(shape))
    # chans=False ravels the portrait (pplib.py:2334-2338) into one row of
    # nchan x nbin samples: ppf_noise_long (four-step for a power-of-two
    # transform, chirp z-transform otherwise; no LDS-size cap).  The
    # restatement is the reference's own NumPy arithmetic
    for shape in ((64, 2048), (512, 2048), (3, 1001), (511, 1023),
                  (512, 1000), (1002,), (8186,), (1022,), (1000,), (2, 3),
                  (5,), (1,)):
        x = np.random.default_rng(4).normal(size=shape)
        F = np.fft.rfft(x.ravel())
        p = np.real(F * np.conj(F)) / x.size
        want = np.sqrt(np.mean(p[int((1 - 4 ** -1) * len(p)):]))
        assert abs(ppl.get_noise(x) / want - 1) < 1e-11, shape


def test_noise_long_rows_match_numpy():
    """ppf_noise_long against NumPy's rFFT at lengths that exercise each
    plan: power-of-two transforms at the four-step's smallest and largest
    splits, chirp z-transforms of prime, odd-composite and even lengths, f32
    input (converted exactly), frac != 4, and several 256-MB row chunks."""
    from pulseportraiture_amd import engine
    rng = np.random.default_rng(9)

    def want(x, frac=4):
        F = np.fft.rfft(x, axis=-1)
        p = np.real(F * np.conj(F)) / x.shape[-1]
        return np.sqrt(np.mean(p[..., int((1 - frac ** -1) * p.shape[-1]):],
                               axis=-1))
    for nrows, nbin in ((3, 128), (2, 1 << 22), (2, 65537), (2, 3 * 5 * 7 * 11 * 13),
                        (4, 2 * 4099), (1, 1 << 25)):
        x = rng.normal(size=(nrows, nbin))
        got = engine.noise_rows_long(x).cpu().numpy()
        np.testing.assert_allclose(got, want(x), rtol=1e-11,
                                   err_msg=str((nrows, nbin)))
    x = rng.normal(size=(2, 3000)).astype(np.float32)
    np.testing.assert_array_equal(
        engine.noise_rows_long(x).cpu().numpy(),
        engine.noise_rows_long(x.astype(np.float64)).cpu().numpy())
    np.testing.assert_allclose(engine.noise_rows_long(x, frac=3).cpu().numpy(),
                               want(x.astype(np.float64), 3), rtol=1e-11)
    # 40 rows of 2^21 samples: 2^20-point transforms, 16 MB per work row,
    # 8 rows per 256-MB chunk -> five chunks
    x = rng.normal(size=(40, 1 << 21)).astype(np.float32)
    np.testing.assert_allclose(engine.noise_rows_long(x).cpu().numpy(),
                               want(x.astype(np.float64)), rtol=1e-11)


def test_noise_fp32_input_equals_fp64(ppl):
    x = np.random.default_rng(3).normal(size=(7, 512)).astype(np.float32)
    a = ppl.get_noise(x, chans=True)
    b = ppl.get_noise(x.astype(np.float64), chans=True)
    np.testing.assert_array_equal(a, b)


def test_rotate_matches_reference(ppl, ppt):
    m = G.misc()
    P0 = 1.0 / 345.67890123456789
    tol = dict(atol=1e-11, rtol=0)
    np.testing.assert_allclose(ppl.rotate_data(m["rot_prof"], 0.123),
                               m["rot1_dm0"], **tol)
    np.testing.assert_allclose(ppl.rotate_data(m["rot_port"], -0.377),
                               m["rot2_dm0"], **tol)
    np.testing.assert_allclose(ppl.rotate_data(m["rot_cube"], 0.05),
                               m["rot4_dm0"], **tol)
    np.testing.assert_allclose(
        ppl.rotate_data(m["rot_prof"], 0.1, 10.0, P0, 1300.0, 1500.0),
        m["rot1_dm"], **tol)
    np.testing.assert_allclose(
        ppl.rotate_data(m["rot_port"], 0.2, 34.5, P0, m["rot_freqs"], 1500.0),
        m["rot2_dm"], **tol)
    np.testing.assert_allclose(
        ppl.rotate_data(m["rot_cube"], -0.3, 12.5, m["rot_Ps"],
                        m["rot_freqs"], 1400.0), m["rot4_dm"], **tol)
    np.testing.assert_allclose(
        ppl.rotate_data(m["rot_cube"], 0.01, 5.0, m["rot_Ps"],
                        m["rot_freqs2"], np.inf), m["rot4_dm_f2"], **tol)
    np.testing.assert_allclose(
        ppl.rotate_portrait(m["rot_port"], 0.25, 20.0, P0, m["rot_freqs"],
                            1450.0), m["rotp_dm"], **tol)
    np.testing.assert_allclose(ppl.rotate_portrait(m["rot_port"], -0.125),
                               m["rotp_nodm"], **tol)
    np.testing.assert_allclose(
        ppt.rotate_portrait_full(m["rot_port"], 0.1, 3.0, 2.0, m["rot_freqs"],
                                 1500., 1600., P0), m["rotf_dmgm"], **tol)


@pytest.mark.parametrize("nbin", [1000, 1022, 2006, 4094, 33, 127, 511,
                                  1001, 1023, 4095,
                                  # round 6: past the LDS transforms
                                  # (ppf_rotate_long, Bluestein both ways)
                                  4097, 8194, 12001, 16384])
def test_rotate_any_nbin_matches_numpy(ppl, nbin):
    """rotate_data (pplib.py:2427-2480) at nbin/2 not a power of two, on
    the mixed-radix (1000) and generic-radix (1022 = 2 x 7 x 73, 2006 =
    2 x 17 x 59, 4094 = 2 x 23 x 89) LDS FFTs, and at odd nbin (33, 127
    prime, 511 = 7 x 73, 1001, 1023, 4095 = 3^2 5 7 13: the row as nbin
    complex points, Hermitian inverse), and past the LDS transforms (4097,
    8194 = 2 x 17 x 241, 12001, 16384: ppf_rotate_long), against its own
    NumPy arithmetic:
    rfft, phasor, irfft -- the irfft WITHOUT a length, as the reference calls
    it (pplib.py:2466, 2508-2512, 2550, 2652; pptoaslib.py:89): at odd nbin
    the public routines return nbin - 1 samples.  The internal full-length
    rotation (engine.rotate_rows, used by the PSRFITS dedispersion) keeps
    nbin samples: irfft(..., n=nbin)."""
    from pulseportraiture_amd import engine, pptoaslib
    x = np.random.default_rng(nbin).normal(size=(3, nbin))
    ph = 0.2718
    k = np.arange(nbin // 2 + 1)
    X = np.fft.rfft(x, axis=-1) * np.exp(2j * np.pi * k * ph)
    want = np.fft.irfft(X, axis=-1)
    assert want.shape[-1] == nbin - (nbin % 2)
    np.testing.assert_allclose(ppl.rotate_data(x, ph), want, atol=1e-11)
    np.testing.assert_allclose(ppl.rotate_data(x[0], ph), want[0], atol=1e-11)
    np.testing.assert_allclose(ppl.rotate_portrait(x, ph), want, atol=1e-11)
    np.testing.assert_allclose(ppl.rotate_profile(x[1], ph), want[1],
                               atol=1e-11)
    # DM != 0 (4-D branch, pplib.py:2467-2512) and rotate_portrait_full
    P0, f = 1.0 / 345.67890123456789, np.array([1300.0, 1400.0, 1500.0])
    phs = ph + ppl.Dconst * 12.5 / P0 * (f ** -2.0 - 1450.0 ** -2.0)
    Xd = np.fft.rfft(x, axis=-1) * np.exp(2j * np.pi * np.outer(phs, k))
    np.testing.assert_allclose(ppl.rotate_data(x, ph, 12.5, P0, f, 1450.0),
                               np.fft.irfft(Xd, axis=-1), atol=1e-10)
    np.testing.assert_allclose(
        pptoaslib.rotate_portrait_full(x, ph, 12.5, 0.0, f, 1450.0, np.inf,
                                       P0), np.fft.irfft(Xd, axis=-1),
        atol=1e-10)
    full = engine.rotate_rows(x, np.full(3, ph)).cpu().numpy()
    np.testing.assert_allclose(full, np.fft.irfft(X, n=nbin, axis=-1),
                               atol=1e-11)


def test_rotate_round_trip_and_bad_shapes(ppl, capsys):
    x = np.random.default_rng(5).normal(size=(4, 2048))
    X = np.fft.rfft(x)
    X[:, -1] = 0.0          # irfft drops Im(Nyquist): band-limit for a clean
    x = np.fft.irfft(X)     # round trip (numpy behaves the same)
    y = ppl.rotate_data(ppl.rotate_data(x, 0.3141), -0.3141)
    np.testing.assert_allclose(y, x, atol=1e-11)
    assert ppl.rotate_data(x, 0.1, 10.0, [1.0, 2.0], np.ones(4) * 1400.0) == 0
    assert "Wrong shape for array of periods." in capsys.readouterr().out


@pytest.mark.parametrize("nbin", [16384, 8193, 8192])
def test_fit_phase_shift_long_rows_match_oracle(ppl, nbin):
    """fit_phase_shift (pplib.py:2136-2182) at nbin past the LDS transforms
    (round 6: the rFFTs on the long transforms, ppf_phase_shift_batch's
    synchronous path) and at 8192 with Ns = nbin (the brute grid in global
    memory beside the LDS transform) against the oracle's restatement of the
    reference (scipy brute + fmin)."""
    from oracle import ppfit_oracle as O
    rng = np.random.default_rng(nbin)
    t = np.arange(nbin) / nbin
    model = np.exp(-0.5 * ((t - 0.4) / 0.01) ** 2) + \
        0.3 * np.exp(-0.5 * ((t - 0.47) / 0.02) ** 2)
    for shift in (0.123, -0.31):
        X = np.fft.rfft(model) * np.exp(2j * np.pi * np.arange(nbin // 2 + 1)
                                        * shift)
        d = 2.5 * np.fft.irfft(X, n=nbin) + rng.normal(0, 0.05, nbin)
        # Ns = nbin (ppalign's): at 16384 the grid leaves the LDS
        for Ns in (100, nbin):
            got = ppl.fit_phase_shift(d, model, Ns=Ns)
            want = O.fit_phase_shift(d, model, Ns=Ns)
            assert abs(G.phase_diff(got.phase, want["phase"])) < \
                0.01 * want["phase_err"]
            assert abs(got.phase_err / want["phase_err"] - 1) < 1e-4
            assert abs(got.scale / want["scale"] - 1) < 1e-6
            assert abs(got.snr / want["snr"] - 1) < 1e-6


def test_fit_phase_shift_matches_reference(ppl):
    m = G.misc()
    for row in m["fps_rows"]:
        d = row[:1024]
        shift, ns, noise, phase, perr, scale, serr, snr, rchi2 = row[1024:1033]
        r = ppl.fit_phase_shift(d, m["fps_model"],
                                None if np.isnan(noise) else noise,
                                Ns=int(ns))
        assert abs(G.phase_diff(r.phase, phase)) < SIG * perr
        assert abs(r.phase_err / perr - 1) < 1e-4
        assert abs(r.scale / scale - 1) < 1e-6
        assert abs(r.snr / snr - 1) < 1e-6


# ------------------------------------------------------- fit_portrait_full ---
@pytest.mark.parametrize("name", G.case_names("fit_portrait_full.npz"))
def test_fit_portrait_full_matches_reference(name, ppt):
    c = G.full_case(name)
    a = G.full_case_args(c)
    a["data_port"] = c["data"]          # float32 amplitudes, as stored
    r = ppt.fit_portrait_full(**a)
    ref = G.ref_bunch(c)
    got = dict(params=r.params, nu_DM=r.nu_DM, nu_GM=r.nu_GM, nu_tau=r.nu_tau)
    dev = G.param_deviation_sigma(got, ref, a["P"], a["log10_tau"])
    assert dev.max() < SIG, (name, dev)
    assert abs(r.red_chi2 / c["out_red_chi2"] - 1) < RCHI2
    assert abs(r.nu_DM / ref["nu_DM"] - 1) < 1e-5
    assert abs(r.nu_tau / ref["nu_tau"] - 1) < 1e-5
    np.testing.assert_allclose(r.param_errs, c["out_param_errs"], rtol=1e-4)
    np.testing.assert_allclose(r.scales, c["out_scales"], rtol=1e-4,
                               atol=1e-3 * np.abs(c["out_scale_errs"]).min())
    np.testing.assert_allclose(r.scale_errs, c["out_scale_errs"], rtol=1e-4)
    np.testing.assert_allclose(r.snr, c["out_snr"], rtol=1e-6)
    cm = c["out_covariance_matrix"]
    np.testing.assert_allclose(r.covariance_matrix, cm, rtol=1e-3,
                               atol=1e-6 * np.abs(cm).max())
    assert r.return_code in (1, 2)


@pytest.mark.parametrize("name", G.case_names("fit_portrait.npz"))
def test_fit_portrait_matches_reference(name, ppl):
    c = G.fp_case(name)
    errs = None if np.all(np.isnan(c["errs"])) else c["errs"]
    r = ppl.fit_portrait(c["data"], c["model"].astype(float), c["init"],
                         float(c["P"]), c["freqs"], None, None, errs)
    # compare at the reference's nu_ref (phase_transform semantics)
    ph = ppl.phase_transform(r.phase, r.DM, r.nu_ref, c["out_nu_ref"],
                             float(c["P"]))
    assert abs(G.phase_diff(ph, c["out_phase"])) < SIG * c["out_phase_err"]
    assert abs(r.DM - c["out_DM"]) < SIG * c["out_DM_err"]
    # the reference's TNC stops at xtol 1e-10: chi2 agrees to its precision
    assert abs(r.red_chi2 / c["out_red_chi2"] - 1) < RCHI2
    np.testing.assert_allclose(r.scales, c["out_scales"], rtol=1e-4)
    np.testing.assert_allclose(r.scale_errs, c["out_scale_errs"], rtol=1e-10)
    np.testing.assert_allclose(r.snr, c["out_snr"], rtol=1e-6)


# ------------------------------------------------------- batched engine -----
def test_batch_equals_single_and_is_deterministic():
    """Shard invariance: a sub-integration's result does not depend on the
    batch it is fitted in (1-vs-N GPU bit-identity rests on this), and
    repeated runs are bitwise identical."""
    from pulseportraiture_amd import engine
    cases = ["pd_64x512", "pd_nuout_64x512", "pdg_64x512"]
    cs = [G.full_case(n) for n in cases]
    data = np.stack([c["data"] for c in cs])
    model = np.stack([c["model"].astype(float) for c in cs])
    freqs = np.stack([c["freqs"] for c in cs])
    P = np.array([float(c["P"]) for c in cs])
    init = np.stack([c["init"] for c in cs])
    flags = np.stack([c["flags"] for c in cs])
    nu_fits = np.stack([c["nu_fits"] for c in cs])
    nu_outs = np.stack([c["nu_outs"] for c in cs])
    kw = dict(nu_fits=nu_fits, nu_outs=nu_outs, model_index=np.arange(3))
    b1 = engine.results_numpy(engine.fit_batch(data, model, freqs, P, init,
                                               flags, **kw))
    b2 = engine.results_numpy(engine.fit_batch(data, model, freqs, P, init,
                                               flags, **kw))
    np.testing.assert_array_equal(b1["results"], b2["results"])
    for i in range(3):
        s = engine.results_numpy(engine.fit_batch(
            data[i:i + 1], model[i:i + 1], freqs[i:i + 1], P[i:i + 1],
            init[i:i + 1], flags[i:i + 1], nu_fits=nu_fits[i:i + 1],
            nu_outs=nu_outs[i:i + 1]))
        np.testing.assert_array_equal(s["results"][0], b1["results"][i])
        np.testing.assert_array_equal(s["scales"][0], b1["scales"][i])
    # an explicit workspace budget below the batch's need splits it into
    # chunks (engine.fit_batch); every table equals the one-call run
    ch = engine.results_numpy(engine.fit_batch(data, model, freqs, P, init,
                                               flags, max_workspace=1 << 16,
                                               **kw))
    for k in ("results", "scales", "scale_errs", "channel_snrs",
              "covariance"):
        np.testing.assert_array_equal(ch[k], b1[k], err_msg=k)


def test_moments_from_x_equal_fused_pass():
    """PPF_OPT_MOM_X (moments from the stored cross spectrum, k_moments)
    lands on the fused pass's fits (k_xmom_g): same stationary point to well
    inside the parity bar (the two sum the same harmonics in another order
    and expand around the exact, not the bin-rounded, centre)."""
    from pulseportraiture_amd import engine, _lib
    cases = ["pd_64x512", "pd_nuout_64x512", "pdg_64x512"]
    cs = [G.full_case(n) for n in cases]
    data = np.stack([c["data"] for c in cs])
    model = np.stack([c["model"].astype(float) for c in cs])
    kw = dict(nu_fits=np.stack([c["nu_fits"] for c in cs]),
              nu_outs=np.stack([c["nu_outs"] for c in cs]),
              model_index=np.arange(3))
    args = (data, model, np.stack([c["freqs"] for c in cs]),
            np.array([float(c["P"]) for c in cs]),
            np.stack([c["init"] for c in cs]), np.stack([c["flags"] for c in cs]))
    a = engine.results_numpy(engine.fit_batch(*args, mom_x=False, **kw))
    b = engine.results_numpy(engine.fit_batch(*args, mom_x=True, **kw))
    I = _lib.RESULT_INDEX
    ra, rb = a["results"], b["results"]
    err = ra[:, I["param_errs"]]
    dp = np.abs(rb[:, I["params"]] - ra[:, I["params"]])
    dp[:, 0] = np.abs((dp[:, 0] + 0.5) % 1.0 - 0.5)
    ok = err > 0
    assert np.all(dp[ok] <= 1e-3 * err[ok]), (dp, err)
    np.testing.assert_allclose(rb[:, I["red_chi2"]], ra[:, I["red_chi2"]],
                               rtol=1e-10)
    np.testing.assert_allclose(b["scales"], a["scales"], rtol=1e-7, atol=0)


def test_masked_channels_equal_subset_fit(ppt):
    """Ragged channel masks in the batch == fitting the channel subset.

    Started near the optimum so both runs stay in one basin: the trust-region
    trajectory from a far start can branch on last-bit differences of the
    channel sums (the reference's own trajectories do the same)."""
    from pulseportraiture_amd import engine, _lib
    import oracle as O
    c = G.full_case("pd_128x1024")
    a = G.full_case_args(c)
    rng = np.random.default_rng(11)
    keep = np.ones(128, dtype=bool)
    keep[rng.choice(128, 17, replace=False)] = False
    lt = a["log10_tau"]          # False: tau = 0 exactly (no scattering)
    ref = O.fit_portrait_full(c["data"][keep].astype(float),
                              a["model_port"][keep], a["init_params"], a["P"],
                              a["freqs"][keep], a["nu_fits"], a["nu_outs"],
                              a["errs"][keep], a["fit_flags"], log10_tau=lt)
    init = np.array(ref["x_fit"]) + np.array([3e-5, 1e-4, 0, 0, 0])
    sub = ppt.fit_portrait_full(c["data"][keep], a["model_port"][keep], init,
                                a["P"], a["freqs"][keep], a["nu_fits"],
                                a["nu_outs"], a["errs"][keep], a["fit_flags"],
                                log10_tau=lt)
    res = engine.results_numpy(engine.fit_batch(
        c["data"][None], a["model_port"][None], a["freqs"][None], [a["P"]],
        init[None], a["fit_flags"], nu_fits=np.asarray(a["nu_fits"])[None],
        errs=a["errs"][None], chan_mask=keep[None].astype(np.uint8)))
    R = res["results"][0]
    I = _lib.RESULT_INDEX
    got = dict(params=R[I["params"]], nu_DM=R[I["nu_out"]][0],
               nu_GM=R[I["nu_out"]][1], nu_tau=R[I["nu_out"]][2])
    for cand in (got, dict(params=sub.params, nu_DM=sub.nu_DM,
                           nu_GM=sub.nu_GM, nu_tau=sub.nu_tau)):
        dev = G.param_deviation_sigma(cand, ref, a["P"], False)
        assert dev.max() < SIG, dev
    assert abs(R[I["red_chi2"]] / ref["red_chi2"] - 1) < RCHI2
    assert R[I["nchanx"]] == keep.sum()
    np.testing.assert_allclose(res["scales"][0][keep], ref["scales"],
                               rtol=1e-6)
    assert np.all(res["scales"][0][~keep] == 0.0)


# ------------------------------------------------------------- get_TOAs -----
class _MJD(object):
    """float-days stand-in for psrchive.MJD (as in the golden generator)."""

    def __init__(self, days=0.0):
        self.days = float(days)

    def __add__(self, other):
        return _MJD(self.days + (other.days if isinstance(other, _MJD)
                                 else other / 86400.0))

    def in_days(self):
        return self.days

    def intday(self):
        return int(self.days)

    def fracday(self):
        return self.days - int(self.days)


def _fake_archives(g):
    from pulseportraiture_amd.pplib import DataBunch, get_noise
    nsub, nchan, nbin = int(g["nsub"]), int(g["nchan"]), int(g["nbin"])
    files = {}
    for f in range(int(g["nfile"])):
        sub = g["f%d_subints" % f].astype(np.float64)[:, None]
        w = g["f%d_weights" % f]
        wn = np.where(w == 0.0, 0.0, 1.0)
        name = "fake%d.fits" % f
        files[name] = DataBunch(
            arch=None, backend="fake_be", backend_delay=0.0, bw=800.0,
            doppler_factors=g["f%d_dfs" % f], DM=float(g["DM0"]), dmc=0,
            epochs=[_MJD(e) for e in g["f%d_epochs" % f]], filename=name,
            flux_prof=np.array([]), freqs=np.tile(g["freqs"], (nsub, 1)),
            frontend="fake_rx", integration_length=60.0 * nsub,
            masks=None, nbin=nbin, nchan=nchan,
            noise_stds=np.array([[get_noise(sub[i, 0], chans=True)]
                                 for i in range(nsub)]),
            npol=1, nsub=nsub, nu0=1500.0,
            ok_ichans=[np.compress(wn[i], list(range(nchan)))
                       for i in range(nsub)],
            ok_isubs=np.arange(nsub), parallactic_angles=np.zeros(nsub),
            phases=None, prof=None, prof_noise=1.0, prof_SNR=100.0,
            Ps=np.ones(nsub) * float(g["P"]),
            SNRs=g["f%d_snrs" % f][:, None, :], source="J1234-5678",
            state="Intensity", subints=sub, subtimes=[60.0] * nsub,
            telescope="GBT", telescope_code="1", weights=w)
        from pulseportraiture_amd.pplib import get_bin_centers
        files[name].phases = get_bin_centers(nbin)
    return files


def _same_printed_number(a, b):
    try:
        fa, fb = float(a), float(b)
    except ValueError:
        return a == b
    dec = len(a.split(".")[1]) if "." in a else 0
    return abs(fa - fb) <= 1.01 * 10 ** (-dec)


def test_get_toas_matches_reference(monkeypatch, tmp_path, capsys):
    import os
    from pulseportraiture_amd import pptoas, pplib
    g = G.gettoas()
    files = _fake_archives(g)
    monkeypatch.setattr(pptoas, "load_data", lambda fn, **kw: files[fn])
    monkeypatch.setattr(pptoas, "_MJD", _MJD)
    meta = tmp_path / "meta.txt"
    meta.write_text("".join(n + "\n" for n in files))
    gm = os.path.join(os.path.dirname(__file__), "golden", "example.gmodel")
    gt = pptoas.GetTOAs(str(meta), gm, quiet=True)
    gt.get_TOAs(quiet=True)
    for f in range(int(g["nfile"])):
        dphi = np.abs(G.phase_diff(gt.phis[f], g["out_phis"][f]))
        assert np.all(dphi < SIG * g["out_phi_errs"][f]), dphi
        assert np.all(np.abs(gt.DMs[f] - g["out_DMs"][f]) <
                      SIG * g["out_DM_errs"][f])
        np.testing.assert_allclose(gt.red_chi2s[f], g["out_red_chi2s"][f],
                                   rtol=RCHI2)
        np.testing.assert_allclose(gt.phi_errs[f], g["out_phi_errs"][f],
                                   rtol=1e-5)
        np.testing.assert_allclose(gt.snrs[f], g["out_snrs"][f], rtol=1e-6)
        np.testing.assert_allclose(np.array(gt.nu_refs[f], dtype=float),
                                   g["out_nu_refs"][f], rtol=1e-6)
        np.testing.assert_allclose(gt.covariances[f], g["out_covariances"][f],
                                   rtol=1e-3, atol=1e-12)
        assert abs(gt.DeltaDM_means[f] - g["out_DeltaDM_means"][f]) < \
            SIG * g["out_DeltaDM_errs"][f]
        np.testing.assert_allclose(gt.DeltaDM_errs[f], g["out_DeltaDM_errs"][f],
                                   rtol=1e-4)
    capsys.readouterr()
    pplib.write_TOAs(gt.TOA_list)
    lines = capsys.readouterr().out.splitlines()
    ref = list(g["out_tim_lines"])
    assert len(lines) == len(ref)
    for a, b in zip(lines, ref):
        ta, tb = a.split(), b.split()
        assert len(ta) == len(tb)
        for i, (x, y) in enumerate(zip(ta, tb)):
            if x.endswith("example.gmodel"):     # -tmplt path differs
                continue
            if i == 1:      # nu_0 (hypersensitive): to 1e-8, see
                assert abs(float(x) / float(y) - 1) < 1e-8, (a, b)
                continue    # test_gpu_fullshape.py
            assert _same_printed_number(x, y), (a, b)


# ------------------------------------------------ full-size properties -----
def test_fullsize_getoas_pipeline_recovers_injected_truth():
    """512x2048 (BASELINE configs[1] shape), device-generated sub-ints, the
    bench pipeline (guess + fit): fitted DMs scatter around the injected
    values with unit pulls, phases at 1500 MHz match, reruns are bitwise
    identical, and a sub-integration's result is independent of its batch."""
    import torch
    from pulseportraiture_amd import engine, synth, _lib
    from pulseportraiture_amd.pplib import guess_fit_freq, phase_transform
    nsub, nchan, nbin = 48, 512, 2048
    b = synth.make_batch(nsub, nchan, nbin, first=1000)
    nu_fit = guess_fit_freq(b["freqs"])
    init = np.zeros((nsub, 5))
    init[:, 1] = synth.DM0
    kw = dict(nu_fits=np.full((nsub, 3), nu_fit), guess=True,
              guess_weights=np.ones((nsub, nchan)),
              guess_DM=np.full(nsub, synth.DM0))
    r1 = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, [1, 1, 0, 0, 0],
        **kw))
    r2 = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, [1, 1, 0, 0, 0],
        **kw))
    np.testing.assert_array_equal(r1["results"], r2["results"])
    I = _lib.RESULT_INDEX
    R = r1["results"]
    assert np.all((R[:, I["status"]].astype(int) & 0xff) == 2)
    pull = (R[:, I["params"]][:, 1] - b["DM_true"]) / R[:, I["param_errs"]][:, 1]
    assert np.sqrt(np.mean(pull ** 2)) < 2.0 and np.all(np.abs(pull) < 6)
    # phase at the 1500 MHz injection reference
    phi1500 = np.array([phase_transform(R[i, I["params"]][0],
                                        R[i, I["params"]][1],
                                        R[i, I["nu_out"]][0], 1500.0,
                                        b["P"][i]) for i in range(nsub)])
    dphi = G.phase_diff(phi1500, b["phi_true"])
    # phi_err at nu_zero is the floor; at 1500 MHz the DM error adds ~2x
    assert np.all(np.abs(dphi) < 10 * R[:, I["param_errs"]][:, 0] + 2e-4)
    # batch independence (same data fitted alone)
    one = engine.results_numpy(engine.fit_batch(
        b["data"][5:6], b["model"], b["freqs"], b["P"][5:6], init[5:6],
        [1, 1, 0, 0, 0], nu_fits=np.full((1, 3), nu_fit), guess=True,
        guess_weights=np.ones((1, nchan)), guess_DM=[synth.DM0]))
    np.testing.assert_array_equal(one["results"][0], R[5])
    # synth keyed by global index: sub 1005 generated alone == in the batch
    b1 = synth.make_batch(1, nchan, nbin, first=1005)
    assert torch.equal(b1["data"][0], b["data"][5])


def test_device_guess_matches_oracle_phase_shift():
    """The on-device GetTOAs phase guess equals the oracle's brute+fmin on
    the dedispersed weighted mean profile (within fmin's xtol)."""
    from pulseportraiture_amd import engine, synth, _lib
    import oracle as O
    from pulseportraiture_amd.pplib import guess_fit_freq
    nsub, nchan, nbin = 4, 64, 512
    b = synth.make_batch(nsub, nchan, nbin, first=77)
    data = b["data"].double().cpu().numpy()
    nu_fit = guess_fit_freq(b["freqs"])
    init = np.zeros((nsub, 5))
    init[:, 1] = synth.DM0
    r = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, [1, 1, 0, 0, 0],
        nu_fits=np.full((nsub, 3), nu_fit), guess=True,
        guess_weights=np.ones((nsub, nchan)), guess_DM=np.full(nsub,
                                                               synth.DM0)))
    for i in range(nsub):
        nu_mean = b["freqs"].mean()
        rot = O.rotate_data(data[i], 0.0, synth.DM0, b["P"][i], b["freqs"],
                            nu_mean)
        prof = np.average(rot, axis=0, weights=np.ones(nchan))
        ph = O.fit_phase_shift(prof, b["model"].mean(axis=0), Ns=100)["phase"]
        ph = O.phase_transform(ph, synth.DM0, nu_mean, nu_fit, b["P"][i],
                               mod=True)
        got = r["results"][i, _lib.RESULT_INDEX["phi_guess"]]
        assert abs(G.phase_diff(got, ph)) < 2e-4, (got, ph)


# ------------------------------------------- wide-band scattering (C3 / C5) --
def _scat_batch(nsub, nchan, nbin, first):
    from pulseportraiture_amd import synth
    from pulseportraiture_amd.pplib import guess_fit_freq, phase_transform
    b = synth.make_batch(nsub, nchan, nbin, first=first, lo=400.0, bw=400.0,
                         tau=5e-3, nu_tau=600.0)
    nu_fit = guess_fit_freq(b["freqs"])
    init = np.zeros((nsub, 5))
    for i in range(nsub):    # start at the injected phase, moved to nu_fit
        init[i, 0] = phase_transform(b["phi_true"][i], b["DM_true"][i],
                                     b["nu_ref"], nu_fit, b["P"][i], mod=True)
    init[:, 1] = synth.DM0
    init[:, 3] = np.log10(1.0 / nbin)           # pptoas.py:488-490
    init[:, 4] = synth.GMODEL_ALPHA
    return b, nu_fit, init


def test_wideband_scattering_2048ch_matches_oracle():
    """configs[4]-style fit (phi, DM, tau, alpha; CHIME-like 400-800 MHz
    band, injected tau = 5e-3 rot at 600 MHz) with 2048 channels -- more
    channel blocks than any golden case -- against the oracle restatement
    on the same float32 data: parameters within 0.01 sigma, chi2_red within
    1e-8 (the reference itself cannot run this width: its dense covariance
    cube, pptoaslib.py:731, would take 2048^3 x 8 B)."""
    import oracle as O
    from pulseportraiture_amd import engine, _lib
    nsub, nchan, nbin = 1, 2048, 256
    b, nu_fit, init = _scat_batch(nsub, nchan, nbin, first=4242)
    flags = [1, 1, 0, 1, 1]
    r = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, flags,
        nu_fits=np.full((nsub, 3), nu_fit), log10_tau=True))
    I = _lib.RESULT_INDEX
    R = r["results"][0]
    data = b["data"][0].double().cpu().numpy()
    ref = O.fit_portrait_full(data, b["model"], list(init[0]), b["P"][0],
                              b["freqs"], nu_fits=(nu_fit,) * 3,
                              fit_flags=flags, log10_tau=True)
    got = dict(params=R[I["params"]], nu_DM=R[I["nu_out"]][0],
               nu_GM=R[I["nu_out"]][1], nu_tau=R[I["nu_out"]][2])
    refd = dict(params=ref["params"], param_errs=ref["param_errs"],
                nu_DM=ref["nu_DM"], nu_GM=ref["nu_GM"], nu_tau=ref["nu_tau"])
    dev = G.param_deviation_sigma(got, refd, b["P"][0], True)
    assert dev.max() < SIG, dev
    assert abs(R[I["red_chi2"]] / ref["red_chi2"] - 1) < RCHI2
    np.testing.assert_allclose(R[I["param_errs"]], ref["param_errs"],
                               rtol=1e-4)
    np.testing.assert_allclose(r["scales"][0], ref["scales"], rtol=1e-4,
                               atol=1e-3 * np.abs(ref["scale_errs"]).min())


def test_chime_shape_16384ch_scattering_fit_properties():
    """configs[4] shape (16384 x 1024, phi+DM+tau+alpha): the fit converges,
    recovers the injected DM / tau / alpha within 6 sigma, is bitwise
    reproducible and independent of its batch."""
    from pulseportraiture_amd import engine, _lib, synth
    nsub, nchan, nbin = 2, 16384, 1024
    b, nu_fit, init = _scat_batch(nsub, nchan, nbin, first=9000)
    flags = [1, 1, 0, 1, 1]
    kw = dict(nu_fits=np.full((nsub, 3), nu_fit), log10_tau=True)
    r1 = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, flags, **kw))
    r2 = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, flags, **kw))
    np.testing.assert_array_equal(r1["results"], r2["results"])
    one = engine.results_numpy(engine.fit_batch(
        b["data"][1:2], b["model"], b["freqs"], b["P"][1:2], init[1:2], flags,
        nu_fits=np.full((1, 3), nu_fit), log10_tau=True))
    np.testing.assert_array_equal(one["results"][0], r1["results"][1])
    I = _lib.RESULT_INDEX
    R = r1["results"]
    assert np.all((R[:, I["status"]].astype(int) & 0xff) == 2)
    p, e = R[:, I["params"]], R[:, I["param_errs"]]
    nuo = R[:, I["nu_out"]][:, 2]
    tau_true = np.log10(5e-3 * (nuo / 600.0) ** synth.GMODEL_ALPHA)
    assert np.all(np.abs((p[:, 1] - b["DM_true"]) / e[:, 1]) < 6)
    assert np.all(np.abs((p[:, 3] - tau_true) / e[:, 3]) < 6)
    assert np.all(np.abs((p[:, 4] - synth.GMODEL_ALPHA) / e[:, 4]) < 6)


# ------------------------------------------------------------- ppalign (C4) --
@pytest.mark.parametrize("nbin", [512, 511])
def test_align_accum_matches_numpy(nbin):
    """ppf_align_accum: sum_s w rotate(x_s, phi_s) per channel (frequency-
    domain accumulation) equals the time-domain rotate-then-sum of the
    oracle to rounding (odd nbin: the unpaired harmonic partials)."""
    import torch
    import oracle as O
    from pulseportraiture_amd import engine
    rng = np.random.default_rng(5)
    nsub, nchan = 37, 12
    x = rng.normal(size=(nsub, nchan, nbin)).astype(np.float32)
    ph = rng.uniform(-0.5, 0.5, size=(nsub, nchan))
    w = rng.uniform(0.1, 2.0, size=(nsub, nchan))
    w[3, 5] = 0.0
    out = torch.zeros((nchan, nbin), dtype=torch.float64, device="cuda")
    ws = torch.zeros(nchan, dtype=torch.float64, device="cuda")
    engine.align_accum(x, ph, w, out, ws)
    engine.align_accum(x, ph, w, out, ws)       # accumulates
    ref = np.zeros((nchan, nbin))
    for s in range(nsub):
        ref += w[s][:, None] * O.rotate_rows(x[s].astype(float), ph[s])
    np.testing.assert_allclose(out.cpu().numpy(), 2 * ref, rtol=0,
                               atol=1e-12 * np.abs(ref).max())
    np.testing.assert_allclose(ws.cpu().numpy(), 2 * w.sum(axis=0), rtol=1e-14)


class _ArchRecorder(object):
    """The PSRCHIVE archive calls of ppalign.py:259-277, recorded."""

    def __init__(self, nchan, nbin):
        self.amps = np.zeros((1, nchan, nbin))
        self.weights = np.full(nchan, -1.0)
        self.dm = None

    def tscrunch(self):
        pass

    def pscrunch(self):
        pass

    def set_dispersion_measure(self, dm):
        self.dm = dm

    def get_npol(self):
        return 1

    def get_nchan(self):
        return self.amps.shape[1]

    def __iter__(self):
        rec = self

        class _S(object):
            def get_Profile(self, ipol, ichan):
                class _P(object):
                    def get_amps(self):
                        return rec.amps[ipol, ichan]
                return _P()

            def set_weight(self, ichan, w):
                rec.weights[ichan] = w
        return iter([_S()])

    def unload(self, outfile):
        self.outfile = outfile


def test_align_archives_matches_reference(monkeypatch):
    """ppalign.align_archives (configs[3] algorithm, 2 iterations, 5 archives
    x 2 sub-ints, one with zapped channels) against the reference's own
    output (tests/golden/align.npz): the aligned portrait to 1e-6 of its peak
    (the fits agree to << 0.01 sigma; a 1e-6 rot phase difference moves this
    portrait by ~1e-4 of its peak), identical channel weights, DM 0."""
    from pulseportraiture_amd import ppalign, pptoas
    c = G.align()
    archives, model_data = G.align_inputs(c)
    rec = _ArchRecorder(int(c["nchan"]), int(c["nbin"]))
    model_data["arch"] = rec
    files = {"arch%d.fits" % i: a for i, a in enumerate(archives)}
    files["guess.fits"] = model_data
    monkeypatch.setattr(pptoas, "load_data", lambda name, **kw: files[name])
    r = ppalign.align_archives(["arch%d.fits" % i for i in
                                range(int(c["nfile"]))], "guess.fits",
                               fit_dm=True, niter=int(c["niter"]),
                               outfile="aligned.fits", quiet=True)
    ref = c["out_aligned"]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(r.port[0], ref, rtol=0, atol=1e-6 * scale)
    np.testing.assert_allclose(rec.amps[0], ref, rtol=0, atol=1e-6 * scale)
    np.testing.assert_array_equal(rec.weights, c["out_weights"])
    assert rec.dm == 0.0 and rec.outfile == "aligned.fits"


# -------------------------------------------------- narrowband TOAs --------
def test_narrowband_toas_match_reference(monkeypatch, tmp_path, capsys):
    """GetTOAs.get_narrowband_TOAs (pptoas.py:794-1189): one FFTFIT per
    usable channel, all channels of an archive in one batched device call,
    against the reference's own run (tests/golden/narrowband.npz): phases
    within 0.01 of their errors, errors / scales / S/N / gof to 1e-6, and
    the .tim lines to their printed precision."""
    import os
    from pulseportraiture_amd import pptoas, pplib
    from pulseportraiture_amd.pplib import DataBunch, get_bin_centers
    g = G.narrowband()
    nsub, nchan, nbin = int(g["nsub"]), int(g["nchan"]), int(g["nbin"])
    files = {}
    for f in range(int(g["nfile"])):
        sub = g["f%d_subints" % f].astype(np.float64)[:, None]
        w = g["f%d_weights" % f]
        wn = np.where(w == 0.0, 0.0, 1.0)
        files["nb%d.fits" % f] = DataBunch(
            arch=None, backend="fake_be", backend_delay=1e-5, bw=800.0,
            doppler_factors=np.ones(nsub), DM=float(g["DM0"]), dmc=0,
            epochs=[_MJD(e) for e in g["f%d_epochs" % f]],
            filename="nb%d.fits" % f, flux_prof=np.array([]),
            freqs=np.tile(g["freqs"], (nsub, 1)), frontend="fake_rx",
            integration_length=60.0 * nsub, masks=None, nbin=nbin,
            nchan=nchan, noise_stds=g["f%d_noise" % f][:, None], npol=1,
            nsub=nsub, nu0=1500.0,
            ok_ichans=[np.compress(wn[i], list(range(nchan)))
                       for i in range(nsub)],
            ok_isubs=np.arange(nsub), parallactic_angles=np.zeros(nsub),
            phases=get_bin_centers(nbin), prof=None, prof_noise=1.0,
            prof_SNR=100.0, Ps=np.ones(nsub) * float(g["P"]),
            SNRs=g["f%d_snrs" % f][:, None, :], source="J1234-5678",
            state="Intensity", subints=sub, subtimes=[60.0] * nsub,
            telescope="GBT", telescope_code="1", weights=w)
    monkeypatch.setattr(pptoas, "load_data", lambda fn, **kw: files[fn])
    monkeypatch.setattr(pptoas, "_MJD", _MJD)
    meta = tmp_path / "meta.txt"
    meta.write_text("".join(n + "\n" for n in files))
    gm = os.path.join(os.path.dirname(__file__), "golden", "example.gmodel")
    gt = pptoas.GetTOAs(str(meta), gm, quiet=True)
    gt.get_narrowband_TOAs(quiet=True)
    for f in range(int(g["nfile"])):
        used = g["out_phi_errs"][f] > 0
        dphi = np.abs(G.phase_diff(gt.phis[f], g["out_phis"][f]))[used]
        assert np.all(dphi < SIG * g["out_phi_errs"][f][used]), dphi
        for key in ("phi_errs", "scales", "scale_errs", "channel_snrs",
                    "channel_red_chi2s"):
            np.testing.assert_allclose(getattr(gt, key)[f],
                                       g["out_" + key][f], rtol=1e-6,
                                       err_msg=key)
    capsys.readouterr()
    pplib.write_TOAs(gt.TOA_list)
    lines = capsys.readouterr().out.splitlines()
    ref = list(g["out_tim_lines"])
    assert len(lines) == len(ref)
    for a, b in zip(lines, ref):
        ta, tb = a.split(), b.split()
        assert len(ta) == len(tb)
        for x, y in zip(ta, tb):
            if x.endswith("example.gmodel"):     # -tmplt path differs
                continue
            assert _same_printed_number(x, y), (a, b)


def _nb_bunch(name, sub, w, noise, snrs, epochs, g, par):
    from pulseportraiture_amd.pplib import DataBunch, get_bin_centers
    nsub = sub.shape[0]
    nchan, nbin = int(g["nchan"]), int(g["nbin"])
    wn = np.where(w == 0.0, 0.0, 1.0)
    return DataBunch(
        arch=None, backend="fake_be", backend_delay=1e-5, bw=800.0,
        doppler_factors=np.ones(nsub), DM=float(g["DM0"]), dmc=0,
        epochs=[_MJD(e) for e in epochs], filename=name,
        flux_prof=np.array([]), freqs=np.tile(g["freqs"], (nsub, 1)),
        frontend="fake_rx", integration_length=60.0 * 3, masks=None,
        nbin=nbin, nchan=nchan, noise_stds=noise[:, None], npol=1, nsub=nsub,
        nu0=1500.0, ok_ichans=[np.compress(wn[i], list(range(nchan)))
                               for i in range(nsub)],
        ok_isubs=np.arange(nsub), parallactic_angles=np.full(nsub, par),
        phases=get_bin_centers(nbin), prof=None, prof_noise=1.0,
        prof_SNR=100.0, Ps=np.ones(nsub) * float(g["P"]),
        SNRs=snrs[:, None, :], source="J1234-5678", state="Intensity",
        subints=sub.astype(np.float64)[:, None],
        subtimes=[60.0 * (3 if nsub == 1 else 1)] * nsub, telescope="GBT",
        telescope_code="1", weights=w)


def test_narrowband_options_match_reference(monkeypatch, tmp_path, capsys):
    """get_narrowband_TOAs' options against the reference's own runs
    (tests/golden/narrowband_opts.npz): print_phase / print_flux raise what
    the reference raises (it reads names that path never defines,
    pptoas.py:1131-1137); tscrunch=True (the loader asked for tscrunched
    archives) with print_parangle and extra flags gives the reference's
    fits and .tim lines."""
    import os
    from pulseportraiture_amd import pptoas, pplib
    g = G.narrowband_opts()
    nf = int(g["nfile"])
    files, ts = {}, {}
    for f in range(nf):
        name = "nb%d.fits" % f
        files[name] = _nb_bunch(name, g["f%d_subints" % f],
                                g["f%d_weights" % f], g["f%d_noise" % f],
                                g["f%d_snrs" % f], g["f%d_epochs" % f], g, 0.0)
        ts[name] = _nb_bunch(name, g["ts_f%d_subints" % f],
                             g["ts_f%d_weights" % f], g["ts_f%d_noise" % f],
                             g["ts_f%d_snrs" % f],
                             [float(g["ts_f%d_epoch" % f])], g, 0.25)
    seen = []

    def load(fn, **kw):
        seen.append(bool(kw.get("tscrunch")))
        return ts[fn] if kw.get("tscrunch") else files[fn]
    monkeypatch.setattr(pptoas, "load_data", load)
    monkeypatch.setattr(pptoas, "_MJD", _MJD)
    meta = tmp_path / "meta.txt"
    meta.write_text("".join(n + "\n" for n in files))
    gm = os.path.join(os.path.dirname(__file__), "golden", "example.gmodel")
    for opt in ("print_phase", "print_flux"):
        gt = pptoas.GetTOAs(str(meta), gm, quiet=True)
        with pytest.raises(Exception) as ei:
            gt.get_narrowband_TOAs(quiet=True, **{opt: True})
        assert "%s: %s" % (ei.type.__name__, ei.value) == \
            str(g["exc_" + opt])
    del seen[:]
    gt = pptoas.GetTOAs(str(meta), gm, quiet=True)
    gt.get_narrowband_TOAs(quiet=True, tscrunch=True, print_parangle=True,
                           addtnl_toa_flags={"pta": "TEST"})
    assert seen and all(seen)
    for f in range(nf):
        used = g["ts_out_phi_errs"][f] > 0
        dphi = np.abs(G.phase_diff(gt.phis[f], g["ts_out_phis"][f]))[used]
        assert np.all(dphi < SIG * g["ts_out_phi_errs"][f][used]), dphi
        for key in ("phi_errs", "scales", "scale_errs", "channel_snrs",
                    "channel_red_chi2s"):
            np.testing.assert_allclose(getattr(gt, key)[f],
                                       g["ts_out_" + key][f], rtol=1e-6,
                                       err_msg=key)
    capsys.readouterr()
    pplib.write_TOAs(gt.TOA_list)
    lines = capsys.readouterr().out.splitlines()
    ref = list(g["ts_out_tim_lines"])
    assert len(lines) == len(ref)
    for a, b in zip(lines, ref):
        ta, tb = a.split(), b.split()
        assert len(ta) == len(tb)
        for x, y in zip(ta, tb):
            if x.endswith("example.gmodel"):     # -tmplt path differs
                continue
            assert _same_printed_number(x, y), (a, b)


# ------------------------------------------------------ channel zapping -----
def _zap_files(g):
    from pulseportraiture_amd.pplib import DataBunch, get_bin_centers
    nsub, nchan, nbin = int(g["nsub"]), int(g["nchan"]), int(g["nbin"])
    files = {}
    for f in range(int(g["nfile"])):
        sub = g["f%d_subints" % f].astype(np.float64)[:, None]
        w = g["f%d_weights" % f]
        wn = np.where(w == 0.0, 0.0, 1.0)
        files["zap%d.fits" % f] = DataBunch(
            arch=None, backend="fake_be", backend_delay=0.0, bw=800.0,
            doppler_factors=g["f%d_dfs" % f], DM=float(g["DM0"]), dmc=0,
            epochs=[_MJD(e) for e in g["f%d_epochs" % f]],
            filename="zap%d.fits" % f, flux_prof=np.array([]),
            freqs=np.tile(g["freqs"], (nsub, 1)), frontend="fake_rx",
            integration_length=60.0 * nsub,
            masks=np.einsum("ij,k", wn, np.ones(nbin))[:, None], nbin=nbin,
            nchan=nchan, noise_stds=g["f%d_noise" % f][:, None], npol=1,
            nsub=nsub, nu0=1500.0,
            ok_ichans=[np.compress(wn[i], list(range(nchan)))
                       for i in range(nsub)],
            ok_isubs=np.arange(nsub), parallactic_angles=np.zeros(nsub),
            phases=get_bin_centers(nbin), prof=None, prof_noise=1.0,
            prof_SNR=100.0, Ps=np.ones(nsub) * float(g["P"]),
            SNRs=g["f%d_snrs" % f][:, None, :], source="J1234-5678",
            state="Intensity", subints=sub, subtimes=[60.0] * nsub,
            telescope="GBT", telescope_code="1", weights=w)
    return files


def test_resid_chi2_kernel_matches_oracle_on_reference_fit():
    """ppf_resid_chi2_batch against the oracle restatement of show_fit +
    get_red_chi2, fed the reference's own fitted parameters
    (tests/golden/zap.npz): every channel chi^2 to 1e-10 relative, fp32 and
    fp64 inputs, and the reference's own chi^2s to 1e-9."""
    import oracle.ppfit_oracle as OO
    from pulseportraiture_amd import engine, pplib as PL
    import os
    g = G.zap()
    nsub, nchan, nbin = int(g["nsub"]), int(g["nchan"]), int(g["nbin"])
    P, freqs = float(g["P"]), g["freqs"]
    gm = os.path.join(os.path.dirname(__file__), "golden", "example.gmodel")
    _, _, model = PL.read_model(gm, PL.get_bin_centers(nbin), freqs, P,
                                quiet=True)
    D = 0.000241 ** -1
    rows, ph, mi, sc, er, ref = [], [], [], [], [], []
    for f in range(int(g["nfile"])):
        w = g["f%d_weights" % f]
        for s in range(nsub):
            ok = np.where(w[s] != 0)[0]
            DM = g["out_DMs"][f][s] / g["out_doppler_fs"][f][s]
            nu_DM = g["out_nu_refs"][f][s][0]
            rows.append(g["f%d_subints" % f][s, ok])
            ph.append(g["out_phis"][f][s] + D * DM * (freqs[ok] ** -2 -
                                                      nu_DM ** -2) / P)
            mi.append(ok)
            sc.append(g["out_scales"][f][s][ok])
            er.append(g["f%d_noise" % f][s][ok])
            ref.append(g["chi2"][0][f][s])
    rows, ph, mi = np.concatenate(rows), np.concatenate(ph), \
        np.concatenate(mi).astype(np.int32)
    sc, er, ref = np.concatenate(sc), np.concatenate(er), np.concatenate(ref)
    want = OO.channel_red_chi2s(rows.astype(np.float64), ph, model[mi], sc,
                                er, nbin - 2)
    for rr in (rows, rows.astype(np.float64)):
        got = engine.resid_chi2_rows(rr, ph, model, mi, sc, er,
                                     nbin - 2).cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=1e-10, atol=0)
        np.testing.assert_allclose(got, ref, rtol=1e-9, atol=0)
    with pytest.raises(ValueError):
        engine.resid_chi2_rows(rows, ph, model, mi + nchan, sc, er, nbin - 2)


def test_channels_to_zap_matches_reference(monkeypatch, tmp_path):
    """GetTOAs.get_TOAs then get_channels_to_zap (pptoas.py:1266-1343) for
    the four (S/N, chi^2, iterate) settings of make_golden_zap.py: channel
    chi^2s within 1e-5 relative of the reference's run (the fitted
    parameters themselves agree to 1e-3 sigma) and the zap lists, in the
    reference's order, identical."""
    import os
    from pulseportraiture_amd import pptoas
    g = G.zap()
    files = _zap_files(g)
    monkeypatch.setattr(pptoas, "load_data", lambda fn, **kw: files[fn])
    monkeypatch.setattr(pptoas, "_MJD", _MJD)
    meta = tmp_path / "meta.txt"
    meta.write_text("".join(n + "\n" for n in files))
    gm = os.path.join(os.path.dirname(__file__), "golden", "example.gmodel")
    gt = pptoas.GetTOAs(str(meta), gm, quiet=True)
    gt.get_TOAs(quiet=True)
    nfile = int(g["nfile"])
    for ic, (snr_t, rchi_t, it) in enumerate(g["calls"]):
        gt.get_channels_to_zap(SNR_threshold=snr_t, rchi2_threshold=rchi_t,
                               iterate=bool(it))
        for f in range(nfile):
            for s in range(int(g["nsub"])):
                np.testing.assert_allclose(
                    gt.channel_red_chi2s[ic * nfile + f][s],
                    g["chi2"][ic][f][s], rtol=1e-5, atol=0)
                assert [int(v) for v in gt.zap_channels[ic * nfile + f][s]] \
                    == g["zap"][ic][f][s], (ic, f, s)
    port, model, ok, freqs, noise = gt.show_fit("zap1.fits", isub=1,
                                                show=False, return_fit=True)
    assert port.shape == model.shape == (int(g["nchan"]), int(g["nbin"]))
    bad = np.setdiff1d(np.arange(int(g["nchan"])), ok)
    assert np.all(port[bad] == 0.0)
    # the ppzap.py command line, model-based branch: get_TOAs +
    # get_channels_to_zap(8, 1.3, iterate) -> paz commands (to a file),
    # identical to the reference's print_paz_cmds of its own zap lists
    from pulseportraiture_amd import ppzap
    paz = tmp_path / "paz.txt"
    assert ppzap.main(["-d", str(meta), "-m", gm, "-o", str(paz),
                       "--quiet"]) == 0
    assert paz.read_text() == str(g["ppzap_paz_out"][0])


# ------------------------------------------------ device model templates ---
# x max|portrait|: exp/log/pow and FFT rounding differ from NumPy's by an
# ulp; a 1-ulp change of an evolved loc moves a sub-bin Gaussian
# (sigma = 1.7e-4 rot in mixed_scat_48x1024) by ~ulp/sigma, i.e. ~1e-12
GAUSS_ATOL = 1e-11


def test_gauss_portraits_match_reference(ppl, tmp_path):
    """k_gauss_port (ppf_gauss_portrait_batch) against the reference's own
    gen_gaussian_portrait / gaussian_profile / read_model outputs
    (tests/golden/make_golden_gauss.py), one portrait per call and all
    same-shape portraits in one batched launch."""
    from pulseportraiture_amd import engine
    g = G.gauss()
    devs = {}
    for name in g["cases"]:
        c = G.gauss_case(g, str(name))
        nbin = c["out"].shape[1]
        out = ppl.gen_gaussian_portrait(c["code"], c["params"], c["alpha"],
                                        np.zeros(nbin), c["freqs"],
                                        c["nu_ref"])
        devs[str(name)] = np.abs(out - c["out"]).max() / \
            np.abs(c["out"]).max()
        # zeroed rows / bins stay exactly zero where the reference's are
        if c["params"][1] == 0.0:
            assert np.array_equal(out == 0.0, c["out"] == 0.0), name
    print("relative max deviation per case:", devs)
    assert max(devs.values()) <= GAUSS_ATOL, devs
    for i in range(int(g["nprof"])):
        nbin, loc, wid = g["prof%d__args" % i]
        ref = g["prof%d__out" % i]
        got = ppl.gaussian_profile(int(nbin), loc, wid)
        np.testing.assert_allclose(got, ref, rtol=0, atol=GAUSS_ATOL)
    # batch: three portraits of one shape (different freqs, nu_ref, tau)
    c = G.gauss_case(g, "example_64x512")
    nbin = c["out"].shape[1]
    prm = np.stack([c["params"]] * 3)
    prm[1, 1] = 5.0
    prm[2, 0] = 0.3
    freqs = np.stack([c["freqs"], c["freqs"][::-1], c["freqs"] * 0.5])
    batch = engine.gauss_portraits(c["code"], prm, [c["alpha"]] * 3, freqs,
                                   [c["nu_ref"], 1500.0, 700.0], nbin)
    batch = batch.cpu().numpy()
    import oracle as O
    for i, nr in enumerate([c["nu_ref"], 1500.0, 700.0]):
        ref = O.gen_gaussian_portrait(c["code"], prm[i], c["alpha"],
                                      np.zeros(nbin), freqs[i], nr)
        np.testing.assert_allclose(batch[i], ref, rtol=0,
                                   atol=GAUSS_ATOL * np.abs(ref).max())
    # read_model with a TAU line: parse, TAU [s] -> [bin], device portrait
    gm = tmp_path / "tau.gmodel"
    gm.write_text(str(g["readmodel__text"]))
    ref = g["readmodel__out"]
    _, ngauss, model = ppl.read_model(str(gm), ppl.get_bin_centers(ref.shape[1]),
                                      g["readmodel__freqs"],
                                      float(g["readmodel__P"]), quiet=True)
    assert ngauss == 2
    np.testing.assert_allclose(model, ref, rtol=0,
                               atol=GAUSS_ATOL * np.abs(ref).max())
    with pytest.raises(KeyError):     # evolve_parameter's unknown code
        ppl.gen_gaussian_portrait("020", c["params"], -4.0, np.zeros(nbin),
                                  c["freqs"], c["nu_ref"])


@pytest.mark.parametrize("nbin", [16384, 8193])
def test_resid_chi2_long_rows_match_oracle(nbin):
    """The zap / show_fit per-channel reduced chi^2 (pplib.py:754-779 after
    rotate_portrait_full) at nbin past the LDS transforms (round 6: the
    rotation on the long transforms) against the oracle, rtol 1e-12."""
    from pulseportraiture_amd import engine
    import oracle as O
    rng = np.random.default_rng(nbin)
    rows = rng.normal(size=(5, nbin))
    mrows = rng.normal(size=(2, nbin))
    phs = rng.uniform(-0.5, 0.5, 5)
    mi = np.array([0, 1, 0, 1, 1], dtype=np.int32)
    sc = rng.uniform(0.5, 2.0, 5)
    er = rng.uniform(0.5, 1.5, 5)
    got = engine.resid_chi2_rows(rows.astype(np.float32), phs, mrows, mi, sc,
                                 er, nbin - 2).cpu().numpy()
    want = O.channel_red_chi2s(rows.astype(np.float32).astype(np.float64),
                               phs, mrows[mi], sc, er, nbin - 2)
    np.testing.assert_allclose(got, want, rtol=1e-12)


@pytest.mark.parametrize("nbin", [16384, 10002])
def test_gauss_portraits_long_scattered_match_oracle(nbin):
    """Scattered Gaussian portraits at even nbin past the LDS transforms
    (round 6: the rows built per bin in LDS, then the convolution with
    1 / (1 + 2 pi i k tau_n) on the long transforms) against the oracle's
    gen_gaussian_portrait (pplib.py:900-960: rfft, scattering_portrait_FT,
    irfft), in one batch with an unscattered portrait; scattered odd rows
    past 4095 are refused (the reference's nbin - 1-bin irfft)."""
    from pulseportraiture_amd import engine
    import oracle as O
    g = G.gauss()
    c = G.gauss_case(g, "example_64x512")
    prm = np.stack([c["params"]] * 2)
    prm[0, 1] = 40.0                      # tau [bin] at nu_ref
    prm[1, 1] = 0.0
    freqs = np.stack([c["freqs"][::8], c["freqs"][::8] * 0.8])
    nus = [c["nu_ref"], 1300.0]
    batch = engine.gauss_portraits(c["code"], prm, [c["alpha"]] * 2, freqs,
                                   nus, nbin).cpu().numpy()
    for i in range(2):
        ref = O.gen_gaussian_portrait(c["code"], prm[i], c["alpha"],
                                      np.zeros(nbin), freqs[i], nus[i])
        np.testing.assert_allclose(batch[i], ref, rtol=0,
                                   atol=GAUSS_ATOL * np.abs(ref).max())
    with pytest.raises(NotImplementedError):
        engine.gauss_portraits(c["code"], prm[:1], [c["alpha"]], freqs[:1],
                               nus[:1], 8193)


# ------------------------------------------------------ harmonic cutoff ---
def _cut_fraction(model):
    """Fraction of harmonics k_model_cut keeps (numpy restatement of its
    rule: last k with |M_k|^2 > 1e-28 max |M|^2, k = 0 excluded)."""
    mp = np.abs(np.fft.rfft(model, axis=1)) ** 2
    mp[:, 0] = 0.0
    above = mp > 1e-28 * mp.max(axis=1, keepdims=True)
    kc = mp.shape[1] - np.argmax(above[:, ::-1], axis=1)
    return kc.mean() / mp.shape[1]


@pytest.mark.parametrize("flags,nbin", [([1, 1, 0, 0, 0], 2048),
                                        ([1, 1, 1, 1, 1], 2048),
                                        ([1, 1, 0, 0, 0], 3001),
                                        ([1, 1, 1, 1, 1], 1001)])
def test_harmonic_cutoff_fits_match_oracle(flags, nbin):
    """The example template at 1100-1900 MHz x 2048 bins has no model power
    above ~1e-14 of its peak past harmonic ~430, so the device sums stop
    there (k_model_cut; DESIGN.md section 4, deviation 7) while the oracle
    sums all 1025 harmonics: the phase+DM moment path (with the device guess)
    and the full scattering fit agree with the oracle to 0.01 sigma and
    chi2_red to 1e-8.  Also at odd nbin (3001, a prime: one generic-radix
    stage of radix 3001; 1001 = 7 x 11 x 13), whose synthetic rows,
    guess profile and spectra all take the full-length complex transforms."""
    import oracle as O
    from pulseportraiture_amd import engine, synth, _lib
    from pulseportraiture_amd.pplib import guess_fit_freq, phase_transform
    nsub, nchan = 2, 128
    scat = flags[3] == 1
    b = synth.make_batch(nsub, nchan, nbin, first=515,
                         tau=2e-3 if scat else 0.0,
                         nu_tau=1500.0 if scat else None)
    assert _cut_fraction(b["model"]) < 0.5          # the cut is active
    nu_fit = guess_fit_freq(b["freqs"])
    init = np.zeros((nsub, 5))
    init[:, 1] = synth.DM0
    if scat:
        for i in range(nsub):
            init[i, 0] = phase_transform(b["phi_true"][i], b["DM_true"][i],
                                         b["nu_ref"], nu_fit, b["P"][i],
                                         mod=True)
        init[:, 3] = np.log10(1.0 / nbin)
        init[:, 4] = synth.GMODEL_ALPHA
    res = engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, flags,
        nu_fits=np.full((nsub, 3), nu_fit), log10_tau=scat,
        guess=not scat, guess_weights=np.ones((nsub, nchan)),
        guess_DM=np.full(nsub, synth.DM0))
    r = engine.results_numpy(res)
    I = _lib.RESULT_INDEX
    if not scat:
        # the oracle's own GetTOAs guess (dedispersed mean profile, brute +
        # fmin), independent of the device's
        og = O.get_toas_archive(b["data"].double().cpu().numpy(), b["model"],
                                np.tile(b["freqs"], (nsub, 1)),
                                np.ones((nsub, nchan)), np.ones((nsub, nchan)),
                                b["P"], synth.DM0, np.ones(nsub))
    for i in range(nsub):
        R = r["results"][i]
        data = b["data"][i].double().cpu().numpy()
        if scat:
            ref = O.fit_portrait_full(data, b["model"], list(init[i]),
                                      b["P"][i], b["freqs"],
                                      nu_fits=(nu_fit,) * 3, fit_flags=flags,
                                      log10_tau=scat)
        else:
            ref = dict(params=[og["phis"][i], og["DMs"][i], 0.0, 0.0, 0.0],
                       param_errs=og["param_errs"][i],
                       nu_DM=og["nu_refs"][i][0], nu_GM=og["nu_refs"][i][1],
                       nu_tau=og["nu_refs"][i][2], red_chi2=og["red_chi2s"][i])
        got = dict(params=R[I["params"]], nu_DM=R[I["nu_out"]][0],
                   nu_GM=R[I["nu_out"]][1], nu_tau=R[I["nu_out"]][2])
        refd = dict(params=ref["params"], param_errs=ref["param_errs"],
                    nu_DM=ref["nu_DM"], nu_GM=ref["nu_GM"],
                    nu_tau=ref["nu_tau"])
        dev = G.param_deviation_sigma(got, refd, b["P"][i], scat)
        assert dev.max() < SIG, (i, dev)
        assert abs(R[I["red_chi2"]] / ref["red_chi2"] - 1) < RCHI2
        np.testing.assert_allclose(R[I["param_errs"]], ref["param_errs"],
                                   rtol=1e-4)


@pytest.mark.gpu
def test_stager_pinned_and_pageable_sources_upload_the_same_rows():
    """GetTOAs' stager: an archive already in page-locked memory
    (engine.pinned_host_array, bench.py --fit gettoas --pinned) is uploaded
    straight from it; a pageable one through the stager's own pinned
    buffers (float64 rows that survive float32 go up as float32)."""
    import torch
    from pulseportraiture_amd import engine, pptoas
    rng = np.random.default_rng(5)
    a = rng.standard_normal((3, 16, 64)).astype(np.float32)
    p = engine.pinned_host_array(a.shape, np.float32)
    p[...] = a
    assert torch.from_numpy(p).is_pinned()
    st = pptoas._Stager()
    try:
        t_pin = st.stage(p).wait()
        t_pag = st.stage(a).wait()
        t_f64 = st.stage(a.astype(np.float64)).wait()
        torch.cuda.synchronize()
        for t in (t_pin, t_pag, t_f64):
            assert t.dtype == torch.float32 and t.is_cuda
            np.testing.assert_array_equal(t.cpu().numpy(), a)
    finally:
        st.close()


@pytest.mark.gpu
def test_copy_from_pinned_and_stage_host():
    """ppf_copy_from_pinned (the fit inputs' kernel copy out of page-locked
    memory, 16-B body + byte tail) moves every byte; engine._stage_host
    returns the same arrays through it as through a copy-engine transfer;
    a pageable source is refused."""
    import ctypes
    import torch
    from pulseportraiture_amd import _lib, engine
    dev = engine.device()
    lib, ctx = _lib.load(), _lib.context(dev.index)
    rng = np.random.default_rng(9)
    for n in (16, 48, 1000, 4096 + 7, (3 << 20) + 13):
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        h.numpy()[:] = rng.integers(0, 256, n, dtype=np.uint8)
        d = torch.full((n + 64,), 0x5A, dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream(dev)
        assert lib.ppf_copy_from_pinned(
            ctx, ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(h.data_ptr()),
            n, ctypes.c_void_p(s.cuda_stream)) == 0
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        np.testing.assert_array_equal(got[:n], h.numpy())
        assert (got[n:] == 0x5A).all()
    pageable = np.zeros(64, dtype=np.uint8)
    d = torch.empty(64, dtype=torch.uint8, device=dev)
    assert lib.ppf_copy_from_pinned(
        ctx, ctypes.c_void_p(d.data_ptr()), pageable.ctypes.data, 64,
        ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) != 0
    items = [(rng.standard_normal((7, 33)), torch.float64),
             (rng.integers(0, 2, (7, 33)).astype(np.uint8), torch.uint8),
             (np.arange(7, dtype=np.int32), torch.int32),
             (rng.standard_normal(5).astype(np.float32), torch.float32)]
    outs = {}
    for kern in (True, False):
        engine._STAGE_KERNEL = kern
        try:
            outs[kern] = [t.cpu().numpy() for t in engine._stage_host(items, dev)]
        finally:
            engine._STAGE_KERNEL = True
    for (a, _), k, c in zip(items, outs[True], outs[False]):
        np.testing.assert_array_equal(k, a)
        np.testing.assert_array_equal(c, a)


@pytest.mark.gpu
def test_lane_trust_region_step_equals_wave_step():
    """Scattering fits of a batch large enough for the lane-per-sub-int
    trust-region step (k_tr_step_l + k_tr_gates: nsub >= 2048, nchan <=
    2048) equal, bitwise, the same sub-ints fitted in a small batch (the
    wave-per-sub-int k_tr_step): a sub-int's fit does not depend on its
    batch, and with one channel block the block sums agree exactly."""
    from pulseportraiture_amd import engine
    nsub, nchan, nbin = 2048, 32, 128
    b, nu_fit, init = _scat_batch(nsub, nchan, nbin, first=777)
    flags = [1, 1, 0, 1, 1]
    kw = dict(nu_fits=np.full((nsub, 3), nu_fit), log10_tau=True)
    big = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, flags, **kw))
    k = 24
    small = engine.results_numpy(engine.fit_batch(
        b["data"][:k], b["model"], b["freqs"], b["P"][:k], init[:k], flags,
        nu_fits=kw["nu_fits"][:k], log10_tau=True))
    for key in ("results", "scales", "scale_errs", "channel_snrs",
                "covariance"):
        np.testing.assert_array_equal(small[key], big[key][:k], err_msg=key)


def test_lane_trust_region_step_equals_wave_step_multiblock():
    """As above with 1024 channels: four 256-channel block partials per
    sub-int, where a block-order sum and the wave reduction's pairwise tree
    round differently.  k_tr_step_l adds them in the tree's
    order, so the big batch equals the small one bitwise."""
    from pulseportraiture_amd import engine
    nsub, nchan, nbin = 2048, 1024, 128
    b, nu_fit, init = _scat_batch(nsub, nchan, nbin, first=991)
    flags = [1, 1, 0, 1, 1]
    kw = dict(nu_fits=np.full((nsub, 3), nu_fit), log10_tau=True)
    big = engine.results_numpy(engine.fit_batch(
        b["data"], b["model"], b["freqs"], b["P"], init, flags, **kw))
    k = 16
    small = engine.results_numpy(engine.fit_batch(
        b["data"][:k], b["model"], b["freqs"], b["P"][:k], init[:k], flags,
        nu_fits=kw["nu_fits"][:k], log10_tau=True))
    for key in ("results", "scales", "scale_errs", "channel_snrs",
                "covariance"):
        np.testing.assert_array_equal(small[key], big[key][:k], err_msg=key)


@pytest.mark.parametrize("nbin", [511, 1001])
def test_odd_nbin_block_kernels_match_oracle(ppl, nbin):
    """The block-FFT kernels at odd nbin (rfft_len: nbin complex points,
    X_k = Z_k, inverse from the Hermitian-filled buffer) against the
    oracle's NumPy restatements: fit_phase_shift (pplib.py:2136-2182),
    the per-channel reduced chi^2 of get_channels_to_zap (pplib.py:754-779),
    and gen_gaussian_portrait with and without scattering
    (pplib.py:886-963)."""
    import oracle as O
    from pulseportraiture_amd import engine
    rng = np.random.default_rng(nbin)
    # fit_phase_shift
    ph = np.linspace(0, 1, nbin, endpoint=False)
    model = np.exp(-0.5 * ((ph - 0.4) / 0.03) ** 2) + \
        0.3 * np.exp(-0.5 * ((ph - 0.55) / 0.05) ** 2)
    data = np.stack([O.rotate_rows(model[None, :] * 2.5, [-s])[0] +
                     rng.normal(scale=0.05, size=nbin)
                     for s in (0.123, -0.31, 0.0)])
    got = engine.phase_shift_batch(data, model).cpu().numpy()
    for i in range(len(data)):
        want = O.fit_phase_shift(data[i], model)
        assert abs(G.phase_diff(got[i, 0], want["phase"])) < \
            SIG * want["phase_err"], (i, got[i], want)
        assert abs(got[i, 1] / want["phase_err"] - 1) < 1e-4
        assert abs(got[i, 2] / want["scale"] - 1) < 1e-6
        assert abs(got[i, 4] / want["snr"] - 1) < 1e-6
    # per-channel reduced chi^2 after rotation
    rows = rng.normal(size=(6, nbin))
    mrows = rng.normal(size=(2, nbin))
    phs = rng.uniform(-0.5, 0.5, 6)
    mi = np.array([0, 1, 0, 1, 1, 0], dtype=np.int32)
    sc = rng.uniform(0.5, 2.0, 6)
    er = rng.uniform(0.5, 1.5, 6)
    got = engine.resid_chi2_rows(rows, phs, mrows, mi, sc, er, 7.0)
    want = O.channel_red_chi2s(rows, phs, mrows[mi], sc, er, 7.0)
    np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-12)
    # Gaussian portraits: the example template, with and without tau
    g = G.gauss()
    c = G.gauss_case(g, "example_64x512")
    for tau in (0.0, 0.02):
        prm = np.array(c["params"], dtype=float)
        prm[1] = tau
        got = ppl.gen_gaussian_portrait(c["code"], prm, c["alpha"],
                                        np.zeros(nbin), c["freqs"],
                                        c["nu_ref"])
        want = O.gen_gaussian_portrait(c["code"], prm, c["alpha"],
                                       np.zeros(nbin), c["freqs"],
                                       c["nu_ref"])
        # (with tau the reference's length-less irfft returns nbin - 1 bins)
        assert got.shape == want.shape == (len(c["freqs"]), nbin - (tau != 0))
        assert np.abs(got - want).max() <= GAUSS_ATOL * np.abs(want).max()


@pytest.mark.parametrize("nbin,log10_tau", [(512, True), (1024, False)])
def test_show_fit_scattered_model_on_device(nbin, log10_tau):
    """show_fit / get_channels_to_zap's model for a fit with scattering
    (pptoas.py:1455-1459): the reference convolves the un-scattered portrait
    with the fitted kernel on the host, irfft(B(tau (nu / nu_ref_tau)^alpha)
    rfft(model)); the drop-in builds the same portrait on the device as
    gen_gaussian_portrait's scattered branch with tau moved to the model's
    reference frequency.  Checked against that host arithmetic (the zap
    goldens hold no scattering fit: parity of this branch is against the
    reference's formula, not a reference run)."""
    import os
    from pulseportraiture_amd import pptoas, pplib
    from pulseportraiture_amd.pplib import DataBunch
    gm = os.path.join(os.path.dirname(__file__), "golden", "example.gmodel")
    nchan = 48
    freqs = np.linspace(1150.0, 1850.0, nchan)
    P = 1.0 / 345.67890123456789
    gt = pptoas.GetTOAs.__new__(pptoas.GetTOAs)
    gt.modelfile, gt.is_FITS_model = gm, False
    gt.add_instrumental_response = False
    gt.ird = {"DM": 0.0, "wids": [], "irf_types": []}
    gt.log10_tau = log10_tau
    tau_rot, alpha, nu_tau = 3.1e-3, -3.7, 1432.5
    gt.taus = [[np.log10(tau_rot) if log10_tau else tau_rot]]
    gt.alphas = [[alpha]]
    gt.nu_refs = [[(1400.0, 1400.0, nu_tau)]]
    data = DataBunch(freqs=freqs[None, :], phases=pplib.get_bin_centers(nbin),
                     Ps=np.array([P]), nbin=nbin)
    _, got = gt._fit_model(data, 0, 0, quiet=True)
    (_, code, nu_ref, _, gparams, _, _, _) = pplib.read_model(gm, quiet=True)
    g0 = np.copy(gparams)
    g0[1] = 0.0
    base = pplib.gen_gaussian_portrait(code, g0, 0.0, data.phases, freqs,
                                       nu_ref)
    want = np.fft.irfft(pplib.scattering_portrait_FT(
        pplib.scattering_times(tau_rot, alpha, freqs, nu_tau), nbin) *
        np.fft.rfft(base, axis=1), axis=1)
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, atol=1e-11 * np.abs(want).max(),
                               rtol=0)

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
    for nb in (256, 2048):
        np.testing.assert_allclose(
            ppl.get_noise(m["noise_in_%d" % nb], chans=True),
            m["noise_out_%d" % nb], rtol=1e-12)
    with pytest.raises(NotImplementedError):     # nbin must be a power of 2
        ppl.get_noise(m["noise_in_1000"], chans=True)


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


def test_rotate_round_trip_and_bad_shapes(ppl, capsys):
    x = np.random.default_rng(5).normal(size=(4, 2048))
    y = ppl.rotate_data(ppl.rotate_data(x, 0.3141), -0.3141)
    np.testing.assert_allclose(y, x, atol=1e-11)
    assert ppl.rotate_data(x, 0.1, 10.0, [1.0, 2.0], np.ones(4) * 1400.0) == 0
    assert "Wrong shape for array of periods." in capsys.readouterr().out


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


def test_masked_channels_equal_subset_fit(ppt):
    """Ragged channel masks in the batch == fitting the channel subset."""
    from pulseportraiture_amd import engine
    c = G.full_case("pd_128x1024")
    a = G.full_case_args(c)
    rng = np.random.default_rng(11)
    keep = np.ones(128, dtype=bool)
    keep[rng.choice(128, 17, replace=False)] = False
    sub = ppt.fit_portrait_full(c["data"][keep], a["model_port"][keep],
                                a["init_params"], a["P"], a["freqs"][keep],
                                a["nu_fits"], a["nu_outs"],
                                a["errs"][keep], a["fit_flags"])
    res = engine.results_numpy(engine.fit_batch(
        c["data"][None], a["model_port"][None], a["freqs"][None], [a["P"]],
        np.asarray(a["init_params"])[None], a["fit_flags"],
        nu_fits=np.asarray(a["nu_fits"])[None], errs=a["errs"][None],
        chan_mask=keep[None].astype(np.uint8)))
    I = G.np  # noqa
    from pulseportraiture_amd import _lib
    R = res["results"][0]
    np.testing.assert_allclose(R[_lib.RESULT_INDEX["params"]], sub.params,
                               rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(res["scales"][0][keep], sub.scales, rtol=1e-10)
    assert np.all(res["scales"][0][~keep] == 0.0)

"""CPU: the oracle (NumPy/SciPy restatement) against golden vectors produced by
the reference itself (tests/golden/make_golden.py).  Pins the checker."""
import numpy as np
import pytest

import goldens as G
import oracle as O

FULL = G.case_names("fit_portrait_full.npz")
# the 512x2048 case takes ~1 s in the oracle; keep the CPU suite fast but
# still cover it once
FULL_FAST = [n for n in FULL]


@pytest.mark.parametrize("name", FULL_FAST)
def test_fit_portrait_full_oracle_vs_reference(name):
    c = G.full_case(name)
    a = G.full_case_args(c)
    msgs = []
    r = O.fit_portrait_full(a["data_port"], a["model_port"], a["init_params"],
                            a["P"], a["freqs"], a["nu_fits"], a["nu_outs"],
                            a["errs"], a["fit_flags"], a["log10_tau"],
                            a["option"], messages=msgs)
    ref = G.ref_bunch(c)
    dev = G.param_deviation_sigma(r, ref, a["P"], a["log10_tau"])
    # the restatement runs the same SciPy trust-ncg: far inside the bar
    assert dev.max() < 1e-3, dev
    assert abs(r["red_chi2"] / c["out_red_chi2"] - 1) < 1e-12
    assert abs(r["nu_DM"] / ref["nu_DM"] - 1) < 1e-6
    np.testing.assert_allclose(r["param_errs"], c["out_param_errs"],
                               rtol=1e-6)
    np.testing.assert_allclose(r["scales"], c["out_scales"], rtol=1e-6,
                               atol=1e-9)
    np.testing.assert_allclose(r["scale_errs"], c["out_scale_errs"],
                               rtol=1e-6)
    np.testing.assert_allclose(r["snr"], c["out_snr"], rtol=1e-9)
    np.testing.assert_allclose(r["channel_snrs"], c["out_channel_snrs"],
                               rtol=1e-6, atol=1e-9)
    cm = c["out_covariance_matrix"]
    np.testing.assert_allclose(r["covariance_matrix"], cm, rtol=1e-5,
                               atol=1e-9 * np.abs(cm).max())
    assert ("Approximating zero-covariance frequencies..." in msgs) == \
        ("Approximating" in str(c["stdout"]))


@pytest.mark.parametrize("name", G.case_names("fit_portrait.npz"))
def test_fit_portrait_oracle_vs_reference(name):
    c = G.fp_case(name)
    errs = None if np.all(np.isnan(c["errs"])) else c["errs"]
    r = O.fit_portrait(c["data"].astype(float), c["model"].astype(float),
                       c["init"], float(c["P"]), c["freqs"], None, None, errs)
    assert abs(G.phase_diff(r["phase"], c["out_phase"])) < \
        0.01 * c["out_phase_err"]
    assert abs(r["DM"] - c["out_DM"]) < 0.01 * c["out_DM_err"]
    assert abs(r["red_chi2"] / c["out_red_chi2"] - 1) < 1e-10
    np.testing.assert_allclose(r["scales"], c["out_scales"], rtol=1e-6)
    np.testing.assert_allclose(r["snr"], c["out_snr"], rtol=1e-9)


def test_rotate_and_noise_oracle_vs_reference():
    m = G.misc()
    P0 = 1.0 / 345.67890123456789
    np.testing.assert_allclose(O.rotate_data(m["rot_prof"], 0.123),
                               m["rot1_dm0"], atol=1e-12)
    np.testing.assert_allclose(O.rotate_data(m["rot_port"], -0.377),
                               m["rot2_dm0"], atol=1e-12)
    np.testing.assert_allclose(O.rotate_data(m["rot_cube"], 0.05),
                               m["rot4_dm0"], atol=1e-12)
    np.testing.assert_allclose(
        O.rotate_data(m["rot_prof"], 0.1, 10.0, P0, 1300.0, 1500.0),
        m["rot1_dm"], atol=1e-12)
    np.testing.assert_allclose(
        O.rotate_data(m["rot_port"], 0.2, 34.5, P0, m["rot_freqs"], 1500.0),
        m["rot2_dm"], atol=1e-12)
    np.testing.assert_allclose(
        O.rotate_data(m["rot_cube"], -0.3, 12.5, m["rot_Ps"], m["rot_freqs"],
                      1400.0), m["rot4_dm"], atol=1e-12)
    np.testing.assert_allclose(
        O.rotate_data(m["rot_cube"], 0.01, 5.0, m["rot_Ps"], m["rot_freqs2"],
                      np.inf), m["rot4_dm_f2"], atol=1e-12)
    np.testing.assert_allclose(O.noise_ps(m["rot_port"]), m["noise_port"],
                               rtol=1e-13)
    for nb in (256, 1000, 2048):
        np.testing.assert_allclose(O.noise_ps(m["noise_in_%d" % nb]),
                                   m["noise_out_%d" % nb], rtol=1e-13)


def test_fit_phase_shift_oracle_vs_reference():
    m = G.misc()
    for row in m["fps_rows"]:
        d = row[:1024]
        shift, ns, noise, phase, perr, scale = row[1024:1030]
        r = O.fit_phase_shift(d, m["fps_model"],
                              None if np.isnan(noise) else noise, Ns=int(ns))
        assert abs(G.phase_diff(r["phase"], phase)) < 1e-12
        assert abs(r["phase_err"] / perr - 1) < 1e-9
        assert abs(r["scale"] / scale - 1) < 1e-9


def test_guess_fit_freq_vs_reference():
    m = G.misc()
    assert abs(O.guess_fit_freq(m["gff_freqs"], m["gff_snrs"]) -
               m["gff_out"][0]) < 1e-9
    assert abs(O.guess_fit_freq(m["gff_freqs"]) - m["gff_out"][1]) < 1e-9


def test_get_toas_oracle_vs_reference():
    g = G.gettoas()
    nsub, nchan, nbin = int(g["nsub"]), int(g["nchan"]), int(g["nbin"])
    import oracle.ppfit_oracle as OO
    freqs = np.tile(g["freqs"], (nsub, 1))
    model = _gmodel_portrait(nchan, nbin, g["freqs"], float(g["P"]))
    for f in range(int(g["nfile"])):
        sub = g["f%d_subints" % f].astype(float)
        out = OO.get_toas_archive(
            sub, model, freqs, g["f%d_weights" % f], g["f%d_snrs" % f],
            np.full(nsub, float(g["P"])), float(g["DM0"]), g["f%d_dfs" % f])
        dev_phi = np.abs(G.phase_diff(out["phis"], g["out_phis"][f])) / \
            g["out_phi_errs"][f]
        dev_dm = np.abs(out["DMs"] - g["out_DMs"][f]) / g["out_DM_errs"][f]
        assert dev_phi.max() < 1e-3 and dev_dm.max() < 1e-3
        np.testing.assert_allclose(out["red_chi2s"], g["out_red_chi2s"][f],
                                   rtol=1e-10)
        assert abs(out["DeltaDM_mean"] - g["out_DeltaDM_means"][f]) < \
            1e-3 * g["out_DeltaDM_errs"][f]


def _gmodel_portrait(nchan, nbin, freqs, P):
    """The example.gmodel portrait GetTOAs builds per sub-integration
    (read_model at full precision, pptoas.py:396-399), regenerated by the
    oracle's gen_gaussian_portrait."""
    from pulseportraiture_amd import pplib as PL
    import oracle as O
    import os
    gm = os.path.join(os.path.dirname(__file__), "golden", "example.gmodel")
    (_, code, nu_ref, _, params, _, alpha, _) = PL.read_model(gm, quiet=True)
    params[1] *= nbin / P                     # read_model's TAU [s] -> [bin]
    return O.gen_gaussian_portrait(code, params, alpha, np.zeros(nbin),
                                   freqs, nu_ref)


def test_oracle_gmodel_matches_reference_model():
    """The oracle's .gmodel portrait generation against the reference's own
    portraits stored (float32-rounded) in the golden cases."""
    for name in ("pd_64x512", "pd_128x1024", "pd_512x2048"):
        c = G.full_case(name)
        nbin = c["model"].shape[1]
        model = _gmodel_portrait(c["model"].shape[0], nbin, c["freqs"],
                                 float(c["P"]))
        ref = c["model"].astype(np.float64)
        ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
        assert np.all(np.abs(model - ref) <= ulp + 1e-12)


def test_oracle_align_archives_matches_reference():
    """The oracle's ppalign iteration (restated from ppalign.py:118-257)
    reproduces the reference's aligned portrait (2 iterations, 5 archives x 2
    sub-ints, one archive with zapped channels)."""
    import oracle as O
    c = G.align()
    archives, model_data = G.align_inputs(c)
    port, tw = O.align_archives(archives, model_data, fit_dm=True,
                                niter=int(c["niter"]))
    ref = c["out_aligned"]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(port[0], ref, rtol=0, atol=1e-6 * scale)
    np.testing.assert_array_equal(tw[:, 0] > 0, c["out_weights"] > 0)


def test_oracle_channels_to_zap_matches_reference():
    """get_channels_to_zap (pptoas.py:1266-1343): the oracle's channel chi^2
    (show_fit + get_red_chi2) and selection, fed the reference's own fitted
    parameters, reproduce the reference's chi^2s and zap lists exactly."""
    import oracle.ppfit_oracle as OO
    g = G.zap()
    nsub, nchan, nbin = int(g["nsub"]), int(g["nchan"]), int(g["nbin"])
    P = float(g["P"])
    freqs = g["freqs"]
    model = _gmodel_portrait(nchan, nbin, freqs, P)
    D = 0.000241 ** -1
    for f in range(int(g["nfile"])):
        sub = g["f%d_subints" % f].astype(float)
        w = g["f%d_weights" % f]
        for s in range(nsub):
            ok = np.where(w[s] != 0)[0]
            df = g["out_doppler_fs"][f][s]
            DM = g["out_DMs"][f][s] / df
            nu_DM, nu_GM, _ = g["out_nu_refs"][f][s]
            ph = g["out_phis"][f][s] + D * DM * (freqs[ok] ** -2 -
                                                   nu_DM ** -2) / P
            chi = OO.channel_red_chi2s(sub[s, ok], ph, model[ok],
                                       g["out_scales"][f][s][ok],
                                       g["f%d_noise" % f][s][ok], nbin - 2)
            for ic, (snr_t, rchi_t, it) in enumerate(g["calls"]):
                np.testing.assert_allclose(chi, g["chi2"][ic][f][s],
                                           rtol=1e-9, atol=0)
                bad = OO.select_zap_channels(
                    g["chi2"][ic][f][s], list(ok), g["out_channel_snrs"][f][s],
                    snr_t, rchi_t, bool(it))
                assert bad == g["zap"][ic][f][s], (ic, f, s)


def test_ppzap_host_logic_matches_reference(tmp_path):
    """ppzap.get_zap_channels (noise-median iteration, ppzap.py:23-53) and
    print_paz_cmds (ppzap.py:56-106) against the reference's own output on
    the zap archives: identical channel lists and identical paz text."""
    import contextlib
    import io
    from pulseportraiture_amd import ppzap
    from pulseportraiture_amd.pplib import DataBunch
    g = G.zap()
    nsub, nfile = int(g["nsub"]), int(g["nfile"])
    zl = []
    for nstd in (1.0, 3.0):
        for f in range(nfile):
            w = g["f%d_weights" % f]
            d = DataBunch(ok_isubs=np.arange(nsub),
                          ok_ichans=[np.where(w[i] != 0)[0]
                                     for i in range(nsub)],
                          noise_stds=g["f%d_noise" % f][:, None])
            zl.append(ppzap.get_zap_channels(d, nstd=nstd))
    flat = [int(v) for a in zl for s in a for v in s]
    assert flat == list(g["ppzap_noise_zap"])
    assert [len(s) for a in zl for s in a] == list(g["ppzap_noise_zap_n"])
    files = ["zap0.fits", "zap1.fits"]
    outs = iter(g["ppzap_paz_out"])
    for zap_list in (g["zap"][0], zl[:2]):
        for all_subs in (False, True):
            for modify in (False, True):
                buf = io.StringIO()
                with contextlib.redirect_stdout(buf):
                    ppzap.print_paz_cmds(files, zap_list, all_subs=all_subs,
                                         modify=modify)
                assert buf.getvalue() == str(next(outs))
    out = tmp_path / "paz.txt"
    ppzap.print_paz_cmds(files, zl[:2], outfile=str(out), quiet=True)
    assert out.read_text() == str(g["ppzap_paz_out"][5])


def test_oracle_gaussian_portraits_match_reference(tmp_path):
    """The oracle's gen_gaussian_portrait / gaussian_profile reproduce the
    reference's own outputs bit for bit (both evolution codes, wrapped and
    out-of-range locs, widths through zero, scattering), and read_model's
    parse + TAU scaling feeds it the reference's parameters."""
    import oracle as O
    from pulseportraiture_amd import pplib as PL
    g = G.gauss()
    for name in g["cases"]:
        c = G.gauss_case(g, str(name))
        nbin = c["out"].shape[1]
        out = O.gen_gaussian_portrait(c["code"], c["params"], c["alpha"],
                                      np.zeros(nbin), c["freqs"], c["nu_ref"])
        np.testing.assert_array_equal(out, c["out"])
    for i in range(int(g["nprof"])):
        nbin, loc, wid = g["prof%d__args" % i]
        np.testing.assert_array_equal(O.gaussian_profile(int(nbin), loc, wid),
                                      g["prof%d__out" % i])
    gm = tmp_path / "tau.gmodel"
    gm.write_text(str(g["readmodel__text"]))
    (_, code, nu_ref, ngauss, params, _, alpha, _) = PL.read_model(str(gm),
                                                                   quiet=True)
    ref = g["readmodel__out"]
    nbin, P = ref.shape[1], float(g["readmodel__P"])
    assert ngauss == 2 and params[1] != 0.0
    params[1] *= nbin / P
    out = O.gen_gaussian_portrait(code, params, alpha, np.zeros(nbin),
                                  g["readmodel__freqs"], nu_ref)
    np.testing.assert_array_equal(out, ref)

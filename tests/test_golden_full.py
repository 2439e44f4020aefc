"""CPU checks of the full-shape golden vectors (tests/golden/full.npz,
oracle_c5.npz): the inputs rebuild bit for bit from their stored parameters
(SHA-256), the oracle reproduces the reference's full-shape outputs
(parity pinning of the checker at the BASELINE shapes), and the host
get_scales_full matches the reference's."""
import os

import numpy as np
import pytest

import fullshape as F
import goldens as G
import oracle as O

SIG, RCHI2 = G.SIGMA_TOL, G.RCHI2_RTOL


@pytest.mark.parametrize("name", ["c3_all_512x2048_a", "c3_all_512x2048_b",
                                  "c3_pdta_512x2048", "narrow_pd_512x2048",
                                  "pd_64x4096", "pdta_64x128", "pd_128x1000",
                                  "pdta_128x1536", "pd_128x1022",
                                  "pdta_64x2006", "pd_128x1023",
                                  "pdta_64x1001"])
def test_fit_inputs_rebuild(name):
    F.fit_case(name)


@pytest.mark.parametrize("name", [c["name"] for c in F.FI.TOAS])
def test_toa_inputs_rebuild(name):
    F.toa_case(name)


@pytest.mark.parametrize("name", ["c4", "dup"])
def test_align_inputs_rebuild(name):
    F.align_case(name)


@pytest.mark.parametrize("name", ["c5_a", "c5_b"])
def test_c5_inputs_rebuild(name):
    F.c5_case(name)


def _oracle_fit(c, data, model, freqs):
    lt = bool(c["log10_tau"])
    return O.fit_portrait_full(data.astype(np.float64), model,
                               list(c["init"]), float(c["P"]), freqs,
                               [float(c["nu_fit"])] * 3, [None] * 3,
                               c["errs"], [int(v) for v in c["flags"]],
                               log10_tau=lt)


@pytest.mark.parametrize("name", ["c3_pdta_512x2048", "narrow_pd_512x2048",
                                  "pd_64x4096", "pdta_64x128",
                                  "lowsnr_pd_512x2048", "lowsnr_pd_64x512",
                                  "pd_128x1000", "pdta_128x1536",
                                  "pd_128x1022", "pdta_64x2006",
                                  "pd_128x1023", "pdta_64x1001"])
def test_oracle_matches_reference_fullshape_fits(name):
    c, data, model, freqs = F.fit_case(name)
    r = _oracle_fit(c, data, model, freqs)
    dev = G.param_deviation_sigma(r, G.ref_bunch(c), float(c["P"]),
                                  bool(c["log10_tau"]))
    assert dev.max() < SIG, dev
    assert abs(r["red_chi2"] / c["out_red_chi2"] - 1) < RCHI2


def test_oracle_matches_reference_example_gettoas():
    """configs[0] (examples/example.py shape, scintillation): the oracle's
    GetTOAs loop against the reference's get_TOAs(DM0=DM0)."""
    c, files, freqs, gm = F.toa_case("c1")
    model = _gmodel_portrait(gm, freqs, int(c["nbin"]))
    for f, fi in enumerate(files):
        nsub = fi["subints"].shape[0]
        o = O.get_toas_archive(fi["subints"].astype(np.float64), model,
                               np.tile(freqs, (nsub, 1)), fi["weights"],
                               fi["snrs"], np.full(nsub, float(c["P"])),
                               float(c["DM0"]), fi["dfs"],
                               noise_stds=fi["noise"], DM0=float(c["DM0"]))
        dphi = np.abs(G.phase_diff(o["phis"], c["out_phis"][f]))
        assert np.all(dphi < SIG * c["out_phi_errs"][f])
        assert np.all(np.abs(o["DMs"] - c["out_DMs"][f]) <
                      SIG * c["out_DM_errs"][f])
        np.testing.assert_allclose(o["red_chi2s"], c["out_red_chi2s"][f],
                                   rtol=RCHI2)
        assert abs(o["DeltaDM_mean"] - c["out_DeltaDM_means"][f]) < \
            SIG * c["out_DeltaDM_errs"][f]


def test_oracle_matches_reference_scatfix_gettoas():
    """configs[4]'s band (400-800 MHz, 128 x 1024): the oracle's GetTOAs loop
    with scat_guess and alpha held (fit_flags [1, 1, 0, 1, 0]) against the
    reference's get_TOAs(fit_scat=True, fix_alpha=True, scat_guess=...)."""
    c, files, freqs, gm = F.toa_case("scatfix")
    kw = F.toa_conf("scatfix")["kw"]
    model = _gmodel_portrait(gm, freqs, int(c["nbin"]))
    fi = files[0]
    nsub = fi["subints"].shape[0]
    o = O.get_toas_archive(fi["subints"].astype(np.float64), model,
                           np.tile(freqs, (nsub, 1)), fi["weights"],
                           fi["snrs"], np.full(nsub, float(c["P"])),
                           float(c["DM0"]), fi["dfs"], noise_stds=fi["noise"],
                           fit_flags=(1, 1, 0, 1, 0), log10_tau=True,
                           scat_guess=kw["scat_guess"])
    dphi = np.abs(G.phase_diff(o["phis"], c["out_phis"][0]))
    assert np.all(dphi < SIG * c["out_phi_errs"][0])
    for key, ix in (("DMs", 1), ("taus", 3)):
        err = c["out_" + key[:-1] + "_errs"][0]
        assert np.all(np.abs(o[key] - c["out_" + key][0]) < SIG * err), key
        np.testing.assert_allclose(o["param_errs"][:, ix], err, rtol=1e-5)
    np.testing.assert_array_equal(o["alphas"], c["out_alphas"][0])
    np.testing.assert_allclose(o["red_chi2s"], c["out_red_chi2s"][0],
                               rtol=RCHI2)


def _gmodel_portrait(path, freqs, nbin):
    import synth_np as S
    code, nu_ref, params, alpha = S.read_gmodel(path)
    return O.gen_gaussian_portrait(code, params, alpha,
                                   O.get_bin_centers(nbin), freqs, nu_ref)


def test_oracle_matches_reference_align_duplicate_channels():
    """ppalign with archive channels mapping two-to-one onto the template
    (ADVICE round 1): the oracle fits the full ichans list, duplicates
    included, and accumulates only the last of each duplicate, like the
    reference."""
    c, archives, model_data = F.align_case("dup")
    port, _ = O.align_archives(archives, model_data, fit_dm=True,
                               niter=int(c["niter"]))
    ref = c["out_aligned"]
    np.testing.assert_allclose(port[0], ref, rtol=0,
                               atol=1e-6 * np.abs(ref).max())


def test_oracle_get_scales_full_matches_reference():
    """The oracle's get_scales_full (pptoaslib.py:953-971) against the
    reference's own output on a scattering case's spectra: log10 and linear
    tau, tau = 0 (B = 1), fitted and arbitrary parameters (the device path
    is checked against the same vectors in test_gpu_fullshape.py)."""
    g = F.case("scales", "scales")
    c = G.full_case(str(g["case"]))
    data = c["data"].astype(np.float64)
    model = c["model"].astype(np.float64)
    nbin = data.shape[1]
    dFT = np.fft.rfft(data, axis=1)
    dFT[:, 0] *= 0
    mFT = np.fft.rfft(model, axis=1)
    mFT[:, 0] *= 0
    errs_FT = c["errs"] * np.sqrt(nbin / 2.0)
    for i in range(4):
        nus = g["s%d_nus" % i]
        got = O.get_scales_full(list(g["s%d_params" % i]), dFT, mFT,
                                errs_FT, float(c["P"]), c["freqs"],
                                nus[0], nus[1], nus[2],
                                bool(g["s%d_log10_tau" % i]))
        np.testing.assert_allclose(got, g["s%d_out" % i], rtol=1e-12,
                                   atol=1e-14 * np.abs(g["s%d_out" % i]).max())


def test_spline_model_file():
    """tests/golden/spline.spl (the make_spline_model-type template the
    spline goldens were made with) reads back through read_spline_model
    (pplib.py:3060-3096) as the parts full_inputs.spline_parts() builds, and
    read_model rejects it with the UnicodeDecodeError GetTOAs catches to
    fall back to the spline reader (pptoas.py:416)."""
    import full_inputs as FI
    from pulseportraiture_amd import pplib
    name, src, df, mean_prof, eigvec, tck = pplib.read_spline_model(
        FI.SPLINE_MODEL, quiet=True)
    parts = FI.spline_parts()
    assert (name, src, df) == parts[:3]
    np.testing.assert_allclose(mean_prof, parts[3], rtol=1e-12)
    np.testing.assert_allclose(np.abs(eigvec), np.abs(parts[4]), atol=1e-10)
    assert eigvec.shape == (FI.SPLINE_NBIN, FI.SPLINE_NCOMP)
    assert int(tck[2]) == 3 and len(tck[1]) == FI.SPLINE_NCOMP
    with pytest.raises(UnicodeDecodeError):
        pplib.read_model(FI.SPLINE_MODEL, quiet=True)


def test_read_model_missing_line_unbound(tmp_path):
    """A .gmodel without its DC line leaves the reference's local unbound
    (pplib.py:3022): UnboundLocalError, as GetTOAs expects."""
    from pulseportraiture_amd import pplib
    src = open(os.path.join(G.GOLDEN, "example.gmodel")).read().splitlines()
    bad = tmp_path / "nodc.gmodel"
    bad.write_text("\n".join(l for l in src if not l.startswith("DC")) +
                   "\n")
    with pytest.raises(UnboundLocalError):
        pplib.read_model(str(bad), quiet=True)

"""GetTOAs' whole-array host paths (pptoas.FAST_HOST: _gather_uniform,
_book_uniform) against the per-sub-int loops they replace
(pptoas.py:384-711), bit for bit, on synthetic archives and result tables
(no device: the fit's output table is synthetic)."""
import numpy as np
import pytest

from pulseportraiture_amd import _lib, pplib, pptoas


def _gt(fit_flags, bary, log10_tau, scat_guess):
    class G(pptoas.GetTOAs):
        def __init__(self):
            for a in pptoas._ATTRS:
                setattr(self, a, [])
            self.quiet = True

    g = G()
    g.fit_flags = list(fit_flags)
    g.fit_DM, g.fit_GM = bool(fit_flags[1]), bool(fit_flags[2])
    g.nfit = int(sum(fit_flags))
    g.bary, g.log10_tau, g.scat_guess = bary, log10_tau, scat_guess
    g.modelfile = "t.gmodel"
    g.model_nu_ref = 1500.0
    g.gparams = [0.0, 1e-4]
    g._ff = [None]
    return g


def _archive(rng, nsub, nchan, nbin, ok_common=True):
    freqs = np.linspace(1100.0, 1900.0, nchan)
    chans = np.arange(nchan)
    if ok_common == "all":
        ok = [chans] * nsub
    elif ok_common:
        ok = [chans[chans % 7 != 3]] * nsub
    else:
        ok = [chans[(chans + i) % 5 != 0] for i in range(nsub)]
    return pplib.DataBunch(
        nsub=nsub, nchan=nchan, nbin=nbin, freqs=np.tile(freqs, (nsub, 1)),
        SNRs=rng.uniform(1, 50, (nsub, 1, nchan)),
        Ps=rng.uniform(0.002, 0.003, nsub),
        doppler_factors=1 + rng.uniform(-1e-4, 1e-4, nsub),
        epochs=[pplib.MJD(57000, 0.1 + 1e-3 * i) for i in range(nsub)],
        ok_ichans=ok, ok_isubs=np.arange(nsub), backend="be", frontend="fe",
        backend_delay=1e-7, bw=800.0, subtimes=list(10.0 + np.arange(nsub)),
        telescope="GBT", telescope_code="1", parallactic_angles=np.zeros(nsub),
        nu0=1500.0)


def _table(rng, nok, nchan):
    I = _lib.RESULT_INDEX
    R = rng.normal(size=(nok, _lib.RESULT_DOUBLES))
    R[:, I["status"]] = 0
    R[:, I["nfeval"]] = rng.integers(3, 40, nok)
    R[:, I["nu_out"]] = rng.uniform(1200, 1800, (nok, 3))
    R[:, I["snr"]] = rng.uniform(10, 100, nok)
    R[:, I["red_chi2"]] = rng.uniform(0.8, 1.2, nok)
    return dict(results=R, scales=rng.normal(size=(nok, nchan)),
                scale_errs=rng.uniform(size=(nok, nchan)),
                channel_snrs=rng.normal(size=(nok, nchan)),
                covariance=rng.normal(size=(nok, 5, 5)), batch_duration=0.37)


def _ctx(nu_refs, bary, fit_scat, print_phase, print_flux=False):
    return dict(quiet=True, tscrunch=False, fit_scat=fit_scat,
                method="trust-ncg", bounds=[None], by_archive=False,
                nu_fit_tuple=None, nu_ref_tuple=nu_refs, bary=bary,
                print_phase=print_phase, print_flux=print_flux,
                print_parangle=True, addtnl_toa_flags={"pta": "X"})


def _run(fast, flags, bary, log10_tau, scat_guess, nu_refs, print_phase,
         ok_common=True, print_flux=False):
    rng = np.random.default_rng(17)
    nsub, nchan, nbin = 9, 24, 256
    d = _archive(rng, nsub, nchan, nbin, ok_common)
    g = _gt(flags, bary, log10_tau, scat_guess)
    ctx = _ctx(nu_refs, bary, bool(flags[3]), print_phase, print_flux)
    models = np.random.default_rng(5).normal(2.0, 1.0, (2, nchan, 8))
    ok_isubs = list(d.ok_isubs)
    nu_fits_a = list(np.zeros([nsub, 3]))
    nu_refs_a = list(np.zeros([nsub, 3]))
    pptoas.FAST_HOST = fast
    try:
        gat = g._gather_uniform(d, ok_isubs, ctx, nu_fits_a, nu_refs_a,
                                10.0) if fast else None
        used = gat is not None
        if gat is None:
            gat = g._gather_rows(d, ok_isubs, ctx, nu_fits_a, nu_refs_a,
                                 10.0)
        mask, init, flags_b, nu_fit_b, nu_out_b, guess_tau = gat
        job = dict(d=d, datafile="a.fits", nsub=nsub, nchan=nchan, nbin=nbin,
                   obs=None, nu_fits_a=nu_fits_a, nu_refs_a=nu_refs_a,
                   MJDs=np.zeros(nsub), DM0=10.0, ok_isubs=ok_isubs,
                   nok=len(ok_isubs), models=models,
                   model_index=np.arange(len(ok_isubs)) % 2,
                   mask=mask, flags_b=flags_b, fit_duration=0.0)
        g._book_archive(job, _table(rng, len(ok_isubs), nchan), ctx, 0.0)
    finally:
        pptoas.FAST_HOST = True
    return used, gat, nu_fits_a, g


def _same(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        a, b = np.asarray(a), np.asarray(b)
        assert a.dtype == b.dtype and a.shape == b.shape
        if a.dtype == object:
            assert [repr(x) for x in a.ravel()] == \
                [repr(x) for x in b.ravel()]
        else:
            np.testing.assert_array_equal(a, b)
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            _same(x, y)
    else:
        assert type(a) is type(b) and repr(a) == repr(b), (a, b)


CASES = [
    ([1, 1, 0, 0, 0], True, False, None, None, False, True),
    ([1, 1, 0, 0, 0], False, False, None, (1400.0, 1400.0, 1400.0), True),
    ([1, 1, 1, 0, 0], True, False, None, None, True),
    ([1, 0, 0, 0, 0], True, False, None, None, False),
    ([1, 1, 0, 1, 1], True, True, (1e-4, 1500.0, -4.0), None, False),
    ([1, 1, 0, 1, 1], True, False, None, (1500.0, 1500.0, 1500.0), False),
    ([1, 1, 0, 1, 0], False, True, None, None, True, True),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("chans", [True, "all"])
def test_uniform_paths_equal_loops(case, chans):
    flags, bary, log10_tau, sg, nu_refs, pp = case[:6]
    pf = case[6] if len(case) > 6 else False
    used, gf, nf_f, fast = _run(True, flags, bary, log10_tau, sg, nu_refs, pp,
                                ok_common=chans, print_flux=pf)
    assert used
    _, gs, nf_s, slow = _run(False, flags, bary, log10_tau, sg, nu_refs, pp,
                             ok_common=chans, print_flux=pf)
    if pf:
        assert np.all(np.asarray(fast.fluxes[0]) != 0.0)
    _same(list(gf), list(gs))
    _same(nf_f, nf_s)
    for a in pptoas._ATTRS:
        if a == "TOA_list":
            continue
        _same(getattr(fast, a), getattr(slow, a))
    assert len(fast.TOA_list) == len(slow.TOA_list) == 9
    for t, u in zip(fast.TOA_list, slow.TOA_list):
        for k in ("archive", "frequency", "TOA_error", "telescope",
                  "telescope_code", "DM", "DM_error"):
            _same(getattr(t, k), getattr(u, k))
        assert repr(t.MJD) == repr(u.MJD)
        assert list(t.flags) == list(u.flags)
        for k in t.flags:
            _same(t.flags[k], u.flags[k])


def test_ragged_channels_take_the_loop():
    used, *_ = _run(True, [1, 1, 0, 0, 0], True, False, None, None, False,
                    ok_common=False)
    assert not used


def test_flux_is_the_scattered_model_mean():
    """print_flux takes each model row's mean: the scattered model's mean
    (the reference's rfft / irfft round trip, pptoas.py:628-636) is the same
    number up to rounding."""
    from pulseportraiture_amd.pplib import (scattering_portrait_FT,
                                            scattering_times)
    rng = np.random.default_rng(2)
    model = rng.normal(3.0, 1.0, (16, 256))
    freqs = np.linspace(1100.0, 1900.0, 16)
    scat = np.fft.irfft(scattering_portrait_FT(scattering_times(
        0.03, -4.0, freqs, 1500.0), 256) * np.fft.rfft(model, axis=1),
        axis=1)
    np.testing.assert_allclose(scat.mean(axis=1), model.mean(axis=1),
                               rtol=1e-14)


def test_substituted_epoch_type_takes_the_object_path(monkeypatch):
    """With pptoas._MJD replaced (PSRCHIVE's MJD, or a test's own type) the
    TOA epochs are built one object at a time; the same values here."""
    used, _, _, fast = _run(True, [1, 1, 0, 0, 0], True, False, None, None,
                            False, ok_common="all")
    monkeypatch.setattr(pptoas, "_MJD", lambda days: pplib.MJD(days))
    assert not pptoas._MJD_is_plain()
    _, _, _, obj = _run(True, [1, 1, 0, 0, 0], True, False, None, None,
                        False, ok_common="all")
    assert [repr(t.MJD) for t in fast.TOA_list] == \
        [repr(t.MJD) for t in obj.TOA_list]


def test_noise_length_rule():
    """get_noise_PS(chans=False) sends a flattened row to the LDS FFT only
    when its transform length has no prime factor above NOISE_MAX_PRIME
    (8186 = 2 x 4093 was a 4093-point direct DFT per row); the
    rest take the device FFT library."""
    from pulseportraiture_amd import engine
    ok = [2048, 1000, 1536, 4096, 8192, 1023, 4095, 33, 2006]
    lib = [8186, 1022, 4094, 127, 1002, 30, 8194, 4097]
    assert all(engine.noise_len_supported(n) for n in ok)
    assert not any(engine.noise_len_supported(n) for n in lib)
    assert engine._max_prime_factor(2 * 3 * 167) == 167
    assert engine._max_prime_factor(1) == 1

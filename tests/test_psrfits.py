"""PSRFITS fast path (pulseportraiture_amd/psrfits.py): the FITS reader and
writer on the CPU, and on the GPU the device unpack against its NumPy
restatement and GetTOAs on a PSRFITS file against GetTOAs on the same rows
handed over as a host DataBunch.

Parity note: no PSRFITS fixture and no PSRCHIVE exist here, so what PSRCHIVE
itself would return for a file (epochs referred to the predictor, Doppler
factors, its own S/N) is unpinned; these tests pin the fast path to its
documented restatement and to the DataBunch path that the reference goldens
pin."""
import os

import numpy as np
import pytest

from pulseportraiture_amd import psrfits as PF


def _archive(tmp, nsub=4, npol=2, nchan=32, nbin=256, seed=1, elem="I",
             wvals=False):
    rng = np.random.default_rng(seed)
    b = np.arange(nbin)
    prof = np.exp(-0.5 * ((b - 0.3 * nbin) / (0.02 * nbin)) ** 2)
    rows = 20.0 * prof[None, None, None] * rng.uniform(0.5, 1.5, (nsub, 1, nchan, 1)) \
        + rng.normal(0, 1.0, (nsub, npol, nchan, nbin)) + 7.0
    q, scl, offs = PF.quantize(rows)
    fr = np.tile(np.linspace(1100.0, 1900.0, nchan), (nsub, 1))
    wts = np.ones((nsub, nchan))
    if wvals:
        wts = np.round(rng.uniform(0.5, 2.0, (nsub, nchan)), 2)
        wts[:, 7] = 0.0                                # zapped everywhere
    wts[1, 3] = 0.0
    fn = os.path.join(str(tmp), "a.fits")
    PF.write_psrfits(fn, q, scl, offs, fr, wts, np.full(nsub, 0.00289),
                     5.0 + 10.0 * np.arange(nsub), np.full(nsub, 10.0),
                     stt_imjd=57000, stt_smjd=3600, stt_offs=0.25, npol=npol,
                     pol_type="AABBCRCI" if npol == 4 or npol == 2 else "AA+BB",
                     dm=12.5, be_delay=1e-6)
    return fn, q, scl, offs, fr, wts


def test_fits_round_trip(tmp_path):
    fn, q, scl, offs, fr, wts = _archive(tmp_path)
    f = PF.PSRFITS(fn)
    assert (f.nsub, f.npol, f.nchan, f.nbin) == q.shape
    raw, dt = f.data_bytes()
    got = np.ascontiguousarray(raw).view(dt).reshape(q.shape)
    np.testing.assert_array_equal(got, q)
    s, o = f.scales_offsets()
    np.testing.assert_array_equal(s, scl)
    np.testing.assert_array_equal(o, offs)
    np.testing.assert_array_equal(f.freqs(), fr)
    np.testing.assert_array_equal(f.weights(), wts)
    np.testing.assert_array_equal(f.periods(), 0.00289)
    imjd, frac = f.epochs()
    np.testing.assert_array_equal(imjd, 57000)
    np.testing.assert_allclose(frac, (3600.25 + 5.0 + 10.0 * np.arange(4)) / 86400.0,
                               rtol=0, atol=1e-15)
    assert f.primary["TELESCOP"] == "GBT" and f.subint.header["DM"] == 12.5
    f.close()


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_read_data_into_native_reader(tmp_path, threads, monkeypatch):
    """ppf_read_rows (native positioned reads, no device) returns the DATA
    bytes of every row, at any thread count, into a strided buffer, and
    fails loudly on a truncated file or a bad destination."""
    fn, q, scl, offs, fr, wts = _archive(tmp_path, nsub=5, npol=2, nchan=16,
                                         nbin=128)
    monkeypatch.setattr(PF, "_READ_THREADS", threads)
    f = PF.PSRFITS(fn)
    raw, dt = f.data_bytes()
    nbytes = 1 * 16 * 128 * 2                 # pol 0 only: the first block
    dst = np.full((5, nbytes + 64), 0xAB, dtype=np.uint8)
    f.read_data_into(nbytes, dst)
    np.testing.assert_array_equal(dst[:, :nbytes], np.asarray(raw)[:, :nbytes])
    assert (dst[:, nbytes:] == 0xAB).all()
    full = raw.shape[1]
    dst2 = np.zeros((5, full), dtype=np.uint8)
    f.read_data_into(full, dst2)
    np.testing.assert_array_equal(dst2, np.asarray(raw))
    with pytest.raises(ValueError):
        f.read_data_into(nbytes, np.zeros((4, nbytes), dtype=np.uint8))
    f.close()
    # a file cut inside the last row's DATA: the read comes up short
    f = PF.PSRFITS(fn)
    t = f.subint
    cut = t._off + 4 * t.rowbytes + t.columns["DATA"][0] + 100
    f.close()
    with open(fn, "r+b") as fh:
        fh.truncate(cut)
    with open(fn, "rb") as fh:
        from pulseportraiture_amd import _lib
        rc = _lib.load().ppf_read_rows(
            fh.fileno(), t._off + t.columns["DATA"][0], t.rowbytes, nbytes,
            5, dst.ctypes.data, dst.strides[0], threads)
        assert rc == -5                                   # PPF_EIO
        assert _lib.load().ppf_read_rows(fh.fileno(), 0, 10, 20, 1,
                                         dst.ctypes.data, 64, 1) == -1


def test_unpack_host_restatement(tmp_path):
    fn, q, scl, offs, fr, wts = _archive(tmp_path)
    f = PF.PSRFITS(fn)
    raw, dt = f.data_bytes()
    u = PF.unpack_host(raw, dt, *f.scales_offsets(), f.npol, f.nchan, f.nbin)
    s4 = scl.reshape(4, 2, 32, 1)
    o4 = offs.reshape(4, 2, 32, 1)
    want = (q.astype(np.float32) * s4).astype(np.float32) + o4
    np.testing.assert_array_equal(u, want[:, 0] + want[:, 1])
    f.close()


def test_mjd_arithmetic():
    from pulseportraiture_amd.pplib import MJD
    m = MJD(57000, 0.999999) + MJD(0.5 / 86400.0 * 86400.0 / 86400.0)
    assert m.intday() == 57001 and abs(m.fracday() - (0.999999 + 0.5 / 86400 - 1)) < 1e-15
    t = MJD(57000, 0.25) + 3600.0                       # seconds
    assert t.intday() == 57000 and abs(t.fracday() - (0.25 + 1 / 24.0)) < 1e-15


def test_load_data_rejects_psrchive_only_options(tmp_path):
    fn = _archive(tmp_path)[0]
    for kw in (dict(fscrunch=True), dict(state="Stokes")):
        with pytest.raises(NotImplementedError):
            PF.load_data(fn, pscrunch=True, **kw)
    with pytest.raises(NotImplementedError):
        PF.load_data(fn, pscrunch=False)              # npol 2, not scrunched


def _host_baseline(u, wts, frac=0.15):
    """NumPy restatement of k_base_window + k_row_stats."""
    nsub, nchan, nbin = u.shape
    W = min(nbin - 1, max(1, int(np.rint(frac * nbin))))
    out, stats, w0s, mins = np.empty_like(u), np.empty((nsub, nchan, 3)), [], []
    for s in range(nsub):
        tot = (wts[s][:, None] * u[s].astype(float)).sum(axis=0)
        ext = np.concatenate([tot, tot[:W]])
        cs = np.concatenate([[0.0], np.cumsum(ext)])
        sums = cs[W:W + nbin] - cs[:nbin]
        w0s.append(int(np.argmin(sums)))
        mins.append((sums, tot))
    return W, w0s, mins


@pytest.mark.gpu
@pytest.mark.parametrize("npol,elem", [(2, "I"), (1, "I")])
def test_device_unpack_matches_restatement(tmp_path, npol, elem):
    import torch
    from pulseportraiture_amd import engine
    fn, q, scl, offs, fr, wts = _archive(tmp_path, npol=npol)
    f = PF.PSRFITS(fn)
    raw, dt = f.data_bytes()
    s, o = f.scales_offsets()
    raw_d = torch.from_numpy(np.ascontiguousarray(raw)).cuda()
    res = engine.unpack_psrfits(raw_d, 0, npol, f.nchan, f.nbin, s, o,
                                wts=wts.astype(np.float32),
                                pol_mode=1 if npol == 2 else 0, rm_baseline=True)
    rows = res["rows"].cpu().numpy()
    st = res["stats"].cpu().numpy()
    w0 = res["wstart"].cpu().numpy()
    u = PF.unpack_host(raw, dt, s, o, npol, f.nchan, f.nbin)
    W, w0h, mins = _host_baseline(u, wts)
    for k in range(f.nsub):
        sums, tot = mins[k]
        np.testing.assert_allclose(res["total"].cpu().numpy()[k], tot, rtol=1e-12,
                                   atol=1e-9)
        # the device window is a minimum of the window sums (ties aside)
        assert sums[w0[k]] <= sums.min() + 1e-9 * abs(sums).max()
        idx = (w0[k] + np.arange(W)) % f.nbin
        mean = u[k][:, idx].astype(float).mean(axis=1)
        want = (u[k].astype(float) - mean[:, None]).astype(np.float32)
        np.testing.assert_allclose(rows[k], want, rtol=0,
                                   atol=2 * np.spacing(np.abs(want).max()))
        np.testing.assert_allclose(st[k, :, 0], mean, rtol=1e-12)
        sig = u[k][:, idx].astype(float).std(axis=1)
        np.testing.assert_allclose(st[k, :, 1], sig, rtol=1e-10)
        on = np.ones(f.nbin, bool)
        on[idx] = False
        snr = (u[k][:, on].astype(float) - mean[:, None]).sum(axis=1) / \
            (sig * np.sqrt(on.sum()))
        np.testing.assert_allclose(st[k, :, 2], snr, rtol=1e-9)
    f.close()


@pytest.mark.gpu
def test_gettoas_psrfits_equals_databunch_path(tmp_path, monkeypatch):
    """get_TOAs on a PSRFITS file (rows unpacked on the device, fitted
    without leaving HBM) == get_TOAs on the same rows and metadata as a
    host DataBunch (staged through pinned memory), bitwise."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import synth_np as SN
    from pulseportraiture_amd import pptoas, pplib
    nsub, nchan, nbin = 6, 64, 512
    model, freqs = SN.template(nchan, nbin)
    rng = np.random.default_rng(5)
    P = 0.0028929
    phis = rng.uniform(-0.2, 0.2, nsub)
    port = np.stack([SN.rotate(model, -(phis[i] + 4148.808 * 10.0 *
                                        (freqs ** -2 - 1500.0 ** -2) / P))
                     for i in range(nsub)])
    rows = 40.0 * port[:, None] + rng.normal(0, 1.0, (nsub, 2, nchan, nbin))
    q, scl, offs = PF.quantize(rows)
    fn = str(tmp_path / "p.fits")
    PF.write_psrfits(fn, q, scl, offs, np.tile(freqs, (nsub, 1)),
                     np.ones((nsub, nchan)), np.full(nsub, P),
                     5.0 + 10.0 * np.arange(nsub), np.full(nsub, 10.0),
                     npol=2, pol_type="AABBCRCI", dm=10.0)
    gm = str(tmp_path / "t.gmodel")
    SN.write_gmodel(gm, *SN.read_gmodel())
    meta = tmp_path / "meta.txt"
    meta.write_text(fn + "\n")
    fast = pptoas.GetTOAs(str(meta), gm, quiet=True)
    fast.get_TOAs(quiet=True, bary=False)
    # as get_TOAs loads it (rm_baseline = bool(F0_fact) = False,
    # pptoas.py:36-39)
    d = pplib.load_data(fn, pscrunch=True, rm_baseline=False, quiet=True)
    host = pplib.DataBunch(**{k: v for k, v in d.items()})
    host["subints"] = np.asarray(d.subints).copy()
    monkeypatch.setattr(pptoas, "load_data", lambda f_, **kw: host)
    slow = pptoas.GetTOAs(str(meta), gm, quiet=True)
    slow.get_TOAs(quiet=True, bary=False)
    for key in ("phis", "phi_errs", "DMs", "DM_errs", "red_chi2s", "snrs"):
        np.testing.assert_array_equal(np.asarray(getattr(fast, key)[0]),
                                      np.asarray(getattr(slow, key)[0]), err_msg=key)
    a = [str(t.MJD.intday()) + repr(t.MJD.fracday()) for t in fast.TOA_list]
    b = [str(t.MJD.intday()) + repr(t.MJD.fracday()) for t in slow.TOA_list]
    assert a == b
    # the fits converged on data of unit reduced chi^2
    rc = np.asarray(fast.red_chi2s[0])
    assert np.all((rc > 0.8) & (rc < 1.25)), rc


def _baseline_removed(R, wts, frac=0.15):
    """k_base_window + k_row_stats restated over float32 rows [nsub, nchan,
    nbin]: (rows minus their window mean, float32; S/N; window starts)."""
    nsub, nchan, nbin = R.shape
    W = min(nbin - 1, max(1, int(np.rint(frac * nbin))))
    out, snr, w0 = np.empty_like(R), np.empty((nsub, nchan)), []
    for s in range(nsub):
        tot = (wts[s][:, None] * R[s].astype(float)).sum(axis=0)
        cs = np.concatenate([[0.0], np.cumsum(np.concatenate([tot, tot[:W]]))])
        k = int(np.argmin(cs[W:W + nbin] - cs[:nbin]))
        w0.append(k)
        idx = (k + np.arange(W)) % nbin
        mean = R[s][:, idx].astype(float).mean(axis=1)
        sig = R[s][:, idx].astype(float).std(axis=1)
        on = np.ones(nbin, bool)
        on[idx] = False
        snr[s] = (R[s][:, on].astype(float) - mean[:, None]).sum(axis=1) / \
            (sig * np.sqrt(on.sum()))
        out[s] = (R[s].astype(float) - mean[:, None]).astype(np.float32)
    return out, snr, w0


@pytest.mark.gpu
def test_load_data_dedisperse_tscrunch(tmp_path):
    """load_data(dedisperse, tscrunch) on the device against the DataBunch
    rows transformed on the host side of the API: rotate_data (pplib.py:
    2427-2515) by the stored DM to OBSFREQ per sub-int period, the baseline
    measured after the rotation (pplib.py:2786-2791), then the
    DAT_WTS-weighted mean over sub-ints (PSRCHIVE's weighted Profile
    average; PSRCHIVE parity itself unpinned)."""
    from pulseportraiture_amd import pplib
    fn = _archive(tmp_path, wvals=True)[0]
    f = PF.PSRFITS(fn)
    wts = f.weights()                # DAT_WTS as stored (float32 values)
    f.close()
    base = PF.load_data(fn, pscrunch=True, rm_baseline=False, quiet=True)
    U = np.asarray(base.subints)[:, 0]
    nsub, nchan, nbin = U.shape
    nu0 = base.nu0
    R = pplib.rotate_data(U[:, None], 0.0, 12.5, base.Ps, base.freqs,
                          nu0)[:, 0].astype(np.float32)
    Rb, snr, _ = _baseline_removed(R, wts)
    sp = 2 * np.spacing(np.float32(np.abs(Rb).max()))
    # dedisperse
    dd = PF.load_data(fn, pscrunch=True, rm_baseline=True, dedisperse=True,
                      quiet=True)
    assert dd.dmc == 1 and dd.nsub == nsub
    np.testing.assert_allclose(np.asarray(dd.subints)[:, 0], Rb, rtol=0,
                               atol=sp)
    np.testing.assert_allclose(dd.SNRs[:, 0], snr, rtol=1e-6)
    # tscrunch (no dedispersion, no baseline removal)
    ts = PF.load_data(fn, pscrunch=True, rm_baseline=False, tscrunch=True,
                      quiet=True)
    wsum = wts.sum(axis=0)
    mean = (wts[:, :, None] * U.astype(float)).sum(axis=0) / \
        np.where(wsum > 0, wsum, 1.0)[:, None]
    assert ts.nsub == 1 and ts.dmc == 0 and len(ts.epochs) == 1
    np.testing.assert_allclose(np.asarray(ts.subints)[0, 0],
                               mean.astype(np.float32), rtol=0,
                               atol=4 * np.spacing(np.float32(
                                   np.abs(mean).max())))
    np.testing.assert_array_equal(ts.weights[0], wsum)
    assert list(ts.ok_ichans[0]) == [c for c in range(nchan) if wsum[c]]
    # the middle of the span: sub-int centres 5 + 10 i s, 10 s each
    assert ts.epochs[0].intday() == 57000
    assert abs(ts.epochs[0].fracday() - (3600.25 + 20.0) / 86400.0) < 1e-12
    assert ts.subtimes == [40.0] and ts.Ps[0] == 0.00289
    np.testing.assert_allclose(ts.noise_stds[0, 0], pplib.get_noise(
        np.asarray(ts.subints)[0, 0].astype(float), chans=True), rtol=1e-9)
    # both: the weighted mean of the dedispersed, baseline-removed rows
    both = PF.load_data(fn, pscrunch=True, rm_baseline=True, dedisperse=True,
                        tscrunch=True, quiet=True)
    mb = (wts[:, :, None] * Rb.astype(float)).sum(axis=0) / \
        np.where(wsum > 0, wsum, 1.0)[:, None]
    np.testing.assert_allclose(np.asarray(both.subints)[0, 0],
                               mb.astype(np.float32), rtol=0,
                               atol=4 * np.spacing(np.float32(
                                   np.abs(mb).max())))
    assert both.dmc == 1 and both.nsub == 1


@pytest.mark.gpu
def test_gettoas_tscrunch_psrfits_equals_databunch_path(tmp_path,
                                                        monkeypatch):
    """get_TOAs(tscrunch=True) on a PSRFITS file (tscrunched on the device)
    == get_TOAs on the same tscrunched rows and metadata as a host
    DataBunch, bitwise."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import synth_np as SN
    from pulseportraiture_amd import pptoas, pplib
    nsub, nchan, nbin = 6, 64, 512
    model, freqs = SN.template(nchan, nbin)
    rng = np.random.default_rng(9)
    P = 0.0028929
    port = np.stack([SN.rotate(model, -(0.1 + 4148.808 * 10.0 *
                                        (freqs ** -2 - 1500.0 ** -2) / P))
                     for _ in range(nsub)])
    rows = 15.0 * port[:, None] + rng.normal(0, 1.0, (nsub, 1, nchan, nbin))
    q, scl, offs = PF.quantize(rows)
    fn = str(tmp_path / "t.fits")
    PF.write_psrfits(fn, q, scl, offs, np.tile(freqs, (nsub, 1)),
                     np.ones((nsub, nchan)), np.full(nsub, P),
                     5.0 + 10.0 * np.arange(nsub), np.full(nsub, 10.0),
                     npol=1, pol_type="AA+BB", dm=10.0)
    gm = str(tmp_path / "t.gmodel")
    SN.write_gmodel(gm, *SN.read_gmodel())
    meta = tmp_path / "meta.txt"
    meta.write_text(fn + "\n")
    fast = pptoas.GetTOAs(str(meta), gm, quiet=True)
    fast.get_TOAs(quiet=True, bary=False, tscrunch=True)
    assert len(fast.TOA_list) == 1
    d = pplib.load_data(fn, pscrunch=True, rm_baseline=False, tscrunch=True,
                        quiet=True)
    host = pplib.DataBunch(**{k: v for k, v in d.items()})
    host["subints"] = np.asarray(d.subints).copy()
    monkeypatch.setattr(pptoas, "load_data", lambda f_, **kw: host)
    slow = pptoas.GetTOAs(str(meta), gm, quiet=True)
    slow.get_TOAs(quiet=True, bary=False, tscrunch=True)
    for key in ("phis", "phi_errs", "DMs", "DM_errs", "red_chi2s", "snrs"):
        np.testing.assert_array_equal(np.asarray(getattr(fast, key)[0]),
                                      np.asarray(getattr(slow, key)[0]),
                                      err_msg=key)


@pytest.mark.gpu
def test_failed_load_releases_pinned_slot(tmp_path, monkeypatch):
    """A load that fails after it reserved a pinned slot (here: the read
    cannot be submitted) releases the slot: the loads after it, which rotate
    through every slot including the failed one, complete (an
    unset ticket blocked the next user of the slot for ever)."""
    import threading
    fn = _archive(tmp_path)[0]

    class _Refuse(object):
        def submit(self, *a, **k):
            raise RuntimeError("read refused")

    real = PF._read_master
    monkeypatch.setattr(PF, "_read_master", lambda: _Refuse())
    with pytest.raises(RuntimeError):
        PF.load_data(fn, pscrunch=True, quiet=True)
    monkeypatch.setattr(PF, "_read_master", real)
    done = []

    def good():
        for _ in range(PF._PIN_SLOTS + 1):
            d = PF.load_data(fn, pscrunch=True, quiet=True)
            done.append(d.subints.shape)

    t = threading.Thread(target=good, daemon=True)
    t.start()
    t.join(60.0)
    assert not t.is_alive(), "a load after the failed one blocked"
    assert len(done) == PF._PIN_SLOTS + 1

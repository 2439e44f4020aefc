"""CPU, world_size 2 over gloo: the sharding / result all-gather used by the
multi-GPU path (pulseportraiture_amd/dist.py) reassembles per-sub-integration
records in global order, and a per-sub-integration computation sharded over
ranks equals the serial one (shard invariance)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pulseportraiture_amd import dist as pdist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def per_subint(first, count, nchan=8, nbin=64):
    """Deterministic per-sub-integration work (the oracle noise estimate of a
    seeded synthetic portrait), keyed by the global index."""
    import oracle as O
    out = []
    for g in range(first, first + count):
        x = np.random.default_rng(1000 + g).normal(size=(nchan, nbin))
        out.append(np.concatenate([[g], O.noise_ps(x)]))
    return torch.tensor(np.array(out).reshape(count, nchan + 1),
                        dtype=torch.float64)


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    sys.path.insert(0, os.path.dirname(__file__))
    pdist.init("gloo")
    first, count = pdist.shard(n_total, rank, world)
    local = per_subint(first, count)
    full = pdist.allgather_rows(local, n_total, world)
    t = pdist.max_over_ranks(float(rank) + 0.5)
    if rank == 0:
        q.put((full.numpy(), t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [7, 10])
def test_allgather_reassembles_global_order(n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q))
             for r in range(2)]
    for p in procs:
        p.start()
    full, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    serial = per_subint(0, n_total).numpy()
    np.testing.assert_array_equal(full, serial)
    assert tmax == 1.5


def test_shard_is_a_balanced_partition():
    for n in (1, 7, 10000, 80000):
        for w in (1, 2, 3, 8):
            got = [pdist.shard(n, r, w) for r in range(w)]
            assert sum(c for _, c in got) == n
            assert got[0][0] == 0
            for (f0, c0), (f1, _) in zip(got, got[1:]):
                assert f0 + c0 == f1
            assert max(c for _, c in got) - min(c for _, c in got) <= 1


def _align_worker(rank, world, port, n_total, q):
    """ppalign's exchange: each rank accumulates the weighted rotated rows of
    its archives (oracle rotation on CPU), then allreduce_sum_ of the
    portrait and the weights."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    pdist.init("gloo")
    out, w = _align_partial(*pdist.shard(n_total, rank, world))
    pdist.allreduce_sum_(out, w)
    if rank == 0:
        q.put((out.numpy(), w.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _align_partial(first, count, nchan=6, nbin=64):
    import oracle as O
    out = torch.zeros((nchan, nbin), dtype=torch.float64)
    w = torch.zeros(nchan, dtype=torch.float64)
    for g in range(first, first + count):
        rng = np.random.default_rng(500 + g)
        x = rng.normal(size=(nchan, nbin))
        ph = rng.uniform(-0.5, 0.5, nchan)
        wt = rng.uniform(0.5, 1.5, nchan)
        out += torch.as_tensor(wt[:, None] * O.rotate_rows(x, ph))
        w += torch.as_tensor(wt)
    return out, w


def test_align_allreduce_equals_serial():
    n_total = 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_align_worker, args=(r, 2, port, n_total, q))
             for r in range(2)]
    for p in procs:
        p.start()
    out, w = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    ref, rw = _align_partial(0, n_total)
    np.testing.assert_allclose(out, ref.numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(w, rw.numpy(), rtol=1e-14)


def _table_worker(rank, world, port, n_total, nchan, q):
    """GetTOAs' exchange: each rank packs its share's result tables
    (pptoas._pack layout) and all-gathers them over gloo."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    from pulseportraiture_amd import pptoas
    pdist.init("gloo")
    first, count = pdist.shard(n_total, rank, world)
    res = _fake_results(first, count, nchan)
    full = pdist.allgather_rows(pptoas._pack(res), n_total, world)
    if rank == 0:
        q.put(full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _fake_results(first, count, nchan):
    g = torch.arange(first, first + count, dtype=torch.float64)
    return dict(results=g[:, None] + torch.arange(32.0)[None] / 100,
                scales=g[:, None] * 10 + torch.arange(nchan)[None],
                scale_errs=-g[:, None] - torch.arange(nchan)[None],
                channel_snrs=g[:, None] * 1000 + torch.arange(nchan)[None],
                covariance=(g[:, None] + torch.arange(25.0)[None] * 1e-3)
                .reshape(count, 5, 5))


def test_gettoas_table_gather_matches_serial():
    """The packed GetTOAs result tables all-gathered from 2 ranks unpack to
    the serial tables (global sub-int order, every field)."""
    from pulseportraiture_amd import pptoas
    n_total, nchan = 7, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_table_worker,
                         args=(r, 2, port, n_total, nchan, q))
             for r in range(2)]
    for p in procs:
        p.start()
    full = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = pptoas._unpack(full, nchan)
    ref = {k: v.numpy() for k, v in _fake_results(0, n_total, nchan).items()}
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


# ---------------------------------------------------------------------------
# GetTOAs sharded by archive (pptoas.GetTOAs.get_TOAs with world > 1 and at
# least as many archives as ranks): each rank runs only its own block of
# archives; the per-archive attributes and TOAs are gathered in archive order
# ---------------------------------------------------------------------------
class _UnpicklableMJD(object):
    """Stands in for a PSRCHIVE MJD (a SWIG object pickle refuses)."""

    def __init__(self, days):
        self.days = days

    def intday(self):
        return int(self.days)

    def fracday(self):
        return self.days - int(self.days)

    def __reduce__(self):
        raise TypeError("cannot pickle a SWIG object")


def _fake_gettoas(nfile, skip=()):
    """A GetTOAs whose device stages are replaced by deterministic per-archive
    bookkeeping (values keyed by the archive index): exercises get_TOAs'
    archive partition, its error path and _gather_archives."""
    from pulseportraiture_amd import pptoas

    class G(pptoas.GetTOAs):
        def __init__(self):
            for a in pptoas._ATTRS:
                setattr(self, a, [])
            self.datafiles = ["a%d.fits" % i for i in range(nfile)]
            self.quiet = True
            self.seen = []

        def _prep_archive(self, iarch, datafile, ctx, stager, loaded=None):
            self.seen.append(iarch)
            # get_TOAs' loader thread already ran load_data on this archive
            assert loaded is not None and loaded.result() == datafile
            if iarch in skip:                 # load_data failed: skipped
                return None
            self.ok_idatafiles.append(iarch)
            return dict(iarch=iarch, datafile=datafile, nsub=2 + iarch % 3)

        def _fit_archive(self, job, ctx):
            return None

        def _book_archive(self, job, r, ctx, start):
            i, n = job["iarch"], job["nsub"]
            for a in pptoas._ATTRS:
                if a in ("ok_idatafiles", "TOA_list", "channel_red_chi2s",
                         "zap_channels"):
                    continue
                getattr(self, a).append(np.arange(n) * 1.5 + 100 * i +
                                        len(a))
            self.ok_isubs[-1] = np.arange(n)
            for s in range(n):
                self.TOA_list.append(pptoas.TOA(
                    job["datafile"], 1400.0 + s, _UnpicklableMJD(
                        57000.0 + i + s / 7.0), 0.5, "GBT", "1", 34.5 + s,
                    1e-3, {"subint": s}))
    return G()


def _recording_loader(log):
    def load(filename, **kw):
        log.append(filename)
        return filename
    return load


def _summary(gt):
    from pulseportraiture_amd import pptoas
    out = {a: [np.asarray(v).tolist() for v in getattr(gt, a)]
           for a in pptoas._ATTRS if a != "TOA_list"}
    out["TOA_list"] = [(t.archive, t.frequency, t.MJD.intday(),
                        t.MJD.fracday(), t.DM, dict(t.flags))
                       for t in gt.TOA_list]
    return out


def _archive_worker(rank, world, port, nfile, skip, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    sys.path.insert(0, os.path.dirname(__file__))
    import test_dist_gloo as T
    pdist.init("gloo")
    from pulseportraiture_amd import pptoas
    loaded = []
    pptoas.load_data = T._recording_loader(loaded)
    gt = T._fake_gettoas(nfile, skip)
    gt.get_TOAs(quiet=True)
    # each rank's loader read exactly its own archives, once each
    assert sorted(loaded) == sorted(gt.datafiles[i] for i in gt.seen), loaded
    q.put((rank, gt.seen, T._summary(gt)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("nfile,skip", [(5, ()), (4, (1,)), (2, ())])
def test_gettoas_archive_sharding_equals_serial(nfile, skip):
    """Every rank loads only its contiguous block of archives (none twice,
    none missed) and ends with exactly the serial run's per-archive
    attributes and TOA list (archive order; skipped archives absent; PSRCHIVE
    MJDs that cannot be pickled travel as their printed int/frac day)."""
    from pulseportraiture_amd import pptoas
    loaded, real = [], pptoas.load_data
    pptoas.load_data = _recording_loader(loaded)
    try:
        serial = _fake_gettoas(nfile, skip)
        serial.get_TOAs(quiet=True)
    finally:
        pptoas.load_data = real
    assert sorted(loaded) == sorted(serial.datafiles)
    ref = _summary(serial)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_archive_worker,
                         args=(r, 2, port, nfile, skip, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (seen, summ)) for r, seen, summ in
               (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(got[0][0] + got[1][0]) == list(range(nfile))
    assert got[0][0] == list(range(len(got[0][0])))
    for r in (0, 1):
        assert got[r][1] == ref


# ---------------------------------------------------------------------------
# GetTOAs' own batch gathering, sharding, table all-gather and bookkeeping
# for the scattering fits (configs[2] full: phi, DM, GM, tau, alpha;
# configs[4] scat: phi, DM, tau, alpha), with the device fit replaced by a
# deterministic CPU function of each sub-int's inputs: two ranks over gloo
# end with the serial run's attributes and TOAs, bit for bit
# ---------------------------------------------------------------------------
def _fit_fake(data, models, freqs, Ps, init, flags, nu_fits=None,
              nu_outs=None, errs=None, chan_mask=None, guess_tau=None,
              guess_weights=None, **kw):
    """ppf_fit_batch's output records as a function of the per-sub-int
    inputs only (never of the row's position in the batch)."""
    from pulseportraiture_amd import _lib
    x = np.asarray(data, dtype=np.float64)
    n, nchan = x.shape[:2]
    init, flags = np.asarray(init, float), np.asarray(flags, float)
    nu_fits, nu_outs = np.asarray(nu_fits, float), np.asarray(nu_outs, float)
    mask = np.asarray(chan_mask, float)
    tg = np.zeros(n) if guess_tau is None else np.asarray(guess_tau, float)
    rs = (x.sum(axis=2) * mask).sum(axis=1)
    I = _lib.RESULT_INDEX
    R = np.zeros((n, _lib.RESULT_DOUBLES))
    R[:, I["params"]] = init + 1e-6 * rs[:, None] * flags
    R[:, I["param_errs"]] = 1e-3 + 1e-4 * flags + tg[:, None]
    R[:, I["nu_out"]] = np.where(np.isnan(nu_outs), nu_fits, nu_outs)
    R[:, I["nu_fit"]] = nu_fits
    R[:, I["chi2"]] = rs
    R[:, I["red_chi2"]] = 1.0 + 1e-3 * mask.sum(axis=1)
    R[:, I["snr"]] = 10.0 + 1e-3 * rs
    R[:, I["nfeval"]] = 5 + flags.sum(axis=1)
    R[:, I["status"]] = 2
    cov = 1e-6 * (init[:, :, None] + init[:, None, :] + np.eye(5))
    t = torch.from_numpy
    return dict(results=t(R), scales=t(x.mean(axis=2) * mask),
                scale_errs=t(np.asarray(errs, float) * mask),
                channel_snrs=t(np.asarray(guess_weights, float) *
                               np.asarray(freqs, float) * 1e-3),
                covariance=t(cov))


class _CPUStaged(object):
    def __init__(self, rows):
        self.rows = rows

    def wait(self):
        return torch.from_numpy(np.ascontiguousarray(self.rows))

    def release(self):
        self.rows = None


class _CPUStager(object):
    def stage(self, rows):
        return _CPUStaged(np.asarray(rows))

    def close(self):
        pass


def _scat_archives(nfile):
    from pulseportraiture_amd.pplib import DataBunch, MJD
    out = {}
    for f in range(nfile):
        rng = np.random.default_rng(300 + f)
        nsub, nchan, nbin = 5, 6, 32
        ok = np.arange(nchan) if f % 2 == 0 else np.array([0, 1, 2, 4, 5])
        wts = np.ones((nsub, nchan))
        wts[:, np.setdiff1d(np.arange(nchan), ok)] = 0.0
        name = "s%d.fits" % f
        out[name] = DataBunch(
            arch=None, backend="be", backend_delay=0.0, bw=400.0,
            doppler_factors=1.0 + rng.uniform(-1e-4, 1e-4, nsub), DM=30.0,
            dmc=0, epochs=[MJD(57000 + f, 0.01 * i) for i in range(nsub)],
            filename=name, flux_prof=np.array([]),
            freqs=np.tile(np.linspace(400.0, 800.0, nchan), (nsub, 1)),
            frontend="fe", integration_length=50.0, masks=None, nbin=nbin,
            nchan=nchan, noise_stds=rng.uniform(0.5, 1.5, (nsub, 1, nchan)),
            npol=1, nsub=nsub, nu0=600.0, ok_ichans=[ok] * nsub,
            ok_isubs=np.arange(nsub), parallactic_angles=np.zeros(nsub),
            phases=np.arange(nbin) / nbin, prof=np.zeros(nbin),
            prof_noise=1.0, prof_SNR=20.0,
            Ps=np.full(nsub, 0.005) + 1e-6 * f,
            SNRs=rng.uniform(5, 50, (nsub, 1, nchan)), source="J0000+0000",
            state="Intensity",
            subints=rng.normal(size=(nsub, 1, nchan, nbin)).astype(np.float32),
            subtimes=[10.0] * nsub, telescope="GBT", telescope_code="1",
            weights=wts)
    return out


def _scat_gettoas(nfile):
    from pulseportraiture_amd import pptoas

    class G(pptoas.GetTOAs):
        def __init__(self):
            for a in pptoas._ATTRS:
                setattr(self, a, [])
            self.datafiles = ["s%d.fits" % i for i in range(nfile)]
            self.quiet = True
            self.modelfile = "t.gmodel"
            self.gparams = [0.0, 2e-3]
            self.model_nu_ref = 600.0
            self.ird = {"DM": 0.0, "wids": [], "irf_types": []}

        def _models(self, d, ok_isubs, fit_scat, quiet, host=True):
            return (np.zeros((1, d.nchan, d.nbin)),
                    np.zeros(len(ok_isubs), dtype=np.int32))
    return G()


def _scat_run(mode, nfile):
    from pulseportraiture_amd import engine, pptoas
    files = _scat_archives(nfile)
    saved = (pptoas.load_data, pptoas._Stager, pptoas._worker_stream,
             engine.device, engine.fit_batch)
    pptoas.load_data = lambda fn, **kw: files[fn]
    pptoas._Stager = _CPUStager
    pptoas._worker_stream = lambda dev: None
    engine.device = lambda *a, **k: -1       # torch.cuda.device(-1): no-op
    engine.fit_batch = _fit_fake
    try:
        gt = _scat_gettoas(nfile)
        gt.get_TOAs(quiet=True, fit_DM=True, fit_GM=(mode == "full"),
                    fit_scat=True)
        return _summary(gt)
    finally:
        (pptoas.load_data, pptoas._Stager, pptoas._worker_stream,
         engine.device, engine.fit_batch) = saved


def _scat_worker(rank, world, port, mode, nfile, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    sys.path.insert(0, os.path.dirname(__file__))
    import test_dist_gloo as T
    pdist.init("gloo")
    q.put((rank, T._scat_run(mode, nfile)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,nfile", [("full", 3), ("scat", 3),
                                        ("scat", 1)])
def test_gettoas_scattering_fits_sharded_equal_serial(mode, nfile):
    """full (fit_DM + fit_GM: sharded by sub-int in every archive) and scat
    (3 archives: sharded by archive; 1 archive: by sub-int), with ragged
    shards (5 sub-ints) and zapped channels: the 2-rank attributes, the
    scattering TOA flags and the tau guesses each sub-int was fitted from
    equal the serial run's."""
    serial = _scat_run(mode, nfile)
    assert len(serial["TOA_list"]) == 5 * nfile
    assert "scat_time" in serial["TOA_list"][0][5]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scat_worker,
                         args=(r, 2, port, mode, nfile, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        for k in serial:
            if k != "fit_durations":            # wall-clock times
                assert repr(got[r][k]) == repr(serial[k]), (r, k)


# ---- the bench.py self-launcher (dist.launch_local), CPU / gloo ----------

def _launch(argv, nproc, timeout=180):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = os.path.join(root, "tests", "launch_probe.py")
    code = ("import sys; sys.path.insert(0, %r); "
            "from pulseportraiture_amd import dist; "
            "sys.exit(dist.launch_local(%r, %r, %d, "
            "local_ranks=lambda r: 0))" % (root, probe, argv, nproc))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-c", code], capture_output=True,
                         text=True, timeout=timeout, env=env)
    lines = [json.loads(ln) for ln in out.stdout.splitlines()
             if ln.startswith("{")]
    return out.returncode, lines, out.stdout, out.stderr


@pytest.mark.parametrize("nproc", [2, 3])
def test_self_launcher_starts_ranks_and_forwards_rank0(nproc):
    """bench.py --gpus N without torchrun: N child ranks, each with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set, gathered rows in global order,
    exactly one JSON line (rank 0's) on the launcher's stdout."""
    rc, lines, so, se = _launch(["11"], nproc)
    assert rc == 0, se
    assert len(lines) == 1, so
    d = lines[0]
    assert d["world"] == nproc and d["rank"] == 0 and d["local_rank"] == 0
    assert d["launcher"] == "bench-self" and d["master"] == "127.0.0.1"
    assert d["first_col"] == [float(i) for i in range(11)]
    for r in range(1, nproc):
        assert "[rank %d] rank %d local 0 done" % (r, r) in se


def test_self_launcher_fails_when_a_rank_fails():
    """A rank that exits non-zero fails the launch (its exit code), and the
    ranks left waiting in the all-gather are stopped, not left hanging."""
    import time
    t0 = time.monotonic()
    rc, lines, so, se = _launch(["11", "1"], 2, timeout=120)
    assert rc == 3, (so, se)
    assert lines == []
    assert "rank 1 exited with 3" in se
    assert time.monotonic() - t0 < 100

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

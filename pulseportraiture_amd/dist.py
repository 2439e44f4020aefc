"""Multi-GPU sharding: one process per GPU, torch.distributed over RCCL.

Sub-integrations (and archives) are independent:
nothing couples two of them inside the fit, so each rank fits a contiguous
block of the global sub-integration index with NO data-path collective; the
only exchange is one all-gather of the fixed-size result records at the end
of a batch (``backend="nccl"`` is RCCL over xGMI on ROCm).  ``gloo`` runs the
same code on CPU tensors for tests.
"""
import os

import torch
import torch.distributed as dist


def env_rank_world():
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    return rank, world, local


def init(backend="nccl"):
    """Initialise the process group from torchrun's env (no-op at world 1)."""
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device(
                "cuda", local))
        else:
            dist.init_process_group(backend)
    elif backend == "nccl" and torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def shard(n_total, rank, world):
    """Contiguous, balanced block of [0, n_total) for `rank`: (first, count).
    Ranks differ by at most one sub-integration."""
    base, extra = divmod(n_total, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def allgather_rows(local, n_total, world):
    """All-gather per-sub-integration rows [count, ...] from every rank into
    [n_total, ...] in global order (blocks padded to equal size for the
    collective, then trimmed)."""
    if world == 1:
        return local
    if local.is_cuda and backend() == "gloo":      # (rehearsals: gloo is CPU-only)
        return allgather_rows(local.cpu(), n_total, world).to(local.device)
    per = -(-n_total // world)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    pad[:local.shape[0]] = local
    out = torch.empty((per * world,) + tuple(local.shape[1:]),
                      dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad)
    rows = []
    for r in range(world):
        first, count = shard(n_total, r, world)
        rows.append(out[r * per:r * per + count])
    return torch.cat(rows, 0)


def barrier():
    if dist.is_initialized():
        dist.barrier()


def collective_device(device=None):
    """Device of a small tensor handed to a collective: None (CPU) under
    gloo; under nccl (RCCL has no CPU path) the given device, else this
    rank's current HIP device."""
    b = backend()
    if b == "gloo":
        return None
    if device is None and b == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return device


def max_over_ranks(x, device=None):
    """Max of a python float over ranks (used for timings)."""
    if not dist.is_initialized():
        return x
    device = collective_device(device)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def is_dist():
    return dist.is_initialized() and dist.get_world_size() > 1


def allreduce_sum_(*tensors):
    """In-place sum over ranks (ppalign's aligned portrait and channel
    weights: the one exchange of the alignment iteration)."""
    if not is_dist():
        return tensors
    for t in tensors:
        if t.is_cuda and backend() == "gloo":       # (rehearsals)
            c = t.cpu()
            dist.all_reduce(c, op=dist.ReduceOp.SUM)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return tensors


def raise_if_any_failed(err, device=None):
    """Collective error check: every rank calls this with its own exception
    (or None) BEFORE the next collective, so a failure on one rank raises on
    every rank instead of leaving the others blocked in that collective."""
    if not is_dist():
        if err is not None:
            raise err
        return
    device = collective_device(device)
    t = torch.tensor([1.0 if err is not None else 0.0], dtype=torch.float64,
                     device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if err is not None:
        raise err
    if t.item() > 0.0:
        raise RuntimeError("another rank failed (its exception is raised "
                           "there)")


def backend():
    """The process group's backend ('nccl' = RCCL, 'gloo'), or None."""
    return dist.get_backend() if dist.is_initialized() else None


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local(script, argv, nproc, local_ranks=None, poll_s=0.2):
    """Start `nproc` ranks of `script` on this node and wait for them: the
    launcher `bench.py --gpus N` uses when nothing set WORLD_SIZE (as
    ``torch.distributed.run --nnodes 1 --nproc-per-node N`` would).

    This process never touches a GPU and never re-execs: each rank is a child
    process (``sys.executable script argv``) with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR (127.0.0.1) / MASTER_PORT set.  LOCAL_RANK is
    the rank (one GPU per rank) unless `local_ranks` maps it (the one-GPU
    gloo rehearsal puts every rank on device 0).  Rank 0's stdout is
    forwarded to this process's stdout line by line (it carries the bench
    JSON line); the other ranks' stdout goes to stderr with a rank prefix.
    If any rank fails, the others are terminated (by their own PIDs) so none
    waits forever in a collective.  Returns 0, or the first failing rank's
    exit code (1 if that was a signal)."""
    import subprocess
    import sys
    import threading
    import time
    port = free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nproc),
                   LOCAL_RANK=str(local_ranks(r) if local_ranks else r),
                   LOCAL_WORLD_SIZE=str(nproc), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   PPF_LAUNCHER="bench-self")
        procs.append(subprocess.Popen([sys.executable, script] + list(argv),
                                      env=env, stdout=subprocess.PIPE,
                                      text=True, bufsize=1))

    def pump(r, p):
        dst = sys.stdout if r == 0 else sys.stderr
        for ln in p.stdout:
            dst.write(ln if r == 0 else "[rank %d] %s" % (r, ln))
            dst.flush()

    pumps = [threading.Thread(target=pump, args=(r, p), daemon=True)
             for r, p in enumerate(procs)]
    for t in pumps:
        t.start()
    rc = 0
    t_term = None
    live = list(range(nproc))
    while live:
        for r in list(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.remove(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print("[launcher] rank %d exited with %d; stopping the "
                      "others" % (r, c), file=sys.stderr, flush=True)
                for q in live:
                    procs[q].terminate()
                t_term = time.monotonic()
        if live and t_term is not None and time.monotonic() - t_term > 30.0:
            for q in live:                  # ignored SIGTERM (e.g. in a collective)
                procs[q].kill()
        if live:
            time.sleep(poll_s)
    for t in pumps:
        t.join(timeout=10)
    return rc

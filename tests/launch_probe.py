"""A rank of the launcher tests (tests/test_dist_gloo.py): started by
pulseportraiture_amd.dist.launch_local, it joins the gloo group from the
environment the launcher set, shards a small deterministic table as bench.py
does, all-gathers it, and rank 0 prints one JSON line.
    argv: N_TOTAL [fail-rank]   (fail-rank: that rank exits 3 before the
    gather, the others block in it until the launcher stops them)"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pulseportraiture_amd import dist as pdist  # noqa: E402


def main():
    n_total = int(sys.argv[1])
    fail = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    rank, world, local = pdist.init("gloo")
    if rank == fail:
        sys.exit(3)
    first, count = pdist.shard(n_total, rank, world)
    rows = torch.arange(first, first + count, dtype=torch.float64)[:, None] * \
        torch.ones((1, 4), dtype=torch.float64)
    full = pdist.allgather_rows(rows, n_total, world)
    if rank == 0:
        print(json.dumps(dict(
            world=world, rank=rank, local_rank=local,
            launcher=os.environ.get("PPF_LAUNCHER"),
            master=os.environ.get("MASTER_ADDR"),
            rows_sha256=hashlib.sha256(full.numpy().tobytes()).hexdigest(),
            first_col=full[:, 0].tolist())), flush=True)
    else:
        print("rank %d local %d done" % (rank, local), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py to
per-unit HBM traffic (profiles/pmc_summary.json, read by bench.py).

    python profiles/pmc_reduce.py <fetch_dir> <write_dir> <bench_json_log> \
        [--nchan 512] [--out profiles/pmc_summary.json]

Counter handling follows MI355X_MICROARCH.md (HBM section): counters are in
KiB; FETCH_SIZE counts half of the bytes of wide coalesced streaming reads on
gfx950, so it is doubled; WRITE_SIZE is taken as is.  Unit: one
sub-integration; a launch processes `chunk` sub-integrations (bench config).
  xmom -- the first (full) fused moment pass k_xmom_g<*, *, *, true>
  dsum -- the guess-profile pass k_dsum_w
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                  recursive=True)[0]
    rows = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        rows[r["Kernel_Name"]].append(r)
    return rows


def pick(rows, key):
    return [r for k, v in rows.items() if key in k for r in v]


KERNELS = {"xmom": ("k_xmom_g<", ", true>"), "dsum": ("k_dsum_w<", "")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("bench_log")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(
        os.path.abspath(__file__)), "pmc_summary.json"))
    a = ap.parse_args()
    line = [l for l in open(a.bench_log) if l.startswith("{")][-1]
    bench = json.loads(line)
    per_launch = min(bench["config"]["chunk"], bench["config"]["nsub_per_gpu"])
    fr, wr = load(a.fetch_dir), load(a.write_dir)
    KiB = 1024.0
    out = dict(source=dict(fetch=a.fetch_dir, write=a.write_dir,
                           bench=bench["config"]["workload"],
                           correction="FETCH_SIZE x2 (gfx950 wide reads), "
                                      "WRITE_SIZE x1, KiB -> bytes"),
               kernels={})
    for key, (pre, post) in KERNELS.items():
        sel = lambda rows: [r for k, v in rows.items()
                            if pre in k and post in k for r in v]
        f, w = sel(fr), sel(wr)
        if not f or not w:
            continue
        fb = sum(float(r["Counter_Value"]) for r in f) * KiB * 2 / len(f)
        wb = sum(float(r["Counter_Value"]) for r in w) * KiB / len(w)
        out["kernels"][key] = dict(
            unit="sub-integration", subints_per_launch=per_launch,
            fetch_bytes=fb / per_launch, write_bytes=wb / per_launch,
            hbm_bytes=(fb + wb) / per_launch, launches=len(f),
            kernel=sorted({r["Kernel_Name"] for r in f}))
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

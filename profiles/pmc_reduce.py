#!/usr/bin/env python
"""Reduce the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of a
tools/prof.sh run of bench.py to HBM traffic per unit of work
(profiles/pmc_summary.json, read by bench.py for `roofline.traffic`).

    python profiles/pmc_reduce.py gpurun_out/prof_TAG [--out ...]

Counter handling follows MI355X_MICROARCH.md (HBM section): counters are in
KiB; FETCH_SIZE counts half of the bytes of wide coalesced streaming reads on
gfx950, so it is doubled; WRITE_SIZE is taken as is.  Entries are keyed by
the bench fit mode (phase+DM, full, scat) and kernel:
  xmom  -- the first (full) fused moment pass k_xmom_g<*, *, *, true>;
           unit = one sub-integration
  dsum  -- the guess-profile pass k_dsum_w; unit = one sub-integration
  xspec -- the cross-spectrum pass k_xspec_w; unit = one sub-integration
  pass  -- the streaming trust-region evaluation k_pass<true>; unit = one
           evaluation of one sub-integration (the run's launches process
           nsub x mean_passes_per_fit evaluations per call)
  moments -- k_moments (moments from the stored cross spectrum): every
           launch, re-centring launches included, per sub-integration of a
           launch (so a lower bound per first-pass sub-integration)
"""
import argparse
import collections
import csv
import glob
import json
import os

KERNELS = {"xmom": ("k_xmom_g<", ", true>"), "dsum": ("k_dsum_w<", ""),
           "xspec": ("k_xspec_w", ""), "pass": ("k_pass<true>", ""),
           "moments": ("k_moments", ""), "accum": ("k_align", ""), "noise": ("k_noise_w<", "")}


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                  recursive=True)[0]
    rows = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        rows[r["Kernel_Name"]].append(r)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(
        os.path.abspath(__file__)), "pmc_summary.json"))
    a = ap.parse_args()
    line = [ln for ln in open(os.path.join(a.prof_dir, "ks.log"))
            if ln.startswith("{")][-1]
    bench = json.loads(line)
    cfg = bench["config"]
    # (non-power-of-two nbin: its own entry, e.g. "phase+DM@1000")
    nb = cfg.get("nbin", 2048)
    mode = cfg["fit"] if nb & (nb - 1) == 0 else "%s@%d" % (cfg["fit"], nb)
    calls = bench["steps"] + bench["warmup"]
    per_launch = min(cfg.get("chunk", cfg["nsub_per_gpu"]), cfg["nsub_per_gpu"])
    fr = load(os.path.join(a.prof_dir, "fetch"))
    wr = load(os.path.join(a.prof_dir, "write"))
    KiB = 1024.0
    old = json.load(open(a.out)) if os.path.exists(a.out) else {}
    out = old if "modes" in old else {"modes": {}}
    ent = dict(source=dict(prof=a.prof_dir, bench=cfg["workload"],
                           correction="FETCH_SIZE x2 (gfx950 wide reads), "
                                      "WRITE_SIZE x1, KiB -> bytes"),
               kernels={})
    for key, (pre, post) in KERNELS.items():
        def sel(rows):
            return [r for k, v in rows.items() if pre in k and post in k
                    for r in v]
        f, w = sel(fr), sel(wr)
        if not f or not w:
            continue
        fb = sum(float(r["Counter_Value"]) for r in f) * KiB * 2
        wb = sum(float(r["Counter_Value"]) for r in w) * KiB
        if key == "pass":
            units = calls * cfg["nsub_per_gpu"] * bench["mean_passes_per_fit"]
            unit = "sub-integration evaluation"
        else:
            units = len(f) * per_launch
            unit = "sub-integration"
        ent["kernels"][key] = dict(
            unit=unit, units=units, launches=len(f),
            fetch_bytes=fb / units, write_bytes=wb / units,
            hbm_bytes=(fb + wb) / units,
            kernel=sorted({r["Kernel_Name"] for r in f}))
    out["modes"][mode] = ent
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()

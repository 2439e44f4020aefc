#!/usr/bin/env python
"""Reduce the SQ counter passes of a tools/prof.sh run of bench.py to the
fp64 work per unit of each hot kernel (profiles/fp64_summary.json, read by
bench.py for its `fp64` roofline object).

    python profiles/fp64_reduce.py gpurun_out/prof_TAG [--out ...]

Per kernel, summed over its dispatches in the run:
  valu_f64  -- f64 VALU wave-instructions (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64)
  flops     -- 64 lanes x (ADD + MUL + TRANS + 2 FMA) + 512 x
               SQ_INSTS_VALU_MFMA_MOPS_F64 (one MOP = 512 flops: a
               v_mfma_f64_16x16x4 is 4 MOPS = 16 x 16 x 4 x 2 flops)
  valu_active_per_wave -- SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (the fraction
               of a wave's life it issues VALU; x waves per SIMD = the SIMD's
               VALU-issue fraction)
  clock_ghz -- GRBM_GUI_ACTIVE per dispatch and XCD / the kernel's mean
               duration (the shader clock the chip held)
Units follow pmc_reduce.py: xmom/dsum/xspec per sub-integration of a launch,
pass per sub-integration evaluation.
"""
import argparse
import collections
import csv
import glob
import json
import os

KERNELS = {"xmom": ("k_xmom_g<", ", true>"), "dsum": ("k_dsum_w<", ""),
           "xspec": ("k_xspec_w", ""), "pass": ("k_pass<true>", ""),
           "tr_mom": ("k_tr_mom", ""), "postfit": ("k_postfit", ""),
           "moments": ("k_moments", ""), "accum": ("k_align", "")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(
        os.path.abspath(__file__)), "fp64_summary.json"))
    a = ap.parse_args()
    line = [ln for ln in open(os.path.join(a.prof_dir, "ks.log"))
            if ln.startswith("{")][-1]
    bench = json.loads(line)
    cfg = bench["config"]
    calls = bench["steps"] + bench["warmup"]
    per_launch = min(cfg.get("chunk", cfg["nsub_per_gpu"]), cfg["nsub_per_gpu"])
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    grbm_rows = collections.defaultdict(int)
    files = sorted(glob.glob(os.path.join(a.prof_dir, "*", "*counter_collection.csv")))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                grbm_rows[k] += 1
    dur = {}
    ks = glob.glob(os.path.join(a.prof_dir, "ks", "*kernel_stats.csv"))
    if ks:
        for r in csv.DictReader(open(ks[0])):
            dur[r["Name"]] = float(r["AverageNs"])
    old = json.load(open(a.out)) if os.path.exists(a.out) else {}
    out = old if "modes" in old else {"modes": {}}
    ent = dict(source=dict(prof=a.prof_dir, bench=cfg["workload"]), kernels={})
    for key, (pre, post) in KERNELS.items():
        names = [k for k in cnt if pre in k and post in k]
        if not names:
            continue
        v = collections.defaultdict(float)
        for k in names:
            for c, x in cnt[k].items():
                v[c] += x
        # dispatches of the run = distinct ids in one counter pass
        nd = max(len({r["Dispatch_Id"] for r in csv.DictReader(open(f))
                      if r["Kernel_Name"] in names}) for f in files)
        if key == "pass":
            units = calls * cfg["nsub_per_gpu"] * bench["mean_passes_per_fit"]
            unit = "sub-integration evaluation"
        else:
            units = nd * per_launch
            unit = "sub-integration"
        valu = (v["SQ_INSTS_VALU_ADD_F64"] + v["SQ_INSTS_VALU_MUL_F64"] +
                v["SQ_INSTS_VALU_FMA_F64"] + v["SQ_INSTS_VALU_TRANS_F64"])
        flops = 64.0 * (valu + v["SQ_INSTS_VALU_FMA_F64"]) + \
            512.0 * v["SQ_INSTS_VALU_MFMA_MOPS_F64"]
        e = dict(unit=unit, units=units, dispatches=nd,
                 valu_f64_per_unit=valu / units,
                 mfma_f64_per_unit=v["SQ_INSTS_VALU_MFMA_MOPS_F64"] / 4.0 / units,
                 valu_all_per_unit=v["SQ_INSTS_VALU"] / units,
                 flops_per_unit=flops / units,
                 valu_active_per_wave=(v["SQ_ACTIVE_INST_VALU"] /
                                       v["SQ_WAVE_CYCLES"]) if v["SQ_WAVE_CYCLES"] else None,
                 kernel=sorted(names))
        dn = [dur[k] for k in names if k in dur]
        if dn and grbm_rows.get(names[0]):
            rows = sum(grbm_rows[k] for k in names)
            # GRBM_GUI_ACTIVE rows sum the 8 XCDs
            e["clock_ghz"] = v["GRBM_GUI_ACTIVE"] / rows / 8.0 / (sum(dn) / len(dn))
        ent["kernels"][key] = e
    # (non-power-of-two nbin: its own entry, e.g. "phase+DM@1000")
    nb = cfg.get("nbin", 2048)
    out["modes"][cfg["fit"] if nb & (nb - 1) == 0 else "%s@%d" % (cfg["fit"], nb)] = ent
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()

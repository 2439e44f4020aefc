#!/usr/bin/env python
"""Per-kernel table of a tools/prof.sh run: dispatches, average duration
(kernel trace), per-dispatch averages of every PMC counter, plus derived
figures (HBM bytes with the gfx950 FETCH_SIZE x2 correction, L2 hit rate,
f64 ops).  usage: python tools/pmc_table.py gpurun_out/prof_TAG [filter]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    ks = glob.glob(os.path.join(d, "ks", "*kernel_stats.csv"))[0]
    dur = {}
    for r in csv.DictReader(open(ks)):
        dur[r["Name"]] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"], r["Dispatch_Id"])
            disp[key][r["Counter_Name"]] = disp[key].get(
                r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (name, _), cs in disp.items():
            for c, v in cs.items():
                ctr[name][c].append(v)
    for name in sorted(dur, key=lambda n: -dur[n][0] * dur[n][1]):
        if filt not in name:
            continue
        calls, us = dur[name]
        print("%-60s calls %5d  avg %9.2f us  total %8.2f ms" %
              (name[:60], calls, us, calls * us / 1e3))
        cs = ctr.get(name, {})
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(avg):
            print("    %-32s %16.1f" % (c, avg[c]))
        if "FETCH_SIZE" in avg:
            rd = avg["FETCH_SIZE"] * 1024 * 2
            wr = avg.get("WRITE_SIZE", 0.0) * 1024
            print("    HBM read %.3f MB (x2 corr), write %.3f MB, %.1f GB/s"
                  % (rd / 1e6, wr / 1e6, (rd + wr) / (us * 1e3)))
        if "TCC_HIT_sum" in avg:
            h, m = avg["TCC_HIT_sum"], avg["TCC_MISS_sum"]
            print("    L2 hit rate %.3f" % (h / max(1.0, h + m)))
        f64 = sum(avg.get(c, 0.0) * w for c, w in (
            ("SQ_INSTS_VALU_ADD_F64", 64), ("SQ_INSTS_VALU_MUL_F64", 64),
            ("SQ_INSTS_VALU_FMA_F64", 128), ("SQ_INSTS_VALU_TRANS_F64", 64)))
        if f64:
            print("    f64 VALU %.3f GFLOP -> %.2f TFLOP/s" %
                  (f64 / 1e9, f64 / (us * 1e-6) / 1e12))
        if "SQ_BUSY_CYCLES" in avg and "SQ_WAVE_CYCLES" in avg:
            print("    wave-cycles/busy %.2f  valu/wave-cycles %.3f  "
                  "wait/wave-cycles %.3f" % (
                      avg["SQ_WAVE_CYCLES"] / max(1, avg["SQ_BUSY_CYCLES"]),
                      avg.get("SQ_ACTIVE_INST_VALU", 0) / max(
                          1, avg["SQ_WAVE_CYCLES"]),
                      avg.get("SQ_WAIT_ANY", 0) / max(1, avg["SQ_WAVE_CYCLES"])))


if __name__ == "__main__":
    main()

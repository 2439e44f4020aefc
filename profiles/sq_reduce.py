"""Per-kernel sums of rocprofv3 --pmc counter passes (SQ_* / GRBM_*), for
the issue/wait split of the fit kernels.
    python profiles/sq_reduce.py DIR [DIR ...]   (each DIR holds one
    *_counter_collection.csv) -> a table on stdout, kernels with >= 1% of
the total SQ_BUSY_CYCLES / SQ_WAVE_CYCLES, and the derived ratios."""
import collections
import csv
import glob
import os
import sys


def load(d):
    f = glob.glob(os.path.join(d, "*_counter_collection.csv"))[0]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
    return tot, calls


def main():
    tot = collections.defaultdict(dict)
    calls = {}
    for d in sys.argv[1:]:
        t, c = load(d)
        for k, v in t.items():
            tot[k].update(v)
            calls[k] = len(c[k])
    key = "SQ_WAVE_CYCLES"
    allw = sum(v.get(key, 0.0) for v in tot.values()) or 1.0
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get(key, 0.0)):
        if v.get(key, 0.0) < 0.01 * allw:
            continue
        print("%s  calls %d" % (k, calls[k]))
        for c in sorted(v):
            print("   %-22s %.4g" % (c, v[c]))
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in v:
                    print("   %-22s %.3f of wave cycles" % (c, v[c] / wc))
        if v.get("SQ_INSTS_LDS"):
            print("   LDS bank conflicts per LDS instruction %.3f"
                  % (v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_INSTS_LDS"]))


if __name__ == "__main__":
    main()

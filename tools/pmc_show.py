"""Summarise tools/pmc_sq.sh output per kernel: python tools/pmc_show.py <dir> [substr...]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
keys = sys.argv[2:] or ["xspec", "xmom", "dsum", "guess", "tr_mom"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(d + "/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if not any(s in k for s in keys):
        continue
    W = v["SQ_WAVE_CYCLES"] or 1
    nw = v["SQ_WAVES"] or 1
    print("%-40s waves %8d valu/w %6.0f lds/w %5.0f mfma/w %4.0f | wait %.2f winst %.2f act %.2f valu %.2f lds %.2f | bconf/lds %.2f wlds %.2f mfmabusy %.3g gui %.3g" % (
        k, nw, v["SQ_INSTS_VALU"] / nw, v["SQ_INSTS_LDS"] / nw, v["SQ_INSTS_MFMA"] / nw,
        v["SQ_WAIT_ANY"] / W, v["SQ_WAIT_INST_ANY"] / W, v["SQ_ACTIVE_INST_ANY"] / W,
        v["SQ_ACTIVE_INST_VALU"] / W, v["SQ_ACTIVE_INST_LDS"] / W,
        v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_INSTS_LDS"]), v["SQ_WAIT_INST_LDS"] / W,
        v["SQ_VALU_MFMA_BUSY_CYCLES"], v["GRBM_GUI_ACTIVE"]))

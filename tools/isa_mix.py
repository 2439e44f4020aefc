"""Static instruction mix of one kernel in a hipcc --save-temps .s file, per
basic block (so the per-row loop body can be read off):
    python tools/isa_mix.py file.s <kernel-substring> [--blocks]"""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_") and "f64" in op:
        return "valu64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read().split("\n")
    start = next(i for i, l in enumerate(s) if re.match(r"^_Z\S*%s\S*:" % re.escape(pat), l))
    end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
    print(s[start].split(":")[0])
    blocks = collections.OrderedDict()
    cur = "entry"
    blocks[cur] = collections.Counter()
    for l in s[start + 1:end]:
        t = l.strip()
        if re.match(r"^\.LBB\S*:", t):
            cur = t.split(":")[0]
            blocks[cur] = collections.Counter()
            continue
        if not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        blocks[cur][classify(op)] += 1
        blocks[cur]["_n"] += 1
    tot = collections.Counter()
    for c in blocks.values():
        tot.update(c)
    print("total", dict(tot))
    if "--blocks" in sys.argv:
        for k, c in blocks.items():
            if c["_n"] >= 40:
                print(k, dict(c))


if __name__ == "__main__":
    main()

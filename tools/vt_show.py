"""Per-kernel durations (us) of the last bench step from tools/var_trace.sh traces:
python tools/vt_show.py gpurun_out/vt_*"""
import collections, csv, glob, sys
for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    if not f:
        continue
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last ppf_fit_batch call: from the last k_rfft_rows on
    last = max(i for i, r in enumerate(rows) if "k_rfft_rows" in r["Kernel_Name"])
    tot = collections.OrderedDict()
    for r in rows[last:]:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ppf::", "")[:28]
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot.setdefault(n, []).append(dt)
    print(d.split("/")[-1], " ".join("%s=%s" % (k, "+".join("%.0f" % x for x in v[:3]) + ("..%d" % len(v) if len(v) > 3 else "")) for k, v in tot.items() if sum(v) > 20))

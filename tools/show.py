#!/usr/bin/env python
"""Print the key fields of bench.py JSON lines: python tools/show.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        ln = [x for x in open(f) if x.startswith("{")][-1]
    except (OSError, IndexError):
        print(f, "-- no JSON line")
        continue
    d = json.loads(ln)
    r = d.get("roofline") or {}
    c = d.get("cpu_baseline") or {}
    print("%s: %s %s %s/step=%sms stages=%s" % (
        f, d["value"], d["unit"], d["config"].get("fit"), d["ms_per_step"],
        d.get("stage_ms")))
    if r:
        print("   roofline %s %.1f GB/s frac %.3f traffic %s alg/launch %.0f "
              "launch %.3f ms x%s" % (r["kernel"], r["achieved"], r["frac"],
                                      r["traffic"],
                                      r["algorithmic_bytes_per_launch"],
                                      r["avg_launch_ms"], r.get("launches")))
    if c:
        print("   cpu %.4g %s (ref-equiv %s, all-core %s)" % (
            c["value"], c["sample"], c.get("reference_equiv_value"),
            (c.get("all_core") or {}).get("value")))
    if d.get("parity"):
        print("   parity", d["parity"])
    if d.get("kernels"):
        print("   kernels", {k: (v["avg_launch_ms"], v.get("gbs"))
                            for k, v in d["kernels"].items()})

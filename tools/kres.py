"""Per-kernel VGPR / AGPR / scratch / occupancy of a HIP source:
python tools/kres.py file.hip [regex] [-- extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "--" else "."
extra = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
       "-ffp-contract=fast", "-munsafe-fp-atomics", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for ln in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", ln)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if re.search(pat, r["name"]):
        print("%-60s vgpr %4s agpr %4s scratch %5s occ %s" % (
            r["name"][:60], r.get("VGPRs"), r.get("AGPRs"),
            r.get("ScratchSize [bytes/lane]"), r.get("Occupancy [waves/SIMD]")))

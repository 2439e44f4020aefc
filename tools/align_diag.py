"""C4 diagnostics: distance from the guess to the fitted point vs data passes
(run on the GPU box; writes gpurun_out/align_diag.npz)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from pulseportraiture_amd import _lib

captured = {}
orig = bench.ppalign._fit_rows if hasattr(bench, "ppalign") else None
from pulseportraiture_amd import ppalign
real = ppalign._fit_rows


def spy(rows, model, mi, dc, fit_dm, nbin, dev):
    out = real(rows, model, mi, dc, fit_dm, nbin, dev)
    captured.setdefault("r", []).append(dc["last_results"].cpu().numpy())
    return out


ppalign._fit_rows = spy
sys.argv = ["bench.py", "--fit", "align", "--nsub", "1000", "--nchan", "256",
            "--nbin", "1024", "--steps", "3", "--warmup", "0"]
bench.main()
I = _lib.RESULT_INDEX
for it, r in enumerate(captured["r"]):
    dphi = (r[:, I["x_fit_phi"]] - r[:, I["phi_guess"]] + 0.5) % 1.0 - 0.5
    npass = r[:, I["npass"]].astype(int)
    dm = r[:, I["params"]][:, 1] - 34.56789
    print("iter", it, "npass hist", np.bincount(npass).tolist())
    for k in range(1, npass.max() + 1):
        sel = npass == k
        if sel.any():
            print("  npass=%d n=%d |dphi|*nbin median %.3f max %.3f  |dDM| median %.2e  niter med %.1f" % (
                k, sel.sum(), np.median(abs(dphi[sel])) * 1024, abs(dphi[sel]).max() * 1024,
                np.median(abs(dm[sel])), np.median(r[sel, I["niter"]])))
np.savez("gpurun_out/align_diag.npz", *captured["r"])

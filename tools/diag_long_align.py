"""Diagnostic: synthetic ppalign (device) vs the oracle at several nbin,
printing the worst aligned-portrait difference and the per-sub-int phases."""
import sys, time
sys.path[:0] = ['.', 'tests']
import numpy as np
import fullshape as F
from oracle import ppfit_oracle as O
from pulseportraiture_amd import ppalign, pptoas

import os
NCH = int(os.environ.get("NCH", 8))
NOISE = float(os.environ.get("NOISE", 0.5))
for nbin in [int(x) for x in sys.argv[1:]]:
    t = time.time()
    archives, model_data = F.align_synthetic(NCH, nbin, 1, 2, 71, NOISE)
    files = {"arch%d.fits" % i: a for i, a in enumerate(archives)}
    files["guess.fits"] = model_data
    pptoas.load_data = lambda n, **kw: files[n]
    r = ppalign.align_archives(["arch0.fits", "arch1.fits"], "guess.fits",
                               fit_dm=True, niter=1, outfile=None, quiet=True)
    ref, tw = O.align_archives(archives, model_data, fit_dm=True, niter=1)
    d = np.abs(r.port[0] - ref[0]).max() / np.abs(ref).max()
    dw = np.abs(r.total_weights - tw).max() / np.abs(tw).max()
    print("nchan %d noise %g nbin %d: port rel %.3e  weights rel %.3e  (%.1f s)" % (NCH, NOISE, nbin, d, dw, time.time() - t), flush=True)

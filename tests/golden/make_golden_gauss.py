#!/usr/bin/env python
"""Golden vectors for the Gaussian-component model portraits
(pplib.gen_gaussian_portrait pplib.py:886-963, gaussian_profile 801-856,
read_model 2971-3057), produced by running the REFERENCE in this container
(never on the GPU box) with the import shims of make_golden.py.

Cases cover both evolution codes for each of loc/wid/amp, locs outside
[0, 1) and next to the wrap, widths that evolve through zero (the zeroout
branch), narrow (< 1 bin) and wide components, non-zero TAU (the scattering
convolution, read_model's TAU [s] -> [bin] scaling through a .gmodel file
with a TAU line) and standalone gaussian_profile calls.

Usage:  python tests/golden/make_golden_gauss.py
"""
import contextlib
import io
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (imports the reference with the shims)
import numpy as np  # noqa: E402

pplib = mg.pplib


def comp(loc, mloc, wid, mwid, amp, mamp):
    return [loc, mloc, wid, mwid, amp, mamp]


def params_of(dc, tau, comps):
    return np.array([dc, tau] + [v for c in comps for v in c], dtype=float)


EXAMPLE = mg.pplib.read_model(mg.GMODEL, quiet=True)   # (name, code, nu_ref, ngauss, params, ...)

CASES = {
    # the example template GetTOAs builds for every sub-integration
    "example_64x512": dict(code=EXAMPLE[1], params=EXAMPLE[4], alpha=EXAMPLE[6],
                           nu_ref=EXAMPLE[2], freqs=mg.channel_freqs(64), nbin=512),
    # linear evolution everywhere; locs outside [0, 1) and at the wrap
    "linear_32x256": dict(code="111", params=params_of(0.05, 0.0, [
        comp(1.30, 2e-4, 0.05, 1e-5, 3.0, -1e-3),
        comp(-0.20, -1e-4, 0.02, 0.0, 1.5, 2e-3),
        comp(0.985, 3e-5, 0.03, -2e-5, 2.0, 0.0)]), alpha=-4.0,
        nu_ref=1400.0, freqs=mg.channel_freqs(32, 1000.0, 800.0), nbin=256),
    # width evolving through zero (zeroout), narrow sub-bin component,
    # scattering with a shallow index
    "mixed_scat_48x1024": dict(code="010", params=params_of(-0.01, 3.0, [
        comp(0.40, 0.5, 0.04, -1e-4, 4.0, -1.2),
        comp(0.70, -0.3, 4e-4, 0.0, 6.0, 0.8),
        comp(0.10, 0.0, 0.20, 0.0, 0.5, -2.0)]), alpha=-3.5,
        nu_ref=1300.0, freqs=mg.channel_freqs(48, 1100.0, 800.0), nbin=1024),
    # strong scattering (power laws) at low frequencies, 2048 bins
    "scat_16x2048": dict(code="000", params=params_of(0.0, 40.0, [
        comp(0.25, -0.01, 0.03, -1.5, 5.0, -1.6),
        comp(0.30, 0.02, 0.06, 0.5, 2.0, -0.5),
        comp(0.60, 0.0, 0.015, 0.0, 1.0, 0.0),
        comp(0.95, 0.0, 0.10, 0.3, 0.7, 1.0),
        comp(0.05, 0.0, 0.01, 0.0, 3.0, -3.0)]), alpha=-4.0,
        nu_ref=600.0, freqs=mg.channel_freqs(16, 400.0, 400.0), nbin=2048),
    # one channel, 32 bins, a component wider than the profile
    "tiny_1x32": dict(code="001", params=params_of(1.0, 0.0, [
        comp(0.5, 0.0, 0.7, 0.0, 1.0, 0.0),
        comp(0.02, 0.0, 0.01, 0.0, 2.0, 0.01)]), alpha=-4.0,
        nu_ref=1500.0, freqs=np.array([1500.0]), nbin=32),
}

PROFILES = [(512, 0.3, 0.05), (512, 1.7, 0.01), (256, -0.4, 0.2),
            (128, 0.999, 0.002), (1024, 0.5, 0.0), (64, 0.0, 1.5)]

GMODEL_TAU = """MODEL   SCAT_TEST
CODE    000
FREQ    1500.00000
DC      0.01 1
TAU     0.00050000 1
ALPHA  -4.400      0
COMP01  0.30 1  -0.01 1   0.04 1  -1.0 1    5.0 1   -1.5 1
COMP02  0.55 1   0.00 1   0.02 1   0.5 1    2.0 1    0.3 1
"""


def main():
    out = {}
    for name, c in CASES.items():
        with contextlib.redirect_stdout(io.StringIO()):
            port = pplib.gen_gaussian_portrait(
                c["code"], np.array(c["params"], dtype=float), c["alpha"],
                pplib.get_bin_centers(c["nbin"]), c["freqs"], c["nu_ref"])
        out[name + "__code"] = np.array(c["code"])
        out[name + "__params"] = np.array(c["params"], dtype=float)
        out[name + "__alpha"] = np.float64(c["alpha"])
        out[name + "__nu_ref"] = np.float64(c["nu_ref"])
        out[name + "__freqs"] = np.asarray(c["freqs"], dtype=float)
        out[name + "__out"] = port
    for i, (nbin, loc, wid) in enumerate(PROFILES):
        out["prof%d__args" % i] = np.array([nbin, loc, wid], dtype=float)
        out["prof%d__out" % i] = pplib.gaussian_profile(nbin, loc, wid)
    # read_model with a TAU line (TAU [s] -> [bin] via P, pplib.py:3050-3055)
    with tempfile.NamedTemporaryFile("w", suffix=".gmodel", delete=False) as fh:
        fh.write(GMODEL_TAU)
        gpath = fh.name
    nbin, P = 1024, mg.P0
    freqs = mg.channel_freqs(24, 1100.0, 800.0)
    with contextlib.redirect_stdout(io.StringIO()):
        _, ngauss, model = pplib.read_model(gpath, pplib.get_bin_centers(nbin),
                                            freqs, P, quiet=True)
    os.unlink(gpath)
    out["readmodel__text"] = np.array(GMODEL_TAU)
    out["readmodel__freqs"] = freqs
    out["readmodel__P"] = np.float64(P)
    out["readmodel__out"] = model
    out["cases"] = np.array(sorted(CASES))
    out["nprof"] = np.int64(len(PROFILES))
    path = os.path.join(HERE, "gauss.npz")
    np.savez_compressed(path, **out)
    print("wrote %s (%d cases, %d profiles)" % (path, len(CASES), len(PROFILES)))


if __name__ == "__main__":
    main()

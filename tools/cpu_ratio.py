#!/usr/bin/env python
"""Measure, in THIS container, the single-core speed ratio of the reference's
GetTOAs loop to the oracle restatement on identical inputs (the configs[1]
sub-int shape, 512 x 2048, phase + DM), so bench.py can report its CPU
baseline (the oracle, timed on the GPU box's host) also as a
reference-equivalent rate (SURVEY.md 8(d) "report it both ways").

Writes profiles/cpu_ratio.json.  Needs /root/reference (never on the GPU
box); bench.py only reads the JSON.

Usage: python tools/cpu_ratio.py [nsub]
"""
import contextlib
import io
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
os.environ.setdefault("OMP_NUM_THREADS", "1")
from threadpoolctl import threadpool_limits  # noqa: E402
import numpy as np  # noqa: E402


def main():
    import make_golden_full as MGF
    import oracle as O
    from full_inputs import TOAS
    c = dict([t for t in TOAS if t["name"] == "c2"][0])
    c["nsub"] = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    with threadpool_limits(1):
        t0 = time.perf_counter()
        out = MGF.run_toas(c)           # reference get_TOAs (timed inside)
        ref_s = float(out["ref_seconds"])
        files, freqs = MGF.toa_inputs(c)
        fi = files[0]
        nsub = c["nsub"]
        t0 = time.perf_counter()
        O.get_toas_archive(fi["subints"], MGF.S.template(512, 2048)[0],
                           np.tile(freqs, (nsub, 1)), fi["weights"],
                           out["f0_snrs"], np.full(nsub, MGF.S.P0), MGF.S.DM0,
                           fi["dfs"], noise_stds=out["f0_noise"])
        orc_s = time.perf_counter() - t0
        # the scattering fits (bench --fit full / scat): the reference's
        # fit_portrait_full against the oracle's on the C3 golden inputs
        from full_inputs import FITS
        scat = {}
        for mode, name in (("full", "c3_all_512x2048_a"),
                           ("scat", "c3_pdta_512x2048")):
            fc = [f for f in FITS if f["name"] == name][0]
            r = MGF.run_fit(fc)
            data, model, freqs, P, _, init, nu_fit = MGF.fit_inputs(fc)
            t0 = time.perf_counter()
            O.fit_portrait_full(data.astype(np.float64), model, list(init), P,
                                freqs, [nu_fit] * 3, [None] * 3, r["errs"],
                                list(fc["flags"]), log10_tau=True)
            o_s = time.perf_counter() - t0
            scat[mode] = dict(case=name, flags=list(fc["flags"]),
                              reference_s_per_fit=float(r["ref_seconds"]),
                              oracle_s_per_fit=o_s,
                              reference_over_oracle_time=float(
                                  r["ref_seconds"]) / o_s)
    res = dict(shape="512x2048 phase+DM GetTOAs loop", nsub=nsub,
               reference_s_per_fit=ref_s / nsub,
               oracle_s_per_fit=orc_s / nsub,
               reference_over_oracle_time=ref_s / orc_s,
               cpu=platform.processor() or platform.machine(),
               threads=1, numpy=np.__version__,
               note="measured in the build container (the reference never "
                    "travels to the GPU box); bench.py divides the oracle's "
                    "rate on the GPU box host by this ratio",
               scattering_fits=scat)
    path = os.path.join(ROOT, "profiles", "cpu_ratio.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    with contextlib.redirect_stderr(io.StringIO()):
        main()

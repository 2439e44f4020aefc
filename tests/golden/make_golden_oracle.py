#!/usr/bin/env python
"""Oracle-produced golden vectors for shapes the REFERENCE cannot run.

configs[4] (16384 channels x 1024 bins): the reference's covariance step
allocates a (5+nchan)^2 nchan float64 cube (pptoaslib.py:731; 3.5e13 B at
16384 channels), so these fits are produced by the oracle restatement
(oracle/ppfit_oracle.py: same objective, derivatives, SciPy trust-ncg and
zero-covariance algebra, O(nchan) Schur-complement covariance), which is
itself pinned to the reference's golden vectors at <= 512 channels
(tests/test_oracle_golden.py).  Inputs are rebuilt by full_inputs.c5_inputs
and checked by SHA-256 in the tests.  About two minutes per fit here.

Usage:  python tests/golden/make_golden_oracle.py
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
import synth_np as S  # noqa: E402
from full_inputs import C5, c5_inputs  # noqa: E402


def main():
    store = {}
    for c in C5:
        data, model, freqs, P, truth, init, nu_fit = c5_inputs(c)
        t0 = time.time()
        r = O.fit_portrait_full(data, model, init, P, freqs, [nu_fit] * 3,
                                [None] * 3, None, c["flags"], log10_tau=True)
        dt = time.time() - t0
        key = "c5_" + c["name"]
        store[key + "/sha"] = np.array(S.sha(data.astype(np.float32),
                                             model.astype(np.float32)))
        store[key + "/init"] = np.array(init, dtype=float)
        store[key + "/nu_fit"] = np.float64(nu_fit)
        store[key + "/truth"] = truth
        store[key + "/oracle_seconds"] = np.float64(dt)
        for k in ("params", "param_errs", "nu_DM", "nu_GM", "nu_tau",
                  "red_chi2", "chi2", "snr", "scales", "scale_errs",
                  "channel_snrs", "covariance_matrix", "nfeval"):
            store[key + "/out_" + k] = np.asarray(r[k], dtype=np.float64)
        print(key, "%.1f s" % dt, r["params"], flush=True)
    np.savez_compressed(os.path.join(HERE, "oracle_c5.npz"), **store)


if __name__ == "__main__":
    main()

"""GPU probe of the any-nbin paths, one step per line (flushed), so that a
fault names the step that caused it: block-FFT noise and rotate at nbin with
large prime factors, then the wave mixed-radix fit at 1000 and 1022 bins.
usage: python tools/nbin_probe.py [step ...]   (steps: noise rotate fit1000
fit1022 fit2006)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def say(*a):
    print(time.strftime("%H:%M:%S"), *a, flush=True)


def main(steps):
    from pulseportraiture_amd import pplib as ppl
    from pulseportraiture_amd import pptoaslib
    import fullshape as F
    for st in steps:
        say("start", st)
        if st == "noise":
            for nb in (1002, 1022, 4094):
                x = np.random.default_rng(nb).normal(size=(2, nb))
                say(" noise", nb, ppl.get_noise(x, chans=True))
        elif st == "rotate":
            for nb in (1000, 1022, 2006):
                x = np.random.default_rng(nb).normal(size=(3, nb))
                say(" rotate", nb, float(np.abs(ppl.rotate_data(x, 0.27)).sum()))
        elif st.startswith("fit"):
            name = {"fit1000": "pd_128x1000", "fit1022": "pd_128x1022",
                    "fit2006": "pdta_64x2006"}[st]
            c, data, model, freqs = F.fit_case(name)
            lt = bool(c["log10_tau"])
            nu_fit = float(c["nu_fit"])
            r = pptoaslib.fit_portrait_full(data, model, list(c["init"]),
                                            float(c["P"]), freqs, [nu_fit] * 3,
                                            [None] * 3, c["errs"],
                                            [int(v) for v in c["flags"]],
                                            log10_tau=lt)
            say(" fit", name, r.params, r.red_chi2)
        say("done", st)


if __name__ == "__main__":
    main(sys.argv[1:] or ["noise", "rotate", "fit1000", "fit1022", "fit2006"])

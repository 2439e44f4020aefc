"""Diagnostic: ppalign's batched fit (fit_batch with the k_guess guess at
Ns = nbin, guess_ref = 1) vs the oracle's guess and fit, per archive."""
import sys
sys.path[:0] = ['.', 'tests']
import numpy as np
import fullshape as F
from oracle import ppfit_oracle as O
from pulseportraiture_amd import engine, _lib

I = _lib.RESULT_INDEX
for nbin in [int(x) for x in sys.argv[1:]]:
    archives, model_data = F.align_synthetic(8, nbin, 1, 2, 71)
    model_port = (model_data.masks * model_data.subints)[0, 0]
    for f, data in enumerate(archives):
        ichans = data.ok_ichans[0]
        port = data.subints[0, 0, ichans]
        freqs = data.freqs[0, ichans]
        P = data.Ps[0]
        errs = data.noise_stds[0, 0, ichans]
        DMg = data.DM
        w = data.weights[0, ichans]
        nu_fit = O.guess_fit_freq(freqs, data.SNRs[0, 0, ichans])
        rot = O.rotate_data(port, 0.0, DMg, P, freqs, nu_fit)
        prof = np.average(rot, axis=0, weights=w)
        po = O.fit_phase_shift(prof, model_port[ichans].mean(axis=0), Ns=nbin)
        ro = O.fit_portrait_full(port, model_port[ichans], [po["phase"], DMg, 0, 0, 0], P, freqs,
                                 [nu_fit] * 3, [None] * 3, errs, [1, 1, 0, 0, 0], log10_tau=False)
        res = engine.results_numpy(engine.fit_batch(
            port[None], model_port[ichans], freqs[None], np.array([P]),
            np.array([[0.0, DMg, 0, 0, 0]]), [1, 1, 0, 0, 0],
            nu_fits=np.full((1, 3), nu_fit), nu_outs=np.full((1, 3), np.nan),
            errs=errs[None], log10_tau=False, is_toa=True, guess=True,
            guess_weights=w[None], guess_DM=np.array([DMg]), guess_Ns=nbin,
            guess_ref=1, n_x=0))
        r = res["results"][0]
        print("nbin %d arch %d: guess oracle %.12f dev %.12f" % (nbin, f, po["phase"], r[I["phi_guess"]]))
        print("   oracle phi %.12f DM %.12f scale0 %.9e" % (ro["phi"], ro["DM"], ro["scales"][0]))
        print("   dev    phi %.12f DM %.12f scale0 %.9e" % (r[I["params"]][0], r[I["params"]][1],
                                                         res["scales"][0][0]), flush=True)

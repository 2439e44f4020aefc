"""Diagnostic: the pieces of one ppalign sub-int (guess FFTFIT, portrait
fit) on the device vs the oracle at several nbin."""
import sys
sys.path[:0] = ['.', 'tests']
import numpy as np
import fullshape as F
from oracle import ppfit_oracle as O
from pulseportraiture_amd import pplib, pptoaslib

for nbin in [int(x) for x in sys.argv[1:]]:
    archives, model_data = F.align_synthetic(8, nbin, 1, 2, 71)
    data = archives[0]
    model_port = (model_data.masks * model_data.subints)[0, 0]
    ichans = data.ok_ichans[0]
    port = data.subints[0, 0, ichans]
    freqs = data.freqs[0, ichans]
    P = data.Ps[0]
    errs = data.noise_stds[0, 0, ichans]
    DMg = data.DM
    nu_fit = O.guess_fit_freq(freqs, data.SNRs[0, 0, ichans])
    rot = O.rotate_data(port, 0.0, DMg, P, freqs, nu_fit)
    prof = np.average(rot, axis=0, weights=data.weights[0, ichans])
    mm = model_port[ichans].mean(axis=0)
    po = O.fit_phase_shift(prof, mm, Ns=nbin)
    pd = pplib.fit_phase_shift(prof, mm, Ns=nbin)
    print("nbin %d guess: oracle %.12f dev %.12f  err %.3e" % (nbin, po["phase"], pd.phase, po["phase_err"]), flush=True)
    for pg in (po["phase"], pd.phase):
        ro = O.fit_portrait_full(port, model_port[ichans], [pg, DMg, 0, 0, 0], P, freqs, [nu_fit] * 3,
                                 [None] * 3, errs, [1, 1, 0, 0, 0], log10_tau=False)
        rd = pptoaslib.fit_portrait_full(port, model_port[ichans], [pg, DMg, 0, 0, 0], P, freqs, [nu_fit] * 3,
                                         [None] * 3, errs, [1, 1, 0, 0, 0], log10_tau=False)
        print("   fit from %.9f: oracle phi %.12f DM %.12f chi2 %.9e | dev phi %.12f DM %.12f chi2 %.9e" % (
            pg, ro["phi"], ro["DM"], ro.get("chi2", np.nan), rd.phi, rd.DM, getattr(rd, "chi2", np.nan)), flush=True)

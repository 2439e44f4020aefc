"""Debug: ppalign duplicate-channel path, first iteration, device vs oracle
per-row fits."""
import os, sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"]
import numpy as np
import fullshape as F
import oracle as O
from pulseportraiture_amd import ppalign, engine
c, archives, model_data = F.align_case("dup")
dev = engine.device()
R = ppalign._Rows(archives, model_data, 1, dev)
model_port = (model_data.masks * model_data.subints)[0, 0]
ph, w = ppalign._fit_and_weights(R, model_port, True, int(c["nbin"]), dev)
ph, w = ph.cpu().numpy(), w.cpu().numpy()
nbin = int(c["nbin"])
row = 0
for data in archives:
    for isub in data.ok_isubs:
        ichans = data.ok_ichans[isub]
        mok = model_data.ok_ichans[0]
        mch = np.array([mok[np.argmin(abs(model_data.freqs[0][mok] - data.freqs[isub, ic]))] for ic in ichans])
        port = data.subints[isub, 0, ichans]
        freqs = data.freqs[isub, ichans]
        model = model_port[mch]
        P = data.Ps[isub]
        errs = data.noise_stds[isub, 0, ichans]
        nu_fit = O.guess_fit_freq(freqs, data.SNRs[isub, 0, ichans])
        rot = O.rotate_data(port, 0.0, data.DM, P, freqs, nu_fit)
        pg = O.fit_phase_shift(np.average(rot, axis=0, weights=data.weights[isub, ichans]), model.mean(axis=0), Ns=nbin)["phase"]
        r = O.fit_portrait_full(port, model, [pg, data.DM, 0, 0, 0], P, freqs, [nu_fit]*3, [None]*3, errs, [1,1,0,0,0], log10_tau=False)
        last = {}
        for i, m in enumerate(mch): last[int(m)] = i
        for m, i in sorted(last.items()):
            phr = r["phi"] + O.DCONST * r["DM"] / P * (freqs[i] ** -2 - r["nu_DM"] ** -2)
            wr = r["scales"][i] / errs[i] ** 2
            print(row, m, i, "dphase %.3e" % (((ph[row, m] - phr + 0.5) % 1) - 0.5), "w %.6g %.6g" % (w[row, m], wr))
            break
        print(row, "pg", pg, "phi", r["phi"], "DM", r["DM"], "nu", r["nu_DM"])
        row += 1

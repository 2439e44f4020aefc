"""Host-side cost of one GetTOAs-sized ppf_fit_batch call (GPU box): 64
sub-ints x 512 ch x 2048 bins resident on the device, the per-sub-int inputs
as host arrays (as GetTOAs passes them), timed per call with and without the
library's stage events, plus the pieces of engine.fit_batch.
    python tools/fitcall_probe.py [nsub]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pulseportraiture_amd import _lib, engine, synth
    from pulseportraiture_amd.pplib import guess_fit_freq
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = engine.device()
    b = synth.make_batch(n, 512, 2048, dev=dev)
    model = torch.as_tensor(b["model"], dtype=torch.float64, device=dev)[None]
    freqs = np.tile(b["freqs"], (n, 1))
    P = np.asarray(b["P"], dtype=float)
    init = np.zeros((n, 5))
    init[:, 1] = synth.DM0
    flags = np.tile(np.array([1, 1, 0, 0, 0], np.int32), (n, 1))
    nu = guess_fit_freq(b["freqs"])
    nu_fits = np.full((n, 3), nu)
    nu_outs = np.full((n, 3), np.nan)
    errs = engine.noise_rows(b["data"]).cpu().numpy()
    mask = np.ones((n, 512), np.uint8)
    mi = np.zeros(n, np.int32)
    gw = np.ones((n, 512))
    gdm = np.full(n, synth.DM0)
    ws = None

    def call():
        nonlocal ws
        r = engine.fit_batch(b["data"], model, freqs, P, init, flags,
                             nu_fits=nu_fits, nu_outs=nu_outs, errs=errs,
                             chan_mask=mask, model_index=mi, is_toa=True,
                             guess=True, guess_weights=gw, guess_DM=gdm,
                             guess_Ns=100, dev=dev, workspace=ws,
                             max_workspace=1 << 36)
        ws = r["workspace"]
        return r
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    for prof in (0, 1):
        lib = _lib.load()
        lib.ppf_set_profiling(_lib.context(dev.index), prof)
        ts, tl = [], []
        for _ in range(20):
            t0 = time.perf_counter()
            r = call()
            t1 = time.perf_counter()
            r["results"].cpu()
            t2 = time.perf_counter()
            ts.append(t1 - t0)
            tl.append(t2 - t0)
        print("profiling=%d: fit_batch returns after %.3f ms (median), "
              "results on the host after %.3f ms" % (
                  prof, 1e3 * np.median(ts), 1e3 * np.median(tl)), flush=True)
        if prof:
            ctx = _lib.context(dev.index)
            h = np.zeros((20, 4))
            got = lib.ppf_stage_ms_history(ctx, 20, h.ctypes.data)
            print("  device stages (model_rfft, xspec, guess, solve) ms:",
                  np.round(np.median(h[:got], axis=0), 3), flush=True)
            p = np.zeros((20, 2))
            got = lib.ppf_pass_ms_history(ctx, 20, p.ctypes.data)
            print("  solver passes per call:", np.median(p[:got, 1]),
                  "pass ms", np.round(np.median(p[:got, 0]), 3), flush=True)
    # pieces of the host path
    t0 = time.perf_counter()
    for _ in range(20):
        engine._stage_host([(freqs, torch.float64), (P, torch.float64),
                            (init, torch.float64), (flags, torch.int32),
                            (nu_fits, torch.float64), (nu_outs, torch.float64),
                            (errs, torch.float64), (mask, torch.uint8),
                            (mi, torch.int32), (gw, torch.float64),
                            (gdm, torch.float64)], dev)
    torch.cuda.synchronize()
    print("_stage_host: %.3f ms" % (1e3 * (time.perf_counter() - t0) / 20))


if __name__ == "__main__":
    main()

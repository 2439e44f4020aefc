"""Time k_gauss_port (ppf_gauss_portrait_batch): nport example.gmodel
portraits of nchan x nbin on cuda:0, with and without scattering.
usage: python tools/gauss_bench.py [nport nchan nbin]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pulseportraiture_amd import engine, synth  # noqa: E402


def main():
    nport, nchan, nbin = (int(v) for v in (sys.argv[1:4] or (64, 512, 2048)))
    dev = torch.device("cuda", 0)
    params = np.asarray(synth.GMODEL_PARAMS, dtype=float)
    freqs = np.stack([synth.channel_freqs(nchan)] * nport)
    for tau in (0.0, 3.0):
        p = np.tile(params, (nport, 1))
        p[:, 1] = tau
        pt = torch.as_tensor(p, device=dev)
        ft = torch.as_tensor(freqs, device=dev)
        args = (synth.GMODEL_CODE, pt, [synth.GMODEL_ALPHA] * nport, ft,
                [synth.GMODEL_NU_REF] * nport, nbin)
        engine.gauss_portraits(*args, dev=dev)
        torch.cuda.synchronize(dev)
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            out = engine.gauss_portraits(*args, dev=dev)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        rows = nport * nchan
        print("k_gauss_port tau=%g: %d x %d x %d in %.3f ms: %.1f Mrows/s, "
              "%.1f GB/s written" % (tau, nport, nchan, nbin, dt * 1e3,
                                     rows / dt / 1e6,
                                     out.numel() * 8 / dt / 1e9), flush=True)


if __name__ == "__main__":
    main()

"""Where the PSRFITS fast path spends its time (GPU box): writes a few
configs[1]-shape 16-bit archives, times load_data's stages on one of them,
then profiles GetTOAs.get_TOAs over all of them with cProfile.
    python tools/psrfits_prof.py [narchives]"""
import cProfile
import os
import pstats
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pulseportraiture_amd import engine, pptoas, psrfits, synth
    na = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = engine.device()
    tmp = tempfile.mkdtemp()
    names = []
    for f in range(na):
        b = synth.make_batch(64, 512, 2048, first=f * 64, dev=dev)
        names.append(bench._write_psrfits(os.path.join(tmp, "a%02d.fits" % f),
                                          b, f, 64))
        del b
    torch.cuda.synchronize()
    fn = names[0]
    for rep in range(3):
        t = [time.perf_counter()]
        pf = psrfits.PSRFITS(fn)
        t.append(time.perf_counter())
        raw, edt = pf.data_bytes()
        scl, offs = pf.scales_offsets()
        w = pf.weights()
        t.append(time.perf_counter())
        nbytes = 512 * 2048 * 2
        host = torch.empty((64, nbytes), dtype=torch.uint8, pin_memory=True)
        t.append(time.perf_counter())
        host.copy_(torch.from_numpy(raw[:, :nbytes]))
        t.append(time.perf_counter())
        d = host.to(dev)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        out = engine.unpack_psrfits(d, 0, 1, 512, 2048, scl, offs,
                                    wts=w.astype(np.float32))
        nz = engine.noise_rows(out["rows"])
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        data = psrfits.load_data(fn, pscrunch=True, rm_baseline=False,
                                 quiet=True)
        t.append(time.perf_counter())
        print("open %.2f  columns %.2f  pin-alloc %.2f  pinned copy %.2f  H2D "
              "%.2f  unpack+noise %.2f  load_data %.2f ms" % tuple(
                  1e3 * (t[i + 1] - t[i]) for i in range(len(t) - 1)),
              flush=True)
        pf.close()
    gm = synth.write_gmodel(os.path.join(tmp, "t.gmodel"))
    meta = os.path.join(tmp, "meta.txt")
    with open(meta, "w") as fh:
        fh.write("".join(n + "\n" for n in names))
    gt = pptoas.GetTOAs(meta, gm, quiet=True)
    gt.get_TOAs(quiet=True)
    t0 = time.perf_counter()
    pr = cProfile.Profile()
    pr.enable()
    gt = pptoas.GetTOAs(meta, gm, quiet=True)
    gt.get_TOAs(quiet=True)
    pr.disable()
    dt = time.perf_counter() - t0
    print("get_TOAs over %d archives: %.1f ms (%.0f TOAs/s)" %
          (na, dt * 1e3, na * 64 / dt))
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()

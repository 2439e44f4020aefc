"""Bounds of the PSRFITS fast path on the GPU box: the positioned DATA read
into a page-locked buffer (psrfits.PSRFITS.read_data_into) at several reader
thread counts, the pinned host-to-device upload of one archive (one copy and
16-MiB chunks), and both at once (read of archive i+1 beside the upload of
archive i), each as GB/s of DATA bytes.
    python tools/psrfits_bw.py [reps]"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pulseportraiture_amd import engine, psrfits, synth
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = engine.device()
    tmp = tempfile.mkdtemp()
    names = []
    for f in range(2):
        b = synth.make_batch(64, 512, 2048, first=f * 64, dev=dev)
        names.append(bench._write_psrfits(os.path.join(tmp, "a%d.fits" % f),
                                          b, f, 64))
        del b
    torch.cuda.synchronize()
    nbytes = 512 * 2048 * 2
    tot = 64 * nbytes
    pins = [torch.empty((64, nbytes), dtype=torch.uint8, pin_memory=True)
            for _ in range(2)]
    dbuf = torch.empty((64, nbytes), dtype=torch.uint8, device=dev)
    files = [psrfits.PSRFITS(n) for n in names]

    def gbs(dt):
        return tot / dt / 1e9

    for nt in (1, 2, 4, 8, 12, 16):
        psrfits._READ_THREADS = nt
        ts = []
        for r in range(reps):
            t0 = time.perf_counter()
            files[r % 2].read_data_into(nbytes, pins[r % 2].numpy())
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print("read  %2d threads: median %.2f ms = %.1f GB/s (best %.1f)" % (
            nt, 1e3 * ts[len(ts) // 2], gbs(ts[len(ts) // 2]), gbs(ts[0])),
            flush=True)
    psrfits._READ_THREADS = 8
    st = torch.cuda.Stream(dev)
    for chunk in (0, 16, 4):
        ts = []
        for r in range(reps):
            with torch.cuda.stream(st):
                e0, e1 = torch.cuda.Event(enable_timing=True), \
                    torch.cuda.Event(enable_timing=True)
                e0.record(st)
                if chunk:
                    step = max(1, (chunk << 20) // nbytes)
                    for r0 in range(0, 64, step):
                        dbuf[r0:r0 + step].copy_(pins[0][r0:r0 + step],
                                                 non_blocking=True)
                else:
                    dbuf.copy_(pins[0], non_blocking=True)
                e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        ts.sort()
        print("H2D chunk %2d MiB: median %.2f ms = %.1f GB/s" % (
            chunk, 1e3 * ts[len(ts) // 2], gbs(ts[len(ts) // 2])), flush=True)
    # both at once: upload slot 0 while reading file 1 into slot 1
    for nt in (4, 8, 16):
        psrfits._READ_THREADS = nt
        tr, tu, tw = [], [], []
        for r in range(reps):
            torch.cuda.synchronize()
            w0 = time.perf_counter()
            with torch.cuda.stream(st):
                e0, e1 = torch.cuda.Event(enable_timing=True), \
                    torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for r0 in range(0, 64, 8):
                    dbuf[r0:r0 + 8].copy_(pins[0][r0:r0 + 8],
                                          non_blocking=True)
                e1.record(st)
            t0 = time.perf_counter()
            files[1].read_data_into(nbytes, pins[1].numpy())
            tr.append(time.perf_counter() - t0)
            e1.synchronize()
            tu.append(e0.elapsed_time(e1) * 1e-3)
            tw.append(time.perf_counter() - w0)
        m = lambda v: sorted(v)[len(v) // 2]
        print("read %2d threads beside the upload: read %.2f ms (%.1f GB/s), "
              "upload %.2f ms (%.1f GB/s), both %.2f ms" % (
                  nt, 1e3 * m(tr), gbs(m(tr)), 1e3 * m(tu), gbs(m(tu)),
                  1e3 * m(tw)), flush=True)
    for f in files:
        f.close()


if __name__ == "__main__":
    main()

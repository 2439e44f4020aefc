"""Host staging bandwidth on the GPU box (GetTOAs from in-memory float32
archives, pptoas._Stager): a 268 MB archive (64 x 512 x 2048 float32) copied
from pageable numpy memory into a page-locked buffer by torch's copy_ and by
the native ppf_host_copy at several thread counts, the pinned upload alone,
and copy + upload of the other buffer at once (the pipeline's steady state).
    python tools/host_copy_bw.py"""
import ctypes
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from pulseportraiture_amd import _lib
    lib = _lib.load()
    n = 64 * 512 * 2048
    src = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    nb = src.nbytes
    pins = [torch.empty(nb, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    dev = torch.device("cuda:0")
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)

    def best(fn, reps=7):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2]

    def torch_copy():
        pins[0][:nb].view(torch.float32).copy_(torch.from_numpy(src))

    def native(nt):
        return lambda: lib.ppf_host_copy(ctypes.c_void_p(pins[0].data_ptr()),
                                         src.ctypes.data, nb, nt)

    def upload():
        with torch.cuda.stream(st):
            d.copy_(pins[1], non_blocking=True)
        st.synchronize()

    print("torch threads %d" % torch.get_num_threads(), flush=True)
    t = best(torch_copy)
    print("torch copy_          %6.2f ms  %5.1f GB/s" % (t * 1e3, nb / t / 1e9), flush=True)
    for nt in (1, 4, 8, 16, 32):
        t = best(native(nt))
        print("ppf_host_copy x%-2d     %6.2f ms  %5.1f GB/s" % (nt, t * 1e3, nb / t / 1e9),
              flush=True)
    t = best(upload)
    print("pinned upload        %6.2f ms  %5.1f GB/s" % (t * 1e3, nb / t / 1e9), flush=True)
    for name, fn in (("torch", torch_copy), ("native x8", native(8)),
                     ("native x16", native(16))):
        def both():
            th = threading.Thread(target=upload)
            th.start()
            fn()
            th.join()
        t = best(both)
        print("copy (%s) + upload at once %6.2f ms  %5.1f GB/s each" % (
            name, t * 1e3, nb / t / 1e9), flush=True)


if __name__ == "__main__":
    main()

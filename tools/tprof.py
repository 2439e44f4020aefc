"""Section cycle profile of k_tr_mom from a PPF_TM_PROF build (thread 0 of
every workgroup, shader-clock cycles summed over workgroups):
    tools/build_variant.sh tprof -DPPF_TM_PROF=1
    PPFIT_LIB=varlib/libppfit_tprof.so python tools/tprof.py [bench args]
(default bench args: the C4 ppalign shape, one step)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (the HIP runtime comes up through torch first)
    from pulseportraiture_amd import _lib
    _lib.load()
    dll = ctypes.CDLL(os.environ["PPFIT_LIB"])
    get = dll.ppf_debug_tprof
    get.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = np.zeros(8, dtype=np.uint64)
    args = sys.argv[1:] or ["--fit", "align", "--nsub", "1000", "--nchan", "256",
                            "--nbin", "1024", "--steps", "1", "--warmup", "1",
                            "--cpu-sample", "0"]
    sys.argv = ["bench.py"] + args
    import bench
    get(out.ctypes.data, 1)
    bench.main()
    get(out.ctypes.data, 1)
    names = ["state in", "radius check", "evaluation pass", "block sum",
             "TR update (t0)", "barrier", "state out", "-"]
    tot = float(out[:7].sum())
    for i, nm in enumerate(names[:7]):
        print("%-16s %14d  %5.1f%%" % (nm, out[i], 100.0 * out[i] / tot))


if __name__ == "__main__":
    main()

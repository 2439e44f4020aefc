"""Section cycle profile of k_xmom_g from a PPF_XM_PROF build:
PPFIT_LIB=varlib/libppfit_xprof.so python tools/xprof.py (tools/build_variant.sh xprof -DPPF_XM_PROF=1)
Runs bench.py's workload for one 2500-sub-int chunk (after a warmup call) and
prints the cycles per section summed over all waves (shader clock)."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pulseportraiture_amd import _lib
    lib = _lib.load()
    dll = ctypes.CDLL(os.environ["PPFIT_LIB"])
    get = dll.ppf_debug_xprof
    get.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = np.zeros(8, dtype=np.uint64)
    # BENCH_ARGS: another workload (e.g. C4: "--fit align --nsub 1000
    # --nchan 256 --nbin 1024")
    extra = os.environ.get("BENCH_ARGS", "--nsub 2500").split()
    sys.argv = ["bench.py"] + extra + ["--steps", "1", "--warmup", "0", "--cpu-sample", "0"]
    import bench
    get(out.ctypes.data, 1)
    bench.main()
    get(out.ctypes.data, 1)
    names = os.environ.get("XP_NAMES", "load issue,fft,pair+noise,barrier1,mfma issue,epilogue,wait+convert,-").split(",")
    tot = float(out[:8].sum())
    for i, nm in enumerate(names):
        print("%-14s %14d  %5.1f%%" % (nm, out[i], 100.0 * out[i] / tot))


if __name__ == "__main__":
    main()

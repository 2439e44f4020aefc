#!/bin/bash
# Kernel traces of bench.py for library variants: tools/var_trace.sh lib1.so [lib2.so ...]
# -> gpurun_out/vt_<name>/ (kernel_trace.csv); summarise with tools/vt_show.py
export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename $lib .so)
  export PPFIT_LIB=$lib
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/vt_$name -o run --output-format csv -- python3 bench.py --nsub 2500 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/vt_$name.log 2>&1 || { echo "FAIL $lib"; exit 1; }
done

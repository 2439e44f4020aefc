#!/bin/bash
# rocprof kernel stats of bench.py under several library variants:
# tools/var_prof.sh TAG "<bench args>" lib1.so [lib2.so ...] -> gpurun_out/vp_TAG_<name>/
export TMPDIR=/tmp
tag=$1; args=$2; shift 2
for lib in "$@"; do
  name=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/vp_${tag}_$name -o run --output-format csv -- python3 bench.py $args --cpu-sample 0 > gpurun_out/vp_${tag}_$name.log 2>&1 || { echo "FAIL $lib"; exit 1; }
done

#!/bin/bash
# Kernel traces of bench.py under environment settings: tools/env_trace.sh name1 "VAR=1 VAR2=2" name2 "..."
# -> gpurun_out/vt_<name>/ ; summarise with tools/vt_show.py
export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  name=$1; envs=$2; shift 2
  ( for kv in $envs; do export "$kv"; done
    timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/vt_$name -o run --output-format csv -- python3 bench.py --nsub 2500 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/vt_$name.log 2>&1 ) || { echo "FAIL $name"; exit 1; }
done

#!/bin/bash
# Round-2 profiling: kernel stats + SQ counter passes over a short C2 bench.
# usage: tools/prof_r2.sh TAG [extra bench args]
set -e
tag=${1:-r2}; shift || true
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
args="--nsub 2500 --steps 1 --warmup 1 --passes 1 --cpu-sample 0 $@"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/ks -o ks --output-format csv -- python3 bench.py $args > $out/ks.log 2>&1
p1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
p2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for p in "$p1" "$p2" "$@PMC3"; do
  [ "$p" = "@PMC3" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p -d $out/p$i -o p$i --output-format csv -- python3 bench.py $args > $out/p$i.log 2>&1
done

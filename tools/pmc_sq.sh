#!/bin/bash
# SQ-counter passes over a short bench run (one rocprofv3 --pmc pass per set).
# usage: tools/pmc_sq.sh <outdir> [bench args...]
set -e
out=${1:-gpurun_out/pmc_sq}; shift || true
args=${@:---nsub 2500 --steps 1 --warmup 1 --cpu-sample 0}
export TMPDIR=/tmp
p1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
p2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
mkdir -p $out
i=0
for p in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $p -d $out/p$i -o p$i --output-format csv -- python3 bench.py $args > $out/p$i.log 2>&1
done

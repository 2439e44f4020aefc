#!/bin/bash
# Round-2 profiling: kernel stats + SQ counter passes over a short C2 bench.
# usage: tools/prof_r2.sh TAG [extra bench args]   (PPFIT_LIB selects a variant)
set -e
tag=${1:-r2}; shift || true
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
args="--nsub 2500 --steps 1 --warmup 1 --passes 1 --cpu-sample 0 $@"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/ks -o ks --output-format csv -- python3 bench.py $args > $out/ks.log 2>&1
i=0
while read -r p; do
  [ -z "$p" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p -d $out/p$i -o p$i --output-format csv -- python3 bench.py $args > $out/p$i.log 2>&1 || echo "pass $i failed: $p"
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_ACTIVE_INST_MISC SQ_INSTS_SALU
SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT
PASSES

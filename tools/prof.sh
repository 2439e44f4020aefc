#!/bin/bash
# Kernel stats + PMC passes (HBM bytes, SQ/f64 utilisation, L2 hit rate) of a
# short bench.py run.  usage: tools/prof.sh TAG [bench args]
# Output: gpurun_out/prof_TAG/{ks,fetch,write,sq1,sq2,tcc}; each pass its own
# rocprofv3 run (no trace domains beside --pmc), each under its own timeout.
set -e
tag=${1:-r2}; shift || true
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
args="--steps 1 --warmup 1 --cpu-sample 0 $@"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/ks -o ks --output-format csv -- python3 bench.py $args > $out/ks.log 2>&1
run() {
  name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $out/$name -o $name --output-format csv -- python3 bench.py $args > $out/$name.log 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD
run sq2 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
run tcc TCC_HIT_sum TCC_MISS_sum
echo prof_done

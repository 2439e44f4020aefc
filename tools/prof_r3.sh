#!/bin/bash
# Round-3 profiles: rocprofv3 kernel statistics of the C2, C3 and C5 bench
# commands, then FETCH_SIZE / WRITE_SIZE passes (each its own run, no trace
# domains beside --pmc) for C2 and C3.  usage: tools/prof_r3.sh TAG
set -e
tag=${1:-r3}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
c2="--steps 1 --warmup 1 --cpu-sample 0"
c3="--fit full --nsub 10000 --steps 1 --warmup 1 --cpu-sample 0"
c5="--fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 1 --warmup 1 --cpu-sample 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/ks_c2 -o ks --output-format csv -- python3 bench.py $c2 > $out/ks_c2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks_c3 -o ks --output-format csv -- python3 bench.py $c3 > $out/ks_c3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks_c5 -o ks --output-format csv -- python3 bench.py $c5 > $out/ks_c5.log 2>&1
for m in c2 c3 c5; do
  args=$c2; [ $m = c3 ] && args=$c3; [ $m = c5 ] && args=$c5
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch_$m -o fetch --output-format csv -- python3 bench.py $args > $out/fetch_$m.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $out/write_$m -o write --output-format csv -- python3 bench.py $args > $out/write_$m.log 2>&1
done

# SQ counters of the C3 command (k_xspec_w / k_pass issue and wait split)
p1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
p2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for p in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $p -d $out/sq${i}_c3 -o sq$i --output-format csv -- python3 bench.py $c3 > $out/sq${i}_c3.log 2>&1
done
echo sq_done

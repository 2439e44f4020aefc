#!/bin/bash
# Reduce the round-4 profiling runs (tools/prof_r4.sh TAG c2 c3 c5 c4, merged
# back into gpurun_out/) into the tracked summaries: kernel statistics per
# config, the PMC HBM-traffic summary and the SQ / fp64 summary bench.py reads,
# and the SQ issue/wait tables.   usage: profiles/collect_r4.sh TAG
tag=${1:-a}
cd "$(dirname "$0")/.."
for c in c2 c3 c5 c4; do
  d=gpurun_out/prof_r4${tag}_$c
  [ -d $d ] || continue
  ks=$(ls $d/ks/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$ks" ] && cp $ks profiles/r04/kernel_stats_${c}_${tag}.csv
  grep '^{' $d/ks.log | tail -1 > profiles/r04/bench_under_rocprof_${c}_${tag}.json
  python profiles/pmc_reduce.py $d > profiles/r04/pmc_${c}_${tag}.json || true
  python profiles/fp64_reduce.py $d > profiles/r04/fp64_${c}_${tag}.json || true
  python profiles/sq_reduce.py $d/sq1 $d/sq2 > profiles/r04/sq_${c}_${tag}.txt 2>&1 || true
done
ls profiles/r04

#!/bin/bash
# Reduce a round's profiling runs (tools/prof_round.sh TAG c2 c3 c5 c4 nb1000,
# merged back into gpurun_out/prof_TAG_CONFIG) into the tracked summaries:
# kernel statistics per config, the PMC HBM-traffic summary and the SQ / fp64
# summary bench.py reads, and the SQ issue/wait tables.
#   usage: profiles/collect.sh ROUND TAG      (e.g. profiles/collect.sh r05 r5a)
round=${1:-r05}; tag=${2:-a}
cd "$(dirname "$0")/.."
mkdir -p profiles/$round
for c in c2 c3 c5 c4 nb1000 nb1536 nb1023; do
  d=gpurun_out/prof_${tag}_$c
  [ -d $d ] || continue
  ks=$(ls $d/ks/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$ks" ] && cp $ks profiles/$round/kernel_stats_${c}_${tag}.csv
  grep '^{' $d/ks.log | tail -1 > profiles/$round/bench_under_rocprof_${c}_${tag}.json
  python profiles/pmc_reduce.py $d > profiles/$round/pmc_${c}_${tag}.json || true
  python profiles/fp64_reduce.py $d > profiles/$round/fp64_${c}_${tag}.json || true
  python profiles/sq_reduce.py $d/sq1 $d/sq2 > profiles/$round/sq_${c}_${tag}.txt 2>&1 || true
done
ls profiles/$round

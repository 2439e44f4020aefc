#!/bin/bash
# Evidence run: the GPU parity suite and smoke(), then every bench line with its
# CPU baseline and parity sample (C2 headline, single-call latency, C3 and C5
# with >= 5 timed steps, C4 ppalign, GetTOAs from 16-bit PSRFITS and from
# float32 archives, phase+DM at the mixed-radix nbin 1000 and 1536 and the
# odd nbin 1023).
# usage: [PART=a|b] tools/evid.sh TAG [tests|notests]
tag=${1:-a}
mode=${2:-tests}
export TMPDIR=/tmp
mkdir -p gpurun_out
st=gpurun_out/evid_${tag}_status.txt
if [ "$mode" = tests ] && [ "${PART:-ab}" != b ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/gpu_tests_$tag.log)" >> $st
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
run() {
  name=$1; lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > gpurun_out/bench_${name}_$tag.log 2>&1
  rc=$?
  echo "$name rc=$rc $(python tools/show.py gpurun_out/bench_${name}_$tag.log | head -1)" >> $st
  [ $rc -eq 0 ] || exit $rc
}
if [ "$mode" = tests ] && [ "${PART:-ab}" != b ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.txt 2>&1
  rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/smoke_$tag.txt)" >> $st
  [ $rc -eq 0 ] || exit $rc
fi
# PART=a: the parity suite, smoke and C2 / single / C3 / C5; PART=b: the
# rest (each part fits one gpurun call); unset: everything
if [ "${PART:-ab}" != b ]; then
run c2 300
run single 200 --fit single --cpu-sample 1
# C3 / C5: 16 / 4 one-core oracle sub-ints for the line's own parity
run c3 500 --fit full --nsub 10000 --steps 5 --warmup 1 --cpu-sample 192
run c5 600 --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 5 --warmup 1 --cpu-sample 192
fi
[ "${PART:-ab}" = a ] && { echo end >> $st; exit 0; }
# C4: 50 timed steps (a 5-step region of ~3-ms steps is host-jitter bound)
run c4 300 --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 50 --warmup 5
run gettoaspsrfits 300 --fit gettoas --psrfits --steps 4 --warmup 1 --timeline gpurun_out/gettoas_psrfits_timeline_$tag.json
run gettoas 300 --fit gettoas --steps 3 --warmup 1
run c2nb1000 300 --nbin 1000 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 8
run c2nb1536 300 --nbin 1536 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 8
run c2nb1023 300 --nbin 1023 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 8
echo end >> $st

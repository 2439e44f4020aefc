#!/bin/bash
# channel-subset Newton warm start (in-tree) vs every-channel evaluations
# (varlib nosub): scattering parity tests, C3 / C5 benches; then the PSRFITS
# fast-path stage profile.  usage: tools/ab_r3c.sh TAG
set -e
tag=${1:-a}
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_fullshape.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -m gpu -k "scat or full or c5 or branches or lowsnr" > gpurun_out/gpu_sub_$tag.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_sub_$tag.log; }
tail -1 gpurun_out/gpu_sub_$tag.log
$T 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 2 > gpurun_out/bench_c3_$tag.log 2>&1
$T 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 1 > gpurun_out/bench_c5_$tag.log 2>&1
PPFIT_LIB=varlib/libppfit_nosub.so $T 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3nosub_$tag.log 2>&1
PPFIT_LIB=varlib/libppfit_nosub.so $T 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5nosub_$tag.log 2>&1
for c in c3 c5 c3nosub c5nosub; do
  f=gpurun_out/bench_${c}_$tag.log
  echo "$c $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), d.get('mean_passes_per_fit'), d.get('mean_evals_per_fit'), d.get('bytes_per_fit'), (d.get('roofline') or {}).get('frac'), (k.get('pass') or {}).get('total_ms'), (d.get('parity') or {}).get('ok'))")"
done
$T 300 python tools/psrfits_prof.py 8 > gpurun_out/psrfits_prof_$tag.log 2>&1 || true
head -8 gpurun_out/psrfits_prof_$tag.log

#!/bin/bash
# Round-3 A/B on one box: scattering parity tests + C3 Newton vs scipy path;
# moment-path Newton (varlib nm) vs base on C2/C4 with its parity subset;
# k_xmom_g static priority (prio) on C2; direct-store k_xspec_w (xd, xd3) on
# C3/C5 with the scattering parity tests.  usage: tools/ab_r3.sh TAG
set -e
tag=${1:-a}
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_fullshape.py tests/test_psrfits.py -x -q --timeout 200 --timeout-method thread -m gpu -k "branches or full or scat or c5 or psrfits or unpack" > gpurun_out/gpu_scat_$tag.log 2>&1 || { tail -3 gpurun_out/gpu_scat_$tag.log; grep -E "^E  " gpurun_out/gpu_scat_$tag.log | head -20; }
tail -1 gpurun_out/gpu_scat_$tag.log
$T 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 2 > gpurun_out/bench_c3_$tag.log 2>&1
$T 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 --solver scipy > gpurun_out/bench_c3scipy_$tag.log 2>&1
for v in base nm; do
  PPFIT_LIB=varlib/libppfit_$v.so $T 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4${v}_$tag.log 2>&1
  PPFIT_LIB=varlib/libppfit_$v.so $T 300 python bench.py --cpu-sample 0 --steps 3 > gpurun_out/bench_c2${v}_$tag.log 2>&1
done
PPFIT_LIB=varlib/libppfit_prio.so $T 300 python bench.py --cpu-sample 0 --steps 3 > gpurun_out/bench_c2prio_$tag.log 2>&1
for v in base xd xd3; do
  PPFIT_LIB=varlib/libppfit_$v.so $T 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3${v}_$tag.log 2>&1
  PPFIT_LIB=varlib/libppfit_$v.so $T 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5${v}_$tag.log 2>&1
done
PPFIT_LIB=varlib/libppfit_xd.so $T 300 python -u -m pytest tests/test_gpu_fullshape.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -m gpu -k "scat or full or c5 or branches" > gpurun_out/gpu_xd_$tag.log 2>&1 || true
tail -1 gpurun_out/gpu_xd_$tag.log
PPFIT_LIB=varlib/libppfit_nm.so $T 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullshape.py -k "not branches" > gpurun_out/gpu_nm_$tag.log 2>&1 || true
tail -1 gpurun_out/gpu_nm_$tag.log
grep -E "^FAILED" gpurun_out/gpu_nm_$tag.log gpurun_out/gpu_xd_$tag.log | head -20 || true
for c in c3 c3scipy c4base c4nm c2base c2nm c2prio c3base c3xd c3xd3 c5base c5xd c5xd3; do
  f=gpurun_out/bench_${c}_$tag.log
  echo "$c $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), d.get('mean_passes_per_fit'), d.get('mean_evals_per_fit'), (d.get('roofline') or {}).get('frac'), (k.get('xspec') or {}).get('avg_launch_ms'), (k.get('pass') or {}).get('total_ms'), (d.get('parity') or {}).get('ok'))")"
done

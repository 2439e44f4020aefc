cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psrfits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g12_pytest.log 2>&1 || exit 1
for v in "base" "HSA_ENABLE_SDMA=0" "PPF_UPLOAD_CHUNK_MB=16" "PPF_LOAD_DEPTH=2"; do
  e=""; [ "$v" != base ] && e="$v"
  timeout -k 10 300 env $e python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g12_tl_${v%%=*}.json > gpurun_out/g12_gt_${v%%=*}.json 2> gpurun_out/g12_gt_${v%%=*}.err || exit 2
  echo "$v $(python tools/show.py gpurun_out/g12_gt_${v%%=*}.json)" >> gpurun_out/g12_status.txt
done
for c in c5 c4; do
  for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_dsum1.so; do
    v=$(basename $lib .so)
    if [ $c = c5 ]; then a="--fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 3 --warmup 1 --cpu-sample 0"; else a="--fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 5 --warmup 2 --cpu-sample 0"; fi
    PPFIT_LIB=$lib timeout -k 10 300 python bench.py $a > gpurun_out/g12_${c}_$v.json 2> gpurun_out/g12_${c}_$v.err || exit 3
    echo "$c $v $(python tools/show.py gpurun_out/g12_${c}_$v.json | head -1)" >> gpurun_out/g12_status.txt
  done
done
echo "end" >> gpurun_out/g12_status.txt

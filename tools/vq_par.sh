#!/bin/bash
# parity subset + C2 timing of every varlib/ build
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
for lib in varlib/*.so; do
  nm=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_fullshape.py::test_c2_bench_pipeline_matches_oracle \
    "tests/test_gpu_fullshape.py::test_fullshape_gettoas_matches_reference" \
    tests/test_gpu_parity.py::test_get_toas_matches_reference \
    tests/test_gpu_parity.py::test_batch_equals_single_and_is_deterministic \
    tests/test_gpu_parity.py::test_device_guess_matches_oracle_phase_shift \
    tests/test_gpu_parity.py::test_align_archives_matches_reference \
    tests/test_gpu_parity.py::test_fit_portrait_full_matches_reference \
    tests/test_gpu_parity.py::test_harmonic_cutoff_fits_match_oracle \
    tests/test_gpu_fullshape.py::test_fullshape_fit_matches_reference \
    tests/test_gpu_fullshape.py::test_fullshape_align_matches_reference \
    > gpurun_out/vp_${tag}_$nm.log 2>&1 || { echo "FAIL $nm"; tail -30 gpurun_out/vp_${tag}_$nm.log; exit 1; }
  echo "$nm tests: $(tail -1 gpurun_out/vp_${tag}_$nm.log)"
done
bash tools/vq.sh $tag
bash tools/vq_al.sh $tag

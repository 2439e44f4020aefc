cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "lane_trust_region or wideband_scattering" > gpurun_out/g35_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/g35_pytest.log; exit $rc

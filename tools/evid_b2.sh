# round 6 final: the align / guess parity tests on the final build, the
# evidence lines of part B, then the chirp-grid guess at nbin 512 / 2048
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "align or c4 or guess or phase_shift or gettoas" > gpurun_out/pre_b_tests_r6b.log 2>&1 || exit 1
PART=b bash tools/evid.sh r6b tests || exit 1
TESTK= bash tools/ab.sh czn "c4n512 c4n2048" "base lib:varlib/libppfit_nocz.so" 1

# round 6: k_pass harmonic batch (KB 4 spills 40 B at three waves per SIMD)
TESTK="c3_bench or c5" bash tools/ab.sh kb "c3 c5" "base lib:varlib/libppfit_kb2.so lib:varlib/libppfit_kb3.so lib:varlib/libppfit_kb2w4.so" 2

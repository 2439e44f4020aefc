# round 6: the C3 / C5 lines on the final build (k_pass KB = 3), with their
# oracle parity sub-ints
export TMPDIR=/tmp
mkdir -p gpurun_out; st=gpurun_out/evid_r6c_status.txt
timeout -k 10 500 python bench.py --fit full --nsub 10000 --steps 5 --warmup 1 --cpu-sample 192 > gpurun_out/bench_c3_r6c.log 2>&1
rc=$?; echo "c3 rc=$rc $(python tools/show.py gpurun_out/bench_c3_r6c.log 2>/dev/null | head -1)" >> $st
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 5 --warmup 1 --cpu-sample 192 > gpurun_out/bench_c5_r6c.log 2>&1
rc=$?; echo "c5 rc=$rc $(python tools/show.py gpurun_out/bench_c5_r6c.log 2>/dev/null | head -1)" >> $st
echo end >> $st

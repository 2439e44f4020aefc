cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/g10_trace -o gt -- python3 bench.py --fit gettoas --psrfits --steps 1 --warmup 1 > gpurun_out/g10_gt.json 2> gpurun_out/g10_gt.err
echo "end rc=$?" >> gpurun_out/g10_status.txt

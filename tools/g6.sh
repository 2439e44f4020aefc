cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/g6_prof -o gt -- python3 bench.py --fit gettoas --psrfits --steps 1 --warmup 1 > gpurun_out/g6_gt.json 2> gpurun_out/g6_gt.err
echo "end rc=$?" >> gpurun_out/g6_status.txt

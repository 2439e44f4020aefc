cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 240 python -u tools/psrfits_bw.py 8 > gpurun_out/g17_bw.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g17_tl.json > gpurun_out/g17_gt.json 2> gpurun_out/g17_gt.err || exit 3
echo end

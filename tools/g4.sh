cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --mom-x > gpurun_out/g4_c2_momx.json 2> gpurun_out/g4_c2_momx.err &&
timeout -k 10 300 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/g4_c4.json 2> gpurun_out/g4_c4.err &&
timeout -k 10 300 env PPF_MOM_X=1 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/g4_c4_momx.json 2> gpurun_out/g4_c4_momx.err &&
timeout -k 10 400 python bench.py --fit gettoas --psrfits --steps 2 --warmup 1 --timeline gpurun_out/g4_tl_psrfits.json > gpurun_out/g4_gt_psrfits.json 2> gpurun_out/g4_gt_psrfits.err &&
timeout -k 10 400 python bench.py --fit gettoas --steps 2 --warmup 1 --timeline gpurun_out/g4_tl_f32.json > gpurun_out/g4_gt_f32.json 2> gpurun_out/g4_gt_f32.err
echo "end rc=$?" >> gpurun_out/g4_status.txt

#!/bin/bash
# Does X stay in the MALL across passes when a call's cross spectrum fits in
# it?  C3 shape with 80 sub-ints (X ~180 MB) vs 2500: k_pass time and HBM
# bytes per evaluation.
set -e
export TMPDIR=/tmp
bash tools/prof.sh c3m80 --fit full --nsub 80 --steps 3 > /dev/null
python profiles/pmc_reduce.py gpurun_out/prof_c3m80 --out gpurun_out/pm_c3m80.json | python -c "import json,sys; d=json.load(sys.stdin); print({k:(round(v['hbm_bytes']), v['units']) for k,v in d['kernels'].items()})"
grep "k_pass" gpurun_out/prof_c3m80/ks/ks_kernel_stats.csv

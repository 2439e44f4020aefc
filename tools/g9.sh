cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python tools/fitcall_probe.py 64 > gpurun_out/g9_probe.log 2>&1
echo "end rc=$?" >> gpurun_out/g9_status.txt

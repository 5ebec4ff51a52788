set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/stamp.py forging-control_amd/lib/libfcr_stamp.so > gpurun_out/stamp.log 2>&1
cat gpurun_out/stamp.log | grep -v amdgpu.ids

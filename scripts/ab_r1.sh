set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python scripts/kbench.py forging-control_amd/lib/libfcr_v2.so forging-control_amd/lib/libfcr_s0.so forging-control_amd/lib/libfcr_s4.so forging-control_amd/lib/libfcr_s8.so forging-control_amd/lib/libfcr_s14.so forging-control_amd/lib/libfcr_s0p2.so --rounds 5 > gpurun_out/kbench.log 2>&1
cat gpurun_out/kbench.log | grep lib

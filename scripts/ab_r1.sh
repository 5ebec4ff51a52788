# GPU A/B: parity tests on the default build, then kernel timing of the variants in lib/
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
LIBS="forging-control_amd/lib/libfcr.so $(ls forging-control_amd/lib/libfcr_*.so)"
timeout -k 10 400 python scripts/kbench.py $LIBS --rounds 2 --sustain 40 > gpurun_out/kbench.log 2>&1
grep lib gpurun_out/kbench.log

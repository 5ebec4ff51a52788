# GPU A/B: parity suite on the default build, then interleaved kernel timing of libfcr.so against the
# other variants in lib/ (kbench, sustained back-to-back launches)
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
LIBS="forging-control_amd/lib/libfcr.so $(ls forging-control_amd/lib/libfcr_*.so)"
timeout -k 10 400 python scripts/kbench.py $LIBS --rounds 2 --sustain ${SUSTAIN:-30} > gpurun_out/kbench.log 2>&1
grep lib gpurun_out/kbench.log

# Captured-step tests (+ the surrogate/wide-path tests after the rocBLAS atomics change) and the
# eager-vs-graphed step timings, 1 GPU
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_graphed.py tests/test_surrogate.py > gpurun_out/graphed_tests.log 2>&1
tail -3 gpurun_out/graphed_tests.log
timeout -k 10 300 python -u scripts/bench_graphed.py > gpurun_out/graphed_bench.log 2>&1
cat gpurun_out/graphed_bench.log | grep workload

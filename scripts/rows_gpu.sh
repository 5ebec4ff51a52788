# GPU: parity tests of the §8(f) rows (plant, windows, inference) + their benchmark lines
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/rows
timeout -k 10 300 python -m pytest tests/test_plant.py tests/test_windows.py tests/test_gpu_inference.py -m gpu -x -q > gpurun_out/rows/pytest.log 2>&1 || { tail -30 gpurun_out/rows/pytest.log; exit 1; }
tail -2 gpurun_out/rows/pytest.log
timeout -k 10 200 python scripts/bench_windows.py > gpurun_out/rows/bench_windows.log 2>&1 || { tail -20 gpurun_out/rows/bench_windows.log; exit 1; }
tail -1 gpurun_out/rows/bench_windows.log

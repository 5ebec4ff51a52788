# Config 5 (H = 256, N = 25): wide-path parity tests, the benchmark line and its kernel statistics, 1 GPU
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-c5}
mkdir -p $R/gpurun_out/c5
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_surrogate.py tests/test_graphed.py > gpurun_out/c5/tests.log 2>&1
tail -2 gpurun_out/c5/tests.log
timeout -k 10 300 python bench.py --hidden 256 --horizon 25 --batch 65536 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5/bench_c5.log 2>&1
tail -1 gpurun_out/c5/bench_c5.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c5/prof -o $TAG -- python3 $R/bench.py --hidden 256 --horizon 25 --batch 65536 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/c5/prof.log 2>&1
echo done

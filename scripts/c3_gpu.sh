set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
timeout -k 10 300 python bench.py --precision f16 --batch 262144 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
timeout -k 10 300 python bench.py --batch 262144 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3_fp32.log 2>&1 || { tail -20 gpurun_out/bench_c3_fp32.log; exit 1; }
tail -1 gpurun_out/bench_c3_fp32.log

# SURVEY config 5 (H = 256, N = 25, B = 65536) and a smaller-batch point, 1 GPU
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --hidden 256 --horizon 25 --batch 65536 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1
tail -1 gpurun_out/bench_c5.log

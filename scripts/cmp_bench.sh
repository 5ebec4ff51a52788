set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/cmp_bench.log 2>&1
L=forging-control_amd/lib
timeout -k 10 300 python scripts/kbench.py $L/libfcr.so --rounds 1 --sustain 40 > gpurun_out/cmp_kbench.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/cmp_bench2.log 2>&1
grep -h -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' gpurun_out/cmp_bench.log gpurun_out/cmp_bench2.log
grep lib gpurun_out/cmp_kbench.log

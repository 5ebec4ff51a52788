# GPU: benchmark lines of the SURVEY §8(f) rows (plant, closed loop, windows, surrogate), one file each
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/rows
for b in plant closed_loop windows surrogate; do
  timeout -k 10 300 python scripts/bench_$b.py > gpurun_out/rows/bench_$b.log 2>&1 || { echo "bench_$b failed"; tail -20 gpurun_out/rows/bench_$b.log; exit 1; }
  echo "$b: $(grep -v amdgpu.ids gpurun_out/rows/bench_$b.log | tail -1 | cut -c1-300)"
done

set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r05}
cd $R
mkdir -p gpurun_out/sur
timeout -k 10 300 python -m pytest tests/test_surrogate.py -m gpu -x -q > gpurun_out/sur/pytest.log 2>&1 || { tail -30 gpurun_out/sur/pytest.log; exit 1; }
tail -1 gpurun_out/sur/pytest.log
timeout -k 10 300 python scripts/bench_surrogate.py > gpurun_out/sur/bench.log 2>&1 || { tail -20 gpurun_out/sur/bench.log; exit 1; }
cat gpurun_out/sur/bench.log | grep metric
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sur/trace -o $TAG -- python3 $R/scripts/bench_surrogate.py --B 256 65536 --steps 20 --cpu-budget 0.2 > $R/gpurun_out/sur/trace.log 2>&1
echo done

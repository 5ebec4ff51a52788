# GPU: plant parity tests, benchmark line, rocprofv3 kernel stats + PMC (VALU instructions, HBM bytes)
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r05}
cd $R
mkdir -p gpurun_out/plant
timeout -k 10 300 python -m pytest tests/test_plant.py -m gpu -x -q > gpurun_out/plant/pytest.log 2>&1 || { tail -30 gpurun_out/plant/pytest.log; exit 1; }
tail -2 gpurun_out/plant/pytest.log
timeout -k 10 300 python scripts/bench_plant.py > gpurun_out/plant/bench.log 2>&1 || { tail -20 gpurun_out/plant/bench.log; exit 1; }
tail -1 gpurun_out/plant/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/plant/trace -o $TAG -- python3 $R/scripts/bench_plant.py --cpu-budget 0.5 > $R/gpurun_out/plant/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $R/gpurun_out/plant/valu -o $TAG -- python3 $R/scripts/bench_plant.py --cpu-budget 0.5 --iters 2 > $R/gpurun_out/plant/valu.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 --output-format csv -d $R/gpurun_out/plant/f64 -o $TAG -- python3 $R/scripts/bench_plant.py --cpu-budget 0.5 --iters 2 > $R/gpurun_out/plant/f64.log 2>&1 || echo "f64 counters unavailable"
echo done

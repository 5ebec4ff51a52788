# GPU suite + default benchmark line (one gpurun call): scripts/gpu_check.sh TAG [pytest -k expr]
set -e -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-check}
K=${2:-}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rP -k "$K" > $OUT/pytest.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rP > $OUT/pytest.log 2>&1
fi
tail -3 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
tail -c 3000 $OUT/bench.log

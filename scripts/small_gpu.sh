# Small-batch kernels: their GPU tests, then config-1 bench lines (B = 15, 256, 4096) with both kernel families.
# usage: scripts/small_gpu.sh TAG -> gpurun_out/small_TAG/
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/small_${1:-x}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for b in 15 256 4096; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --grad-check off --batch $b --steps 50 --warmup 5 > $O/b$b.log 2>&1
  timeout -k 10 300 python3 bench.py --small-limit 0 --no-cpu-baseline --grad-check off --batch $b --steps 50 --warmup 5 > $O/b${b}_fused.log 2>&1
done
for f in $O/b*.log; do echo "== $f"; python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('value %.4g' % d['value'], '| ms %.3f' % d['ms_per_step'], '| kernels', d['kernels_ms'].get('fwd'), d['kernels_ms'].get('bwd'))
"; done

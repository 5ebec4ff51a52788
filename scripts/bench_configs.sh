# Benchmark lines of the BASELINE configs other than the default (one gpurun call):
# config 3 (B = 262 144) in its two precision modes, config 5 (N = 25, H = 256), config 1 batches (B = 15, 256:
# small-batch kernels eager and HIP-graph replayed, and the fused kernels at B = 15 for comparison).
# usage: scripts/bench_configs.sh TAG -> gpurun_out/cfg_TAG/*.log
set -e -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-round2}
O=$R/gpurun_out/cfg_$TAG
mkdir -p $O
cd $R
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 300 $B --batch 262144 --precision f16 --steps 10 --warmup 3 > $O/c3_f16.log 2>&1
timeout -k 10 300 $B --batch 262144 --steps 10 --warmup 3 > $O/c3_fp32.log 2>&1
timeout -k 10 300 $B --batch 15 --steps 50 --warmup 5 > $O/c1_b15.log 2>&1
timeout -k 10 300 $B --batch 15 --steps 100 --warmup 5 --graphed > $O/c1_b15_graphed.log 2>&1
timeout -k 10 300 $B --batch 15 --steps 50 --warmup 5 --small-limit 0 > $O/c1_b15_fused.log 2>&1
timeout -k 10 300 $B --batch 256 --steps 50 --warmup 5 > $O/c1_b256.log 2>&1
timeout -k 10 300 $B --batch 256 --steps 100 --warmup 5 --graphed > $O/c1_b256_graphed.log 2>&1
timeout -k 10 600 $B --horizon 25 --hidden 256 --steps 5 --warmup 2 > $O/c5.log 2>&1
timeout -k 10 600 $B --horizon 25 --hidden 256 --steps 5 --warmup 2 --wide-keep-budget max > $O/c5max.log 2>&1
for f in $O/*.log; do echo "== $f"; python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print(d['config']['workload'], '| value %.4g' % d['value'], '| ms %.3f' % d['ms_per_step'], '| kernels', d['kernels_ms'].get('fwd'), d['kernels_ms'].get('bwd'), '| grad_err', d.get('grad_max_rel_err'), '| frac %.3f' % d['roofline']['frac'])
"; done

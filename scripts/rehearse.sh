# N > 1 rehearsal on a 1-GPU box: bench.py --gpus N --share-gpu (every rank on cuda:0 over gloo; the launcher, barriers,
# grad all-reduce, max-over-ranks clock and the per-rank table), one gpurun step: scripts/rehearse.sh TAG [N]
set -e -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-rehearse}
NR=${2:-2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py --gpus $NR --share-gpu --steps 10 --warmup 3 --grad-check off > $OUT/rehearse_$NR.log 2>&1
grep '^{' $OUT/rehearse_$NR.log | tail -c 1500

# Round 3 profile, part 2 (one gpurun call): the config-4 rehearsal (8 ranks time-sharing cuda:0 over gloo, grad
# check on), then config 5 (every window kept: --wide-keep-budget max): its bench line (10 timed steps), rocprofv3
# kernel statistics and HBM PMC passes.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-round3}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py --gpus 8 --share-gpu --steps 10 --warmup 2 > $O/rehearse8.log 2>&1
grep '^{' $O/rehearse8.log | tail -c 600
cd /tmp && export TMPDIR=/tmp
C5="python3 $R/bench.py --hidden 256 --horizon 25 --batch 65536 --wide-keep-budget max"
timeout -k 10 400 $C5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1
grep '^{' $O/bench_c5.log | tail -c 300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5trace -o c5 -- $C5 --steps 3 --warmup 1 --no-cpu-baseline --grad-check off > $O/c5trace.log 2>&1
echo trace ok
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5fetch -o c5 -- $C5 --steps 1 --warmup 1 --no-cpu-baseline --grad-check off > $O/c5fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5write -o c5 -- $C5 --steps 1 --warmup 1 --no-cpu-baseline --grad-check off > $O/c5write.log 2>&1
echo pmc ok
mkdir -p $O/c5 && ln -sfn ../c5fetch $O/c5/fetch && ln -sfn ../c5write $O/c5/write   # relative: valid on the box and here
(cd $R && python3 scripts/pmc_c5_summary.py $TAG $O/c5 > $O/c5summary.log 2>&1)
tail -20 $O/c5summary.log

# Round 3 profile, part 1 (one gpurun call): the GPU suite, then the default benchmark's bench line, the rocprofv3
# kernel statistics of that SAME command (with the bench line it printed under the profiler), and PMC passes.
# usage: scripts/profile_round3.sh TAG   -> gpurun_out/prof_TAG/ (copy the summaries into profiles/)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-round3}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -1 $O/gputest.log
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 20 --warmup 5"
SHORT="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --grad-check off"
timeout -k 10 300 $CMD > $O/bench.log 2>&1
tail -c 300 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o $TAG -- $CMD > $O/trace.log 2>&1
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o $TAG -- $SHORT > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o $TAG -- $SHORT > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/inst -o $TAG -- $SHORT > $O/inst.log 2>&1
echo pmc ok
(cd $R && python3 scripts/pmc_summary.py $TAG $O > $O/summary.log 2>&1)
head -40 $O/summary.log

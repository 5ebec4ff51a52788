# Round profile of the default benchmark (one gpurun call): bench line, rocprofv3 kernel statistics of the SAME
# command, and PMC passes (HBM bytes; MFMA / VALU instruction counts and the clock) on the H = 50 kernels.
# usage: scripts/profile_round.sh TAG   -> gpurun_out/prof_TAG/ (copy the summaries into profiles/)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-round2}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 20 --warmup 5"
SHORT="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --grad-check off"
timeout -k 10 300 $CMD > $O/bench.log 2>&1
tail -c 400 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o $TAG -- $CMD > $O/trace.log 2>&1
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o $TAG -- $SHORT > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o $TAG -- $SHORT > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/inst -o $TAG -- $SHORT > $O/inst.log 2>&1
echo pmc ok
(cd $R && python3 scripts/pmc_summary.py $TAG $O > $O/summary.log 2>&1)
cat $O/summary.log | head -60

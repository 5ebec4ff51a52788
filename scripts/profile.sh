# Profile of one benchmark configuration, in ONE gpurun call: [the GPU suite], the bench line, then the SAME command
# under rocprofv3 --kernel-trace --stats with the post-timing grad check and the CPU baseline off (so the statistics
# hold the product's kernels only), the timed dispatches of that trace, and the HBM / instruction PMC passes (each
# counter group its own run, MI355X_MICROARCH.md). Summaries: profiles/TAG[_CFG]_{kernel_stats.csv,timed_kernels.json,
# pmc.json} (copied here from gpurun_out/ after the call).
#   usage: scripts/profile.sh TAG [CONFIG] [gputest]
#   CONFIG: c2 (default: B 65 536, N 10, H 50, fp32) | c3 (B 262 144, f16) |
#           c3fp32 (B 262 144, fp32) | c5 (H 256, N 25, library keep budget) | c5max (c5, every window kept)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:?tag}
CFG=${2:-c2}
case $CFG in
  c2) ARGS=""; SUF="" ;;
  c3) ARGS="--batch 262144 --precision f16"; SUF="_c3f16" ;;
  c3fp32) ARGS="--batch 262144"; SUF="_c3fp32" ;;
  c5) ARGS="--hidden 256 --horizon 25"; SUF="_c5" ;;
  c5max) ARGS="--hidden 256 --horizon 25 --wide-keep-budget max"; SUF="_c5" ;;
  *) echo "unknown config $CFG"; exit 2 ;;
esac
case $CFG in c5*) K=10; W=2; KS=3; KP=1 ;; *) K=20; W=5; KS=20; KP=3 ;; esac
O=$R/gpurun_out/prof_${TAG}_$CFG
mkdir -p $O
cd $R
if [ "${3:-}" = gputest ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
  tail -1 $O/gputest.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 $R/bench.py $ARGS --steps $K --warmup $W > $O/bench.log 2>&1
grep '^{' $O/bench.log | tail -c 400
QUIET="--no-cpu-baseline --grad-check off"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o $TAG -- python3 $R/bench.py $ARGS --steps $KS --warmup $W $QUIET > $O/trace.log 2>&1
grep '^{' $O/trace.log | tail -c 300
echo trace ok
SHORT="python3 $R/bench.py $ARGS --steps $KP --warmup 1 $QUIET"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o $TAG -- $SHORT > $O/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o $TAG -- $SHORT > $O/write.log 2>&1
case $CFG in
  c5*) timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/inst -o $TAG -- $SHORT > $O/inst.log 2>&1 ;;
  *) timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/inst -o $TAG -- $SHORT > $O/inst.log 2>&1
     timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/wait -o $TAG -- $SHORT > $O/wait.log 2>&1 ;;
esac
echo pmc ok
cd $R
case $CFG in
  c5*) python3 scripts/pmc_c5_summary.py $TAG $O > $O/summary.log 2>&1 ;;
  *) python3 scripts/pmc_summary.py $TAG$SUF $O $ARGS > $O/summary.log 2>&1
     python3 scripts/trace_timed.py $(ls $O/trace/*kernel_trace.csv $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1) $W $KS profiles/$TAG${SUF}_timed_kernels.json > $O/timed.log 2>&1 ;;
esac
tail -30 $O/summary.log

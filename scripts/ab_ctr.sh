set -e
bash $GRAFT_REPO_ROOT/scripts/ab_r1.sh
rm -rf $GRAFT_REPO_ROOT/gpurun_out/ctr
bash $GRAFT_REPO_ROOT/scripts/counters.sh > /dev/null
cd $GRAFT_REPO_ROOT && python3 scripts/ctr_summary.py

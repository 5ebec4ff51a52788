# kernel trace of the B = 15 training step (config 1, the reference's batch): every kernel and gap of a step
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_b15 -o t -- python3 $R/bench.py --batch 15 --steps 30 --warmup 5 --no-cpu-baseline > $R/gpurun_out/tr_b15.log 2>&1

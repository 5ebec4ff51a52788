# Round 2f: full GPU suite on the final tree, config-5 bench line and its rocprofv3 kernel statistics
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2f
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -2 $O/gputest.log
timeout -k 10 300 python $R/bench.py --hidden 256 --horizon 25 --batch 65536 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.log 2>&1
tail -c 300 $O/bench_c5.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5trace -o c5 -- python3 $R/bench.py --hidden 256 --horizon 25 --batch 65536 --steps 2 --warmup 1 --no-cpu-baseline --grad-check off > $O/c5trace.log 2>&1
echo trace ok

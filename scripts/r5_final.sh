# Round-5 closing call: the whole GPU suite, the smoke, then config 5's two lines and the default bench line.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final5
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -1 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py --horizon 25 --hidden 256 --steps 10 --warmup 2 --wide-keep-budget max > $O/c5max.log 2>&1
tail -c 300 $O/c5max.log
timeout -k 10 600 python3 bench.py --horizon 25 --hidden 256 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_default.log 2>&1
tail -c 300 $O/c5_default.log
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
tail -c 300 $O/bench.log

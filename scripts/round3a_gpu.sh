# Round 3a: GPU suite on the new parity checks, the default bench line, the 8-rank --share-gpu rehearsal of
# config 4 (grad check on), and the config-5 line at the new default kept-window budget.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3a
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rP > $O/gputest.log 2>&1
tail -2 $O/gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
tail -c 1500 $O/bench.log
timeout -k 10 600 python bench.py --gpus 8 --share-gpu --steps 10 --warmup 2 > $O/rehearse8.log 2>&1
tail -c 1500 $O/rehearse8.log
timeout -k 10 400 python bench.py --hidden 256 --horizon 25 --batch 65536 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1
tail -c 1500 $O/bench_c5.log

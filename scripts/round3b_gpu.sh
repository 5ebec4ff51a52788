# Round 3b: GPU suite on the own-h backward + hi-only last transposed tile, then an A/B of the H = 50 kernels
# against the previous build (one process, interleaved rounds, then sustained back-to-back launches)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3b
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rP > $O/gputest.log 2>&1
tail -2 $O/gputest.log
timeout -k 10 300 python scripts/kbench.py lib_ab/base.so lib_ab/own.so --rounds 5 --sustain 20 > $O/kb.log 2>&1
cat $O/kb.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
tail -c 1200 $O/bench.log

# Round 3c: forward pointwise with shared reciprocals: GPU parity suite, then A/B against the previous build
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rP > $O/gputest.log 2>&1
tail -2 $O/gputest.log
timeout -k 10 300 python scripts/kbench.py lib_ab/own.so lib_ab/fwdrcp.so --rounds 5 --sustain 20 > $O/kb.log 2>&1
cat $O/kb.log
timeout -k 10 300 python scripts/kbench.py lib_ab/own.so lib_ab/fwdrcp.so --rounds 3 --batch 262144 --precision 1 > $O/kb_c3.log 2>&1
cat $O/kb_c3.log

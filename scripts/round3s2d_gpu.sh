# Carried backward scale (FCR_BWD_CARRY=1, the working tree): the whole GPU suite, then A/B against the session-start
# build and the permlane-free variant
set -o pipefail
O=gpurun_out/r3s2d
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -2 $O/gputest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/gputest.log | head -80; exit $rc; }
timeout -k 10 500 python -u scripts/kbench.py lib_ab/base.so lib_ab/cr.so lib_ab/crb.so lib_ab/pl.so --rounds 3 --sustain 30 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep lib $O/kbench.log

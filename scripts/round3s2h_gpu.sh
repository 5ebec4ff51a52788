# Time-major layers 0+1 in the H <= 52 forward (FCR_FWD_TM=1, the working tree): the whole GPU suite, then A/B
# against the session-start build (fp32-accurate and f16 mode)
set -o pipefail
O=gpurun_out/r3s2h
mkdir -p $O
cp lib_ab/tm.so forging-control_amd/lib/libfcr.so && timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -2 $O/gputest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/gputest.log | head -60; exit $rc; }
timeout -k 10 500 python -u scripts/kbench.py lib_ab/base.so lib_ab/tm.so --rounds 5 --sustain 40 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
timeout -k 10 500 python -u scripts/kbench.py lib_ab/tm.so lib_ab/base.so --rounds 5 --sustain 40 > $O/kbench2.log 2>&1 || { tail -20 $O/kbench2.log; exit 1; }
timeout -k 10 500 python -u scripts/kbench.py lib_ab/base.so lib_ab/tm.so --rounds 3 --sustain 20 --precision 1 --batch 262144 > $O/kbench_f16.log 2>&1 || { tail -20 $O/kbench_f16.log; exit 1; }
grep lib $O/kbench.log $O/kbench2.log $O/kbench_f16.log

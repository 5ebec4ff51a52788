# f16 mode: all three layers time-major in the forward (every layer resident): the whole GPU suite with it, then A/B
# against the two-layer time-major build at config 3 (B = 262 144, f16) and at config 2 (fp32, must be unchanged)
set -o pipefail
O=gpurun_out/r3s2i
mkdir -p $O
cp lib_ab/lp3.so forging-control_amd/lib/libfcr.so && timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -2 $O/gputest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/gputest.log | head -60; exit $rc; }
timeout -k 10 500 python -u scripts/kbench.py lib_ab/tm.so lib_ab/lp3.so --rounds 3 --sustain 20 --precision 1 --batch 262144 > $O/kbench_f16.log 2>&1 || { tail -20 $O/kbench_f16.log; exit 1; }
timeout -k 10 500 python -u scripts/kbench.py lib_ab/lp3.so lib_ab/tm.so --rounds 3 --sustain 20 --precision 1 --batch 262144 > $O/kbench_f16b.log 2>&1 || { tail -20 $O/kbench_f16b.log; exit 1; }
grep lib $O/kbench_f16.log $O/kbench_f16b.log

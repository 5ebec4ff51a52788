# Config 5: c_t rebuilt in the backward cell kernel instead of read (FCR_WIDE_CREC=1, the working tree): wide parity
# tests and the config-5 full batch, then A/B against the session-start build (kept windows at the default budget)
set -o pipefail
O=gpurun_out/r3s2f
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "wide or config5 or nonfinite or unscaled" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/tests.log | head -60; exit $rc; }
timeout -k 10 600 python -u scripts/kbench.py lib_ab/base.so lib_ab/crec.so --hidden 256 --horizon 25 --rounds 2 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep lib $O/kbench.log

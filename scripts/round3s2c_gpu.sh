# permlane lane-group reductions (FCR_PERMLANE=1, the working tree): parity + small-batch suites, then A/B against
# the session-start build, with and without the forward's read-first fence
set -o pipefail
O=gpurun_out/r3s2c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/kbench.py lib_ab/base.so lib_ab/pl.so lib_ab/plrf.so --rounds 3 --sustain 30 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep lib $O/kbench.log

# Minimal-shift range guard restored; surrogate guard test held to 4x torch fp32 (ill-conditioned case); suite, bench
R=$(pwd)
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_surrogate.py > $O/sur_tests.log 2>&1
rc=$?; tail -3 $O/sur_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1
rc2=$?; tail -3 $O/gpu_suite.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then echo "suite rc=$rc2: stop"; exit $rc2; fi
timeout -k 10 300 python -u scripts/bench_surrogate.py --B 256 65536 --steps 50 > $O/sur_bench.log 2>&1 || { tail -20 $O/sur_bench.log; exit 1; }
cat $O/sur_bench.log
exit $((rc + rc2))

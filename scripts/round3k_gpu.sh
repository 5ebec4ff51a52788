# Surrogate on the fused kernels: its GPU tests, the B = 256 / 65 536 step bench, and the 65 536 step's kernel statistics
R=$(pwd)
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_surrogate.py > $O/sur_tests.log 2>&1
rc=$?
tail -5 $O/sur_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
timeout -k 10 300 python -u scripts/bench_surrogate.py --B 256 65536 --steps 50 > $O/sur_bench.log 2>&1 || { tail -20 $O/sur_bench.log; exit 1; }
cat $O/sur_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o sur -- python3 $R/scripts/bench_surrogate.py --B 65536 --steps 20 --cpu-budget 0.2 > $R/$O/trace.log 2>&1 || { tail -20 $R/$O/trace.log; exit 1; }
echo "trace ok"

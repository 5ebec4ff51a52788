# Surrogate fixes (saturated output gate, coalesced partial sums, readout gradients): its tests, the rollout's GPU
# suite (the med3 in lstm_point_grad_h), a same-box rollout A/B against HEAD, the surrogate bench and kernel trace
R=$(pwd)
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_surrogate.py > $O/sur_tests.log 2>&1
rc=$?; tail -3 $O/sur_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
timeout -k 10 300 python -u scripts/kbench.py lib_ab/head.so lib_ab/cur.so --rounds 5 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
tail -6 $O/kbench.log
timeout -k 10 300 python -u scripts/bench_surrogate.py --B 256 4096 65536 --steps 50 > $O/sur_bench.log 2>&1 || { tail -20 $O/sur_bench.log; exit 1; }
cat $O/sur_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o sur -- python3 $R/scripts/bench_surrogate.py --B 65536 --steps 20 --cpu-budget 0.2 > $R/$O/trace.log 2>&1 || { tail -20 $R/$O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace256 -o sur -- python3 $R/scripts/bench_surrogate.py --B 256 --steps 20 --cpu-budget 0.2 > $R/$O/trace256.log 2>&1 || { tail -20 $R/$O/trace256.log; exit 1; }
echo "trace ok"
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1
rc=$?; tail -3 $O/gpu_suite.log; exit $rc

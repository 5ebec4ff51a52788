# Config 5 line again (it now finds round3b's committed PMC traffic) and config 3 at B = 262 144 in the
# fp32-accurate and the f16 modes
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 600 python -u bench.py --hidden 256 --horizon 25 --steps 10 --warmup 2 --no-cpu-baseline --wide-keep-budget max > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log | tail -1 | cut -c1-300
for p in fp32 f16 f16fwd; do
  timeout -k 10 400 python -u bench.py --batch 262144 --steps 10 --warmup 2 --no-cpu-baseline --precision $p > $O/bench_c3_$p.log 2>&1 || { tail -20 $O/bench_c3_$p.log; exit 1; }
  grep '^{' $O/bench_c3_$p.log | tail -1 | cut -c1-300
done
timeout -k 10 300 python -u scripts/bench_graphed.py > $O/graphed.log 2>&1 || { tail -20 $O/graphed.log; exit 1; }
tail -8 $O/graphed.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_surrogate.py > $O/sur_tests.log 2>&1; rc=$?; tail -2 $O/sur_tests.log; exit $rc

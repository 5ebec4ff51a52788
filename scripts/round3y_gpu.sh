# Config 5 per-row dgate scales, the row max on DPP: A/B against the global-scale and the shuffle builds; tests; line
# against the global-scale build, wide parity tests, and the config-5 line's gradient error
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 500 python -u scripts/kbench.py lib_ab/bufst2.so lib_ab/rowsc.so lib_ab/rowsc2.so --hidden 256 --horizon 25 --rounds 2 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
tail -3 $O/kbench.log
cp lib_ab/rowsc2.so forging-control_amd/lib/libfcr.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --hidden 256 --horizon 25 --steps 5 --warmup 1 --no-cpu-baseline --wide-keep-budget max > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log | tail -1 | cut -c1-200

# Final tree: smoke(), the default bench line, and config 3's f16 line
set -o pipefail
O=gpurun_out/r3s2j
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-300
timeout -k 10 300 python3 -u bench.py --precision f16 --batch 262144 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3_f16.log 2>&1 || { tail -20 $O/bench_c3_f16.log; exit 1; }
grep '^{' $O/bench_c3_f16.log | tail -1 | cut -c1-300

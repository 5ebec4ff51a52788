# Config 5 with the kept-window opt-in (--wide-keep-budget max): bench line (10 steps) with its grad check
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 600 python -u bench.py --hidden 256 --horizon 25 --steps 10 --warmup 2 --no-cpu-baseline --wide-keep-budget max > $O/bench_c5_keepmax.log 2>&1 || { tail -20 $O/bench_c5_keepmax.log; exit 1; }
tail -1 $O/bench_c5_keepmax.log | cut -c1-600

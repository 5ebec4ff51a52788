# Session-2 re-entry check: the GPU suite on the restored tree, then the default bench line
set -o pipefail
O=gpurun_out/r3s2a
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
tail -3 $O/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-400

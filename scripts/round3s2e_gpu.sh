# Longer A/B of the carried backward scale against the session-start build (two libraries only, 60 sustained steps)
set -o pipefail
O=gpurun_out/r3s2e
mkdir -p $O
timeout -k 10 500 python -u scripts/kbench.py lib_ab/base.so lib_ab/cr.so --rounds 5 --sustain 60 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
timeout -k 10 500 python -u scripts/kbench.py lib_ab/cr.so lib_ab/base.so --rounds 5 --sustain 60 > $O/kbench2.log 2>&1 || { tail -20 $O/kbench2.log; exit 1; }
grep lib $O/kbench.log $O/kbench2.log

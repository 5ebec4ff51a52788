# A/B: the next cell's own h kept in registers (FCR_OWN_REG 1) vs re-read from the slab (0)
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 400 python -u scripts/kbench.py lib_ab/own0.so lib_ab/own1.so --rounds 7 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
tail -4 $O/kbench.log

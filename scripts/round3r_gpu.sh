# A/B: half-block transposed tiles from duplicate LDS reads (no operand copies) vs the register-kept own h build
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 400 python -u scripts/kbench.py lib_ab/own1.so lib_ab/half.so --rounds 7 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
tail -4 $O/kbench.log

# A/B: the two waves of a SIMD delayed against each other after every phase barrier (FCR_STAGGER x 64 cycles of
# s_sleep on waves 4-7), with and without the cell-by-cell priority alternation
set -o pipefail
O=gpurun_out/r3s2g
mkdir -p $O
timeout -k 10 600 python -u scripts/kbench.py lib_ab/base.so lib_ab/st16.so lib_ab/st60.so lib_ab/st16np.so --rounds 3 --sustain 40 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep lib $O/kbench.log

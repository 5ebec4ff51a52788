# Round 3e: (1) A/B of loop unrolling on the H = 50 kernels; (2) parity of the hand-written config-5 gradient
# product (fcr_wbwd.h) on every wide test; (3) config-5 A/B hand-written vs rocBLAS backward product
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3e
mkdir -p $O
cd $R
true
true
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_inference.py -x -v --timeout 300 --timeout-method thread -rP -k "wide or config5 or golden or h256 or inference" > $O/wide_tests.log 2>&1
tail -3 $O/wide_tests.log
timeout -k 10 600 python scripts/kbench.py lib_ab/blasbwd.so lib_ab/hwbwd.so --hidden 256 --horizon 25 --rounds 2 > $O/kb_c5.log 2>&1
cat $O/kb_c5.log

# Config 5 forward cell GEMM with the split four-half mainloop (8 waves, 3-stage 48 KB ring): A/B against the
# K-concatenated build at B = 65536, N = 25, H = 256, then the wide-path parity tests on it
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 500 python -u scripts/kbench.py lib_ab/bufst2.so lib_ab/wg4.so --hidden 256 --horizon 25 --rounds 3 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
tail -3 $O/kbench.log
cp lib_ab/wg4.so forging-control_amd/lib/libfcr.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "wide or h256 or H64 or 64 or 256 or config5" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; exit $rc

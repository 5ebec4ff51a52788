# A/B: backward dx stores through the dseq buffer descriptor vs the buffer-forward build; tests
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 400 python -u scripts/kbench.py lib_ab/bufst.so lib_ab/bufst2.so --rounds 7 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
tail -4 $O/kbench.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_surrogate.py tests/test_gpu_parity.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; exit $rc

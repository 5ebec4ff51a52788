set -e -o pipefail
mkdir -p gpurun_out/chk
FCR_LIB=$PWD/lib_ab/wb512.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_cell.py tests/test_gpu_parity.py -m gpu -k "wide or cell or h256" > gpurun_out/chk/wb512_tests.log 2>&1
tail -1 gpurun_out/chk/wb512_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_cell.py tests/test_gpu_parity.py tests/test_surrogate.py tests/test_gpu_small.py -m gpu > gpurun_out/chk/prod_tests.log 2>&1
tail -1 gpurun_out/chk/prod_tests.log
timeout -k 10 600 python3 bench.py --horizon 25 --hidden 256 --steps 10 --warmup 2 --wide-keep-budget max > gpurun_out/chk/c5max.log 2>&1
tail -c 400 gpurun_out/chk/c5max.log

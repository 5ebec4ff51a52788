set -e -o pipefail
mkdir -p gpurun_out/wb512
export FCR_LIB=$PWD/lib_ab/wb512.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_cell.py tests/test_gpu_parity.py tests/test_surrogate.py tests/test_gpu_small.py -m gpu > gpurun_out/wb512/tests.log 2>&1
tail -3 gpurun_out/wb512/tests.log
unset FCR_LIB
timeout -k 10 400 python scripts/kbench.py lib_ab/prod.so lib_ab/wb512.so --batch 65536 --horizon 25 --hidden 256 --rounds 3 --keep-budget 272000000000 > gpurun_out/wb512/ab_keepall.log 2>&1
tail -6 gpurun_out/wb512/ab_keepall.log
for v in fwd_no_act fwd_hot_rec fwd_no_cst; do
timeout -k 10 400 python scripts/kbench.py lib_ab/prod.so lib_ab/$v.so --batch 65536 --horizon 25 --hidden 256 --rounds 2 --keep-budget 272000000000 > gpurun_out/wb512/ab_$v.log 2>&1
tail -4 gpurun_out/wb512/ab_$v.log
done

# Tests of candidate lib_ab/$1.so (FCR_LIB), then one kbench process timing prod, $1 and $2 at config 5 keep-all and
# default budget. usage: scripts/r5_ab3.sh CAND OTHER
set -e -o pipefail
N=$1; M=$2
mkdir -p gpurun_out/$N
FCR_LIB=$PWD/lib_ab/$N.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_wide_cell.py tests/test_gpu_parity.py tests/test_surrogate.py tests/test_gpu_small.py -m gpu > gpurun_out/$N/tests.log 2>&1
tail -2 gpurun_out/$N/tests.log
timeout -k 10 500 python scripts/kbench.py lib_ab/prod.so lib_ab/$N.so lib_ab/$M.so --batch 65536 --horizon 25 --hidden 256 --rounds 2 --keep-budget 272000000000 > gpurun_out/$N/ab_keepall.log 2>&1
tail -3 gpurun_out/$N/ab_keepall.log
timeout -k 10 500 python scripts/kbench.py lib_ab/prod.so lib_ab/$N.so lib_ab/$M.so --batch 65536 --horizon 25 --hidden 256 --rounds 2 > gpurun_out/$N/ab_default.log 2>&1
tail -3 gpurun_out/$N/ab_default.log

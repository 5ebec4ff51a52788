# Same-process A/B of a candidate build against lib_ab/prod.so: its wide GPU tests first (FCR_LIB), then config 5
# keep-all and default budget. usage: scripts/r5_ab.sh NAME [rounds]
# (lib_ab/prod.so: a copy of the current forging-control_amd/lib/libfcr.so; lib_ab/NAME.so: the candidate, e.g. from
# scripts/build_patch_variant.py or hipcc with a -D option)
set -e -o pipefail
N=$1; RND=${2:-3}
mkdir -p gpurun_out/$N
FCR_LIB=$PWD/lib_ab/$N.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_wide_cell.py tests/test_gpu_parity.py tests/test_surrogate.py tests/test_gpu_small.py -m gpu > gpurun_out/$N/tests.log 2>&1
tail -2 gpurun_out/$N/tests.log
bash scripts/ab_c5.sh gpurun_out/$N lib_ab/prod.so lib_ab/$N.so $RND

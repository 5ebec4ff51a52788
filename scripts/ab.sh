# Same-process A/B of library builds (scripts/kbench.py: interleaved rounds, one device, one batch), optionally after
# the GPU tests of every candidate. The first library is the reference of the comparison (outputs are checked against
# it); lib_ab/prod.so is normally a copy of forging-control_amd/lib/libfcr.so, the others come from
# scripts/build_patch_variant.py, scripts/build_variant.sh or scripts/build_head.sh.
#   usage: scripts/ab.sh OUTDIR CONFIG LIB_A LIB_B [LIB_C ...] [--rounds R] [--tests]
#   CONFIG: c2 (B 65 536, N 10, H 50) | c3 (B 262 144, f16) | c3fp32 (B 262 144) | c1 (B 15) |
#           c5 (B 65 536, N 25, H 256: every window kept, then the library's default keep budget) | c5max (kept only)
#   --tests: tests/test_wide_cell.py, test_gpu_parity.py, test_surrogate.py and test_gpu_small.py against each of
#            LIB_B ... (FCR_DEV=1 FCR_LIB=...) before any timing; a red candidate stops the call
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:?outdir}; CFG=${2:?config}; shift 2
LIBS=(); RND=3; TESTS=0
while [ $# -gt 0 ]; do
  case $1 in
    --rounds) RND=$2; shift 2 ;;
    --tests) TESTS=1; shift ;;
    *) LIBS+=("$1"); shift ;;
  esac
done
[ ${#LIBS[@]} -ge 2 ] || { echo "need at least two libraries"; exit 2; }
mkdir -p $OUT
cd $R
if [ $TESTS = 1 ]; then
  for L in "${LIBS[@]:1}"; do
    n=$(basename $L .so)
    FCR_DEV=1 FCR_LIB=$(realpath $L) timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_wide_cell.py tests/test_gpu_parity.py tests/test_surrogate.py tests/test_gpu_small.py -m gpu \
      > $OUT/tests_$n.log 2>&1
    echo "tests $n: $(tail -1 $OUT/tests_$n.log)"
  done
fi
KB="timeout -k 10 500 python scripts/kbench.py ${LIBS[*]} --rounds $RND"
case $CFG in
  c2) $KB > $OUT/ab_c2.log 2>&1; tail -6 $OUT/ab_c2.log ;;
  c3) $KB --batch 262144 --precision 1 > $OUT/ab_c3.log 2>&1; tail -6 $OUT/ab_c3.log ;;
  c3fp32) $KB --batch 262144 > $OUT/ab_c3fp32.log 2>&1; tail -6 $OUT/ab_c3fp32.log ;;
  c1) $KB --batch 15 > $OUT/ab_c1.log 2>&1; tail -6 $OUT/ab_c1.log ;;
  c5|c5max)
    $KB --batch 65536 --horizon 25 --hidden 256 --keep-budget 272000000000 > $OUT/ab_c5_keepall.log 2>&1
    tail -6 $OUT/ab_c5_keepall.log
    if [ $CFG = c5 ]; then
      $KB --batch 65536 --horizon 25 --hidden 256 > $OUT/ab_c5_default.log 2>&1
      tail -6 $OUT/ab_c5_default.log
    fi ;;
  *) echo "unknown config $CFG"; exit 2 ;;
esac

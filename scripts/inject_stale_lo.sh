# Fault injection for tests/test_wide_cell.py: build lib_ab/inject_stale_lo.so from a copy of the
# sources whose fused backward cell (csrc/fcr_wbwd.h) reads its lo-half A fragments from the OTHER ring slot at K step
# nk - 2 — the stale lo stage the round-4 variant (c) read at that step through its off-by-one vmcnt — and run the
# per-element tests against it: they must FAIL (the product's own build passes them).
#   usage: bash scripts/inject_stale_lo.sh build      (here: hipcc cross-compiles; the .so travels with the tree)
#          bash scripts/inject_stale_lo.sh OUTDIR     (on the GPU box: the tests against the injected build)
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$R/gpurun_out/inject}
if [ "$OUT" = build ]; then
mkdir -p $R/lib_ab
T=$(mktemp -d)
cp -r $R/forging-control_amd/csrc $T/csrc
python3 - $T/csrc/fcr_wbwd.h <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
a = "al[i] = *reinterpret_cast<const f16x8 *>(st + kWbStageA + wb_off(r, fq));"
b = ("al[i] = *reinterpret_cast<const f16x8 *>((ks == nk - 2 ? lds + (buf ^ 1) * kWbStage : st) + kWbStageA + "
     "wb_off(r, fq));")
assert s.count(a) == 1, "injection site moved"
open(p, "w").write(s.replace(a, b))
PY
/opt/rocm/bin/hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -std=c++17 -shared -fPIC -I $R/include -I $T/csrc \
  $T/csrc/fcr_abi.hip $T/csrc/fcr_rows.hip -o $R/lib_ab/inject_stale_lo.so
rm -rf $T
exit 0
fi
mkdir -p $OUT
cd $R
set +e
FCR_DEV=1 FCR_LIB=$R/lib_ab/inject_stale_lo.so timeout -k 10 300 python -u -m pytest tests/test_wide_cell.py -m gpu -v \
  --timeout 120 --timeout-method thread -k layer_cell > $OUT/inject_stale_lo.log 2>&1
rc=$?
set -e
tail -12 $OUT/inject_stale_lo.log
if [ $rc -eq 0 ]; then echo "INJECTED FAULT NOT DETECTED"; exit 1; fi
echo "injected stale lo stage detected (pytest rc $rc)"

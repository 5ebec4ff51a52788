# Round 3g: isolated gradient-product check with small dgates; h256 golden case on hw / hw+dg3 / rocBLAS builds
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3g
mkdir -p $O
cd $R
#timeout -k 10 300 python scripts/wb_check.py lib_ab/wbtest.so > $O/wb_check.log 2>&1
#cat $O/wb_check.log
cat > /tmp/h256.py <<'PY'
import sys; sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from conftest import load_case, relerr
from test_gpu_parity import run, GRADS, FEATS
for name in ("h256_b8_n25", "h64_b24_n3"):
    c, params = load_case(name)
    o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"])
    print(name, {k: f"{relerr(o[k], c[k + '_64']):.2e}" for k in ("loss", "xhat") + tuple(g for g, _ in GRADS)})
PY
for v in wbl1 wbl6 hwbwd; do
  cp lib_ab/$v.so forging-control_amd/lib/libfcr.so
  timeout -k 10 120 python /tmp/h256.py > $O/h256_$v.log 2>&1; echo $v; tail -2 $O/h256_$v.log
done

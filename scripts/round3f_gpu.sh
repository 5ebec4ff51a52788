# Round 3f: the config-5 gradient product kernel in isolation (scripts/wb_check.py), then the h256 golden case on
# the hand-written and on the rocBLAS backward product (error printed for both)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3f
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/wb_check.py lib_ab/wbtest.so > $O/wb_check.log 2>&1
cat $O/wb_check.log
cat > /tmp/h256.py <<'PY'
import sys; sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from conftest import load_case, relerr
from test_gpu_parity import run, GRADS, FEATS
c, params = load_case("h256_b8_n25")
o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"])
print({k: f"{relerr(o[k], c[k + '_64']):.2e}" for k in ("loss", "prediction", "xhat") + tuple(g for g, _ in GRADS)})
PY
timeout -k 10 120 python /tmp/h256.py > $O/h256_hw.log 2>&1; cat $O/h256_hw.log | tail -1
cp lib_ab/blasbwd.so forging-control_amd/lib/libfcr.so
timeout -k 10 120 python /tmp/h256.py > $O/h256_blas.log 2>&1; cat $O/h256_blas.log | tail -1

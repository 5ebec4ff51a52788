# Round 3h: diagnostic build comparing the hand-written and rocBLAS layer>=1 products (h256 case), with one call's
# operands dumped for an offline fp64 check
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3h
mkdir -p $O
cd $R
cp lib_ab/wbtwice.so forging-control_amd/lib/libfcr.so
cat > /tmp/cmp.py <<'PY'
import sys, ctypes; sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
from conftest import load_case, relerr
from test_gpu_parity import run, GRADS
import forging_control_amd as fca
lib = fca._native.load()
c, params = load_case("h256_b8_n25")
o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"])
out = (ctypes.c_float * 4)()
lib.fcr_debug_wbdiff(out)
print(list(out))
B, H = 8, 256
buf = np.zeros(B * 12 * H * 2 + B * 2 * H * 4 * 2, np.uint8)
print("dump rows", lib.fcr_debug_dump(buf.ctypes.data_as(ctypes.c_void_p)))
np.save("gpurun_out/r3h/dump.npy", buf)
cd = (ctypes.c_float * 4096)()
lib.fcr_debug_calldiff(cd)
cd = np.array(cd).reshape(2048, 2)
for j in range(25):
    for l in (1, 2):
        for t in range(10):
            i = (j * 3 + l) * 10 + t
            if cd[i, 0] > 3e-6:
                print("call j=%d l=%d t=%d row-part rel diff %.3e (max |blas| %.3e)" % (j, l, t, cd[i, 0], cd[i, 1]))
PY
timeout -k 10 120 python /tmp/cmp.py > $O/cmp.log 2>&1; tail -3 $O/cmp.log

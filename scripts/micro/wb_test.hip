// Stand-alone harness of the config-5 gradient product kernel (fcr_wbwd.h): launches wide_bwd_gemm_kernel on
// caller-provided device buffers (scripts/wb_check.py compares it with an fp64 torch product).
#include <hip/hip_runtime.h>
#include "fcr_wbwd.h"
using namespace fcr;
extern "C" int wb_run(const _Float16 *ahi, const _Float16 *alo, const _Float16 *b, float *out, int lda, int ldb, int lo_off,
                      int ldo, int NB, int NO, int K, void *stream) {
    static bool set = false;
    if (!set) {
        if (hipFuncSetAttribute((const void *)wide_bwd_gemm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kWbLds))
            return -3;
        set = true;
    }
    WbArgs a{ahi, alo, b, out, lda, ldb, lo_off, ldo, NB, NO, K};
    const int nx = (NB + kWbN - 1) / kWbN, ny = (NO + kWbM - 1) / kWbM;
    hipLaunchKernelGGL(wide_bwd_gemm_kernel, dim3(nx * ny), dim3(kWbThreads), kWbLds, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

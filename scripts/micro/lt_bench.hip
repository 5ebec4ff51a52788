// Config-5 split-f16 GEMM shapes (fcr_abi.hip gemm16_fwd / gemm16_bwd): rocblas_gemm_ex against the
// hipBLASLt heuristic's candidates, f16 in, fp32 accumulate and out. Prints us and TFLOP/s per shape.
//   hipcc --offload-arch=gfx950 -O2 lt_bench.hip -o lt_bench -lrocblas -lhipblaslt
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        auto e_ = (x);                                                          \
        if ((int)e_ != 0) {                                                     \
            std::printf("error %d at %s:%d\n", (int)e_, __FILE__, __LINE__);   \
            return 1;                                                           \
        }                                                                       \
    } while (0)

template <class F>
static float time_us(F f, hipStream_t s, int reps = 20) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return 1000.0f * ms / reps;
}

// C (m x n, ld m, fp32) = op(A) . B with A stored [k][m] (transA) or [m][k]... as rocBLAS column-major:
// transA: A is k x m column-major (lda = k); B is k x n column-major (ldb = k).
static int run(rocblas_handle rb, hipblasLtHandle_t lt, hipStream_t s, const char *name, int m, int n, int k,
               bool transA, void *A, void *B, float *C, void *ws, size_t wsb) {
    const float one = 1.0f, zero = 0.0f;
    const int lda = transA ? k : m, ldb = k;
    const double fl = 2.0 * m * n * k;
    float t_rb = time_us([&] {
        rocblas_gemm_ex(rb, transA ? rocblas_operation_transpose : rocblas_operation_none, rocblas_operation_none, m, n,
                        k, &one, A, rocblas_datatype_f16_r, lda, B, rocblas_datatype_f16_r, ldb, &zero, C,
                        rocblas_datatype_f32_r, m, C, rocblas_datatype_f32_r, m, rocblas_datatype_f32_r,
                        rocblas_gemm_algo_standard, 0, 0);
    }, s);
    std::printf("%s m=%d n=%d k=%d  rocblas %.1f us %.0f TF/s\n", name, m, n, k, t_rb, fl / t_rb * 1e-6);

    hipblasLtMatmulDesc_t md;
    CK(hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16F, transA ? k : m, transA ? m : k, lda));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16F, k, n, ldb));
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, m, n, m));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsl = wsb;
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsl, sizeof(wsl)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(32);
    int nres = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(lt, md, la, lb, lc, lc, pref, 32, res.data(), &nres));
    float best = 1e30f;
    int besti = -1;
    for (int i = 0; i < nres; ++i) {
        if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > wsb) continue;
        hipblasStatus_t st = HIPBLAS_STATUS_SUCCESS;
        float t = time_us([&] {
            st = hipblasLtMatmul(lt, md, &one, A, la, B, lb, &zero, C, lc, C, lc, &res[i].algo, ws, wsb, s);
        }, s, 10);
        if (st != HIPBLAS_STATUS_SUCCESS) continue;
        if (i < 3) std::printf("   lt algo %d: %.1f us %.0f TF/s (ws %zu)\n", i, t, fl / t * 1e-6, res[i].workspaceSize);
        if (t < best) {
            best = t;
            besti = i;
        }
    }
    std::printf("   hipblaslt best of %d: algo %d %.1f us %.0f TF/s  (%.2fx rocblas)\n", nres, besti, best,
                fl / best * 1e-6, t_rb / best);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatmulDescDestroy(md);
    return 0;
}

int main() {
    const int H = 256, B = 65536;
    hipStream_t s;
    hipStreamCreate(&s);
    rocblas_handle rb;
    rocblas_create_handle(&rb);
    rocblas_set_stream(rb, s);
    rocblas_set_atomics_mode(rb, rocblas_atomics_not_allowed);
    hipblasLtHandle_t lt;
    CK(hipblasLtCreate(&lt));
    const size_t wsb = 64u << 20;
    void *A, *Bm, *ws;
    float *C;
    CK(hipMalloc(&A, sizeof(_Float16) * 12 * H * 2 * H));
    CK(hipMalloc(&Bm, sizeof(_Float16) * (size_t)B * 12 * H));
    CK(hipMalloc(&C, sizeof(float) * (size_t)B * 4 * H));
    CK(hipMalloc(&ws, wsb));
    CK(hipMemset(A, 0x11, sizeof(_Float16) * 12 * H * 2 * H));
    CK(hipMemset(Bm, 0x11, sizeof(_Float16) * (size_t)B * 12 * H));
    // forward: G (4H x B) = A^T (A [4H][6H] row-major = 6H x 4H col-major) . XB (6H x B)
    if (run(rb, lt, s, "fwd K=6H", 4 * H, B, 6 * H, true, A, Bm, C, ws, wsb)) return 1;
    if (run(rb, lt, s, "fwd K=3H", 4 * H, B, 3 * H, true, A, Bm, C, ws, wsb)) return 1;
    // backward: dX (H x B) = A (H x 12H col-major = [12H][H] row-major) . dGs (12H x B)
    if (run(rb, lt, s, "bwd N=H", H, B, 12 * H, false, A, Bm, C, ws, wsb)) return 1;
    // both backward products in one GEMM: [dX | dH] (2H x B) = [A_ih | A_hh] (2H x 12H) . dGs
    if (run(rb, lt, s, "bwd N=2H", 2 * H, B, 12 * H, false, A, Bm, C, ws, wsb)) return 1;
    std::printf("done\n");
    return 0;
}

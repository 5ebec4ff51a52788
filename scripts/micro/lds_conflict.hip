// Micro-test: LDS bank conflicts of the backward's image read patterns (fcr_img.h), one kernel per
// pattern so rocprofv3 --pmc SQ_LDS_BANK_CONFLICT attributes them. Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "fcr_img.h"
using namespace fcr;

template <int MODE, int RB>
__global__ void pat(float *out, int iters) {
    extern __shared__ __attribute__((aligned(16))) float lw[];
    for (int i = threadIdx.x; i < 163840 / 4; i += blockDim.x) lw[i] = (float)i;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const ImgLane<RB> L = img_lane<RB>(lds_offset(lw), lane);
    float acc = 0.0f;
    for (int it = 0; it < iters; ++it) {
        uint32_t fb = L.fb, tb = L.tb;
        asm volatile("" : "+v"(fb), "+v"(tb));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            f16x4 v;
            if (MODE == 0) v = lds_b64_f16((fb ^ (8u * (8 * ((k >> 1) % (RB / 64)) + (k & 1)))) + (k & 3) * 16 * RB);  // forward
            else if (MODE == 1) v = lds_tr_f16((tb ^ (8u * (8 * ((k % (RB / 32 - 1)) >> 1) + ((k % (RB / 32 - 1)) & 1)))) + (k & 3) * 16 * RB);  // tr
            else v = lds_b64_f16(lds_offset(lw) + lane * 8 + k * 512);   // linear reference
            acc += (float)v[0] + (float)v[1] + (float)v[2] + (float)v[3];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    float *out;
    hipMalloc(&out, 1024 * 512 * 4);
    auto run = [&](auto k, const char *name) {
        hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
        hipLaunchKernelGGL(k, dim3(256), dim3(512), 163840, 0, out, 2000);
        hipDeviceSynchronize();
        printf("%s %s\n", name, hipGetErrorString(hipGetLastError()));
    };
    run(pat<0, 256>, "fwd256");
    run(pat<1, 256>, "tr256");
    run(pat<0, 128>, "fwd128");
    run(pat<1, 128>, "tr128");
    run(pat<2, 256>, "linear");
    return 0;
}

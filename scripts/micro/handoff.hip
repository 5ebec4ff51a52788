// Micro-benchmark: the latency of handing a value between two waves, as a ping-pong of flag + payload, in shader-clock
// cycles (s_memtime counts the core clock; s_memrealtime the 100 MHz wall clock, both read here). Prices two schedules the rollout kernels could take:
//   lds   — two waves of ONE workgroup on different SIMDs pass a 16-B-per-lane record and a flag through LDS (the
//           pairing a 16-wave fcr_fwd/fcr_bwd geometry would need once per cell);
//   l2    — two workgroups (one wave each) on the same XCD pass the same through global memory (device-scope release /
//           acquire), the hand-off a layer-wavefront B = 15 schedule needs between the CUs that hold its layers' images;
//   xcd   — the same between workgroups on two different XCDs (each XCD has its own L2).
// Every spin is bounded (kMaxSpin polls), so a wave whose partner never arrives still ends; the host reports such a
// timeout. Vector memory instructions only. Diagnostic, not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/micro/handoff scripts/micro/handoff.hip && scripts/micro/handoff
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kIters = 2000;
constexpr int kMaxSpin = 1 << 22;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ unsigned long long wall() { return __builtin_amdgcn_s_memrealtime(); }

// two waves of one workgroup (threads 0..63 and 64..127 land on different SIMDs)
__global__ __launch_bounds__(128) void lds_pingpong(unsigned long long *out, int *timeouts) {
    __shared__ float rec[2][64 * 4];
    __shared__ int flag[2];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < 2) flag[threadIdx.x] = -1;
    __syncthreads();
    float v = (float)lane;
    int bad = 0;
    const unsigned long long t0 = now(), r0 = wall();
    for (int i = 0; i < kIters; ++i) {
        if ((i & 1) == w) {   // my turn to send: payload, then the flag after the payload's writes completed
            *reinterpret_cast<float4 *>(&rec[i & 1][lane * 4]) = make_float4(v, v + 1, v + 2, v + 3);
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
            if (lane == 0) __hip_atomic_store(&flag[w], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {               // wait for the partner's flag, then read its payload
            int s = 0;   // wave-uniform spin (readfirstlane): a scalar branch, no per-lane exec juggling
            while (__builtin_amdgcn_readfirstlane(
                       __hip_atomic_load(&flag[w ^ 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < i &&
                   ++s < kMaxSpin) {
            }
            bad |= s >= kMaxSpin;
            const float4 r = *reinterpret_cast<const float4 *>(&rec[i & 1][lane * 4]);
            v = r.x + r.w * 1e-9f;
        }
    }
    const unsigned long long t1 = now(), r1 = wall();
    if (lane == 0) {
        out[w] = t1 - t0;
        out[2 + w] = r1 - r0;
        if (bad) atomicAdd(timeouts, 1);
    }
    if (v == -1.0f) out[4] = 0;   // keep v live
}

// two workgroups, one wave each: blockIdx.x == 0 and blockIdx.x == partner play; the others exit at once
__global__ __launch_bounds__(64) void gmem_pingpong(float *rec, int *flag, int partner, unsigned long long *out,
                                                   int *timeouts) {
    const int me = blockIdx.x == 0 ? 0 : blockIdx.x == (unsigned)partner ? 1 : -1;
    if (me < 0) return;
    const int lane = threadIdx.x;
    float v = (float)lane;
    int bad = 0;
    const unsigned long long t0 = now(), r0 = wall();
    for (int i = 0; i < kIters && !bad; ++i) {
        if ((i & 1) == me) {
            reinterpret_cast<float4 *>(rec + (size_t)(i & 1) * 256)[lane] = make_float4(v, v + 1, v + 2, v + 3);
            __atomic_thread_fence(__ATOMIC_RELEASE);   // device scope: payload visible before the flag
            if (lane == 0) __hip_atomic_store(&flag[me], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            int s = 0;
            while (__builtin_amdgcn_readfirstlane(
                       __hip_atomic_load(&flag[me ^ 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < i &&
                   ++s < kMaxSpin) {
            }
            bad |= s >= kMaxSpin;
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            const float4 r = reinterpret_cast<const float4 *>(rec + (size_t)(i & 1) * 256)[lane];
            v = r.x + r.w * 1e-9f;
        }
    }
    const unsigned long long t1 = now(), r1 = wall();
    if (lane == 0) {
        out[me] = t1 - t0;
        out[2 + me] = r1 - r0;
        if (bad) atomicAdd(timeouts, 1);
    }
    if (v == -1.0f) out[4] = 0;
}

int main() {
    unsigned long long *out;
    int *timeouts, *flag;
    float *rec;
    hipMalloc(&out, 5 * sizeof(unsigned long long));
    hipMalloc(&timeouts, sizeof(int));
    hipMalloc(&flag, 2 * sizeof(int));
    hipMalloc(&rec, 2 * 256 * sizeof(float));
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, 0);   // s_memrealtime ticks per ms (kHz)
    auto report = [&](const char *name) {
        unsigned long long h[4];
        int t = 0;
        hipMemcpy(h, out, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        hipMemcpy(&t, timeouts, sizeof(int), hipMemcpyDeviceToHost);
        const double cyc = (double)(h[0] > h[1] ? h[0] : h[1]) / kIters;   // one one-way hand-off
        const double ns = (double)(h[2] > h[3] ? h[2] : h[3]) / kIters * 1e6 / clk;
        printf("%-28s one-way hand-off %7.1f shader cycles = %6.1f ns (%.2f GHz)%s\n", name, cyc, ns, cyc / ns,
               t ? "  (TIMEOUTS)" : "");
    };
    for (int rep = 0; rep < 3; ++rep) {
        hipMemset(timeouts, 0, sizeof(int));
        hipLaunchKernelGGL(lds_pingpong, dim3(1), dim3(128), 0, 0, out, timeouts);
        hipDeviceSynchronize();
        report("lds (two waves, one CU)");
        for (int partner : {8, 1}) {   // workgroup ids go round-robin over the 8 XCDs: 8 = same XCD, 1 = the next one
            hipMemset(timeouts, 0, sizeof(int));
            hipMemset(flag, 0xff, 2 * sizeof(int));
            hipLaunchKernelGGL(gmem_pingpong, dim3(partner + 1), dim3(64), 0, 0, rec, flag, partner, out, timeouts);
            hipDeviceSynchronize();
            report(partner == 8 ? "l2 (same XCD)" : "xcd (two XCDs)");
        }
    }
    printf("s_memrealtime clock %d kHz; %s\n", clk, hipGetErrorString(hipGetLastError()));
    return 0;
}

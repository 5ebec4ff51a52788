// fcr_plant.h — the open-die forging press as a batched fp64 RK4 integrator.
//
// Reference: FeasibilityRecovery.forging_model (Functions.py:1615-1740) / template_model
// (template_model.py:19-149, pressures floored by smooth_relu, :106-118), integrated by
// FeasibilityRecovery.Ruge_Kuta (Functions.py:1743-1781): M = 4 RK4 sub-steps of TS/M with the command
// held, all in fp64 as CasADi's SX evaluation is.
//
// One lane owns one trajectory for the whole horizon: its 5 states stay in VGPRs across the S steps
// and 4·S right-hand sides; HBM sees the command (8 B) in and the state (40 B) out per step. Each
// right-hand side is ~500 fp64-path VALU instructions (3 logs, 2 exps, 2 square roots, 5 divisions, all
// software sequences; constant divisors are folded into reciprocal products) — the kernel is bound by
// VALU issue, not by HBM (48 B per 16 right-hand sides).
//
// The algebra of the deformation force is regrouped so one log of the height ratio feeds every power:
//   r = H0/h1, e = log r, r^A = exp(A e), H0/h1 · W0/w1 = r / r^A,
//   e^M2 · ė^M3 · exp(M1 T) · exp(M4/e) = exp(M1 T + M2 log e + M3 log ė + M4/e)
// (ė = 0 -> log ė = -inf -> exp(-inf) = 0 = 0^M3, as the reference); results agree with the literal
// restatement (oracle/plant_np.py) to a few ulp per step.
#pragma once
#include <hip/hip_runtime.h>

namespace fcr {
namespace plant {

constexpr double kPi = 3.14159265358979323846;
constexpr double M_MASS = 90000.0, B_DAMP = 25000.0, FT = 200000.0;   // Functions.py:1636-1643
constexpr double D1 = 0.6, D2 = 0.5, G = 9.81;
constexpr double A1 = kPi * D1 * D1 / 4, A2 = kPi * D2 * D2 / 4;
constexpr double KB = 22e9, V1_0 = 0.3, V2_0 = 0.1, KL_1 = 8e-13, KL_2 = 14e-14;   // :1646-1650
constexpr double CD = 0.63, RHO = 858.0, D = 0.006;                           // :1653-1655
constexpr double PS = 32e6, PT = 101325.0;                                    // :1660-1661
constexpr double MU = 0.3, K = 1.115, W0 = 0.2, H0 = 0.5, B0 = 0.1;          // :1664-1668
constexpr double A = 0.14 + 0.36 * (B0 / W0) - 0.054 * (B0 / W0) * (B0 / W0);   // :1671
constexpr double T_DEF = 900.0, T1 = 0.005;                                   // :1677, :1680
constexpr double M0 = 1200e6, M1 = -0.0025, M2 = -0.0587, M3 = 0.1165, M4 = -0.0065;   // :1691-1695
constexpr double kSmoothEps = 1e-6;                                           // template_model.py:113
constexpr double kFlowC = kPi * D * CD;                                       // q = kFlowC·z·sqrt(2|a|/RHO)·sign(a)
constexpr double kTwoOverRho = 2.0 / RHO;
constexpr double kPress1 = 3 * kPi * D1 * D1 / 4, kPress2 = kPi * D2 * D2 / 2;

// xdot = f(x, u), Functions.py:1633-1738 (SMOOTH: template_model.py:116-139)
template <bool SMOOTH>
__device__ __forceinline__ void forging_rhs(const double (&x)[5], double u, double (&f)[5]) {
    const double y = x[0], yd = x[1], z = x[4];
    double p1 = x[2], p2 = x[3];
    if (SMOOTH) {
        p1 = 0.5 * (p1 + sqrt(p1 * p1 + kSmoothEps));
        p2 = 0.5 * (p2 + sqrt(p2 * p2 + kSmoothEps));
    }
    // Fd_article = if_else(y > 0 && y_dot >= 0, Kd·Ad·M0·exp(M1 T)·e^M2·ė^M3·exp(M4/e), 0)   :1698-1704
    double fd = 0.0;
    if (y > 0.0 && yd >= 0.0) {
        const double rh = 1.0 / (H0 - y);                    // 1/h1
        const double r = H0 * rh;                            // H0/h1
        const double e = log(r);                             // strain, :1698
        const double ra = exp(A * e);                        // (H0/h1)^A
        const double w1 = W0 * ra;                           // :1673
        const double b1 = B0 * (1.0 + 0.67 * (r / ra - 1.0));   // :1674
        // Kd = K (1 + MU b1/(2y) + y/(4 b1)) over one division, :1686
        const double kd = K * (1.0 + (2.0 * MU * b1 * b1 + y * y) / (4.0 * y * b1));
        const double ad = w1 * b1;                           // :1687
        const double ed = yd * rh;                           // e_dot, :1699
        fd = kd * ad * M0 * exp(M1 * T_DEF + M2 * log(e) + M3 * log(ed) + M4 / e);
    }
    // servo-valve flows, :1709-1719: the spool direction picks the pressure differences
    const bool work = z >= 0.0;
    const double apb = work ? PS - p1 : p1 - PT;
    const double aat = work ? p2 - PT : PS - p2;
    const double qpb = kFlowC * z * copysign(sqrt(kTwoOverRho * fabs(apb)), apb);
    const double qat = kFlowC * z * copysign(sqrt(kTwoOverRho * fabs(aat)), aat);
    const double v1 = V1_0 / 2 + A1 * y;                     // :1722-1723
    const double v2 = V2_0 / 2 - A2 * y;
    const double ft = fabs(yd) <= 0.5 ? FT * yd / 0.5 : FT;  // :1726
    f[0] = yd;                                               // :1729-1733
    f[1] = (kPress1 * p1 - kPress2 * p2 - B_DAMP * yd - ft - fd) * (1.0 / M_MASS) + G;
    f[2] = KB / v1 * (qpb * (1.0 / 3.0) - A1 * yd - KL_1 * p1);
    f[3] = KB / v2 * (-0.5 * qat + A2 * yd - KL_2 * p2);
    f[4] = (u - z) * (1.0 / T1);
}

// One TS step of Ruge_Kuta (Functions.py:1758-1776): `substeps` RK4 stages of dt = TS/substeps.
template <bool SMOOTH>
__device__ __forceinline__ void rk4_step(double (&x)[5], double u, double dt, int substeps) {
    for (int m = 0; m < substeps; ++m) {
        double k1[5], k2[5], k3[5], k4[5], xs[5];
        forging_rhs<SMOOTH>(x, u, k1);
#pragma unroll
        for (int i = 0; i < 5; ++i) xs[i] = x[i] + dt / 2 * k1[i];
        forging_rhs<SMOOTH>(xs, u, k2);
#pragma unroll
        for (int i = 0; i < 5; ++i) xs[i] = x[i] + dt / 2 * k2[i];
        forging_rhs<SMOOTH>(xs, u, k3);
#pragma unroll
        for (int i = 0; i < 5; ++i) xs[i] = x[i] + dt * k3[i];
        forging_rhs<SMOOTH>(xs, u, k4);
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = x[i] + dt / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
    }
}

constexpr int kPlantBlock = 256;

// x (B, S+1, 5): x[b, 0] = x0[b], x[b, t+1] = F(x[b, t], u[b, t]) for u (B, S)
template <bool SMOOTH>
__global__ __launch_bounds__(kPlantBlock) void plant_rk4_kernel(int B, int S, double dt, int substeps,
                                                                const double *__restrict__ x0,
                                                                const double *__restrict__ u,
                                                                double *__restrict__ xo) {
    const int b = blockIdx.x * kPlantBlock + threadIdx.x;
    if (b >= B) return;
    double x[5];
    double *o = xo + (size_t)b * (S + 1) * 5;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        x[i] = x0[(size_t)b * 5 + i];
        o[i] = x[i];
    }
    const double *ub = u + (size_t)b * S;
    double un = S > 0 ? ub[0] : 0.0;
    for (int t = 0; t < S; ++t) {
        const double ut = un;
        if (t + 1 < S) un = ub[t + 1];                       // next command in flight during the step
        rk4_step<SMOOTH>(x, ut, dt, substeps);
        o += 5;
#pragma unroll
        for (int i = 0; i < 5; ++i) o[i] = x[i];
    }
}

}  // namespace plant
}  // namespace fcr

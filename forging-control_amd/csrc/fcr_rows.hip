// fcr_rows.hip — C ABI of the SURVEY.md §8(f) rows that need no rollout state: the batched press plant
// (fcr_plant.h), the controller + press closed loop (fcr_closed_loop.h) and the training-window gather
// (fcr_window.h). Validation before any device call; stream-ordered launches; no allocation.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fcr.h"
#include "fcr_closed_loop.h"
#include "fcr_host.h"
#include "fcr_plant.h"
#include "fcr_window.h"

using namespace fcr;

extern "C" {

int fcr_plant_rk4(int32_t B, int32_t S, double ts, int32_t substeps, int32_t smooth, const double *x0,
                  const double *u, double *x, void *stream) {
    if (B < 0 || S < 0) return fail(FCR_EINVAL, "fcr_plant_rk4: B=%d, S=%d must be >= 0", B, S);
    if (substeps < 1 || substeps > 4096) return fail(FCR_EINVAL, "fcr_plant_rk4: substeps=%d must be 1..4096", substeps);
    if (!(ts > 0.0) || ts > 1e6) return fail(FCR_EINVAL, "fcr_plant_rk4: ts=%g must be a positive time step", ts);
    if (smooth != 0 && smooth != 1) return fail(FCR_EINVAL, "fcr_plant_rk4: smooth=%d must be 0 or 1", smooth);
    if ((long long)B * (S + 1) * 5 > (1LL << 40)) return fail(FCR_EINVAL, "fcr_plant_rk4: B*(S+1) too large");
    if (B == 0) return FCR_OK;
    if (!x0 || !x || (S > 0 && !u)) return fail(FCR_EINVAL, "fcr_plant_rk4: a required pointer is NULL");
    if ((((uintptr_t)x0) | ((uintptr_t)u) | ((uintptr_t)x)) & 7)
        return fail(FCR_EINVAL, "fcr_plant_rk4: buffers must be 8-byte aligned (fp64)");
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((B + plant::kPlantBlock - 1) / plant::kPlantBlock);
    const double dt = ts / substeps;
    if (smooth)
        hipLaunchKernelGGL(plant::plant_rk4_kernel<true>, grid, dim3(plant::kPlantBlock), 0, s, B, S, dt, substeps, x0, u, x);
    else
        hipLaunchKernelGGL(plant::plant_rk4_kernel<false>, grid, dim3(plant::kPlantBlock), 0, s, B, S, dt, substeps, x0, u, x);
    return launch_check("plant_rk4_kernel");
}

int fcr_window_gather(const fcr_windows *t, int32_t B, const int64_t *idx, float *x, float *y, float *z,
                      int32_t *bad, void *stream) {
    if (!t) return fail(FCR_EINVAL, "fcr_window_gather: tables is NULL");
    if (t->rows < 1 || t->traj_len < 1 || t->rows % t->traj_len)
        return fail(FCR_EINVAL, "fcr_window_gather: rows=%lld must be a positive multiple of traj_len=%d",
                    (long long)t->rows, t->traj_len);
    if (t->lookback < 1 || t->lookback > 4096) return fail(FCR_EINVAL, "fcr_window_gather: lookback=%d must be 1..4096", t->lookback);
    if (t->nx < 0 || t->ny < 0 || t->nz < 0 || t->nx > 4096 || t->ny > 4096 || t->nz > 4096)
        return fail(FCR_EINVAL, "fcr_window_gather: feature counts %d/%d/%d must be 0..4096", t->nx, t->ny, t->nz);
    if (B < 0) return fail(FCR_EINVAL, "fcr_window_gather: B=%d must be >= 0", B);
    if ((t->nx && !t->X) || (t->ny && !t->Y) || (t->nz && !t->Z) || !bad ||
        (B && (!idx || (t->nx && !x) || (t->ny && !y) || (t->nz && !z))))
        return fail(FCR_EINVAL, "fcr_window_gather: a required pointer is NULL");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(bad, 0, sizeof(int32_t), s) != hipSuccess) return fail(FCR_EHIP, "hipMemsetAsync failed");
    const long long per = t->nx + t->ny + (long long)t->lookback * t->nz;
    if (B == 0 || per == 0) return FCR_OK;
    window::WinArgs a{t->X, t->Y, t->Z, (long long)t->rows, t->traj_len, t->lookback, t->nx, t->ny, t->nz,
                      B, (const long long *)idx, x, y, z, bad};
    const long long n = (long long)B * per;
    if (n > (1LL << 40)) return fail(FCR_EINVAL, "fcr_window_gather: batch too large");
    hipLaunchKernelGGL(window::window_gather_kernel, dim3((unsigned)((n + window::kWinBlock - 1) / window::kWinBlock)),
                       dim3(window::kWinBlock), 0, s, a);
    return launch_check("window_gather_kernel");
}

int fcr_closed_loop_run(const fcr_closed_loop *c, void *stream) {
    if (!c) return fail(FCR_EINVAL, "fcr_closed_loop_run: args is NULL");
    if (c->B < 0 || c->T < 0) return fail(FCR_EINVAL, "fcr_closed_loop_run: B=%d, T=%d must be >= 0", c->B, c->T);
    if (c->substeps < 1 || c->substeps > 4096) return fail(FCR_EINVAL, "fcr_closed_loop_run: substeps=%d must be 1..4096", c->substeps);
    if (!(c->ts > 0.0) || c->ts > 1e6) return fail(FCR_EINVAL, "fcr_closed_loop_run: ts=%g must be a positive time step", c->ts);
    if (c->smooth != 0 && c->smooth != 1) return fail(FCR_EINVAL, "fcr_closed_loop_run: smooth=%d must be 0 or 1", c->smooth);
    if (c->ctrl_hidden < 1 || c->ctrl_hidden > closed_loop::kClMaxHidden)
        return fail(FCR_EUNSUPPORTED, "fcr_closed_loop_run: ctrl_hidden=%d: built for 1..%d", c->ctrl_hidden,
                    closed_loop::kClMaxHidden);
    if (!(c->in_scale[0] > 0.0) || !(c->in_scale[1] > 0.0) || !(c->ref_scale > 0.0) || !(c->out_scale > 0.0))
        return fail(FCR_EINVAL, "fcr_closed_loop_run: scaler scales must be positive");
    if (c->B == 0) return FCR_OK;
    if (!c->x0 || !c->x || !c->ctrl_w_inp || !c->ctrl_b_inp || !c->ctrl_w_out || (c->T > 0 && (!c->ref || !c->u)))
        return fail(FCR_EINVAL, "fcr_closed_loop_run: a required pointer is NULL");
    if ((((uintptr_t)c->x0) | ((uintptr_t)c->ref) | ((uintptr_t)c->x) | ((uintptr_t)c->u)) & 7)
        return fail(FCR_EINVAL, "fcr_closed_loop_run: fp64 buffers must be 8-byte aligned");
    closed_loop::ClArgs a{c->B, c->T, c->substeps, c->ctrl_hidden, c->ts / c->substeps, c->x0, c->ref,
                          c->ctrl_w_inp, c->ctrl_b_inp, c->ctrl_w_out, c->in_scale[0], c->in_scale[1],
                          c->ref_scale, c->out_scale, c->x, c->u};
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((c->B + closed_loop::kClBlock - 1) / closed_loop::kClBlock);
    if (c->smooth)
        hipLaunchKernelGGL(closed_loop::closed_loop_kernel<true>, grid, dim3(closed_loop::kClBlock), 0, s, a);
    else
        hipLaunchKernelGGL(closed_loop::closed_loop_kernel<false>, grid, dim3(closed_loop::kClBlock), 0, s, a);
    return launch_check("closed_loop_kernel");
}

}  // extern "C"

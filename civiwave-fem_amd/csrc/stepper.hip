// stepper.hip -- node-wise Newmark phases of cwf::gpu::newmark::Stepper (CPU branch semantics,
// src/gpu/newmark_stepper.cpp:1162-1314). fp64 math on f32 state, rounded exactly where the
// reference rounds; compiled with -ffp-contract=off so the parity mode stays bit-exact.
#include "cwf_internal.hpp"

namespace cwf
{
namespace
{
constexpr int kBlock = 256;
inline unsigned grid_for(uint32_t n) { return (n + kBlock - 1) / kBlock; }

// write_predictor (:1245-1286): u~ = (u + dt v) + ((0.5-beta) dt^2) a ; v~ = v + ((1-gamma) dt) a
__global__ __launch_bounds__(kBlock) void k_predictor(uint32_t D, const float *__restrict__ u,
                                                      const float *__restrict__ v, const float *__restrict__ a,
                                                      float *__restrict__ up, float *__restrict__ vp, double dt,
                                                      double dt_sq, double disp_factor, double vel_factor)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= D)
        return;
    const double uu = u[i], vv = v[i], aa = a[i];
    up[i] = (float)(uu + dt * vv + disp_factor * dt_sq * aa);
    vp[i] = (float)(vv + vel_factor * dt * aa);
}

// assemble_rhs node loop (:1174-1198)
__global__ __launch_bounds__(kBlock) void k_assemble_rhs(uint32_t N, const float *__restrict__ mass,
                                                         const float *__restrict__ u, const float *__restrict__ v,
                                                         const float *__restrict__ a, const float *__restrict__ f,
                                                         float *__restrict__ rhs, float *__restrict__ damp, double a0,
                                                         double a1, double a2, double a3, double a4, double a5,
                                                         double ralpha)
{
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= N)
        return;
    const double m = (double)mass[n];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const uint32_t i = 3u * n + k;
        const double uu = u[i], vv = v[i], aa = a[i];
        const double mass_term = m * (a0 * uu + a2 * vv + a3 * aa);
        const double damping_term = a1 * uu + a4 * vv + a5 * aa;
        const double force = (double)f[i];
        const double total = force + mass_term + ralpha * m * damping_term;
        rhs[i] = (float)total;
        damp[i] = (float)damping_term;
    }
}

// rhs += f32(beta_R) * (K d) in f32 (:1210-1213)
__global__ __launch_bounds__(kBlock) void k_rhs_damping(uint32_t D, float *__restrict__ rhs,
                                                        const float *__restrict__ kd, float bf)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= D)
        return;
    rhs[i] = rhs[i] + bf * kd[i];
}

// clamp_dirichlet_rhs (:1219-1243): rhs_c = bc_value_c - u_c (f32)
__global__ __launch_bounds__(kBlock) void k_clamp(uint32_t N, const uint32_t *__restrict__ mask,
                                                  const float *__restrict__ bcv, const float *__restrict__ u,
                                                  float *__restrict__ rhs)
{
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= N)
        return;
    const uint32_t mk = mask[n];
    if (mk == 0u)
        return;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (mk & (1u << k))
            rhs[3u * n + k] = bcv[3u * n + k] - u[3u * n + k];
}

// apply_state_update (:1288-1314), f32
__global__ __launch_bounds__(kBlock) void k_state_update(uint32_t D, const float *__restrict__ x,
                                                         const float *__restrict__ up,
                                                         const float *__restrict__ vp, float *__restrict__ u,
                                                         float *__restrict__ v, float *__restrict__ a, float ib,
                                                         float gob)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= D)
        return;
    const float dx = x[i];
    u[i] = up[i] + dx;
    a[i] = ib * dx;
    v[i] = vp[i] + gob * dx;
}

// external_force = safe_cast(base + scale * pattern) (loads.cpp:87-174 with one curve-scaled load pattern,
// then pack.cpp:41-57): the per-step rewrite of nodes.external_force the viewer does on the host
// (viewer.cpp:262-266), on the device
__global__ __launch_bounds__(kBlock) void k_scaled_load(uint32_t D, const double *__restrict__ base,
                                                        const double *__restrict__ pattern, double scale,
                                                        float *__restrict__ f)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= D)
        return;
    const double v = base[i] + scale * pattern[i];
    const double fmax = 3.4028234663852886e38;  // FLT_MAX
    float out;
    if (!isfinite(v))
        out = v > 0.0 ? __int_as_float(0x7f800000) : v < 0.0 ? __int_as_float((int)0xff800000u) : __int_as_float(0x7fc00000);
    else if (v > fmax)
        out = 3.4028234663852886e38f;
    else if (v < -fmax)
        out = -3.4028234663852886e38f;
    else
        out = (float)v;
    f[i] = out;
}
}  // namespace

void stepper_predictor(uint32_t D, const float *u, const float *v, const float *a, float *up, float *vp, double dt,
                       double beta, double gamma, hipStream_t st)
{
    if (!D)
        return;
    const double dt_sq = dt * dt;
    k_predictor<<<grid_for(D), kBlock, 0, st>>>(D, u, v, a, up, vp, dt, dt_sq, 0.5 - beta, 1.0 - gamma);
}

void stepper_assemble_rhs(uint32_t N, const float *mass, const float *u, const float *v, const float *a,
                          const float *f, float *rhs, float *damp, const double *c6, double ralpha, hipStream_t st)
{
    if (!N)
        return;
    k_assemble_rhs<<<grid_for(N), kBlock, 0, st>>>(N, mass, u, v, a, f, rhs, damp, c6[0], c6[1], c6[2], c6[3],
                                                   c6[4], c6[5], ralpha);
}

void stepper_rhs_damping(uint32_t D, float *rhs, const float *kd, float bf, hipStream_t st)
{
    if (D)
        k_rhs_damping<<<grid_for(D), kBlock, 0, st>>>(D, rhs, kd, bf);
}

void stepper_clamp(uint32_t N, const uint32_t *mask, const float *bcv, const float *u, float *rhs, hipStream_t st)
{
    if (N)
        k_clamp<<<grid_for(N), kBlock, 0, st>>>(N, mask, bcv, u, rhs);
}

void stepper_update(uint32_t D, const float *x, const float *up, const float *vp, float *u, float *v, float *a,
                    float ib, float gob, hipStream_t st)
{
    if (D)
        k_state_update<<<grid_for(D), kBlock, 0, st>>>(D, x, up, vp, u, v, a, ib, gob);
}

void stepper_scaled_load(uint32_t D, const double *base, const double *pattern, double scale, float *f, hipStream_t st)
{
    if (D)
        k_scaled_load<<<grid_for(D), kBlock, 0, st>>>(D, base, pattern, scale, f);
}

}  // namespace cwf

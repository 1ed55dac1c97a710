// spmv_tiles.hip -- FAST-mode K_eff and the fused FAST PCG iteration (2 kernels / iteration).
//
// k_keff_tiles_pipe (the default; persistent, XCD-aware, software-pipelined; tiles of <= 2 NT
// Morton-ordered tets and <= NT nodes):
//   a) tile-node phase: the node's coordinates and value go to LDS: x (apply_keff) or, inside PCG, the new
//      search direction p = z + beta p_old formed on the fly (the p-update pass of pcg.cpp:897-914 is
//      fused here); the next tile's records are already in flight;
//   b) element phase: 8-B corner-id records, gradients and volume recomputed from the tile-relative
//      coordinates (cofactor rows, one stress scale), fp32 strain -> stress -> 12 nodal forces, each
//      corner's 3 forces pushed to its position in the tile's local CSR (epos);
//   c) fold phase: every tile node sums its contiguous run (ascending element, deterministic, no atomics)
//      and stores a 12-B partial at its node-major slot; PCG adds the tile's fp64 share of p.Ap.
// k_keff_tiles: one workgroup per tile, 48-B gradient records and a local-CSR fold; the path for meshes
//   without coordinates that reproduce their gradients.
// k_keff_hex_tiles (hex8_tiles.inc): the native hex8 element on the same tile machinery.
// k_keff_finalize (apply_keff): y = node's partials (ascending tile) + m s_M x, Dirichlet identity rows.
// k_pcg_update_tiles (PCG, 256-thread workgroups, resident grid-stride): Ap from the node-major partials
//   (never stored), the same p expression, x += alpha p, r -= alpha Ap, Dirichlet, z = M^-1 r, store
//   x r z p, fp64 r.r / r.z shares.
// Scalars without atomics or fences: every consumer workgroup folds the producer's partials itself in a
// fixed order (alpha in the update kernel, |r| / convergence / beta in the tiles-kernel preamble,
// pcg.cpp:840-895); the host passes the iteration index and rho is double-buffered by parity, so no
// device scalar is read after being written inside one kernel.
#include <algorithm>

#include <hip/hip_ext.h>

#include "blockinv_pack.hpp"
#include "cwf_internal.hpp"
#include "lattice_common.hpp"
#include "reduce.hpp"

namespace cwf
{
namespace
{
constexpr int kMaxM = 16;
#ifndef CWF_UPD_THREADS
#define CWF_UPD_THREADS 256
#endif
constexpr int kUpdThreads = CWF_UPD_THREADS;  // update-pass workgroup size (its per-workgroup shares are refolded by every consumer workgroup)
constexpr unsigned kMaxUpdateBlocks = 2048;  // 8 resident per CU (grid-stride beyond); <= 2048 shares to fold

// buffer descriptor over a whole allocation (base pointer wave-uniform: a kernel argument)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t whole_rsrc(const void *base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, -1, 0x00020000);
}

// 12-B store at float index 3 q; wt: write-through (sc1), so the line leaves L2 during the kernel instead of
// in the end-of-kernel write-back the next launch waits for (the update pass's x / r / z: C2 +2.7% PCG it/s,
// C3 neutral, same-box A/B; the tiles kernel's scattered partial / p stores measured 5% slower that way)
// (one buffer_store_dwordx3 either way; base: the buffer the descriptor covers)
__device__ __forceinline__ void store3(float *base, __amdgpu_buffer_rsrc_t rs, uint64_t q, float a, float b, float c,
                                       bool wt)
{
    (void)base;
    const u32x3 v = {__float_as_uint(a), __float_as_uint(b), __float_as_uint(c)};
    if (wt)
        __builtin_amdgcn_raw_buffer_store_b96(v, rs, (uint32_t)(12ull * q), 0, 16);
    else
        __builtin_amdgcn_raw_buffer_store_b96(v, rs, (uint32_t)(12ull * q), 0, 0);
}

// pcg.cpp:862-895 for iteration `it` >= 1 from the update kernel's r.r / r.z shares (stride 1), or
// from the all-gathered per-rank {r.r, r.z} pairs of a sharded system (stride 2, rank order).
// Returns false when the solve is over (converged or rho breakdown); *beta_out = beta for this iteration. pre: the
// control words prefetched by the caller (ctl_prefetch); then !pre->active (tested after the fold) also returns false.
template <int NT, int B = 4>
__device__ __forceinline__ bool residual_step(Ctl *ctl, const double *__restrict__ prr, const double *__restrict__ prz,
                                              unsigned nparts, unsigned stride, unsigned it,
                                              double *__restrict__ hist, double *red, float *beta_out,
                                              bool dry = false, const CtlPre *pre = nullptr)
{
    if (it == 0)
    {
        *beta_out = 0.f;
        return pre ? pre->active != 0 : true;
    }
    double rr, rz;
    fold_all2<NT, B>(prr, prz, nparts, red, stride, rr, rz);
    if (pre && !pre->active)
        return false;
    const double res = sqrt(rr);
    const double rho_old = pre ? pre->rho_old : ctl->rho2[(it - 1) & 1u];
    const bool conv = res <= (pre ? pre->tol : ctl->tol);
    const bool err = !conv && fabs(rho_old) < 1.0e-18;
    const double beta = (conv || err) ? 0.0 : rz / rho_old;
    if (dry)  // diagnostic timing: full work, no side effects
    {
        *beta_out = (float)beta;
        return true;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
    {
        ctl->res = res;
        ctl->iterations = it;
        hist[it] = res;
        if (conv)
        {
            ctl->converged = 1;
            ctl->active = 0;
        }
        else if (err)
        {
            ctl->error = CWF_ERR_RHO_ZERO;
            ctl->error_iter = (int)it - 1;
            ctl->active = 0;
        }
        else
        {
            ctl->rho2[it & 1u] = rz;
            ctl->beta = beta;
            ctl->beta_last = beta;
        }
    }
    *beta_out = (float)beta;
    return !(conv || err);
}

template <bool ISO>
__device__ __forceinline__ void stress_f32(const float *Dm, const float e[6], float s[6])
{
    if constexpr (ISO)
    {
#pragma unroll
        for (int r = 0; r < 3; ++r)
            s[r] = fmaf(Dm[3 * r + 2], e[2], fmaf(Dm[3 * r + 1], e[1], Dm[3 * r] * e[0]));
#pragma unroll
        for (int r = 3; r < 6; ++r)
            s[r] = Dm[6 + r] * e[r];
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 6; ++r)
        {
            float sum = 0.0f;
#pragma unroll
            for (int c = 0; c < 6; ++c)
                sum = fmaf(Dm[6 * r + c], e[c], sum);
            s[r] = sum;
        }
    }
}

__device__ __forceinline__ uint32_t dsrc(bool iso, uint32_t t)
{
    return iso ? (t < 9 ? (t / 3) * 6 + (t % 3) : (t - 6) * 7) : t;
}

// value of one tile node: x (apply, optionally sanitised) or p_new = z + beta p_old (PCG)
template <bool SANITIZE, int MODE>
__device__ __forceinline__ void gather_node(const DevSys &s, const float *__restrict__ x, const float *__restrict__ z,
                                            float beta, uint32_t g, float u[3])
{
    if constexpr (MODE == 1)
    {
        // constrained dofs stay 0 (z_c = 0, p_c = 0)
        u[0] = fmaf(beta, x[3u * g + 0], z[3u * g + 0]);
        u[1] = fmaf(beta, x[3u * g + 1], z[3u * g + 1]);
        u[2] = fmaf(beta, x[3u * g + 2], z[3u * g + 2]);
    }
    else
    {
        u[0] = x[3u * g + 0];
        u[1] = x[3u * g + 1];
        u[2] = x[3u * g + 2];
        if constexpr (SANITIZE)
        {
            const uint32_t mk = s.mask[g];
            u[0] = (mk & 1u) ? 0.f : u[0];
            u[1] = (mk & 2u) ? 0.f : u[1];
            u[2] = (mk & 4u) ? 0.f : u[2];
        }
    }
}

// strain -> stress -> 12 nodal forces of one tet from its corner gradients g[12] (corner-major xyz), its
// local corner ids and V s_K; corner values from LDS, forces stored to LDS as f[12][kTileElems]
// (fp32 counterpart of pcg.cpp:140-220)
template <bool ISO>
__device__ __forceinline__ void element_force_values(const DevSys &s, const float g[12], const uint32_t li[4], float vol,
                                                     uint32_t mi, const float *sp, uint32_t ms, const float *dtab,
                                                     float f[12])
{
    constexpr int kTab = ISO ? 12 : 36;
    float eps[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 4; ++a)
    {
        const float u0 = sp[li[a]], u1 = sp[ms + li[a]], u2 = sp[2 * ms + li[a]];
        const float gx = g[3 * a], gy = g[3 * a + 1], gz = g[3 * a + 2];
        eps[0] = fmaf(gx, u0, eps[0]);
        eps[1] = fmaf(gy, u1, eps[1]);
        eps[2] = fmaf(gz, u2, eps[2]);
        eps[3] = fmaf(gx, u1, fmaf(gy, u0, eps[3]));
        eps[4] = fmaf(gy, u2, fmaf(gz, u1, eps[4]));
        eps[5] = fmaf(gx, u2, fmaf(gz, u0, eps[5]));
    }
    float sig[6];
    if (mi < (uint32_t)kMaxM)
        stress_f32<ISO>(dtab + kTab * mi, eps, sig);
    else
    {
        float tab[36];
        for (int t = 0; t < kTab; ++t)
            tab[t] = (float)s.dmat[36u * mi + dsrc(ISO, t)];
        stress_f32<ISO>(tab, eps, sig);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
    {
        const float ax = g[3 * a], ay = g[3 * a + 1], az = g[3 * a + 2];
        f[3 * a + 0] = vol * fmaf(az, sig[5], fmaf(ay, sig[3], ax * sig[0]));
        f[3 * a + 1] = vol * fmaf(az, sig[4], fmaf(ax, sig[3], ay * sig[1]));
        f[3 * a + 2] = vol * fmaf(ax, sig[5], fmaf(ay, sig[4], az * sig[2]));
    }
}

template <bool ISO>
__device__ __forceinline__ void element_forces(const DevSys &s, const float g[12], const uint32_t li[4], float vol,
                                               uint32_t mi, uint32_t j, const float *sp, uint32_t ms,
                                               const float *dtab, float *sf)
{
    float f[12];
    element_force_values<ISO>(s, g, li, vol, mi, sp, ms, dtab, f);
#pragma unroll
    for (int c = 0; c < 12; ++c)
        sf[c * kTileElems + j] = f[c];
}

// 48-B record {idx01, idx23, g0x, g0y}{g0z g1x g1y g1z}{g2x g2y g2z vol}: gradients as stored
__device__ __forceinline__ void record_geometry(uint4 q0, uint4 q1, uint4 q2, float g[12], uint32_t li[4], float *vol)
{
    g[0] = __uint_as_float(q0.z);
    g[1] = __uint_as_float(q0.w);
    g[2] = __uint_as_float(q1.x);
    g[3] = __uint_as_float(q1.y);
    g[4] = __uint_as_float(q1.z);
    g[5] = __uint_as_float(q1.w);
    g[6] = __uint_as_float(q2.x);
    g[7] = __uint_as_float(q2.y);
    g[8] = __uint_as_float(q2.z);
    g[9] = -(g[0] + g[3] + g[6]);
    g[10] = -(g[1] + g[4] + g[7]);
    g[11] = -(g[2] + g[5] + g[8]);
    li[0] = q0.x & 0xffffu;
    li[1] = q0.x >> 16;
    li[2] = q0.y & 0xffffu;
    li[3] = q0.y >> 16;
    *vol = __uint_as_float(q2.w);
}

// on-the-fly geometry of a linear tet from its corner coordinates (tile-relative f32, staged in LDS):
// with edge columns c_k = x_k - x_0, the rows of [c1 c2 c3]^-1 are the gradients of N_1..N_3
// (r1 = c2 x c3 / det, r2 = c3 x c1 / det, r3 = c1 x c2 / det), grad N_0 = -(r1 + r2 + r3) and
// V = |det| / 6 -- the quantities preprocess.cpp:284-379 tabulates, recomputed instead of streamed
__device__ __forceinline__ void coord_geometry(uint2 id, const float *sx, uint32_t ms, float g[12], uint32_t li[4],
                                               float *vol)
{
    li[0] = id.x & 0xffffu;
    li[1] = id.x >> 16;
    li[2] = id.y & 0xffffu;
    li[3] = id.y >> 16;
    float c[3][3];  // c[k] = x_{k+1} - x_0
    const float x0 = sx[li[0]], y0 = sx[ms + li[0]], z0 = sx[2 * ms + li[0]];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        c[k][0] = sx[li[k + 1]] - x0;
        c[k][1] = sx[ms + li[k + 1]] - y0;
        c[k][2] = sx[2 * ms + li[k + 1]] - z0;
    }
    float r[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const float *u = c[(k + 1) % 3], *v = c[(k + 2) % 3];
        r[k][0] = u[1] * v[2] - u[2] * v[1];
        r[k][1] = u[2] * v[0] - u[0] * v[2];
        r[k][2] = u[0] * v[1] - u[1] * v[0];
    }
    const float det = c[0][0] * r[0][0] + c[0][1] * r[0][1] + c[0][2] * r[0][2];
    const float inv = 1.0f / det;
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        g[3 * (k + 1) + 0] = r[k][0] * inv;
        g[3 * (k + 1) + 1] = r[k][1] * inv;
        g[3 * (k + 1) + 2] = r[k][2] * inv;
    }
    g[0] = -(g[3] + g[6] + g[9]);
    g[1] = -(g[4] + g[7] + g[10]);
    g[2] = -(g[5] + g[8] + g[11]);
    *vol = fabsf(det) * (1.0f / 6.0f);
}

struct PcgArgs
{
    const float *z;           // z (PCG); x holds p_old
    Ctl *ctl;
    double *part_dot;         // out: per-tile p.Ap share
    const double *prr, *prz;  // in: folded {r.r, r.z} of the previous update (per rank)
    unsigned nupd;
    unsigned stride;
    unsigned it;
    double *hist;
    unsigned abl;  // diagnostic ablation bits (ablate(); the dry-run bit 32), 0 in solves
    float *pnew;   // out (PCG): the owner slot of every tile node stores the new p = z + beta p_old here
};

// Ablation bits (tools/ablate.py): phases of the tiles kernels skipped for diagnostic timing. They are compiled
// in only by the ablation build (make ABLATION=1, -DCWF_ABLATION=1); release kernels test a constant 0. Bit 32
// (a side-effect-free residual step, the dry timing of cwf_hip_keff_timed) is not a phase and stays live.
#ifndef CWF_ABLATION
#define CWF_ABLATION 0
#endif
__device__ __forceinline__ bool ablate(const PcgArgs &pa, unsigned bit) { return CWF_ABLATION && (pa.abl & bit); }

// Pipelined-kernel element body (GEO). With edge columns c_k = x_k - x_0 and r_k their cofactor rows
// (r_1 = c_2 x c_3, ...), the gradients are g_a = r_a / det and V = |det| / 6, so
//   f_a = V B(g_a)^T D B(g) u = B(r_a)^T D (sum_b B(r_b) u_b) * s_K / (6 |det|):
// the strain is built from the unscaled r_a and ONE scale lands on the 6 stresses (no per-gradient
// division, no per-force volume multiply). FAST arithmetic: FMA contractions and the hardware
// reciprocal (1 ulp), tolerance-checked against the oracle.
// the element body from register operands: corners X[a] = {x, y, z, p_x}, Q[a] = {p_y, p_z}
template <bool ISO>
__device__ __forceinline__ void tet_forces_reg(const DevSys &s, const float4 X[4], const float2 Q[4], float sK6,
                                               uint32_t mi, const float *dtab, float f[12])
{
    constexpr int kTab = ISO ? 12 : 36;
    float c[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        c[k][0] = X[k + 1].x - X[0].x;
        c[k][1] = X[k + 1].y - X[0].y;
        c[k][2] = X[k + 1].z - X[0].z;
    }
    float g[4][3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const float *u = c[(k + 1) % 3], *v = c[(k + 2) % 3];
        g[k + 1][0] = fmaf(u[1], v[2], -u[2] * v[1]);
        g[k + 1][1] = fmaf(u[2], v[0], -u[0] * v[2]);
        g[k + 1][2] = fmaf(u[0], v[1], -u[1] * v[0]);
    }
    const float det = fmaf(c[0][0], g[1][0], fmaf(c[0][1], g[1][1], c[0][2] * g[1][2]));
    const float scale = sK6 * __builtin_amdgcn_rcpf(fabsf(det));
#pragma unroll
    for (int q = 0; q < 3; ++q)
        g[0][q] = -(g[1][q] + g[2][q] + g[3][q]);
    float eps[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 4; ++a)
    {
        const float u0 = X[a].w, u1 = Q[a].x, u2 = Q[a].y;
        const float gx = g[a][0], gy = g[a][1], gz = g[a][2];
        eps[0] = fmaf(gx, u0, eps[0]);
        eps[1] = fmaf(gy, u1, eps[1]);
        eps[2] = fmaf(gz, u2, eps[2]);
        eps[3] = fmaf(gx, u1, fmaf(gy, u0, eps[3]));
        eps[4] = fmaf(gy, u2, fmaf(gz, u1, eps[4]));
        eps[5] = fmaf(gx, u2, fmaf(gz, u0, eps[5]));
    }
    float sig[6];
    if (s.M == 1)  // uniform branch: D from the kernel arguments (SGPR operands, no LDS reads)
        stress_f32<ISO>(s.d1, eps, sig);
    else if (mi < (uint32_t)kMaxM)
        stress_f32<ISO>(dtab + kTab * mi, eps, sig);
    else
    {
        float tab[36];
        for (int t = 0; t < kTab; ++t)
            tab[t] = (float)s.dmat[36u * mi + dsrc(ISO, t)];
        stress_f32<ISO>(tab, eps, sig);
    }
#pragma unroll
    for (int r = 0; r < 6; ++r)
        sig[r] *= scale;
#pragma unroll
    for (int a = 0; a < 4; ++a)
    {
        const float ax = g[a][0], ay = g[a][1], az = g[a][2];
        f[3 * a + 0] = fmaf(az, sig[5], fmaf(ay, sig[3], ax * sig[0]));
        f[3 * a + 1] = fmaf(az, sig[4], fmaf(ax, sig[3], ay * sig[1]));
        f[3 * a + 2] = fmaf(ax, sig[5], fmaf(ay, sig[4], az * sig[2]));
    }
}

template <bool ISO>
__device__ __forceinline__ void geo_element_forces(const DevSys &s, uint2 id, const float4 *sxp, const float2 *sq,
                                                   float sK6, uint32_t mi, const float *dtab, float f[12])
{
    const uint32_t li[4] = {id.x & 0xffffu, id.x >> 16, id.y & 0xffffu, id.y >> 16};
    // one ds_read_b128 {x, y, z, p_x} + one ds_read_b64 {p_y, p_z} per corner
    float4 X[4];
    float2 Q[4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
    {
        X[a] = sxp[li[a]];
        Q[a] = sq[li[a]];
    }
    tet_forces_reg<ISO>(s, X, Q, sK6, mi, dtab, f);
}

// MODE 0: apply (gather x, optional sanitize); MODE 1: PCG (gather z, p_old -> p_new).
// GEO: 8-B element records + per-tile-node coordinates (geometry recomputed); else 48-B records.
template <bool ISO, bool SANITIZE, int MODE, int NT, bool GEO>
__global__ __launch_bounds__(NT) void k_keff_tiles(DevSys s, const float *__restrict__ x, PcgArgs pa)
{
    constexpr int kTab = ISO ? 12 : 36;
    extern __shared__ float lds[];
    const DevTiles &T = s.t;
    const uint32_t ms = T.max_tile_nodes;
    float *sf = lds;                                                     // [12][kTileElems]
    uint16_t *sc = reinterpret_cast<uint16_t *>(lds + 12 * kTileElems);  // [4*kTileElems] local CSR
    float *sp = lds + 14 * kTileElems;                                   // [3][ms] node values
    float *sx = sp + 3 * ms;                                             // [3][ms] node coordinates (GEO)
    __shared__ float dtab[kMaxM * kTab];
    __shared__ double red[2 * (NT / 64)];
    if constexpr (MODE == 1)
    {
        if (!pa.ctl->active)
            return;
    }
    const uint4 hd = T.hdr[blockIdx.x];
    const uint32_t e0 = hd.x, ne = hd.y, nb = hd.z, nn = hd.w;
    const float sK = (float)s.sK;
    // (a) issue every load that does not depend on beta: the first tile-node record, its coordinates
    //     and value(s), the thread's element records and the tile's local CSR (staged into LDS)
    const uint32_t i0 = threadIdx.x;
    uint2 tn0 = uint2{0u, 0u};
    float v0[3] = {0.f, 0.f, 0.f}, w0[3] = {0.f, 0.f, 0.f};
    if (i0 < nn)
    {
        tn0 = T.tnode[nb + i0];
        const uint32_t g = tn0.x & 0x7fffffffu;
        v0[0] = x[3u * g + 0];
        v0[1] = x[3u * g + 1];
        v0[2] = x[3u * g + 2];
        if constexpr (MODE == 1)
        {
            w0[0] = pa.z[3u * g + 0];
            w0[1] = pa.z[3u * g + 1];
            w0[2] = pa.z[3u * g + 2];
        }
        else if constexpr (SANITIZE)
        {
            const uint32_t mk = s.mask[g];
            v0[0] = (mk & 1u) ? 0.f : v0[0];
            v0[1] = (mk & 2u) ? 0.f : v0[1];
            v0[2] = (mk & 4u) ? 0.f : v0[2];
        }
    }
    if constexpr (GEO)
    {
        const uint32_t T3 = T.total_tile_nodes;
        for (uint32_t i = threadIdx.x; i < nn; i += NT)
        {
            sx[i] = T.tcoord[nb + i];
            sx[ms + i] = T.tcoord[T3 + nb + i];
            sx[2 * ms + i] = T.tcoord[2 * T3 + nb + i];
        }
    }
    constexpr int kPer = kTileElems / NT;
    uint4 pq[kPer][GEO ? 1 : 3];
    uint2 pid[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k)
    {
        const uint32_t j = threadIdx.x + k * NT;
        const uint32_t e = e0 + (j < ne ? j : 0u);
        if constexpr (GEO)
            pid[k] = T.eid[e];
        else
        {
            const uint4 *P = T.planes;
            pq[k][0] = P[e];
            pq[k][GEO ? 0 : 1] = P[T.E + e];
            pq[k][GEO ? 0 : 2] = P[2u * T.E + e];
        }
    }
    {
        const uint2 *src = reinterpret_cast<const uint2 *>(T.csr_ent + 4ull * e0);  // 8-B aligned
        uint2 *dst = reinterpret_cast<uint2 *>(sc);
        for (uint32_t k = threadIdx.x; k < ne; k += NT)
            dst[k] = src[k];
    }
    const uint32_t nm = s.M < kMaxM ? s.M : kMaxM;
    for (uint32_t i = threadIdx.x; i < nm * kTab; i += NT)
        dtab[i] = (float)s.dmat[36u * (i / kTab) + dsrc(ISO, i % kTab)];
    float beta = 0.f;
    if constexpr (MODE == 1)
    {
        // pcg.cpp:862-895 of the previous update; its fold latency overlaps the loads above
        if (ablate(pa, 1u))
            beta = (float)pa.ctl->beta;
        else if (!residual_step<NT>(pa.ctl, pa.prr, pa.prz, pa.nupd, pa.stride, pa.it, pa.hist, red, &beta,
                                    pa.abl & 32u))
            return;
    }
    if (i0 < nn)
    {
        if constexpr (MODE == 1)
        {
            // p_new = z + beta p_old; constrained dofs stay 0 (z_c = 0, p_c = 0)
            v0[0] = fmaf(beta, v0[0], w0[0]);
            v0[1] = fmaf(beta, v0[1], w0[1]);
            v0[2] = fmaf(beta, v0[2], w0[2]);
        }
        sp[i0] = v0[0];
        sp[ms + i0] = v0[1];
        sp[2 * ms + i0] = v0[2];
    }
    for (uint32_t i = i0 + NT; i < nn; i += NT)
    {
        const uint2 tn = T.tnode[nb + i];
        float u[3];
        gather_node<SANITIZE, MODE>(s, x, pa.z, beta, tn.x & 0x7fffffffu, u);
        sp[i] = u[0];
        sp[ms + i] = u[1];
        sp[2 * ms + i] = u[2];
    }
    __syncthreads();
    // (b) elements
    if (!ablate(pa, 16u))
    {
#pragma unroll
        for (int k = 0; k < kPer; ++k)
        {
            const uint32_t j = threadIdx.x + k * NT;
            if (j < ne)
            {
                float g[12], vol;
                uint32_t li[4];
                if constexpr (GEO)
                    coord_geometry(pid[k], sx, ms, g, li, &vol);
                else
                    record_geometry(pq[k][0], pq[k][GEO ? 0 : 1], pq[k][GEO ? 0 : 2], g, li, &vol);
                element_forces<ISO>(s, g, li, vol * sK, T.mat ? T.mat[e0 + j] : 0u, j, sp, ms, dtab, sf);
            }
        }
    }
    __syncthreads();
    // (c) fold per tile node (tile-major partials: the tile's block is one contiguous store)
    double pap = 0.0;
    const float sM = (float)s.sM;
    for (uint32_t i = threadIdx.x; i < (ablate(pa, 8u) ? 0u : nn); i += NT)
    {
        const uint2 tn = i == threadIdx.x ? tn0 : T.tnode[nb + i];
        float a0 = 0.f, a1 = 0.f, a2 = 0.f;
        const uint32_t qe = tn.y >> 16;
        uint32_t q = tn.y & 0xffffu;
        // 4 independent (entry, force) LDS chains in flight; the sums stay in ascending-entry order
        for (; q + 4 <= qe; q += 4)
        {
            uint32_t ent[4];
            float f[4][3];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                ent[u] = sc[q + u];
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                const uint32_t el = ent[u] >> 2, c = 3u * (ent[u] & 3u);
                f[u][0] = sf[(c + 0) * kTileElems + el];
                f[u][1] = sf[(c + 1) * kTileElems + el];
                f[u][2] = sf[(c + 2) * kTileElems + el];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                a0 += f[u][0];
                a1 += f[u][1];
                a2 += f[u][2];
            }
        }
        for (; q < qe; ++q)
        {
            const uint32_t ent = sc[q];
            const uint32_t el = ent >> 2, c = 3u * (ent & 3u);
            a0 += sf[(c + 0) * kTileElems + el];
            a1 += sf[(c + 1) * kTileElems + el];
            a2 += sf[(c + 2) * kTileElems + el];
        }
        float *o = T.part + 3ull * (nb + i);
        o[0] = a0;
        o[1] = a1;
        o[2] = a2;
        if (MODE == 1 && pa.pnew && (tn.x & 0x80000000u))  // owner slot: the new p for the update pass
        {
            float *q = pa.pnew + 3ull * (tn.x & 0x7fffffffu);
            q[0] = sp[i];
            q[1] = sp[ms + i];
            q[2] = sp[2 * ms + i];
        }
        if (MODE == 1 && !ablate(pa, 4u) && (tn.x & 0x7fffffffu) < s.Nown)  // ghosts: another rank's row
        {
            const float p0 = sp[i], p1 = sp[ms + i], p2 = sp[2 * ms + i];
            pap += (double)fmaf(p2, a2, fmaf(p1, a1, p0 * a0));  // fp32 per node, fp64 across nodes
            if (tn.x & 0x80000000u)  // the node's owner slot adds its mass term m s_M |p|^2 once
            {
                const float m = s.mass[tn.x & 0x7fffffffu] * sM;
                pap += (double)(m * p0) * (double)p0 + (double)(m * p1) * (double)p1 +
                       (double)(m * p2) * (double)p2;
            }
        }
    }
    if constexpr (MODE == 1)
    {
        const double t = block_sum<NT>(pap, red);
        if (threadIdx.x == 0)
            pa.part_dot[blockIdx.x] = t;
    }
}

// Persistent, software-pipelined form of k_keff_tiles (GEO records, push fold; the default FAST path).
// A resident grid (occupancy x CUs) walks the tiles; while a workgroup computes tile t from LDS, the
// loads of its next tile t' (tile-node records, coordinates, corner ids, local CSR, then the z/p
// gathers) are already in flight in registers, so each tile's memory chain overlaps the previous
// tile's element and fold work instead of being exposed. Tiles are dealt XCD-contiguously (workgroup
// b runs on XCD b % 8 and walks that XCD's eighth of the Morton-ordered tiles) so neighbouring tiles,
// which share nodes, share an L2. beta (the residual step) and the material table are set up once
// per workgroup; the p.Ap share is one per workgroup.
// Sum of a node's contiguous run [q, qe) of pushed corner forces, in ascending order: {f_x, f_y} pairs
// accumulate with v_pk_add_f32 straight from ds_read2_b64 (component-wise, so the same order and
// bits as three scalar sums), f_z from its own plane.
__device__ __forceinline__ void fold_run(const float2 *sfxy, const float *sfz, uint32_t q, uint32_t qe, float &a0,
                                         float &a1, float &a2)
{
    typedef float pair_t __attribute__((ext_vector_type(2)));
    const pair_t *pxy = reinterpret_cast<const pair_t *>(sfxy);
    // runs start on even slots: two entries per step, {f_x, f_y} x 2 in one ds_read_b128 (4 LDS cycles) and
    // f_z x 2 in one ds_read_b64 (2 cycles) instead of merged ds_read2_b64 / ds_read2_b32 (8 + 4)
    typedef float quad_t __attribute__((ext_vector_type(4)));
    pair_t axy = {0.f, 0.f};
    float az = 0.f;
#pragma unroll 1
    for (; q + 2 <= qe; q += 2)
    {
        const quad_t f2 = *reinterpret_cast<const quad_t *>(pxy + q);
        const pair_t z2 = *reinterpret_cast<const pair_t *>(sfz + q);
        axy += f2.xy;
        az += z2.x;
        axy += f2.zw;
        az += z2.y;
    }
    if (q < qe)
    {
        axy += pxy[q];
        az += sfz[q];
    }
    a0 = axy.x;
    a1 = axy.y;
    a2 = az;
}

struct PipeNext
{
    uint2 tn;          // record of tile node threadIdx.x
    float c[3];        // its coordinates
    float v[3], w[3];  // x / p_old and z (MODE 1) at that node
    float m;           // its lumped mass (MODE 1: the owner slot's m s_M |p|^2 share of p.Ap)
    uint2 id[2];       // corner ids of elements threadIdx.x, threadIdx.x + 256
    uint2 pos[2];      // local-CSR positions of the corners of elements threadIdx.x, + NT
    uint32_t slot;     // node-major partial slot of tile node threadIdx.x
    uint32_t mat[2];   // material of elements threadIdx.x, threadIdx.x + 256 (0 when M == 1)
};

template <int NT, bool SANITIZE, int MODE>
__device__ __forceinline__ void pipe_issue_records(const DevSys &s, uint4 hd, PipeNext &n)
{
    const DevTiles &T = s.t;
    const uint32_t e0 = hd.x, ne = hd.y, nb = hd.z, nn = hd.w;
    const uint32_t i = threadIdx.x;
    n.tn = i < nn ? T.tnode[nb + i] : uint2{0u, 0u};
    n.slot = i < nn ? T.tslot[nb + i] : 0u;
    const uint32_t T3 = T.total_tile_nodes;
    const uint32_t q = nb + (i < nn ? i : 0u);
    n.c[0] = T.tcoord[q];
    n.c[1] = T.tcoord[T3 + q];
    n.c[2] = T.tcoord[2 * T3 + q];
#pragma unroll
    for (int k = 0; k < 2; ++k)
    {
        const uint32_t j = i + k * (uint32_t)NT;
        n.id[k] = T.eid[e0 + (j < ne ? j : 0u)];
        // prefetched with the records: a load inside the element phase would make its wait drain
        // every record load in flight for the next tile
        n.mat[k] = T.mat ? T.mat[e0 + (j < ne ? j : 0u)] : 0u;
        n.pos[k] = T.epos[e0 + (j < ne ? j : 0u)];
    }
}

template <bool SANITIZE, int MODE>
__device__ __forceinline__ void pipe_issue_gather(const DevSys &s, const float *__restrict__ x,
                                                  const float *__restrict__ z, uint32_t nn, PipeNext &n)
{
    const uint32_t g = n.tn.x & 0x7fffffffu;  // node 0 for idle lanes (harmless, in range)
    n.m = 0.f;
    (void)nn;
    n.v[0] = x[3u * g + 0];
    n.v[1] = x[3u * g + 1];
    n.v[2] = x[3u * g + 2];
    if constexpr (MODE == 1)
    {
        n.w[0] = z[3u * g + 0];
        n.w[1] = z[3u * g + 1];
        n.w[2] = z[3u * g + 2];
        n.m = s.mass[g];
    }
    else if constexpr (SANITIZE)
    {
        const uint32_t mk = s.mask[g];
        n.v[0] = (mk & 1u) ? 0.f : n.v[0];
        n.v[1] = (mk & 2u) ? 0.f : n.v[1];
        n.v[2] = (mk & 4u) ? 0.f : n.v[2];
    }
}

// NT threads per workgroup, tiles of <= TE = 2 NT elements and <= NT nodes (one node per lane)
// Push fold: each element stores its 4 corner forces at their tile-relative local-CSR positions (epos),
// so a node's forces sit contiguously in ascending element order and the fold reads them without a
// dependent CSR-entry lookup (the order of a local-CSR fold, without its index stream).
template <bool ISO, bool SANITIZE, int MODE, int NT>
__global__ __launch_bounds__(NT) void k_keff_tiles_pipe(DevSys s, const float *__restrict__ x, PcgArgs pa,
                                                        const uint4 *__restrict__ hdr)
{
    constexpr int TE = 2 * NT;
    constexpr int SP = 4 * TE + 2 * NT;  // slots per component plane: (element, corner) pairs + run pads
    constexpr int kTab = ISO ? 12 : 36;
    extern __shared__ float lds[];
    const DevTiles &T = s.t;
    const uint32_t ms = T.max_tile_nodes;
    // pushed corner forces: {f_x, f_y} pairs (one ds_write_b64 / ds_read2_b64 per two, summed with
    // v_pk_add_f32 without repacking) and an f_z plane
    float2 *sfxy = reinterpret_cast<float2 *>(lds);           // [SP]
    float *sfz = lds + 2 * SP;                                // [SP]
    float4 *sxp = reinterpret_cast<float4 *>(lds + 3 * SP);  // [ms] {x, y, z, v_x}
    float2 *sq = reinterpret_cast<float2 *>(sxp + ms);                   // [ms] {v_y, v_z}
    __shared__ float dtab[kMaxM * kTab];
    __shared__ double red[2 * (NT / 64)];
    if constexpr (MODE == 1)
    {
        if (!pa.ctl->active)
            return;
    }
    // this workgroup's tiles: XCD-contiguous ranges, stride = workgroups per XCD
    const uint32_t nxcd = 8u, xcd = blockIdx.x % nxcd, lb = blockIdx.x / nxcd, nbx = gridDim.x / nxcd;
    const uint32_t t_end = (uint32_t)(((uint64_t)(xcd + 1) * T.ntiles) / nxcd);
    uint32_t t = (uint32_t)(((uint64_t)xcd * T.ntiles) / nxcd) + lb;
    PipeNext cur;
    uint4 hd = t < t_end ? hdr[t] : uint4{0u, 0u, 0u, 0u};
    // header of the tile after next, loaded one tile early so phase (b) never waits on it
    uint4 hd2 = t + nbx < t_end ? hdr[t + nbx] : uint4{0u, 0u, 0u, 0u};
    if (t < t_end)
    {
        pipe_issue_records<NT, SANITIZE, MODE>(s, hd, cur);
        pipe_issue_gather<SANITIZE, MODE>(s, x, pa.z, hd.w, cur);
    }
    const uint32_t nm = s.M < kMaxM ? s.M : kMaxM;
    for (uint32_t i = threadIdx.x; i < nm * kTab; i += NT)
        dtab[i] = (float)s.dmat[36u * (i / kTab) + dsrc(ISO, i % kTab)];
    float beta = 0.f;
    if constexpr (MODE == 1)
    {
        // pcg.cpp:862-895 of the previous update, once per workgroup
        if (!residual_step<NT>(pa.ctl, pa.prr, pa.prz, pa.nupd, pa.stride, pa.it, pa.hist, red, &beta, pa.abl & 32u))
            return;
    }
    const float sK6 = (float)(s.sK / 6.0), sM = (float)s.sM;
    double pap = 0.0;
    for (; t < t_end; t += nbx)
    {
        const uint32_t ne = hd.y, nn = hd.w;
        // (a) LDS fill of tile t from the prefetched registers (second node slot, if any, loads directly)
        const uint32_t i0 = threadIdx.x;
        if (i0 < nn)
        {
            float v0 = cur.v[0], v1 = cur.v[1], v2 = cur.v[2];
            if constexpr (MODE == 1)
            {
                v0 = fmaf(beta, v0, cur.w[0]);
                v1 = fmaf(beta, v1, cur.w[1]);
                v2 = fmaf(beta, v2, cur.w[2]);
            }
            sxp[i0] = float4{cur.c[0], cur.c[1], cur.c[2], v0};
            sq[i0] = float2{v1, v2};
        }
        const uint2 id0 = cur.id[0], id1 = cur.id[1];
        const uint2 pos0 = cur.pos[0], pos1 = cur.pos[1];
        const uint32_t mat0 = cur.mat[0], mat1 = cur.mat[1];
        const uint2 tn_own = cur.tn;
        const uint32_t slot_own = cur.slot;
        const float m_own = cur.m;
        __syncthreads();
        // (b) next tile's records in flight during this tile's element and fold work
        const uint32_t tn_next = t + nbx;
        const uint4 hdn = hd2;
        if (tn_next < t_end)
            pipe_issue_records<NT, SANITIZE, MODE>(s, hdn, cur);
        hd2 = tn_next + nbx < t_end ? hdr[tn_next + nbx] : uint4{0u, 0u, 0u, 0u};
        // (c) elements of tile t (ablation bit 64: skipped, diagnostic timing only)
#pragma unroll
        for (int k = 0; k < 2; ++k)
        {
            const uint32_t j = threadIdx.x + k * NT;
            if (j < ne && !ablate(pa, 64u))
            {
                float f[12];
                geo_element_forces<ISO>(s, k ? id1 : id0, sxp, sq, sK6, k ? mat1 : mat0, dtab, f);
                const uint2 ps = k ? pos1 : pos0;
                const uint32_t pq[4] = {ps.x & 0xffffu, ps.x >> 16, ps.y & 0xffffu, ps.y >> 16};
#pragma unroll
                for (int a = 0; a < 4; ++a)
                {
                    sfxy[pq[a]] = float2{f[3 * a], f[3 * a + 1]};
                    sfz[pq[a]] = f[3 * a + 2];
                }
            }
        }
        __syncthreads();
        // (d) next tile's gathers (its node records have arrived by now; ablation bit 256: skipped)
        if (tn_next < t_end && !ablate(pa, 256u))
            pipe_issue_gather<SANITIZE, MODE>(s, x, pa.z, hdn.w, cur);
        // (e) fold per tile node -> node-major partials (+ p.Ap) (ablation bit 128: skipped)
        if (threadIdx.x < (ablate(pa, 128u) ? 0u : nn))  // nn <= 256: one tile node per lane
        {
            const uint32_t i = threadIdx.x;
            const uint2 tn = tn_own;
            float a0, a1, a2;
            fold_run(sfxy, sfz, tn.y & 0xffffu, tn.y >> 16, a0, a1, a2);
            float p0 = 0.f, p1 = 0.f, p2 = 0.f;
            if constexpr (MODE == 1)
            {
                p0 = sxp[i].w;
                p1 = sq[i].x;
                p2 = sq[i].y;
                if (tn.x & 0x80000000u)  // the node's owner slot carries its mass term m s_M p (once)
                {
                    const float m = m_own * sM;
                    a0 = fmaf(m, p0, a0);
                    a1 = fmaf(m, p1, a1);
                    a2 = fmaf(m, p2, a2);
                    if (pa.pnew)  // and stores the new p for the update pass (no z / p_old re-read there)
                    {
                        float *q = pa.pnew + 3ull * (tn.x & 0x7fffffffu);
                        q[0] = p0;
                        q[1] = p1;
                        q[2] = p2;
                    }
                }
            }
            // ablation (diagnostic timing only): 512 = no partial store, 1024 = tile-major store position
            if (!ablate(pa, 512u))
            {
                float *o = T.part + 3ull * (ablate(pa, 1024u) ? hd.z + i : slot_own);
                o[0] = a0;
                o[1] = a1;
                o[2] = a2;
            }
            if (MODE == 1 && (tn.x & 0x7fffffffu) < s.Nown)  // ghosts: another rank's row
                pap += (double)fmaf(p2, a2, fmaf(p1, a1, p0 * a0));  // fp32 per node, fp64 across nodes
        }
        __syncthreads();  // LDS is refilled by the next tile
        hd = hdn;
    }
    if constexpr (MODE == 1)
    {
        const double tt = block_sum<NT>(pap, red);
        if (threadIdx.x == 0)
            pa.part_dot[blockIdx.x] = tt;
    }
}

// ---- fan groups (groups.cpp) ----
// Persistent, XCD-aware, software-pipelined like k_keff_tiles_pipe, over tiles of <= NT fan groups (one per
// lane) and <= 2 NT nodes (two per lane). A lane loads its group's <= 8 nodes {x y z v_x}{v_y v_z} from LDS,
// runs the group's f <= 6 tets {a, b, r_i, r_(i+1) mod 6} in packed fp32 (v_pk_fma_f32: tets i and i + 3 of
// the fan side by side, so a closed Kuhn fan is three packed tet pairs), sums the forces per node in
// registers and pushes one force per node to its position in the tile's local CSR (the node's run start,
// kept in LDS, plus the group's 4-bit rank in the run from the 16-B record); the node fold, partial stores,
// p.Ap share and owner p store are those of k_keff_tiles_pipe.

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat(float v) { return f2{v, v}; }

struct GroupNext
{
    uint2 tn[2];          // records of tile nodes threadIdx.x, threadIdx.x + NT
    uint32_t slot[2];     // their node-major partial slots
    float c[2][3];        // their tile-relative coordinates
    float v[2][3], w[2][3], m[2];  // x / p_old, z and lumped mass at them
    uint4 g;              // record of group threadIdx.x
};

template <int NT>
__device__ __forceinline__ void group_issue_records(const DevSys &s, uint4 hd, GroupNext &n)
{
    const DevTiles &T = s.t;
    const uint32_t g0 = hd.x, ng = hd.y, nb = hd.z, nn = hd.w;
    const uint32_t T3 = T.total_tile_nodes;
#pragma unroll
    for (int k = 0; k < 2; ++k)
    {
        const uint32_t i = threadIdx.x + k * (uint32_t)NT;
        const uint32_t q = nb + (i < nn ? i : 0u);
        n.tn[k] = i < nn ? T.tnode[q] : uint2{0u, 0u};
        n.slot[k] = T.tslot[q];
        n.c[k][0] = T.tcoord[q];
        n.c[k][1] = T.tcoord[T3 + q];
        n.c[k][2] = T.tcoord[2 * T3 + q];
    }
    n.g = T.grec[g0 + (threadIdx.x < ng ? threadIdx.x : 0u)];
}

// one 12-B node triple per lane in a single buffer_load_dwordx3 (three dword gathers cost three address
// walks of the wave's 64 scattered lines)
__device__ __forceinline__ void load3(__amdgpu_buffer_rsrc_t rs, uint32_t q, float v[3])
{
    const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(rs, 12u * q, 0, 0);
    v[0] = __uint_as_float(w.x);
    v[1] = __uint_as_float(w.y);
    v[2] = __uint_as_float(w.z);
}

template <bool SANITIZE, int MODE>
__device__ __forceinline__ void group_issue_gather(const DevSys &s, const float *__restrict__ x,
                                                   const float *__restrict__ z, GroupNext &n)
{
    const __amdgpu_buffer_rsrc_t rx = whole_rsrc(x);
#pragma unroll
    for (int k = 0; k < 2; ++k)
    {
        const uint32_t g = n.tn[k].x & 0x7fffffffu;  // node 0 for idle lanes (harmless, in range)
        n.m[k] = 0.f;
        load3(rx, g, n.v[k]);
        if constexpr (MODE == 1)
        {
            load3(whole_rsrc(z), g, n.w[k]);
            n.m[k] = s.mass[g];
        }
        else if constexpr (SANITIZE)
        {
            const uint32_t mk = s.mask[g];
            n.v[k][0] = (mk & 1u) ? 0.f : n.v[k][0];
            n.v[k][1] = (mk & 2u) ? 0.f : n.v[k][1];
            n.v[k][2] = (mk & 4u) ? 0.f : n.v[k][2];
        }
    }
}

// Ring nodes k and k + 3 side by side: edge vectors d from a, values du relative to a's, w = e x d.
struct RingPair
{
    f2 d[3], du[3], w[3];
};

__device__ __forceinline__ RingPair ring_pair(const float4 *sxp, const float2 *sq, uint32_t l0, uint32_t l1,
                                              const float xa[3], const float ua[3], const float e[3])
{
    const float4 X0 = sxp[l0], X1 = sxp[l1];
    const float2 Q0 = sq[l0], Q1 = sq[l1];
    RingPair P;
    P.d[0] = f2{X0.x - xa[0], X1.x - xa[0]};
    P.d[1] = f2{X0.y - xa[1], X1.y - xa[1]};
    P.d[2] = f2{X0.z - xa[2], X1.z - xa[2]};
    P.du[0] = f2{X0.w - ua[0], X1.w - ua[0]};
    P.du[1] = f2{Q0.x - ua[1], Q1.x - ua[1]};
    P.du[2] = f2{Q0.y - ua[2], Q1.y - ua[2]};
    P.w[0] = pk_fma(splat(e[1]), P.d[2], -(splat(e[2]) * P.d[1]));
    P.w[1] = pk_fma(splat(e[2]), P.d[0], -(splat(e[0]) * P.d[2]));
    P.w[2] = pk_fma(splat(e[0]), P.d[1], -(splat(e[1]) * P.d[0]));
    return P;
}

__device__ __forceinline__ RingPair swap_pair(const RingPair &P)
{
    RingPair S;
#pragma unroll
    for (int q = 0; q < 3; ++q)
    {
        S.d[q] = P.d[q].yx;
        S.du[q] = P.du[q].yx;
        S.w[q] = P.w[q].yx;
    }
    return S;
}

// F += B(g)^T sig (g the corner's unscaled gradient, sig the scaled stress), packed over a tet pair
__device__ __forceinline__ void corner_acc(const f2 g[3], const f2 sig[6], f2 F[3])
{
    F[0] = pk_fma(g[2], sig[5], pk_fma(g[1], sig[3], pk_fma(g[0], sig[0], F[0])));
    F[1] = pk_fma(g[2], sig[4], pk_fma(g[0], sig[3], pk_fma(g[1], sig[1], F[1])));
    F[2] = pk_fma(g[0], sig[5], pk_fma(g[1], sig[4], pk_fma(g[2], sig[2], F[2])));
}

// Tets i (.x) and i + 3 (.y) of the fan: corners {a, b, r_i, r_j} with ring pairs I = (r_i, r_(i+3)) and
// J = (r_j, r_(j+3)), j = i + 1. With e = x_b - x_a, d_k = x_(r_k) - x_a and w_k = e x d_k, the cofactor rows
// (unscaled gradients) of corners b, r_i, r_j are d_i x d_j, -w_j and w_i, corner a's minus their sum, so
// the strain is sum over {b, r_i, r_j} of B(g_k) (u_k - u_a). The stress carries s_K / (6 |det|), masked to 0
// in a half whose tet does not exist. Forces accumulate on b (Fb), r_i (Fi) and r_j (Fj); corner a's is
// minus the group's other forces (partition of unity), formed once per group.
template <bool ISO>
__device__ __forceinline__ void tet_pair(const RingPair &I, const RingPair &J, const float e[3], const float db[3],
                                         const float *Dm, float sK6, bool vx, bool vy, f2 Fb[3], f2 Fi[3], f2 Fj[3])
{
    f2 g1[3];
    g1[0] = pk_fma(I.d[1], J.d[2], -(I.d[2] * J.d[1]));
    g1[1] = pk_fma(I.d[2], J.d[0], -(I.d[0] * J.d[2]));
    g1[2] = pk_fma(I.d[0], J.d[1], -(I.d[1] * J.d[0]));
    const f2 det = pk_fma(splat(e[0]), g1[0], pk_fma(splat(e[1]), g1[1], splat(e[2]) * g1[2]));
    f2 sc = {sK6 * __builtin_amdgcn_rcpf(fabsf(det.x)), sK6 * __builtin_amdgcn_rcpf(fabsf(det.y))};
    sc.x = vx ? sc.x : 0.f;
    sc.y = vy ? sc.y : 0.f;
    const f2 db0 = splat(db[0]), db1 = splat(db[1]), db2 = splat(db[2]);
    f2 eps[6];
    eps[0] = pk_fma(-J.w[0], I.du[0], pk_fma(I.w[0], J.du[0], g1[0] * db0));
    eps[1] = pk_fma(-J.w[1], I.du[1], pk_fma(I.w[1], J.du[1], g1[1] * db1));
    eps[2] = pk_fma(-J.w[2], I.du[2], pk_fma(I.w[2], J.du[2], g1[2] * db2));
    eps[3] = pk_fma(g1[0], db1, g1[1] * db0);
    eps[3] = pk_fma(I.w[0], J.du[1], pk_fma(I.w[1], J.du[0], eps[3]));
    eps[3] = pk_fma(-J.w[0], I.du[1], pk_fma(-J.w[1], I.du[0], eps[3]));
    eps[4] = pk_fma(g1[1], db2, g1[2] * db1);
    eps[4] = pk_fma(I.w[1], J.du[2], pk_fma(I.w[2], J.du[1], eps[4]));
    eps[4] = pk_fma(-J.w[1], I.du[2], pk_fma(-J.w[2], I.du[1], eps[4]));
    eps[5] = pk_fma(g1[0], db2, g1[2] * db0);
    eps[5] = pk_fma(I.w[0], J.du[2], pk_fma(I.w[2], J.du[0], eps[5]));
    eps[5] = pk_fma(-J.w[0], I.du[2], pk_fma(-J.w[2], I.du[0], eps[5]));
#pragma unroll
    for (int r = 0; r < 6; ++r)
        eps[r] *= sc;
    f2 sig[6];
    if constexpr (ISO)
    {
#pragma unroll
        for (int r = 0; r < 3; ++r)
            sig[r] = pk_fma(splat(Dm[3 * r + 2]), eps[2], pk_fma(splat(Dm[3 * r + 1]), eps[1], splat(Dm[3 * r]) * eps[0]));
#pragma unroll
        for (int r = 3; r < 6; ++r)
            sig[r] = splat(Dm[6 + r]) * eps[r];
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 6; ++r)
        {
            f2 acc = splat(Dm[6 * r]) * eps[0];
#pragma unroll
            for (int c = 1; c < 6; ++c)
                acc = pk_fma(splat(Dm[6 * r + c]), eps[c], acc);
            sig[r] = acc;
        }
    }
    const f2 mwj[3] = {-J.w[0], -J.w[1], -J.w[2]};
    corner_acc(g1, sig, Fb);
    corner_acc(mwj, sig, Fi);
    corner_acc(I.w, sig, Fj);
}

// One fan group around edge (a, b). Record g: slot s (0 = a, 1 = b, 2 + k = ring node k) has the 9-bit local
// id s % 3 of word s / 3 and rank nibble s of g.w; f = g.x >> 27 tets {a, b, r_i, r_(i+1)}, i < f (ring slot 6
// is ring slot 0: a closed 6-fan; a closed fan of f < 6 repeats r_0 in ring slot f). Used slots: a, b and
// ring slots 0 .. min(f + 1, 6) - 1.
template <bool ISO>
__device__ __forceinline__ void group_forces(uint4 g, const float4 *sxp, const float2 *sq, const uint16_t *sst,
                                             float sK6, const float *Dm, float2 *sfxy, float *sfz)
{
    const auto lid = [&](int k) { return ((k < 3 ? g.x : k < 6 ? g.y : g.z) >> (9 * (k % 3))) & 0x1ffu; };
    const auto push = [&](int k, float fx, float fy, float fz) {
        const uint32_t l = lid(k);
        const uint32_t q = (uint32_t)sst[l] + ((g.w >> (4 * k)) & 15u);
        sfxy[q] = float2{fx, fy};
        sfz[q] = fz;
    };
    const int f = (int)((g.x >> 27) & 7u);
    const float4 Xa = sxp[lid(0)], Xb = sxp[lid(1)];
    const float2 Qa = sq[lid(0)], Qb = sq[lid(1)];
    const float xa[3] = {Xa.x, Xa.y, Xa.z};
    const float ua[3] = {Xa.w, Qa.x, Qa.y};
    const float e[3] = {Xb.x - Xa.x, Xb.y - Xa.y, Xb.z - Xa.z};
    const float db[3] = {Xb.w - ua[0], Qb.x - ua[1], Qb.y - ua[2]};
    const RingPair P0 = ring_pair(sxp, sq, lid(2), lid(5), xa, ua, e);
    const RingPair P1 = ring_pair(sxp, sq, lid(3), lid(6), xa, ua, e);
    f2 Fb[3] = {}, F0[3] = {}, F1[3] = {}, F2[3] = {}, F3[3] = {};
    // pair 0: tets 0, 3 (ring pairs 0, 1)
    tet_pair<ISO>(P0, P1, e, db, Dm, sK6, f > 0, f > 3, Fb, F0, F1);
    const RingPair P2 = ring_pair(sxp, sq, lid(4), lid(7), xa, ua, e);
    // pair 1: tets 1, 4 (ring pairs 1, 2); ring nodes 1 and 4 are complete after it
    tet_pair<ISO>(P1, P2, e, db, Dm, sK6, f > 1, f > 4, Fb, F1, F2);
    push(3, F1[0].x, F1[1].x, F1[2].x);
    if (f >= 4)
        push(6, F1[0].y, F1[1].y, F1[2].y);
    // pair 2: tets 2, 5 (ring pairs 2, 3 = ring pair 0 swapped: ring slot 6 is ring slot 0)
    tet_pair<ISO>(P2, swap_pair(P0), e, db, Dm, sK6, f > 2, f > 5, Fb, F2, F3);
    if (f >= 2)
        push(4, F2[0].x, F2[1].x, F2[2].x);
    if (f >= 5)
        push(7, F2[0].y, F2[1].y, F2[2].y);
    // ring node 0 = F0.x + F3.y, ring node 3 = F0.y + F3.x; a = -(everything else)
    float r0[3], r3[3], fb[3], fa[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
    {
        r0[q] = F0[q].x + F3[q].y;
        r3[q] = F0[q].y + F3[q].x;
        fb[q] = Fb[q].x + Fb[q].y;
        const f2 s12 = F1[q] + F2[q];
        fa[q] = -(((fb[q] + r0[q]) + r3[q]) + (s12.x + s12.y));
    }
    push(2, r0[0], r0[1], r0[2]);
    if (f >= 3)
        push(5, r3[0], r3[1], r3[2]);
    push(0, fa[0], fa[1], fa[2]);
    push(1, fb[0], fb[1], fb[2]);
}

// MONO: one material, D from the kernel arguments (SGPR operands); otherwise the group's material selects
// a row of the LDS table (<= 16 materials, abi.cpp)
template <bool ISO, bool SANITIZE, int MODE, int NT, bool MONO>
__global__ __launch_bounds__(NT, kGroupWavesPerSimd) void k_keff_groups_pipe(DevSys s, const float *__restrict__ x, PcgArgs pa,
                                                         const uint4 *__restrict__ hdr)
{
    constexpr int kTab = ISO ? 12 : 36;
    constexpr int SP = (int)kGroupSlotsPerLane * NT, MS = 2 * NT;
    extern __shared__ float lds[];
    const DevTiles &T = s.t;
    float2 *sfxy = reinterpret_cast<float2 *>(lds);           // [SP]
    float *sfz = lds + 2 * SP;                                // [SP]
    float4 *sxp = reinterpret_cast<float4 *>(lds + 3 * SP);  // [MS] {x, y, z, v_x}
    float2 *sq = reinterpret_cast<float2 *>(sxp + MS);       // [MS] {v_y, v_z}
    uint16_t *sst = reinterpret_cast<uint16_t *>(sq + MS);   // [MS] run start in the local CSR
    __shared__ float dtab[MONO ? 1 : kMaxM * kTab];
    __shared__ double red[2 * (NT / 64)];
    const uint32_t nxcd = 8u, xcd = blockIdx.x % nxcd, lb = blockIdx.x / nxcd, nbx = gridDim.x / nxcd;
    const uint32_t t_end = (uint32_t)(((uint64_t)(xcd + 1) * T.ntiles) / nxcd);
    uint32_t t = (uint32_t)(((uint64_t)xcd * T.ntiles) / nxcd) + lb;
    GroupNext cur;
    // the control flag and the first two tile headers: scalar loads issued together, one round trip (the flag was
    // a round trip of its own in front of the headers)
    const int active = MODE == 1 ? pa.ctl->active : 1;
    uint4 hd = t < t_end ? hdr[t] : uint4{0u, 0u, 0u, 0u};
    uint4 hd2 = t + nbx < t_end ? hdr[t + nbx] : uint4{0u, 0u, 0u, 0u};
    if (!active)
        return;
    if (t < t_end)
    {
        group_issue_records<NT>(s, hd, cur);
        group_issue_gather<SANITIZE, MODE>(s, x, pa.z, cur);
    }
    if constexpr (!MONO)
    {
        const uint32_t nm = s.M < kMaxM ? s.M : kMaxM;
        for (uint32_t i = threadIdx.x; i < nm * kTab; i += NT)
            dtab[i] = (float)s.dmat[36u * (i / kTab) + dsrc(ISO, i % kTab)];
    }
    float beta = 0.f;
    if constexpr (MODE == 1)
    {
        if (!residual_step<NT, 8>(pa.ctl, pa.prr, pa.prz, pa.nupd, pa.stride, pa.it, pa.hist, red, &beta, pa.abl & 32u))
            return;
    }
    const float sK6 = (float)(s.sK / 6.0), sM = (float)s.sM;
    double pap = 0.0;
    for (; t < t_end; t += nbx)
    {
        const uint32_t ng = hd.y, nn = hd.w;
        // (a) LDS fill of tile t's nodes (two per lane) from the prefetched registers
#pragma unroll
        for (int k = 0; k < 2; ++k)
        {
            const uint32_t i = threadIdx.x + k * NT;
            if (i < nn)
            {
                float v0 = cur.v[k][0], v1 = cur.v[k][1], v2 = cur.v[k][2];
                if constexpr (MODE == 1)
                {
                    v0 = fmaf(beta, v0, cur.w[k][0]);
                    v1 = fmaf(beta, v1, cur.w[k][1]);
                    v2 = fmaf(beta, v2, cur.w[k][2]);
                }
                sxp[i] = float4{cur.c[k][0], cur.c[k][1], cur.c[k][2], v0};
                sq[i] = float2{v1, v2};
                sst[i] = (uint16_t)(cur.tn[k].y & 0xffffu);
            }
        }
        const uint4 gr = cur.g;
        const uint2 tn_own[2] = {cur.tn[0], cur.tn[1]};
        const uint32_t slot_own[2] = {cur.slot[0], cur.slot[1]};
        const float m_own[2] = {cur.m[0], cur.m[1]};
        __syncthreads();
        // (b) next tile's records in flight during this tile's group and fold work
        const uint32_t tn_next = t + nbx;
        const uint4 hdn = hd2;
        if (tn_next < t_end)
            group_issue_records<NT>(s, hdn, cur);
        hd2 = tn_next + nbx < t_end ? hdr[tn_next + nbx] : uint4{0u, 0u, 0u, 0u};
        // (c) this lane's group (ablation bit 64: skipped, diagnostic timing only)
        if (threadIdx.x < ng && !ablate(pa, 64u))
        {
            const float *Dm = MONO ? s.d1 : dtab + kTab * (gr.y >> 27);
            group_forces<ISO>(gr, sxp, sq, sst, sK6, Dm, sfxy, sfz);
        }
        __syncthreads();
        // (d) next tile's gathers (ablation bit 256: skipped)
        if (tn_next < t_end && !ablate(pa, 256u))
            group_issue_gather<SANITIZE, MODE>(s, x, pa.z, cur);
        // (e) fold per tile node -> node-major partials (+ p.Ap) (ablation bit 128: skipped)
#pragma unroll
        for (int k = 0; k < 2; ++k)
        {
            const uint32_t i = threadIdx.x + k * NT;
            if (i < (ablate(pa, 128u) ? 0u : nn))
            {
                const uint2 tn = tn_own[k];
                float a0, a1, a2;
                fold_run(sfxy, sfz, tn.y & 0xffffu, tn.y >> 16, a0, a1, a2);
                float p0 = 0.f, p1 = 0.f, p2 = 0.f;
                if constexpr (MODE == 1)
                {
                    p0 = sxp[i].w;
                    p1 = sq[i].x;
                    p2 = sq[i].y;
                    if (tn.x & 0x80000000u)  // the node's owner slot carries its mass term m s_M p (once)
                    {
                        const float m = m_own[k] * sM;
                        a0 = fmaf(m, p0, a0);
                        a1 = fmaf(m, p1, a1);
                        a2 = fmaf(m, p2, a2);
                        if (pa.pnew)  // and stores the new p for the update pass
                            store3(pa.pnew, whole_rsrc(pa.pnew), tn.x & 0x7fffffffu, p0, p1, p2, false);
                    }
                }
                if (!ablate(pa, 512u))
                    store3(T.part, whole_rsrc(T.part), slot_own[k], a0, a1, a2, T.wt_part != 0);
                if (MODE == 1 && (tn.x & 0x7fffffffu) < s.Nown)  // ghosts: another rank's row
                    pap += (double)fmaf(p2, a2, fmaf(p1, a1, p0 * a0));  // fp32 per node, fp64 across nodes
            }
        }
        __syncthreads();  // LDS is refilled by the next tile
        hd = hdn;
    }
    if constexpr (MODE == 1)
    {
        const double tt = block_sum<NT>(pap, red);
        if (threadIdx.x == 0)
            pa.part_dot[blockIdx.x] = tt;
    }
}

// pcg.cpp:862-895 for the last iteration of a batch (the next batch's tiles kernel repeats it
// idempotently): one workgroup
__global__ __launch_bounds__(256) void k_pcg_check(Ctl *ctl, const double *__restrict__ prr,
                                                   const double *__restrict__ prz, unsigned nparts, unsigned stride,
                                                   unsigned it, double *__restrict__ hist)
{
    __shared__ double red[8];
    if (!ctl->active)
        return;
    float beta;
    (void)residual_step<256>(ctl, prr, prz, nparts, stride, it, hist, red, &beta);
}

// one workgroup: out[0] = fold(a[0..n)), out[1] = fold(b[0..n)) (b may be NULL), fixed order
__global__ __launch_bounds__(1024) void k_fold_pair(const double *__restrict__ a, const double *__restrict__ b,
                                                    unsigned n, double *__restrict__ out)
{
    __shared__ double red[16];
    const double ta = fold_all<1024>(a, n, red);
    const double tb = b ? fold_all<1024>(b, n, red) : 0.0;
    if (threadIdx.x == 0)
    {
        out[0] = ta;
        if (b)
            out[1] = tb;
    }
}

// FAST: symmetrise the block inverse (upper triangle wins, so k_precond and the update agree) and pack
// it to 16 B per node for the update pass in the Jacobi-scaled form of blockinv_pack.hpp (fp32 scale,
// fp16 row scales and correlations; a flagged fp32 fallback for blocks that form does not hold). The
// operator the solve applies is written back to the 9-float copy, so the prologue's z (k_precond) and
// the update's z use the same symmetric preconditioner.
__global__ __launch_bounds__(256) void k_sym_inverse(uint32_t N, const uint32_t *__restrict__ mask,
                                                     float *__restrict__ inv9, float *__restrict__ inv6)
{
    const uint32_t n = blockIdx.x * 256u + threadIdx.x;
    if (n >= N)
        return;
    float *a = inv9 + 9ull * n;
    const float v[6] = {a[0], a[1], a[2], a[4], a[5], a[8]};  // a00 a01 a02 a11 a12 a22
    uint32_t w[4];
    float d[6];
    (void)pack_block_inverse(v, mask[n], w, d);
    a[0] = d[0];
    a[1] = a[3] = d[1];
    a[2] = a[6] = d[2];
    a[4] = d[3];
    a[5] = a[7] = d[4];
    a[8] = d[5];
    reinterpret_cast<uint4 *>(inv6)[n] = make_uint4(w[0], w[1], w[2], w[3]);
}

// a lattice handle's per-class block inverse (packed record and the 9-float operator) from one representative node
// of each class (every node of a class has the same diagonal blocks and mass: lattice.cpp)
__global__ __launch_bounds__(256) void k_lat_class_inverse(const uint32_t *__restrict__ rep,
                                                           const float *__restrict__ inv6, const float *__restrict__ inv9,
                                                           uint4 *__restrict__ cinv6, float *__restrict__ cinv9,
                                                           float4 *__restrict__ cz)
{
    for (uint32_t c = threadIdx.x; c < kLatClasses; c += 256)
    {
        const uint32_t n = rep[c];
        if (n == 0xFFFFFFFFu)
            continue;
        const uint4 iw = reinterpret_cast<const uint4 *>(inv6)[n];
        float a9[9];
        for (int q = 0; q < 9; ++q)
            a9[q] = inv9[9ull * n + q];
        cinv6[c] = iw;
        for (int q = 0; q < 9; ++q)
            cinv9[9 * c + q] = a9[q];
        // the operator k_pcg_update_tiles applies (its unpack, or the flagged block's fp32 copy)
        float bv[6];
        if ((int)iw.x >= 0)
            unpack_block_inverse(iw.y, iw.z, iw.w, __uint_as_float(iw.x), bv);
        else
        {
            bv[0] = a9[0];
            bv[1] = a9[1];
            bv[2] = a9[2];
            bv[3] = a9[4];
            bv[4] = a9[5];
            bv[5] = a9[8];
        }
        if (cz)
        {
            cz[2 * c] = float4{bv[0], bv[1], bv[2], bv[3]};
            cz[2 * c + 1] = float4{bv[4], bv[5], 0.f, 0.f};
        }
    }
}

__global__ __launch_bounds__(256) void k_halo_pack(const uint32_t *__restrict__ idx, uint64_t n,
                                                   const float *__restrict__ v, float *__restrict__ out)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull)
    {
        const uint32_t q = idx[i];
        out[3 * i + 0] = v[3ull * q + 0];
        out[3 * i + 1] = v[3ull * q + 1];
        out[3 * i + 2] = v[3ull * q + 2];
    }
}

template <bool SANITIZE>
__global__ __launch_bounds__(256) void k_keff_finalize(DevSys s, const float *__restrict__ x, float *__restrict__ y)
{
    const DevTiles &T = s.t;
    const uint32_t n = blockIdx.x * 256 + threadIdx.x;
    if (n >= s.N)
        return;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (uint32_t q = T.node_part_off[n] & kPartOffBits; q < (T.node_part_off[n + 1] & kPartOffBits); ++q)
    {
        const float *pp = T.part + 3ull * (T.node_major ? q : T.part_slot[q]);
        a0 += pp[0];
        a1 += pp[1];
        a2 += pp[2];
    }
    const uint32_t mk = s.mask[n];
    const float m = s.mass[n] * (float)s.sM;
    const float x0 = x[3u * n + 0], x1 = x[3u * n + 1], x2 = x[3u * n + 2];
    float y0 = fmaf(m, (SANITIZE && (mk & 1u)) ? 0.f : x0, a0);
    float y1 = fmaf(m, (SANITIZE && (mk & 2u)) ? 0.f : x1, a1);
    float y2 = fmaf(m, (SANITIZE && (mk & 4u)) ? 0.f : x2, a2);
    y[3u * n + 0] = (mk & 1u) ? x0 : y0;
    y[3u * n + 1] = (mk & 2u) ? x1 : y1;
    y[3u * n + 2] = (mk & 4u) ? x2 : y2;
}

// The four rotating search-direction buffers: p_j lives in p[(j + 1) % 4] (fast_p_buf)
struct PBufs
{
    const float *p[4];
};

// Per-node state of the update pass, loaded in phases so that U nodes per thread have their loads in
// flight together (the pass is latency-bound: node_part_off -> partial run is a dependent chain)
struct UpdNode
{
    uint32_t n, q0, q1, mk;
    bool ok;
    float rv0[3], pa[3], pb[3], pv[3], m;
    uint4 iw;
    float xv[3], pj[kXLag][3];
};

// pcg.cpp:840-895 per owned node: Ap from the node-major partials (folded in ascending tile order),
// r -= alpha Ap, Dirichlet, z = M^-1 r (16-B Jacobi-scaled block, blockinv_pack.hpp), r.r / r.z shares;
// x += alpha_j p_j for the last `lag` iterations every lag-th iteration (lazy x, 1 = every iteration; the
// FMA chain in iteration order is bitwise the eager update), fast_flush_x applies the rest after the solve.
template <int U, bool XF, bool LAT, bool NOZ = false>
__global__ __launch_bounds__(kUpdThreads) void k_pcg_update_tiles(
    DevSys s, const float *__restrict__ rhs, const float *__restrict__ inv, const float *__restrict__ inv9,
    float *__restrict__ x, float *__restrict__ r, float *__restrict__ z, const float *__restrict__ pold,
    float *__restrict__ pnew, Ctl *__restrict__ ctl, const double *__restrict__ part_dot, unsigned ntp,
    double *__restrict__ prr, double *__restrict__ prz, unsigned it, int wt, PBufs pbuf, unsigned lag)
{
    __shared__ double red[2 * (kUpdThreads / 64)];
    __shared__ uint4 cinv[LAT ? kLatClasses : 1];
    const DevTiles &T = s.t;
    const __amdgpu_buffer_rsrc_t rctl = ctl_rsrc(ctl);
    // this iteration's beta (the K_eff kernel's residual step wrote it), as a vector load like every control word here
    const float beta = (float)ctl_f64(rctl, (uint32_t)offsetof(Ctl, beta));
    const float sM = (float)s.sM;
    const __amdgpu_buffer_rsrc_t rpart = whole_rsrc(T.part);
    // XF: this iteration applies the lazy x update (a separate instantiation, so the three iterations in four
    // that do not keep the registers of the update pass's occupancy)
    constexpr bool xflush = XF;
    const uint32_t step = gridDim.x * kUpdThreads * U;
    uint32_t base = blockIdx.x * kUpdThreads * U + threadIdx.x;
    UpdNode v[U];
    // (1) + (2): every load of the U nodes that does not need alpha (issued for the first trip before the
    // p.Ap fold below, so its latency hides under the fold's)
    const auto load_nodes = [&](uint32_t b0) {
#pragma unroll
        for (int u = 0; u < U; ++u)  // the partial-run bounds (and the Dirichlet mask in their top bits)
        {
            v[u].n = b0 + u * kUpdThreads;
            v[u].ok = v[u].n < s.Nown;
            const uint32_t n = v[u].ok ? v[u].n : 0u;
            if constexpr (LAT)  // one row value per node; the mask and the block inverse from the node's class
            {
                v[u].q0 = n;
                v[u].q1 = n + 1u;
                v[u].mk = T.lcls[n];  // class << 3 | mask
            }
            else
            {
                const uint32_t o0 = T.node_part_off[n], o1 = T.node_part_off[n + 1];
                v[u].q0 = o0 & kPartOffBits;
                v[u].q1 = o1 & kPartOffBits;
                v[u].mk = T.off_mask ? o0 >> 29 : s.mask[n];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            UpdNode &w = v[u];
            const uint32_t n = w.ok ? w.n : 0u;
#pragma unroll
            for (int k = 0; k < 3; ++k)
                w.rv0[k] = r[3u * n + k];
            if constexpr (LAT)
                load3(rpart, n, w.pa);
            else
            {
                w.iw = reinterpret_cast<const uint4 *>(inv)[n];
                // first two partials unconditionally (the part buffer carries 2 padding slots)
                if (T.node_major)
                {
                    load3(rpart, w.q0, w.pa);
                    load3(rpart, w.q0 + 1, w.pb);
                }
            }
            // a node of no element forms p_it here (Ap = m s_M p); the tiles kernel folded the mass term
            // into every other node's owner partial
            w.m = 0.f;
            w.pv[0] = w.pv[1] = w.pv[2] = 0.f;
            if (!LAT && w.q0 == w.q1)
            {
                w.m = s.mass[n] * sM;
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    w.pv[k] = fmaf(beta, pold[3u * n + k], z[3u * n + k]);
            }
            if (xflush)
            {
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    w.xv[k] = x[3u * n + k];
#pragma unroll
                for (unsigned j = 0; j < kXLag; ++j)
                    if (j < lag)
                    {
                        const float *pj = pbuf.p[(it + 2u - lag + j) % 4u];
#pragma unroll
                        for (int k = 0; k < 3; ++k)
                            w.pj[j][k] = pj[3u * n + k];
                    }
            }
        }
    };
    if (base < s.Nown)
        load_nodes(base);
    // LAT (structured block): the packed block inverse of each (boundary class, mask), lattice.cpp; thread c loads
    // class c's with the node loads in flight (one prologue round trip for the nodes, the class table, the control
    // block and the p.Ap shares, instead of three)
    static_assert(!LAT || kLatClasses <= kUpdThreads, "one class per thread");
    uint4 cw = {0u, 0u, 0u, 0u};
    if constexpr (LAT)
        cw = T.lcinv6[min((uint32_t)threadIdx.x, kLatClasses - 1u)];
    // control words (ctl_rsrc): the flag, rho and the lazy-x alphas, in flight with the node loads and the fold's
    const int active = (int)__builtin_amdgcn_raw_buffer_load_b32(rctl, (uint32_t)offsetof(Ctl, active), 0, 0);
    const double rho = ctl_f64(rctl, (uint32_t)(offsetof(Ctl, rho2) + 8u * (it & 1u)));
    double ah[kXLag];
#pragma unroll
    for (unsigned j = 0; j < kXLag; ++j)
        ah[j] = xflush ? ctl_f64(rctl, (uint32_t)(offsetof(Ctl, alpha_h) + 8u * j)) : 0.0;
    // pcg.cpp:840-852: alpha = rho / (p . Ap)
    const double denom = fold_all<kUpdThreads, 12>(part_dot, ntp, red);  // <= 3,072 K_eff shares in one trip
    if (!active)
        return;
    if constexpr (LAT)
    {
        if (threadIdx.x < kLatClasses)
            cinv[threadIdx.x] = cw;
        __syncthreads();
    }
    if (fabs(denom) < 1.0e-18)
    {
        if (blockIdx.x == 0 && threadIdx.x == 0)
        {
            ctl->denom = denom;
            ctl->error = CWF_ERR_DENOM_ZERO;
            ctl->error_iter = (int)it;
            ctl->active = 0;
        }
        return;
    }
    const double alpha_d = rho / denom;
    if (blockIdx.x == 0 && threadIdx.x == 0)
    {
        ctl->denom = denom;
        ctl->alpha = alpha_d;
        ctl->alpha_last = alpha_d;
        ctl->alpha_h[it % kXLag] = alpha_d;
    }
    float aj[kXLag];  // alpha of iteration it + 1 - lag + j
#pragma unroll
    for (unsigned j = 0; j < kXLag; ++j)
    {
        const unsigned ij = it + 1u - lag + j;
        aj[j] = j < lag ? (float)(ij == it ? alpha_d : ah[ij % kXLag]) : 0.f;
    }
    const float alpha = (float)alpha_d;
    double rr = 0.0, rz = 0.0;
    for (; base < s.Nown; base += step)
    {
        if (base != blockIdx.x * kUpdThreads * U + threadIdx.x)
            load_nodes(base);
        // (3) fold, update, precondition, store
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            UpdNode &w = v[u];
            if (!w.ok)
                continue;
            const uint32_t n = w.n, mk = LAT ? w.mk & 7u : w.mk;
            if constexpr (LAT)
                w.iw = cinv[w.mk];
            if (!LAT && w.q0 == w.q1)
                store3(pnew, whole_rsrc(pnew), n, w.pv[0], w.pv[1], w.pv[2], false);
            if (xflush)  // x and the lag p_j were loaded with the rest; the FMA chain in iteration order
            {
#pragma unroll
                for (unsigned j = 0; j < kXLag; ++j)
                    if (j < lag)
#pragma unroll
                        for (int k = 0; k < 3; ++k)
                            w.xv[k] = fmaf(aj[j], w.pj[j][k], w.xv[k]);
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    if (mk & (1u << k))
                        w.xv[k] = rhs[3u * n + k];
                store3(x, whole_rsrc(x), n, w.xv[0], w.xv[1], w.xv[2], wt);
            }
            float a0 = 0.f, a1 = 0.f, a2 = 0.f;
            const uint32_t cnt = w.q1 - w.q0;
            if (LAT)
            {
                a0 = w.pa[0];
                a1 = w.pa[1];
                a2 = w.pa[2];
            }
            else if (T.node_major)
            {
                if (cnt > 0)
                {
                    a0 = w.pa[0];
                    a1 = w.pa[1];
                    a2 = w.pa[2];
                }
                if (cnt > 1)
                {
                    a0 += w.pb[0];
                    a1 += w.pb[1];
                    a2 += w.pb[2];
                }
                for (uint32_t q = 2; q < cnt; ++q)
                {
                    float d[3];
                    load3(rpart, w.q0 + q, d);
                    a0 += d[0];
                    a1 += d[1];
                    a2 += d[2];
                }
            }
            else
                for (uint32_t q = w.q0; q < w.q1; ++q)
                {
                    const float *pp = T.part + 3ull * T.part_slot[q];
                    a0 += pp[0];
                    a1 += pp[1];
                    a2 += pp[2];
                }
            const float av[3] = {a0, a1, a2};
            float rv[3];
#pragma unroll
            for (int k = 0; k < 3; ++k)
            {
                const float apk = cnt == 0 ? w.m * w.pv[k] : av[k];
                rv[k] = (mk & (1u << k)) ? 0.0f : fmaf(-alpha, apk, w.rv0[k]);
            }
            store3(r, whole_rsrc(r), n, rv[0], rv[1], rv[2], wt);
            // symmetric block inverse {a00 a01 a02 a11 a12 a22}; a flagged block (negative scale) reads its
            // fp32 copy instead
            float bv[6];
            if ((int)w.iw.x >= 0)
                unpack_block_inverse(w.iw.y, w.iw.z, w.iw.w, __uint_as_float(w.iw.x), bv);
            else
            {
                const float *a9 = LAT ? T.lcinv9 + 9u * w.mk : inv9 + 9ull * n;
                bv[0] = a9[0];
                bv[1] = a9[1];
                bv[2] = a9[2];
                bv[3] = a9[4];
                bv[4] = a9[5];
                bv[5] = a9[8];
            }
            const float iv[9] = {bv[0], bv[1], bv[2], bv[1], bv[3], bv[4], bv[2], bv[4], bv[5]};
            float zs[3];
#pragma unroll
            for (int k = 0; k < 3; ++k)
            {
                float zk = fmaf(iv[3 * k + 2], rv[2], fmaf(iv[3 * k + 1], rv[1], iv[3 * k] * rv[0]));
                zk = (mk & (1u << k)) ? 0.0f : zk;
                zs[k] = zk;
                rr += (double)rv[k] * (double)rv[k];
                rz += (double)rv[k] * (double)zk;
            }
            if constexpr (!NOZ)  // NOZ (lattice lzr): the K_eff pass forms z from r itself
                store3(z, whole_rsrc(z), n, zs[0], zs[1], zs[2], wt);
        }
    }
    // ghost nodes of a shard: only the search direction (the tiles kernel's p) is kept
    for (uint32_t n = s.Nown + blockIdx.x * kUpdThreads + threadIdx.x; n < s.N; n += gridDim.x * kUpdThreads)
    {
#pragma unroll
        for (int k = 0; k < 3; ++k)
            pnew[3u * n + k] = fmaf(beta, pold[3u * n + k], z[3u * n + k]);
    }
    double t0, t1;
    block_sum2<kUpdThreads>(rr, rz, red, t0, t1);
    if (threadIdx.x == 0)
    {
        prr[blockIdx.x] = t0;
        prz[blockIdx.x] = t1;
    }
}

inline unsigned grid_for(uint32_t n, uint32_t b) { return (n + b - 1) / b; }

inline size_t tiles_lds(const DevSys &s)
{
    // element forces [12][kTileElems] f32 + local CSR [4*kTileElems] u16 + node values [3][ms]
    // (+ node coordinates [3][ms] with GEO records)
    return sizeof(float) * (14 * kTileElems + (s.t.geo ? 6 : 3) * (size_t)s.t.max_tile_nodes);
}

template <bool ISO, bool SAN, int MODE, bool GEO>
void launch_tiles_g(const DevSys &s, const float *x, const PcgArgs &pa, int nt, hipStream_t st)
{
    const size_t lds = tiles_lds(s);
    if (nt == 512)
        k_keff_tiles<ISO, SAN, MODE, 512, GEO><<<s.t.ntiles, 512, lds, st>>>(s, x, pa);
    else
        k_keff_tiles<ISO, SAN, MODE, 256, GEO><<<s.t.ntiles, 256, lds, st>>>(s, x, pa);
}

#include "hex8_tiles.inc"
#include "lattice.inc"
#include "lattice_fused.inc"

// pipelined kernel: element forces + local CSR + per tile node {x y z v_x}{v_y v_z}
inline size_t pipe_lds(const DevSys &s)
{
    const size_t ms = s.t.max_tile_nodes, te = 2 * (size_t)s.t.pipe_nt;
    // 3 component planes of 4 te (element, corner) slots + one pad per tile node (odd runs), then the tile
    // nodes {x y z v_x}{v_y v_z}
    return sizeof(float) * 3 * (4 * te + 2 * (size_t)s.t.pipe_nt) + ms * (16 + 8);
}

template <bool ISO, int NT>
unsigned pipe_grid_query(const DevSys &s)
{
    int dev = 0, bpc = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k_keff_tiles_pipe<ISO, false, 1, NT>, NT,
                                                       pipe_lds(s));
    unsigned g = (unsigned)((bpc > 0 ? bpc : 1) * (cus > 0 ? cus : 1));
    g = g < 8u ? 8u : g - g % 8u;  // whole XCD groups
    const unsigned need = ((s.t.ntiles + 7u) / 8u) * 8u;
    return g < need ? g : (need ? need : 8u);
}

template <bool ISO, bool SAN, int MODE, int NT>
void launch_pipe(const DevSys &s, const float *x, const PcgArgs &pa, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    const size_t lds = pipe_lds(s);
    if (e0 && e1)
        hipExtLaunchKernelGGL(k_keff_tiles_pipe<ISO, SAN, MODE, NT>, dim3(s.t.pipe_grid), dim3(NT),
                              (uint32_t)lds, st, e0, e1, 0, s, x, pa, s.t.hdr);
    else
        k_keff_tiles_pipe<ISO, SAN, MODE, NT><<<s.t.pipe_grid, NT, lds, st>>>(s, x, pa, s.t.hdr);
}

// pushed forces {f_x, f_y} + f_z per slot, then per tile node {x y z v_x} {v_y v_z} and its u16 run start
constexpr size_t group_lds(int nt) { return sizeof(float) * 3 * kGroupSlotsPerLane * nt + 2 * nt * (16 + 8 + 2); }

template <bool ISO, bool MONO, int NT>
unsigned group_grid_query()
{
    int dev = 0, bpc = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k_keff_groups_pipe<ISO, false, 1, NT, MONO>, NT,
                                                       group_lds(NT));
    unsigned g = (unsigned)((bpc > 0 ? bpc : 1) * (cus > 0 ? cus : 1));
    return g < 8u ? 8u : g - g % 8u;  // whole XCD groups
}

template <bool ISO, bool SAN, int MODE, bool MONO, int NT>
void launch_groups_m(const DevSys &s, const float *x, const PcgArgs &pa, hipStream_t st, hipEvent_t e0,
                     hipEvent_t e1)
{
    constexpr uint32_t lds = (uint32_t)group_lds(NT);
    if (e0 && e1)
        hipExtLaunchKernelGGL(k_keff_groups_pipe<ISO, SAN, MODE, NT, MONO>, dim3(s.t.pipe_grid), dim3(NT), lds, st,
                              e0, e1, 0, s, x, pa, s.t.hdr);
    else
        k_keff_groups_pipe<ISO, SAN, MODE, NT, MONO><<<s.t.pipe_grid, NT, lds, st>>>(s, x, pa, s.t.hdr);
}

template <bool ISO, bool SAN, int MODE>
void launch_groups(const DevSys &s, const float *x, const PcgArgs &pa, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    if (s.t.pipe_nt == 256)
        s.M == 1 ? launch_groups_m<ISO, SAN, MODE, true, 256>(s, x, pa, st, e0, e1)
                 : launch_groups_m<ISO, SAN, MODE, false, 256>(s, x, pa, st, e0, e1);
    else
        s.M == 1 ? launch_groups_m<ISO, SAN, MODE, true, 128>(s, x, pa, st, e0, e1)
                 : launch_groups_m<ISO, SAN, MODE, false, 128>(s, x, pa, st, e0, e1);
}

template <bool ISO, bool MONO>
unsigned group_grid(int nt)
{
    return nt == 256 ? group_grid_query<ISO, MONO, 256>() : group_grid_query<ISO, MONO, 128>();
}

// e0/e1 (optional): hipExtLaunchKernel stamps them from the dispatch packet itself, so the timed
// interval is the kernel's own execution (what rocprofv3 --kernel-trace reports), not marker latency
template <bool ISO, bool SAN, int MODE>
void launch_tiles(const DevSys &s, const float *x, const PcgArgs &pa, int nt, hipStream_t st,
                  hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr)
{
    if (s.t.lat)
    {
        launch_lattice<MODE, SAN>(s, x, pa, st, e0, e1);
        return;
    }
    if (s.t.grp)
    {
        launch_groups<ISO, SAN, MODE>(s, x, pa, st, e0, e1);
        return;
    }
    if (s.t.hex)
    {
        launch_hex<ISO, SAN, MODE>(s, x, pa, st, e0, e1);
        return;
    }
    if (s.t.pipe)
    {
        if (s.t.pipe_nt == 128)
            launch_pipe<ISO, SAN, MODE, 128>(s, x, pa, st, e0, e1);
        else
            launch_pipe<ISO, SAN, MODE, 256>(s, x, pa, st, e0, e1);
        return;
    }
    if (e0)
        (void)hipEventRecord(e0, st);
    if (s.t.geo)
        launch_tiles_g<ISO, SAN, MODE, true>(s, x, pa, nt, st);
    else
        launch_tiles_g<ISO, SAN, MODE, false>(s, x, pa, nt, st);
    if (e1)
        (void)hipEventRecord(e1, st);
}
}  // namespace

unsigned fast_tile_blocks(const DevSys &s)
{
    return s.t.lat ? s.t.lnwork : (s.t.pipe || s.t.hex) ? s.t.pipe_grid : s.t.ntiles;
}

unsigned fast_pipe_grid(const DevSys &s)
{
    if (s.t.grp)
    {
        const int nt = s.t.pipe_nt;
        const unsigned g = s.iso ? (s.M == 1 ? group_grid<true, true>(nt) : group_grid<true, false>(nt))
                                 : (s.M == 1 ? group_grid<false, true>(nt) : group_grid<false, false>(nt));
        const unsigned need = ((s.t.ntiles + 7u) / 8u) * 8u;
        return g < need ? g : (need ? need : 8u);
    }
    if (s.t.hex)
        return s.iso ? hex_grid_query<true>(s) : hex_grid_query<false>(s);
    if (s.t.pipe_nt == 128)
        return s.iso ? pipe_grid_query<true, 128>(s) : pipe_grid_query<false, 128>(s);
    return s.iso ? pipe_grid_query<true, 256>(s) : pipe_grid_query<false, 256>(s);
}
// the update pass is grid-stride: at most one resident wave of workgroups (occupancy x CUs), so no
// workgroup waits for a slot behind the others' whole node ranges
template <int U, bool XF>
unsigned update_resident()
{
    int dev = 0, bpc = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k_pcg_update_tiles<U, XF, false>, kUpdThreads, 0);
    const unsigned r = (unsigned)((bpc > 0 ? bpc : 1) * (cus > 0 ? cus : 1));
    return r < kMaxUpdateBlocks ? r : kMaxUpdateBlocks;
}

// flush: the grid of the lazy-x instantiation (its own occupancy); the consumers of the update's r.r / r.z
// shares ask with the flag of the iteration that produced them
unsigned fast_update_blocks(const DevSys &s, bool flush)
{
    static const unsigned resident[2] = {update_resident<1, false>(), update_resident<1, true>()};
    constexpr unsigned cap = kMaxUpdateBlocks;
    const unsigned res = std::min(resident[flush ? 1 : 0], cap);
    const unsigned g = grid_for(s.N, kUpdThreads);
    return g < res ? (g ? g : 1u) : res;
}

// workgroup size of the one-tile-per-workgroup per-tet kernel (k_keff_tiles)
static int tile_threads() { return 256; }

void fast_keff_ds(const DevSys &s, const float *x, float *y, bool sanitize, const Ctl *ctl, double *part,
                  hipStream_t st)
{
    (void)ctl;
    (void)part;
    if (s.N == 0)
        return;
    if (s.t.ntiles)
    {
        PcgArgs none{};
        const int nt = tile_threads();
        if (s.iso)
            sanitize ? launch_tiles<true, true, 0>(s, x, none, nt, st) : launch_tiles<true, false, 0>(s, x, none, nt, st);
        else
            sanitize ? launch_tiles<false, true, 0>(s, x, none, nt, st)
                     : launch_tiles<false, false, 0>(s, x, none, nt, st);
    }
    const unsigned g = grid_for(s.N, 256);
    if (sanitize)
        k_keff_finalize<true><<<g, 256, 0, st>>>(s, x, y);
    else
        k_keff_finalize<false><<<g, 256, 0, st>>>(s, x, y);
}

// FAST search directions rotate over four buffers: p_j (iteration j's) lives in {p, p2, p3, p4}[(j + 1) % 4],
// so iteration `it` reads p_old from [it % 4] (the prologue's p is in p) and writes the new p to
// [(it + 1) % 4], and the last kXLag directions stay readable for the lazy x update
inline float *fast_p_buf(cwf_hip_system *h, unsigned k)
{
    float *const b[4] = {h->p, h->p2, h->p3, h->p4};
    return b[k % 4u];
}
inline float *fast_p_old(cwf_hip_system *h, unsigned it) { return fast_p_buf(h, it); }
inline float *fast_p_new(cwf_hip_system *h, unsigned it) { return fast_p_buf(h, it + 1u); }
static_assert(kXLag <= 4, "p_(it - lag + 1) .. p_it must still be in the four rotating buffers");
inline PBufs fast_p_bufs(cwf_hip_system *h) { return PBufs{{h->p, h->p2, h->p3, h->p4}}; }

// CWF_XLAG=1..4 (diagnostic): iterations per lazy x update (default kXLag)
static unsigned x_lag()
{
    static const unsigned v = [] {
        const char *e = knob("CWF_XLAG");
        const int k = e ? atoi(e) : (int)kXLag;
        return (unsigned)(k < 1 ? 1 : k > (int)kXLag ? (int)kXLag : k);
    }();
    return v;
}

// iteration j's update applies the lazy x terms
inline bool x_flush_iter(unsigned j) { return (j + 1u) % x_lag() == 0u; }

// the lazy x terms of the iterations after the last flush: j = n - n % lag .. n - 1, n = completed
// iterations (the device control block's count, so the host needs no iteration count)
__global__ __launch_bounds__(256) void k_x_flush(DevSys s, const float *__restrict__ rhs, float *__restrict__ x,
                                                 const Ctl *__restrict__ ctl, PBufs pb, unsigned lag)
{
    const unsigned n_it = (unsigned)ctl->iterations, j0 = n_it - n_it % lag;
    if (j0 == n_it)
        return;
    for (uint32_t n = blockIdx.x * 256 + threadIdx.x; n < s.Nown; n += gridDim.x * 256)
    {
        float xv[3] = {x[3u * n + 0], x[3u * n + 1], x[3u * n + 2]};
        for (unsigned j = j0; j < n_it; ++j)
        {
            const float *pj = pb.p[(j + 1u) % 4u];
            const float a = (float)ctl->alpha_h[j % kXLag];
#pragma unroll
            for (int k = 0; k < 3; ++k)
                xv[k] = fmaf(a, pj[3u * n + k], xv[k]);
        }
        const uint32_t mk = s.mask[n];
#pragma unroll
        for (int k = 0; k < 3; ++k)
        {
            if (mk & (1u << k))
                xv[k] = rhs[3u * n + k];
            x[3u * n + k] = xv[k];
        }
    }
}

// x / r / z of the update pass are stored write-through (store3; C2 +2.7% PCG it/s, C3 neutral)
static bool update_write_through() { return true; }

// iteration `it`: residual step of it-1's update (beta, convergence) + p_new + tile partials + p.Ap shares
void fast_tiles_pcg(cwf_hip_system *h, unsigned it, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    const DevSys &s = h->ds;
    if (!s.t.ntiles)
        return;
    const unsigned abl = 0u;
    // beta / convergence: a single handle folds the update kernel's per-workgroup {r.r, r.z} shares
    // directly; a shard reads the all-gathered per-rank pairs
    // lzr: the lattice kernel forms z from r (pa.z carries r)
    const float *pz = s.t.lzr ? h->r : h->z;
    PcgArgs pa = fast_direct_fold(h)
                     ? PcgArgs{pz, h->ctl, h->part0, h->part1, h->part2,
                               fast_update_blocks(s, it && x_flush_iter(it - 1u)), 1u, it, h->hist, abl,
                               fast_p_new(h, it)}
                     : PcgArgs{pz, h->ctl, h->part0, h->g_rrz, h->g_rrz + 1,
                               (unsigned)h->nranks, 2u, it, h->hist, abl, fast_p_new(h, it)};
    if (s.iso)
        launch_tiles<true, false, 1>(s, fast_p_old(h, it), pa, tile_threads(), st, e0, e1);
    else
        launch_tiles<false, false, 1>(s, fast_p_old(h, it), pa, tile_threads(), st, e0, e1);
}

void fast_update_pcg(cwf_hip_system *h, const float *rhs, unsigned it, hipStream_t st)
{
    const DevSys &s = h->ds;
    const bool direct = fast_direct_fold(h);
    const bool xf = x_flush_iter(it);
    const bool lat = s.t.lcls != nullptr;
    const auto k = lat && s.t.lzr ? (xf ? k_pcg_update_tiles<1, true, true, true> : k_pcg_update_tiles<1, false, true, true>)
                   : lat ? (xf ? k_pcg_update_tiles<1, true, true> : k_pcg_update_tiles<1, false, true>)
                         : (xf ? k_pcg_update_tiles<1, true, false> : k_pcg_update_tiles<1, false, false>);
    k<<<fast_update_blocks(s, xf), kUpdThreads, 0, st>>>(
        s, rhs, h->inv6, h->inv, h->x, h->r, h->z, fast_p_old(h, it), fast_p_new(h, it), h->ctl,
        direct ? h->part0 : h->g_pap, direct ? fast_tile_blocks(s) : (unsigned)h->nranks, h->part1, h->part2, it,
        update_write_through(), fast_p_bufs(h), x_lag());
}

void fast_flush_x(cwf_hip_system *h, const float *rhs, hipStream_t st)
{
    const DevSys &s = h->ds;
    if (!s.Nown)
        return;
    const unsigned g = std::min<unsigned>(grid_for(s.Nown, 256), 2048u);
    k_x_flush<<<g, 256, 0, st>>>(s, rhs, h->x, h->ctl, fast_p_bufs(h), x_lag());
}

// diagnostic: `reps` PCG-mode tiles launches with side-effect-free preambles (ablation bits | 32)
void fast_tiles_pcg_dry(cwf_hip_system *h, unsigned abl, int reps, hipStream_t st)
{
    const DevSys &s = h->ds;
    PcgArgs pa{s.t.lzr ? h->r : h->z, h->ctl, h->part0, h->g_rrz, h->g_rrz + 1, (unsigned)h->nranks, 2u, 1u,
               h->hist, abl | 32u};
    for (int i = 0; i < reps; ++i)
        launch_tiles<true, false, 1>(s, h->p, pa, tile_threads(), st);
}

// ---- the fused lattice iteration (lattice_fused.inc) --------------------------------------------------------
unsigned pcg_lattice_resident_count(const DevSys &s) { return lattice_resident_count(s); }

// CWF_FUSED=0: the two-kernel iteration on a structured block; CWF_FUSED_MAXWG: the largest grid that fuses (every
// workgroup folds five shares of each of the previous launch's workgroups)
bool fast_fused(const cwf_hip_system *h)
{
    const DevTiles &t = h->ds.t;
    if (!(h->mode == CWF_MODE_FAST && t.lat && t.lcls && t.lcz && h->r2 && h->fsh && h->g_fsh && t.ntiles))
        return false;
    if (h->fused_grid == 0 || h->fused_items != t.lnwork)  // per handle and plan (attach re-plans a shard's items)
    {
        cwf_hip_system *m = const_cast<cwf_hip_system *>(h);
        const char *on = knob("CWF_FUSED"), *cap = knob("CWF_FUSED_MAXWG");
        m->fused_grid = pcg_lattice_grid(h->ds, cap && atoi(cap) > 0 ? (unsigned)atoi(cap) : 1024u);
        m->fused_items = t.lnwork;
        // default: fused where one round of workgroups covers the work items (C2 fused 46.6k vs two-kernel 46.9k
        // PCG it/s, same box: one launch and one exchange per iteration for the same time). Beyond one round the
        // persistent walk (234-248 VGPRs, 2 waves/SIMD) loses to the two kernels: C3 8.3k vs 10.8k it/s
        // (profiles/r05b). CWF_FUSED=2 forces it, 0 turns it off
        const int v = on ? atoi(on) : 1;
        m->fused_on = v == 2 || (v == 1 && m->fused_grid >= t.lnwork);
    }
    return h->fused_on;
}

namespace
{
#if CWF_ABLATION
// diagnostic (ablation build): CWF_FUSED_TRACE=path appends the stamps of one launch (CWF_FUSED_TRACE_IT, default
// 50) of every solve: one line per workgroup "wg kind|planes<<8 hw_id xcc_id t0 t1 t2 t3 t4" (s_memrealtime, 100 MHz)
uint64_t *g_ftrace = nullptr;
unsigned g_ftrace_n = 0;
uint64_t *fused_trace_buffer(const cwf_hip_system *h)
{
    if (!knob("CWF_FUSED_TRACE"))
        return nullptr;
    if (g_ftrace_n < h->fused_grid)
    {
        if (g_ftrace)
            (void)hipFree(g_ftrace);
        g_ftrace = nullptr;
        if (hipMalloc(reinterpret_cast<void **>(&g_ftrace), 128ull * h->fused_grid) != hipSuccess)
            return nullptr;
        g_ftrace_n = h->fused_grid;
    }
    return g_ftrace;
}
void fused_trace_dump(cwf_hip_system *h, unsigned it, hipStream_t st)
{
    const char *path = knob("CWF_FUSED_TRACE"), *at = knob("CWF_FUSED_TRACE_IT");
    if (!path || !g_ftrace || it != (unsigned)(at ? atoi(at) : 50))
        return;
    std::vector<uint64_t> v(16ull * h->fused_grid);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(v.data(), g_ftrace, v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return;
    if (FILE *f = std::fopen(path, "a"))
    {
        std::fprintf(f, "# launch %u grid %u\n", it + 1u, h->fused_grid);
        for (unsigned b = 0; b < h->fused_grid; ++b)
        {
            const uint64_t *w = &v[16ull * b];
            std::fprintf(f, "%u %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", b,
                         (unsigned long long)w[5], (unsigned long long)w[6], (unsigned long long)w[7],
                         (unsigned long long)w[0], (unsigned long long)w[1], (unsigned long long)w[2],
                         (unsigned long long)w[3], (unsigned long long)w[4], (unsigned long long)w[8],
                         (unsigned long long)w[9], (unsigned long long)w[10], (unsigned long long)w[11],
                         (unsigned long long)w[12], (unsigned long long)w[13]);
        }
        std::fclose(f);
    }
}
#endif
// launch j of the fused iteration: r_j -> {r2, r}[j & 1], Ap_j -> {Ap, ap2}[j & 1], p_j -> p[(j + 1) % 4], shares
// -> fsh[j & 1]; launch j reads launch j - 1's (launch 0 reads r from r and Ap from ap2, zeroed at init)
FusedArgs fused_args(cwf_hip_system *h, unsigned j)
{
    const unsigned W = h->ds.t.lnwork;
    float *const R[2] = {h->r2, h->r}, *const A[2] = {h->Ap, h->ap2};
    FusedArgs fa{};
    fa.ctl = h->ctl;
    fa.sstride = W;
    fa.grid = h->fused_grid;
    if (h->sharded())  // every rank folds the all-gathered rank totals, in rank order
    {
        fa.sin = h->g_fsh;
        if (h->px_agreed == 1)  // PEER in-kernel: the totals land in the mailbox's gather area (previous epoch)
        {
            const double *gp = nullptr;
            peer_fused_args(h, j, fa.pe, &gp);
            fa.px = 1;
            fa.sin = gp;
        }
        fa.nin = (unsigned)h->nranks;
        fa.sin_stride = 1;
        fa.sis = kFusedSlot;
    }
    else
    {
        fa.sin = h->fsh + (size_t)((j + 1u) & 1u) * 5 * W;
        fa.nin = h->fused_grid;
        fa.sin_stride = W;
        fa.sis = 1;
    }
    fa.sout = h->fsh + (size_t)(j & 1u) * 5 * W;
    fa.j = j;
    fa.hist = h->hist;
    fa.rin = R[(j + 1u) & 1u];
    fa.rout = R[j & 1u];
    fa.ain = A[(j + 1u) & 1u];
    fa.aout = A[j & 1u];
    fa.pin = fast_p_buf(h, j);
    fa.pout = fast_p_buf(h, j + 1u);
    fa.x = h->x;
    fa.trace = nullptr;
#if CWF_ABLATION
    fa.trace = fused_trace_buffer(h);
#endif
    return fa;
}
}  // namespace

void fast_fused_init(cwf_hip_system *h, const float *rhs, double rel_tol, hipStream_t st, bool launch0)
{
    const DevSys &s = h->ds;
    const uint32_t nbD = fast_dot_blocks(s.D);
    fast_block_inverse(h, st);
    fast_keff(h, h->x, h->Ap, true, nullptr, nullptr, st);
    launch_init_residual(h, rhs, st);  // r_0 = rhs - A x (Dirichlet: x = rhs, r = 0) into h->r
    fast_dot(rhs, rhs, nullptr, s.D, h->part0, nullptr, st);
    fast_dot(h->r, h->r, nullptr, s.D, h->part1, nullptr, st);
    fast_init_scalars_strided(h, h->part0, h->part1, nbD, 1u, rel_tol, st);
    // launch 0 reads p_(-1) and Ap_(-1) (times beta = alpha = 0): zero, so no stale non-finite value enters
    if (launch0)  // (the resident solve runs its phase 0 itself)
        fast_fused_launch0(h, st);
}

void fast_fused_iteration(cwf_hip_system *h, unsigned it, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    launch_pcg_lattice(h->ds, fused_args(h, it + 1u), st, e0, e1);
#if CWF_ABLATION
    fused_trace_dump(h, it, st);
#endif
}

void fast_fused_launch0(cwf_hip_system *h, hipStream_t st)
{
    (void)hipMemsetAsync(h->p, 0, sizeof(float) * h->ds.D, st);
    (void)hipMemsetAsync(h->ap2, 0, sizeof(float) * h->ds.D, st);
    launch_pcg_lattice(h->ds, fused_args(h, 0), st, nullptr, nullptr);
}

// a shard's ghost class bytes from their owners (once per handle, before its first fused solve): the owned classes
// as floats in tmp's x components, a halo, and the ghosts' back into lcls (a ghost's local class is a boundary type
// of the shard's sub-lattice; its owner's is the node's class in the whole block, the one its z_j is formed with)
__global__ __launch_bounds__(256) void k_cls_out(const uint8_t *__restrict__ cls, uint32_t n, float *__restrict__ t)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        t[3u * i] = (float)cls[i];
}
__global__ __launch_bounds__(256) void k_cls_in(const float *__restrict__ t, uint32_t n0, uint32_t n1,
                                                uint8_t *__restrict__ cls)
{
    for (uint32_t i = n0 + blockIdx.x * 256u + threadIdx.x; i < n1; i += gridDim.x * 256u)
        cls[i] = (uint8_t)t[3u * i];
}
void fast_fused_cls_out(cwf_hip_system *h, hipStream_t st)
{
    if (h->ds.Nown)
        k_cls_out<<<std::min<unsigned>(grid_for(h->ds.Nown, 256), 1024u), 256, 0, st>>>(h->ds.t.lcls, h->ds.Nown, h->tmp);
}
void fast_fused_cls_in(cwf_hip_system *h, hipStream_t st)
{
    if (h->ds.N > h->ds.Nown)
        k_cls_in<<<std::min<unsigned>(grid_for(h->ds.N - h->ds.Nown, 256), 1024u), 256, 0, st>>>(
            h->tmp, h->ds.Nown, h->ds.N, const_cast<uint8_t *>(h->ds.t.lcls));
}

// a shard's launch j: its Ap_j (the vector the exchange after it carries) and its rank totals into g_fsh[rank]
float *fast_fused_ap(cwf_hip_system *h, unsigned j) { return (j & 1u) ? h->ap2 : h->Ap; }
void fast_fused_rank_totals(cwf_hip_system *h, unsigned j, hipStream_t st)
{
    const unsigned W = h->ds.t.lnwork;
    k_fused_rank_totals<<<1, 256, 0, st>>>(h->fsh + (size_t)(j & 1u) * 5 * W, h->fused_grid, W,
                                           h->g_fsh + (size_t)kFusedSlot * h->rank);
}
const double *fast_fused_shares(const cwf_hip_system *h, unsigned j, unsigned *stride, unsigned *count)
{
    *stride = h->ds.t.lnwork;
    *count = h->fused_grid;
    return h->fsh + (size_t)(j & 1u) * 5 * h->ds.t.lnwork;
}

// the convergence of the batch's last launch (it iterations enqueued: launch it's r)
void fast_fused_check(cwf_hip_system *h, unsigned it, hipStream_t st)
{
    k_fused_check<<<1, 256, 0, st>>>(fused_args(h, it + 1u));
}

void fast_fused_finish(cwf_hip_system *h, hipStream_t st)
{
    const uint32_t D = h->ds.D;
    if (D)
        k_fused_finish<<<std::min<unsigned>(grid_for(D, 256), 1024u), 256, 0, st>>>(h->ctl, h->r2, h->r, D);
}

void fast_check_pcg(cwf_hip_system *h, unsigned it, hipStream_t st)
{
    if (fast_direct_fold(h))
        k_pcg_check<<<1, 256, 0, st>>>(h->ctl, h->part1, h->part2,
                                       fast_update_blocks(h->ds, it && x_flush_iter(it - 1u)), 1u, it, h->hist);
    else
        k_pcg_check<<<1, 256, 0, st>>>(h->ctl, h->g_rrz, h->g_rrz + 1, (unsigned)h->nranks, 2u, it, h->hist);
}

void fast_block_inverse(cwf_hip_system *h, hipStream_t st)
{
    if (h->inv_fast && h->inv_sK == h->ds.sK && h->inv_sM == h->ds.sM)
        return;  // built for these scalars (C2: one 350-us fp64 setup per Newmark step saved)
    h->inv_fast = true;
    h->inv_sK = h->ds.sK;
    h->inv_sM = h->ds.sM;
    if (h->ds.hex)
        hex_block_jacobi(h, h->inv, st);
    else
        parity_block_jacobi(h, h->inv, st);
    if (h->ds.N)
        k_sym_inverse<<<grid_for(h->ds.N, 256), 256, 0, st>>>(h->ds.N, h->ds.mask, h->inv, h->inv6);
    if (h->ds.t.lcls)  // structured block: one representative node per (boundary class, mask)
        k_lat_class_inverse<<<1, 256, 0, st>>>(h->ds.t.lrep, h->inv6, h->inv, h->ds.t.lcinv6, h->ds.t.lcinv9,
                                               h->ds.t.lcz);
}

void fold_pair(const double *a, const double *b, uint32_t n, double *out, hipStream_t st)
{
    k_fold_pair<<<1, 1024, 0, st>>>(a, b, n, out);
}

// a single (unsharded) handle skips the per-rank fold kernels: every consumer workgroup refolds the
// producer's per-workgroup shares itself (<= 2048 doubles, L2-served), two launches fewer per iteration
// (C2 +11% PCG it/s against fold kernels, same-box A/B, round 2)
bool fast_direct_fold(const cwf_hip_system *h) { return !h->sharded(); }

void fast_fold_pap(cwf_hip_system *h, hipStream_t st)
{
    if (fast_direct_fold(h))
        return;
    fold_pair(h->part0, nullptr, fast_tile_blocks(h->ds), h->g_pap + h->rank, st);
}

unsigned fast_rrz_shares(const DevSys &s, unsigned it) { return fast_update_blocks(s, x_flush_iter(it)); }

void fast_fold_rrz(cwf_hip_system *h, unsigned it, hipStream_t st)
{
    if (fast_direct_fold(h))
        return;
    fold_pair(h->part1, h->part2, fast_update_blocks(h->ds, x_flush_iter(it)), h->g_rrz + 2 * h->rank, st);
}

void halo_pack(cwf_hip_system *h, const float *v, hipStream_t st, float *dst)
{
    if (!h->nsend)
        return;
    const uint64_t g = std::min<uint64_t>((h->nsend + 255) / 256, 1024);
    k_halo_pack<<<(unsigned)g, 256, 0, st>>>(h->send_idx, h->nsend, v, dst ? dst : h->sendbuf);
}

}  // namespace cwf

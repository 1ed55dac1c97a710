// lattice_common.hpp -- what the structured-block kernels share across translation units (spmv_tiles.hip: the
// K_eff / fused-iteration kernels; resident.hip: the resident solve): vector types, the control-block reads, the
// lattice element kinds and their class-table preconditioner, and the fused iteration's per-node arithmetic and
// scalar decision. Device code only, in an anonymous namespace per including unit.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

#include "cwf_internal.hpp"
#include "reduce.hpp"

namespace cwf
{
namespace
{
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef float f2 __attribute__((ext_vector_type(2)));

// Control-block words as vector (buffer) loads. A consumer prologue issues them with its gathers and the scalar
// fold's loads, and they return with those: one memory round trip. As scalar loads they cost one of their own, in
// front of the fold's loads (every s_waitcnt lgkmcnt(0) for a kernel argument the fold needs waits for them) or
// after the fold (where their value is used).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ctl_rsrc(const Ctl *c)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<Ctl *>(c), 0, (int)sizeof(Ctl), 0x00020000);
}
__device__ __forceinline__ double ctl_f64(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0),
                   hi = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4u, 0, 0);
    return __hiloint2double((int)hi, (int)lo);
}
// what residual_step reads of the control block for iteration it >= 1
struct CtlPre
{
    int active;
    double rho_old, tol;  // rho2[(it - 1) & 1], tol
};
__device__ __forceinline__ CtlPre ctl_prefetch(const Ctl *ctl, unsigned it)
{
    const __amdgpu_buffer_rsrc_t rs = ctl_rsrc(ctl);
    CtlPre p;
    p.active = (int)__builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)offsetof(Ctl, active), 0, 0);
    p.rho_old = ctl_f64(rs, (uint32_t)(offsetof(Ctl, rho2) + 8u * ((it - 1u) & 1u)));
    p.tol = ctl_f64(rs, (uint32_t)offsetof(Ctl, tol));
    return p;
}

constexpr int kLatNT = kLatThreads, kLatBX = kLatBrickX;
constexpr int kLatRing = 6;
// element kinds of a structured block: the offsets of a row (the node first, then (+d, -d) pairs), the cell's
// corner pairs (c, c') in (c, c') order with their offset index, and where each corner's pairs start
struct LatKuhn
{
    static constexpr int nOff = kLatOffsets, nPairs = kLatPairs, coefPairs = 9 * kLatOffsets;
    static constexpr const int (&off)[kLatOffsets][3] = kLatOff;
    static constexpr const int (&pair)[kLatPairs][2] = kLatPair;
    static constexpr const int (&pairOff)[kLatPairs] = kLatPairOff;
    static constexpr int pairStart[9] = {0, 8, 13, 18, 23, 28, 33, 38, 46};
};
struct LatHex
{
    static constexpr int nOff = kLatHexOffsets, nPairs = kLatHexPairs, coefPairs = 9 * kLatHexOffsets;
    static constexpr const int (&off)[kLatHexOffsets][3] = kLatHexOff;
    static constexpr int pair[kLatHexPairs][2] = {
#define P8(c) {c, 0}, {c, 1}, {c, 2}, {c, 3}, {c, 4}, {c, 5}, {c, 6}, {c, 7}
        P8(0), P8(1), P8(2), P8(3), P8(4), P8(5), P8(6), P8(7)
#undef P8
    };
    static constexpr const int (&pairOff)[kLatHexPairs] = kLatHexPairOff;
    static constexpr int pairStart[9] = {0, 8, 16, 24, 32, 40, 48, 56, 64};
};
constexpr uint32_t kLatOob3 = 0x15555555u;  // 12 * kLatOob3 = 0xFFFFFFFC: past any 12-B-per-node buffer
constexpr uint32_t kLatOob1 = 0x3FFFFFFFu;  // 4 * kLatOob1: past any 4-B-per-node buffer

// storage index of node (0, 0, k). AFF (the PCG loop on an affine block, DevTiles::lpstride): arithmetic, so no scalar
// load stands in front of the brick's first gathers. A template parameter, not a branch on lpstride: a uniform branch
// around the load in front of every plane's gathers splits the prologue into blocks whose joins make the waitcnt pass
// wait for gathers in flight.
template <bool AFF>
__device__ __forceinline__ uint32_t lat_plane(const DevTiles &T, const uint32_t *__restrict__ plane, int k)
{
    if constexpr (AFF)
        return (uint32_t)k * T.lpstride;
    else
        return plane[k];
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sized_rsrc(const void *base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
}

// ZR: the update pass does not store z; the K_eff pass forms z = M^-1 r from r and the node's class (boundary
// type << 3 | Dirichlet mask) with the class's block inverse, in exactly the update pass's arithmetic
// (k_pcg_update_tiles: the same unpacked 6 floats, DevTiles::lcz, the same FMA order, the masked components 0)
__device__ __forceinline__ void lat_z(const float4 A, const float2 B, uint32_t cls, const float r[3], float z[3])
{
    const float iv[9] = {A.x, A.y, A.z, A.y, A.w, B.x, A.z, B.x, B.y};
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const float zk = fmaf(iv[3 * k + 2], r[2], fmaf(iv[3 * k + 1], r[1], iv[3 * k] * r[0]));
        z[k] = (cls >> k) & 1u ? 0.0f : zk;
    }
}

enum
{
    kFR = 0,   // r_j . z_j (the direct rho_j)
    kFRR = 1,  // r_j . r_j
    kFPA = 2,  // p_j . Ap_j
    kFZA = 3,  // z_j . Ap_j
    kFAMA = 4, // Ap_j . M^-1 Ap_j
    kFusedShares = 5,
    kFusedSlot = 8  // doubles per rank of the all-gathered totals (the PEER step's slot)
};

// pcg.cpp:840-895 from the folded shares v of the launch (or resident phase) before j: alpha_(j-1), beta_j and the
// convergence of r_(j-1); block 0's thread 0 records them (and the history). Every caller holds the same v, so every
// workgroup takes the same decision. Returns false when the solve is over.
__device__ __forceinline__ bool fused_decide(Ctl *ctl, double *hist, unsigned j, const CtlPre &pre,
                                             const double v[kFusedShares], float *alpha_out, float *beta_out)
{
    const unsigned it = j - 1u;  // the completed updates r_(j-1) carries (launch 0 made none)
    const double res = sqrt(v[kFRR]);
    // the prologue tested r_0; r_(j-1) of an update is tested here (residual_step's place in the two-kernel loop)
    const bool conv = it > 0 && res <= pre.tol;
    const double rho = v[kFR], denom = v[kFPA];
    const bool derr = !conv && fabs(denom) < 1.0e-18;
    const bool rerr = !conv && !derr && fabs(rho) < 1.0e-18;
    const double alpha = (conv || derr || rerr) ? 0.0 : rho / denom;
    const double rho_next = rho - 2.0 * alpha * v[kFZA] + alpha * alpha * v[kFAMA];
    const double beta = (conv || derr || rerr) ? 0.0 : rho_next / rho;
    if (blockIdx.x == 0 && threadIdx.x == 0)
    {
        if (it > 0)
        {
            ctl->res = res;
            ctl->iterations = it;
            hist[it] = res;
        }
        ctl->denom = denom;
        if (conv)
        {
            ctl->converged = 1;
            ctl->active = 0;
        }
        else if (derr)  // pcg.cpp:846-849
        {
            ctl->error = CWF_ERR_DENOM_ZERO;
            ctl->error_iter = (int)it;
            ctl->active = 0;
        }
        else if (rerr)  // pcg.cpp:889-892
        {
            ctl->error = CWF_ERR_RHO_ZERO;
            ctl->error_iter = (int)it;
            ctl->active = 0;
        }
        else
        {
            ctl->alpha = alpha;
            ctl->alpha_last = alpha;
            ctl->rho2[it & 1u] = rho;
            ctl->beta = beta;
            ctl->beta_last = beta;
        }
    }
    *alpha_out = (float)alpha;
    *beta_out = (float)beta;
    return !(conv || derr || rerr);
}

// r_j, z_j, p_j of one entry (rz: the class's block inverse {a00 a01 a02 a11} {a12 a22})
__device__ __forceinline__ void fused_form(const float4 *czA, const float2 *czB, uint32_t cls, float alpha,
                                           float beta, const float r[3], const float a[3], const float p[3],
                                           float rn[3], float z[3], float pn[3])
{
#pragma unroll
    for (int c = 0; c < 3; ++c)
        rn[c] = (cls >> c) & 1u ? 0.f : fmaf(-alpha, a[c], r[c]);
    lat_z(czA[cls], czB[cls], cls, rn, z);
#pragma unroll
    for (int c = 0; c < 3; ++c)
        pn[c] = fmaf(beta, p[c], z[c]);
}

// the dots of one owned row (row value a = Ap_j, the node's p_j, z_j and class)
__device__ __forceinline__ void fused_row_dots(const float4 *czA, const float2 *czB, uint32_t cls, const float u[3],
                                               const float z[3], const float a[3], double d[kFusedShares])
{
    float am[3], w[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
        am[c] = (cls >> c) & 1u ? 0.f : a[c];
    lat_z(czA[cls], czB[cls], cls, am, w);
    // each node's 3-term products in fp32 (one FMA chain), fp64 across nodes: the tiles kernels' p.Ap convention. The
    // per-component fp64 form (two conversions, a multiply and an add per term, 41 fp64 operations per node) was a
    // third of the launch's VALU time (half-rate fp64)
    d[kFPA] += (double)fmaf(u[2], a[2], fmaf(u[1], a[1], u[0] * a[0]));
    d[kFZA] += (double)fmaf(z[2], am[2], fmaf(z[1], am[1], z[0] * am[0]));
    d[kFAMA] += (double)fmaf(am[2], w[2], fmaf(am[1], w[1], am[0] * w[0]));
}

__device__ __forceinline__ void fused_entry_dots(const float rn[3], const float z[3], double d[kFusedShares])
{
    d[kFR] += (double)fmaf(rn[2], z[2], fmaf(rn[1], z[1], rn[0] * z[0]));
    d[kFRR] += (double)fmaf(rn[2], rn[2], fmaf(rn[1], rn[1], rn[0] * rn[0]));
}

}  // namespace
}  // namespace cwf

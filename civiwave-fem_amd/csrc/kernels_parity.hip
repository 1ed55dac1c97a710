// kernels_parity.hip -- reference-order (bit-exact) kernels for gfx950.
//
// Every fold reproduces /root/reference/src/gpu/pcg.cpp in order:
//  * node-centric gather over the ascending node->element CSR reproduces the scatter-add of
//    pcg.cpp:653-661 (an fp64 accumulator per DOF that receives element contributions in
//    ascending element order, starting at +0.0);
//  * element math is fp64 on fp32 inputs with the reference operand order; structural zeros
//    of B (and of an isotropic D) are skipped, which is exact: every fold starts at +0.0, a
//    round-to-nearest sum that starts at +0.0 is never -0.0, so adding a +-0 term is a no-op;
//  * this TU is compiled with -ffp-contract=off (no FMA contraction), IEEE fp64 div/sqrt.
#include "cwf_internal.hpp"
#include "knobs.hpp"

#include <algorithm>
#include <type_traits>

namespace cwf
{
namespace
{

constexpr int kBlock = 256;
constexpr int kMaxLdsMaterials = 16;

struct Grad
{
    float g[12];  // g[3a+k]
    uint32_t c[4];
};

__device__ __forceinline__ void load_erec(const uint4 *__restrict__ erec, uint32_t e, Grad &r)
{
    const uint4 q0 = erec[4u * e + 0u];
    const uint4 q1 = erec[4u * e + 1u];
    const uint4 q2 = erec[4u * e + 2u];
    const uint4 q3 = erec[4u * e + 3u];
    r.c[0] = q0.x;
    r.c[1] = q0.y;
    r.c[2] = q0.z;
    r.c[3] = q0.w;
    r.g[0] = __uint_as_float(q1.x);
    r.g[1] = __uint_as_float(q1.y);
    r.g[2] = __uint_as_float(q1.z);
    r.g[3] = __uint_as_float(q1.w);
    r.g[4] = __uint_as_float(q2.x);
    r.g[5] = __uint_as_float(q2.y);
    r.g[6] = __uint_as_float(q2.z);
    r.g[7] = __uint_as_float(q2.w);
    r.g[8] = __uint_as_float(q3.x);
    r.g[9] = __uint_as_float(q3.y);
    r.g[10] = __uint_as_float(q3.z);
    r.g[11] = __uint_as_float(q3.w);
}

// stress = D strain (pcg.cpp:632-640). ISO: 12-entry table [D00 D01 D02 D10 D11 D12 D20 D21 D22 D33 D44 D55].
template <bool ISO>
__device__ __forceinline__ void stress_fp64(const double *Dm, const double e[6], double s[6])
{
    if constexpr (ISO)
    {
#pragma unroll
        for (int r = 0; r < 3; ++r)
        {
            double sum = 0.0;
            sum += Dm[3 * r + 0] * e[0];
            sum += Dm[3 * r + 1] * e[1];
            sum += Dm[3 * r + 2] * e[2];
            s[r] = sum;
        }
#pragma unroll
        for (int r = 3; r < 6; ++r)
        {
            double sum = 0.0;
            sum += Dm[6 + r] * e[r];
            s[r] = sum;
        }
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 6; ++r)
        {
            double sum = 0.0;
#pragma unroll
            for (int c = 0; c < 6; ++c)
                sum += Dm[6 * r + c] * e[c];
            s[r] = sum;
        }
    }
}

// f[col] = (sum_r B[r][col] sigma_r) * vol for one corner (pcg.cpp:643-651), the term the scatter adds
__device__ __forceinline__ void corner_force(double ax, double ay, double az, const double sig[6], double vol,
                                             double f[3])
{
    double fx = 0.0, fy = 0.0, fz = 0.0;
    fx += ax * sig[0];
    fx += ay * sig[3];
    fx += az * sig[5];
    fy += ay * sig[1];
    fy += ax * sig[3];
    fy += az * sig[4];
    fz += az * sig[2];
    fz += ay * sig[4];
    fz += ax * sig[5];
    f[0] = fx * vol;
    f[1] = fy * vol;
    f[2] = fz * vol;
}

// a tet's operands: its record (corner ids, f32 gradients), the f32 corner values and (SANITIZE) the corners'
// Dirichlet masks, its volume and material. Gathered first so a pipelined kernel can have them in flight while it
// works on the previous tet (k_keff_parity_tile).
template <bool SANITIZE>
struct TetIn
{
    Grad G;
    float u[12];
    uint32_t mk[SANITIZE ? 4 : 1];
    float vol;
    uint32_t mat;
};

// the loads of the corner values (needs G.c) and of the volume and material
template <bool SANITIZE>
__device__ __forceinline__ void tet_gather(const DevSys &s, const float *__restrict__ x, uint32_t e, TetIn<SANITIZE> &t)
{
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        const uint32_t m = t.G.c[q];
        const float *xp = x + 3u * m;
        t.u[3 * q + 0] = xp[0];
        t.u[3 * q + 1] = xp[1];
        t.u[3 * q + 2] = xp[2];
        if constexpr (SANITIZE)
            t.mk[q] = s.mask[m];
    }
    t.vol = s.vol[e];
    t.mat = s.mat[e];
}

// strain / stress of a tet from its operands (pcg.cpp:574-640): gradients g{x,y,z}[4] in fp64, stress sig[6]
template <bool ISO, bool SANITIZE>
__device__ __forceinline__ void tet_stress_in(const DevSys &s, const TetIn<SANITIZE> &t, const double *dtab,
                                              double gx[4], double gy[4], double gz[4], double sig[6])
{
    constexpr int kTab = ISO ? 12 : 36;
    const uint32_t mi = t.mat;
    double u[12];
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        double u0 = (double)t.u[3 * q + 0], u1 = (double)t.u[3 * q + 1], u2 = (double)t.u[3 * q + 2];
        if constexpr (SANITIZE)
        {
            const uint32_t mk = t.mk[q];
            if (mk & 1u)
                u0 = 0.0;
            if (mk & 2u)
                u1 = 0.0;
            if (mk & 4u)
                u2 = 0.0;
        }
        u[3 * q + 0] = u0;
        u[3 * q + 1] = u1;
        u[3 * q + 2] = u2;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        gx[q] = (double)t.G.g[3 * q + 0];
        gy[q] = (double)t.G.g[3 * q + 1];
        gz[q] = (double)t.G.g[3 * q + 2];
    }
    double eps[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        eps[0] += gx[q] * u[3 * q + 0];
        eps[1] += gy[q] * u[3 * q + 1];
        eps[2] += gz[q] * u[3 * q + 2];
        eps[3] += gy[q] * u[3 * q + 0];
        eps[3] += gx[q] * u[3 * q + 1];
        eps[4] += gz[q] * u[3 * q + 1];
        eps[4] += gy[q] * u[3 * q + 2];
        eps[5] += gz[q] * u[3 * q + 0];
        eps[5] += gx[q] * u[3 * q + 2];
    }
    if (mi < (uint32_t)kMaxLdsMaterials)
        stress_fp64<ISO>(dtab + kTab * mi, eps, sig);
    else
    {
        double tab[36];
        for (int t2 = 0; t2 < kTab; ++t2)
        {
            uint32_t src;
            if constexpr (ISO)
                src = t2 < 9 ? (t2 / 3) * 6 + (t2 % 3) : (t2 - 6) * 7;
            else
                src = t2;
            tab[t2] = s.dmat[36u * mi + src];
        }
        stress_fp64<ISO>(tab, eps, sig);
    }
}

template <bool ISO>
__device__ __forceinline__ void stage_dtab(const DevSys &s, double *dtab)
{
    constexpr int kTab = ISO ? 12 : 36;
    const uint32_t nm = s.M < kMaxLdsMaterials ? s.M : kMaxLdsMaterials;
    for (uint32_t i = threadIdx.x; i < nm * kTab; i += kBlock)
    {
        const uint32_t m = i / kTab, t = i % kTab;
        uint32_t src;
        if constexpr (ISO)
            src = t < 9 ? (t / 3) * 6 + (t % 3) : (t - 6) * 7;  // (3,3) (4,4) (5,5)
        else
            src = t;
        dtab[i] = s.dmat[36u * m + src];
    }
}

// A 256-thread workgroup of consecutive nodes covers 768 DOFs = three whole 256-DOF reduction chunks (workgroup b:
// chunks 3b .. 3b + 2), so the node kernels that produce a dot's operands also produce its chunk partials. Every
// thread stages the fp64 products of its own DOFs in LDS (chunk k at row 257 k, against bank conflicts); a
// product of two fp32 values is exact in fp64, so staging (double)a * (double)b is bitwise the term
// pcg.cpp:189-199 adds. Lanes 0..2 then fold one chunk each, sequentially in DOF order, adds only (the chains
// are the critical path: staging the fp32 operands and forming the products in the chains measured 22 us for
// the C2 update pass against 14 us without the partials). DOFs of nodes at or past `nlim` (the owned nodes of
// a shard, or N) are staged as +0.0, an exact no-op in a fold from +0.0. NV = 2: two dots per DOF, {ab, ac}.
// Streamed scalar folds (the single-handle PCG loop, 256-DOF chunks; kernels below): a producing pass stores each
// chunk partial as a tagged 16-B granule {partial lo, hi, tag, 0} in ONE write-through (sc1) store, and its
// workgroup 0 polls them (sc1 loads, served past L1 and the per-XCD L2) and folds them in chunk order while the other
// workgroups still produce: each granule carries its own tag, so no counter and no ordering between granules is
// needed (the hand-off form of resident.hip / MI355X_MICROARCH.md). Granule of chunk k, operand c: NC k + c.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gran_rsrc(const double *g)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(g), 0, -1, 0x00020000);
}
__device__ __forceinline__ void gran_store(__amdgpu_buffer_rsrc_t rs, uint32_t idx, double v, uint32_t tag)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const u32x4 w = {(uint32_t)b, (uint32_t)(b >> 32), tag, 0u};
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, 16u * idx, 0, 16);  // sc1: write-through
}

constexpr int kChunkRow = 257;
template <int NV>
using ChunkTerm = std::conditional_t<NV == 2, double2, double>;

__device__ __forceinline__ uint32_t chunk_slot(uint32_t d)  // LDS index of the workgroup's d-th DOF
{
    return (d >> 8) * kChunkRow + (d & 255u);
}

template <int NV>
__device__ __forceinline__ void wg_chunk_partials(const ChunkTerm<NV> *st, uint32_t chunks, double *pab, double *pac,
                                                  uint32_t blk, const double *gran = nullptr, uint32_t tag = 0)
{
    if (threadIdx.x >= 3u)
        return;
    const uint32_t k = 3u * blk + threadIdx.x;
    if (k >= chunks)
        return;
    const ChunkTerm<NV> *row = st + threadIdx.x * kChunkRow;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 16
    for (uint32_t i = 0; i < 256u; ++i)
    {
        if constexpr (NV == 2)
        {
            const double2 t = row[i];
            s0 += t.x;
            s1 += t.y;
        }
        else
            s0 += row[i];
    }
    if (gran)  // streamed: the granules the folding workgroup polls
    {
        const __amdgpu_buffer_rsrc_t rs = gran_rsrc(gran);
        gran_store(rs, NV * k, s0, tag);
        if constexpr (NV == 2)
            gran_store(rs, NV * k + 1u, s1, tag);
        return;
    }
    pab[k] = s0;
    if constexpr (NV == 2)
        pac[k] = s1;
}

// K_eff x (pcg.cpp:505-694) over node tiles: workgroup b owns nodes [256 b, 256 b + 256) (thread t node 256 b + t)
// and walks the tile's incident tets in ascending element order, 256 at a time. In each batch thread t computes one
// tet's strain and stress in fp64 (the reference's operand order) and the corner forces of its corners inside the
// tile, each the exact fp64 term pcg.cpp:643-661 adds, into LDS; then every node thread adds its incidences that
// fall in the batch, in ascending element order, to its fp64 accumulators (started at +0.0). Batches run in
// element order, so each node's sum is the reference's left fold over its incident elements: y is bit-identical.
// Then the mass term, the Dirichlet identity rows and the cast (pcg.cpp:664-691); DOT (the PCG loop): the chunk
// partials of x . y (the p . Ap of pcg.cpp:840), three whole 256-DOF chunks per workgroup (wg_chunk_partials).
// Halo tets (those with corners in two tiles) are computed once per tile that needs them (~2.4 tets per tet on a
// Kuhn block); nothing but y leaves the workgroup. Round 3 stored every corner force to HBM (96 B per tet written
// and read back by a node pass: 76 + 36 us on C2); round 2 gathered every incident tet per node (4x the element
// work, 293 us).
constexpr int kTileTets = 256;
constexpr int kIncAhead = 4;  // a node's next incidence entries held in registers
// The PCG loop's compact-tile instantiation (ISO, no sanitize, SET) is held to 128 VGPRs: 4 waves per SIMD instead
// of 3 at 132, no spill (C3 PARITY K_eff 1,260 -> 1,124 us, C2 121 -> 124 us, same box: profiles/r04zg_*); the
// others spill at 128 and keep their registers.
template <bool ISO, bool SANITIZE, bool DOT, bool SET>
__global__ __launch_bounds__(kBlock, ISO && !SANITIZE && SET ? 4 : 1) void k_keff_parity_tile(DevSys s, const float *__restrict__ x,
                                                             float *__restrict__ y, const Ctl *__restrict__ ctl,
                                                             double *__restrict__ pdot, uint32_t nlim,
                                                             uint32_t chunks)
{
    __shared__ double dtab[kMaxLdsMaterials * 36];
    __shared__ double fs[3][4 * kTileTets];  // [component][batch tet * 4 + corner]
    __shared__ double sxy[DOT ? 3 * kChunkRow : 1];
    if (ctl && !ctl->active)
        return;
    stage_dtab<ISO>(s, dtab);
    // XCD-aware tile order: consecutive tiles (which share halo tets) on one XCD
    const uint32_t ntile = gridDim.x, xcd = blockIdx.x & 7u, per = ntile >> 3, rem = ntile & 7u;
    const uint32_t tile = xcd * per + min(xcd, rem) + (blockIdx.x >> 3);
    // SET (compact tiles): the tile's nodes from ptile_nodes (pads are ~0 >= N); else 256 consecutive nodes
    const uint32_t n0 = tile * kBlock, n = SET ? s.ptile_nodes[n0 + threadIdx.x] : n0 + threadIdx.x;
    static_assert(!(SET && DOT), "compact tiles are not runs of consecutive DOFs");
    const uint32_t t0 = s.ptile_off[tile], nt = s.ptile_off[tile + 1] - t0;
    uint32_t j = 0, jend = 0;
    if (n < s.N)
    {
        j = s.off[n];
        jend = s.off[n + 1];
    }
    // the node's next kIncAhead incidence entries (tile-local tet << 2 | corner; ~0 past its last), refilled after
    // each batch's fold so their loads are in flight during the next batch's element work
    uint32_t qa[kIncAhead];
#pragma unroll
    for (int i = 0; i < kIncAhead; ++i)
        qa[i] = j + i < jend ? s.pinc[j + i] : 0xFFFFFFFFu;
    // software pipeline over batches: batch b's operands were gathered during batch b - 1; the next batch's record
    // is issued before this batch's math and its corner gathers before the fold
    const uint32_t tid = threadIdx.x;
    TetIn<SANITIZE> cur;
    uint32_t e_cur = tid < nt ? s.ptile_tets[t0 + tid] : 0u;
    if (tid < nt)
    {
        load_erec(s.erec, e_cur, cur.G);
        tet_gather<SANITIZE>(s, x, e_cur, cur);
    }
    uint32_t e_nxt = kTileTets + tid < nt ? s.ptile_tets[t0 + kTileTets + tid] : 0u;
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
    __syncthreads();  // dtab
    for (uint32_t base = 0; base < nt; base += kTileTets)
    {
        const bool has_nxt = base + kTileTets + tid < nt;
        TetIn<SANITIZE> nxt;
        if (has_nxt)
            load_erec(s.erec, e_nxt, nxt.G);
        const uint32_t e_nn = base + 2 * kTileTets + tid < nt ? s.ptile_tets[t0 + base + 2 * kTileTets + tid] : 0u;
        if (base + tid < nt)
        {
            double gx[4], gy[4], gz[4], sig[6];
            tet_stress_in<ISO, SANITIZE>(s, cur, dtab, gx, gy, gz, sig);
            const double vol = (double)cur.vol * s.sK;  // pcg.cpp:642
#pragma unroll
            for (int a = 0; a < 4; ++a)
                if (SET || cur.G.c[a] - n0 < (uint32_t)kBlock)  // a corner of this tile (SET: every corner)
                {
                    double f[3];
                    corner_force(gx[a], gy[a], gz[a], sig, vol, f);
                    const uint32_t sl = 4u * tid + (uint32_t)a;
                    fs[0][sl] = f[0];
                    fs[1][sl] = f[1];
                    fs[2][sl] = f[2];
                }
        }
        if (has_nxt)
            tet_gather<SANITIZE>(s, x, e_nxt, nxt);
        __syncthreads();
        // incidences are ascending in element order, so in tile-local tet order: the node's entries below lim are
        // this batch's, consumed in order
        const uint32_t lim = (base + kTileTets) << 2;
        int used = 0;
#pragma unroll
        for (int i = 0; i < kIncAhead; ++i)
            if (qa[i] < lim && used == i)
            {
                const uint32_t sl = qa[i] - (base << 2);
                acc0 += fs[0][sl];
                acc1 += fs[1][sl];
                acc2 += fs[2][sl];
                ++used;
            }
        j += (uint32_t)used;
        if (used == kIncAhead)  // more in this batch than the register window holds (rare): straight from memory
        {
            uint32_t q = j < jend ? s.pinc[j] : 0xFFFFFFFFu;
            while (q < lim)
            {
                const uint32_t sl = q - (base << 2);
                acc0 += fs[0][sl];
                acc1 += fs[1][sl];
                acc2 += fs[2][sl];
                ++j;
                q = j < jend ? s.pinc[j] : 0xFFFFFFFFu;
            }
        }
#pragma unroll
        for (int i = 0; i < kIncAhead; ++i)
            qa[i] = j + i < jend ? s.pinc[j + i] : 0xFFFFFFFFu;
        __syncthreads();
        cur = nxt;
        e_nxt = e_nn;
    }
    float yv[3] = {0.f, 0.f, 0.f}, xv[3] = {0.f, 0.f, 0.f};
    if (n < s.N)
    {
        const uint32_t mk = s.mask[n];
        const double m = (double)s.mass[n] * s.sM;
        const float x0 = x[3u * n + 0], x1 = x[3u * n + 1], x2 = x[3u * n + 2];
        const double s0 = (SANITIZE && (mk & 1u)) ? 0.0 : (double)x0;
        const double s1 = (SANITIZE && (mk & 2u)) ? 0.0 : (double)x1;
        const double s2 = (SANITIZE && (mk & 4u)) ? 0.0 : (double)x2;
        acc0 += m * s0;
        acc1 += m * s1;
        acc2 += m * s2;
        if (mk & 1u)
            acc0 = (double)x0;
        if (mk & 2u)
            acc1 = (double)x1;
        if (mk & 4u)
            acc2 = (double)x2;
        yv[0] = (float)acc0;
        yv[1] = (float)acc1;
        yv[2] = (float)acc2;
        y[3u * n + 0] = yv[0];
        y[3u * n + 1] = yv[1];
        y[3u * n + 2] = yv[2];
        xv[0] = x0;
        xv[1] = x1;
        xv[2] = x2;
    }
    if constexpr (DOT)
    {
        // the tile's chunks are 3 tile, 3 tile + 1, 3 tile + 2
        const bool own = n < nlim;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            sxy[chunk_slot(3u * threadIdx.x + k)] = own ? (double)xv[k] * (double)yv[k] : 0.0;
        __syncthreads();
        wg_chunk_partials<1>(sxy, chunks, pdot, nullptr, tile);
    }
}

__device__ void invert_spd_3x3(double m[9], double inv[9])
{
    // pcg.cpp:215-268
    const double kDetTol = 1.0e-12;
    auto det3 = [&]() {
        return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
               m[2] * (m[3] * m[7] - m[4] * m[6]);
    };
    double det = det3();
    if (fabs(det) < kDetTol)
    {
        const double md = fmax(fmax(m[0], m[4]), m[8]);
        const double eps = fmax(1.0e-6, md * 1.0e-6 + 1.0e-12);
        m[0] += eps;
        m[4] += eps;
        m[8] += eps;
        det = det3();
    }
    if (fabs(det) < kDetTol)
    {
        for (int i = 0; i < 9; ++i)
            inv[i] = 0.0;
        inv[0] = 1.0 / fmax(m[0], 1.0e-6);
        inv[4] = 1.0 / fmax(m[4], 1.0e-6);
        inv[8] = 1.0 / fmax(m[8], 1.0e-6);
        return;
    }
    const double id = 1.0 / det;
    inv[0] = (m[4] * m[8] - m[5] * m[7]) * id;
    inv[1] = (m[2] * m[7] - m[1] * m[8]) * id;
    inv[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    inv[3] = (m[5] * m[6] - m[3] * m[8]) * id;
    inv[4] = (m[0] * m[8] - m[2] * m[6]) * id;
    inv[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    inv[6] = (m[3] * m[7] - m[4] * m[6]) * id;
    inv[7] = (m[1] * m[6] - m[0] * m[7]) * id;
    inv[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

// Block-Jacobi inverse, one thread per node (pcg.cpp:270-408): the node's diagonal 3x3 block of
// every incident K_e in ascending element order, + m*s_M, fp64 inverse, constrained rows -> identity.
__global__ __launch_bounds__(kBlock) void k_block_jacobi_parity(DevSys s, float *__restrict__ inv_out)
{
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    double blk[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t j = s.off[n]; j < s.off[n + 1]; ++j)
    {
        const uint32_t inc = s.inc[j];
        const uint32_t e = inc >> 2, a = inc & 3u;
        const uint4 *rec = s.erec + 4u * e;
        const float *gf = reinterpret_cast<const float *>(rec + 1);
        const double gx = (double)gf[3 * a + 0], gy = (double)gf[3 * a + 1], gz = (double)gf[3 * a + 2];
        const double *Dm = s.dmat + 36u * s.mat[e];
        // nonzero rows of B column 3a+k, ascending: k=0 {0:gx,3:gy,5:gz} k=1 {1:gy,3:gx,4:gz} k=2 {2:gz,4:gy,5:gx}
        const int rows[3][3] = {{0, 3, 5}, {1, 3, 4}, {2, 4, 5}};
        const double vals[3][3] = {{gx, gy, gz}, {gy, gx, gz}, {gz, gy, gx}};
        double DB[6][3];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k)
            {
                double sum = 0.0;
#pragma unroll
                for (int t = 0; t < 3; ++t)
                    sum += Dm[6 * r + rows[k][t]] * vals[k][t];
                DB[r][k] = sum;
            }
        const double sv = (double)s.vol[e] * s.sK;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int k = 0; k < 3; ++k)
            {
                double sum = 0.0;
#pragma unroll
                for (int t = 0; t < 3; ++t)
                    sum += vals[i][t] * DB[rows[i][t]][k];
                blk[3 * i + k] += sum * sv;
            }
    }
    const double m = (double)s.mass[n] * s.sM;
    blk[0] += m;
    blk[4] += m;
    blk[8] += m;
    double iv[9];
    invert_spd_3x3(blk, iv);
    const uint32_t mk = s.mask[n];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (mk & (1u << k))
            for (int c = 0; c < 3; ++c)
                iv[3 * k + c] = (k == c) ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i)
        inv_out[9u * n + i] = (float)iv[i];
}

// Native hex8 block-Jacobi (FAST only; parity unpinned: the reference rejects hex8). One
// thread per node, incident hexes in ascending element order (inc = element << 3 | corner): the
// corner's diagonal 3x3 block of K_e = sum_gp |det J| B_a^T D B_a s_K in fp64 (2x2x2 Gauss), then the
// same m s_M diagonal, regularised fp64 inverse and constrained-row identity as the tet path.
__global__ __launch_bounds__(kBlock) void k_block_jacobi_hex(DevSys s, float *__restrict__ inv_out)
{
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    const double sg[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
                             {-1, -1, 1},  {1, -1, 1},  {1, 1, 1},  {-1, 1, 1}};
    const double r3 = 0.57735026918962576;  // 1 / sqrt(3)
    double blk[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t j = s.off[n]; j < s.off[n + 1]; ++j)
    {
        const uint32_t inc = s.inc[j];
        const uint32_t e = inc >> 3, a = inc & 7u;
        double X[8][3];
        for (int c = 0; c < 8; ++c)
        {
            const uint32_t v = s.hconn[8ull * e + c];
            X[c][0] = s.hcoord[3ull * v + 0];
            X[c][1] = s.hcoord[3ull * v + 1];
            X[c][2] = s.hcoord[3ull * v + 2];
        }
        const double *Dm = s.dmat + 36u * s.mat[e];
        for (int p = 0; p < 8; ++p)
        {
            const double q[3] = {(p & 1) ? r3 : -r3, (p & 2) ? r3 : -r3, (p & 4) ? r3 : -r3};
            double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, dNa[3] = {0, 0, 0};
            for (int c = 0; c < 8; ++c)
            {
                const double f0 = 1.0 + sg[c][0] * q[0], f1 = 1.0 + sg[c][1] * q[1], f2 = 1.0 + sg[c][2] * q[2];
                const double d0 = 0.125 * sg[c][0] * f1 * f2, d1 = 0.125 * f0 * sg[c][1] * f2,
                             d2 = 0.125 * f0 * f1 * sg[c][2];
                for (int m = 0; m < 3; ++m)
                {
                    J[m][0] += X[c][m] * d0;
                    J[m][1] += X[c][m] * d1;
                    J[m][2] += X[c][m] * d2;
                }
                if ((uint32_t)c == a)
                {
                    dNa[0] = d0;
                    dNa[1] = d1;
                    dNa[2] = d2;
                }
            }
            double A[3][3];
            A[0][0] = J[1][1] * J[2][2] - J[1][2] * J[2][1];
            A[0][1] = J[0][2] * J[2][1] - J[0][1] * J[2][2];
            A[0][2] = J[0][1] * J[1][2] - J[0][2] * J[1][1];
            A[1][0] = J[1][2] * J[2][0] - J[1][0] * J[2][2];
            A[1][1] = J[0][0] * J[2][2] - J[0][2] * J[2][0];
            A[1][2] = J[0][2] * J[1][0] - J[0][0] * J[1][2];
            A[2][0] = J[1][0] * J[2][1] - J[1][1] * J[2][0];
            A[2][1] = J[0][1] * J[2][0] - J[0][0] * J[2][1];
            A[2][2] = J[0][0] * J[1][1] - J[0][1] * J[1][0];
            const double det = J[0][0] * A[0][0] + J[0][1] * A[1][0] + J[0][2] * A[2][0];
            double g[3];
            for (int m = 0; m < 3; ++m)
                g[m] = (dNa[0] * A[0][m] + dNa[1] * A[1][m] + dNa[2] * A[2][m]) / det;
            // B_a (6x3), rows xx yy zz xy yz xz
            const double B[6][3] = {{g[0], 0, 0}, {0, g[1], 0}, {0, 0, g[2]},
                                    {g[1], g[0], 0}, {0, g[2], g[1]}, {g[2], 0, g[0]}};
            const double w = fabs(det) * s.sK;
            for (int i = 0; i < 3; ++i)
                for (int k = 0; k < 3; ++k)
                {
                    double sum = 0.0;
                    for (int r = 0; r < 6; ++r)
                    {
                        double db = 0.0;
                        for (int c = 0; c < 6; ++c)
                            db += Dm[6 * r + c] * B[c][k];
                        sum += B[r][i] * db;
                    }
                    blk[3 * i + k] += sum * w;
                }
        }
    }
    const double m = (double)s.mass[n] * s.sM;
    blk[0] += m;
    blk[4] += m;
    blk[8] += m;
    double iv[9];
    invert_spd_3x3(blk, iv);
    const uint32_t mk = s.mask[n];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (mk & (1u << k))
            for (int c = 0; c < 3; ++c)
                iv[3 * k + c] = (k == c) ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i)
        inv_out[9u * n + i] = (float)iv[i];
}

// ---- reductions (pcg.cpp:170-207): sequential fp64 fold inside each reduction_block chunk ----

// generic chunk size: one thread per chunk, sequential loads
template <int NV>
__global__ __launch_bounds__(kBlock) void k_dot_chunks_generic(const float *__restrict__ a,
                                                               const float *__restrict__ b,
                                                               const float *__restrict__ c, uint32_t D,
                                                               uint32_t B, uint32_t chunks, double *__restrict__ pab,
                                                               double *__restrict__ pac, const Ctl *__restrict__ ctl)
{
    if (ctl && !ctl->active)
        return;
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= chunks)
        return;
    const uint32_t beg = k * B, end = min(beg + B, D);
    double s0 = 0.0, s1 = 0.0;
    for (uint32_t i = beg; i < end; ++i)
    {
        const double av = (double)a[i];
        s0 += av * (double)b[i];
        if constexpr (NV == 2)
            s1 += av * (double)c[i];
    }
    pab[k] = s0;
    if constexpr (NV == 2)
        pac[k] = s1;
}

// chunk = 256 DOFs: a 256-thread workgroup per 32 chunks. The workgroup stages the 32 x 256 values of every
// operand through LDS with coalesced loads (rows padded to 257 floats, so the 32 folding lanes hit 32 different
// banks), then lane c of wave 0 folds chunk c sequentially, in DOF order (pcg.cpp:189-199); the fp32 x fp32
// products are exact in fp64. Values past D are staged as 0: +0.0 * +0.0 added to a fold that started at +0.0 is
// exact (such a fold is never -0.0), so the tail chunk equals the reference's shorter loop.
constexpr int kDotChunksPerBlock = 32;
constexpr int kDotRow = 257;
// (CPB chunks per block; no early return, so a persistent caller can loop over blocks with a barrier in between)
template <int NV, int CPB = kDotChunksPerBlock>
__device__ __forceinline__ void dot_chunks256(const float *__restrict__ a, const float *__restrict__ b,
                                              const float *__restrict__ c, uint32_t D, uint32_t chunks,
                                              double *__restrict__ pab, double *__restrict__ pac, uint32_t bx,
                                              const double *gran, uint32_t tag)
{
    __shared__ float sa[CPB * kDotRow];
    __shared__ float sb[CPB * kDotRow];
    __shared__ float sc[NV == 2 ? CPB * kDotRow : 1];
    const uint64_t base = (uint64_t)bx * CPB * 256u;
    // 16-B loads (4 DOFs per lane and step) when the operands are 16-B aligned (a caller's device pointer need
    // not be); a block's range starts 32 KB into the vector, the tail past D goes scalar
    const bool al = ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                      reinterpret_cast<uintptr_t>(NV == 2 ? c : a)) & 15u) == 0;
    for (uint32_t i = 4u * threadIdx.x; i < CPB * 256u; i += 1024u)
    {
        const uint64_t gi = base + i;
        const uint32_t l = (i >> 8) * kDotRow + (i & 255u);  // 4 consecutive DOFs stay in one row
        if (al && gi + 4u <= D)
        {
            const float4 va = *reinterpret_cast<const float4 *>(a + gi);
            const float4 vb = *reinterpret_cast<const float4 *>(b + gi);
            sa[l] = va.x, sa[l + 1] = va.y, sa[l + 2] = va.z, sa[l + 3] = va.w;
            sb[l] = vb.x, sb[l + 1] = vb.y, sb[l + 2] = vb.z, sb[l + 3] = vb.w;
            if constexpr (NV == 2)
            {
                const float4 vc = *reinterpret_cast<const float4 *>(c + gi);
                sc[l] = vc.x, sc[l + 1] = vc.y, sc[l + 2] = vc.z, sc[l + 3] = vc.w;
            }
        }
        else
            for (uint32_t u = 0; u < 4u; ++u)
            {
                const bool ok = gi + u < D;
                sa[l + u] = ok ? a[gi + u] : 0.0f;
                sb[l + u] = ok ? b[gi + u] : 0.0f;
                if constexpr (NV == 2)
                    sc[l + u] = ok ? c[gi + u] : 0.0f;
            }
    }
    __syncthreads();
    const uint32_t k = bx * CPB + threadIdx.x;
    if (threadIdx.x >= (uint32_t)CPB || k >= chunks)
        return;
    const float *ra = sa + threadIdx.x * kDotRow, *rb = sb + threadIdx.x * kDotRow;
    const float *rc = sc + (NV == 2 ? threadIdx.x * kDotRow : 0u);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 16
    for (uint32_t i = 0; i < 256u; ++i)
    {
        const double av = (double)ra[i];
        s0 += av * (double)rb[i];
        if constexpr (NV == 2)
            s1 += av * (double)rc[i];
    }
    if (gran)
    {
        const __amdgpu_buffer_rsrc_t rs = gran_rsrc(gran);
        gran_store(rs, NV * k, s0, tag);
        if constexpr (NV == 2)
            gran_store(rs, NV * k + 1u, s1, tag);
    }
    else
    {
        pab[k] = s0;
        if constexpr (NV == 2)
            pac[k] = s1;
    }
}

template <int NV>
__global__ __launch_bounds__(256) void k_dot_chunks256(const float *__restrict__ a, const float *__restrict__ b,
                                                       const float *__restrict__ c, uint32_t D, uint32_t chunks,
                                                       double *__restrict__ pab, double *__restrict__ pac,
                                                       const Ctl *__restrict__ ctl)
{
    if (ctl && !ctl->active)
        return;
    dot_chunks256<NV>(a, b, c, D, chunks, pab, pac, blockIdx.x, nullptr, 0u);
}

// The ordered chain over one block of NB partials in LDS, fully unrolled with scheduling barriers. A loop of two
// alternating register sets is rotated by LLVM so that both sets load at the top of each trip: every 32 adds then
// wait a full LDS round trip (C2's 4,020-partial folds took 28-30 us in the streamed kernels, ~6 ns per add). Here
// the next set's eight 16-B reads are pinned in front of the current set's 16 dependent adds.
template <uint32_t NB, uint32_t H = 8>  // H: double2 per register set (2 sets: 4 H VGPRs)
__device__ __forceinline__ void fold_block(const double2 *v, double &acc)
{
    double2 A[H], B[H];
#pragma unroll
    for (uint32_t u = 0; u < H; ++u)
        A[u] = v[u];
#pragma unroll
    for (uint32_t i = 0; i < NB / 2u; i += 2u * H)
    {
#pragma unroll
        for (uint32_t u = 0; u < H; ++u)
            B[u] = v[i + H + u];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (uint32_t u = 0; u < H; ++u)
        {
            acc += A[u].x;
            acc += A[u].y;
        }
        __builtin_amdgcn_sched_barrier(0);
        if (i + 2u * H < NB / 2u)
        {
#pragma unroll
            for (uint32_t u = 0; u < H; ++u)
                A[u] = v[i + 2u * H + u];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (uint32_t u = 0; u < H; ++u)
        {
            acc += B[u].x;
            acc += B[u].y;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

constexpr int kFoldThreads = 256;
constexpr uint32_t kFoldBlock = 4096;  // partials per staged block and operand (one block: C2's 4,030 chunks)
constexpr uint32_t kFoldSub = 256;     // partials per fold_block (a staged block is padded with +0.0 to a multiple)
template <int NC>
__device__ void fold_seq(const double *__restrict__ p0, const double *__restrict__ p1, uint32_t count, double &t0,
                         double &t1)
{
    // a staged block is padded with +0.0 to a multiple of kFoldSub (a sequential sum from +0.0 is never -0.0, so
    // adding +0.0 is exact) and folded by fold_block, branch-free. Two operands (NC = 2) are two independent chains,
    // run by thread 0 (operand 0) and thread 64 (operand 1) in different waves: interleaved in one thread they
    // measured no faster than back to back (C2 beta 39 us; a ping-pong of both 42-45).
    constexpr uint32_t W = 16, kRow = kFoldBlock + W;
    constexpr uint32_t kStage = NC == 2 ? 128u : 64u;  // the first thread of the staging waves
    __shared__ double2 buf[2][NC][kRow / 2];
    __shared__ double other;
    const uint32_t nb = (count + kFoldBlock - 1u) / kFoldBlock;
    const auto stage = [&](uint32_t blk, uint32_t first, uint32_t step) {
        const uint32_t b0 = blk * kFoldBlock, n = min(kFoldBlock, count - b0);
        const uint32_t npad = (n + kFoldSub - 1u) / kFoldSub * kFoldSub;
        double *d0 = reinterpret_cast<double *>(buf[blk & 1u][0]);
        double *d1 = reinterpret_cast<double *>(buf[blk & 1u][NC - 1]);
        for (uint32_t i = first; i < npad; i += step)
        {
            d0[i] = i < n ? p0[b0 + i] : 0.0;
            if constexpr (NC == 2)
                d1[i] = i < n ? p1[b0 + i] : 0.0;
        }
    };
    // whole kFoldSub-partial sub-blocks through fold_block (its next reads pinned ahead of the adds)
    const auto chain = [](const double2 *v, uint32_t npad, double &acc) {
        for (uint32_t i = 0; i < npad; i += kFoldSub)
            fold_block<kFoldSub>(v + i / 2u, acc);
    };
    double acc = 0.0;
    if (nb)
        stage(0, threadIdx.x, kFoldThreads);
    __syncthreads();
    for (uint32_t blk = 0; blk < nb; ++blk)
    {
        const uint32_t n = min(kFoldBlock, count - blk * kFoldBlock);
        const uint32_t npad = (n + kFoldSub - 1u) / kFoldSub * kFoldSub;
        if (threadIdx.x >= kStage)  // the staging waves; the folding threads' waves do nothing else
        {
            if (blk + 1u < nb)
                stage(blk + 1u, threadIdx.x - kStage, kFoldThreads - kStage);
        }
        else if (threadIdx.x == 0)
            chain(buf[blk & 1u][0], npad, acc);
        else if (NC == 2 && threadIdx.x == 64)
            chain(buf[blk & 1u][NC - 1], npad, acc);
        __syncthreads();
    }
    if (NC == 2 && threadIdx.x == 64)
        other = acc;
    __syncthreads();
    t0 = acc;
    t1 = NC == 2 ? other : 0.0;
}

__global__ __launch_bounds__(kFoldThreads) void k_fold1(const double *__restrict__ p, uint32_t count,
                                                        double *__restrict__ out)
{
    double t0, t1;
    fold_seq<1>(p, nullptr, count, t0, t1);
    if (threadIdx.x == 0)
        out[0] = t0;
}

// ---- PCG scalar phases (one workgroup; thread 0 decides), pcg.cpp:768-895 ----

__global__ __launch_bounds__(kFoldThreads) void k_pcg_init_scalars(Ctl *ctl, const double *__restrict__ p_rhs,
                                                                   const double *__restrict__ p_rr, uint32_t count,
                                                                   double rel_tol, double *__restrict__ hist)
{
    double rhs_sq, rr;
    fold_seq<2>(p_rhs, p_rr, count, rhs_sq, rr);
    if (threadIdx.x)
        return;
    double rhs_norm = sqrt(rhs_sq);
    if (rhs_norm < 1.0e-12)
        rhs_norm = 1.0;
    const double res = sqrt(rr);
    Ctl c{};
    c.res = res;
    c.rhs_norm = rhs_norm;
    c.rhs_norm_raw = sqrt(rhs_sq);
    c.tol = rel_tol * rhs_norm;
    c.iterations = 0;
    c.converged = res <= c.tol ? 1 : 0;
    c.active = c.converged ? 0 : 1;
    c.error = 0;
    c.error_iter = 0;
    hist[0] = res;
    *ctl = c;
}

__global__ __launch_bounds__(kFoldThreads) void k_pcg_init_rho(Ctl *ctl, const double *__restrict__ p_rz,
                                                               uint32_t count)
{
    if (!ctl->active)
        return;
    double rho, unused;
    fold_seq<1>(p_rz, nullptr, count, rho, unused);
    if (threadIdx.x)
        return;
    ctl->rho = rho;
    if (fabs(rho) < 1.0e-18)
    {
        ctl->error = CWF_ERR_RHO_ZERO;
        ctl->error_iter = -1;
        ctl->active = 0;
    }
}

// alpha from the folded p . Ap (pcg.cpp:840-853), thread 0
__device__ __forceinline__ void alpha_decide(Ctl *ctl, double denom)
{
    ctl->denom = denom;
    if (fabs(denom) < 1.0e-18)
    {
        ctl->error = CWF_ERR_DENOM_ZERO;
        ctl->error_iter = (int)ctl->iterations;
        ctl->active = 0;
        return;
    }
    const double alpha = ctl->rho / denom;
    ctl->alpha = alpha;
    ctl->alpha_last = alpha;
}

// residual, convergence and beta from the folded r . r and r . z (pcg.cpp:862-895), thread 0
__device__ __forceinline__ void beta_decide(Ctl *ctl, double rr, double rz, double *__restrict__ hist)
{
    const double res = sqrt(rr);
    const unsigned long long it = ctl->iterations;
    ctl->res = res;
    ctl->iterations = it + 1;
    hist[it + 1] = res;
    if (res <= ctl->tol)
    {
        ctl->converged = 1;
        ctl->active = 0;
        return;
    }
    if (fabs(ctl->rho) < 1.0e-18)
    {
        ctl->error = CWF_ERR_RHO_ZERO;
        ctl->error_iter = (int)it;
        ctl->active = 0;
        return;
    }
    const double beta = rz / ctl->rho;
    ctl->beta = beta;
    ctl->beta_last = beta;
    ctl->rho = rz;
}

__global__ __launch_bounds__(kFoldThreads) void k_pcg_alpha(Ctl *ctl, const double *__restrict__ p_pAp, uint32_t count)
{
    if (!ctl->active)
        return;
    double denom, unused;
    fold_seq<1>(p_pAp, nullptr, count, denom, unused);
    if (threadIdx.x == 0)
        alpha_decide(ctl, denom);
}

__global__ __launch_bounds__(kFoldThreads) void k_pcg_beta(Ctl *ctl, const double *__restrict__ p_rr,
                                                           const double *__restrict__ p_rz, uint32_t count,
                                                           double *__restrict__ hist)
{
    if (!ctl->active)
        return;
    double rr, rz;
    fold_seq<2>(p_rr, p_rz, count, rr, rz);
    if (threadIdx.x == 0)
        beta_decide(ctl, rr, rz, hist);
}

// The streamed form of fold_seq, run by workgroup 0 of the producing pass. Wave c < NC folds operand c (its lane 0,
// wave-uniform LDS addresses). The S = 4 - NC other waves stage: staging wave w polls the granules of blocks w,
// w + S, ... (kStreamBlock chunks each; a block's slot is claimed first, then every lane polls its NC kStreamBlock / 64
// granules at once, re-polling only those that do not carry the launch's tag yet, and stores each landed value to
// LDS) into a ring of kStreamRing LDS slots, and publishes the block with an LDS flag; the folding waves wait on the
// flag and count the block folded when done. So S blocks' polls are in flight while the chains run, decoupled by
// LDS flags instead of workgroup barriers. The chain is fold_block, in chunk order: bitwise fold_seq over the
// partial arrays. Bounded: a granule that never arrives ends the poll (the block is published anyway, the fold
// returns false and the solve fails).
#ifndef CWF_ALPHA_FOLD_H
#define CWF_ALPHA_FOLD_H 16
#endif
constexpr uint32_t kAlphaFoldH = CWF_ALPHA_FOLD_H;  // (a build macro for the same-box A/B of the register sets)
constexpr uint32_t kStreamBlock = 256;
constexpr uint32_t kStreamCPB = 8;         // chunks per block of the streamed p.Ap pass
// the producing workgroups of the streamed p.Ap / update passes (persistent, in block order). Production, not the
// chain, bounds both passes (C2, rocprofv3 means, same box: p.Ap + alpha 25.5 / 21.9 / 24.0 us at 128 / 256 / 512;
// update + beta 31.9 / 28.1 / 29.4 us at 256 / 512 / 768, 29.5 with one workgroup per node block)
constexpr uint32_t kStreamDotWG = 256;
constexpr uint32_t kStreamUpdWG = 512;
// (kStreamBlock: chunks per fold block; C2's 4,020 chunks in 16 blocks)
constexpr uint32_t kStreamRing = 6;              // LDS slots
constexpr uint32_t kStreamRow = kStreamBlock + 16u;  // + the chain's W spare slots
constexpr uint32_t kStreamMaxRounds = 4000000u;  // poll rounds per block before giving up (>= 4 s)
template <int NC>
constexpr uint32_t fold_stream_lds()  // double2 entries of the caller's staging buffer
{
    return kStreamRing * NC * (kStreamRow / 2u);
}
// bufp: fold_stream_lds<NC>() double2 of LDS (the caller's, so a producing workgroup reuses it for its own staging);
// t0 (operand 0) and t1 (operand 1) are valid in thread 0
template <int NC>
__device__ bool fold_stream(const double *gran, uint32_t count, uint32_t tag, double2 *bufp, double &t0, double &t1)
{
    constexpr uint32_t W = 16, kRow = kStreamRow, kStagers = kFoldThreads / 64 - NC;
    constexpr uint32_t P = kStreamBlock * NC / 64u;  // granules per staging lane and block
    static_assert(P <= 32u && kStreamBlock % (2u * W) == 0u, "stream block");
    double *buf = reinterpret_cast<double *>(bufp);  // slot s, operand c: buf + (s NC + c) kRow
    __shared__ uint32_t ready[kStreamRing], consumed[NC], fail;
    __shared__ double other;
    const __amdgpu_buffer_rsrc_t rs = gran_rsrc(gran);
    const uint32_t nb = (count + kStreamBlock - 1u) / kStreamBlock, lane = threadIdx.x % 64u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);  // wave-uniform (scalar LDS addresses)
    if (threadIdx.x < kStreamRing)
        ready[threadIdx.x] = 0u;
    if (threadIdx.x < (uint32_t)NC)
        consumed[threadIdx.x] = 0u;
    if (threadIdx.x == 0)
        fail = 0u;
    __syncthreads();
    // the producing workgroups' waves share these SIMDs: the chain's dependent adds (and the polls feeding it) issue
    // first
    if (wave < (uint32_t)NC)
        __builtin_amdgcn_s_setprio(3);
    else
        __builtin_amdgcn_s_setprio(2);
    if (wave >= (uint32_t)NC)
    {
        for (uint32_t blk = wave - NC; blk < nb; blk += kStagers)
        {
            const uint32_t b0 = blk * kStreamBlock, n = min(kStreamBlock, count - b0), slot = blk % kStreamRing;
            // the slot is free once the chain has folded block blk - kStreamRing (the polls of the next slots are
            // still ahead of the chain: kStreamRing / kStagers blocks per staging wave)
            const auto folded = [&]() {  // blocks both chains have folded
                uint32_t c = __hip_atomic_load(&consumed[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if constexpr (NC == 2)
                    c = min(c, __hip_atomic_load(&consumed[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                return c;
            };
            while (blk >= kStreamRing && folded() + kStreamRing <= blk)
                __builtin_amdgcn_s_sleep(1);
            double *row = buf + slot * NC * kRow;
            uint32_t pending = 0;
#pragma unroll
            for (uint32_t u = 0; u < P; ++u)
            {
                const uint32_t q = lane + 64u * u;
                if (q / NC < n)
                    pending |= 1u << u;
                else
                    row[(q % NC) * kRow + q / NC] = 0.0;  // +0.0 pads: the chain always folds kStreamBlock terms
            }
            for (uint32_t round = 0; pending; ++round)
            {
                u32x4 g[P];
#pragma unroll
                for (uint32_t u = 0; u < P; ++u)
                    if ((pending >> u) & 1u)
                        g[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * (NC * b0 + lane + 64u * u), 0, 16);
#pragma unroll
                for (uint32_t u = 0; u < P; ++u)
                    if (((pending >> u) & 1u) && g[u].z == tag)
                    {
                        const uint32_t q = lane + 64u * u;
                        row[(q % NC) * kRow + q / NC] = __hiloint2double((int)g[u].y, (int)g[u].x);
                        pending &= ~(1u << u);
                    }
                if (!pending)
                    break;
                if (round >= kStreamMaxRounds)
                {
                    __hip_atomic_store(&fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0)
                __hip_atomic_store(&ready[slot], blk + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    else if (lane == 0)
    {
        double acc = 0.0;
        for (uint32_t blk = 0; blk < nb; ++blk)
        {
            const uint32_t slot = blk % kStreamRing;
            while (__hip_atomic_load(&ready[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != blk + 1u)
                __builtin_amdgcn_s_sleep(1);
            // the alpha pass (NC = 1) runs at 2 waves / SIMD (its LDS): 32-partial register sets; the update pass
            // keeps 16 (its VGPRs set its occupancy)
            fold_block<kStreamBlock, NC == 1 ? kAlphaFoldH : 8u>(
                reinterpret_cast<const double2 *>(buf + (slot * NC + wave) * kRow), acc);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __hip_atomic_store(&consumed[wave], blk + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (wave == 1)
            other = acc;
        t0 = acc;
    }
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    t1 = NC == 2 ? other : 0.0;
    return fail == 0u;
}

__device__ __forceinline__ void stream_fail(Ctl *ctl)
{
    ctl->error = CWF_ERR_HIP;
    ctl->error_iter = (int)ctl->iterations;
    ctl->active = 0;
}

// the p . Ap chunk partials (k_dot_chunks256, workgroups 1..) streamed into alpha (k_pcg_alpha, workgroup 0)
__global__ __launch_bounds__(256) void k_dot_alpha_stream(const float *__restrict__ p, const float *__restrict__ Ap,
                                                          uint32_t D, uint32_t chunks, Ctl *ctl,
                                                          const double *gran, uint32_t tag)
{
    if (!ctl->active)
        return;
    if (blockIdx.x == 0)
    {
        __shared__ double2 fbuf[fold_stream_lds<1>()];
        double denom = 0.0, unused;
        const bool ok = fold_stream<1>(gran, chunks, tag, fbuf, denom, unused);
        if (threadIdx.x == 0)
            ok ? alpha_decide(ctl, denom) : stream_fail(ctl);
        return;
    }
    // workgroups 1..G walk the blocks in order (block j G + b - 1 in their j-th step), so the partials land roughly in
    // chunk order while workgroup 0 folds: 8 chunks per block, the first step's land after one round trip
    const uint32_t nblk = (chunks + kStreamCPB - 1u) / kStreamCPB, G = gridDim.x - 1u;
    for (uint32_t bx = blockIdx.x - 1u; bx < nblk; bx += G)
    {
        dot_chunks256<1, kStreamCPB>(p, Ap, nullptr, D, chunks, nullptr, nullptr, bx, gran, tag);
        __syncthreads();  // the staging rows are refilled by the next block
    }
}

// ---- node-wise vector phases ----

// r = rhs - Ap (f32), then enforce_dirichlet_solution (pcg.cpp:761-766, 458-475)
__global__ __launch_bounds__(kBlock) void k_init_residual(DevSys s, const float *__restrict__ rhs,
                                                          const float *__restrict__ Ap, float *__restrict__ x,
                                                          float *__restrict__ r)
{
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    const uint32_t mk = s.mask[n];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const uint32_t d = 3u * n + k;
        float rv = rhs[d] - Ap[d];
        if (mk & (1u << k))
        {
            x[d] = rhs[d];
            rv = 0.0f;
        }
        r[d] = rv;
    }
}

__device__ __forceinline__ void precond_node(const float *__restrict__ inv, uint32_t n, uint32_t mk, const float rv[3],
                                             float z[3])
{
    // pcg.cpp:426-453
    const double r0 = (double)rv[0], r1 = (double)rv[1], r2 = (double)rv[2];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        double sum = 0.0;
        sum += (double)inv[9u * n + 3 * k + 0] * r0;
        sum += (double)inv[9u * n + 3 * k + 1] * r1;
        sum += (double)inv[9u * n + 3 * k + 2] * r2;
        z[k] = (mk & (1u << k)) ? 0.0f : (float)sum;
    }
}

__global__ __launch_bounds__(kBlock) void k_precond(DevSys s, const float *__restrict__ inv,
                                                    const float *__restrict__ r, float *__restrict__ z,
                                                    const Ctl *__restrict__ ctl)
{
    if (ctl && !ctl->active)
        return;
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    const float rv[3] = {r[3u * n], r[3u * n + 1], r[3u * n + 2]};
    float zv[3];
    precond_node(inv, n, s.mask[n], rv, zv);
    z[3u * n] = zv[0];
    z[3u * n + 1] = zv[1];
    z[3u * n + 2] = zv[2];
}

// p = z, constrained -> 0 (pcg.cpp:815-828)
__global__ __launch_bounds__(kBlock) void k_p_init(DevSys s, const float *__restrict__ z, float *__restrict__ p,
                                                   const Ctl *__restrict__ ctl)
{
    if (!ctl->active)
        return;
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    const uint32_t mk = s.mask[n];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        p[3u * n + k] = (mk & (1u << k)) ? 0.0f : z[3u * n + k];
}

// x += f32(alpha p); r -= f32(alpha Ap); enforce; z = M^-1 r  (pcg.cpp:854-860, 877), and the chunk partials of
// r . r and r . z (pcg.cpp:862, 883) from the workgroup's own DOFs (wg_chunk_partials)
// STREAM: workgroup 0 folds the r . r and r . z granules of workgroups 1.. (their nodes: blockIdx - 1) into the
// residual check and beta (k_pcg_beta's work, fold_stream), gran / tag / hist its arguments
template <bool STREAM>
__global__ __launch_bounds__(kBlock) void k_update(DevSys s, const float *__restrict__ rhs,
                                                   const float *__restrict__ inv, const float *__restrict__ p,
                                                   const float *__restrict__ Ap, float *__restrict__ x,
                                                   float *__restrict__ r, float *__restrict__ z,
                                                   Ctl *__restrict__ ctl, double *__restrict__ prr,
                                                   double *__restrict__ prz, uint32_t nlim, uint32_t chunks,
                                                   const double *gran, uint32_t tag, double *__restrict__ hist)
{
    constexpr uint32_t kSh = STREAM ? std::max<uint32_t>(6u * kChunkRow, fold_stream_lds<2>()) : 3u * kChunkRow;
    __shared__ double2 srz[kSh];
    if (!ctl->active)
        return;
    if constexpr (STREAM)
        if (blockIdx.x == 0)
        {
            double rr = 0.0, rz;
            const bool ok = fold_stream<2>(gran, chunks, tag, srz, rr, rz);
            if (threadIdx.x == 0)
                ok ? beta_decide(ctl, rr, rz, hist) : stream_fail(ctl);
            return;
        }
    // one node block: x, r, z and (prr) the staged fp64 products of its DOFs in st
    const auto nodes = [&](uint32_t bx, double2 *st) {
        const uint32_t n = bx * kBlock + threadIdx.x;
        float rv[3] = {0.f, 0.f, 0.f}, zv[3] = {0.f, 0.f, 0.f};
        if (n < s.N)
        {
            const double alpha = ctl->alpha;
            const uint32_t mk = s.mask[n];
#pragma unroll
            for (int k = 0; k < 3; ++k)
            {
                const uint32_t d = 3u * n + k;
                float xv = x[d] + (float)(alpha * (double)p[d]);
                float rr = r[d] - (float)(alpha * (double)Ap[d]);
                if (mk & (1u << k))
                {
                    xv = rhs[d];
                    rr = 0.0f;
                }
                x[d] = xv;
                r[d] = rr;
                rv[k] = rr;
            }
            precond_node(inv, n, mk, rv, zv);
            z[3u * n] = zv[0];
            z[3u * n + 1] = zv[1];
            z[3u * n + 2] = zv[2];
        }
        if (!prr)  // a reduction chunk other than 256 DOFs: the partials are a separate pass
            return;
        const bool own = n < nlim;
#pragma unroll
        for (int k = 0; k < 3; ++k)
        {
            const double r = (double)rv[k];
            st[chunk_slot(3u * threadIdx.x + k)] = own ? double2{r * r, r * (double)zv[k]} : double2{0.0, 0.0};
        }
    };
    if constexpr (STREAM)
    {
        // workgroups 1..G walk the node blocks in order (block j G + b - 1 in their j-th step), so the partials
        // land roughly in chunk order while workgroup 0 folds them. The staging rows alternate by step: wave 0's
        // lanes 0-2 fold block j's chunks while waves 1-3 already load and form block j + G (wave 0 reaches step
        // j + 1's barrier only after its chains, so block j + 2 G never restages rows still being folded)
        const uint32_t nblk = (s.N + kBlock - 1u) / kBlock, G = gridDim.x - 1u;
        uint32_t j = 0;
        for (uint32_t bx = blockIdx.x - 1u; bx < nblk; bx += G, ++j)
        {
            double2 *st = srz + (j & 1u) * (3u * kChunkRow);
            nodes(bx, st);
            __syncthreads();
            wg_chunk_partials<2>(st, chunks, prr, prz, bx, gran, tag);
        }
    }
    else
    {
        nodes(blockIdx.x, srz);
        if (!prr)
            return;
        __syncthreads();
        wg_chunk_partials<2>(srz, chunks, prr, prz, blockIdx.x);
    }
}

// p = f32(double(z) + beta double(p)), constrained -> 0 (pcg.cpp:897-914)
__global__ __launch_bounds__(kBlock) void k_p_update(DevSys s, const float *__restrict__ z, float *__restrict__ p,
                                                     const Ctl *__restrict__ ctl)
{
    if (!ctl->active)
        return;
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    const double beta = ctl->beta;
    const uint32_t mk = s.mask[n];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const uint32_t d = 3u * n + k;
        const float pv = (float)((double)z[d] + beta * (double)p[d]);
        p[d] = (mk & (1u << k)) ? 0.0f : pv;
    }
}

inline unsigned grid_for(uint32_t n, uint32_t b) { return (n + b - 1) / b; }

inline bool knob_off(const char *name)
{
    const char *v = knob(name);
    return v && v[0] == '0';
}

}  // namespace

uint32_t parity_chunk_count(const cwf_hip_system *h)
{
    const uint64_t B = h->reduction_block ? h->reduction_block : 1;
    return (uint32_t)((h->ds.D + B - 1) / B);
}

// the node-tile K_eff (the handle builds its tiles whenever it runs PARITY: abi.cpp parity_force_buffer)
template <bool SAN, bool DOT>
void launch_parity_tile(const DevSys &s, const float *x, float *y, const Ctl *ctl, double *pdot, uint32_t nlim,
                        uint32_t chunks, hipStream_t st)
{
    const dim3 b(kBlock);
    if (s.ptile_nodes && !DOT)
    {
        const dim3 gn(s.pntile);
        if (s.iso)
            k_keff_parity_tile<true, SAN, false, true><<<gn, b, 0, st>>>(s, x, y, ctl, pdot, nlim, chunks);
        else
            k_keff_parity_tile<false, SAN, false, true><<<gn, b, 0, st>>>(s, x, y, ctl, pdot, nlim, chunks);
        return;
    }
    const dim3 gn(grid_for(s.N, kBlock));
    if (s.iso)
        k_keff_parity_tile<true, SAN, DOT, false><<<gn, b, 0, st>>>(s, x, y, ctl, pdot, nlim, chunks);
    else
        k_keff_parity_tile<false, SAN, DOT, false><<<gn, b, 0, st>>>(s, x, y, ctl, pdot, nlim, chunks);
}

void parity_keff_ds(const DevSys &s, const float *x, float *y, bool sanitize, const Ctl *ctl, hipStream_t st)
{
    if (s.N == 0)
        return;
    sanitize ? launch_parity_tile<true, false>(s, x, y, ctl, nullptr, 0u, 0u, st)
             : launch_parity_tile<false, false>(s, x, y, ctl, nullptr, 0u, 0u, st);
}

// the PCG loop's K_eff p with the chunk partials of p . Ap over nodes [0, Nown) into pdot: fused into the node fold
// when the reduction chunk is 256 DOFs (every workgroup then owns three whole chunks), a separate pass otherwise
void parity_keff_dot(const cwf_hip_system *h, const float *p, float *Ap, const Ctl *ctl, double *pdot, hipStream_t st)
{
    const DevSys &s = h->ds;
    if (h->reduction_block != 256 || s.ptile_nodes)  // compact tiles: the partials in their own pass
    {
        parity_keff_ds(s, p, Ap, false, ctl, st);
        parity_dot_partials_n(3u * s.Nown, (uint32_t)h->reduction_block, p, Ap, nullptr, pdot, nullptr, ctl, st);
        return;
    }
    if (s.N == 0)
        return;
    launch_parity_tile<false, true>(s, p, Ap, ctl, pdot, s.Nown, grid_for(3u * s.Nown, 256u), st);
}

void parity_keff(const cwf_hip_system *h, const float *x, float *y, bool sanitize, const Ctl *ctl, hipStream_t st)
{
    parity_keff_ds(h->ds, x, y, sanitize, ctl, st);
}

void hex_block_jacobi(const cwf_hip_system *h, float *inv, hipStream_t st)
{
    if (h->ds.N == 0)
        return;
    k_block_jacobi_hex<<<grid_for(h->ds.N, kBlock), kBlock, 0, st>>>(h->ds, inv);
}

void parity_block_jacobi(const cwf_hip_system *h, float *inv, hipStream_t st)
{
    if (h->ds.N == 0)
        return;
    k_block_jacobi_parity<<<grid_for(h->ds.N, kBlock), kBlock, 0, st>>>(h->ds, inv);
}

void parity_dot_partials_n(uint32_t D, uint32_t B, const float *a, const float *b, const float *c, double *pab,
                           double *pac, const Ctl *ctl, hipStream_t st)
{
    B = B ? B : 1;
    const uint32_t chunks = (uint32_t)(((uint64_t)D + B - 1) / B);
    if (chunks == 0)
        return;
    if (B == 256)
    {
        if (c)
            k_dot_chunks256<2><<<grid_for(chunks, kDotChunksPerBlock), 256, 0, st>>>(a, b, c, D, chunks, pab, pac, ctl);
        else
            k_dot_chunks256<1><<<grid_for(chunks, kDotChunksPerBlock), 256, 0, st>>>(a, b, c, D, chunks, pab, pac, ctl);
    }
    else
    {
        if (c)
            k_dot_chunks_generic<2><<<grid_for(chunks, kBlock), kBlock, 0, st>>>(a, b, c, D, B, chunks, pab, pac,
                                                                                ctl);
        else
            k_dot_chunks_generic<1><<<grid_for(chunks, kBlock), kBlock, 0, st>>>(a, b, c, D, B, chunks, pab, pac,
                                                                                ctl);
    }
}

void parity_dot_partials(const cwf_hip_system *h, const float *a, const float *b, const float *c, double *pab,
                         double *pac, const Ctl *ctl, hipStream_t st)
{
    parity_dot_partials_n(h->ds.D, (uint32_t)h->reduction_block, a, b, c, pab, pac, ctl, st);
}

void parity_fold(const double *part, uint32_t count, double *out, hipStream_t st)
{
    k_fold1<<<1, kFoldThreads, 0, st>>>(part, count, out);
}

void launch_init_residual(const cwf_hip_system *h, const float *rhs, hipStream_t st)
{
    k_init_residual<<<grid_for(h->ds.N, kBlock), kBlock, 0, st>>>(h->ds, rhs, h->Ap, h->x, h->r);
}

void launch_precond(const cwf_hip_system *h, const Ctl *ctl, hipStream_t st)
{
    k_precond<<<grid_for(h->ds.N, kBlock), kBlock, 0, st>>>(h->ds, h->inv, h->r, h->z, ctl);
}

void launch_p_init(const cwf_hip_system *h, hipStream_t st)
{
    k_p_init<<<grid_for(h->ds.N, kBlock), kBlock, 0, st>>>(h->ds, h->z, h->p, h->ctl);
}

// solve_pcg prologue (pcg.cpp:744-828). Requires x (warm start or zeroed) on device.
void parity_pcg_init(cwf_hip_system *h, const float *rhs, double rel_tol, hipStream_t st)
{
    const DevSys &s = h->ds;
    const uint32_t chunks = parity_chunk_count(h);
    if (!h->fgran && h->reduction_block == 256 && !knob_off("CWF_PARITY_STREAM"))
    {
        // the streamed folds' granules: 2 per chunk, tag 0 (the first streamed launch's tag is 1)
        void *q = nullptr;
        const size_t bytes = 32ull * chunks + 64u;
        if (hipMalloc(&q, bytes) == hipSuccess)
        {
            h->owned.push_back(q);
            h->bytes += bytes;
            h->fgran = static_cast<double *>(q);
            h->fgran_tag = 0;
            (void)hipMemsetAsync(q, 0, bytes, st);
        }
    }
    parity_block_jacobi(h, h->inv, st);
    h->inv_fast = false;  // inv now holds the PARITY inverse (not symmetrised, no inv6)
    parity_keff(h, h->x, h->Ap, true, nullptr, st);
    k_init_residual<<<grid_for(s.N, kBlock), kBlock, 0, st>>>(s, rhs, h->Ap, h->x, h->r);
    parity_dot_partials(h, rhs, rhs, nullptr, h->part0, nullptr, nullptr, st);
    parity_dot_partials(h, h->r, h->r, nullptr, h->part1, nullptr, nullptr, st);
    k_pcg_init_scalars<<<1, kFoldThreads, 0, st>>>(h->ctl, h->part0, h->part1, chunks, rel_tol, h->hist);
    k_precond<<<grid_for(s.N, kBlock), kBlock, 0, st>>>(s, h->inv, h->r, h->z, h->ctl);
    parity_dot_partials(h, h->r, h->z, nullptr, h->part0, nullptr, h->ctl, st);
    k_pcg_init_rho<<<1, kFoldThreads, 0, st>>>(h->ctl, h->part0, chunks);
    k_p_init<<<grid_for(s.N, kBlock), kBlock, 0, st>>>(s, h->z, h->p, h->ctl);
}

// ---- the scalar and node phases of solve_pcg, for the sharded PARITY schedule (comm.cpp), which folds the
// all-gathered chunk partials of every rank in global chunk order ----
void parity_init_scalars(cwf_hip_system *h, const double *p_rhs, const double *p_rr, uint32_t count, double rel_tol,
                         hipStream_t st)
{
    k_pcg_init_scalars<<<1, kFoldThreads, 0, st>>>(h->ctl, p_rhs, p_rr, count, rel_tol, h->hist);
}

void parity_init_rho(cwf_hip_system *h, const double *p_rz, uint32_t count, hipStream_t st)
{
    k_pcg_init_rho<<<1, kFoldThreads, 0, st>>>(h->ctl, p_rz, count);
}

void parity_alpha(cwf_hip_system *h, const double *p_pap, uint32_t count, hipStream_t st)
{
    k_pcg_alpha<<<1, kFoldThreads, 0, st>>>(h->ctl, p_pap, count);
}

void parity_update(cwf_hip_system *h, const float *rhs, double *prr, double *prz, hipStream_t st)
{
    const uint32_t nlim = h->ds.Nown;
    const bool fused = h->reduction_block == 256;
    k_update<false><<<grid_for(h->ds.N, kBlock), kBlock, 0, st>>>(h->ds, rhs, h->inv, h->p, h->Ap, h->x, h->r, h->z,
                                                                  h->ctl, fused ? prr : nullptr, prz, nlim,
                                                                  grid_for(3u * nlim, 256u), nullptr, 0u, nullptr);
    if (!fused)
        parity_dot_partials_n(3u * nlim, (uint32_t)h->reduction_block, h->r, h->r, h->z, prr, prz, h->ctl, st);
}

void parity_beta(cwf_hip_system *h, const double *p_rr, const double *p_rz, uint32_t count, hipStream_t st)
{
    k_pcg_beta<<<1, kFoldThreads, 0, st>>>(h->ctl, p_rr, p_rz, count, h->hist);
}

void parity_p_update(cwf_hip_system *h, hipStream_t st)
{
    k_p_update<<<grid_for(h->ds.N, kBlock), kBlock, 0, st>>>(h->ds, h->z, h->p, h->ctl);
}

// one PCG iteration (pcg.cpp:830-915); no-op once ctl->active == 0
void parity_pcg_iteration(cwf_hip_system *h, const float *rhs, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    const DevSys &s = h->ds;
    const uint32_t chunks = parity_chunk_count(h);
    if (h->fgran && h->reduction_block == 256 && s.ptile_nodes && s.Nown == s.N)
    {
        // streamed folds: alpha folded by the p . Ap pass's workgroup 0, beta by the update pass's (the same
        // partials in the same order as below: bitwise the same scalars), two launches fewer per iteration
        if (e0)
            (void)hipEventRecord(e0, st);
        parity_keff_ds(s, h->p, h->Ap, false, h->ctl, st);
        if (e1)
            (void)hipEventRecord(e1, st);
        const uint32_t t1 = ++h->fgran_tag, t2 = ++h->fgran_tag;
        const uint32_t gd = std::min(grid_for(chunks, kStreamCPB), kStreamDotWG);
        const uint32_t gu = std::min(grid_for(s.N, kBlock), kStreamUpdWG);
        k_dot_alpha_stream<<<1u + gd, 256, 0, st>>>(h->p, h->Ap, 3u * s.N, chunks, h->ctl, h->fgran, t1);
        k_update<true><<<1u + gu, kBlock, 0, st>>>(s, rhs, h->inv, h->p, h->Ap, h->x, h->r, h->z,
                                                                      h->ctl, h->part0, h->part1, s.N, chunks,
                                                                      h->fgran, t2, h->hist);
        k_p_update<<<grid_for(s.N, kBlock), kBlock, 0, st>>>(s, h->z, h->p, h->ctl);
        return;
    }
    if (e0)
        (void)hipEventRecord(e0, st);
    parity_keff_dot(h, h->p, h->Ap, h->ctl, h->part0, st);  // + the p . Ap chunk partials
    if (e1)
        (void)hipEventRecord(e1, st);
    k_pcg_alpha<<<1, kFoldThreads, 0, st>>>(h->ctl, h->part0, chunks);
    parity_update(h, rhs, h->part0, h->part1, st);  // + the r . r and r . z chunk partials
    k_pcg_beta<<<1, kFoldThreads, 0, st>>>(h->ctl, h->part0, h->part1, chunks, h->hist);
    k_p_update<<<grid_for(s.N, kBlock), kBlock, 0, st>>>(s, h->z, h->p, h->ctl);
}

}  // namespace cwf

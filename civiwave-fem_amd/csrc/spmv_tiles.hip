// spmv_tiles.hip -- FAST-mode K_eff and the fused FAST PCG iteration (2 kernels / iteration).
//
// k_keff_tiles (256-thread workgroups looping over tiles of <= 512 Morton-ordered tets):
//   a) gather the tile's distinct nodes into LDS: x (apply_keff) or, inside PCG, the on-the-fly
//      search direction p_new = z + beta p_old (the p-update pass of pcg.cpp:897-914 is fused here);
//   b) every element: stream its 48-B record from 3 SoA planes (each dwordx4 wave-load is one
//      contiguous 1 KiB run), corners' values from LDS, fp32 strain -> stress -> 12 nodal forces
//      scaled by V*s_K, stored to LDS as f[12][512] (bank-conflict free);
//   c) every tile node: fold its (element, corner) forces in ascending element order through the
//      tile's local CSR (deterministic, no atomics) and store the 12-B tile-node partial;
//   d) PCG only: the workgroup's fp64 share of p.Ap (one partial per workgroup).
// k_keff_finalize (apply_keff only): y = sum of the node's tile partials (ascending tile) + m s_M x,
//   Dirichlet identity rows.
// k_pcg_update_tiles (PCG only, grid-stride over nodes): Ap from the partials (never stored),
//   recompute p_new, x += alpha p, r -= alpha Ap, Dirichlet enforce, z = M^-1 r, store x r z p;
//   fp64 r.r and r.z shares per workgroup.
// Scalars without atomics or fences: every workgroup of a consumer kernel folds the producer's
// (<= 2048) workgroup partials itself in a fixed order, so alpha (update kernel) and |r|,
// convergence, beta (tiles-kernel preamble, pcg.cpp:862-895) are computed identically everywhere;
// the host passes the iteration index, and rho is double-buffered by iteration parity, so no
// device scalar is read after being written inside one kernel.
#include "cwf_internal.hpp"

namespace cwf
{
namespace
{
constexpr int kBlock = 256;
constexpr int kMaxM = 16;
constexpr unsigned kMaxTileBlocks = 2048;
constexpr unsigned kMaxUpdateBlocks = 1024;

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    return v;
}

// 256-thread block sum, fixed order; result valid in every thread
__device__ __forceinline__ double block_sum(double v, double *red4)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0)
        red4[threadIdx.x >> 6] = v;
    __syncthreads();
    const double t = (red4[0] + red4[1]) + (red4[2] + red4[3]);
    __syncthreads();
    return t;
}

// fixed-order fold of `count` doubles by the whole block (valid in every thread)
__device__ __forceinline__ double fold_all(const double *__restrict__ p, unsigned count, double *red4)
{
    double v = 0.0;
    for (unsigned i = threadIdx.x; i < count; i += kBlock)
        v += p[i];
    return block_sum(v, red4);
}

// pcg.cpp:862-895 for iteration `it` >= 1 from the update kernel's r.r / r.z shares.
// Returns false when the solve is over (converged or rho breakdown); writes beta for this iteration.
__device__ __forceinline__ bool residual_step(Ctl *ctl, const double *__restrict__ prr, const double *__restrict__ prz,
                                              unsigned nparts, unsigned it, double *__restrict__ hist, double *red4,
                                              float *beta_out)
{
    if (it == 0)
    {
        *beta_out = 0.f;
        return true;
    }
    const double rr = fold_all(prr, nparts, red4);
    const double rz = fold_all(prz, nparts, red4);
    const double res = sqrt(rr);
    const double rho_old = ctl->rho2[(it - 1) & 1u];
    const bool conv = res <= ctl->tol;
    const bool err = !conv && fabs(rho_old) < 1.0e-18;
    const double beta = (conv || err) ? 0.0 : rz / rho_old;
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

struct PcgArgs
{
    const float *z;           // z (PCG) -- x holds p_old
    Ctl *ctl;
    double *part_dot;         // out: per-workgroup p.Ap share
    const double *prr, *prz;  // in: update kernel's r.r / r.z shares of the previous iteration
    unsigned nupd;
    unsigned it;
    double *hist;
};

// MODE 0: apply (gather x, optional sanitize); MODE 1: PCG (gather z, p_old -> p_new)
template <bool ISO, bool SANITIZE, int MODE>
__global__ __launch_bounds__(kBlock) void k_keff_tiles(DevSys s, const float *__restrict__ x, PcgArgs pa)
{
    constexpr int kTab = ISO ? 12 : 36;
    extern __shared__ float lds[];
    float *sf = lds;                    // [12][kTileElems]
    float *sp = lds + 12 * kTileElems;  // [3][max_tile_nodes]
    __shared__ float dtab[kMaxM * 36];
    __shared__ double red[4];
    float beta = 0.f;
    if constexpr (MODE == 1)
    {
        if (!pa.ctl->active)
            return;
        if (!residual_step(pa.ctl, pa.prr, pa.prz, pa.nupd, pa.it, pa.hist, red, &beta))
            return;
    }
    const DevTiles &T = s.t;
    const uint32_t ms = T.max_tile_nodes;
    const uint32_t nm = s.M < kMaxM ? s.M : kMaxM;
    for (uint32_t i = threadIdx.x; i < nm * kTab; i += kBlock)
        dtab[i] = (float)s.dmat[36u * (i / kTab) + dsrc(ISO, i % kTab)];
    const float sK = (float)s.sK, sM = (float)s.sM;
    const uint4 *P0 = T.planes, *P1 = T.planes + T.E, *P2 = T.planes + 2u * T.E;
    double pap = 0.0;
    for (uint32_t tile = blockIdx.x; tile < T.ntiles; tile += gridDim.x)
    {
        const uint32_t e0 = T.tile_elem_off[tile], ne = T.tile_elem_off[tile + 1] - e0;
        const uint32_t nb = T.tile_node_off[tile], nn = T.tile_node_off[tile + 1] - nb;
        __syncthreads();  // previous tile's LDS reads are done
        for (uint32_t i = threadIdx.x; i < nn; i += kBlock)
        {
            const uint32_t g = T.tile_nodes[nb + i] & 0x7fffffffu;
            float u0, u1, u2;
            if constexpr (MODE == 1)
            {
                // p_new = z + beta p_old; constrained dofs stay 0 (z_c = 0, p_c = 0)
                u0 = fmaf(beta, x[3u * g + 0], pa.z[3u * g + 0]);
                u1 = fmaf(beta, x[3u * g + 1], pa.z[3u * g + 1]);
                u2 = fmaf(beta, x[3u * g + 2], pa.z[3u * g + 2]);
            }
            else
            {
                u0 = x[3u * g + 0];
                u1 = x[3u * g + 1];
                u2 = x[3u * g + 2];
                if constexpr (SANITIZE)
                {
                    const uint32_t mk = s.mask[g];
                    u0 = (mk & 1u) ? 0.f : u0;
                    u1 = (mk & 2u) ? 0.f : u1;
                    u2 = (mk & 4u) ? 0.f : u2;
                }
            }
            sp[i] = u0;
            sp[ms + i] = u1;
            sp[2 * ms + i] = u2;
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < ne; j += kBlock)
        {
            const uint32_t e = e0 + j;
            const uint4 q0 = P0[e], q1 = P1[e], q2 = P2[e];
            float g[12];
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
            const uint32_t li[4] = {q0.x & 0xffffu, q0.x >> 16, q0.y & 0xffffu, q0.y >> 16};
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
            const uint32_t mi = T.mat ? T.mat[e] : 0u;
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
            const float vol = __uint_as_float(q2.w) * sK;
#pragma unroll
            for (int a = 0; a < 4; ++a)
            {
                const float ax = g[3 * a], ay = g[3 * a + 1], az = g[3 * a + 2];
                sf[(3 * a + 0) * kTileElems + j] = vol * fmaf(az, sig[5], fmaf(ay, sig[3], ax * sig[0]));
                sf[(3 * a + 1) * kTileElems + j] = vol * fmaf(az, sig[4], fmaf(ax, sig[3], ay * sig[1]));
                sf[(3 * a + 2) * kTileElems + j] = vol * fmaf(ax, sig[5], fmaf(ay, sig[4], az * sig[2]));
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nn; i += kBlock)
        {
            float a0 = 0.f, a1 = 0.f, a2 = 0.f;
            const uint32_t qb = T.csr_off[nb + i], qe = T.csr_off[nb + i + 1];
            for (uint32_t q = qb; q < qe; ++q)
            {
                const uint32_t ent = T.csr_ent[q];
                const uint32_t el = ent >> 2, c = 3u * (ent & 3u);
                a0 += sf[(c + 0) * kTileElems + el];
                a1 += sf[(c + 1) * kTileElems + el];
                a2 += sf[(c + 2) * kTileElems + el];
            }
            float *o = T.part + 3ull * (nb + i);
            o[0] = a0;
            o[1] = a1;
            o[2] = a2;
            if constexpr (MODE == 1)
            {
                const float p0 = sp[i], p1 = sp[ms + i], p2 = sp[2 * ms + i];
                pap += (double)p0 * (double)a0 + (double)p1 * (double)a1 + (double)p2 * (double)a2;
                const uint32_t tg = T.tile_nodes[nb + i];
                if (tg & 0x80000000u)  // the node's owner slot adds its mass term m s_M |p|^2 once
                {
                    const float m = s.mass[tg & 0x7fffffffu] * sM;
                    pap += (double)(m * p0) * (double)p0 + (double)(m * p1) * (double)p1 +
                           (double)(m * p2) * (double)p2;
                }
            }
        }
    }
    if constexpr (MODE == 1)
    {
        const double t = block_sum(pap, red);
        if (threadIdx.x == 0)
            pa.part_dot[blockIdx.x] = t;
    }
}

// pcg.cpp:862-895 for the last iteration of a batch (the next batch's tiles kernel repeats it
// idempotently): one workgroup
__global__ __launch_bounds__(kBlock) void k_pcg_check(Ctl *ctl, const double *__restrict__ prr,
                                                      const double *__restrict__ prz, unsigned nparts, unsigned it,
                                                      double *__restrict__ hist)
{
    __shared__ double red[4];
    if (!ctl->active)
        return;
    float beta;
    (void)residual_step(ctl, prr, prz, nparts, it, hist, red, &beta);
}

template <bool SANITIZE>
__global__ __launch_bounds__(kBlock) void k_keff_finalize(DevSys s, const float *__restrict__ x,
                                                          float *__restrict__ y)
{
    const DevTiles &T = s.t;
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (uint32_t q = T.node_part_off[n]; q < T.node_part_off[n + 1]; ++q)
    {
        const float *pp = T.part + 3ull * T.node_part_slot[q];
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

__global__ __launch_bounds__(kBlock) void k_pcg_update_tiles(DevSys s, const float *__restrict__ rhs,
                                                             const float *__restrict__ inv, float *__restrict__ x,
                                                             float *__restrict__ r, float *__restrict__ z,
                                                             float *__restrict__ p, Ctl *__restrict__ ctl,
                                                             const double *__restrict__ part_dot, unsigned ntp,
                                                             double *__restrict__ prr, double *__restrict__ prz,
                                                             unsigned it)
{
    __shared__ double red[4];
    if (!ctl->active)
        return;
    // pcg.cpp:840-852: alpha = rho / (p . Ap)
    const double denom = fold_all(part_dot, ntp, red);
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
    const double alpha_d = ctl->rho2[it & 1u] / denom;
    if (blockIdx.x == 0 && threadIdx.x == 0)
    {
        ctl->denom = denom;
        ctl->alpha = alpha_d;
        ctl->alpha_last = alpha_d;
    }
    const DevTiles &T = s.t;
    const float alpha = (float)alpha_d, beta = (float)ctl->beta;
    const float sM = (float)s.sM;
    double rr = 0.0, rz = 0.0;
    for (uint32_t n = blockIdx.x * kBlock + threadIdx.x; n < s.N; n += gridDim.x * kBlock)
    {
        float a0 = 0.f, a1 = 0.f, a2 = 0.f;
        for (uint32_t q = T.node_part_off[n]; q < T.node_part_off[n + 1]; ++q)
        {
            const float *pp = T.part + 3ull * T.node_part_slot[q];
            a0 += pp[0];
            a1 += pp[1];
            a2 += pp[2];
        }
        const uint32_t mk = s.mask[n];
        const float m = s.mass[n] * sM;
        const float av[3] = {a0, a1, a2};
        float rv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k)
        {
            const uint32_t d = 3u * n + k;
            const float pk = fmaf(beta, p[d], z[d]);  // same expression as the tiles gather
            const float apk = (mk & (1u << k)) ? pk : fmaf(m, pk, av[k]);
            float xv = fmaf(alpha, pk, x[d]);
            float rw = fmaf(-alpha, apk, r[d]);
            if (mk & (1u << k))
            {
                xv = rhs[d];
                rw = 0.0f;
            }
            x[d] = xv;
            r[d] = rw;
            p[d] = pk;
            rv[k] = rw;
        }
        const float *iv = inv + 9u * n;
#pragma unroll
        for (int k = 0; k < 3; ++k)
        {
            float zk = fmaf(iv[3 * k + 2], rv[2], fmaf(iv[3 * k + 1], rv[1], iv[3 * k] * rv[0]));
            zk = (mk & (1u << k)) ? 0.0f : zk;
            z[3u * n + k] = zk;
            rr += (double)rv[k] * (double)rv[k];
            rz += (double)rv[k] * (double)zk;
        }
    }
    const double t0 = block_sum(rr, red);
    const double t1 = block_sum(rz, red);
    if (threadIdx.x == 0)
    {
        prr[blockIdx.x] = t0;
        prz[blockIdx.x] = t1;
    }
}

inline unsigned grid_for(uint32_t n, uint32_t b) { return (n + b - 1) / b; }

inline size_t tiles_lds(const DevSys &s)
{
    return sizeof(float) * (12 * kTileElems + 3 * (size_t)s.t.max_tile_nodes);
}
}  // namespace

unsigned fast_tile_blocks(const DevSys &s) { return s.t.ntiles < kMaxTileBlocks ? s.t.ntiles : kMaxTileBlocks; }
unsigned fast_update_blocks(const DevSys &s)
{
    const unsigned g = grid_for(s.N, kBlock);
    return g < kMaxUpdateBlocks ? (g ? g : 1u) : kMaxUpdateBlocks;
}

void fast_keff_ds(const DevSys &s, const float *x, float *y, bool sanitize, const Ctl *ctl, double *part,
                  hipStream_t st)
{
    (void)ctl;
    (void)part;
    if (s.N == 0)
        return;
    if (s.t.ntiles)
    {
        const size_t lds = tiles_lds(s);
        const unsigned g = fast_tile_blocks(s);
        PcgArgs none{};
        if (s.iso)
            sanitize ? k_keff_tiles<true, true, 0><<<g, kBlock, lds, st>>>(s, x, none)
                     : k_keff_tiles<true, false, 0><<<g, kBlock, lds, st>>>(s, x, none);
        else
            sanitize ? k_keff_tiles<false, true, 0><<<g, kBlock, lds, st>>>(s, x, none)
                     : k_keff_tiles<false, false, 0><<<g, kBlock, lds, st>>>(s, x, none);
    }
    const unsigned g = grid_for(s.N, kBlock);
    if (sanitize)
        k_keff_finalize<true><<<g, kBlock, 0, st>>>(s, x, y);
    else
        k_keff_finalize<false><<<g, kBlock, 0, st>>>(s, x, y);
}

// iteration `it`: residual step of it-1's update (beta, convergence) + p_new + tile partials + p.Ap shares
void fast_tiles_pcg(cwf_hip_system *h, unsigned it, hipStream_t st)
{
    const DevSys &s = h->ds;
    PcgArgs pa{h->z, h->ctl, h->part0, h->part1, h->part2, fast_update_blocks(s), it, h->hist};
    const unsigned g = fast_tile_blocks(s);
    const size_t lds = tiles_lds(s);
    if (s.iso)
        k_keff_tiles<true, false, 1><<<g, kBlock, lds, st>>>(s, h->p, pa);
    else
        k_keff_tiles<false, false, 1><<<g, kBlock, lds, st>>>(s, h->p, pa);
}

void fast_update_pcg(cwf_hip_system *h, const float *rhs, unsigned it, hipStream_t st)
{
    const DevSys &s = h->ds;
    k_pcg_update_tiles<<<fast_update_blocks(s), kBlock, 0, st>>>(s, rhs, h->inv, h->x, h->r, h->z, h->p, h->ctl,
                                                                 h->part0, fast_tile_blocks(s), h->part1, h->part2,
                                                                 it);
}

void fast_check_pcg(cwf_hip_system *h, unsigned it, hipStream_t st)
{
    k_pcg_check<<<1, kBlock, 0, st>>>(h->ctl, h->part1, h->part2, fast_update_blocks(h->ds), it, h->hist);
}

}  // namespace cwf

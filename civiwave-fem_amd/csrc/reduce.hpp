// reduce.hpp -- fixed-order fp64 reductions shared by the consumer kernels (spmv_tiles.hip) and the PEER exchange
// step (peer.hip): every workgroup that folds the same shares gets the same bits, and the PEER step's fold of a
// rank's shares equals k_fold_pair's (the LOCAL / RCCL schedules') bit for bit.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cwf
{
// fp64 lane exchange through DPP (both halves): CTRL is a GFX9 dpp_ctrl
template <int CTRL> __device__ __forceinline__ double dpp_f64(double v)
{
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_f64(double v, int lane)
{
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                            __builtin_amdgcn_readlane(__double2loint(v), lane));
}
// Wave sum in a fixed order, the same value in every lane (all 64 lanes active). Inside each 16-lane row a butterfly
// through DPP: quad_perm xor 1, xor 2, then row_half_mirror and row_mirror, which act as xor 4 and xor 8 on values
// already uniform over quads / half-rows; each lane adds the same two operands (a + b == b + a bitwise), so every
// lane of a row holds the same row sum. Then ((row0 + row1) + row2) + row3 from readlanes. The ds_bpermute butterfly
// it replaces (__shfl_xor, six LDS-routed rounds of two 32-bit permutes) sat on the critical path of every consumer
// prologue's scalar fold and every producer's share.
__device__ __forceinline__ double wave_sum(double v)
{
    v += dpp_f64<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += dpp_f64<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += dpp_f64<0x141>(v);  // row_half_mirror
    v += dpp_f64<0x140>(v);  // row_mirror
    return ((lane_f64(v, 0) + lane_f64(v, 16)) + lane_f64(v, 32)) + lane_f64(v, 48);
}

// NT-thread block sum in a fixed order; result valid in every thread. red: NT/64 doubles.
template <int NT> __device__ __forceinline__ double block_sum(double v, double *red)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0)
        red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w)
        t += red[w];
    __syncthreads();
    return t;
}

// the pair {a, b} in one pass (one LDS round, two barriers); red: 2 NT / 64 doubles
template <int NT> __device__ __forceinline__ void block_sum2(double a, double b, double *red, double &ta, double &tb)
{
    a = wave_sum(a);
    b = wave_sum(b);
    if ((threadIdx.x & 63) == 0)
    {
        red[2 * (threadIdx.x >> 6)] = a;
        red[2 * (threadIdx.x >> 6) + 1] = b;
    }
    __syncthreads();
    double x = 0.0, y = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w)
    {
        x += red[2 * w];
        y += red[2 * w + 1];
    }
    __syncthreads();
    ta = x;
    tb = y;
}

// Thread t sums p[t], p[t + NT], ... in that order, B loads in flight at a time; the last, partial batch is one
// more batch of B loads (indices clamped into the array, the values past count replaced by +0.0: exact, a sum that
// starts at +0.0 is never -0.0), so a fold of count shares costs ceil(count / (B NT)) memory round trips. (The
// one-load-per-trip tail it replaces cost C3's update pass four dependent round trips for its 2,903 K_eff shares.)
template <int NT, int B = 8>
__device__ __forceinline__ double fold_all(const double *__restrict__ p, unsigned count, double *red,
                                           unsigned stride = 1)
{
    double v = 0.0;
    unsigned i = threadIdx.x;
    for (; i + (B - 1u) * NT < count; i += B * NT)
    {
        double q[B];
#pragma unroll
        for (int u = 0; u < B; ++u)
            q[u] = p[(size_t)(i + u * NT) * stride];
#pragma unroll
        for (int u = 0; u < B; ++u)
            v += q[u];
    }
    if (i < count)
    {
        // loads only for the rows some lane of this wave needs (a wave-uniform bound: a 12-load batch for a
        // 436-share fold issued ten loads per lane for nothing, C2 -5%)
        const unsigned w0 = i - (threadIdx.x & 63u), nb = (count - w0 + NT - 1u) / NT;
        double q[B];
#pragma unroll
        for (int u = 0; u < B; ++u)
            q[u] = (unsigned)u < nb ? p[(size_t)min(i + u * NT, count - 1u) * stride] : 0.0;
#pragma unroll
        for (int u = 0; u < B; ++u)
            v += i + u * NT < count ? q[u] : 0.0;
    }
    return block_sum<NT>(v, red);
}

// the two folds of fold_all in one pass: every load of both arrays in flight together, one block reduction of
// the pair (red: 2 NT / 64 doubles); fixed order, so every workgroup gets the same pair
template <int NT, int B = 4>
__device__ __forceinline__ void fold_all2(const double *__restrict__ pa, const double *__restrict__ pb, unsigned count,
                                          double *red, unsigned stride, double &ta, double &tb)
{
    double va = 0.0, vb = 0.0;
    unsigned i = threadIdx.x;
    for (; i + (B - 1u) * NT < count; i += B * NT)
    {
        double qa[B], qb[B];
#pragma unroll
        for (int u = 0; u < B; ++u)
        {
            qa[u] = pa[(size_t)(i + u * NT) * stride];
            qb[u] = pb[(size_t)(i + u * NT) * stride];
        }
#pragma unroll
        for (int u = 0; u < B; ++u)
        {
            va += qa[u];
            vb += qb[u];
        }
    }
    if (i < count)  // the partial batch, as in fold_all
    {
        const unsigned w0 = i - (threadIdx.x & 63u), nb = (count - w0 + NT - 1u) / NT;
        double qa[B], qb[B];
#pragma unroll
        for (int u = 0; u < B; ++u)
        {
            const size_t k = (size_t)min(i + u * NT, count - 1u) * stride;
            qa[u] = (unsigned)u < nb ? pa[k] : 0.0;
            qb[u] = (unsigned)u < nb ? pb[k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < B; ++u)
        {
            va += i + u * NT < count ? qa[u] : 0.0;
            vb += i + u * NT < count ? qb[u] : 0.0;
        }
    }
    va = wave_sum(va);
    vb = wave_sum(vb);
    if ((threadIdx.x & 63) == 0)
    {
        red[2 * (threadIdx.x >> 6)] = va;
        red[2 * (threadIdx.x >> 6) + 1] = vb;
    }
    __syncthreads();
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w)
    {
        a += red[2 * w];
        b += red[2 * w + 1];
    }
    __syncthreads();
    ta = a;
    tb = b;
}

// K folds of fold_all's order in one pass: element i of array q is p[q stride + i istride] (i < count), thread t
// sums its elements t, t + NT, ... in that order, 2K loads in flight per trip (two rows per array), then each
// array's wave and block sums as block_sum. red: K NT / 64 doubles. The fused PCG iteration's five scalars
// (lattice_fused.inc): a workgroup's shares (istride 1) or the all-gathered per-rank totals (stride 1, istride K).
// NTV < NT: the fold of an NTV-thread block, bitwise (threads >= NTV hold +0.0, and adding +0.0 to a sum from +0.0
// changes nothing): the PEER step's 1024-thread workgroup folds a rank's shares as a 256-thread one does.
template <int NT, int K, int NTV = NT>
__device__ __forceinline__ void fold_k(const double *__restrict__ p, unsigned count, unsigned stride, double *red,
                                       double out[K], unsigned istride = 1)
{
    double v[K];
#pragma unroll
    for (int q = 0; q < K; ++q)
        v[q] = 0.0;
    for (unsigned i = threadIdx.x; threadIdx.x < (unsigned)NTV && i < count; i += 2u * NTV)
    {
        const bool two = i + NTV < count;
        const unsigned i2 = two ? i + NTV : i;
        double a[K], b[K];
#pragma unroll
        for (int q = 0; q < K; ++q)
        {
            a[q] = p[(size_t)q * stride + (size_t)i * istride];
            b[q] = p[(size_t)q * stride + (size_t)i2 * istride];
        }
#pragma unroll
        for (int q = 0; q < K; ++q)
        {
            v[q] += a[q];
            v[q] += two ? b[q] : 0.0;
        }
    }
#pragma unroll
    for (int q = 0; q < K; ++q)
    {
        v[q] = wave_sum(v[q]);
        if ((threadIdx.x & 63) == 0)
            red[K * (threadIdx.x >> 6) + q] = v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < K; ++q)
    {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w)
            t += red[K * w + q];
        out[q] = t;
    }
    __syncthreads();
}

// K block sums in one LDS round (the order of block_sum per value); red: K NT / 64 doubles
template <int NT, int K> __device__ __forceinline__ void block_sum_k(double v[K], double *red)
{
#pragma unroll
    for (int q = 0; q < K; ++q)
    {
        v[q] = wave_sum(v[q]);
        if ((threadIdx.x & 63) == 0)
            red[K * (threadIdx.x >> 6) + q] = v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < K; ++q)
    {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w)
            t += red[K * w + q];
        v[q] = t;
    }
    __syncthreads();
}

}  // namespace cwf

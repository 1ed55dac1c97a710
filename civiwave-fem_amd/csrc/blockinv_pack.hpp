// blockinv_pack.hpp -- FAST mode's 16-B per-node block-Jacobi inverse (host and device share this code).
//
// The reference's preconditioner (pcg.cpp:270-408) is a per-node 3x3 inverse B stored as
// 9 f32, with the rows of constrained axes replaced by identity. The FAST update pass reads B once per
// node per PCG iteration, so it is packed to 16 B in a Jacobi-scaled form:
//
//   S   = max over free axes of B_kk                    (fp32, word 0)
//   t_k = sqrt(B_kk / S)   in (0, 1]                    (fp16; 0 on a constrained axis)
//   C_ij = B_ij / sqrt(B_ii B_jj)   in (-1, 1)          (fp16, i < j; 0 when i or j is constrained)
//   dequantised  B~_kk = S (t_k t_k),  B~_ij = S ((t_i t_j) C_ij)
//
// Every entry keeps ~2^-11 precision relative to its own row and column scale, whatever the spread of
// the block's diagonal: a block with free entries ~1e-10 next to a constrained axis (a node fixed only in
// z, config.hpp:208 constrain_axis) or with diagonal entries 1e3 apart keeps its small entries. Only the
// free-free sub-block is stored: a constrained axis has z = 0 and r = 0 there (pcg.cpp:452, 466-472), so
// its row and column never act.
//
// Fallback: when the block is not usable in this form -- a free diagonal entry not > 0 or not finite,
// t_k below fp16's normal range (a diagonal spread > 2^28), |C_ij| >= 1, or a dequantised correlation
// matrix C~ whose determinant is below 1/16 (near-singular: the 2^-12 quantisation step could move its
// smallest eigenvalue by more than ~3%) -- word 0 holds -1.0f and the update pass reads the node's
// symmetrised fp32 block from the 9-float copy instead.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace cwf
{

constexpr float kInvPackMinDet = 0.0625f;

// v: {a00 a01 a02 a11 a12 a22} (upper triangle of B); mk: bit k = axis k constrained.
// w: packed record; d: the operator the solve applies, {a00 a01 a02 a11 a12 a22}. Returns false on fallback.
__host__ __device__ inline bool pack_block_inverse(const float v[6], uint32_t mk, uint32_t w[4], float d[6])
{
    const int di[3] = {0, 3, 5};            // diagonal slots in v
    const int oi[3] = {1, 2, 4};            // off-diagonal slots: (0,1) (0,2) (1,2)
    const int oa[3] = {0, 0, 1}, ob[3] = {1, 2, 2};
    bool ok = true;
    float S = 0.f;
    for (int k = 0; k < 3; ++k)
        if (!(mk & (1u << k)))
        {
            const float b = v[di[k]];
            if (!(b > 0.f) || !(b < INFINITY))
                ok = false;
            else
                S = S > b ? S : b;
        }
    _Float16 qt[3] = {(_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
    _Float16 qc[3] = {(_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
    if (ok && S > 0.f)
    {
        for (int k = 0; k < 3; ++k)
            if (!(mk & (1u << k)))
            {
                const double t = sqrt((double)v[di[k]] / (double)S);
                qt[k] = (_Float16)(float)t;
                if ((float)qt[k] < 6.103515625e-05f)  // 2^-14: below fp16's normal range
                    ok = false;
            }
        for (int j = 0; j < 3; ++j)
        {
            const int a = oa[j], b = ob[j];
            if ((mk & (1u << a)) || (mk & (1u << b)))
                continue;
            const double c = (double)v[oi[j]] / sqrt((double)v[di[a]] * (double)v[di[b]]);
            if (!(fabs(c) < 1.0))
                ok = false;
            else
                qc[j] = (_Float16)(float)c;
        }
        if (ok)
        {
            const double c01 = (float)qc[0], c02 = (float)qc[1], c12 = (float)qc[2];
            const double det = 1.0 + 2.0 * c01 * c02 * c12 - c01 * c01 - c02 * c02 - c12 * c12;
            if (!(det >= (double)kInvPackMinDet) || !(1.0 - c01 * c01 > 0.0))
                ok = false;
        }
    }
    if (!ok)
    {
        w[0] = __builtin_bit_cast(uint32_t, -1.0f);
        w[1] = w[2] = w[3] = 0u;
        for (int k = 0; k < 6; ++k)
            d[k] = v[k];
        for (int k = 0; k < 3; ++k)
            if (mk & (1u << k))
            {
                d[di[k]] = 0.f;
                for (int j = 0; j < 3; ++j)
                    if (oa[j] == k || ob[j] == k)
                        d[oi[j]] = 0.f;
            }
        return false;
    }
    w[0] = __builtin_bit_cast(uint32_t, S);
    w[1] = (uint32_t)__builtin_bit_cast(uint16_t, qt[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, qt[1]) << 16);
    w[2] = (uint32_t)__builtin_bit_cast(uint16_t, qt[2]) | ((uint32_t)__builtin_bit_cast(uint16_t, qc[0]) << 16);
    w[3] = (uint32_t)__builtin_bit_cast(uint16_t, qc[1]) | ((uint32_t)__builtin_bit_cast(uint16_t, qc[2]) << 16);
    const float t0 = (float)qt[0], t1 = (float)qt[1], t2 = (float)qt[2];
    d[0] = S * (t0 * t0);
    d[3] = S * (t1 * t1);
    d[5] = S * (t2 * t2);
    d[1] = S * ((t0 * t1) * (float)qc[0]);
    d[2] = S * ((t0 * t2) * (float)qc[1]);
    d[4] = S * ((t1 * t2) * (float)qc[2]);
    return true;
}

// the update pass's decode of a non-fallback record: bit for bit the d[] of pack_block_inverse
__host__ __device__ inline void unpack_block_inverse(const uint32_t w1, const uint32_t w2, const uint32_t w3,
                                                     const float S, float d[6])
{
    const auto h = [](uint32_t x, int hi) {
        return (float)__builtin_bit_cast(_Float16, (uint16_t)(hi ? x >> 16 : x & 0xffffu));
    };
    const float t0 = h(w1, 0), t1 = h(w1, 1), t2 = h(w2, 0);
    d[0] = S * (t0 * t0);
    d[3] = S * (t1 * t1);
    d[5] = S * (t2 * t2);
    d[1] = S * ((t0 * t1) * h(w2, 1));
    d[2] = S * ((t0 * t2) * h(w3, 0));
    d[4] = S * ((t1 * t2) * h(w3, 1));
}

}  // namespace cwf

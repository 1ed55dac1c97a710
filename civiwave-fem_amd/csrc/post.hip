// post.hip -- derived fields on the device, bit-exact with src/post/derived_fields.cpp:139-211.
//
// Per element (derived_fields.cpp:157-186): strain from grad(N) . u in fp64 (the reference's
// per-corner statement order, shear pairs summed before they are added), stress = D strain as the
// full row fold (structural zeros of an isotropic D skipped, exact -- see kernels_parity.hip),
// von Mises from the fp64 stress, all stored as f32 {strain[6], stress[6], vm} (the 52-B layout of
// cwf::post::ElementField).
// Per node (derived_fields.cpp:188-210): the reference scatters V*strain, V*stress and V into fp64
// accumulators in ascending element order; one thread per node gathers its ascending CSR from +0.0
// (the same fold order), recomputing each incident element's fp64 strain/stress (bitwise the values
// the element pass produced), then divides by the volume weight and re-evaluates von Mises from the
// averaged stress. This TU inherits -ffp-contract=off and IEEE fp64 div/sqrt from the Makefile.
#include "cwf_internal.hpp"

namespace cwf
{
namespace
{

constexpr int kBlock = 256;

struct ElemTensors
{
    double strain[6];
    double stress[6];
};

// derived_fields.cpp:164-180 + stiffness_mul :66-80 for element e (tet4: 4 local nodes). HEX (native
// hex8, SURVEY 8f4, parity unpinned): the same statement order over 8 corners with the element-centre
// gradients cwf_preprocess_hex8 stores in the 24 gradient slots, i.e. the centroid strain.
template <bool ISO, bool HEX = false>
__device__ __forceinline__ void element_tensors(const DevSys &s, const float *__restrict__ u, uint32_t e,
                                                ElemTensors &t)
{
    constexpr int K = HEX ? 8 : 4;
    uint32_t c[K];
    float g[3 * K];
    if constexpr (HEX)
    {
#pragma unroll
        for (int a = 0; a < 8; ++a)
            c[a] = s.hconn[8ull * e + a];
#pragma unroll
        for (int i = 0; i < 24; ++i)
            g[i] = s.hgrad[24ull * e + i];
    }
    else
    {
        const uint4 q0 = s.erec[4u * e + 0u];
        const uint4 g0 = s.erec[4u * e + 1u], g1 = s.erec[4u * e + 2u], g2 = s.erec[4u * e + 3u];
        const uint32_t cc[4] = {q0.x, q0.y, q0.z, q0.w};
        const float gg[12] = {__uint_as_float(g0.x), __uint_as_float(g0.y), __uint_as_float(g0.z),
                              __uint_as_float(g0.w), __uint_as_float(g1.x), __uint_as_float(g1.y),
                              __uint_as_float(g1.z), __uint_as_float(g1.w), __uint_as_float(g2.x),
                              __uint_as_float(g2.y), __uint_as_float(g2.z), __uint_as_float(g2.w)};
#pragma unroll
        for (int a = 0; a < 4; ++a)
            c[a] = cc[a];
#pragma unroll
        for (int i = 0; i < 12; ++i)
            g[i] = gg[i];
    }
    double e6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int a = 0; a < K; ++a)
    {
        const double ux = (double)u[3ull * c[a] + 0], uy = (double)u[3ull * c[a] + 1], uz = (double)u[3ull * c[a] + 2];
        const double gx = (double)g[3 * a], gy = (double)g[3 * a + 1], gz = (double)g[3 * a + 2];
        e6[0] += gx * ux;
        e6[1] += gy * uy;
        e6[2] += gz * uz;
        e6[3] += gy * ux + gx * uy;
        e6[4] += gz * uy + gy * uz;
        e6[5] += gz * ux + gx * uz;
    }
    const double *D = s.dmat + 36ull * s.mat[e];
#pragma unroll
    for (int r = 0; r < 6; ++r)
    {
        t.strain[r] = e6[r];
        double acc = 0.0;
        if constexpr (ISO)
        {
            if (r < 3)
            {
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    acc += D[6 * r + k] * e6[k];
            }
            else
                acc += D[6 * r + r] * e6[r];
        }
        else
        {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                acc += D[6 * r + k] * e6[k];
        }
        t.stress[r] = acc;
    }
}

// derived_fields.cpp:47-63
__device__ __forceinline__ double von_mises(const double s[6])
{
    const double dxy = s[0] - s[1], dyz = s[1] - s[2], dzx = s[2] - s[0];
    const double energy = 0.5 * (dxy * dxy + dyz * dyz + dzx * dzx) + 3.0 * (s[3] * s[3] + s[4] * s[4] + s[5] * s[5]);
    return sqrt(energy < 0.0 ? 0.0 : energy);  // std::max(energy, 0.0), NaN passes through
}

template <bool ISO, bool HEX>
__global__ __launch_bounds__(kBlock) void k_derived_elements(DevSys s, const float *__restrict__ u,
                                                             float *__restrict__ out)
{
    const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= s.E)
        return;
    ElemTensors t;
    element_tensors<ISO, HEX>(s, u, e, t);
    float *o = out + 13ull * e;
#pragma unroll
    for (int c = 0; c < 6; ++c)
    {
        o[c] = (float)t.strain[c];
        o[6 + c] = (float)t.stress[c];
    }
    o[12] = (float)von_mises(t.stress);
}

template <bool ISO, bool HEX>
__global__ __launch_bounds__(kBlock) void k_derived_nodes(DevSys s, const float *__restrict__ u, float *__restrict__ out)
{
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    double ws = 0.0, as[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, at[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (uint32_t q = s.off[n]; q < s.off[n + 1]; ++q)
    {
        const uint32_t e = s.inc[q] >> (HEX ? 3 : 2);
        ElemTensors t;
        element_tensors<ISO, HEX>(s, u, e, t);
        const double vol = (double)s.vol[e];
        ws += vol;  // accumulate_node (derived_fields.cpp:82-95)
#pragma unroll
        for (int c = 0; c < 6; ++c)
        {
            as[c] += t.strain[c] * vol;
            at[c] += t.stress[c] * vol;
        }
    }
    float *o = out + 13ull * n;
    if (ws <= 0.0)  // finalize_node (derived_fields.cpp:110-134): isolated node -> zero field
    {
#pragma unroll
        for (int c = 0; c < 13; ++c)
            o[c] = 0.0f;
        return;
    }
    const double inv = 1.0 / ws;
    double avg[6];
#pragma unroll
    for (int c = 0; c < 6; ++c)
    {
        o[c] = (float)(as[c] * inv);
        avg[c] = at[c] * inv;
        o[6 + c] = (float)avg[c];
    }
    o[12] = (float)von_mises(avg);
}

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

template <bool HEX>
void derived_fields_k(const DevSys &s, const float *u, float *elem_out, float *node_out, hipStream_t st)
{
    if (s.E && elem_out)
    {
        if (s.iso)
            k_derived_elements<true, HEX><<<grid_for(s.E), kBlock, 0, st>>>(s, u, elem_out);
        else
            k_derived_elements<false, HEX><<<grid_for(s.E), kBlock, 0, st>>>(s, u, elem_out);
    }
    if (s.N && node_out)
    {
        if (s.iso)
            k_derived_nodes<true, HEX><<<grid_for(s.N), kBlock, 0, st>>>(s, u, node_out);
        else
            k_derived_nodes<false, HEX><<<grid_for(s.N), kBlock, 0, st>>>(s, u, node_out);
    }
}
}  // namespace

void derived_fields(cwf_hip_system *h, const float *u, float *elem_out, float *node_out, hipStream_t st)
{
    if (h->ds.hex)
        derived_fields_k<true>(h->ds, u, elem_out, node_out, st);
    else
        derived_fields_k<false>(h->ds, u, elem_out, node_out, st);
}

}  // namespace cwf

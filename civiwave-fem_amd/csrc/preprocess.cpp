// preprocess.cpp -- host-side mesh preprocessing for the hot path: tet gradients, volumes,
// lumped masses and the ascending node->element CSR, restating mesh::pre::run
// (src/mesh/preprocess.cpp:268-405) and the fp64->fp32 casts of pack::build_packed_buffers
// (src/mesh/pack.cpp:41-57,176-200) so the packed f32 arrays are bit-identical to the reference's.
// Compiled with -ffp-contract=off (no FMA) like the rest of the parity path.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "cwf_internal.hpp"

namespace
{
inline void sub3(const double *a, const double *b, double *o)
{
    o[0] = a[0] - b[0];
    o[1] = a[1] - b[1];
    o[2] = a[2] - b[2];
}
inline void cross3(const double *l, const double *r, double *o)  // math.hpp:124-128
{
    o[0] = (l[1] * r[2]) - (l[2] * r[1]);
    o[1] = (l[2] * r[0]) - (l[0] * r[2]);
    o[2] = (l[0] * r[1]) - (l[1] * r[0]);
}
inline double dot3(const double *l, const double *r) { return (l[0] * r[0]) + (l[1] * r[1]) + (l[2] * r[2]); }
inline float safe_f32(double v)  // pack.cpp:41-57
{
    if (!std::isfinite(v))
        return v > 0 ? std::numeric_limits<float>::infinity()
                     : (v < 0 ? -std::numeric_limits<float>::infinity() : std::numeric_limits<float>::quiet_NaN());
    if (v > (double)FLT_MAX)
        return FLT_MAX;
    if (v < -(double)FLT_MAX)
        return -FLT_MAX;
    return (float)v;
}
}  // namespace

extern "C" int cwf_preprocess_tets(uint64_t N, uint64_t E, const double *coords, const uint32_t *tets,
                                   const uint32_t *material_index, const double *density, uint64_t material_count,
                                   float *grads24, float *volume, double *mass64, float *mass32, uint32_t *offsets,
                                   uint32_t *adj_elem, uint8_t *adj_local, uint32_t *conn8)
{
    using cwf::set_error;
    if ((N && (!coords || !mass64 || !mass32 || !offsets)) ||
        (E && (!tets || !material_index || !density || !grads24 || !volume || !adj_elem || !adj_local)))
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (N == 0)
        return set_error(nullptr, CWF_ERR_SIZE, "mesh has zero nodes", "mesh");
    if (E == 0)
        return set_error(nullptr, CWF_ERR_SIZE, "mesh has zero elements", "mesh");
    std::vector<uint32_t> counts(N, 0);
    for (uint64_t n = 0; n < N; ++n)
        mass64[n] = 0.0;
    for (uint64_t e = 0; e < E; ++e)
    {
        const double *p[4];
        for (int a = 0; a < 4; ++a)
        {
            const uint32_t n = tets[e * 4 + a];
            if (n >= N)
                return set_error(nullptr, CWF_ERR_NODE_RANGE, "element references node out of range",
                                 "elements [" + std::to_string(e) + "]");
            p[a] = coords + 3 * (uint64_t)n;
            ++counts[n];
        }
        if (material_index[e] >= material_count)
            return set_error(nullptr, CWF_ERR_MATERIAL_RANGE, "element physical group missing assignment",
                             "elements [" + std::to_string(e) + "]");
        double e0[3], e1[3], e2[3], c12[3];
        sub3(p[1], p[0], e0);
        sub3(p[2], p[0], e1);
        sub3(p[3], p[0], e2);
        cross3(e1, e2, c12);
        const double volume6 = dot3(e0, c12);
        const double vol = std::fabs(volume6) / 6.0;
        if (vol <= DBL_EPSILON)
            return set_error(nullptr, CWF_ERR_SIZE, "tetrahedron volume non-positive",
                             "elements [" + std::to_string(e) + "]");
        const double inv6 = -1.0 / volume6;  // compute_tet_gradients (:268-280)
        double g[4][3], a0[3], b0[3];
        sub3(p[2], p[1], a0);
        sub3(p[3], p[1], b0);
        cross3(a0, b0, g[0]);
        sub3(p[3], p[0], a0);
        sub3(p[2], p[0], b0);
        cross3(a0, b0, g[1]);
        sub3(p[1], p[0], a0);
        sub3(p[3], p[0], b0);
        cross3(a0, b0, g[2]);
        sub3(p[2], p[0], a0);
        sub3(p[1], p[0], b0);
        cross3(a0, b0, g[3]);
        float *gr = grads24 + e * 24;
        for (int a = 0; a < 4; ++a)
            for (int k = 0; k < 3; ++k)
                gr[3 * a + k] = safe_f32(g[a][k] * inv6);
        std::memset(gr + 12, 0, 12 * sizeof(float));
        volume[e] = safe_f32(vol);
        const double lump = density[material_index[e]] * vol / 4.0;
        for (int a = 0; a < 4; ++a)
            mass64[tets[e * 4 + a]] += lump;
        if (conn8)
            for (int a = 0; a < 8; ++a)
                conn8[e * 8 + a] = a < 4 ? tets[e * 4 + a] : 0xFFFFFFFFu;
    }
    uint32_t acc = 0;
    for (uint64_t n = 0; n < N; ++n)
    {
        offsets[n] = acc;
        acc += counts[n];
        counts[n] = 0;
        mass32[n] = safe_f32(mass64[n]);
    }
    offsets[N] = acc;
    for (uint64_t e = 0; e < E; ++e)
        for (int a = 0; a < 4; ++a)
        {
            const uint32_t n = tets[e * 4 + a];
            const uint32_t w = offsets[n] + counts[n]++;
            adj_elem[w] = (uint32_t)e;
            adj_local[w] = (uint8_t)a;
        }
    return 0;
}

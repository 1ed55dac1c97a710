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

// ---- native hex8 ---------------------------------------------------------------
// The reference stops here ("only tetrahedron elements supported in Phase 3", preprocess.cpp:326-330);
// this is the trilinear isoparametric element (Gmsh/VTK corner order, 2x2x2 Gauss) the FAST hex8
// kernels integrate: V = sum_gp det J, lumped mass rho V / 8 per corner, grads24 = dN_a/dx at the
// element centre (the 8 x 3 gradient slots the packed layout reserves, pcg.hpp:67-86; the post
// stack's centroid strain reads them). Parity unpinned (no reference arithmetic exists).
namespace
{
const double kHexSign[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
                               {-1, -1, 1},  {1, -1, 1},  {1, 1, 1},  {-1, 1, 1}};

// dN_a/dx at reference point q of the hex with corners X; returns det J
double hex_grads(const double X[8][3], const double q[3], double g[8][3])
{
    double dN[8][3], J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int a = 0; a < 8; ++a)
    {
        const double *s = kHexSign[a];
        const double f0 = 1.0 + s[0] * q[0], f1 = 1.0 + s[1] * q[1], f2 = 1.0 + s[2] * q[2];
        dN[a][0] = 0.125 * s[0] * f1 * f2;
        dN[a][1] = 0.125 * f0 * s[1] * f2;
        dN[a][2] = 0.125 * f0 * f1 * s[2];
        for (int m = 0; m < 3; ++m)
            for (int l = 0; l < 3; ++l)
                J[m][l] += X[a][m] * dN[a][l];
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
    for (int a = 0; a < 8; ++a)
        for (int m = 0; m < 3; ++m)
            g[a][m] = (dN[a][0] * A[0][m] + dN[a][1] * A[1][m] + dN[a][2] * A[2][m]) / det;
    return det;
}
}  // namespace

extern "C" int cwf_preprocess_hex8(uint64_t N, uint64_t E, const double *coords, const uint32_t *hexes,
                                   const uint32_t *material_index, const double *density, uint64_t material_count,
                                   float *grads24, float *volume, double *mass64, float *mass32, uint32_t *offsets,
                                   uint32_t *adj_elem, uint8_t *adj_local, uint32_t *conn8)
{
    using cwf::set_error;
    if ((N && (!coords || !mass64 || !mass32 || !offsets)) ||
        (E && (!hexes || !material_index || !density || !grads24 || !volume || !adj_elem || !adj_local)))
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (N == 0)
        return set_error(nullptr, CWF_ERR_SIZE, "mesh has zero nodes", "mesh");
    if (E == 0)
        return set_error(nullptr, CWF_ERR_SIZE, "mesh has zero elements", "mesh");
    const double r = 1.0 / std::sqrt(3.0);
    std::vector<uint32_t> counts(N, 0);
    for (uint64_t n = 0; n < N; ++n)
        mass64[n] = 0.0;
    for (uint64_t e = 0; e < E; ++e)
    {
        double X[8][3], g[8][3];
        for (int a = 0; a < 8; ++a)
        {
            const uint32_t n = hexes[e * 8 + a];
            if (n >= N)
                return set_error(nullptr, CWF_ERR_NODE_RANGE, "element references node out of range",
                                 "elements [" + std::to_string(e) + "]");
            for (int m = 0; m < 3; ++m)
                X[a][m] = coords[3 * (uint64_t)n + m];
            ++counts[n];
        }
        if (material_index[e] >= material_count)
            return set_error(nullptr, CWF_ERR_MATERIAL_RANGE, "element physical group missing assignment",
                             "elements [" + std::to_string(e) + "]");
        double vol = 0.0;
        for (int p = 0; p < 8; ++p)
        {
            const double q[3] = {(p & 1) ? r : -r, (p & 2) ? r : -r, (p & 4) ? r : -r};
            const double det = hex_grads(X, q, g);
            if (!(det > 0.0))
                return set_error(nullptr, CWF_ERR_SIZE, "hexahedron Jacobian non-positive (inverted or degenerate)",
                                 "elements [" + std::to_string(e) + "]");
            vol += det;
        }
        const double q0[3] = {0.0, 0.0, 0.0};
        (void)hex_grads(X, q0, g);
        float *gr = grads24 + e * 24;
        for (int a = 0; a < 8; ++a)
            for (int m = 0; m < 3; ++m)
                gr[3 * a + m] = safe_f32(g[a][m]);
        volume[e] = safe_f32(vol);
        const double lump = density[material_index[e]] * vol / 8.0;
        for (int a = 0; a < 8; ++a)
            mass64[hexes[e * 8 + a]] += lump;
        if (conn8)
            for (int a = 0; a < 8; ++a)
                conn8[e * 8 + a] = hexes[e * 8 + a];
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
        for (int a = 0; a < 8; ++a)
        {
            const uint32_t n = hexes[e * 8 + a];
            const uint32_t w = offsets[n] + counts[n]++;
            adj_elem[w] = (uint32_t)e;
            adj_local[w] = (uint8_t)a;
        }
    return 0;
}

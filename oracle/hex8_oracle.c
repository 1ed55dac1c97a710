/*
 * hex8_oracle.c -- CPU restatement of the native trilinear hex8 operator.
 *
 * TEST INFRASTRUCTURE ONLY (same rules as cwf_oracle.c): loaded by tests/ as the checker.
 *
 * PARITY UNPINNED: the reference rejects hex8 elements ("only tetrahedron elements supported in
 * Phase 3", src/mesh/preprocess.cpp:326-330) although its loader reads them (mesh.cpp:234-260,
 * gmsh type 5) and its packed layout reserves 8 corner slots and 24 gradient floats per element
 * (pcg.hpp:67-86). There is no reference arithmetic to reproduce, so this file is the textbook
 * isoparametric element, written for clarity rather than speed, in fp64:
 *   - corners in Gmsh/VTK order: 0(-,-,-) 1(+,-,-) 2(+,+,-) 3(-,+,-) 4(-,-,+) 5(+,-,+) 6(+,+,+) 7(-,+,+);
 *   - N_a = (1 + xi xi_a)(1 + eta eta_a)(1 + zeta zeta_a) / 8, full 2x2x2 Gauss (points +-1/sqrt(3), w = 1);
 *   - B, D and the Voigt order (xx, yy, zz, xy, yz, xz; engineering shear) of the tet path
 *     (pcg.cpp:592-651): f_a = sum_gp |det J| B_a^T D B u * s_K.
 * The GPU kernel (spmv_tiles.hip, k_keff_hex_tiles) evaluates the same integrals with sum
 * factorisation in fp32; tests compare both and check the operator's physics (patch test, rigid
 * modes, symmetry, convergence towards the oracle Kuhn-tet solution).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "cwf_oracle.h"

static const double kSign[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
                                   {-1, -1, 1},  {1, -1, 1},  {1, 1, 1},  {-1, 1, 1}};

/* dN_a/dxi_l at (xi, eta, zeta) */
static void ref_grads(const double q[3], double dN[8][3])
{
    for (int a = 0; a < 8; ++a)
    {
        const double s0 = kSign[a][0], s1 = kSign[a][1], s2 = kSign[a][2];
        const double f0 = 1.0 + s0 * q[0], f1 = 1.0 + s1 * q[1], f2 = 1.0 + s2 * q[2];
        dN[a][0] = 0.125 * s0 * f1 * f2;
        dN[a][1] = 0.125 * f0 * s1 * f2;
        dN[a][2] = 0.125 * f0 * f1 * s2;
    }
}

/* physical gradients g[a][m] = dN_a/dx_m and det J at reference point q; returns det J */
static double phys_grads(const double X[8][3], const double q[3], double g[8][3])
{
    double dN[8][3], J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    ref_grads(q, dN);
    for (int a = 0; a < 8; ++a)
        for (int m = 0; m < 3; ++m)
            for (int l = 0; l < 3; ++l)
                J[m][l] += X[a][m] * dN[a][l]; /* J[m][l] = dx_m / dxi_l */
    double A[3][3]; /* adjugate: A = det * J^-1 */
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
    /* dN/dx_m = sum_l dN/dxi_l * (J^-1)[l][m] */
    for (int a = 0; a < 8; ++a)
        for (int m = 0; m < 3; ++m)
        {
            double s = 0.0;
            for (int l = 0; l < 3; ++l)
                s += dN[a][l] * A[l][m];
            g[a][m] = s / det;
        }
    return det;
}

static void gauss_point(int p, double q[3])
{
    const double r = 1.0 / sqrt(3.0);
    q[0] = (p & 1) ? r : -r;
    q[1] = (p & 2) ? r : -r;
    q[2] = (p & 4) ? r : -r;
}

static int load_corners(const double *coords, const uint32_t *conn8, uint64_t N, uint64_t e, double X[8][3])
{
    for (int a = 0; a < 8; ++a)
    {
        const uint32_t n = conn8[8 * e + a];
        if (n >= N)
            return -1;
        for (int m = 0; m < 3; ++m)
            X[a][m] = coords[3 * (uint64_t)n + m];
    }
    return 0;
}

int orc_hex8_preprocess(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8,
                        const uint32_t *material_index, const double *density, uint64_t material_count,
                        double *volume, double *mass64, float *grads24)
{
    for (uint64_t n = 0; n < N; ++n)
        mass64[n] = 0.0;
    for (uint64_t e = 0; e < E; ++e)
    {
        double X[8][3], g[8][3], q[3];
        if (load_corners(coords, conn8, N, e, X) || material_index[e] >= material_count)
            return -1;
        double v = 0.0;
        for (int p = 0; p < 8; ++p)
        {
            gauss_point(p, q);
            const double det = phys_grads(X, q, g);
            if (!(det > 0.0))
                return -2;
            v += det;
        }
        volume[e] = v;
        const double q0[3] = {0.0, 0.0, 0.0};
        (void)phys_grads(X, q0, g);
        for (int a = 0; a < 8; ++a)
            for (int m = 0; m < 3; ++m)
                grads24[24 * e + 3 * a + m] = (float)g[a][m];
        const double share = density[material_index[e]] * v / 8.0;
        for (int a = 0; a < 8; ++a)
            mass64[conn8[8 * e + a]] += share;
    }
    return 0;
}

/* y = K_eff x with apply_keff's boundary semantics (pcg.cpp:530-546, 664-691); acc: [3N] fp64 result.
 * x is f32 (x32) or fp64 (x64, then y may be NULL and acc is the fp64 product). */
static int hex8_apply_impl(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8,
                           const uint32_t *material_index, const double *D36, double sK, double sM, const float *mass,
                           const uint32_t *mask, const float *x32, const double *x64, float *y, double *acc)
{
#define XV(d) (x32 ? (double)x32[d] : x64[d])
    for (uint64_t n = 0; n < N; ++n)
        for (int k = 0; k < 3; ++k)
            acc[3 * n + k] = 0.0;
    for (uint64_t e = 0; e < E; ++e)
    {
        double X[8][3], g[8][3], q[3], u[8][3];
        if (load_corners(coords, conn8, N, e, X))
            return -1;
        for (int a = 0; a < 8; ++a)
        {
            const uint32_t n = conn8[8 * e + a];
            for (int k = 0; k < 3; ++k)
                u[a][k] = (mask[n] & (1u << k)) ? 0.0 : XV(3 * (uint64_t)n + k);
        }
        const double *D = D36 + 36 * material_index[e];
        double f[8][3];
        memset(f, 0, sizeof f);
        for (int p = 0; p < 8; ++p)
        {
            gauss_point(p, q);
            const double det = phys_grads(X, q, g);
            double eps[6] = {0, 0, 0, 0, 0, 0};
            for (int a = 0; a < 8; ++a)
            {
                eps[0] += g[a][0] * u[a][0];
                eps[1] += g[a][1] * u[a][1];
                eps[2] += g[a][2] * u[a][2];
                eps[3] += g[a][1] * u[a][0] + g[a][0] * u[a][1];
                eps[4] += g[a][2] * u[a][1] + g[a][1] * u[a][2];
                eps[5] += g[a][2] * u[a][0] + g[a][0] * u[a][2];
            }
            double sig[6];
            for (int r = 0; r < 6; ++r)
            {
                double s = 0.0;
                for (int c = 0; c < 6; ++c)
                    s += D[6 * r + c] * eps[c];
                sig[r] = s * fabs(det) * sK;
            }
            for (int a = 0; a < 8; ++a)
            {
                f[a][0] += g[a][0] * sig[0] + g[a][1] * sig[3] + g[a][2] * sig[5];
                f[a][1] += g[a][1] * sig[1] + g[a][0] * sig[3] + g[a][2] * sig[4];
                f[a][2] += g[a][2] * sig[2] + g[a][1] * sig[4] + g[a][0] * sig[5];
            }
        }
        for (int a = 0; a < 8; ++a)
            for (int k = 0; k < 3; ++k)
                acc[3 * (uint64_t)conn8[8 * e + a] + k] += f[a][k];
    }
    for (uint64_t n = 0; n < N; ++n)
        for (int k = 0; k < 3; ++k)
        {
            const uint64_t d = 3 * n + k;
            const double s = (mask[n] & (1u << k)) ? 0.0 : XV(d);
            acc[d] += (double)mass[n] * sM * s;
            if (mask[n] & (1u << k))
                acc[d] = XV(d);
            if (y)
                y[d] = (float)acc[d];
        }
#undef XV
    return 0;
}

int orc_hex8_apply(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8, const uint32_t *material_index,
                   const double *D36, double sK, double sM, const float *mass, const uint32_t *mask, const float *x,
                   float *y, double *acc)
{
    return hex8_apply_impl(N, E, coords, conn8, material_index, D36, sK, sM, mass, mask, x, NULL, y, acc);
}

/* fp64 in / fp64 out (acc), for reference solves in the tests */
int orc_hex8_apply64(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8,
                     const uint32_t *material_index, const double *D36, double sK, double sM, const float *mass,
                     const uint32_t *mask, const double *x, double *y)
{
    return hex8_apply_impl(N, E, coords, conn8, material_index, D36, sK, sM, mass, mask, NULL, x, NULL, y);
}

/* node diagonal 3x3 blocks of sum_e K_e (stiffness only, x s_K), row-major [9N] */
int orc_hex8_diag_blocks(uint64_t N, uint64_t E, const double *coords, const uint32_t *conn8,
                         const uint32_t *material_index, const double *D36, double sK, double *blocks)
{
    for (uint64_t i = 0; i < 9 * N; ++i)
        blocks[i] = 0.0;
    for (uint64_t e = 0; e < E; ++e)
    {
        double X[8][3], g[8][3], q[3];
        if (load_corners(coords, conn8, N, e, X))
            return -1;
        const double *D = D36 + 36 * material_index[e];
        for (int p = 0; p < 8; ++p)
        {
            gauss_point(p, q);
            const double det = phys_grads(X, q, g);
            const double w = fabs(det) * sK;
            for (int a = 0; a < 8; ++a)
            {
                /* B_a (6x3): rows xx, yy, zz, xy, yz, xz */
                const double B[6][3] = {{g[a][0], 0, 0}, {0, g[a][1], 0}, {0, 0, g[a][2]},
                                        {g[a][1], g[a][0], 0}, {0, g[a][2], g[a][1]}, {g[a][2], 0, g[a][0]}};
                double *blk = blocks + 9 * (uint64_t)conn8[8 * e + a];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                    {
                        double s = 0.0;
                        for (int r = 0; r < 6; ++r)
                        {
                            double db = 0.0;
                            for (int c = 0; c < 6; ++c)
                                db += D[6 * r + c] * B[c][j];
                            s += B[r][i] * db;
                        }
                        blk[3 * i + j] += s * w;
                    }
            }
        }
    }
    return 0;
}

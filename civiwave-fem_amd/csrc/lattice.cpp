// lattice.cpp -- structured-block specialisation of the FAST operator ("structured-block
// specialisation with a single shared K_e").
//
// The reference's operator is the element loop of pcg.cpp:561-662: per tet, f = vol s_K B^T D B u, scattered to
// its 4 corners. On a Kuhn block (every hex cell split into the 6 tets {0,1,3,7} {0,1,5,7} {0,2,3,7} {0,2,6,7}
// {0,4,5,7} {0,4,6,7} of its corner bits (i, j, k)) whose tets of one Kuhn type all carry the same gradients and
// volume, every cell contributes the same 24 x 24 cell stiffness Kc = sum of its 6 K_e (fp64, from the desc's own
// f32 gradients and volumes, the reference's B / D / vol products), and K u = sum over cells of Kc u_cell. Regrouped
// by node pair, an interior node's row is 15 3x3 blocks (the Kuhn edges: +-x, +-y, +-z, +-(1,1,0), +-(1,0,1),
// +-(0,1,1), +-(1,1,1), and the node itself):
//   (K u)_n = sum_d S_d u_(n+d),  S_d = sum over the cell corners c with c + d a corner of Kc[c][c + d].
// The kernel (lattice.inc) forms it in difference form, sum_(d != 0) S_d (u_(n+d) - u_n) (rigid translations
// are in the null space of every row), so each fp32 term is strain-sized as in the element loop. A node on the
// block's surface misses some of its 8 cells: its row is formed in the cell form instead, each existing cell's
// blocks Kc[c][c'] on the same differences. The regrouping changes the fp32 summation order only (FAST's
// tolerance contract, tests/test_lattice.py on the CPU, tests/test_gpu_lattice.py).
//
// detect_lattice() decides it for a desc: integer lattice coordinates of every node (from the first tet's cell
// size), a bijection onto an nx * ny * nz lattice, every tet one Kuhn tet of one cell (each of a cell's 6 types
// exactly once), one material, and every tet's gradients / volume within 1e-6 (relative) of the first tet of its
// Kuhn type. Storage order: lexicographic (i fastest) inside each k plane, planes anywhere (a shard's local order:
// owned planes, then its ghost planes; shard.cpp), or, when the handle may renumber, any order (perm).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "cwf_internal.hpp"

namespace cwf
{
namespace
{
constexpr int kKuhn[6][4] = {{0, 1, 3, 7}, {0, 1, 5, 7}, {0, 2, 3, 7}, {0, 2, 6, 7}, {0, 4, 5, 7}, {0, 4, 6, 7}};

// 6x3 strain-displacement block of one corner (the reference's B rows: xx, yy, zz, xy, yz, zx;
// pcg.cpp:622-630)
void b_block(const double g[3], double B[6][3])
{
    std::memset(B, 0, sizeof(double) * 18);
    B[0][0] = g[0];
    B[1][1] = g[1];
    B[2][2] = g[2];
    B[3][0] = g[1];
    B[3][1] = g[0];
    B[4][1] = g[2];
    B[4][2] = g[1];
    B[5][0] = g[2];
    B[5][2] = g[0];
}
}  // namespace

// kLatPair (cwf_internal.hpp) lists exactly the corner pairs that share a Kuhn tet, in (c, c') order, and
// kLatPairOff names each pair's offset c' - c
bool lattice_tables_ok()
{
    int q = 0;
    for (int c = 0; c < 8; ++c)
        for (int c2 = 0; c2 < 8; ++c2)
        {
            bool edge = c == c2;
            for (int t = 0; t < 6 && !edge; ++t)
            {
                bool a = false, b = false;
                for (int s = 0; s < 4; ++s)
                {
                    a |= kKuhn[t][s] == c;
                    b |= kKuhn[t][s] == c2;
                }
                edge = a && b;
            }
            if (!edge)
                continue;
            if (q >= kLatPairs || kLatPair[q][0] != c || kLatPair[q][1] != c2)
                return false;
            const int o = kLatPairOff[q];
            if (kLatOff[o][0] != (c2 & 1) - (c & 1) || kLatOff[o][1] != ((c2 >> 1) & 1) - ((c >> 1) & 1) ||
                kLatOff[o][2] != ((c2 >> 2) & 1) - ((c >> 2) & 1))
                return false;
            ++q;
        }
    return q == kLatPairs;
}

// storage order: lexicographic inside every k plane (the caller's order: plane[k] = its node (0, 0, k)), or, when
// the handle may renumber, the lexicographic order (perm = at)
bool storage_order(uint64_t N, const uint32_t nn[3], const std::vector<uint32_t> &at, bool allow_perm, Lattice &L)
{
    const uint64_t nx = nn[0], ny = nn[1], nz = nn[2];
    L.nx = (uint32_t)nx;
    L.ny = (uint32_t)ny;
    L.nz = (uint32_t)nz;
    L.plane.assign(nz, 0);
    L.perm.clear();
    bool caller_order = true;
    for (uint64_t k = 0; k < nz && caller_order; ++k)
    {
        const uint32_t base = at[k * nx * ny];
        L.plane[k] = base;
        if ((uint64_t)base + nx * ny > N)
            caller_order = false;
        for (uint64_t j = 0; j < ny && caller_order; ++j)
            for (uint64_t i = 0; i < nx; ++i)
                if (at[(k * ny + j) * nx + i] != base + j * nx + i)
                {
                    caller_order = false;
                    break;
                }
    }
    if (caller_order)
        return true;
    if (!allow_perm)
        return false;
    L.perm = at;
    for (uint64_t k = 0; k < nz; ++k)
        L.plane[k] = (uint32_t)(k * nx * ny);
    return true;
}

// stencil blocks S_d = sum over the corners c with c + d a corner of Kc[c][c + d], then the cell-pair blocks
template <int NOFF, int NPAIR>
void stencil_tables(const double Kc[8][8][3][3], const int (&off)[NOFF][3], const int (&pair)[NPAIR][2], Lattice &L)
{
    double S[NOFF][9] = {};
    double smax = 0.0;
    for (int o = 0; o < NOFF; ++o)
    {
        for (int c = 0; c < 8; ++c)
        {
            const int cx = (c & 1) + off[o][0], cy = ((c >> 1) & 1) + off[o][1], cz = ((c >> 2) & 1) + off[o][2];
            if (cx < 0 || cx > 1 || cy < 0 || cy > 1 || cz < 0 || cz > 1)
                continue;
            const int c2 = cx | cy << 1 | cz << 2;
            for (int r = 0; r < 3; ++r)
                for (int k = 0; k < 3; ++k)
                    S[o][3 * r + k] += Kc[c][c2][r][k];
        }
        for (double v : S[o])
            smax = std::max(smax, std::fabs(v));
    }
    // paired directions: S_(-d) = S_d^T always; S_d symmetric (S_(-d) = S_d) for an isotropic block. The two are
    // summed over the cells in different orders, so they agree to fp64 rounding: within 1e-10 of the largest
    // entry they are taken as equal and both set to their fp64 mean before the f32 rounding
    L.sym = true;
    for (int o = 1; o < NOFF; o += 2)
        for (int j = 0; j < 9; ++j)
            L.sym = L.sym && std::fabs(S[o][j] - S[o + 1][j]) <= 1e-10 * smax;
    if (L.sym)
        for (int o = 1; o < NOFF; o += 2)
            for (int j = 0; j < 9; ++j)
                S[o][j] = S[o + 1][j] = 0.5 * (S[o][j] + S[o + 1][j]);
    for (int o = 0; o < NOFF; ++o)
        for (int j = 0; j < 9; ++j)
            L.coef[9 * o + j] = (float)S[o][j];
    for (int p = 0; p < NPAIR; ++p)
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k)
                L.coef[9 * (NOFF + p) + 3 * r + k] = (float)Kc[pair[p][0]][pair[p][1]][r][k];
}

constexpr int kHexPair[kLatHexPairs][2] = {
#define P8(c) {c, 0}, {c, 1}, {c, 2}, {c, 3}, {c, 4}, {c, 5}, {c, 6}, {c, 7}
    P8(0), P8(1), P8(2), P8(3), P8(4), P8(5), P8(6), P8(7)
#undef P8
};

// native hex8 cells (Gmsh / VTK corner order; slot s sits at corner bits kHexSlotBits[s]): one hex per cell, the
// cell stiffness from the first hex's corner coordinates (the lattice's, to 1e-6 of the cell: every cell is a
// translate), 2 x 2 x 2 Gauss in fp64 (the textbook element of oracle/hex8_oracle.c and k_keff_hex_tiles)
bool detect_hex_cells(const cwf_system_desc *d, const std::vector<uint32_t> &q, const uint32_t nn[3],
                      const std::vector<uint32_t> &at, bool allow_perm, Lattice &L, std::string *why)
{
    const auto fail = [&](const char *m) {
        if (why)
            *why = m;
        return false;
    };
    constexpr int kHexSlotBits[8] = {0, 1, 3, 2, 4, 5, 7, 6};
    const uint64_t N = d->node_count, E = d->element_count, nx = nn[0], ny = nn[1], nz = nn[2];
    if (E != (nx - 1) * (ny - 1) * (nz - 1))
        return fail("element count is not one hex per cell");
    const uint32_t *conn = d->element_connectivity;
    std::vector<uint8_t> seen(E, 0);
    for (uint64_t e = 0; e < E; ++e)
    {
        const uint32_t *c = &q[3ull * conn[8 * e]];  // slot 0 is the cell's corner (0, 0, 0)
        if (c[0] >= nx - 1 || c[1] >= ny - 1 || c[2] >= nz - 1)
            return fail("a hex is not a cell");
        for (int s = 1; s < 8; ++s)
        {
            const uint32_t *qs = &q[3ull * conn[8 * e + s]];
            const uint32_t ox = qs[0] - c[0], oy = qs[1] - c[1], oz = qs[2] - c[2];
            if (ox > 1 || oy > 1 || oz > 1 || (int)(ox | oy << 1 | oz << 2) != kHexSlotBits[s])
                return fail("a hex is not a cell in Gmsh corner order");
        }
        const uint64_t cell = ((uint64_t)c[2] * (ny - 1) + c[1]) * (nx - 1) + c[0];
        if (seen[cell])
            return fail("two hexes on one cell");
        seen[cell] = 1;
    }
    if (!storage_order(N, nn, at, allow_perm, L))
        return fail("node order is not lexicographic within planes");
    double Xc[8][3];  // corner coordinates of the first hex by corner bits
    for (int s = 0; s < 8; ++s)
        for (int k = 0; k < 3; ++k)
            Xc[kHexSlotBits[s]][k] = d->node_coords[3ull * conn[s] + k];
    const double *D = d->material_stiffness + 36ull * d->element_material_index[0];
    double Kc[8][8][3][3];
    std::memset(Kc, 0, sizeof Kc);
    const double gq = 1.0 / std::sqrt(3.0);
    for (int gp = 0; gp < 8; ++gp)
    {
        const double qp[3] = {(gp & 1) ? gq : -gq, (gp & 2) ? gq : -gq, (gp & 4) ? gq : -gq};
        double dN[8][3], J[3][3] = {};
        for (int a = 0; a < 8; ++a)
        {
            const double sg[3] = {(a & 1) ? 1.0 : -1.0, (a & 2) ? 1.0 : -1.0, (a & 4) ? 1.0 : -1.0};
            const double f[3] = {1.0 + sg[0] * qp[0], 1.0 + sg[1] * qp[1], 1.0 + sg[2] * qp[2]};
            dN[a][0] = 0.125 * sg[0] * f[1] * f[2];
            dN[a][1] = 0.125 * f[0] * sg[1] * f[2];
            dN[a][2] = 0.125 * f[0] * f[1] * sg[2];
            for (int m = 0; m < 3; ++m)
                for (int l = 0; l < 3; ++l)
                    J[m][l] += Xc[a][m] * dN[a][l];
        }
        double A[3][3];  // adjugate
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
        if (!(std::fabs(det) > 0.0))
            return fail("degenerate hex");
        double g[8][3];
        for (int a = 0; a < 8; ++a)
            for (int m = 0; m < 3; ++m)
            {
                double sum = 0.0;
                for (int l = 0; l < 3; ++l)
                    sum += dN[a][l] * A[l][m];
                g[a][m] = sum / det;
            }
        for (int a = 0; a < 8; ++a)
            for (int b = 0; b < 8; ++b)
            {
                double Ba[6][3], Bb[6][3];
                b_block(g[a], Ba);
                b_block(g[b], Bb);
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k)
                    {
                        double sum = 0.0;
                        for (int i = 0; i < 6; ++i)
                            for (int j = 0; j < 6; ++j)
                                sum += Ba[i][r] * D[6 * i + j] * Bb[j][k];
                        Kc[a][b][r][k] += std::fabs(det) * sum;
                    }
            }
    }
    stencil_tables(Kc, kLatHexOff, kHexPair, L);
    L.hex = true;
    return true;
}

bool detect_lattice(const cwf_system_desc *d, bool allow_perm, Lattice &L, std::string *why)
{
    const auto fail = [&](const char *m) {
        if (why)
            *why = m;
        return false;
    };
    const uint64_t N = d->node_count, E = d->element_count;
    static const bool tables_ok = lattice_tables_ok();
    if (!tables_ok)
        return fail("lattice tables inconsistent");
    if (!E || N < 8 || !d->node_coords)
        return fail("no elements or no node coordinates");
    const bool hex = d->element_connectivity[4] != 0xFFFFFFFFu;
    const int K = hex ? 8 : 4;
    const uint32_t *conn = d->element_connectivity;
    const double *X = d->node_coords;
    const uint32_t m0 = d->element_material_index[0];
    for (uint64_t e = 0; e < E; ++e)
        if (d->element_material_index[e] != m0)
            return fail("more than one material");
    // cell size from the first element (a Kuhn tet spans its whole cell: it holds corners 0 and 7)
    double h[3], lo[3];
    for (int k = 0; k < 3; ++k)
    {
        double a = X[3ull * conn[0] + k], b = a;
        for (int s = 1; s < K; ++s)
        {
            a = std::min(a, X[3ull * conn[s] + k]);
            b = std::max(b, X[3ull * conn[s] + k]);
        }
        h[k] = b - a;
        if (!(h[k] > 0.0))
            return fail("degenerate first element");
        lo[k] = X[k];
    }
    for (uint64_t n = 1; n < N; ++n)
        for (int k = 0; k < 3; ++k)
            lo[k] = std::min(lo[k], X[3 * n + k]);
    std::vector<uint32_t> q(3 * N);
    uint32_t nn[3] = {0, 0, 0};
    for (uint64_t n = 0; n < N; ++n)
        for (int k = 0; k < 3; ++k)
        {
            // tets: the element records define the operator (checked below), so coordinates only place the nodes;
            // hex8: the operator is formed from the coordinates, so they must be the lattice's
            const double f = (X[3 * n + k] - lo[k]) / h[k];
            const double r = std::nearbyint(f);
            if (!(std::fabs(f - r) <= (hex ? 1e-6 : 1e-3)) || r >= 1048576.0)
                return fail("nodes off the lattice");
            q[3 * n + k] = (uint32_t)r;
            nn[k] = std::max(nn[k], (uint32_t)r + 1u);
        }
    if (nn[0] < 2 || nn[1] < 2 || nn[2] < 2 || (uint64_t)nn[0] * nn[1] * nn[2] != N)
        return fail("nodes do not fill a box lattice");
    const uint64_t nx = nn[0], ny = nn[1], nz = nn[2];
    std::vector<uint32_t> at(N, 0xFFFFFFFFu);  // lexicographic lattice index -> node
    for (uint64_t n = 0; n < N; ++n)
    {
        const uint64_t li = ((uint64_t)q[3 * n + 2] * ny + q[3 * n + 1]) * nx + q[3 * n];
        if (at[li] != 0xFFFFFFFFu)
            return fail("two nodes on one lattice point");
        at[li] = (uint32_t)n;
    }
    const uint64_t C = (nx - 1) * (ny - 1) * (nz - 1);
    if (hex)
        return detect_hex_cells(d, q, nn, at, allow_perm, L, why);
    if (E != 6 * C)
        return fail("element count is not 6 per cell");
    // every tet a Kuhn tet of one cell, each of a cell's 6 types once; gradients / volume per type
    int type_of[256];
    std::fill(type_of, type_of + 256, -1);
    for (int t = 0; t < 6; ++t)
    {
        int m = 0;
        for (int s = 0; s < 4; ++s)
            m |= 1 << kKuhn[t][s];
        type_of[m] = t;
    }
    std::vector<uint8_t> seen(C, 0);
    double G[6][8][3];
    double V[6], gmax[6];
    bool have[6] = {false, false, false, false, false, false};
    const float *grad = d->element_gradients;
    for (uint64_t e = 0; e < E; ++e)
    {
        uint32_t c[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        for (int s = 0; s < 4; ++s)
            for (int k = 0; k < 3; ++k)
                c[k] = std::min(c[k], q[3ull * conn[8 * e + s] + k]);
        int bits[4], m = 0;
        for (int s = 0; s < 4; ++s)
        {
            const uint32_t *qs = &q[3ull * conn[8 * e + s]];
            const uint32_t ox = qs[0] - c[0], oy = qs[1] - c[1], oz = qs[2] - c[2];
            if (ox > 1 || oy > 1 || oz > 1)
                return fail("an element spans more than one cell");
            bits[s] = (int)(ox | oy << 1 | oz << 2);
            m |= 1 << bits[s];
        }
        const int t = type_of[m];
        if (t < 0 || c[0] >= nx - 1 || c[1] >= ny - 1 || c[2] >= nz - 1)
            return fail("an element is not a Kuhn tet of a cell");
        const uint64_t cell = ((uint64_t)c[2] * (ny - 1) + c[1]) * (nx - 1) + c[0];
        if (seen[cell] & (1u << t))
            return fail("a cell holds one Kuhn type twice");
        seen[cell] |= (uint8_t)(1u << t);
        const float *g = grad + 24 * e;
        const double vol = d->element_volume[e];
        if (!have[t])
        {
            have[t] = true;
            V[t] = vol;
            gmax[t] = 0.0;
            for (int s = 0; s < 4; ++s)
                for (int k = 0; k < 3; ++k)
                {
                    G[t][bits[s]][k] = g[3 * s + k];
                    gmax[t] = std::max(gmax[t], std::fabs((double)g[3 * s + k]));
                }
            if (!(V[t] > 0.0) || !(gmax[t] > 0.0))
                return fail("degenerate element");
            continue;
        }
        if (!(std::fabs(vol - V[t]) <= 1e-6 * V[t]))
            return fail("element volumes differ within a Kuhn type");
        for (int s = 0; s < 4; ++s)
            for (int k = 0; k < 3; ++k)
                if (!(std::fabs((double)g[3 * s + k] - G[t][bits[s]][k]) <= 1e-6 * gmax[t]))
                    return fail("element gradients differ within a Kuhn type");
    }
    if (!storage_order(N, nn, at, allow_perm, L))
        return fail("node order is not lexicographic within planes");
    L.hex = false;
    // cell stiffness Kc[c][c'] = sum over the cell's tets of vol B_c^T D B_c' (fp64, pcg.cpp:622-651 products)
    const double *D = d->material_stiffness + 36ull * m0;
    double Kc[8][8][3][3];
    std::memset(Kc, 0, sizeof Kc);
    for (int t = 0; t < 6; ++t)
        for (int sa = 0; sa < 4; ++sa)
            for (int sb = 0; sb < 4; ++sb)
            {
                const int a = kKuhn[t][sa], b = kKuhn[t][sb];
                double Ba[6][3], Bb[6][3];
                b_block(G[t][a], Ba);
                b_block(G[t][b], Bb);
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k)
                    {
                        double sum = 0.0;
                        for (int i = 0; i < 6; ++i)
                            for (int j = 0; j < 6; ++j)
                                sum += Ba[i][r] * D[6 * i + j] * Bb[j][k];
                        Kc[a][b][r][k] += V[t] * sum;
                    }
            }
    // every block outside the Kuhn pattern is structurally zero (never accumulated): nothing to check
    stencil_tables(Kc, kLatOff, kLatPair, L);
    return true;
}

// Work items: the surface shell of the computed planes [lk0, lk1), one node per thread (256-thread workgroups,
// rounded up to whole XCD groups so the bricks after them keep the XCD mapping), then 32 x 8 column bricks of the
// strict interior times L planes. L = 6 while the brick columns are fewer than one round of resident workgroups
// (1024: four per CU), else one column's planes per brick (about kLatTargetItems bricks). Measured (PCG it/s, same
// box, two passes, k_keff_lattice with the uniform mass): C2 (27 columns) L = 3 / 4 / 5 / 6 / 7 / 8: 40.2k / 40.1k
// / 41.6k / 41.6k / 39.3k / 39.5k; C3 (95 columns) L = 5 / 6 / 7 / 8 / 9 / 11 / 14 / 20 / 28: 58.8-60.9 / 54.3-57.9
// / 56.4-61.0 / 54.0-58.0 / 55.1-55.9 / 56.0-59.8 / 55.4-59.9 / 60.1-62.4 / 67.0-69.0 us; C3 hex8 L = 6 / 12 /
// 14 / 24: 65.4 / 66.6 / 68.0 / 75.4 us; C5 (1250 columns) L = 6 / 12 / 24 / 48 (all): 252 / 242 / 267 / 224 us
void lattice_plan(DevTiles &t)
{
    constexpr uint64_t kLatTargetItems = 262144 / kLatThreads;  // 1024 bricks of 256 threads
    const uint64_t nx = t.lnx, ny = t.lny, nz = t.lnz;
    const uint64_t k0 = t.lk0, k1 = std::max(t.lk1, t.lk0);
    t.lkI0 = (uint32_t)std::max<uint64_t>(k0, 1);
    t.lkI1 = (uint32_t)std::max<uint64_t>(std::min<uint64_t>(k1, nz - 1), t.lkI0);
    uint64_t shell = 0;
    if (k0 == 0 && k1 > 0)
        shell += nx * ny;
    if (k1 == nz && nz > 1 && k1 > k0)
        shell += nx * ny;
    shell += (uint64_t)(t.lkI1 - t.lkI0) * (2 * nx + 2 * (ny - 2));
    t.lnshell = (uint32_t)shell;
    t.lnsb = (uint32_t)(((shell + kLatThreads - 1) / kLatThreads + 7) / 8 * 8);
    t.lnbx = (uint32_t)((nx - 2 + kLatBrickX - 1) / kLatBrickX);
    t.lnby = (uint32_t)((ny - 2 + kLatBrickY - 1) / kLatBrickY);
    const uint64_t planes = t.lkI1 - t.lkI0, cols = (uint64_t)t.lnbx * t.lnby;
    uint64_t L = cols < kLatTargetItems ? 6 : (planes * cols + kLatTargetItems - 1) / kLatTargetItems;
    const char *lk = knob("CWF_LAT_L");
    if (lk && atoi(lk) > 0)
        L = (uint64_t)atoi(lk);
    L = std::max<uint64_t>(lk && atoi(lk) > 0 ? 2 : 4, std::min<uint64_t>(L, 64));
    t.lL = (uint32_t)L;
    t.lnwm = (uint32_t)(cols * ((planes + L - 1) / L));
    t.lnwork = t.lnsb + t.lnwm;
    // the shell workgroups lead the bricks when the grid takes several rounds of resident workgroups (C3: 2.8
    // rounds, shell last -2.6%) and follow them when it fits in one (C2: 436 workgroups, shell last +6.2%, keff 14.2
    // -> 12.9 us; same box, two passes)
    // several rounds of many k-chunks: each chunk's perimeter workgroups right after its bricks (C3 +0.5-1.4%, C3
    // hex8 +1.5% over the shell first, same box: the perimeter gathers find the chunk's lines in the XCD's L2;
    // profiles/r04w_*). Not with few chunks: each XCD takes a contiguous share of the items, so C5's one chunk put
    // its 1,250 whole-column bricks on three XCDs and the end planes on the rest (K_eff 241 -> 476 us, r04z)
    const uint64_t nchunks = (planes + L - 1) / L;
    t.lshl = t.lnwork <= kLatTargetItems ? 1 : nchunks >= 16 ? 2 : 0;
    t.lnsc = 0;
    if (t.lshl == 2)  // interleaved: per k-chunk its bricks, then the perimeters of its planes; the end planes last
    {
        const uint64_t per = 2 * nx + 2 * (ny - 2), nchunk = (planes + L - 1) / L;
        const uint64_t nlo = (k0 == 0 && k1 > 0) ? nx * ny : 0, nhi = (k1 == nz && nz > 1 && k1 > k0) ? nx * ny : 0;
        t.lnsc = (uint32_t)((L * per + kLatThreads - 1) / kLatThreads);
        t.lnwork = (uint32_t)(nchunk * (cols + t.lnsc) + (nlo + kLatThreads - 1) / kLatThreads +
                              (nhi + kLatThreads - 1) / kLatThreads);
    }
    t.ntiles = t.lnwork;
}

}  // namespace cwf

extern "C" int cwf_lattice_describe(const cwf_system_desc *desc, int renumber, uint32_t dims[3], float *coef,
                                    uint32_t *plane)
{
    static_assert(cwf::kLatCoef == CWF_LATTICE_COEFS, "cwf_hip.h CWF_LATTICE_COEFS");
    if (!desc || !dims || !coef || !desc->element_connectivity || !desc->element_gradients || !desc->element_volume ||
        !desc->element_material_index || !desc->material_stiffness)
        return CWF_ERR_ARGUMENT;
    // tet4 blocks (the reference's element; native hex8 blocks run the 27-point instantiation and are not described)
    if (desc->mode != CWF_MODE_FAST || desc->node_count >= 0x15555555ull || !desc->element_count ||
        desc->element_connectivity[4] != 0xFFFFFFFFu)
        return 0;
    for (uint64_t e = 0; e < desc->element_count; ++e)
    {
        if (desc->element_material_index[e] >= desc->material_count)
            return CWF_ERR_MATERIAL_RANGE;
        for (int a = 0; a < 4; ++a)
            if (desc->element_connectivity[8 * e + a] >= desc->node_count)
                return CWF_ERR_NODE_RANGE;
    }
    cwf::Lattice L;
    if (!cwf::detect_lattice(desc, renumber != 0, L))
        return 0;
    dims[0] = L.nx;
    dims[1] = L.ny;
    dims[2] = L.nz;
    std::memcpy(coef, L.coef, sizeof(float) * cwf::kLatCoef);
    dims[0] |= L.sym ? 0x80000000u : 0u;
    if (plane)
        std::memcpy(plane, L.plane.data(), L.plane.size() * sizeof(uint32_t));
    return 1;
}

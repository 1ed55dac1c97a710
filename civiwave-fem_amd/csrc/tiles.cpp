// tiles.cpp -- host-side build of the FAST-mode element tiles.
//
// The fast K_eff is element-centric: one workgroup per tile of <= kTileElems consecutive
// elements. With node coordinates, tet tiles are the leaves of a recursive coordinate bisection of
// the element centroids (cuts at the widest centroid gap near the balanced count, so they run between
// element layers), each leaf in Morton order inside; hex tiles are segments of the Morton curve. Per
// tile the host precomputes
//   * the tile's distinct nodes (sorted global ids) -> the workgroup gathers their p into LDS,
//   * every element's 4 corners as u16 indices into that node list,
//   * a local CSR  tile-node -> (element_local * 4 + corner), ascending element, so the LDS fold of
//     the element forces into tile-node partial sums is deterministic (no atomics),
//   * the node -> (tile, slot) list, ascending tile, used by the finalize pass that adds a node's
//     2..8 tile partials in a fixed order.
// Element records are stored as 4 SoA planes of uint4 so every dwordx4 load of a wave is one
// contiguous 1 KiB run:  plane0 = {idx01, idx23, vol_bits, material}, planes1..3 = the 12 gradients.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "cwf_internal.hpp"

namespace cwf
{
uint64_t spread21(uint64_t v)
{
    v &= 0x1fffff;
    v = (v | v << 32) & 0x1f00000000ffffull;
    v = (v | v << 16) & 0x1f0000ff0000ffull;
    v = (v | v << 8) & 0x100f00f00f00f00full;
    v = (v | v << 4) & 0x10c30c30c30c30c3ull;
    v = (v | v << 2) & 0x1249249249249249ull;
    return v;
}

namespace
{

// Recursive coordinate bisection of the elements into leaves of at most max_elems (target max_elems
// (1 - 1/tdiv), tdiv = 0: max_elems). Each range is cut along the longest axis of its centroid box near the
// count n * L1 / L (L leaves, L1 = L / 2), at the widest gap between consecutive centroid coordinates within
// +-n/wdiv of that count.
// A cut through such a gap runs between element layers instead of through them, so the two sides share
// one node layer rather than the nodes of a whole sliced layer: for a Kuhn block the tile halo (T / N)
// drops from ~2.5 (Morton-curve segments) to ~1.8. The leaves come out in k-d-tree order, so consecutive
// tiles are neighbours. c: centroids [3E]; lo/hi: per-element min/max node coordinate [3E] (extent);
// leaf_end receives each leaf's end in `order`.
void rcb(const std::vector<double> &c, const double ext[3], std::vector<uint32_t> &order, uint64_t b, uint64_t e,
         uint64_t max_elems, std::vector<uint64_t> &leaf_end, int tdiv = 16, int wdiv = 16)
{
    const uint64_t n = e - b;
    if (n <= max_elems)
    {
        if (n)
            leaf_end.push_back(e);
        return;
    }
    const uint64_t target = std::max<uint64_t>(1, tdiv > 0 ? max_elems - max_elems / (uint64_t)tdiv : max_elems);
    const uint64_t Lr = std::max<uint64_t>((n + target - 1) / target, 2);
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (uint64_t i = b; i < e; ++i)
        for (int k = 0; k < 3; ++k)
        {
            lo[k] = std::min(lo[k], c[3ull * order[i] + k]);
            hi[k] = std::max(hi[k], c[3ull * order[i] + k]);
        }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (hi[k] - lo[k] > hi[ax] - lo[ax])
            ax = k;
    const auto less = [&](uint32_t x, uint32_t y) {
        const double cx = c[3ull * x + ax], cy = c[3ull * y + ax];
        return cx < cy || (cx == cy && x < y);  // ties by element id: deterministic
    };
    const uint64_t L1 = Lr / 2;
    const uint64_t m = b + (n * L1 + Lr / 2) / Lr;
    const uint64_t w = n / (uint64_t)(wdiv > 0 ? wdiv : 16);
    uint64_t cut = m;
    std::nth_element(order.begin() + b, order.begin() + m, order.begin() + e, less);
    if (w >= 2)
    {
        // candidates: the elements whose centroid lies within 1.5 mean element extents of the median's,
        // sorted; everything before that band is <, after it > (two partitions, O(n))
        const double vm = c[3ull * order[m] + ax], dl = 1.5 * ext[ax];
        const auto mid = std::partition(order.begin() + b, order.begin() + e,
                                        [&](uint32_t x) { return c[3ull * x + ax] < vm - dl; });
        const auto top = std::partition(mid, order.begin() + e, [&](uint32_t x) { return c[3ull * x + ax] <= vm + dl; });
        std::sort(mid, top, less);
        const uint64_t wb = std::max<uint64_t>((uint64_t)(mid - order.begin()), m - w);
        const uint64_t we = std::min<uint64_t>((uint64_t)(top - order.begin()), m + w + 1);
        double best = -1.0;
        cut = std::min(std::max(m, wb), we > wb ? we - 1 : wb);
        for (uint64_t i = wb + 1; i < we; ++i)
        {
            const double gap = c[3ull * order[i] + ax] - c[3ull * order[i - 1] + ax];
            const uint64_t dist = i > m ? i - m : m - i, bdist = cut > m ? cut - m : m - cut;
            if (gap > best * (1.0 + 1e-9) || (gap >= best * (1.0 - 1e-9) && dist < bdist))
            {
                best = gap;
                cut = i;
            }
        }
    }
    cut = std::min(std::max(cut, b + 1), e - 1);  // both sides non-empty (n > max_elems >= 1)
    rcb(c, ext, order, b, cut, max_elems, leaf_end, tdiv, wdiv);
    rcb(c, ext, order, cut, e, max_elems, leaf_end, tdiv, wdiv);
}
}  // namespace

void rcb_partition(const std::vector<double> &c, const double ext[3], std::vector<uint32_t> &order,
                   uint64_t max_elems, std::vector<uint64_t> &leaf_end, int tdiv, int wdiv)
{
    rcb(c, ext, order, 0, order.size(), max_elems, leaf_end, tdiv, wdiv);
}

int build_tiles(const cwf_system_desc *d, HostTiles &out, uint32_t max_nodes, uint32_t max_elems, int corners)
{
    const uint64_t N = d->node_count, E = d->element_count;
    const int K = corners == 8 ? 8 : 4;  // tet4 or hex8 (slots 0..K-1 of the 8-slot connectivity)
    std::vector<uint32_t> order(E);
    std::iota(order.begin(), order.end(), 0u);
    std::vector<uint64_t> leaf_end;  // RCB leaf boundaries in `order` (empty: one run, greedy cuts only)
    if (d->node_coords && E)
    {
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (uint64_t n = 0; n < N; ++n)
            for (int k = 0; k < 3; ++k)
            {
                lo[k] = std::min(lo[k], d->node_coords[3 * n + k]);
                hi[k] = std::max(hi[k], d->node_coords[3 * n + k]);
            }
        double ext = 0.0;
        for (int k = 0; k < 3; ++k)
            ext = std::max(ext, hi[k] - lo[k]);
        const double scale = ext > 0 ? (double)((1u << 21) - 1) / ext : 0.0;
        std::vector<uint64_t> key(E);
        for (uint64_t e = 0; e < E; ++e)
        {
            double c[3] = {0, 0, 0};
            for (int a = 0; a < K; ++a)
                for (int k = 0; k < 3; ++k)
                    c[k] += d->node_coords[3 * (uint64_t)d->element_connectivity[e * 8 + a] + k];
            uint64_t q[3];
            for (int k = 0; k < 3; ++k)
                q[k] = (uint64_t)std::llround((c[k] / K - lo[k]) * scale);
            key[e] = spread21(q[0]) | spread21(q[1]) << 1 | spread21(q[2]) << 2;
        }
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
        static const int tile_order = [] {  // CWF_TILE_ORDER=morton|rcb (diagnostic; default by element)
            const char *v = knob("CWF_TILE_ORDER");
            return !v ? -1 : std::string(v) == "morton" ? 0 : 1;
        }();
        // tets: RCB leaves (C3 tiles kernel 223 -> 200 us, same-box A/B); hex8: Morton segments, whose
        // 128-hex tiles are already compact octant blocks (RCB measured 4% slower there)
        if (tile_order == 1 || (tile_order == -1 && K == 4))
        {
            // tiles = RCB leaves (each kept in Morton order inside); the greedy pass below still splits
            // a leaf whose node list exceeds max_nodes
            std::vector<double> cen(3 * E);
            double ext[3] = {0.0, 0.0, 0.0};  // mean element extent per axis
            for (uint64_t e = 0; e < E; ++e)
                for (int k = 0; k < 3; ++k)
                {
                    double v = 0.0, mn = 1e300, mx = -1e300;
                    for (int a = 0; a < K; ++a)
                    {
                        const double x = d->node_coords[3 * (uint64_t)d->element_connectivity[e * 8 + a] + k];
                        v += x;
                        mn = std::min(mn, x);
                        mx = std::max(mx, x);
                    }
                    cen[3 * e + k] = v / K;
                    ext[k] += mx - mn;
                }
            for (int k = 0; k < 3; ++k)
                ext[k] /= (double)E;
            rcb(cen, ext, order, 0, E, max_elems, leaf_end);
            uint64_t b = 0;
            for (const uint64_t le : leaf_end)
            {
                std::stable_sort(order.begin() + b, order.begin() + le,
                                 [&](uint32_t x, uint32_t y) { return key[x] < key[y]; });
                b = le;
            }
        }
    }

    out = HostTiles{};
    out.tile_elem_off.push_back(0);
    out.tile_node_off.push_back(0);
    out.csr_off.push_back(0);
    if (K == 4)
    {
        for (int q = 0; q < 3; ++q)
            out.planes[q].resize(E);
        out.eid.resize(E);
        out.epos.resize(E);
    }
    else
    {
        out.eid8.resize(E);
        out.epos8.resize(E);
    }
    if (d->material_count > 1)
        out.mat.resize(E);
    out.csr_ent.reserve(E * K);
    std::vector<uint32_t> stamp(N, 0xFFFFFFFFu), local(N, 0);
    std::vector<uint32_t> nodes;
    std::vector<uint32_t> cnt;
    uint64_t e = 0;
    uint32_t tile = 0;
    size_t leaf = 0;
    while (e < E)
    {
        // greedy: up to kTileElems elements of the current RCB leaf while the tile's node list fits
        // kMaxTileNodes
        nodes.clear();
        const uint64_t e0 = e;
        while (leaf < leaf_end.size() && leaf_end[leaf] <= e0)
            ++leaf;
        const uint64_t stop = leaf < leaf_end.size() ? leaf_end[leaf] : E;
        while (e < stop && e - e0 < (uint64_t)max_elems)
        {
            const uint32_t src = order[e];
            uint32_t add = 0;
            for (int a = 0; a < K; ++a)
                add += stamp[d->element_connectivity[(uint64_t)src * 8 + a]] != tile ? 1u : 0u;
            if (nodes.size() + add > (size_t)max_nodes)
                break;
            for (int a = 0; a < K; ++a)
            {
                const uint32_t g = d->element_connectivity[(uint64_t)src * 8 + a];
                if (stamp[g] != tile)
                {
                    stamp[g] = tile;
                    nodes.push_back(g);
                }
            }
            ++e;
        }
        std::sort(nodes.begin(), nodes.end());
        for (uint32_t i = 0; i < nodes.size(); ++i)
            local[nodes[i]] = i;
        const uint32_t ne = (uint32_t)(e - e0), nn = (uint32_t)nodes.size();
        // element records + local CSR
        cnt.assign(nn + 1, 0);
        for (uint32_t j = 0; j < ne; ++j)
        {
            const uint32_t src = order[e0 + j];
            uint32_t li[8];
            for (int a = 0; a < K; ++a)
            {
                li[a] = local[d->element_connectivity[(uint64_t)src * 8 + a]];
                ++cnt[li[a] + 1];
            }
            if (!out.mat.empty())
                out.mat[e0 + j] = d->element_material_index[src];
            if (K == 8)
            {
                out.eid8[e0 + j] = uint4{li[0] | (li[1] << 16), li[2] | (li[3] << 16), li[4] | (li[5] << 16),
                                         li[6] | (li[7] << 16)};
                continue;
            }
            const float *g = d->element_gradients + (uint64_t)src * 24;
            uint4 q0, q1, q2;
            q0.x = li[0] | (li[1] << 16);
            q0.y = li[2] | (li[3] << 16);
            std::memcpy(&q0.z, g + 0, 8);   // g0x g0y
            std::memcpy(&q1, g + 2, 16);    // g0z g1x g1y g1z
            std::memcpy(&q2, g + 6, 12);    // g2x g2y g2z
            std::memcpy(&q2.w, &d->element_volume[src], 4);
            out.eid[e0 + j] = uint2{q0.x, q0.y};
            out.planes[0][e0 + j] = q0;
            out.planes[1][e0 + j] = q1;
            out.planes[2][e0 + j] = q2;
        }
        for (uint32_t i = 0; i < nn; ++i)
            cnt[i + 1] += cnt[i];
        const uint64_t base = out.csr_ent.size();
        out.csr_ent.resize(base + (uint64_t)K * ne);
        std::vector<uint32_t> cur(cnt.begin(), cnt.end() - 1);
        for (uint32_t j = 0; j < ne; ++j)
        {
            const uint32_t src = order[e0 + j];
            uint32_t epos[8];
            for (int a = 0; a < K; ++a)
            {
                const uint32_t l = local[d->element_connectivity[(uint64_t)src * 8 + a]];
                epos[a] = cur[l];  // the corner's tile-relative local-CSR position (PUSH)
                out.csr_ent[base + cur[l]++] = (uint16_t)(j * K + a);
            }
            if (K == 8)
                out.epos8[e0 + j] = uint4{epos[0] | (epos[1] << 16), epos[2] | (epos[3] << 16),
                                          epos[4] | (epos[5] << 16), epos[6] | (epos[7] << 16)};
            else
                out.epos[e0 + j] = uint2{epos[0] | (epos[1] << 16), epos[2] | (epos[3] << 16)};
        }
        for (uint32_t i = 0; i < nn; ++i)
        {
            out.tile_nodes.push_back(nodes[i]);
            out.csr_off.push_back((uint32_t)(base + cnt[i + 1]));
        }
        if (d->node_coords && nn)
        {
            // tile-relative f32 coordinates (origin = the tile's first node) keep the edge vectors exact
            const double *o = d->node_coords + 3ull * nodes[0];
            for (uint32_t i = 0; i < nn; ++i)
                for (int k = 0; k < 3; ++k)
                    out.tcoord[k].push_back((float)(d->node_coords[3ull * nodes[i] + k] - o[k]));
        }
        if (K == 8)
        {
            // parallelepiped test: the trilinear map's bilinear/trilinear ("hourglass") coefficients
            // x_0 - x_1 + x_2 - x_3 (bottom face), ..., all ~0 -> J is constant over the hex. Tolerance
            // 1e-7 of the element's extent: below fp32 rounding of the kernel's own J.
            bool aff = d->node_coords != nullptr;
            for (uint64_t j = e0; aff && j < e; ++j)
            {
                const uint32_t *c = d->element_connectivity + 8ull * order[j];
                for (int m = 0; m < 3 && aff; ++m)
                {
                    double v[8];  // lexicographic corner L = i + 2 j + 4 k (Gmsh order 0 1 3 2 4 5 7 6)
                    const int lex[8] = {0, 1, 3, 2, 4, 5, 7, 6};
                    for (int a = 0; a < 8; ++a)
                        v[lex[a]] = d->node_coords[3ull * c[a] + m];
                    const double hxy0 = v[0] - v[1] - v[2] + v[3], hxy1 = v[4] - v[5] - v[6] + v[7];
                    const double hxz = v[0] - v[1] - v[4] + v[5], hyz = v[0] - v[2] - v[4] + v[6];
                    const double ext = std::fabs(v[1] - v[0]) + std::fabs(v[2] - v[0]) + std::fabs(v[4] - v[0]);
                    const double tol = 1e-7 * ext;
                    aff = std::fabs(hxy0) <= tol && std::fabs(hxy1) <= tol && std::fabs(hxz) <= tol &&
                          std::fabs(hyz) <= tol;
                }
            }
            out.tile_affine.push_back(aff ? 1 : 0);
        }
        out.max_tile_nodes = std::max(out.max_tile_nodes, nn);
        out.tile_elem_off.push_back((uint32_t)e);
        out.tile_node_off.push_back((uint32_t)out.tile_nodes.size());
        ++tile;
    }
    out.ntiles = tile;
    // node -> slots (ascending tile)
    const uint64_t total = out.tile_nodes.size();
    out.node_part_off.assign(N + 1, 0);
    for (uint64_t s = 0; s < total; ++s)
        ++out.node_part_off[out.tile_nodes[s] + 1];
    for (uint64_t n = 0; n < N; ++n)
        out.node_part_off[n + 1] += out.node_part_off[n];
    out.node_part_slot.resize(total);
    std::vector<uint32_t> cur(out.node_part_off.begin(), out.node_part_off.end() - 1);
    for (uint64_t s = 0; s < total; ++s)
        out.node_part_slot[cur[out.tile_nodes[s]]++] = (uint32_t)s;
    // node-major partial position of every tile node: the update pass then streams a node's
    // partials contiguously (part[node_part_off[n] .. node_part_off[n+1]), ascending tile)
    out.tile_slot.resize(total);
    for (uint64_t q = 0; q < total; ++q)
        out.tile_slot[out.node_part_slot[q]] = (uint32_t)q;
    // owner slot = the node's first (lowest-tile) slot: bit 31 of tile_nodes
    for (uint64_t n = 0; n < N; ++n)
        if (out.node_part_off[n + 1] > out.node_part_off[n])
            out.tile_nodes[out.node_part_slot[out.node_part_off[n]]] |= 0x80000000u;
    return 0;
}

bool geometry_matches(const cwf_system_desc *d)
{
    if (!d->node_coords)
        return false;
    const double *X = d->node_coords;
    for (uint64_t e = 0; e < d->element_count; ++e)
    {
        const uint32_t *c = d->element_connectivity + 8 * e;
        double ed[3][3];
        for (int k = 0; k < 3; ++k)
            for (int q = 0; q < 3; ++q)
                ed[k][q] = X[3ull * c[k + 1] + q] - X[3ull * c[0] + q];
        double r[3][3];
        for (int k = 0; k < 3; ++k)
        {
            const double *u = ed[(k + 1) % 3], *v = ed[(k + 2) % 3];
            r[k][0] = u[1] * v[2] - u[2] * v[1];
            r[k][1] = u[2] * v[0] - u[0] * v[2];
            r[k][2] = u[0] * v[1] - u[1] * v[0];
        }
        const double det = ed[0][0] * r[0][0] + ed[0][1] * r[0][1] + ed[0][2] * r[0][2];
        if (!(std::fabs(det) > 0.0))
            return false;
        double g[4][3];
        for (int k = 0; k < 3; ++k)
            for (int q = 0; q < 3; ++q)
                g[k + 1][q] = r[k][q] / det;
        for (int q = 0; q < 3; ++q)
            g[0][q] = -(g[1][q] + g[2][q] + g[3][q]);
        double gmax = 0.0;
        for (int a = 0; a < 4; ++a)
            for (int q = 0; q < 3; ++q)
                gmax = std::max(gmax, std::fabs(g[a][q]));
        const float *G = d->element_gradients + 24 * e;
        for (int a = 0; a < 4; ++a)
            for (int q = 0; q < 3; ++q)
                if (std::fabs((double)G[3 * a + q] - g[a][q]) > 1e-5 * gmax)
                    return false;
        const double vol = std::fabs(det) / 6.0;
        if (std::fabs((double)d->element_volume[e] - vol) > 1e-5 * vol)
            return false;
    }
    return true;
}

}  // namespace cwf

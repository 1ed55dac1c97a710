// groups.cpp -- host build of the FAST-mode tet fan groups and their tiles (GroupTiles, cwf_internal.hpp).
//
// The reference's operator is a loop over tets that scatters 12 forces per tet (pcg.cpp:561-662). The
// tiles kernel of round 1 pushes those 12 forces through LDS one (tet, corner) at a time and reads every
// corner's coordinates and value from LDS, so LDS traffic, not HBM, bounds it on small meshes. A fan group
// gathers the tets around one edge (a, b): tet i = {a, b, r_i, r_{(i+1) mod 6}}, i < f <= 6, so a lane
// holds the group's <= 8 nodes in registers, computes its f tets with static register indices, sums the
// forces per node and pushes one force per node. A Kuhn-split hex is one closed 6-tet fan around its
// diagonal (8 nodes for 24 corners); an unstructured mesh forms fans around its edges (~5 tets each).
// The element math per tet is unchanged (fp32, corner order free: the gradients and |det| are intrinsic).
//
// Grouping: tets in Morton order of their centroids; an unassigned tet seeds a group on the edge whose
// fan of unassigned, same-material tets (walked both ways around the edge from the seed) is longest
// (closed fans preferred); a closed fan of f < 6 tets repeats r_0 in slot f, an open fan holds <= 5 tets.
// Tiles: recursive coordinate bisection of the group centroids (rcb_partition) into <= nt groups, split
// further while a tile's node list exceeds max_nodes or a node's run exceeds kGroupMaxRun pushes; the local
// CSR of pushed forces is ordered by (node, group), the fold order, and every run is padded as for the tet
// tiles (abi.cpp). A group's push position for slot s is its node's run start (kept in LDS by the kernel)
// plus the group's rank in that run, so the 16-B record carries 4-bit ranks instead of 16-bit positions.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "cwf_internal.hpp"

namespace cwf
{
namespace
{
struct Fan
{
    uint32_t a = 0, b = 0;
    uint32_t r[7] = {};  // ring nodes in walk order
    int nr = 0;
    uint32_t t[6] = {};  // tets in fan order: t[i] = {a, b, r[i], r[i + 1]} (closed: r[f] == r[0])
    int f = 0;
    bool closed = false;
};

// the two nodes of tet `t` other than u, v
inline void others(const uint32_t *c, uint32_t u, uint32_t v, uint32_t &p, uint32_t &q)
{
    uint32_t o[2];
    int k = 0;
    for (int i = 0; i < 4; ++i)
        if (c[i] != u && c[i] != v && k < 2)
            o[k++] = c[i];
    p = o[0];
    q = k > 1 ? o[1] : o[0];
}

// longest fan of unassigned same-material tets around edge (u, v) through seed tet t
Fan walk_fan(const uint32_t *conn, const std::vector<uint32_t> &off, const std::vector<uint32_t> &lst,
             const std::vector<uint32_t> &group, const uint32_t *mat, uint32_t t, uint32_t u, uint32_t v,
             std::vector<uint32_t> &star)
{
    // star = tets of u that also contain v, unassigned, same material as t (both lists ascending)
    star.clear();
    for (uint32_t i = off[u], j = off[v]; i < off[u + 1] && j < off[v + 1];)
    {
        if (lst[i] < lst[j])
            ++i;
        else if (lst[i] > lst[j])
            ++j;
        else
        {
            const uint32_t s = lst[i];
            if (group[s] == ~0u && (!mat || mat[s] == mat[t]))
                star.push_back(s);
            ++i;
            ++j;
        }
    }
    Fan F;
    F.a = u;
    F.b = v;
    uint32_t p, q;
    others(conn + 8ull * t, u, v, p, q);
    uint32_t R[13];
    uint32_t TT[12];
    int head = 6, tail = 7;  // R[head..tail], TT[head..tail-1]
    R[6] = p;
    R[7] = q;
    TT[6] = t;
    std::vector<char> used(star.size(), 0);
    for (size_t k = 0; k < star.size(); ++k)
        used[k] = star[k] == t;
    const auto next = [&](uint32_t from, uint32_t &to, uint32_t &tet) -> bool {
        for (size_t k = 0; k < star.size(); ++k)
            if (!used[k])
            {
                uint32_t x, y;
                others(conn + 8ull * star[k], u, v, x, y);
                if (x == from || y == from)
                {
                    used[k] = 1;
                    to = x == from ? y : x;
                    tet = star[k];
                    return true;
                }
            }
        return false;
    };
    bool closed = false;
    // forward from q
    while (tail - head < 6)
    {
        uint32_t to, tet;
        if (!next(R[tail], to, tet))
            break;
        if (to == R[head])  // back at the start: the ring closes
        {
            TT[tail] = tet;
            closed = true;
            break;
        }
        if (tail - head == 5)  // an open fan holds <= 5 tets (<= 6 ring slots); leave this one
        {
            break;
        }
        ++tail;
        R[tail] = to;
        TT[tail - 1] = tet;
    }
    if (!closed)
        while (tail - head < 5)  // backward from p
        {
            uint32_t to, tet;
            if (!next(R[head], to, tet))
                break;
            if (to == R[tail])
                break;  // closing from this side would need the forward tet already tried
            --head;
            R[head] = to;
            TT[head] = tet;
        }
    F.closed = closed;
    F.nr = tail - head + 1;
    for (int i = 0; i < F.nr; ++i)
        F.r[i] = R[head + i];
    F.f = closed ? F.nr : F.nr - 1;
    for (int i = 0; i < F.f; ++i)
        F.t[i] = TT[head + i];
    return F;
}

// ds_read_b128 lane groups of a wave64 access (MI355X_MICROARCH.md §LDS): {0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31}, and the same two + 32
inline uint32_t lane_group128(uint32_t l)
{
    const uint32_t h = (l & 63u) >= 32u ? 2u : 0u;
    l &= 31u;
    const bool g0 = l < 4u || (l >= 12u && l < 16u) || (l >= 20u && l < 28u);
    return h + (g0 ? 0u : 1u);
}

// The fan kernel reads every group's 8 slot nodes from LDS by local id, all lanes in lockstep per slot:
// {x y z v_x} by ds_read_b128 (bank 4 lid mod 64: conflict-free when the 16 lanes of a lane group have
// distinct lid mod 16), {v_y v_z} by ds_read_b64 (32-lane groups, lid mod 32) and the u16 run start
// (32-lane groups, (lid / 2) mod 32); then it pushes one force per used slot, {f_x, f_y} by ds_write_b64
// (16-lane groups, bank 2 q mod 32) and f_z by ds_write_b32 (32-lane groups, q mod 32) at q = the node's run
// start + the group's rank in the run. In RCB order those addresses collide often: the C2 kernel's group
// phase spent 1.16M extra LDS cycles per launch on bank conflicts (tools/lds_ablate.sh; tools/tile_stats.cpp
// models the same count: 0.51M from the reads, 0.63M from the pushes). Greedy, lane by lane: take, among the
// next W unplaced groups, the one adding the fewest same-bank accesses to its lane groups (ranks follow the
// placement order, so a candidate's push positions are known; ties: the earliest, so RCB order is the
// fallback). The fold order follows the new lane order.
template <typename SlotNode, typename SlotsUsed>
void order_lanes_by_bank(const std::vector<Fan> &fans, const SlotNode &slot_node, const SlotsUsed &slots_used,
                         const std::vector<uint32_t> &local, const std::vector<uint32_t> &start,
                         std::vector<uint32_t> &placed, uint32_t *grp, uint32_t ng)
{
    constexpr uint32_t W = 32;
    const uint32_t nw = (ng + 63u) / 64u;
    std::vector<uint8_t> c128(nw * 4u * 8u * 16u, 0), c64(nw * 2u * 8u * 32u, 0), c16(nw * 2u * 8u * 32u, 0);
    std::vector<uint8_t> cw64(nw * 4u * 8u * 16u, 0), cw32(nw * 2u * 8u * 32u, 0);
    uint32_t lid[8], q[8];
    const auto slots = [&](const Fan &F) {  // local ids and push positions of F placed next
        const int su = slots_used(F);
        for (int s = 0; s < 8; ++s)
        {
            lid[s] = local[slot_node(F, s)];
            uint32_t dup = 0;  // a closing repeat pushes to r_0 twice
            for (int r = 0; r < s; ++r)
                dup += r < su && lid[r] == lid[s];
            q[s] = s < su ? start[lid[s]] + placed[lid[s]] + dup : ~0u;
        }
    };
    for (uint32_t L = 0; L < ng; ++L)
    {
        const uint32_t w = L / 64u, g128 = lane_group128(L), g32 = (L & 63u) >> 5, g16 = (L & 63u) >> 4;
        uint8_t *a = &c128[(w * 4u + g128) * 8u * 16u];
        uint8_t *b = &c64[(w * 2u + g32) * 8u * 32u];
        uint8_t *c = &c16[(w * 2u + g32) * 8u * 32u];
        uint8_t *d = &cw64[(w * 4u + g16) * 8u * 16u];
        uint8_t *e = &cw32[(w * 2u + g32) * 8u * 32u];
        uint32_t best = L, best_cost = ~0u;
        const uint32_t end = std::min(ng, L + W);
        for (uint32_t k = L; k < end && best_cost; ++k)
        {
            slots(fans[grp[k]]);
            uint32_t cost = 0;
            for (int s = 0; s < 8; ++s)
            {
                cost += a[s * 16 + (lid[s] & 15u)] + b[s * 32 + (lid[s] & 31u)] + c[s * 32 + ((lid[s] >> 1) & 31u)];
                if (q[s] != ~0u)
                    cost += d[s * 16 + (q[s] & 15u)] + e[s * 32 + (q[s] & 31u)];
            }
            if (cost < best_cost)
            {
                best_cost = cost;
                best = k;
            }
        }
        std::rotate(grp + L, grp + best, grp + best + 1);
        slots(fans[grp[L]]);
        for (int s = 0; s < 8; ++s)
        {
            ++a[s * 16 + (lid[s] & 15u)];
            ++b[s * 32 + (lid[s] & 31u)];
            ++c[s * 32 + ((lid[s] >> 1) & 31u)];
            if (q[s] != ~0u)
            {
                ++d[s * 16 + (q[s] & 15u)];
                ++e[s * 32 + (q[s] & 31u)];
            }
        }
        for (int s = 0; s < 8; ++s)
            if (q[s] != ~0u)
                ++placed[lid[s]];
    }
}
}  // namespace

int build_group_tiles(const cwf_system_desc *d, GroupTiles &out, uint32_t nt, uint32_t max_nodes,
                      uint32_t slot_budget, bool order_lanes)
{
    out = GroupTiles{};
    const uint64_t N = d->node_count, E = d->element_count;
    const uint32_t *conn = d->element_connectivity;
    const uint32_t *mat = d->material_count > 1 ? d->element_material_index : nullptr;
    if (!d->node_coords || !E || max_nodes > 512 || d->material_count > 32)
        return -1;
    // node -> tets, ascending tet
    std::vector<uint32_t> off(N + 1, 0), lst(4 * E);
    for (uint64_t e = 0; e < E; ++e)
        for (int a = 0; a < 4; ++a)
            ++off[conn[8 * e + a] + 1];
    for (uint64_t n = 0; n < N; ++n)
        off[n + 1] += off[n];
    {
        std::vector<uint32_t> cur(off.begin(), off.end() - 1);
        for (uint64_t e = 0; e < E; ++e)
            for (int a = 0; a < 4; ++a)
                lst[cur[conn[8 * e + a]]++] = (uint32_t)e;
    }
    // seed order: Morton order of the tet centroids
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
        uint64_t q[3];
        for (int k = 0; k < 3; ++k)
        {
            double c = 0.0;
            for (int a = 0; a < 4; ++a)
                c += d->node_coords[3ull * conn[8 * e + a] + k];
            q[k] = (uint64_t)std::llround((c / 4.0 - lo[k]) * scale);
        }
        key[e] = spread21(q[0]) | spread21(q[1]) << 1 | spread21(q[2]) << 2;
    }
    std::vector<uint32_t> seed(E);
    std::iota(seed.begin(), seed.end(), 0u);
    std::stable_sort(seed.begin(), seed.end(), [&](uint32_t x, uint32_t y) { return key[x] < key[y]; });
    key.clear();
    key.shrink_to_fit();

    // fans
    std::vector<uint32_t> group(E, ~0u);
    std::vector<Fan> fans;
    fans.reserve(E / 4 + 1);
    std::vector<uint32_t> star;
    static const int EDGES[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
    for (const uint32_t t : seed)
    {
        if (group[t] != ~0u)
            continue;
        const uint32_t *c = conn + 8ull * t;
        Fan best;
        for (int q = 0; q < 6; ++q)
        {
            const Fan F = walk_fan(conn, off, lst, group, mat, t, c[EDGES[q][0]], c[EDGES[q][1]], star);
            if (F.f > best.f || (F.f == best.f && F.closed && !best.closed))
                best = F;
        }
        const uint32_t g = (uint32_t)fans.size();
        for (int i = 0; i < best.f; ++i)
            group[best.t[i]] = g;
        fans.push_back(best);
    }
    const uint64_t G = fans.size();
    out.ngroups = (uint32_t)G;
    out.tets_per_group = (double)E / (double)G;
    // slots of a group: 0 = a, 1 = b, 2 + i = ring node i (closed f < 6: ring slot f repeats r_0);
    // used: a, b and ring slots 0 .. min(f + 1, 6) - 1
    const auto slot_node = [&](const Fan &F, int s) -> uint32_t {
        if (s == 0)
            return F.a;
        if (s == 1)
            return F.b;
        const int i = s - 2;
        if (i < F.nr)
            return F.r[i];
        return F.closed && i == F.nr ? F.r[0] : F.a;  // the closing repeat; unused slots point at a
    };
    const auto slots_used = [](const Fan &F) { return 2 + std::min(F.f + 1, 6); };
    // group centroids and extents for the RCB
    std::vector<double> cen(3 * G);
    double gext[3] = {0.0, 0.0, 0.0};
    for (uint64_t g = 0; g < G; ++g)
    {
        const Fan &F = fans[g];
        const int su = slots_used(F);
        for (int k = 0; k < 3; ++k)
        {
            double v = 0.0, mn = 1e300, mx = -1e300;
            for (int s = 0; s < su; ++s)
            {
                const double x = d->node_coords[3ull * slot_node(F, s) + k];
                v += x;
                mn = std::min(mn, x);
                mx = std::max(mx, x);
            }
            cen[3 * g + k] = v / su;
            gext[k] += mx - mn;
        }
    }
    for (int k = 0; k < 3; ++k)
        gext[k] /= (double)G;
    std::vector<uint32_t> order(G);
    std::iota(order.begin(), order.end(), 0u);
    std::vector<uint64_t> leaf_end;
    // leaves aimed at the full lane count with a +-n/32 layer-gap window: C3 14.3k tiles at 90% lane fill
    // against 15.9k at 81% for the per-tet tiles' 15/16 target and +-n/16 window, same T/N (K_eff 111.4 ->
    // 105.6 us, +3.7% PCG it/s); C2 2.9k tiles against 3.2k (T/N 1.73 -> 1.76, +1.2%) (same-box A/B).
    const int tdiv = 0, wdiv = 32;  // the RCB leaf target and layer-gap window (measured best, rounds 2-3)
    rcb_partition(cen, gext, order, nt, leaf_end, tdiv, wdiv);

    // lanes of a tile ordered against LDS bank conflicts (order_lanes_by_bank)
    const bool lanes_by_bank = order_lanes;
    // tiles: each RCB leaf, split greedily while its node list would exceed max_nodes
    std::vector<uint32_t> stamp(N, ~0u), local(N, 0), tcnt(N, 0), placed;
    std::vector<uint32_t> nodes, cnt, cur;
    out.hdr.clear();
    out.grec.resize(G);
    uint64_t p = 0;
    uint32_t tile = 0;
    size_t leaf = 0;
    std::vector<uint32_t> gorder;  // groups in tile order
    gorder.reserve(G);
    while (p < G)
    {
        while (leaf < leaf_end.size() && leaf_end[leaf] <= p)
            ++leaf;
        const uint64_t stop = leaf < leaf_end.size() ? leaf_end[leaf] : G;
        nodes.clear();
        const uint64_t p0 = p;
        uint32_t pslots = 0;  // the tile's slots with runs padded to even lengths (the layout below without spread)
        while (p < stop && p - p0 < nt)
        {
            const Fan &F = fans[order[p]];
            uint32_t add = 0, dslots = 0;
            bool long_run = false;
            for (int s = 0; s < slots_used(F); ++s)
            {
                const uint32_t n = slot_node(F, s);
                if (stamp[n] != tile)
                {
                    stamp[n] = tile;
                    tcnt[n] = 0;
                    ++add;
                    nodes.push_back(n);
                }
                dslots += (tcnt[n] & 1u) ? 0u : 2u;  // an even run grows by a padded pair
                long_run |= ++tcnt[n] > kGroupMaxRun;
            }
            // a slot budget below 10 per lane (the 4-wave LDS layout) closes the tile at the budget too
            if (nodes.size() > max_nodes || long_run || pslots + dslots > slot_budget)
            {
                // undo this group's pushes and new nodes and close the tile before it
                for (int s = 0; s < slots_used(F); ++s)
                    --tcnt[slot_node(F, s)];
                for (uint32_t k = 0; k < add; ++k)
                {
                    stamp[nodes.back()] = ~0u;
                    nodes.pop_back();
                }
                break;
            }
            pslots += dslots;
            ++p;
        }
        if (p == p0)
            return -2;  // one group alone exceeds max_nodes (cannot happen: <= 8 nodes)
        std::sort(nodes.begin(), nodes.end());
        const uint32_t nn = (uint32_t)nodes.size(), ng = (uint32_t)(p - p0);
        for (uint32_t i = 0; i < nn; ++i)
            local[nodes[i]] = i;
        // push entries per node, ascending group within the tile
        cnt.assign(nn, 0);
        for (uint64_t q = p0; q < p; ++q)
        {
            const Fan &F = fans[order[q]];
            for (int s = 0; s < slots_used(F); ++s)
                ++cnt[local[slot_node(F, s)]];
        }
        // padded runs: even starts, 2 (mod 4) slots where the budget allows (the tet tiles' rule, abi.cpp)
        std::vector<uint32_t> start(nn);
        for (int spread = 1; spread >= 0; --spread)
        {
            uint32_t padded = 0;
            for (uint32_t i = 0; i < nn; ++i)
            {
                start[i] = padded;
                uint32_t len = (cnt[i] + 1u) & ~1u;
                if (spread && (len / 2u) % 2u == 0u)
                    len += 2u;
                padded += len;
            }
            out.max_tile_slots = std::max(out.max_tile_slots, padded);
            if (padded <= slot_budget || !spread)
                break;
        }
        if (out.max_tile_slots > slot_budget)
            return -3;  // cannot happen: the tile closed at the budget (padded without spread)
        cur.assign(start.begin(), start.end());
        if (lanes_by_bank)
        {
            placed.assign(nn, 0);
            order_lanes_by_bank(fans, slot_node, slots_used, local, start, placed, order.data() + p0, ng);
        }
        const uint32_t nb = (uint32_t)out.tile_nodes.size();
        for (uint64_t q = p0; q < p; ++q)
        {
            const uint32_t g = order[q];
            const Fan &F = fans[g];
            const uint64_t gi = gorder.size();
            gorder.push_back(g);
            uint32_t id[8], ranks = 0;
            for (int s = 0; s < 8; ++s)
            {
                id[s] = local[slot_node(F, s)];
                if (s < slots_used(F))
                    ranks |= (cur[id[s]]++ - start[id[s]]) << (4 * s);  // < kGroupMaxRun (tile loop above)
            }
            out.grec[gi] = uint4{id[0] | id[1] << 9 | id[2] << 18 | (uint32_t)F.f << 27,
                                 id[3] | id[4] << 9 | id[5] << 18 | (mat ? mat[F.t[0]] : 0u) << 27,
                                 id[6] | id[7] << 9, ranks};
        }
        const double *o = d->node_coords + 3ull * nodes[0];
        for (uint32_t i = 0; i < nn; ++i)
        {
            out.tile_nodes.push_back(nodes[i]);
            out.run.push_back(start[i] | ((start[i] + cnt[i]) << 16));
            for (int k = 0; k < 3; ++k)
                out.tcoord[k].push_back((float)(d->node_coords[3ull * nodes[i] + k] - o[k]));
        }
        out.hdr.push_back(uint4{(uint32_t)p0, ng, nb, nn});
        out.max_tile_nodes = std::max(out.max_tile_nodes, nn);
        ++tile;
    }
    out.ntiles = tile;
    // groups were emitted in tile order: gorder[gi] = fan index; tets map to the emitted index
    std::vector<uint32_t> emitted(G);
    for (uint64_t gi = 0; gi < G; ++gi)
        emitted[gorder[gi]] = (uint32_t)gi;
    out.tet_group.resize(E);
    for (uint64_t e = 0; e < E; ++e)
        out.tet_group[e] = emitted[group[e]];
    // node -> slots ascending tile, node-major slot of every tile node, owner = first slot (bit 31)
    const uint64_t T = out.tile_nodes.size();
    out.node_part_off.assign(N + 1, 0);
    for (uint64_t s = 0; s < T; ++s)
        ++out.node_part_off[out.tile_nodes[s] + 1];
    for (uint64_t n = 0; n < N; ++n)
        out.node_part_off[n + 1] += out.node_part_off[n];
    out.tile_slot.resize(T);
    {
        std::vector<uint32_t> c2(out.node_part_off.begin(), out.node_part_off.end() - 1);
        for (uint64_t s = 0; s < T; ++s)
        {
            const uint32_t n = out.tile_nodes[s];
            if (c2[n] == out.node_part_off[n])
                out.tile_nodes[s] |= 0x80000000u;  // the node's first (lowest-tile) slot owns it
            out.tile_slot[s] = c2[n]++;
        }
    }
    return 0;
}

}  // namespace cwf

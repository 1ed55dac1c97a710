// shard.cpp -- host-side node-range partition of a tet4 or hex8 mesh into rank-local shards (SURVEY.md
// section 8e; no reference counterpart: the reference runs on one device, and its
// src/gpu/sharding.cpp:38-144 only splits packed buffers under Vulkan's 2 GiB buffer cap).
//
// Rank r owns the global nodes [rank_node_begin[r], rank_node_begin[r+1]). Its shard holds
//   * every element touching an owned node, in the input (ascending global) element order, so
//     each owned node sees exactly its global element set and its K_eff row is complete;
//   * local node numbering: owned nodes first (ascending global id), then the ghost nodes grouped by
//     owner rank (ascending), ascending global id inside a group -> the ghosts received from one
//     neighbour are one contiguous range;
//   * the halo plan: neighbour ranks (= owners of ghosts), and per neighbour the owned nodes it needs
//     (owned nodes of a local element that also has a node of that neighbour), ascending global id.
// By construction rank q's ghost range from r and r's send list to q are the same node set in the
// same order: an element holding an r-owned and a q-owned node is in both shards.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "cwf_internal.hpp"

struct cwf_shard
{
    uint64_t owned = 0;
    std::vector<uint64_t> node_global, element_source, node_source;
    std::vector<int32_t> nbr;
    std::vector<uint64_t> send_off, recv_off;
    std::vector<uint32_t> send_nodes;
    // local system arrays
    std::vector<uint32_t> conn8, mat, mask;
    std::vector<float> grads, vol, mass;
    std::vector<double> dmat, coords;
    cwf_system_desc desc{};
};

using namespace cwf;

extern "C" {

int cwf_shard_build(const cwf_system_desc *d, const uint64_t *node_global_ids, const uint64_t *rank_node_begin,
                    int32_t nranks, int32_t rank, cwf_shard **out)
{
    if (!d || !rank_node_begin || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    // tet4 (slots 4..7 = UINT32_MAX) or native hex8 (all 8 slots)
    const int corners = d->element_count && d->element_connectivity && d->element_connectivity[4] != 0xFFFFFFFFu ? 8 : 4;
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "rank out of range",
                         "nranks=" + std::to_string(nranks) + "\nrank=" + std::to_string(rank));
    for (int32_t q = 0; q < nranks; ++q)
        if (rank_node_begin[q + 1] < rank_node_begin[q])
            return set_error(nullptr, CWF_ERR_ARGUMENT, "rank node ranges must be non-decreasing",
                             "rank=" + std::to_string(q));
    const uint64_t N = d->node_count, E = d->element_count;
    if ((E && (!d->element_connectivity || !d->element_gradients || !d->element_volume ||
               !d->element_material_index)) ||
        (N && (!d->lumped_mass || !d->bc_mask)) || !d->material_stiffness || d->material_count == 0)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null system array");
    cwf_shard *s = new (std::nothrow) cwf_shard();
    if (!s)
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    try
    {
        auto gid = [&](uint64_t n) { return node_global_ids ? node_global_ids[n] : n; };
        std::vector<int32_t> owner(N);
        for (uint64_t n = 0; n < N; ++n)
        {
            const uint64_t g = gid(n);
            if (g < rank_node_begin[0] || g >= rank_node_begin[nranks])
            {
                delete s;
                return set_error(nullptr, CWF_ERR_NODE_RANGE, "node outside every rank's range",
                                 "node=" + std::to_string(n) + "\nglobal=" + std::to_string(g));
            }
            owner[n] = (int32_t)(std::upper_bound(rank_node_begin, rank_node_begin + nranks + 1, g) -
                                 rank_node_begin) - 1;
        }
        // elements touching an owned node
        std::vector<uint8_t> used(N, 0);
        for (uint64_t e = 0; e < E; ++e)
        {
            const uint32_t *c = d->element_connectivity + 8 * e;
            if ((c[4] != 0xFFFFFFFFu) != (corners == 8))
            {
                delete s;
                return set_error(nullptr, CWF_ERR_UNSUPPORTED, "mixed tet4/hex8 meshes are not supported",
                                 "element=" + std::to_string(e));
            }
            bool mine = false;
            for (int a = 0; a < corners; ++a)
            {
                if (c[a] >= N)
                {
                    delete s;
                    return set_error(nullptr, CWF_ERR_NODE_RANGE, "element connectivity references node out of range",
                                     "element=" + std::to_string(e) + "\nnode=" + std::to_string(c[a]));
                }
                mine |= owner[c[a]] == rank;
            }
            if (!mine)
                continue;
            s->element_source.push_back(e);
            for (int a = 0; a < corners; ++a)
                used[c[a]] = 1;
        }
        // local numbering: owned (ascending global), ghosts by (owner, global)
        std::vector<uint64_t> own_nodes, ghost_nodes;
        for (uint64_t n = 0; n < N; ++n)
        {
            if (owner[n] == rank)
                own_nodes.push_back(n);
            else if (used[n])
                ghost_nodes.push_back(n);
        }
        std::sort(own_nodes.begin(), own_nodes.end(), [&](uint64_t a, uint64_t b) { return gid(a) < gid(b); });
        std::sort(ghost_nodes.begin(), ghost_nodes.end(), [&](uint64_t a, uint64_t b) {
            return owner[a] != owner[b] ? owner[a] < owner[b] : gid(a) < gid(b);
        });
        const uint64_t NL = own_nodes.size() + ghost_nodes.size();
        s->owned = own_nodes.size();
        std::vector<uint32_t> local(N, 0xFFFFFFFFu);
        std::vector<uint64_t> src_node(NL);
        for (uint64_t i = 0; i < own_nodes.size(); ++i)
            src_node[i] = own_nodes[i];
        for (uint64_t i = 0; i < ghost_nodes.size(); ++i)
            src_node[s->owned + i] = ghost_nodes[i];
        s->node_global.resize(NL);
        s->node_source = src_node;
        for (uint64_t i = 0; i < NL; ++i)
        {
            local[src_node[i]] = (uint32_t)i;
            s->node_global[i] = gid(src_node[i]);
        }
        // neighbours and ghost ranges
        s->recv_off.push_back(0);
        for (uint64_t i = 0; i < ghost_nodes.size(); ++i)
        {
            const int32_t q = owner[ghost_nodes[i]];
            if (s->nbr.empty() || s->nbr.back() != q)
            {
                if (!s->nbr.empty())
                    s->recv_off.push_back(i);
                s->nbr.push_back(q);
            }
        }
        if (!s->nbr.empty())
            s->recv_off.push_back(ghost_nodes.size());
        // send lists: owned nodes of local elements that also hold a node of neighbour q
        const size_t K = s->nbr.size();
        std::vector<std::vector<uint32_t>> send(K);
        std::vector<uint32_t> stamp(NL, 0xFFFFFFFFu);
        for (size_t k = 0; k < K; ++k)
        {
            const int32_t q = s->nbr[k];
            for (uint64_t e : s->element_source)
            {
                const uint32_t *c = d->element_connectivity + 8 * e;
                bool has_q = false;
                for (int a = 0; a < corners; ++a)
                    has_q |= owner[c[a]] == q;
                if (!has_q)
                    continue;
                for (int a = 0; a < corners; ++a)
                {
                    const uint32_t l = local[c[a]];
                    if (l < s->owned && stamp[l] != (uint32_t)k)
                    {
                        stamp[l] = (uint32_t)k;
                        send[k].push_back(l);
                    }
                }
            }
            std::sort(send[k].begin(), send[k].end());  // owned local order == ascending global id
        }
        s->send_off.push_back(0);
        for (size_t k = 0; k < K; ++k)
        {
            s->send_nodes.insert(s->send_nodes.end(), send[k].begin(), send[k].end());
            s->send_off.push_back(s->send_nodes.size());
        }
        // local system arrays
        const uint64_t EL = s->element_source.size();
        s->conn8.assign(EL * 8, 0xFFFFFFFFu);
        s->grads.resize(EL * 24);
        s->vol.resize(EL);
        s->mat.resize(EL);
        for (uint64_t j = 0; j < EL; ++j)
        {
            const uint64_t e = s->element_source[j];
            for (int a = 0; a < corners; ++a)
                s->conn8[8 * j + a] = local[d->element_connectivity[8 * e + a]];
            std::memcpy(&s->grads[24 * j], d->element_gradients + 24 * e, 24 * sizeof(float));
            s->vol[j] = d->element_volume[e];
            s->mat[j] = d->element_material_index[e];
        }
        s->mass.resize(NL);
        s->mask.resize(NL);
        if (d->node_coords)
            s->coords.resize(3 * NL);
        for (uint64_t i = 0; i < NL; ++i)
        {
            s->mass[i] = d->lumped_mass[src_node[i]];
            s->mask[i] = d->bc_mask[src_node[i]];
            if (d->node_coords)
                for (int k = 0; k < 3; ++k)
                    s->coords[3 * i + k] = d->node_coords[3 * src_node[i] + k];
        }
        s->dmat.assign(d->material_stiffness, d->material_stiffness + 36 * d->material_count);
        cwf_system_desc &L = s->desc;
        L = cwf_system_desc{};
        L.node_count = NL;
        L.element_count = EL;
        L.dof_count = 3 * NL;
        L.element_connectivity = s->conn8.data();
        L.element_gradients = s->grads.data();
        L.element_volume = s->vol.data();
        L.element_material_index = s->mat.data();
        L.material_stiffness = s->dmat.data();
        L.material_count = d->material_count;
        L.lumped_mass = s->mass.data();
        L.bc_mask = s->mask.data();
        L.stiffness_scale = d->stiffness_scale;
        L.mass_factor = d->mass_factor;
        L.reduction_block = d->reduction_block ? d->reduction_block : 256;
        L.reduction_partials = std::max<uint64_t>(1, (3 * NL + L.reduction_block - 1) / L.reduction_block);
        L.mode = d->mode;
        L.node_coords = d->node_coords ? s->coords.data() : nullptr;
    }
    catch (const std::bad_alloc &)
    {
        delete s;
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    }
    *out = s;
    return 0;
}

int cwf_shard_get(const cwf_shard *s, cwf_system_desc *local_desc, cwf_shard_info *info)
{
    if (!s)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null shard");
    if (local_desc)
        *local_desc = s->desc;
    if (info)
    {
        info->owned_nodes = s->owned;
        info->local_nodes = s->node_global.size();
        info->local_elements = s->element_source.size();
        info->neighbor_count = (uint32_t)s->nbr.size();
        info->reserved = 0;
        info->neighbor_ranks = s->nbr.data();
        info->send_offsets = s->send_off.data();
        info->send_nodes = s->send_nodes.data();
        info->recv_offsets = s->recv_off.data();
        info->node_global = s->node_global.data();
        info->element_source = s->element_source.data();
        info->node_source = s->node_source.data();
    }
    return 0;
}

void cwf_shard_destroy(cwf_shard *s) { delete s; }

}  // extern "C"

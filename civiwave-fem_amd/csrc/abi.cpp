// abi.cpp -- C-ABI (include/cwf_hip.h) over the gfx950 kernels: handle lifetime (validation, HBM layout and
// upload, the FAST tilings and the structured-block detection), mode / scalar / timing switches and the
// measurement entry points. One HIP stream per handle. The PCG entry points are in abi_pcg.cpp, the Stepper in
// abi_stepper.cpp, the communicators in comm.cpp and peer.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "blockinv_pack.hpp"
#include "cwf_internal.hpp"

namespace cwf
{

static thread_local std::string g_err, g_ctx;

int set_error(cwf_hip_system *h, int code, const std::string &msg, const std::string &ctx)
{
    if (h)
    {
        h->err = msg;
        h->ctx = ctx;
    }
    g_err = msg;
    g_ctx = ctx;
    return code;
}

int hip_fail(cwf_hip_system *h, hipError_t e, const char *what)
{
    return set_error(h, CWF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e), hipGetErrorName(e));
}

// hex8 tile lanes: 256 (<= 256 hexes, <= 512 nodes) from 1M hexes up, else 128. The per-workgroup p.Ap shares
// every update workgroup refolds (and the r.r / r.z shares every hex workgroup refolds) halve with the
// workgroup count: C3 hex8 +2.5-3.9% on 256 lanes, C2 hex8 -2.0-2.5% (same-box A/B, two passes).
// CWF_HEX_NT=128|256 overrides
uint32_t hex_tile_lanes(uint64_t hexes)
{
    const char *e = knob("CWF_HEX_NT");
    if (e)
        return atoi(e) == 256 ? 256u : 128u;
    return hexes >= 1000000ull ? 256u : 128u;
}

}  // namespace cwf

using namespace cwf;

#include "abi_internal.hpp"

namespace cwf
{

bool iso_pattern(const double *D)
{
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c)
        {
            const bool nz = (r < 3 && c < 3) || (r == c);
            if (!nz && D[6 * r + c] != 0.0)
                return false;
        }
    return true;
}

// Built on first use (a PARITY create or set_mode(PARITY)), from the node -> incidence CSR already on the device:
// the node tiles of k_keff_parity_tile. Tile b holds nodes [256 b, 256 b + 256) (three whole 256-DOF reduction
// chunks, so the p.Ap chunk partials stay fused), its incident tets in ascending element order, and for each of its
// nodes' incidences the tet's index in that list. FAST handles never build it.
// above this many tets the host-side breadth-first pass (random reads of 16 B of connectivity per incidence) takes
// tens of seconds: strips there (C5's 96M tets)
constexpr uint64_t kParityCompactMaxTets = 1ull << 25;

// Compact PARITY tiles: greedy breadth-first blobs of <= 256 nodes over the node graph (two nodes adjacent when
// they share a tet), seeded in node order. On C2 the strip tiles (256 consecutive nodes of the caller's
// lexicographic order, one plane thick) evaluate each tet ~2.4 times; blobs fewer.
std::vector<uint32_t> parity_compact_tiles(const std::vector<uint32_t> &off, const std::vector<uint32_t> &inc,
                                           const std::vector<uint32_t> &conn, uint64_t N)
{
    std::vector<uint32_t> nodes;
    nodes.reserve(N + N / 4);
    std::vector<uint8_t> state(N, 0);  // 0 free, 1 queued for the current tile, 2 placed
    std::vector<uint32_t> queue;
    queue.reserve(4096);
    for (uint64_t seed = 0; seed < N; ++seed)
    {
        if (state[seed])
            continue;
        queue.clear();
        queue.push_back((uint32_t)seed);
        state[seed] = 1;
        size_t head = 0, placed = 0;
        while (head < queue.size() && placed < 256)
        {
            const uint32_t u = queue[head++];
            state[u] = 2;
            nodes.push_back(u);
            ++placed;
            for (uint32_t j = off[u]; j < off[u + 1]; ++j)
                for (int c = 0; c < 4; ++c)
                {
                    const uint32_t v = conn[4ull * (inc[j] >> 2) + c];
                    if (!state[v])
                    {
                        state[v] = 1;
                        queue.push_back(v);
                    }
                }
        }
        for (size_t q = head; q < queue.size(); ++q)  // queued but not placed: free again
            state[queue[q]] = 0;
        nodes.resize((nodes.size() + 255) / 256 * 256, 0xFFFFFFFFu);
    }
    return nodes;
}

int parity_incidence_slots(cwf_hip_system *h)
{
    DevSys &s = h->ds;
    const uint64_t N = s.N, E = s.E;
    // compact tiles for single handles (a shard's PCG loop folds p.Ap into rank-ordered chunk partials in the tile
    // kernel, which needs tiles of consecutive nodes); CWF_PARITY_TILES=strip keeps the strips
    const char *pt = knob("CWF_PARITY_TILES");
    const bool compact = !h->sharded() && E <= kParityCompactMaxTets && !(pt && std::strcmp(pt, "strip") == 0);
    std::vector<uint32_t> off, inc, toff, tets, pinc, conn, tnodes;
    try
    {
        off.resize(N + 1);
        inc.resize(4 * E);
        pinc.resize(4 * E);
        tets.reserve(3 * E);
        if (compact)
            conn.resize(4 * E);
    }
    catch (const std::bad_alloc &)
    {
        return set_error(h, CWF_ERR_ALLOC, "host allocation failed");
    }
    HIPTRY(h, hipMemcpy(off.data(), s.off, (N + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIPTRY(h, hipMemcpy(inc.data(), s.inc, 4 * E * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (compact)
    {
        // the corner ids: the first 16 B of every 64-B element record
        HIPTRY(h, hipMemcpy2D(conn.data(), 16, s.erec, 64, 16, E, hipMemcpyDeviceToHost));
        try
        {
            tnodes = parity_compact_tiles(off, inc, conn, N);
        }
        catch (const std::bad_alloc &)
        {
            return set_error(h, CWF_ERR_ALLOC, "host allocation failed");
        }
    }
    const uint64_t nt = compact ? tnodes.size() / 256 : (N + 255) / 256;
    toff.resize(nt + 1);
    std::vector<uint32_t> loc;
    for (uint64_t b = 0; b < nt; ++b)
    {
        toff[b] = (uint32_t)tets.size();
        loc.clear();
        const auto tile_node = [&](uint64_t t) -> uint64_t {
            return compact ? (uint64_t)tnodes[256 * b + t] : 256 * b + t;
        };
        for (uint64_t t = 0; t < 256; ++t)
        {
            const uint64_t n = tile_node(t);
            if (n < N)
                for (uint32_t j = off[n]; j < off[n + 1]; ++j)
                    loc.push_back(inc[j] >> 2);
        }
        std::sort(loc.begin(), loc.end());
        loc.erase(std::unique(loc.begin(), loc.end()), loc.end());
        for (uint64_t t = 0; t < 256; ++t)
        {
            const uint64_t n = tile_node(t);
            if (n < N)
                for (uint32_t j = off[n]; j < off[n + 1]; ++j)
                    pinc[j] = (uint32_t)(std::lower_bound(loc.begin(), loc.end(), inc[j] >> 2) - loc.begin()) << 2 |
                              (inc[j] & 3u);
        }
        try
        {
            tets.insert(tets.end(), loc.begin(), loc.end());
        }
        catch (const std::bad_alloc &)
        {
            return set_error(h, CWF_ERR_ALLOC, "host allocation failed");
        }
        if (tets.size() >= (1ull << 32))
            return set_error(h, CWF_ERR_UNSUPPORTED, "mesh too large for one PARITY handle (shard it)",
                             "tile_tets=" + std::to_string(tets.size()));
    }
    toff[nt] = (uint32_t)tets.size();
    uint32_t *dto, *dte, *dpi, *dtn = nullptr;
    if (int st = upload(h, &dto, toff.data(), nt + 1))
        return st;
    if (int st = upload(h, &dte, tets.data(), tets.size()))
        return st;
    if (int st = upload(h, &dpi, pinc.data(), 4 * E))
        return st;
    if (compact)
        if (int st = upload(h, &dtn, tnodes.data(), tnodes.size()))
            return st;
    s.ptile_off = dto;
    s.ptile_tets = dte;
    s.pinc = dpi;
    s.ptile_nodes = dtn;
    s.pntile = (uint32_t)nt;
    return 0;
}

int parity_force_buffer(cwf_hip_system *h)
{
    if (h->ds.ptile_off || h->ds.hex || !h->ds.E)
        return 0;
    return parity_incidence_slots(h);
}

int check_ready(cwf_hip_system *h)
{
    if (!h)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null handle");
    if (h->unusable)
        return set_error(h, CWF_ERR_ARGUMENT, "handle unusable after a failed attach",
                         "its operator plan was cut to a shard's owned rows; destroy it");
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess)
        return hip_fail(h, e, "hipSetDevice");
    return 0;
}

// stage a DOF vector: host -> device scratch, or use the device pointer directly
int stage_in(cwf_hip_system *h, const float *src, float *scratch, uint64_t n, int kind, const float **out)
{
    if (kind == CWF_PTR_DEVICE)
    {
        *out = src;
        return 0;
    }
    HIPTRY(h, hipMemcpyAsync(scratch, src, n * sizeof(float), hipMemcpyHostToDevice, h->stream));
    *out = scratch;
    return 0;
}

// caller-order node vector (w floats per node, host or device) -> internal order. Without renumbering a
// device input is used in place (*out = src); otherwise it lands in `scratch` (internal order).
int stage_vec(cwf_hip_system *h, const float *src, float *scratch, int kind, int w, const float **out)
{
    const uint64_t n = (uint64_t)w * h->ds.N;
    if (!h->perm)
        return stage_in(h, src, scratch, n, kind, out);
    const float *s = src;
    if (kind != CWF_PTR_DEVICE)
    {
        HIPTRY(h, hipMemcpyAsync(h->pbuf, src, n * sizeof(float), hipMemcpyHostToDevice, h->stream));
        s = h->pbuf;
    }
    perm_gather(h->perm, s, scratch, h->ds.N, w, h->stream);
    *out = scratch;
    return 0;
}

// caller-order input into a fixed internal buffer (always copies)
int vec_in(cwf_hip_system *h, const float *src, float *dst, int kind, int w)
{
    const float *p = nullptr;
    if (int st = stage_vec(h, src, dst, kind, w, &p))
        return st;
    if (p != dst)
        HIPTRY(h, hipMemcpyAsync(dst, p, (uint64_t)w * h->ds.N * sizeof(float), hipMemcpyDeviceToDevice, h->stream));
    return 0;
}

// internal-order device vector -> caller order (host or device)
int vec_out(cwf_hip_system *h, const float *src, float *dst, int kind, int w)
{
    const uint64_t n = (uint64_t)w * h->ds.N;
    if (!h->perm)
    {
        if (src != dst)
            HIPTRY(h, hipMemcpyAsync(dst, src, n * sizeof(float),
                                     kind == CWF_PTR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                     h->stream));
        return 0;
    }
    if (kind == CWF_PTR_DEVICE)
    {
        perm_scatter(h->perm, src, dst, h->ds.N, w, h->stream);
        return 0;
    }
    perm_scatter(h->perm, src, h->pbuf, h->ds.N, w, h->stream);
    HIPTRY(h, hipMemcpyAsync(dst, h->pbuf, n * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    return 0;
}

// Morton order of the node coordinates: perm[i] = caller node of internal node i
std::vector<uint32_t> morton_node_order(const double *X, uint64_t N)
{
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (uint64_t n = 0; n < N; ++n)
        for (int k = 0; k < 3; ++k)
        {
            lo[k] = std::min(lo[k], X[3 * n + k]);
            hi[k] = std::max(hi[k], X[3 * n + k]);
        }
    double ext = 0.0;
    for (int k = 0; k < 3; ++k)
        ext = std::max(ext, hi[k] - lo[k]);
    const double scale = ext > 0 ? (double)((1u << 21) - 1) / ext : 0.0;
    auto spread = [](uint64_t v) {
        v &= 0x1fffff;
        v = (v | v << 32) & 0x1f00000000ffffull;
        v = (v | v << 16) & 0x1f0000ff0000ffull;
        v = (v | v << 8) & 0x100f00f00f00f00full;
        v = (v | v << 4) & 0x10c30c30c30c30c3ull;
        v = (v | v << 2) & 0x1249249249249249ull;
        return v;
    };
    std::vector<uint64_t> key(N);
    for (uint64_t n = 0; n < N; ++n)
    {
        uint64_t q[3];
        for (int k = 0; k < 3; ++k)
            q[k] = (uint64_t)std::llround((X[3 * n + k] - lo[k]) * scale);
        key[n] = spread(q[0]) | spread(q[1]) << 1 | spread(q[2]) << 2;
    }
    std::vector<uint32_t> perm(N);
    std::iota(perm.begin(), perm.end(), 0u);
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
    return perm;
}

// CWF_GROUPS=0 (diagnostic): the per-tet tiles instead of the fan groups
bool groups_enabled()
{
    const char *gv = knob("CWF_GROUPS");
    return !(gv && gv[0] == '0');
}

// fan-group tile lanes: 256 (<= 256 groups, <= 512 nodes: T/N 1.59 against 1.77 on C3, 1.60 against 1.76 on
// C2). 128-lane tiles give C2's resident workgroups two tiles each instead of 1.7, but twice the workgroups
// whose per-workgroup p.Ap shares every update workgroup refolds: with write-through partials C2 runs +2.3%
// on 256 lanes (same-box A/B, two passes; 128 had been +6% before the partials were written through).
// CWF_GROUP_NT=128|256 overrides
uint32_t group_lanes(uint64_t E)
{
    (void)E;
    const char *gn = knob("CWF_GROUP_NT");
    return gn && atoi(gn) == 128 ? 128u : 256u;
}

}  // namespace cwf

extern "C" {

int cwf_hip_abi_version(void) { return CWF_HIP_ABI_VERSION; }

int cwf_hip_device_count(int *count)
{
    if (!count)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess)
    {
        *count = 0;
        return hip_fail(nullptr, e, "hipGetDeviceCount");
    }
    return 0;
}

const char *cwf_hip_last_error(const cwf_hip_system *h) { return h ? h->err.c_str() : g_err.c_str(); }
const char *cwf_hip_last_context(const cwf_hip_system *h) { return h ? h->ctx.c_str() : g_ctx.c_str(); }

void cwf_hip_system_destroy(cwf_hip_system *h)
{
    if (!h)
        return;
    (void)hipSetDevice(h->device);
    if (h->stream)
        (void)hipStreamSynchronize(h->stream);
    if (h->comm && h->comm->kind == 0)  // give the LOCAL communicator's stream back
    {
        h->comm->members[h->rank] = nullptr;
        h->stream = h->own_stream;
    }
    for (void *p : h->owned)
        (void)hipFree(p);
    if (h->hist)
        (void)hipFree(h->hist);
    if (h->ctl_host)
        (void)hipHostFree(h->ctl_host);
    for (hipEvent_t e : h->ev)
        (void)hipEventDestroy(e);
    if (h->stream)
        (void)hipStreamDestroy(h->stream);
    delete h;
}

int cwf_hip_system_create(const cwf_system_desc *d, int device, cwf_hip_system **out)
{
    if (!d || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    const uint64_t N = d->node_count, E = d->element_count;
    // validate_system (pcg.cpp:82-139)
    if (d->dof_count != N * 3)
        return set_error(nullptr, CWF_ERR_SIZE, "dof count mismatch (expected node_count * 3)",
                         "node_count=" + std::to_string(N) + "\ndof_count=" + std::to_string(d->dof_count));
    if (d->material_count == 0 || !d->material_stiffness)
        return set_error(nullptr, CWF_ERR_MATERIALS, "materials table is empty");
    if (d->reduction_block == 0)
        return set_error(nullptr, CWF_ERR_REDUCTION, "reduction block must be >= 1", "reduction_block=0");
    if (d->reduction_partials == 0)
        return set_error(nullptr, CWF_ERR_REDUCTION, "reduction partial count must be >= 1", "reduction_partials=0");
    if ((E && (!d->element_connectivity || !d->element_gradients || !d->element_volume ||
               !d->element_material_index)) ||
        (N && (!d->lumped_mass || !d->bc_mask)))
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null system array");
    if (N * 3 >= (1ull << 32) || E >= (1ull << 30))
        return set_error(nullptr, CWF_ERR_UNSUPPORTED, "mesh too large for one handle (shard it)",
                         "nodes=" + std::to_string(N) + "\nelements=" + std::to_string(E));
    // hex8: all 8 connectivity slots used; tet4 pads slots 4..7 with UINT32_MAX
    const bool hex = E && d->element_connectivity[4] != 0xFFFFFFFFu;
    const int K = hex ? 8 : 4;
    if (hex && d->mode != CWF_MODE_FAST)
        return set_error(nullptr, CWF_ERR_UNSUPPORTED, "hex8 elements run in CWF_MODE_FAST only",
                         "the reference has no hex8 arithmetic to reproduce (preprocess.cpp:326-330)");
    if (hex && !d->node_coords)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "hex8 systems need node_coords");
    for (uint64_t e = 0; e < E; ++e)
    {
        if (d->element_material_index[e] >= d->material_count)
            return set_error(nullptr, CWF_ERR_MATERIAL_RANGE, "element references material out of range",
                             "element=" + std::to_string(e) +
                                 "\nmaterial_index=" + std::to_string(d->element_material_index[e]));
        if ((d->element_connectivity[e * 8 + 4] != 0xFFFFFFFFu) != hex)
            return set_error(nullptr, CWF_ERR_UNSUPPORTED, "mixed tet4/hex8 meshes are not supported",
                             "element=" + std::to_string(e));
        for (int a = 0; a < K; ++a)
            if (d->element_connectivity[e * 8 + a] >= N)
                return set_error(nullptr, CWF_ERR_NODE_RANGE, "element connectivity references node out of range",
                                 "element=" + std::to_string(e) +
                                     "\nnode=" + std::to_string(d->element_connectivity[e * 8 + a]));
    }
    // FAST handles renumber their nodes along a Morton curve (cwf_hip.h CWF_DESC_KEEP_NODE_ORDER): the
    // rest of create then sees a desc in internal order; perm converts at the boundary
    cwf_system_desc rd{};
    std::vector<uint32_t> r_perm, r_conn, r_mask;
    std::vector<float> r_mass;
    std::vector<double> r_coords;
    const char *rn = knob("CWF_RENUMBER");
    const bool may_renumber = d->mode == CWF_MODE_FAST && E && N && d->node_coords &&
                              !(d->reserved & CWF_DESC_KEEP_NODE_ORDER) && !(rn && rn[0] == '0');
    // structured Kuhn block (lattice.cpp): the FAST operator is the node-pair stencil of the one shared cell
    // stiffness (k_keff_lattice). Its nodes stay in the caller's order when that is lexicographic within planes
    // (a shard's local order too); otherwise a handle that may renumber takes the lexicographic order.
    Lattice lat;
    bool is_lat = false;
    {
        const char *lv = knob("CWF_LATTICE");
        if (d->mode == CWF_MODE_FAST && E && N && N < 0x15555555ull && d->node_coords && !(lv && lv[0] == '0'))
        {
            std::string why;
            try
            {
                is_lat = detect_lattice(d, may_renumber, lat, &why);
            }
            catch (const std::bad_alloc &)
            {
                return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
            }
            if (knob("CWF_VERBOSE"))
                fprintf(stderr, "[cwf] lattice: %s (%u x %u x %u nodes%s)\n", is_lat ? "yes" : why.c_str(), lat.nx,
                        lat.ny, lat.nz, is_lat && !lat.perm.empty() ? ", renumbered" : "");
        }
    }
    const bool renumber = may_renumber && (!is_lat || !lat.perm.empty());
    // FAST recomputes tet geometry from node coordinates when they reproduce the desc's gradients (GEO); only
    // then can the tets group into fans (the groups kernel has no gradient stream). Node renumbering does not
    // change it, so it is decided once, on the caller's desc.
    const char *ge = knob("CWF_GEO");
    const bool geo_ok = E && N && d->node_coords && !(ge && ge[0] == '0') &&
                        (d->element_connectivity[4] != 0xFFFFFFFFu || geometry_matches(d));
    if (renumber)
    {
        const auto apply_perm = [&]() {
            std::vector<uint32_t> inv(N);
            for (uint64_t i = 0; i < N; ++i)
                inv[r_perm[i]] = (uint32_t)i;
            r_conn.assign(d->element_connectivity, d->element_connectivity + 8 * E);
            for (auto &c : r_conn)
                if (c != 0xFFFFFFFFu)
                    c = inv[c];
            r_mass.resize(N);
            r_mask.resize(N);
            r_coords.resize(3 * N);
            for (uint64_t i = 0; i < N; ++i)
            {
                const uint64_t n = r_perm[i];
                r_mass[i] = d->lumped_mass[n];
                r_mask[i] = d->bc_mask[n];
                for (int k = 0; k < 3; ++k)
                    r_coords[3 * i + k] = d->node_coords[3 * n + k];
            }
        };
        try
        {
            if (is_lat)  // lexicographic lattice order (lattice.cpp)
            {
                r_perm.swap(lat.perm);
                apply_perm();
            }
            else
            {
            r_perm = morton_node_order(d->node_coords, N);
            apply_perm();
            // fan-group and hex8 meshes: renumber again by (owner tile, Morton) so every tile's owned nodes are one
            // contiguous id range (whole-line owner p / partial stores, coalesced owned gathers). The groups
            // and tiles are built from coordinates and tet order only, so the rebuild after this renumbering
            // gives the same partition.
            if (hex || (d->material_count <= 16 && groups_enabled() && geo_ok))
            {
                cwf_system_desc md = *d;
                md.element_connectivity = r_conn.data();
                md.lumped_mass = r_mass.data();
                md.bc_mask = r_mask.data();
                md.node_coords = r_coords.data();
                std::vector<uint32_t> own;
                if (hex)  // the hex tiles (tiles.cpp, 8 corners): the same owner = first tile of the node
                {
                    HostTiles ht;
                    build_tiles(&md, ht, 2u * hex_tile_lanes(E), hex_tile_lanes(E), 8);
                    own.assign(N, 0xFFFFFFFFu);
                    for (uint32_t tl = 0; tl < ht.ntiles; ++tl)
                        for (uint32_t q = ht.tile_node_off[tl]; q < ht.tile_node_off[tl + 1]; ++q)
                            if (ht.tile_nodes[q] & 0x80000000u)
                                own[ht.tile_nodes[q] & 0x7fffffffu] = tl;
                }
                else
                {
                    GroupTiles gt;
                    const uint32_t gnt = group_lanes(E);
                    if (build_group_tiles(&md, gt, gnt, 2 * gnt, kGroupSlotsPerLane * gnt, false) == 0 &&
                        gt.tets_per_group >= 3.0)
                    {
                        own.assign(N, 0xFFFFFFFFu);
                        for (uint32_t tl = 0; tl < gt.ntiles; ++tl)
                            for (uint32_t q = gt.hdr[tl].z; q < gt.hdr[tl].z + gt.hdr[tl].w; ++q)
                                if (gt.tile_nodes[q] & 0x80000000u)
                                    own[gt.tile_nodes[q] & 0x7fffffffu] = tl;
                    }
                }
                if (!own.empty())
                {
                    std::vector<uint32_t> order(N);
                    std::iota(order.begin(), order.end(), 0u);
                    std::stable_sort(order.begin(), order.end(),
                                     [&](uint32_t a, uint32_t b) { return own[a] < own[b]; });
                    std::vector<uint32_t> p2(N);
                    for (uint64_t i = 0; i < N; ++i)
                        p2[i] = r_perm[order[i]];
                    r_perm.swap(p2);
                    apply_perm();
                }
            }
            }  // !is_lat
        }
        catch (const std::bad_alloc &)
        {
            return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
        }
        rd = *d;
        rd.element_connectivity = r_conn.data();
        rd.lumped_mass = r_mass.data();
        rd.bc_mask = r_mask.data();
        rd.node_coords = r_coords.data();
        rd.adjacency_offsets = nullptr;  // rebuilt in internal order (ascending element per node)
        rd.adjacency_elements = nullptr;
        rd.adjacency_local = nullptr;
        d = &rd;
    }
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess)
        return hip_fail(nullptr, he, "hipSetDevice");

    cwf_hip_system *h = new (std::nothrow) cwf_hip_system();
    if (!h)
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    auto bail = [&](int st) {
        std::string m = h->err, c = h->ctx;
        cwf_hip_system_destroy(h);
        set_error(nullptr, st, m, c);
        return st;
    };
    h->device = device;
    h->mode = d->mode == CWF_MODE_FAST ? CWF_MODE_FAST : CWF_MODE_PARITY;
    h->reduction_block = d->reduction_block;
    h->reduction_partials = d->reduction_partials;
    if ((he = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess)
        return bail(hip_fail(h, he, "hipStreamCreate"));
    if ((he = hipHostMalloc(reinterpret_cast<void **>(&h->ctl_host), sizeof(Ctl), hipHostMallocDefault)) !=
        hipSuccess)
        return bail(hip_fail(h, he, "hipHostMalloc"));

    DevSys &s = h->ds;
    s.N = (uint32_t)N;
    s.Nown = (uint32_t)N;
    s.E = (uint32_t)E;
    s.D = (uint32_t)(3 * N);
    s.M = (uint32_t)d->material_count;
    s.sK = d->stiffness_scale;
    s.sM = d->mass_factor;
    s.iso = 1;
    for (uint64_t m = 0; m < d->material_count; ++m)
        s.iso &= iso_pattern(d->material_stiffness + 36 * m) ? 1 : 0;
    if (s.M == 1)  // table order of the FAST kernels (dsrc): iso = 3x3 normal block + 3 shear diagonals
        for (int t = 0; t < (s.iso ? 12 : 36); ++t)
            s.d1[t] = (float)d->material_stiffness[s.iso ? (t < 9 ? (t / 3) * 6 + (t % 3) : (t - 6) * 7) : t];
    s.hex = hex ? 1 : 0;

    // element records (64 B/tet; the PARITY kernels only, so none for hex8)
    if (!hex)
    {
        std::vector<uint32_t> rec;
        try
        {
            rec.resize(E * 16);
        }
        catch (const std::bad_alloc &)
        {
            return bail(set_error(h, CWF_ERR_ALLOC, "host allocation failed"));
        }
        for (uint64_t e = 0; e < E; ++e)
        {
            uint32_t *r = rec.data() + e * 16;
            for (int a = 0; a < 4; ++a)
                r[a] = d->element_connectivity[e * 8 + a];
            std::memcpy(r + 4, d->element_gradients + e * 24, 12 * sizeof(float));
        }
        uint4 *erec = nullptr;
        if (int st = upload(h, &erec, reinterpret_cast<const uint4 *>(rec.data()), E * 4))
            return bail(st);
        s.erec = erec;
    }
    {
        float *vol;
        uint32_t *mat;
        double *dm;
        float *mass;
        uint32_t *mask;
        if (int st = upload(h, &vol, d->element_volume, E))
            return bail(st);
        if (int st = upload(h, &mat, d->element_material_index, E))
            return bail(st);
        if (int st = upload(h, &dm, d->material_stiffness, 36 * d->material_count))
            return bail(st);
        if (int st = upload(h, &mass, d->lumped_mass, N))
            return bail(st);
        if (int st = upload(h, &mask, d->bc_mask, N))
            return bail(st);
        s.vol = vol;
        s.mat = mat;
        s.dmat = dm;
        s.mass = mass;
        s.mask = mask;
    }
    // node -> element CSR, ascending element per node (preprocess.cpp:380-403)
    {
        std::vector<uint32_t> off(N + 1, 0), inc;
        const uint32_t sh = hex ? 3u : 2u;  // inc = element << sh | corner
        try
        {
            inc.resize(E * K);
        }
        catch (const std::bad_alloc &)
        {
            return bail(set_error(h, CWF_ERR_ALLOC, "host allocation failed"));
        }
        if (d->adjacency_offsets && d->adjacency_elements && d->adjacency_local)
        {
            std::memcpy(off.data(), d->adjacency_offsets, (N + 1) * sizeof(uint32_t));
            if (off[N] != E * K || off[0] != 0)
                return bail(set_error(h, CWF_ERR_SIZE, "adjacency size mismatch",
                                      "expected=" + std::to_string(E * K) + "\nactual=" + std::to_string(off[N])));
            // the caller's CSR must be exactly the node -> (element, corner) incidences in ascending element order
            // (preprocess.cpp:389-400): every later pass indexes through it without bounds checks
            for (uint64_t n = 0; n < N; ++n)
            {
                if (off[n] > off[n + 1])
                    return bail(set_error(h, CWF_ERR_ARGUMENT, "adjacency offsets must be non-decreasing",
                                          "node=" + std::to_string(n)));
                for (uint32_t j = off[n]; j < off[n + 1]; ++j)
                {
                    const uint32_t e = d->adjacency_elements[j], a = d->adjacency_local[j];
                    if (e >= E || a >= (uint32_t)K || d->element_connectivity[8ull * e + a] != n ||
                        (j > off[n] && d->adjacency_elements[j - 1] >= e))
                        return bail(set_error(h, CWF_ERR_ARGUMENT, "adjacency does not match the connectivity",
                                              "node=" + std::to_string(n) + "\nentry=" + std::to_string(j)));
                    inc[j] = (e << sh) | a;
                }
            }
        }
        else
        {
            std::vector<uint32_t> cnt(N, 0);
            for (uint64_t e = 0; e < E; ++e)
                for (int a = 0; a < K; ++a)
                    ++cnt[d->element_connectivity[e * 8 + a]];
            uint32_t acc = 0;
            for (uint64_t n = 0; n < N; ++n)
            {
                off[n] = acc;
                acc += cnt[n];
                cnt[n] = 0;
            }
            off[N] = acc;
            for (uint64_t e = 0; e < E; ++e)
                for (int a = 0; a < K; ++a)
                {
                    const uint32_t n = d->element_connectivity[e * 8 + a];
                    inc[off[n] + cnt[n]++] = ((uint32_t)e << sh) | (uint32_t)a;
                }
        }
        uint32_t *doff, *dinc;
        if (int st = upload(h, &doff, off.data(), N + 1))
            return bail(st);
        if (int st = upload(h, &dinc, inc.data(), E * K))
            return bail(st);
        s.off = doff;
        s.inc = dinc;
    }
    // structured Kuhn block: the stencil blocks, the plane table and one row value per node (lattice.inc)
    if (E && is_lat)
    {
        DevTiles &t = s.t;
        std::vector<uint32_t> npo(N + 1);
        for (uint64_t n = 0; n <= N; ++n)
            npo[n] = (uint32_t)n | (n < N ? (d->bc_mask[n] & 7u) << 29 : 0u);
        uint32_t *dpl, *dnpo;
        float *dcf, *part;
        if (int st = upload(h, &dpl, lat.plane.data(), lat.plane.size()))
            return bail(st);
        // the device copy's stencil blocks are stored row-pair interleaved for the packed rows of k_keff_lattice:
        // per offset {S00 S10 S01 S11 S02 S12 S20 S21 S22}; the cell-pair blocks after them keep row-major order
        std::vector<float> cdev(lat.coef, lat.coef + (lat.hex ? kLatHexCoef : kLatCoef));
        for (int o = 0; o < (lat.hex ? kLatHexOffsets : kLatOffsets); ++o)
            for (int c = 0; c < 3; ++c)
            {
                cdev[9 * o + 2 * c] = lat.coef[9 * o + c];
                cdev[9 * o + 2 * c + 1] = lat.coef[9 * o + 3 + c];
                cdev[9 * o + 6 + c] = lat.coef[9 * o + 6 + c];
            }
        if (int st = upload(h, &dcf, cdev.data(), (uint64_t)cdev.size()))
            return bail(st);
        if (int st = upload(h, &dnpo, npo.data(), npo.size()))
            return bail(st);
        if (int st = dalloc(h, &part, 3 * (N + 2)))  // + 2 padding slots (update pass)
            return bail(st);
        t.lat = 1;
        t.lnx = lat.nx;
        t.lny = lat.ny;
        t.lnz = lat.nz;
        t.lk0 = 0;
        t.lk1 = lat.nz;
        t.lplane = dpl;
        t.lpstride = lat.nx * lat.ny;
        for (uint32_t k = 0; k < lat.nz; ++k)
            if (lat.plane[k] != k * t.lpstride)
                t.lpstride = 0;
        t.lcoef = dcf;
        t.lsym = lat.sym ? 1 : 0;
        t.lhex = lat.hex ? 1 : 0;
        t.node_part_off = dnpo;
        t.off_mask = 1;
        t.node_major = 1;
        t.part = part;
        t.E = (uint32_t)E;
        t.geo = 1;
        t.total_tile_nodes = (uint32_t)N;
        t.wt_part = 0;
        // per-class preconditioner (the update pass reads one byte per node instead of the 16-B record and the
        // partial-run bounds) when the lumped mass is a function of the boundary type
        {
            std::vector<uint8_t> cls(N);
            std::vector<uint32_t> rep(kLatClasses, 0xFFFFFFFFu);
            std::vector<float> tmass(27, 0.f);
            std::vector<uint8_t> tseen(27, 0);
            bool uniform = true;
            for (uint32_t k = 0; k < lat.nz && uniform; ++k)
                for (uint32_t j = 0; j < lat.ny; ++j)
                    for (uint32_t i = 0; i < lat.nx; ++i)
                    {
                        const uint32_t n = lat.plane[k] + j * lat.nx + i;
                        const auto side = [](uint32_t a, uint32_t na) { return a == 0 ? 0u : a + 1 == na ? 2u : 1u; };
                        const uint32_t ty = side(i, lat.nx) + 3 * side(j, lat.ny) + 9 * side(k, lat.nz);
                        const uint32_t c = ty << 3 | (d->bc_mask[n] & 7u);
                        cls[n] = (uint8_t)c;
                        if (rep[c] == 0xFFFFFFFFu || n < rep[c])
                            rep[c] = n;
                        if (!tseen[ty])
                        {
                            tseen[ty] = 1;
                            tmass[ty] = d->lumped_mass[n];
                        }
                        else if (std::memcmp(&tmass[ty], &d->lumped_mass[n], sizeof(float)) != 0)
                            uniform = false;
                    }
            if (uniform && tseen[13])  // type 13: inside along x, y and z (the bricks' nodes)
            {
                t.lmu = 1;
                t.lmass = tmass[13];
                // z from r in the K_eff pass, no z store in the update pass (attach turns it off, comm.cpp): from
                // 2M nodes, where the iteration's vectors leave the 256 MB MALL and the 12 B per node the update
                // pass no longer writes are HBM bytes (C3 +4-5% PCG it/s); on C2 the K_eff pass's class-table fill
                // and the 3 x 3 products per halo entry sit on its latency-bound critical path (-8%), same box
                const char *zr = knob("CWF_LAT_ZR");
                t.lzr = zr ? (zr[0] == '1' ? 1 : 0) : (N >= (1ull << 21) ? 1 : 0);
            }
            if (uniform)
            {
                uint8_t *dcls;
                uint32_t *drep;
                uint4 *dci6;
                float *dci9;
                if (int st = upload(h, &dcls, cls.data(), N))
                    return bail(st);
                if (int st = upload(h, &drep, rep.data(), kLatClasses))
                    return bail(st);
                if (int st = dalloc(h, &dci6, kLatClasses))
                    return bail(st);
                if (int st = dalloc(h, &dci9, 9 * kLatClasses))
                    return bail(st);
                float4 *dcz;
                if (int st = dalloc(h, &dcz, 2 * kLatClasses))
                    return bail(st);
                HIPTRY(h, hipMemset(dcz, 0, 2 * kLatClasses * sizeof(float4)));
                // classes without a node keep zero inverses (k_lat_class_inverse fills only represented ones; halo
                // lanes of the z-from-r and single-launch passes may read any class)
                HIPTRY(h, hipMemset(dci6, 0, kLatClasses * sizeof(uint4)));
                HIPTRY(h, hipMemset(dci9, 0, 9 * kLatClasses * sizeof(float)));
                t.lcls = dcls;
                t.lrep = drep;
                t.lcinv6 = dci6;
                t.lcinv9 = dci9;
                t.lcz = dcz;
            }
        }
        h->lat_plane.swap(lat.plane);
        lattice_plan(t);
    }
    // FAST-mode element tiles (tiles.cpp)
    else if (E)
    {
        HostTiles ht;
        DevTiles &t = s.t;
        // GEO: stream 8-B corner ids + tile-node coordinates and recompute gradients/volume on the fly,
        // when the desc carries coordinates that reproduce its gradients (CWF_GEO=0 forces the records)
        t.geo = hex || geo_ok ? 1 : 0;
        if (hex)  // k_keff_hex_tiles: hex_nt lanes, one hex and two tile nodes per lane, push fold
        {
            t.hex = 1;
            t.hex_nt = (int)hex_tile_lanes(E);
            t.wt_part = 0;
            t.push = 1;
        }
        else
        {
            const char *pp = knob("CWF_TILE_PIPE");  // diagnostic: 0 = the one-tile-per-workgroup kernel
            t.pipe = t.geo && !(pp && pp[0] == '0') ? 1 : 0;
        }
        // fan groups (groups.cpp, k_keff_groups_pipe): the default FAST tet path when the mesh groups into
        // fans of >= 3 tets on average and has <= 16 materials (D from kernel arguments or an LDS table);
        // CWF_GROUPS=0: the per-tet tiles below
        bool grouped = false;
        {
            if (!hex && t.pipe && groups_enabled() && d->material_count <= 16)
            {
                GroupTiles gt;
                int gst = -1;
                const uint32_t gnt = group_lanes(E);
                try
                {
                    gst = build_group_tiles(d, gt, gnt, 2 * gnt, kGroupSlotsPerLane * gnt);
                }
                catch (const std::bad_alloc &)
                {
                    return bail(set_error(h, CWF_ERR_ALLOC, "host allocation failed"));
                }
                if (knob("CWF_VERBOSE"))
                    fprintf(stderr, "[cwf] fan groups: status %d, %u groups (%.2f tets each), %u tiles, %zu tile nodes "
                                    "(%.3f per node), max %u nodes / %u slots per tile\n",
                            gst, gt.ngroups, gt.tets_per_group, gt.ntiles, gt.tile_nodes.size(),
                            N ? (double)gt.tile_nodes.size() / (double)N : 0.0, gt.max_tile_nodes, gt.max_tile_slots);
                if (gst == 0 && gt.tets_per_group >= 3.0)
                {
                    const size_t T = gt.tile_nodes.size();
                    std::vector<uint2> tnode(T);
                    for (size_t q = 0; q < T; ++q)
                        tnode[q] = uint2{gt.tile_nodes[q], gt.run[q]};
                    if (ht_off_mask_ok(gt.node_part_off))
                    {
                        for (uint64_t n = 0; n < N; ++n)
                            gt.node_part_off[n] |= (d->bc_mask[n] & 7u) << 29;
                        t.off_mask = 1;
                    }
                    uint4 *ga, *dh;
                    uint2 *dtn;
                    uint32_t *npo, *tsl;
                    float *tc, *part;
                    if (int st = upload(h, &ga, gt.grec.data(), gt.grec.size()))
                        return bail(st);
                    if (int st = upload(h, &dh, gt.hdr.data(), gt.hdr.size()))
                        return bail(st);
                    if (int st = upload(h, &dtn, tnode.data(), T))
                        return bail(st);
                    if (int st = upload(h, &npo, gt.node_part_off.data(), gt.node_part_off.size()))
                        return bail(st);
                    if (int st = upload(h, &tsl, gt.tile_slot.data(), T))
                        return bail(st);
                    if (int st = dalloc(h, &tc, 3 * T))
                        return bail(st);
                    for (int q = 0; q < 3; ++q)
                        HIPTRY(h, hipMemcpy(tc + q * T, gt.tcoord[q].data(), T * sizeof(float), hipMemcpyHostToDevice));
                    if (int st = dalloc(h, &part, 3 * (T + 2)))  // + 2 padding slots (update pass)
                        return bail(st);
                    t.grp = 1;
                    t.grec = ga;
                    t.hdr = dh;
                    t.tnode = dtn;
                    t.tslot = tsl;
                    t.tcoord = tc;
                    t.node_part_off = npo;
                    t.part = part;
                    t.node_major = 1;
                    t.push = 1;
                    t.pipe = 1;
                    t.pipe_nt = (int)gnt;
                    t.wt_part = E < 4000000ull ? 1 : 0;  // write-through tile partials below 4M tets
                    t.ntiles = gt.ntiles;
                    t.ngroups = gt.ngroups;
                    t.max_tile_nodes = gt.max_tile_nodes;
                    t.total_tile_nodes = (uint32_t)T;
                    t.E = (uint32_t)E;
                    t.pipe_grid = fast_pipe_grid(s);
                    grouped = true;
                }
            }
        }
        if (!grouped)
        {
        try
        {
            // pipelined tiles: 256-thread workgroups over 512-element tiles, or 128 over 256 (128 below 4M
            // tets: the meshes whose 512-element tiles would give each resident workgroup < 8 tiles)
            if (t.pipe)
            {
                t.pipe_nt = E < 4000000ull ? 128 : 256;
                t.push = 1;  // the pipelined kernel folds pushed forces (epos), not local-CSR entries
            }
            if (hex)
                build_tiles(d, ht, 2u * (uint32_t)t.hex_nt, (uint32_t)t.hex_nt, 8);
            else
                build_tiles(d, ht, t.pipe ? (uint32_t)t.pipe_nt : (uint32_t)kMaxTileNodes,
                            t.pipe ? 2u * (uint32_t)t.pipe_nt : (uint32_t)kTileElems);
        }
        catch (const std::bad_alloc &)
        {
            return bail(set_error(h, CWF_ERR_ALLOC, "host allocation failed"));
        }
        if (knob("CWF_VERBOSE"))
            fprintf(stderr, "[cwf] tiles: %u tiles, %zu tile nodes (%.3f per node), max %u nodes/tile, %s records\n",
                    ht.ntiles, ht.tile_nodes.size(), N ? (double)ht.tile_nodes.size() / (double)N : 0.0,
                    ht.max_tile_nodes, t.geo ? "8-B geometric" : "48-B gradient");
        if (t.geo)
        {
            uint2 *eid = nullptr;
            float *tc;
            if (hex)
            {
                uint4 *e8;
                if (int st = upload(h, &e8, ht.eid8.data(), E))
                    return bail(st);
                t.eid8 = e8;
            }
            else if (int st = upload(h, &eid, ht.eid.data(), E))
                return bail(st);
            const size_t T3 = ht.tile_nodes.size();
            if (int st = dalloc(h, &tc, 3 * T3))
                return bail(st);
            for (int q = 0; q < 3; ++q)
                HIPTRY(h, hipMemcpy(tc + q * T3, ht.tcoord[q].data(), T3 * sizeof(float), hipMemcpyHostToDevice));
            t.eid = eid;
            t.tcoord = tc;
        }
        else
        {
            uint4 *planes;
            if (int st = dalloc(h, &planes, 3 * E))
                return bail(st);
            for (int q = 0; q < 3; ++q)
                HIPTRY(h, hipMemcpy(planes + q * E, ht.planes[q].data(), E * sizeof(uint4), hipMemcpyHostToDevice));
            t.planes = planes;
        }
        if (!ht.mat.empty())
        {
            uint32_t *tm;
            if (int st = upload(h, &tm, ht.mat.data(), E))
                return bail(st);
            t.mat = tm;
        }
        // per-tile header (one scalar dwordx4 load) and 8-B tile-node records {node|owner, csr range};
        // partials are tile-major (a tile's block is one contiguous store) and the update pass gathers a
        // node's slots through part_slot
        std::vector<uint4> hdr(ht.ntiles);
        std::vector<uint2> tnode(ht.tile_nodes.size());
        // tet push fold: every node's run of pushed forces starts on an even slot (the fold reads two
        // {f_x, f_y} pairs with one ds_read_b128 and two f_z with one ds_read_b64) and gets 2 (mod 4)
        // slots, so the half-start offsets of side-by-side fold lanes are odd multiples apart and spread
        // over the LDS banks (a uniform stride such as the 24 tets of an interior Kuhn node would put all
        // lanes on a few banks). A tile whose pads would overflow the kernel's slot budget (4 te + 2 nt)
        // only rounds to even. The element corners' positions (epos) shift with their node's run.
        const bool pad_runs = t.push && !hex;
        const uint32_t slot_budget = 8u * (uint32_t)t.pipe_nt + 2u * (uint32_t)t.pipe_nt;
        std::vector<uint32_t> shift;
        for (uint32_t k = 0; k < ht.ntiles; ++k)
        {
            const uint32_t e0 = ht.tile_elem_off[k], nb = ht.tile_node_off[k], nb1 = ht.tile_node_off[k + 1];
            hdr[k] = uint4{e0, ht.tile_elem_off[k + 1] - e0, nb, nb1 - nb};
            if (hex && !ht.tile_affine.empty() && ht.tile_affine[k])
                hdr[k].x |= 0x80000000u;  // hex8 tile of parallelepipeds (k_keff_hex_tiles: constant J)
            shift.assign(nb1 - nb, 0);
            for (int spread = 1; spread >= 0; --spread)
            {
                uint32_t padded = 0;
                for (uint32_t q = nb; q < nb1; ++q)
                {
                    const uint32_t a = ht.csr_off[q] - (uint32_t)K * e0, b = ht.csr_off[q + 1] - (uint32_t)K * e0;
                    const uint32_t start = pad_runs ? padded : a;
                    tnode[q] = uint2{ht.tile_nodes[q], start | ((start + b - a) << 16)};
                    shift[q - nb] = start - a;
                    uint32_t len = (b - a + 1u) & ~1u;  // even
                    if (spread && (len / 2u) % 2u == 0u)
                        len += 2u;  // 2 (mod 4)
                    padded = start + len;
                }
                if (!pad_runs || padded <= slot_budget)
                    break;
            }
            if (pad_runs)
                for (uint32_t j = e0; j < ht.tile_elem_off[k + 1]; ++j)
                {
                    const uint2 id = ht.eid[j];
                    uint2 &ep = ht.epos[j];
                    const uint32_t li[4] = {id.x & 0xffffu, id.x >> 16, id.y & 0xffffu, id.y >> 16};
                    const uint32_t p[4] = {(ep.x & 0xffffu) + shift[li[0]], (ep.x >> 16) + shift[li[1]],
                                           (ep.y & 0xffffu) + shift[li[2]], (ep.y >> 16) + shift[li[3]]};
                    ep = uint2{p[0] | (p[1] << 16), p[2] | (p[3] << 16)};
                }
        }
        uint4 *dh;
        uint2 *dtn;
        uint32_t *npo;
        uint16_t *ce;
        float *part;
        if (int st = upload(h, &dh, hdr.data(), hdr.size()))
            return bail(st);
        if (int st = upload(h, &dtn, tnode.data(), tnode.size()))
            return bail(st);
        ht.csr_ent.resize(ht.csr_ent.size() + 8, 0);  // the pipelined kernel reads a tile's entries as 16-B words
        ce = nullptr;
        if (!t.push)  // PUSH streams the per-element positions (epos) instead
            if (int st = upload(h, &ce, ht.csr_ent.data(), ht.csr_ent.size()))
                return bail(st);
        // the update pass reads each node's partial range anyway: the Dirichlet mask rides in its top bits
        // (one 4-B stream less per PCG iteration) when the offsets leave them free
        if (ht.node_part_off.back() <= kPartOffBits)
        {
            for (uint64_t n = 0; n < N; ++n)
                ht.node_part_off[n] |= (d->bc_mask[n] & 7u) << 29;
            t.off_mask = 1;
        }
        if (int st = upload(h, &npo, ht.node_part_off.data(), ht.node_part_off.size()))
            return bail(st);
        uint32_t *ps;
        if (int st = upload(h, &ps, ht.node_part_slot.data(), ht.node_part_slot.size()))
            return bail(st);
        t.part_slot = ps;
        if (t.push && hex)
        {
            uint4 *ep;
            if (int st = upload(h, &ep, ht.epos8.data(), ht.epos8.size()))
                return bail(st);
            t.epos8 = ep;
        }
        else if (t.push)
        {
            uint2 *ep;
            if (int st = upload(h, &ep, ht.epos.data(), ht.epos.size()))
                return bail(st);
            t.epos = ep;
        }
        if (t.pipe || t.hex)
        {
            uint32_t *tsl;
            if (int st = upload(h, &tsl, ht.tile_slot.data(), ht.tile_slot.size()))
                return bail(st);
            t.tslot = tsl;
            t.node_major = 1;
        }
        if (int st = dalloc(h, &part, 3 * (ht.tile_nodes.size() + 2)))  // + 2 padding slots (update pass)
            return bail(st);
        t.ntiles = ht.ntiles;
        t.hex_all_affine = hex && !ht.tile_affine.empty() &&
                           std::all_of(ht.tile_affine.begin(), ht.tile_affine.end(), [](uint8_t a) { return a != 0; });
        t.max_tile_nodes = ht.max_tile_nodes;
        t.total_tile_nodes = (uint32_t)ht.tile_nodes.size();
        t.E = (uint32_t)E;
        t.hdr = dh;
        t.tnode = dtn;
        t.csr_ent = ce;
        t.node_part_off = npo;
        t.part = part;
        if (t.pipe || t.hex)
            t.pipe_grid = fast_pipe_grid(s);
        }  // !grouped
    }
    if (hex)  // the hex block-Jacobi setup integrates from the global corners (fp64)
    {
        uint32_t *hc;
        double *hx;
        std::vector<uint32_t> conn(E * 8);
        std::memcpy(conn.data(), d->element_connectivity, E * 8 * sizeof(uint32_t));
        if (int st = upload(h, &hc, conn.data(), E * 8))
            return bail(st);
        if (int st = upload(h, &hx, d->node_coords, 3 * N))
            return bail(st);
        float *hg;
        if (int st = upload(h, &hg, d->element_gradients, 24 * E))
            return bail(st);
        s.hconn = hc;
        s.hcoord = hx;
        s.hgrad = hg;
    }
    // solver scratch
    const uint64_t D = 3 * N;
    for (float **v : {&h->x, &h->r, &h->p, &h->p2, &h->p3, &h->p4, &h->z, &h->Ap, &h->rhs, &h->tmp})
        if (int st = dalloc(h, v, D))
            return bail(st);
    if (s.t.lat && s.t.lcls)  // the fused lattice iteration's second r / Ap and its shares (lattice_fused.inc)
    {
        if (int st = dalloc(h, &h->r2, D))
            return bail(st);
        if (int st = dalloc(h, &h->ap2, D))
            return bail(st);
        if (int st = dalloc(h, &h->fsh, 2ull * 5 * std::max<uint32_t>(s.t.lnwork, 1u)))
            return bail(st);
        if (int st = dalloc(h, &h->g_fsh, 8))  // one rank until attach (comm.cpp grows it to [nranks][8])
            return bail(st);
    }
    if (int st = dalloc(h, &h->inv, 9 * N))
        return bail(st);
    if (int st = dalloc(h, &h->inv6, 4 * N))
        return bail(st);
    const uint64_t chunks = (D + d->reduction_block - 1) / d->reduction_block;
    h->part_cap = std::max<uint64_t>(
        {chunks, (uint64_t)fast_block_count(h), (uint64_t)fast_dot_blocks(s.D), (uint64_t)s.t.ntiles,
         (uint64_t)s.t.pipe_grid, 1});
    if (int st = dalloc(h, &h->part0, h->part_cap))
        return bail(st);
    if (int st = dalloc(h, &h->part1, h->part_cap))
        return bail(st);
    if (int st = dalloc(h, &h->part2, h->part_cap))
        return bail(st);
    if (int st = dalloc(h, &h->ctl, 1))
        return bail(st);
    if (int st = dalloc(h, &h->scal, 8))
        return bail(st);
    // folded per-rank scalars (one rank until cwf_hip_system_attach): p.Ap, {r.r, r.z}, {rhs.rhs, r0.r0}, r0.z0
    if (int st = dalloc(h, &h->g_pap, 6))
        return bail(st);
    h->g_rrz = h->g_pap + 1;
    h->g_init = h->g_rrz + 2;
    h->g_rz0 = h->g_init + 2;
    if (renumber)
    {
        if (int st = upload(h, &h->perm, r_perm.data(), N))
            return bail(st);
        if (int st = dalloc(h, &h->pbuf, 13 * N))
            return bail(st);
    }
    if (h->mode == CWF_MODE_PARITY)
        if (int st = parity_force_buffer(h))
            return bail(st);
    HIPTRY(h, hipMemset(h->x, 0, D * sizeof(float)));
    HIPTRY(h, hipMemset(h->ctl, 0, sizeof(Ctl)));
    HIPTRY(h, hipMemset(h->g_pap, 0, 6 * sizeof(double)));
    HIPTRY(h, hipDeviceSynchronize());
    *out = h;
    return 0;
}

int cwf_hip_system_set_scalars(cwf_hip_system *h, double stiffness_scale, double mass_factor)
{
    if (int st = check_ready(h))
        return st;
    h->ds.sK = stiffness_scale;
    h->ds.sM = mass_factor;
    return 0;
}

int cwf_hip_system_set_mode(cwf_hip_system *h, int mode)
{
    if (int st = check_ready(h))
        return st;
    if (h->ds.hex && mode != CWF_MODE_FAST)
        return set_error(h, CWF_ERR_UNSUPPORTED, "hex8 elements run in CWF_MODE_FAST only",
                         "the reference has no hex8 arithmetic to reproduce (preprocess.cpp:326-330)");
    if (h->perm && mode != CWF_MODE_FAST)
        return set_error(h, CWF_ERR_UNSUPPORTED, "a renumbered FAST handle cannot switch to CWF_MODE_PARITY",
                         "create the PARITY handle separately (or with CWF_DESC_KEEP_NODE_ORDER)");
    h->mode = mode == CWF_MODE_FAST ? CWF_MODE_FAST : CWF_MODE_PARITY;
    if (h->mode == CWF_MODE_PARITY)
        return parity_force_buffer(h);
    return 0;
}

int cwf_hip_system_set_timing(cwf_hip_system *h, int enabled)
{
    if (int st = check_ready(h))
        return st;
    h->timing = enabled > 0 ? enabled : 0;  // time every `enabled`-th PCG-loop K_eff launch
    h->keff_ms = 0.0;
    h->keff_count = 0;
    return 0;
}

int cwf_hip_system_timing(cwf_hip_system *h, double *keff_ms, uint64_t *keff_launches)
{
    if (int st = check_ready(h))
        return st;
    if (keff_ms)
        *keff_ms = h->keff_ms;
    if (keff_launches)
        *keff_launches = h->keff_count;
    h->keff_ms = 0.0;
    h->keff_count = 0;
    return 0;
}

int cwf_hip_keff_timed(cwf_hip_system *h, const float *x, float *y, int reps, double *avg_ms)
{
    if (int st = check_ready(h))
        return st;
    if (!x || !y || !avg_ms || reps <= 0)
        return set_error(h, CWF_ERR_ARGUMENT, "bad argument");
    hipEvent_t a, b;
    HIPTRY(h, hipEventCreate(&a));
    HIPTRY(h, hipEventCreate(&b));
    const char *dry = knob("CWF_TIMED_PCG");  // diagnostic: time the PCG-mode tiles kernel instead
    if (dry && h->mode == CWF_MODE_FAST && h->ds.iso)
    {
        Ctl c{};
        c.active = 1;
        c.beta = 0.5;
        c.rho2[0] = c.rho2[1] = 1.0;
        c.tol = 0.0;
        HIPTRY(h, hipMemcpyAsync(h->ctl, &c, sizeof c, hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipMemsetAsync(h->part1, 0, h->part_cap * sizeof(double), h->stream));
        HIPTRY(h, hipMemsetAsync(h->part2, 0, h->part_cap * sizeof(double), h->stream));
        fast_tiles_pcg_dry(h, (unsigned)atoi(dry), 5, h->stream);
    }
    HIPTRY(h, hipEventRecord(a, h->stream));
    for (int i = 0; i < reps; ++i)
    {
        if (dry && h->mode == CWF_MODE_FAST && h->ds.iso)
            fast_tiles_pcg_dry(h, (unsigned)atoi(dry), 1, h->stream);
        else if (h->mode == CWF_MODE_FAST)
            fast_keff(h, x, y, false, nullptr, h->part0, h->stream);
        else
            parity_keff(h, x, y, false, nullptr, h->stream);
    }
    HIPTRY(h, hipEventRecord(b, h->stream));
    HIPTRY(h, hipEventSynchronize(b));
    float ms = 0.f;
    HIPTRY(h, hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *avg_ms = (double)ms / reps;
    return 0;
}

int cwf_hip_bandwidth_probe(int device, uint64_t bytes, int reps, double *gbs)
{
    if (!gbs || bytes < 16 || reps < 1)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "bandwidth probe: bad arguments");
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess)
        return hip_fail(nullptr, e, "hipSetDevice");
    bytes &= ~(uint64_t)15;
    void *a = nullptr, *b = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float ms = 0.f;
    if ((e = hipMalloc(&a, bytes)) == hipSuccess && (e = hipMalloc(&b, bytes)) == hipSuccess &&
        (e = hipMemset(a, 0, bytes)) == hipSuccess && (e = hipEventCreate(&e0)) == hipSuccess &&
        (e = hipEventCreate(&e1)) == hipSuccess)
    {
        copy16(a, b, bytes, nullptr);  // warm
        (void)hipEventRecord(e0, nullptr);
        for (int r = 0; r < reps; ++r)
            copy16(a, b, bytes, nullptr);
        (void)hipEventRecord(e1, nullptr);
        e = hipEventSynchronize(e1);
        if (e == hipSuccess)
            e = hipEventElapsedTime(&ms, e0, e1);
    }
    if (e0)
        (void)hipEventDestroy(e0);
    if (e1)
        (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(b);
    if (e != hipSuccess)
        return hip_fail(nullptr, e, "bandwidth probe");
    *gbs = 2.0 * (double)bytes * reps / ((double)ms * 1e-3) / 1e9;  // read + write
    return 0;
}

int cwf_hip_system_memory(const cwf_hip_system *h, uint64_t *bytes)
{
    if (!h || !bytes)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *bytes = h->bytes;
    return 0;
}

int cwf_hip_system_keff_traffic(const cwf_hip_system *h, uint64_t *layout_bytes, uint64_t *reference_layout_bytes)
{
    if (!h || !layout_bytes || !reference_layout_bytes)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    const DevSys &s = h->ds;
    const uint64_t N = s.N, E = s.E, T = s.t.total_tile_nodes;
    *reference_layout_bytes = 32 * N + 72 * E;
    if (h->mode == CWF_MODE_FAST && s.t.ntiles)
    {
        // per tile: 16-B header; per tet: corner ids (8 B GEO, 48-B records otherwise) + 4 u16 local-CSR
        // entries or (PUSH) positions (+ material id when M > 1); per tile node: {node, csr range} 8 B, coordinates 12 B (GEO), the node-major slot 4 B
        // (pipelined / hex), partial written 12 B; per node: p_old and z read once (24 B) + mass 4 B + the new
        // p written by its owner slot (12 B, PCG mode: the launches bench.py times)
        // hex8: 16-B corner ids + 16-B positions per hex (no material stream for one material)
        // fan groups: 16-B group record (ids, push ranks, tet count, material) instead of the per-tet records
        const uint64_t rec = s.t.hex ? 32 : s.t.geo ? 16 : 56;
        if (s.t.lat && fast_fused(h) && resident_on(h))
        {  // the resident solve (resident.hip), per iteration: only what crosses a CU -- the halo records read, the
           // box-surface records and the shares written, the G x 5 shares read -- the vectors stay on chip
            *layout_bytes = resident_offchip_bytes(h);
            return 0;
        }
        if (s.t.lat && fast_fused(h) && h->fused_agreed != 0)  // the fused iteration (lattice_fused.inc): per owned node r_(j-1), Ap_(j-1),
        {                              // p_(j-1), the class byte and x read, r_j, p_j, Ap_j and x written; the mass
                                       // of the shell's nodes (the strict interior's is one value when lmu)
            *layout_bytes = (uint64_t)s.Nown * (4 * 12 + 1 + 4 * 12) + 4ull * (s.t.lmu ? s.t.lnshell : s.Nown);
            return 0;
        }
        if (s.t.lat)  // per owned node: z and p_old read, the new p and the row value written; the mass read
        {             // (only the shell's when the strict interior's is one value, lmu)
            *layout_bytes = (uint64_t)s.Nown * (12 + 12 + 12 + 12 + (s.t.lmu && s.t.lzr ? 1 : 0)) +
                            4ull * (s.t.lmu ? s.t.lnshell : s.Nown);
            return 0;
        }
        if (s.t.grp)
        {
            *layout_bytes = 16ull * s.t.ntiles + (uint64_t)s.t.ngroups * 16 +
                            T * (8 + 12 + 4 + 12) + N * (24 + 4 + 12);
            return 0;
        }
        *layout_bytes = 16ull * s.t.ntiles + E * (rec + (s.t.mat ? 4 : 0)) +
                        T * (8 + (s.t.geo ? 12 : 0) + (s.t.node_major ? 4 : 0) + 12) + N * (24 + 4 + 12);
    }
    else  // PARITY node tiles (k_keff_parity_tile), compulsory: per tet the 64-B record, vol, its 4 incidence
          // entries (pinc) and its tile-list entry (+ material); per node CSR offset, x in, y out, mass, mask
        *layout_bytes = E * (64 + 4 + 16 + 4 + (s.M > 1 ? 4 : 0)) + N * (4 + 12 + 12 + 4 + 4);
    return 0;
}

#ifndef CWF_FAST_SRC_HASH
#define CWF_FAST_SRC_HASH "unknown"
#endif
#ifndef CWF_PARITY_SRC_HASH
#define CWF_PARITY_SRC_HASH "unknown"
#endif
const char *cwf_hip_system_keff_source_hash(const cwf_hip_system *h)
{
    if (!h)
        return nullptr;
    return h->mode != CWF_MODE_FAST || !h->ds.t.ntiles ? CWF_PARITY_SRC_HASH : CWF_FAST_SRC_HASH;
}

int cwf_hip_system_exchange_schedule(const cwf_hip_system *h)
{
    if (!h || !h->sharded() || h->fused_agreed < 0)
        return -1;
    return h->fused_agreed == 0 ? 0 : h->res_agreed == 1 ? 3 : h->px_agreed == 1 ? 2 : 1;
}

const char *cwf_hip_system_keff_kernel(const cwf_hip_system *h)
{
    if (!h)
        return nullptr;
    const DevTiles &t = h->ds.t;
    if (h->mode != CWF_MODE_FAST || !t.ntiles)  // the PCG-loop instantiation (no sanitize) of the element pass
    {
        // the PCG loop's: strips fuse the p.Ap partials (DOT), compact tiles do not (parity_incidence_slots)
        const char *pt = knob("CWF_PARITY_TILES");
        const bool compact = h->ds.ptile_nodes || (!h->ds.ptile_off && !h->sharded() && h->ds.E <= kParityCompactMaxTets &&
                                                    !(pt && !std::strcmp(pt, "strip")));
        if (compact)
            return h->ds.iso ? "k_keff_parity_tile<true, false, false, true>" : "k_keff_parity_tile<false, false, false, true>";
        return h->ds.iso ? "k_keff_parity_tile<true, false, true, false>" : "k_keff_parity_tile<false, false, true, false>";
    }
    if (t.lat && fast_fused(h) && resident_on(h))
    {  // the resident solve's one launch per solve (resident.hip)
        static thread_local char name[96];
        snprintf(name, sizeof name, "k_pcg_resident<%s, %s, %u, %u, %s>", t.lsym ? "true" : "false",
                 t.lhex ? "LatHex" : "LatKuhn", h->res.npt, h->res.nph, h->res.shard ? "true" : "false");
        return name;
    }
    if (t.lat && fast_fused(h) && h->fused_agreed != 0)  // the fused iteration's one launch (lattice_fused.inc)
    {
        static thread_local char name[112];
        snprintf(name, sizeof name, "k_pcg_lattice<%s, %s, %s, %s, %s, %s>", t.lsym ? "true" : "false",
                 t.lhex ? "LatHex" : "LatKuhn", t.lmu ? "true" : "false", t.lpstride ? "true" : "false",
                 !t.lpstride && h->ds.Nown < h->ds.N ? "true" : "false",
                 h->fused_grid < t.lnwork ? "true" : "false");
        return name;
    }
    if (t.lat)  // as rocprofv3 names it, less the namespaces
    {
        static thread_local char name[96];
        snprintf(name, sizeof name, "k_keff_lattice<1, false, %s, %s, %s, %s, %s>", t.lsym ? "true" : "false",
                 t.lhex ? "LatHex" : "LatKuhn", t.lmu ? "true" : "false", t.lmu && t.lzr ? "true" : "false",
                 t.lpstride ? "true" : "false");
        return name;
    }
    if (t.grp)  // the PCG-mode instantiation, as rocprofv3 names it (so a profile of another one is not taken)
    {
        static thread_local char name[96];
        snprintf(name, sizeof name, "k_keff_groups_pipe<%s, false, 1, %d, %s>", h->ds.iso ? "true" : "false",
                 t.pipe_nt, h->ds.M == 1 ? "true" : "false");
        return name;
    }
    return t.hex ? "k_keff_hex_tiles" : t.pipe ? "k_keff_tiles_pipe" : "k_keff_tiles";
}

int cwf_hip_derived_fields(cwf_hip_system *h, const float *u, uint64_t n, int u_kind, float *elements,
                           float *nodes, int out_kind)
{
    if (int st = check_ready(h))
        return st;
    if (!u || (!elements && !nodes))
        return set_error(h, CWF_ERR_ARGUMENT, "null pointer");
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "displacement span size mismatch",
                         "input=" + std::to_string(n) + "\ndofs=" + std::to_string(h->ds.D));
    const float *uin = nullptr;
    if (int st = stage_vec(h, u, h->tmp, u_kind, 3, &uin))
        return st;
    const uint64_t ne = 13ull * h->ds.E, nn = 13ull * h->ds.N;
    float *de = elements, *dn = nodes;
    if (out_kind != CWF_PTR_DEVICE || h->perm)  // stage through one scratch allocation
    {
        float *scratch = nullptr;
        HIPTRY(h, hipMalloc(reinterpret_cast<void **>(&scratch), (ne + nn + 1) * sizeof(float)));
        de = elements ? scratch : nullptr;
        dn = nodes ? scratch + ne : nullptr;
        derived_fields(h, uin, de, dn, h->stream);
        hipError_t e1 = hipGetLastError();
        const hipMemcpyKind back = out_kind == CWF_PTR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        if (e1 == hipSuccess && elements)
            e1 = hipMemcpyAsync(elements, de, ne * sizeof(float), back, h->stream);
        if (e1 == hipSuccess && nodes)
        {
            if (h->perm)  // node fields back to the caller's node order
                e1 = vec_out(h, dn, nodes, out_kind, 13) ? hipErrorUnknown : hipSuccess;
            else
                e1 = hipMemcpyAsync(nodes, dn, nn * sizeof(float), back, h->stream);
        }
        if (e1 == hipSuccess)
            e1 = hipStreamSynchronize(h->stream);
        (void)hipFree(scratch);
        if (e1 != hipSuccess)
            return hip_fail(h, e1, "derived fields");
        return 0;
    }
    derived_fields(h, uin, de, dn, h->stream);
    HIPTRY(h, hipGetLastError());
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

}  // extern "C"

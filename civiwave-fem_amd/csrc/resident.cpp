// resident.cpp -- the plan of the resident solve (resident.hip): the structured block cut into one box per workgroup
// (at most one per CU, so the persistent grid is co-resident), each box's node list (the thread -> node map its
// registers keep for the whole solve), its halo list (the one-node ring its rows read, each entry pointing at the
// owner's published record) and the publication index of every node some other box reads.
//
// Box choice: every factorisation gx * gy * gz <= CUs of the node lattice, boxes of ceil(n / g) nodes per axis at most,
// scored by the per-workgroup work of a phase (own nodes + 1.5 x halo entries, each halo entry being three 16-B
// loads and a formed p) plus a barrier term growing with the grid (2 per workgroup); the image (box + ring, float4)
// must fit the LDS beside the static tables and the lists the kernel's 4 + 3 entries per thread. C2 (70^3 nodes): 5 x 7 x 7 boxes of
// 14 x 10 x 10 nodes, 245 workgroups.
#include <algorithm>
#include <cstring>

#include "abi_internal.hpp"

namespace cwf
{
namespace
{
constexpr unsigned kResThreads = 512, kResOwn = 4 * kResThreads, kResHalo = 3 * kResThreads;  // resident.hip
// the box image's float4 slots fill the LDS a gfx950 workgroup may hold beside the kernel's static arrays (the own
// entries' r, Ap, x in the 4-node instantiation: 72 KB; the class table; the box's boundary types' stencils, at
// most kResTypesHost of the 27: 8.6 KB with the 15-offset Kuhn stencil, 15.6 KB with the 27-offset hex8 one)
constexpr unsigned kResTypesHost = 12;  // resident.hip kResTypes
constexpr unsigned kResGhostHost = 512;  // resident.hip kResGhostMax: a shard box's ghost halo entries (their r, p in LDS)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kResGhost = 0x80000000u;  // a halo entry's source: a ghost record (resident.hip)
constexpr unsigned kFusedSharesHost = 5;  // kFusedShares (lattice_common.hpp): one 16-B granule each

void split(unsigned n, unsigned g, unsigned q, unsigned &a, unsigned &b)
{
    a = (unsigned)((uint64_t)n * q / g);
    b = (unsigned)((uint64_t)n * (q + 1) / g);
}
}  // namespace

namespace
{
// the plan over the node planes [k0, k1) of the block (a PEER slab shard: its owned planes; the ghost planes beside
// them are the halo entries' only other source, read from the mailbox). False: the solve keeps the other schedules
bool plan_resident(cwf_hip_system *h, bool shard)
{
    ResidentPlan &rp = h->res;
    const DevTiles &t = h->ds.t;
    const uint32_t N = h->ds.N, Nown = h->ds.Nown;
    if (h->mode != CWF_MODE_FAST || !t.lat || !t.lcls || !t.lcz || h->lat_plane.size() != t.lnz)
        return false;
    const unsigned nx = t.lnx, ny = t.lny, per = nx * ny;
    const unsigned k0 = shard ? t.lk0 : 0, k1 = shard ? t.lk1 : t.lnz, nz = k1 - k0;
    if (nx < 2 || ny < 2 || nz < 2 || k1 > t.lnz)
        return false;
    const std::vector<uint32_t> &plane = h->lat_plane;
    if (!shard && (Nown != N || t.lk0 != 0 || t.lk1 != t.lnz))
        return false;
    // a slab shard: its owned nodes are the whole planes [k0, k1), every other plane is ghosts, its send segments
    // (the halo plan's, <= 2 neighbours) disjoint
    std::vector<uint32_t> remote;  // per owned node: neighbour slot << 24 | position in my send segment to it
    if (shard)
    {
        if ((uint64_t)nz * per != Nown || h->nbr.size() > 2 || Nown >= N)
            return false;
        for (unsigned k = 0; k < t.lnz; ++k)
        {
            const bool own = k >= k0 && k < k1;
            if (own ? (uint64_t)plane[k] + per > Nown : plane[k] < Nown || (uint64_t)plane[k] + per > N)
                return false;
        }
        const uint64_t nsend = h->send_off.empty() ? 0 : h->send_off.back();
        std::vector<uint32_t> idx(nsend);
        if (nsend && hipMemcpy(idx.data(), h->send_idx, nsend * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
            return false;
        remote.assign(Nown, kNone);
        for (size_t k = 0; k < h->nbr.size(); ++k)
            for (uint64_t i = h->send_off[k]; i < h->send_off[k + 1]; ++i)
            {
                const uint64_t pos = i - h->send_off[k];
                if (idx[i] >= Nown || remote[idx[i]] != kNone || pos >= (1u << 24))
                    return false;
                remote[idx[i]] = (uint32_t)k << 24 | (uint32_t)pos;
            }
    }
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return false;
    // ranks sharing this device (a 1-GPU rehearsal) split its CUs: every rank's grid is resident at once
    unsigned same = 1;
    if (shard)
        for (int p = 0; p < h->comm->nranks; ++p)
            same += p != h->rank && h->comm->peer_same_device[p] != 0 ? 1u : 0u;
    const unsigned G0 = (unsigned)cus / same;
    if (!G0 || (uint64_t)Nown > (uint64_t)G0 * kResOwn)
        return false;  // more nodes than the grid's registers hold
    // the node classes: the boundary type orders each box's own list (the type-stencil rows first)
    std::vector<uint8_t> cls(N);
    if (hipMemcpy(cls.data(), t.lcls, N, hipMemcpyDeviceToHost) != hipSuccess)
        return false;
    // the box grid; the image's cap from the LDS the instantiation leaves (the 3-node one for boxes it takes)
    int lds_max = 0;
    if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || lds_max <= 0)
        return false;
    const size_t st_small = resident_static_lds(h->ds, true, shard), st_lst = resident_static_lds(h->ds, false, shard);
    if (!st_small || !st_lst || st_small >= (size_t)lds_max || st_lst >= (size_t)lds_max)
        return false;
    const unsigned cap_small = (unsigned)(((size_t)lds_max - st_small) / 16),
                   cap_lst = (unsigned)(((size_t)lds_max - st_lst) / 16);
    const auto slot_cap = [&](uint64_t own, uint64_t halo) {
        return own <= 3ull * kResThreads && halo <= 2ull * kResThreads ? cap_small : cap_lst;
    };
    double best = 1e300;
    unsigned bg[3] = {0, 0, 0};
    for (unsigned gx = 1; gx <= std::min(nx, G0); ++gx)
        for (unsigned gy = 1; gy <= std::min(ny, G0 / gx); ++gy)
            for (unsigned gz = 1; gz <= std::min(nz, G0 / (gx * gy)); ++gz)
            {
                const uint64_t sx = (nx + gx - 1) / gx, sy = (ny + gy - 1) / gy, sz = (nz + gz - 1) / gz;
                const uint64_t own = sx * sy * sz, slots = (sx + 2) * (sy + 2) * (sz + 2), halo = slots - own;
                if (own > kResOwn || halo > kResHalo || slots > slot_cap(own, halo))
                    continue;
                const double cost = (double)own + 1.5 * (double)halo + 2.0 * (double)(gx * gy * gz);
                if (cost < best)
                {
                    best = cost;
                    bg[0] = gx, bg[1] = gy, bg[2] = gz;
                }
            }
    if (!bg[0])
        return false;
    const unsigned G = bg[0] * bg[1] * bg[2];
    const int(*off)[3] = t.lhex ? kLatHexOff : kLatOff;
    const int noff = t.lhex ? kLatHexOffsets : kLatOffsets;
    const auto node = [&](unsigned i, unsigned j, unsigned k) { return plane[k] + j * nx + i; };
    // owner box of every own node, and which nodes another box reads (a ghost has no owner box)
    std::vector<uint32_t> owner(N, kNone);
    std::vector<unsigned> B(6 * (size_t)G);
    for (unsigned b = 0; b < G; ++b)
    {
        const unsigned bx = b % bg[0], by = (b / bg[0]) % bg[1], bz = b / (bg[0] * bg[1]);
        unsigned *q = &B[6 * (size_t)b];
        split(nx, bg[0], bx, q[0], q[1]);
        split(ny, bg[1], by, q[2], q[3]);
        split(nz, bg[2], bz, q[4], q[5]);
        q[4] += k0, q[5] += k0;
        for (unsigned k = q[4]; k < q[5]; ++k)
            for (unsigned j = q[2]; j < q[3]; ++j)
                for (unsigned i = q[0]; i < q[1]; ++i)
                    owner[node(i, j, k)] = b;
    }
    const auto inside = [&](long ii, long jj, long kk) {
        return ii >= 0 && jj >= 0 && kk >= 0 && ii < (long)nx && jj < (long)ny && kk < (long)t.lnz;
    };
    std::vector<uint8_t> needed(N, 0);
    for (unsigned k = k0; k < k1; ++k)
        for (unsigned j = 0; j < ny; ++j)
            for (unsigned i = 0; i < nx; ++i)
            {
                const uint32_t n = node(i, j, k);
                for (int o = 1; o < noff; ++o)
                {
                    const long ii = (long)i + off[o][0], jj = (long)j + off[o][1], kk = (long)k + off[o][2];
                    if (!inside(ii, jj, kk))
                        continue;
                    const uint32_t m = node((unsigned)ii, (unsigned)jj, (unsigned)kk);
                    if (owner[m] != kNone && owner[m] != owner[n])
                        needed[m] = 1;
                }
            }
    // own lists (block-surface nodes first: their type-stencil rows; then the interior's brick rows), publication indices
    // in that order box after box, then the halo lists (sorted by publication index: consecutive lanes, consecutive
    // records; a shard's ghost entries last, by ghost index)
    std::vector<uint32_t> pubidx(N, kNone);
    std::vector<std::vector<uint4>> ownl(G), halol(G);
    std::vector<uint4> hdr(G);
    uint32_t npub = 0;
    unsigned max_own = 0, max_halo = 0;
    size_t max_slots = 0;
    uint64_t remote_sends = 0;
    for (unsigned b = 0; b < G; ++b)
    {
        const unsigned *q = &B[6 * (size_t)b];
        const unsigned PX = q[1] - q[0] + 2, PXY = PX * (q[3] - q[2] + 2), slots = PXY * (q[5] - q[4] + 2);
        hdr[b] = uint4{slots, 0u, PX, PXY};
        max_slots = std::max<size_t>(max_slots, slots);
        for (int pass = 0; pass < 2; ++pass)
            for (unsigned k = q[4]; k < q[5]; ++k)
                for (unsigned j = q[2]; j < q[3]; ++j)
                    for (unsigned i = q[0]; i < q[1]; ++i)
                    {
                        const uint32_t n = node(i, j, k);
                        const bool surface = (cls[n] >> 3) != 13u;
                        if (surface != (pass == 0))  // the surface first: its slower rows land in the first
                            continue;                // wave-slots, one wave per SIMD in turn, not in the last waves
                        const unsigned slot = (k - q[4] + 1) * PXY + (j - q[2] + 1) * PX + (i - q[0] + 1);
                        if (needed[n])
                            pubidx[n] = npub++;
                        const uint32_t rw = shard ? remote[n] : kNone;
                        remote_sends += rw != kNone ? 1u : 0u;
                        ownl[b].push_back(uint4{n, slot, pubidx[n], rw});
                    }
        max_own = std::max<unsigned>(max_own, (unsigned)ownl[b].size());
    }
    uint64_t halo_total = 0, ghost_total = 0;
    std::vector<uint32_t> seen(N, kNone);
    for (unsigned b = 0; b < G; ++b)
    {
        const unsigned *q = &B[6 * (size_t)b];
        const unsigned PX = hdr[b].z, PXY = hdr[b].w;
        for (unsigned k = q[4]; k < q[5]; ++k)
            for (unsigned j = q[2]; j < q[3]; ++j)
                for (unsigned i = q[0]; i < q[1]; ++i)
                    for (int o = 1; o < noff; ++o)
                    {
                        const long ii = (long)i + off[o][0], jj = (long)j + off[o][1], kk = (long)k + off[o][2];
                        if (!inside(ii, jj, kk))
                            continue;
                        const uint32_t m = node((unsigned)ii, (unsigned)jj, (unsigned)kk);
                        if (owner[m] == b || seen[m] == b)
                            continue;
                        seen[m] = b;
                        const unsigned slot = (unsigned)((kk - (long)q[4] + 1) * PXY + (jj - (long)q[2] + 1) * PX +
                                                         (ii - (long)q[0] + 1));
                        // a ghost (m >= Nown): its record in the mailbox, at its ghost index
                        const uint32_t src = m >= Nown ? kResGhost | (m - Nown) : pubidx[m];
                        halol[b].push_back(uint4{m, slot, src, 0u});
                    }
        std::sort(halol[b].begin(), halol[b].end(), [](const uint4 &a, const uint4 &c) { return a.z < c.z; });
        max_halo = std::max<unsigned>(max_halo, (unsigned)halol[b].size());
        halo_total += halol[b].size();
        // the ghost entries are the list's tail: the first one's position (the kernel's index into its ghost state)
        const auto g0 = std::find_if(halol[b].begin(), halol[b].end(), [](const uint4 &e) { return (e.z & kResGhost) != 0; });
        const uint64_t ng = (uint64_t)(halol[b].end() - g0);
        if (ng > kResGhostHost)
            return false;
        hdr[b].y = (uint32_t)(g0 - halol[b].begin());
        ghost_total += ng;
    }
    // the 4-node instantiation (LDS state): each box's boundary types (its block-surface nodes'), in ascending
    // order; the own entry carries the node's index among them in y >> 24 (the kernel's stencil table holds only the
    // box's types: the LDS the image needs). The 3-node one keeps all 27.
    const bool small0 = (max_own + kResThreads - 1) / kResThreads <= 3 && (max_halo + kResThreads - 1) / kResThreads <= 2;
    std::vector<uint8_t> btypes((size_t)G * kResTypesHost, 0);
    for (unsigned b = 0; b < G && !small0; ++b)
    {
        int idx[27];
        std::fill(idx, idx + 27, -1);
        unsigned nt = 0;
        for (const uint4 &e : ownl[b])
            idx[cls[e.x] >> 3] = 0;
        for (unsigned ty = 0; ty < 27; ++ty)
            if (idx[ty] == 0 && ty != 13)
            {
                if (nt == kResTypesHost)
                    return false;
                btypes[(size_t)b * kResTypesHost + nt] = (uint8_t)ty;
                idx[ty] = (int)nt++;
            }
        for (uint4 &e : ownl[b])
        {
            const unsigned ty = cls[e.x] >> 3;
            e.y |= (ty == 13 ? 0u : (uint32_t)idx[ty]) << 24;
        }
    }
    const unsigned npt = (max_own + kResThreads - 1) / kResThreads, nph = (max_halo + kResThreads - 1) / kResThreads;
    if (max_own > kResOwn || max_halo > kResHalo || max_slots > slot_cap(max_own, max_halo) || N - Nown >= kResGhost)
        return false;
    const bool small = npt <= 3 && nph <= 2;
    const unsigned own_stride = (small ? 3u : 4u) * kResThreads, halo_stride = (small ? 2u : 3u) * kResThreads;
    const size_t lds = max_slots * 16;
    // one workgroup per CU at least (the grid waits for all of them every phase)
    if (resident_blocks_per_cu(h->ds, npt, nph, lds, shard) < 1)
        return false;
    std::vector<uint4> own((size_t)G * own_stride, uint4{kNone, 0u, kNone, kNone}),
        halo((size_t)G * halo_stride, uint4{kNone, 0u, kNone, 0u});
    for (unsigned b = 0; b < G; ++b)
    {
        std::copy(ownl[b].begin(), ownl[b].end(), own.begin() + (size_t)b * own_stride);
        std::copy(halol[b].begin(), halol[b].end(), halo.begin() + (size_t)b * halo_stride);
    }
    // the stencil of each boundary type (lattice.inc's shell cell form regrouped): per offset o >= 1, the sum of the
    // pair blocks (c, c') with c' - c = o over the cells that exist around a node of that type, in fp64, stored in the
    // rows' packed order {S00 S10 S01 S11} {S02 S12 S20 S21} {S22 - - -}
    const int npairs = t.lhex ? kLatHexPairs : kLatPairs;
    std::vector<float> cf((size_t)(noff + npairs) * 9);
    if (hipMemcpy(cf.data(), t.lcoef, cf.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
        return false;
    std::vector<float4> tco(27ull * noff * 3, float4{0.f, 0.f, 0.f, 0.f});
    for (unsigned ty = 0; ty < 27; ++ty)
    {
        const unsigned sd[3] = {ty % 3, (ty / 3) % 3, ty / 9};  // 0 lo, 1 inside, 2 hi
        unsigned w8 = 0;
        for (unsigned c8 = 0; c8 < 8; ++c8)
        {
            bool in = true;
            for (int ax = 0; ax < 3; ++ax)
                in = in && (((c8 >> ax) & 1u) ? sd[ax] != 0 : sd[ax] != 2);
            w8 |= (in ? 1u : 0u) << c8;
        }
        for (int o = 1; o < noff; ++o)
        {
            double S[9] = {};
            for (int pp = 0; pp < npairs; ++pp)
            {
                const int c = t.lhex ? pp / 8 : kLatPair[pp][0];
                const int po = t.lhex ? kLatHexPairOff[pp] : kLatPairOff[pp];
                if (po != o || !((w8 >> c) & 1u))
                    continue;
                for (int e = 0; e < 9; ++e)
                    S[e] += (double)cf[(size_t)9 * noff + 9 * pp + e];
            }
            float4 *q = &tco[(size_t)3 * (ty * noff + o)];
            q[0] = float4{(float)S[0], (float)S[3], (float)S[1], (float)S[4]};
            q[1] = float4{(float)S[2], (float)S[5], (float)S[6], (float)S[7]};
            q[2] = float4{(float)S[8], 0.f, 0.f, 0.f};
        }
    }
    std::vector<float4> btco(small ? 0 : (size_t)G * kResTypesHost * noff * 3, float4{0.f, 0.f, 0.f, 0.f});
    for (unsigned b = 0; b < G && !small; ++b)
        for (unsigned k = 0; k < kResTypesHost; ++k)
            std::copy(tco.begin() + (size_t)3 * noff * btypes[(size_t)b * kResTypesHost + k],
                      tco.begin() + (size_t)3 * noff * (btypes[(size_t)b * kResTypesHost + k] + 1),
                      btco.begin() + ((size_t)b * kResTypesHost + k) * 3 * noff);
    float4 *dtc;
    if (small ? upload(h, &dtc, tco.data(), tco.size()) : upload(h, &dtc, btco.data(), btco.size()))
        return false;
    uint4 *dh, *dow, *dha;
    float *dpub;
    double *dsh;
    if (upload(h, &dh, hdr.data(), hdr.size()) || upload(h, &dow, own.data(), own.size()) ||
        upload(h, &dha, halo.data(), halo.size()) || dalloc(h, &dpub, 2ull * 12 * std::max<uint32_t>(npub, 1u)) ||
        dalloc(h, &dsh, 2ull * 2 * kFusedSharesHost * G))
        return false;
    // tags 0: below every tag a solve waits for (the first solve's base is 1, its phases wait for 2 and up)
    if (hipMemset(dsh, 0, 2ull * 2 * kFusedSharesHost * G * sizeof(double)) != hipSuccess ||
        hipMemset(dpub, 0, 2ull * 12 * std::max<uint32_t>(npub, 1u) * sizeof(float)) != hipSuccess)
        return false;
    // a shard's mailbox area (the peers store into it only in a resident solve, after the collective vote that
    // follows this)
    if (shard && peer_resident_clear(h))
        return false;
    rp.G = G;
    rp.npt = small ? 3 : 4;  // the instantiation (resident.hip)
    rp.nph = small ? 2 : 3;
    rp.own_stride = own_stride;
    rp.halo_stride = halo_stride;
    rp.npub = std::max<uint32_t>(npub, 1u);
    rp.lds = lds;
    std::memcpy(rp.dims, bg, sizeof bg);
    rp.max_own = max_own;
    rp.max_halo = max_halo;
    rp.halo_total = halo_total;
    rp.hdr = dh;
    rp.tcoef = dtc;
    rp.own = dow;
    rp.halo = dha;
    rp.pub = dpub;
    rp.sh = dsh;
    rp.shard = shard;
    rp.remote_sends = remote_sends;
    rp.ghost_total = ghost_total;
    rp.state = 1;
    return true;
}

// CWF_RESIDENT=0, or an explicit CWF_FUSED schedule (0: two kernels, 1: the per-launch fused iteration, 2: its
// persistent walk), keeps the launch-per-iteration schedules
bool resident_off()
{
    const char *kn = knob("CWF_RESIDENT");
    return (kn && kn[0] == '0') || knob("CWF_FUSED");
}
}  // namespace

bool resident_ready(cwf_hip_system *h)
{
    ResidentPlan &rp = h->res;
    if (rp.state)
        return rp.state > 0 && !rp.shard;
    if (h->sharded())
        return false;  // a shard plans at the schedule vote (resident_shard_ready)
    rp.state = -1;
    return !resident_off() && plan_resident(h, false);
}

bool resident_shard_ready(cwf_hip_system *h)
{
    ResidentPlan &rp = h->res;
    if (rp.state)
        return rp.state > 0 && rp.shard;
    rp.state = -1;
    // PEER only: the kernel stores its surface records into the neighbours' mailboxes itself
    if (resident_off() || !h->sharded() || !h->comm || h->comm->kind != 2 || h->nranks > kMaxPeers)
        return false;
    return plan_resident(h, true);
}

bool resident_on(const cwf_hip_system *h)
{
    if (h->sharded())
        return h->res_agreed == 1 && h->res.state > 0 && h->res.shard;
    return resident_ready(const_cast<cwf_hip_system *>(h));
}

uint64_t resident_offchip_bytes(const cwf_hip_system *h)
{
    const ResidentPlan &rp = h->res;
    // 48-B records on chip (read by the ring entries, written by the published nodes); a shard's ghost entries read,
    // and its send-plane nodes write, one 16-B Ap granule
    uint64_t b = 48ull * (rp.halo_total - rp.ghost_total + rp.npub) + 16ull * (rp.ghost_total + rp.remote_sends) +
                 80ull * rp.G * (1ull + rp.G);
    if (rp.shard)  // the rank totals: one rank's stores to every rank, every workgroup's poll of all of them
        b += 80ull * h->nranks * (1ull + rp.G);
    return b;
}

}  // namespace cwf

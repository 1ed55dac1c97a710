// resident.hip -- k_pcg_resident: a whole FAST PCG solve of a structured block in ONE launch, with every vector on chip
// (lattice_common.hpp: the fused iteration's per-node arithmetic, run unchanged).
//
// Why: the fused one-launch iteration (lattice_fused.inc) is bound by a per-workgroup chain, not by bytes -- every
// launch re-reads r, Ap, p, x and the class of every node from L2 / MALL (97 B per node), every workgroup refolds the
// previous launch's 436 x 5 shares, and a kernel boundary separates the iterations (C2: 18 us per iteration for 33 MB,
// 0.23 of HBM; VERDICT r5 items 2 and the C3 / 8 strong-scaling bound). A block of up to ~0.5M nodes fits on chip:
// 256 CUs x 160 KB of LDS and 512 KB of VGPRs hold C2's 16.5 MB of r, Ap, p, x many times over. So the solve becomes
// one persistent launch of one 512-thread workgroup per CU, each owning a box of the lattice:
//   - its nodes' r, Ap, p, x, z, class and mass live in registers (NPT nodes per thread) for the whole solve;
//   - per iteration (phase j) it forms r_j, z_j, p_j, x_j exactly as lattice_fused.inc's launch j does (fused_form),
//     writes p_j into an LDS image of the box plus its one-node halo, applies the stencil rows (interior nodes: the
//     brick rows' difference form; block-surface nodes: the shell's cell form), and leaves the five fp64 dots;
//   - the halo's p_j is formed locally from the owners' published (r_(j-1), Ap_(j-1), p_(j-1)) -- the same bits the
//     owner forms -- so ONE synchronisation per iteration carries both the halo and the scalars: each workgroup stores
//     its box-surface records and its five shares write-through (sc1), waits for its stores, and adds one to an
//     arrival counter; the next phase polls the counter (sc1) until every workgroup arrived, reads the G x 5 shares
//     and its halo records (sc1: served past the non-coherent L1 / per-XCD L2), folds the shares in a fixed order
//     (so every workgroup takes the same alpha, beta and stop decision, fused_decide) and goes on.
// The hand-off is MI355X_MICROARCH.md's validated form (sc1 16-B stores, every storing wave's vmcnt(0) before one
// lane's agent-scope add after a workgroup barrier; one lane's sc1 poll, a workgroup barrier, then sc1 16-B loads).
// Every wait is bounded (kResTimeoutTicks): a workgroup that is never scheduled (the grid must be co-resident, one per
// CU; resident_capacity checks the occupancy) ends the solve with CWF_ERR_HIP instead of hanging the GPU.
//
// Results: the per-node arithmetic is lattice_fused.inc's; only the grouping of the fp64 dot sums differs (boxes
// instead of bricks), so alpha / beta differ in their last bits and the solve is tolerance-equal, not bit-equal, to the
// fused schedule (tests/test_gpu_resident.py). Deterministic run to run: no atomics touch a value, the folds' order is
// fixed.
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lattice_common.hpp"

namespace cwf
{
namespace
{
constexpr int kResNT = 512;
constexpr uint32_t kResMaxRounds = 4000000u;  // poll rounds before a phase gives up (>= 4 s: a round is >= 1 us)
constexpr uint32_t kResNone = 0xFFFFFFFFu;
constexpr uint32_t kResOob = 0xFFFFFF00u;  // a byte offset past every range-checked buffer here, +32 included (no wrap)
constexpr uint32_t kResGhost = 0x80000000u;  // a halo entry's source: a shard's ghost record (resident.cpp)
constexpr int kResTypes = 12;  // boundary types one box's own nodes touch, at most (resident.cpp kResTypesHost)
constexpr int kResGhostMax = 512;  // a shard box's ghost halo entries, at most (resident.cpp kResGhostHost)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct ResArgs
{
    Ctl *ctl;
    double *hist;
    const uint4 *hdr;   // [G] {LDS slots, first ghost halo entry (a shard), PX, PXY}: the box's (sx + 2)(sy + 2)(sz + 2)
                        // image and its strides
    const uint4 *own;   // [G][own_stride] {node, image slot, publication index or kResNone, -}
    const uint4 *halo;  // [G][halo_stride] {node, slot, publication index of its owner's record, -}
    const float4 *tcoef;  // the stencil of each boundary type (the block-surface rows), padded blocks: [27][nOff][3]
                          // for the register-state instantiation; for the LDS-state one [G][kResTypes][nOff][3], per
                          // box only the types its nodes have (the own entry's y >> 24 is the node's index there)
    uint32_t own_stride, halo_stride;
    float *pub;         // [2][npub][12] by phase parity: granules {r.xyz, tag} {Ap.xyz, tag} {p.xyz, tag}
    uint32_t npub;
    double *sh;         // [2][G][5] granules {share lo, hi, tag, -} by phase parity
    uint32_t tag0;      // this solve's tag base: phase j's granules carry tag0 + j + 1 (a previous solve's never match)
    float *x, *r;       // in: x_0 (the warm start) and r_0 (fast_fused_init); out: x and r at the stop
    uint32_t max_it;
    uint64_t *trace;    // diagnostic (CWF_RESIDENT_TRACE): per workgroup 8 s_memrealtime stamps of phase trace_j
    uint32_t trace_j;
    // a PEER slab shard (nranks > 1): the send planes' Ap_(j-1) granules stored into the neighbours' mailboxes (a ghost's
    // r and p the receiving box forms itself and keeps, exactly as the owner does), the ghosts' granules read from this
    // rank's, the rank totals stored to every rank and polled from this rank's
    ResPeerArgs pa;
};

__device__ __forceinline__ void st4_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off, u32x4 w)
{
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, off, 0, 16);  // sc1: write-through, past the XCD's L2
}
__device__ __forceinline__ u32x4 pk4(float a, float b, float c, float d)
{
    return u32x4{__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d)};
}
__device__ __forceinline__ u32x4 ld4_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);  // sc1: served past L1
}
// the PEER mailboxes (uncached IPC memory, written by other devices over xGMI): system scope both ways
__device__ __forceinline__ void st4_sys(__amdgpu_buffer_rsrc_t rs, uint32_t off, u32x4 w)
{
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, off, 0, 17);  // sc0 sc1
}
__device__ __forceinline__ u32x4 ld4_sys(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 17);
}

// a workgroup barrier that orders LDS only: no vmcnt wait, so the write-through stores and the polls in flight stay in
// flight across it (__syncthreads' workgroup fence would wait for every store to be acknowledged)
__device__ __forceinline__ void lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// block_sum_k's fixed order (wave sums, then the waves in order) over lds_sync. No trailing barrier: each caller's next
// write of `red` is behind other workgroup barriers of the phase (the halo vote / image barrier, the next phase's polls)
template <int NT, int K>
__device__ __forceinline__ void block_sum_lds(double v[K], double *red)
{
#pragma unroll
    for (int q = 0; q < K; ++q)
    {
        v[q] = wave_sum(v[q]);
        if ((threadIdx.x & 63) == 0)
            red[K * (threadIdx.x >> 6) + q] = v[q];
    }
    lds_sync();
#pragma unroll
    for (int q = 0; q < K; ++q)
    {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w)
            t += red[K * w + q];
        v[q] = t;
    }
}

template <bool SYM, class E, int NPT, int NPH, bool MR>
__global__ __launch_bounds__(kResNT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pcg_resident(DevSys s, ResArgs ra, const float *__restrict__ coef)
{
    extern __shared__ float4 pl[];  // the box + one-node halo image of p_j (out-of-block entries stay 0)
    __shared__ double red[kFusedShares * (kResNT / 64)];
    __shared__ float4 czA[kLatClasses];
    __shared__ float2 czB[kLatClasses];
    constexpr bool LST = NPT > 3;
    constexpr int kTT = LST ? kResTypes : 27;  // the box's boundary types (LST: the LDS the image needs) or all 27
    __shared__ float4 tcf[kTT * E::nOff * 3];  // the boundary types' stencils (not the interior's)
    __shared__ int vote[3];  // the poll rounds' workgroup vote, by round mod 3
    __shared__ double rt[MR ? kFusedShares * kMaxPeers : 1];  // a shard: the ranks' totals, folded in rank order
    __shared__ float4 gst[MR ? 2 * kResGhostMax : 1];  // a shard: each ghost entry's r_j, p_j ({r, -} {p, -})
    // the own entries' r, Ap, x and p: in registers for boxes of <= 3 nodes per thread (C2's 14 x 10 x 10), else
    // (LST) r, Ap, x in LDS (lane-linear: conflict-free) and p in the image (each slot formed by one thread), so 4
    // nodes per thread fit without spilling (the C3 / 8 slab's 19 x 19 x 5; LDS state cost C2 0.9 us per phase)
    __shared__ float st[LST ? 9 : 1][LST ? NPT * kResNT : 1];
    float sreg[LST ? 1 : NPT][LST ? 1 : 12];  // r, Ap, x, p
    const auto S = [&](int u, int q) -> float & {  // q: 0-2 r, 3-5 Ap, 6-8 x (9-11 p: registers only)
        if constexpr (LST)
            return st[q][threadIdx.x + (uint32_t)u * kResNT];
        else
            return sreg[u][q];
    };
    const DevTiles &T = s.t;
    const uint32_t G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
    const uint4 hd = ra.hdr[b];
    const int PX = (int)hd.z, PXY = (int)hd.w;
    // diagnostic phase stamps (a uniform branch; no store unless CWF_RESIDENT_TRACE asked for them)
    const auto stamp = [&](unsigned j, int i) {
        if (ra.trace && j == ra.trace_j && tid == 0)
            __hip_atomic_store(ra.trace + 8ull * b + i, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    for (uint32_t i = tid; i < hd.x; i += kResNT)
        pl[i] = float4{0.f, 0.f, 0.f, 0.f};
    for (uint32_t i = tid; i < (uint32_t)(kTT * E::nOff * 3); i += kResNT)
        tcf[i] = ra.tcoef[(LST ? (size_t)b * (kTT * E::nOff * 3) : 0) + i];

    if (tid < kLatClasses)
    {
        const float4 zA = T.lcz[2u * tid], zB = T.lcz[2u * tid + 1u];
        czA[tid] = zA;
        czB[tid] = float2{zB.x, zB.y};
    }
    const uint32_t vbytes = 12u * s.N;
    constexpr bool multi = MR;  // a PEER slab shard (its own instantiation: the one-block kernel stays as it was)
    const __amdgpu_buffer_rsrc_t rx = sized_rsrc(ra.x, vbytes), rr = sized_rsrc(ra.r, vbytes),
                                 rcls = sized_rsrc(T.lcls, s.N), rmass = sized_rsrc(s.mass, 4u * s.N),
                                 rpub = sized_rsrc(ra.pub, 96u * ra.npub), rsh = sized_rsrc(ra.sh, 160u * G);
    // own nodes: their r, Ap, x in LDS (st), p in the image, for the whole solve; in registers only the node, its
    // image slot and class, publication index and mass (4 per node: 4 nodes per thread fit without spilling)
    uint32_t on[NPT], osc[NPT], opub[NPT];  // node; image slot | class << 16; publication index
    float m[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u)
    {
        const uint32_t e0 = tid + (uint32_t)u * kResNT;
        const uint4 e = ra.own[(size_t)b * ra.own_stride + e0];
        on[u] = e.x;
        opub[u] = e.z;
        const bool v = e.x != kResNone;
        const uint32_t nb = v ? 12u * e.x : 12u * kLatOob3;
        const u32x3 wr = __builtin_amdgcn_raw_buffer_load_b96(rr, nb, 0, 0),
                    wx = __builtin_amdgcn_raw_buffer_load_b96(rx, nb, 0, 0);
        S(u, 0) = __uint_as_float(wr.x), S(u, 1) = __uint_as_float(wr.y), S(u, 2) = __uint_as_float(wr.z);
        S(u, 3) = S(u, 4) = S(u, 5) = 0.f;
        S(u, 6) = __uint_as_float(wx.x), S(u, 7) = __uint_as_float(wx.y), S(u, 8) = __uint_as_float(wx.z);
        if constexpr (!LST)
            sreg[u][9] = sreg[u][10] = sreg[u][11] = 0.f;
        // image slot | class << 16 (| LST: the box's index of the node's boundary type << 24)
        osc[u] = (e.y & (LST ? 0xFF00FFFFu : 0xFFFFu)) |
                 (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rcls, v ? e.x : kResNone, 0, 0) << 16;
        m[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rmass, v ? 4u * e.x : 4u * kLatOob1, 0, 0));
    }
    // halo entries: their owners' records
    uint32_t hn[NPH], hsc[NPH], hpub[NPH];  // node; image slot | class << 16; the owner's publication index
#pragma unroll
    for (int h = 0; h < NPH; ++h)
    {
        const uint4 e = ra.halo[(size_t)b * ra.halo_stride + tid + (uint32_t)h * kResNT];
        hn[h] = e.x;
        hpub[h] = e.z;
        hsc[h] = e.y | (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rcls, e.x != kResNone ? e.x : kResNone, 0, 0)
                           << 16;
    }
    const CtlPre pre = ctl_prefetch(ra.ctl, 1u);  // tol and active (set by fast_fused_init)
    // the node's neighbours in the image (workgroup-uniform)
    int soff[E::nOff];
#pragma unroll
    for (int o = 0; o < E::nOff; ++o)
        soff[o] = E::off[o][0] + E::off[o][1] * PX + E::off[o][2] * PXY;
    // halo entry h's record of the phase of parity par: another box's (pub), or a ghost's in the mailbox (a shard;
    // the out-of-range load of the other source returns 0, so the two combine by OR)
    const auto request = [&](int h, uint32_t par, u32x4 &a, u32x4 &c, u32x4 &e) {
        const bool gh = (hpub[h] & kResGhost) != 0u, v = hn[h] != kResNone;
        const uint32_t po = v && !gh ? 48u * (par * ra.npub + hpub[h]) : kResOob;
        a = ld4_sc1(rpub, po);
        c = ld4_sc1(rpub, po + 16u);
        e = ld4_sc1(rpub, po + 32u);
        if constexpr (multi)  // a ghost: its owner's Ap_(j-1) granule only
        {
            const __amdgpu_buffer_rsrc_t rg = sized_rsrc(par ? ra.pa.grecv[1] : ra.pa.grecv[0], ra.pa.grecv_bytes);
            c |= ld4_sys(rg, v && gh ? 16u * (hpub[h] & ~kResGhost) : kResOob);
        }
    };
    __syncthreads();
    const float sK = (float)s.sK, sM = (float)s.sM;
    bool go = pre.active != 0;
    unsigned j = 0;
    for (; go; ++j)
    {
        float alpha = 0.f, beta = 0.f;
        float hr[NPH][3], ha[NPH][3], hp[NPH][3];
        u32x4 w0[NPH], w1[NPH], w2[NPH];  // phase j - 1's halo records (granules {r, tag} {Ap, tag} {p, tag})
        const uint32_t par = (j - 1u) & 1u, want = ra.tag0 + j;
        // the workgroup's vote on `ok` (slot round mod 3; the next round's slot is reset before this round's
        // barrier: its last readers passed a barrier since). Every thread counts the same rounds: uniform
        uint32_t round = 0;
        const auto all_ok = [&](bool ok) {
            if (tid == 0)
                vote[(round + 1u) % 3u] = 1;
            if (!ok)
                vote[round % 3u] = 0;
            lds_sync();
            return vote[round % 3u] != 0;
        };
        const auto give_up = [&]() {
            if (tid == 0)
            {
                ra.ctl->error = CWF_ERR_HIP;
                ra.ctl->error_iter = (int)j;
                ra.ctl->active = 0;
            }
        };
        if (j == 0)  // phase 0 (alpha = beta = 0; Ap_(-1) = p_(-1) = 0): the halo's r_0 from fast_fused_init's r
        {
#pragma unroll
            for (int h = 0; h < NPH; ++h)
            {
                const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(rr, hn[h] != kResNone ? 12u * hn[h] : 12u * kLatOob3,
                                                                     0, 0);
                hr[h][0] = __uint_as_float(w.x), hr[h][1] = __uint_as_float(w.y), hr[h][2] = __uint_as_float(w.z);
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    ha[h][c] = hp[h][c] = 0.f;
            }
        }
        else
        {
            stamp(j, 0);
            // phase j - 1's five shares of every workgroup and this box's halo records, polled until every granule
            // carries phase j - 1's tag (each 16-B granule is one write-through store with its own tag: no counter,
            // no ordering between granules needed). Bounded: a workgroup that never publishes ends the solve
            u32x4 g[kFusedShares];
            // the five share granules of every workgroup (thread t < G: workgroup t's), polled until all carry
            // phase j - 1's tag; then this box's halo records are requested and arrive while the shares are folded
            // and the own nodes formed (a producer stores its halo records before its shares, so they have nearly
            // always landed by then; a record with another tag is read again below)
            for (;; ++round)
            {
#pragma unroll
                for (int q = 0; q < kFusedShares; ++q)
                    g[q] = ld4_sc1(rsh, tid < G ? 16u * ((par * G + tid) * kFusedShares + (uint32_t)q) : kResOob);
                bool ok = true;
#pragma unroll
                for (int q = 0; q < kFusedShares; ++q)
                    ok = ok && (tid >= G || g[q].z == want);
                if (all_ok(ok))
                    break;
                if (round >= kResMaxRounds)
                {
                    give_up();
                    return;  // x, r are not written: the solve fails
                }
                __builtin_amdgcn_s_sleep(2);
            }
#pragma unroll
            for (int h = 0; h < NPH; ++h)
                request(h, par, w0[h], w1[h], w2[h]);
            stamp(j, 1);
            double v[kFusedShares];
#pragma unroll
            for (int q = 0; q < kFusedShares; ++q)
                v[q] = tid < G ? __hiloint2double((int)g[q].y, (int)g[q].x) : 0.0;
            block_sum_lds<kResNT, kFusedShares>(v, red);  // fixed order: every workgroup the same totals
            if constexpr (multi)  // the rank's totals to every rank (workgroup 0), then every rank's, folded in rank order
            {
                const uint32_t nr = ra.pa.nranks, jp = j & 1u;
                if (b == 0 && tid < (uint32_t)kFusedShares)
                {
                    double t = v[0];
#pragma unroll
                    for (int q = 1; q < kFusedShares; ++q)
                        t = tid == (uint32_t)q ? v[q] : t;
                    const u32x4 w = {(uint32_t)__double2loint(t), (uint32_t)__double2hiint(t), want, 0u};
#pragma unroll
                    for (int p = 0; p < kMaxPeers; ++p)
                        if ((uint32_t)p < nr)
                            st4_sys(sized_rsrc(jp ? ra.pa.tot[p][1] : ra.pa.tot[p][0], 80u * nr),
                                    16u * (kFusedShares * ra.pa.rank + tid), w);
                }
                const __amdgpu_buffer_rsrc_t rtm = sized_rsrc(jp ? ra.pa.tot_mine[1] : ra.pa.tot_mine[0], 80u * nr);
                u32x4 gt;
                for (;; ++round)
                {
                    gt = ld4_sys(rtm, tid < kFusedShares * nr ? 16u * tid : kResOob);
                    if (all_ok(tid >= kFusedShares * nr || gt.z == want))
                        break;
                    if (round >= kResMaxRounds)
                    {
                        give_up();
                        return;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (tid < kFusedShares * nr)
                    rt[tid] = __hiloint2double((int)gt.y, (int)gt.x);
                lds_sync();
#pragma unroll
                for (int q = 0; q < kFusedShares; ++q)
                {
                    double t = 0.0;
                    for (uint32_t p = 0; p < nr; ++p)
                        t += rt[kFusedShares * p + q];
                    v[q] = t;
                }
            }
            stamp(j, 7);
            go = fused_decide(ra.ctl, ra.hist, j, pre, v, &alpha, &beta);
            if (go && j - 1u == ra.max_it)  // max_iterations updates made (the host loop's last launch)
                go = false;
            if (!go)
                break;
            stamp(j, 2);
        }
        // form r_j, z_j, p_j (x_j) of the own nodes and p_j of the halo into the image. The per-node indices are
        // opaque per phase, so no address derived from them is hoisted out of the phase loop into a VGPR
#pragma unroll
        for (int u = 0; u < NPT; ++u)
            asm volatile("" : "+v"(osc[u]), "+v"(opub[u]), "+v"(on[u]));
#pragma unroll
        for (int h = 0; h < NPH; ++h)
            asm volatile("" : "+v"(hsc[h]), "+v"(hpub[h]), "+v"(hn[h]));
        double d[kFusedShares] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int u = 0; u < NPT; ++u)
        {
            __builtin_amdgcn_sched_barrier(0);  // one node's working set at a time (no cross-node hoisting)
            if (on[u] == kResNone)
                continue;
            const uint32_t slot = osc[u] & 0xFFFFu;
            // p_(j-1): this thread formed it last phase (0 at phase 0)
            const float4 po = LST ? pl[slot] : float4{S(u, 9), S(u, 10), S(u, 11), 0.f};
            const float rr0[3] = {S(u, 0), S(u, 1), S(u, 2)}, aa0[3] = {S(u, 3), S(u, 4), S(u, 5)},
                        pp0[3] = {po.x, po.y, po.z};
            float rn[3], zz[3], pn[3];
            fused_form(czA, czB, LST ? (osc[u] >> 16) & 0xFFu : osc[u] >> 16, alpha, beta, rr0, aa0, pp0, rn, zz, pn);
#pragma unroll
            for (int c = 0; c < 3; ++c)
            {
                S(u, 6 + c) = fmaf(alpha, pp0[c], S(u, 6 + c));  // x_j = x_(j-1) + alpha_(j-1) p_(j-1)
                S(u, c) = rn[c];
                if constexpr (!LST)
                    S(u, 9 + c) = pn[c];
            }
            pl[slot] = float4{pn[0], pn[1], pn[2], 0.f};
            fused_entry_dots(rn, zz, d);
        }
        // a shard's ghost entries: their r_(j-1), p_(j-1) as this box formed them last phase (the registers stay as
        // loaded through the re-reads below, so a ghost formed twice stores the same r_j, p_j)
        const auto ghost = [&](int h) { return multi && (hpub[h] & kResGhost) != 0u; };
        const auto gslot = [&](int h) { return 2u * (tid + (uint32_t)h * kResNT - hd.y); };
        if constexpr (multi)
            if (j > 0)
#pragma unroll
                for (int h = 0; h < NPH; ++h)
                    if (hn[h] != kResNone && ghost(h))
                    {
                        const float4 gr = gst[gslot(h)], gp = gst[gslot(h) + 1u];
                        hr[h][0] = gr.x, hr[h][1] = gr.y, hr[h][2] = gr.z;
                        hp[h][0] = gp.x, hp[h][1] = gp.y, hp[h][2] = gp.z;
                    }
        // the halo's p_j: phase 0 from fast_fused_init's r; later phases from the records requested above, each
        // granule checked for its tag (a record that had not landed is read again: a bounded, voted re-read)
        for (;; ++round)
        {
            bool hok = true;
#pragma unroll
            for (int h = 0; h < NPH; ++h)
            {
                if (hn[h] == kResNone)
                    continue;
                if (j > 0)
                {
                    const bool gh = ghost(h);
                    if (w1[h].w != want || (!gh && (w0[h].w != want || w2[h].w != want)))
                    {
                        hok = false;
                        continue;
                    }
                    if (!gh)
                    {
                        hr[h][0] = __uint_as_float(w0[h].x), hr[h][1] = __uint_as_float(w0[h].y);
                        hr[h][2] = __uint_as_float(w0[h].z);
                        hp[h][0] = __uint_as_float(w2[h].x), hp[h][1] = __uint_as_float(w2[h].y);
                        hp[h][2] = __uint_as_float(w2[h].z);
                    }
                    ha[h][0] = __uint_as_float(w1[h].x), ha[h][1] = __uint_as_float(w1[h].y);
                    ha[h][2] = __uint_as_float(w1[h].z);
                }
                float rn[3], zz[3], pn[3];
                fused_form(czA, czB, hsc[h] >> 16, alpha, beta, hr[h], ha[h], hp[h], rn, zz, pn);
                pl[hsc[h] & 0xFFFFu] = float4{pn[0], pn[1], pn[2], 0.f};
                if (ghost(h))
                {
                    gst[gslot(h)] = float4{rn[0], rn[1], rn[2], 0.f};
                    gst[gslot(h) + 1u] = float4{pn[0], pn[1], pn[2], 0.f};
                }
            }
            if (j == 0)
            {
                lds_sync();  // the image complete before the rows
                break;
            }
            if (all_ok(hok))  // (its barrier also completes the image: the own entries were written before it)
                break;
            if (round >= kResMaxRounds)
            {
                give_up();
                return;
            }
#pragma unroll
            for (int h = 0; h < NPH; ++h)
                request(h, par, w0[h], w1[h], w2[h]);
        }
        stamp(j, 3);
        // rows: Ap_j = K_eff p_j, the dots of the row, the box-surface records for the neighbours' next phase
#pragma unroll
        for (int u = 0; u < NPT; ++u)
        {
            __builtin_amdgcn_sched_barrier(0);  // one row's LDS reads in flight at a time (VGPRs)
            if (on[u] == kResNone)
                continue;
            int c0 = (int)(osc[u] & 0xFFFFu);
            asm volatile("" : "+v"(c0));  // opaque per phase: the rows' image addresses are not hoisted out of the phase
                                          // loop (56 loop-invariant addresses would pin as many VGPRs)
            const uint32_t e0 = tid + (uint32_t)u * kResNT;
            const uint32_t rw = multi ? ra.own[(size_t)b * ra.own_stride + e0].w : kResNone;  // a shard's send position
            const float4 q0 = LST ? pl[c0] : float4{S(u, 9), S(u, 10), S(u, 11), 0.f};
            const float u0[3] = {q0.x, q0.y, q0.z};
            float acc[3];
            const uint32_t cls = LST ? (osc[u] >> 16) & 0xFFu : osc[u] >> 16, ty = cls >> 3;  // boundary type
            if (ty != 13u)  // a block-surface node: its type's stencil (the cell form's pair blocks of the cells that
            {               // exist, summed per offset at plan time), every offset on its own
                const float4 *tb = tcf + (LST ? osc[u] >> 24 : ty) * (uint32_t)(E::nOff * 3);
                f2 acc01 = {0.f, 0.f};
                float acc2 = 0.f;
                const f2 u0xy = {u0[0], u0[1]};
#pragma unroll
                for (int o = 1; o < E::nOff; ++o)
                {
                    const float4 q = pl[c0 + soff[o]];
                    const f2 wxy = f2{q.x, q.y} - u0xy;
                    const float wz = q.z - u0[2];
                    const float4 b0 = tb[3 * o], b1 = tb[3 * o + 1], b2 = tb[3 * o + 2];
                    acc01 = __builtin_elementwise_fma(f2{b0.x, b0.y}, f2{wxy.x, wxy.x}, acc01);
                    acc01 = __builtin_elementwise_fma(f2{b0.z, b0.w}, f2{wxy.y, wxy.y}, acc01);
                    acc01 = __builtin_elementwise_fma(f2{b1.x, b1.y}, f2{wz, wz}, acc01);
                    acc2 = fmaf(b1.z, wxy.x, acc2);
                    acc2 = fmaf(b1.w, wxy.y, acc2);
                    acc2 = fmaf(b2.x, wz, acc2);
                }
                acc[0] = acc01.x;
                acc[1] = acc01.y;
                acc[2] = acc2;
            }
            else  // the brick rows' difference form (lattice_fused.inc rows1); the blocks as scalar loads (from LDS
            {     // as well: rows 3.5 -> 4.7 us per phase on C2)
                int zoff;
                asm volatile("s_mov_b32 %0, 0" : "=s"(zoff));
                const float *__restrict__ cf = coef + zoff;
                const f2 u0xy = {u0[0], u0[1]};
                f2 acc01 = {0.f, 0.f};
                float acc2 = 0.f;
#pragma unroll
                for (int o = 1; o < E::nOff; o += (SYM ? 2 : 1))
                {
                    f2 wxy;
                    float wz;
                    {
                        const float4 q = pl[c0 + soff[o]];
                        wxy = f2{q.x, q.y} - u0xy;
                        wz = q.z - u0[2];
                    }
                    if constexpr (SYM)
                    {
                        const float4 q = pl[c0 + soff[o + 1]];
                        wxy += f2{q.x, q.y} - u0xy;
                        wz += q.z - u0[2];
                    }
                    const float *bq = cf + 9 * o;
                    acc01 = __builtin_elementwise_fma(f2{bq[0], bq[1]}, f2{wxy.x, wxy.x}, acc01);
                    acc01 = __builtin_elementwise_fma(f2{bq[2], bq[3]}, f2{wxy.y, wxy.y}, acc01);
                    acc01 = __builtin_elementwise_fma(f2{bq[4], bq[5]}, f2{wz, wz}, acc01);
                    acc2 = fmaf(bq[6], wxy.x, acc2);
                    acc2 = fmaf(bq[7], wxy.y, acc2);
                    acc2 = fmaf(bq[8], wz, acc2);
                }
                acc[0] = acc01.x;
                acc[1] = acc01.y;
                acc[2] = acc2;
            }
            const float mm = m[u] * sM;
            float an[3];
#pragma unroll
            for (int c = 0; c < 3; ++c)
                an[c] = fmaf(mm, u0[c], sK * acc[c]);
#pragma unroll
            for (int c = 0; c < 3; ++c)
                S(u, 3 + c) = an[c];
            const float rj[3] = {S(u, 0), S(u, 1), S(u, 2)};
            float zz[3];  // z_j again from r_j (the form's arithmetic: the same bits)
            lat_z(czA[cls], czB[cls], cls, rj, zz);
            fused_row_dots(czA, czB, cls, u0, zz, an, d);
            const uint32_t po = opub[u] != kResNone ? 48u * ((j & 1u) * ra.npub + opub[u]) : kResOob;
            const uint32_t tag = ra.tag0 + j + 1u;
            const u32x4 g0 = {__float_as_uint(rj[0]), __float_as_uint(rj[1]), __float_as_uint(rj[2]), tag},
                        g1 = {__float_as_uint(an[0]), __float_as_uint(an[1]), __float_as_uint(an[2]), tag},
                        g2 = {__float_as_uint(u0[0]), __float_as_uint(u0[1]), __float_as_uint(u0[2]), tag};
            st4_sc1(rpub, po, g0);
            st4_sc1(rpub, po + 16u, g1);
            st4_sc1(rpub, po + 32u, g2);
            if constexpr (multi)  // a send-plane node: its Ap_j granule into the neighbour's mailbox, at its ghost position
            {
                const uint32_t jp = j & 1u, e = rw >> 24, pos = 16u * (rw & 0xFFFFFFu);
                const __amdgpu_buffer_rsrc_t d0 = sized_rsrc(jp ? ra.pa.rdst[0][1] : ra.pa.rdst[0][0], ra.pa.rdst_bytes[0]),
                                             d1 = sized_rsrc(jp ? ra.pa.rdst[1][1] : ra.pa.rdst[1][0], ra.pa.rdst_bytes[1]);
                const uint32_t o0 = rw != kResNone && e == 0u ? pos : kResOob, o1 = rw != kResNone && e == 1u ? pos : kResOob;
                st4_sys(d0, o0, g1);
                st4_sys(d1, o1, g1);
            }
        }
        stamp(j, 4);
        block_sum_lds<kResNT, kFusedShares>(d, red);
        stamp(j, 5);
        if (tid < (uint32_t)kFusedShares)  // one tagged granule per share: {lo, hi, tag, -}
        {
            double v = d[0];
#pragma unroll
            for (int q = 1; q < kFusedShares; ++q)
                v = tid == (uint32_t)q ? d[q] : v;
            st4_sc1(rsh, 16u * (((j & 1u) * G + b) * kFusedShares + tid),
                    u32x4{(uint32_t)__double2loint(v), (uint32_t)__double2hiint(v), ra.tag0 + j + 1u, 0u});
        }
        stamp(j, 6);
    }
    // the stop at phase j: x_(j-1) and r_(j-1) (phase j made no update)
    const __amdgpu_buffer_rsrc_t wx = sized_rsrc(ra.x, vbytes), wr = sized_rsrc(ra.r, vbytes);
#pragma unroll
    for (int u = 0; u < NPT; ++u)
    {
        const uint32_t nb = on[u] != kResNone ? 12u * on[u] : 12u * kLatOob3;
        const u32x3 vx = {__float_as_uint(S(u, 6)), __float_as_uint(S(u, 7)), __float_as_uint(S(u, 8))},
                    vr = {__float_as_uint(S(u, 0)), __float_as_uint(S(u, 1)), __float_as_uint(S(u, 2))};
        __builtin_amdgcn_raw_buffer_store_b96(vx, wx, nb, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b96(vr, wr, nb, 0, 0);
    }
}

template <bool SYM, class E, int NPT, int NPH, bool MR>
void launch_resident_e(const DevSys &s, const ResArgs &ra, unsigned G, size_t lds, hipStream_t st, hipEvent_t e0,
                       hipEvent_t e1)
{
    const auto k = k_pcg_resident<SYM, E, NPT, NPH, MR>;
    if (e0 && e1)
        hipExtLaunchKernelGGL(k, dim3(G), dim3(kResNT), lds, st, e0, e1, 0, s, ra, s.t.lcoef);
    else
        k<<<G, kResNT, lds, st>>>(s, ra, s.t.lcoef);
}

template <int NPT, int NPH, bool MR>
void launch_resident_n(const DevSys &s, const ResArgs &ra, unsigned G, size_t lds, hipStream_t st, hipEvent_t e0,
                       hipEvent_t e1)
{
    if (s.t.lhex)
        s.t.lsym ? launch_resident_e<true, LatHex, NPT, NPH, MR>(s, ra, G, lds, st, e0, e1)
                 : launch_resident_e<false, LatHex, NPT, NPH, MR>(s, ra, G, lds, st, e0, e1);
    else
        s.t.lsym ? launch_resident_e<true, LatKuhn, NPT, NPH, MR>(s, ra, G, lds, st, e0, e1)
                 : launch_resident_e<false, LatKuhn, NPT, NPH, MR>(s, ra, G, lds, st, e0, e1);
}

template <int NPT, int NPH, bool MR>
size_t res_static_lds(const DevSys &s)
{
    const auto k = s.t.lhex ? (s.t.lsym ? k_pcg_resident<true, LatHex, NPT, NPH, MR>
                                        : k_pcg_resident<false, LatHex, NPT, NPH, MR>)
                            : (s.t.lsym ? k_pcg_resident<true, LatKuhn, NPT, NPH, MR>
                                        : k_pcg_resident<false, LatKuhn, NPT, NPH, MR>);
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k)) == hipSuccess ? a.sharedSizeBytes : 0;
}

template <int NPT, int NPH, bool MR>
int res_bpc(const DevSys &s, size_t lds)
{
    int bpc = 0;
    const auto k = s.t.lhex ? (s.t.lsym ? k_pcg_resident<true, LatHex, NPT, NPH, MR>
                                        : k_pcg_resident<false, LatHex, NPT, NPH, MR>)
                            : (s.t.lsym ? k_pcg_resident<true, LatKuhn, NPT, NPH, MR>
                                        : k_pcg_resident<false, LatKuhn, NPT, NPH, MR>);
    // the image is dynamic LDS beside ~100 KB of static arrays: allow the workgroup its size (gfx950: 160 KB)
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k, kResNT, lds) != hipSuccess)
        return 0;
    return bpc;
}
}  // namespace

// ---- the resident solve (the kernel above): one launch per PCG solve ------------------------------------------------
// the instantiations: <= 3 own + 2 halo entries per thread, state in registers (boxes of <= 1,536 nodes and <= 1,024
// ring entries: C2's 14 x 10 x 10), or <= 4 + 3 with the state in LDS (<= 2,048 nodes, <= 1,536 entries: the C3 / 8
// slab's 19 x 19 x 5); 2 waves per SIMD, one workgroup per CU, no scratch
size_t resident_static_lds(const DevSys &s, bool small, bool shard)
{
    if (small)
        return shard ? res_static_lds<3, 2, true>(s) : res_static_lds<3, 2, false>(s);
    return shard ? res_static_lds<4, 3, true>(s) : res_static_lds<4, 3, false>(s);
}

int resident_blocks_per_cu(const DevSys &s, unsigned npt, unsigned nph, size_t lds, bool shard)
{
    if (npt <= 3 && nph <= 2)
        return shard ? res_bpc<3, 2, true>(s, lds) : res_bpc<3, 2, false>(s, lds);
    if (npt <= 4 && nph <= 3)
        return shard ? res_bpc<4, 3, true>(s, lds) : res_bpc<4, 3, false>(s, lds);
    return 0;
}

void launch_pcg_resident(cwf_hip_system *h, uint32_t max_it, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    const ResidentPlan &rp = h->res;
    ResArgs ra{};
    ra.ctl = h->ctl;
    ra.hist = h->hist;
    ra.hdr = rp.hdr;
    ra.own = rp.own;
    ra.halo = rp.halo;
    ra.tcoef = rp.tcoef;
    ra.own_stride = rp.own_stride;
    ra.halo_stride = rp.halo_stride;
    ra.pub = rp.pub;
    ra.npub = rp.npub;
    ra.sh = rp.sh;
    ra.tag0 = h->res.tag;  // (resident.cpp advances it past this solve's phases)
    ra.x = h->x;
    ra.r = h->r;
    ra.max_it = max_it;
    if (rp.shard)
        peer_resident_args(h, ra.pa);
    else
        ra.pa = ResPeerArgs{};
    static uint64_t *trace = nullptr;  // diagnostic: CWF_RESIDENT_TRACE=path appends phase CWF_FUSED_TRACE_IT's stamps
    static unsigned trace_n = 0;
    const char *tp = knob("CWF_RESIDENT_TRACE");
    if (tp && trace_n < rp.G)
    {
        if (trace)
            (void)hipFree(trace);
        trace = nullptr;
        trace_n = hipMalloc(reinterpret_cast<void **>(&trace), 64ull * rp.G) == hipSuccess ? rp.G : 0u;
    }
    if (tp && trace)
    {
        const char *at = knob("CWF_FUSED_TRACE_IT");
        ra.trace = trace;
        ra.trace_j = at ? (uint32_t)atoi(at) : 50u;
        (void)hipMemsetAsync(trace, 0, 64ull * rp.G, st);
    }
    if (rp.npt <= 3 && rp.nph <= 2)
        rp.shard ? launch_resident_n<3, 2, true>(h->ds, ra, rp.G, rp.lds, st, e0, e1)
                 : launch_resident_n<3, 2, false>(h->ds, ra, rp.G, rp.lds, st, e0, e1);
    else
        rp.shard ? launch_resident_n<4, 3, true>(h->ds, ra, rp.G, rp.lds, st, e0, e1)
                 : launch_resident_n<4, 3, false>(h->ds, ra, rp.G, rp.lds, st, e0, e1);
    if (tp && trace)
    {
        std::vector<uint64_t> v(8ull * rp.G);
        if (hipStreamSynchronize(st) == hipSuccess &&
            hipMemcpy(v.data(), trace, v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess)
            if (FILE *f = std::fopen(tp, "a"))
            {
                std::fprintf(f, "# resident phase %u grid %u boxes %ux%ux%u\n", ra.trace_j, rp.G, rp.dims[0], rp.dims[1],
                             rp.dims[2]);
                for (unsigned b = 0; b < rp.G; ++b)
                {
                    std::fprintf(f, "%u", b);
                    for (int i = 0; i < 8; ++i)
                        std::fprintf(f, " %llu", (unsigned long long)v[8ull * b + i]);
                    std::fprintf(f, "\n");
                }
                std::fclose(f);
            }
    }
}

}  // namespace cwf

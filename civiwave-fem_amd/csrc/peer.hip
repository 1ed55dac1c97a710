// peer.hip -- the PEER communicator: device-initiated exchange steps over IPC-mapped mailboxes (SURVEY.md 8e,
// VERDICT r3 item 4). One process per rank, as RCCL; an exchange step (the all-gathers of per-rank scalar slots
// and the halos of up to three vectors, comm_exchange_vecs) is ONE launch on the rank's stream instead of an RCCL
// group, k_peer_step, in three phases:
//
//   push    every workgroup gathers its share of the send rows straight from the vectors (send_idx: no pack pass)
//           and stores them into the neighbours' mailboxes (write-through system-scope stores: over xGMI to the
//           neighbour's HBM; the same device's memory under IPC on one GPU), workgroup 0 this rank's scalar slots
//           (folded from the rank's shares in the step, PeerFold) into every peer's; each workgroup waits for its
//           stores and takes a ticket; the last one releases at system scope and stores the step's epoch into
//           every peer's flag for this rank (system-scope atomic store);
//   wait    every workgroup polls this rank's flags, one lane per peer, until every peer has reached the epoch
//           (bounded: a peer that has not arrived after 10 s ends the solve with CWF_ERR_COMM instead of a hang), then acquires
//           at system scope;
//   unpack  its share of the received ghost rows and scalar slots into their vectors / slots (system-scope loads).
//
// The fused lattice iteration on PEER shards runs the same protocol inside its own launches instead (lattice_fused.inc
// fused_peer_wait / fused_peer_publish; peer_fused_* below set up their arguments): the launch's Ap send rows and
// rank totals are pushed by the launch, the flags raised by its last workgroup, and the next launch's prologue waits.
//
// Workgroups wait for peers, not for each other, and the grid is small (<= 64 workgroups of 1024 threads, resident
// together), so every workgroup reaches its ticket. The ticket is an agent-scope add (acq_rel in k_peer_step, relaxed in
// the fused launch, where the release's L2 write-back cost 14 us per launch): what it orders are the
// workgroups' write-through (system-scope) stores, each already acknowledged (every storing wave waits vmcnt(0)
// behind a workgroup barrier before its lane takes the ticket), so the last arriver's system-scope release fence and
// flag store come after every workgroup's stores have reached the receiver's memory. Round 4's first form was three launches (push, wait, unpack)
// after the pack pass: 13.7 us per step between two processes on one GPU (profiles/r04ev_peer.log).
//
// A comm error is sticky: a step whose wait times out sets the communicator's device error word, and every
// later step returns at entry (setting the solve's CWF_ERR_COMM again) instead of pushing and spinning to its own
// timeout, so a dead peer ends a queued batch of exchange steps in one timeout, and the prologue's error survives
// the init kernel that rewrites the control block.
//
// A mailbox (one allocation per rank, exported with hipIpcGetMemHandle: uncached device memory,
// hipDeviceMallocUncached, so another device's stores over xGMI are seen without relying on the receiver's L2 holding
// no stale copy; fine-grained or plain device memory where that allocation or its IPC export is refused, recorded in
// cwf_hip_comm_peer_mailbox_kind) is a header with the rank's receive layout
// (where each neighbour's ghosts go, read once by the peers at connect), one 64-B flag line per peer, and two
// copies (by epoch parity) of the scalar-slot area and of the ghost receive area. Two copies suffice: a rank can
// only push step e + 2 after waiting on step e + 1 of the receiver, which the receiver pushes after unpacking step
// e. Only the FAST schedules go through it (slots of <= 8 doubles); PARITY's chunk-partial all-gathers stay on
// RCCL / LOCAL.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cwf_internal.hpp"
#include "reduce.hpp"

#define HIPTRY(h, expr)                                                                                        \
    do                                                                                                         \
    {                                                                                                          \
        hipError_t e__ = (expr);                                                                               \
        if (e__ != hipSuccess)                                                                                 \
            return hip_fail((h), e__, #expr);                                                                  \
    } while (0)

namespace cwf
{
namespace
{
constexpr uint64_t kPeerMagic = 0x43574650454552ull;  // "CWFPEER"
constexpr size_t kHdrBytes = 4096, kFlagLine = 64, kSlot = 8;  // kSlot doubles per rank and gather
constexpr int kMaxPeerGathers = 2;
constexpr int kPeerThreads = 1024;
constexpr uint64_t kPeerTimeoutTicks = 10ull * 100000000ull;  // a wait gives a peer 10 s (s_memrealtime: 100 MHz)  // the fold of a rank's shares is k_fold_pair's 1024-thread fold_all

struct MboxHeader  // at offset 0 of every mailbox
{
    uint64_t magic, nranks, nghost, recv_off[kMaxPeers], recv_cnt[kMaxPeers];
    char bus[32];  // the owner's device (hipDeviceGetPCIBusId): peers on the same device are a rehearsal
};
static_assert(sizeof(MboxHeader) <= kHdrBytes, "mailbox header");

inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
inline size_t off_flags() { return kHdrBytes; }
inline size_t off_gath(int n) { return align256(off_flags() + kFlagLine * (size_t)n); }
inline size_t gath_bytes(int n) { return (size_t)kMaxPeerGathers * n * kSlot * sizeof(double); }  // one parity
inline size_t off_recv(int n) { return align256(off_gath(n) + 2 * gath_bytes(n)); }
inline size_t recv_bytes(uint64_t nghost) { return kMaxHaloVecs * 3 * nghost * sizeof(float); }  // one parity
// the resident solve's area after the receive areas (resident.hip): per parity the rank totals, then the ghosts' Ap
// granules
inline size_t off_res(int n, uint64_t nghost) { return align256(off_recv(n) + 2 * recv_bytes(nghost)); }
inline size_t res_tot_bytes(int n) { return align256(80ull * (size_t)n); }
inline size_t res_par_bytes(int n, uint64_t nghost) { return align256(res_tot_bytes(n) + 16ull * nghost); }

struct PeerStep
{
    // push
    const float *vec[kMaxHaloVecs];  // the halo vectors (node-interleaved, 3 floats per node)
    const uint32_t *send_idx;        // [nsend] owned local node ids, neighbour k's at src_off[k] ..
    uint32_t nv, nnbr;
    float *dst[kMaxPeers];            // per neighbour k: its receive area (this parity), my ghosts' first float
    uint64_t dst_vstride[kMaxPeers];  // floats between vectors there (3 nghost of the neighbour)
    uint64_t src_off[kMaxPeers], cnt[kMaxPeers];  // my send segment for k (nodes)
    uint64_t total;                   // sum over k of cnt (nodes)
    uint32_t ng, gcount[kMaxPeerGathers];
    const double *gsrc[kMaxPeerGathers];  // my slot of gather q
    double *gdst[kMaxPeers];          // per rank p: p's gather area (this parity), my slot of gather 0
    uint32_t *flag[kMaxPeers];        // per rank p: p's flag line for my rank
    uint32_t nranks, rank, epoch;
    uint32_t *cnt_ticket;
    uint32_t *sticky;  // the communicator's device error word (CWF_ERR_COMM once a wait timed out)
    // wait
    const uint32_t *flags;  // my mailbox's flag lines
    Ctl *ctl;
    // unpack
    const float *recv;        // this parity's receive area
    uint64_t nghost, ghost0;  // ghosts are local nodes ghost0 .. ghost0 + nghost
    float *out[kMaxHaloVecs];
    const double *gath;  // this parity's gather area
    double *gbuf[kMaxPeerGathers];
    // fold (fn > 0): gather 0's own slot(s) from the rank's shares fa / fb, folded by workgroup 0
    const double *fa, *fb;
    uint32_t fn, fk5;  // fk5 > 0: five arrays fa[q fk5 + i] (the fused iteration's shares)
};

__global__ __launch_bounds__(kPeerThreads) void k_peer_step(PeerStep a)
{
    constexpr uint32_t NT = kPeerThreads;
    // a peer timed out in an earlier step: push nothing, wait for nothing; end the solve (again) with CWF_ERR_COMM
    if (__hip_atomic_load(a.sticky, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
    {
        if (blockIdx.x == 0 && threadIdx.x == 0)
        {
            a.ctl->error = CWF_ERR_COMM;
            a.ctl->error_iter = (int)a.epoch;
            a.ctl->active = 0;
        }
        return;
    }
    // (0) workgroup 0: this rank's scalars, folded as k_fold_pair folds them, kept for the push and stored locally
    __shared__ double red[5 * (NT / 64)], gv[kSlot];
    if (blockIdx.x == 0 && a.fn && a.fk5)
    {
        double v[5];
        fold_k<NT, 5, 256>(a.fa, a.fn, a.fk5, red, v);  // k_fused_rank_totals' order, bit for bit
        if (threadIdx.x == 0)
        {
            double *own = const_cast<double *>(a.gsrc[0]);
            for (int q = 0; q < (int)kSlot; ++q)
            {
                gv[q] = q < 5 ? v[q] : 0.0;
                own[q] = gv[q];
            }
        }
        __syncthreads();
    }
    else if (blockIdx.x == 0 && a.fn)
    {
        const double ta = fold_all<NT>(a.fa, a.fn, red);
        const double tb = a.fb ? fold_all<NT>(a.fb, a.fn, red) : 0.0;
        if (threadIdx.x == 0)
        {
            gv[0] = ta;
            gv[1] = tb;
            double *own = const_cast<double *>(a.gsrc[0]);
            own[0] = ta;
            if (a.fb)
                own[1] = tb;
        }
        __syncthreads();
    }
    // (1) push: node item t of the flattened (vector, neighbour, node) space, workgroup-strided
    const uint64_t items = a.total * a.nv;
    for (uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x; t < items; t += (uint64_t)gridDim.x * NT)
    {
        uint64_t r = t % a.total;
        const uint32_t v = (uint32_t)(t / a.total);
        uint32_t k = 0;
        while (k + 1 < a.nnbr && r >= a.cnt[k])
            r -= a.cnt[k++];
        const float *src = a.vec[v] + 3ull * a.send_idx[a.src_off[k] + r];
        float *d = a.dst[k] + a.dst_vstride[k] * v + 3 * r;
        const float x0 = src[0], x1 = src[1], x2 = src[2];
        // write-through (system scope): nothing is left dirty in this XCD's L2, so no workgroup needs an L2
        // write-back fence before its ticket
        __hip_atomic_store(d + 0, x0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d + 1, x1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d + 2, x2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (blockIdx.x == 0 && threadIdx.x < a.nranks * kMaxPeerGathers * kSlot)
    {
        const uint32_t p = threadIdx.x / (kMaxPeerGathers * kSlot), q = (threadIdx.x / kSlot) % kMaxPeerGathers,
                       j = threadIdx.x % kSlot;
        if (p != a.rank && q < a.ng && j < a.gcount[q])
            __hip_atomic_store(a.gdst[p] + (size_t)q * a.nranks * kSlot + j, q == 0 && a.fn ? gv[j] : a.gsrc[q][j],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // every storing wave waits for its write-through stores, then one lane takes the workgroup's ticket: the
    // hand-off of the MI355X guide's measured-forms table, row 1 (sc0 sc1 stores, each wave's vmcnt(0), a barrier,
    // one agent-scope add per workgroup, the last adder told by the returned value); the last arriver then orders
    // the whole launch's stores before its flag stores with a system-scope release, and the consumer side keeps
    // its acquire. The ticket is acq_rel as well (the release formally orders the workgroup's
    // stores before its add, the acquire the last arriver's flag stores after every add): measured free here (8.3-9.0
    // us per step relaxed, 8.3-9.4 acq_rel, same round; profiles/r06s_ticket_acq_rel.txt), unlike the fused launch's
    // ticket (lattice_fused.inc fused_peer_publish: +14 us per launch, kept relaxed)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
    {
        // one workgroup (the scalar-only p.Ap step) is its own last arriver: no ticket round trip
        const uint32_t old = gridDim.x == 1 ? 0u
                                            : __hip_atomic_fetch_add(a.cnt_ticket, 1u, __ATOMIC_ACQ_REL,
                                                                     __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == gridDim.x)
        {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
            for (uint32_t p = 0; p < a.nranks; ++p)
                if (p != a.rank)
                    __hip_atomic_store(a.flag[p], a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (gridDim.x > 1)
                __hip_atomic_store(a.cnt_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // (2) wait: wave 0, lane p polls peer p's flag line
    __shared__ int ok_s;
    if (threadIdx.x < 64)
    {
        const uint32_t p = threadIdx.x;
        bool ok = true;
        if (p < a.nranks && p != a.rank)
        {
            const uint32_t *f = a.flags + (kFlagLine / 4) * p;
            uint32_t spins = 0;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz wall clock
            while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch)
            {
                __builtin_amdgcn_s_sleep(4);
                if ((++spins & 63u) == 0u && __builtin_amdgcn_s_memrealtime() - t0 > kPeerTimeoutTicks)
                {
                    ok = false;  // the peer is gone
                    break;
                }
            }
        }
        const bool all = __all(ok);
        if (threadIdx.x == 0)
            ok_s = all ? 1 : 0;
    }
    __syncthreads();
    if (!ok_s)
    {
        if (threadIdx.x == 0)
            __hip_atomic_store(a.sticky, (uint32_t)CWF_ERR_COMM, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (blockIdx.x == 0 && threadIdx.x == 0)
        {
            a.ctl->error = CWF_ERR_COMM;
            a.ctl->error_iter = (int)a.epoch;
            a.ctl->active = 0;
        }
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: an invalidate only (no L2 write-back)
    // (3) unpack
    const uint64_t per = 3 * a.nghost;
    for (uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x; t < per * a.nv; t += (uint64_t)gridDim.x * NT)
    {
        const uint32_t v = (uint32_t)(t / per);
        const uint64_t i = t % per;
        a.out[v][3 * a.ghost0 + i] = __hip_atomic_load(a.recv + per * v + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (blockIdx.x == 0 && threadIdx.x < a.nranks * kMaxPeerGathers * kSlot)
    {
        const uint32_t p = threadIdx.x / (kMaxPeerGathers * kSlot), q = (threadIdx.x / kSlot) % kMaxPeerGathers,
                       j = threadIdx.x % kSlot;
        if (p != a.rank && q < a.ng && j < a.gcount[q])
            a.gbuf[q][(size_t)p * a.gcount[q] + j] = __hip_atomic_load(a.gath + ((size_t)q * a.nranks + p) * kSlot + j,
                                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

// the mailbox memory: uncached device memory first (coherent with another device's xGMI stores by construction),
// then fine-grained, then plain hipMalloc, each only if its IPC export works too (a handle that cannot be exported
// is no mailbox); cm->mbox_kind records which (CWF_PEER_MAILBOX_*)
int peer_alloc_mailbox(cwf_hip_system *h, size_t bytes)
{
    cwf_hip_comm *cm = h->comm;
    const unsigned flags[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
    const int kinds[2] = {CWF_PEER_MAILBOX_UNCACHED, CWF_PEER_MAILBOX_FINEGRAINED};
    for (int i = 0; i < 2; ++i)
    {
        void *p = nullptr;
        if (hipExtMallocWithFlags(&p, bytes, flags[i]) != hipSuccess || !p)
        {
            (void)hipGetLastError();
            continue;
        }
        hipIpcMemHandle_t m;
        if (hipIpcGetMemHandle(&m, p) != hipSuccess)
        {
            (void)hipGetLastError();
            (void)hipFree(p);
            continue;
        }
        cm->mbox = p;
        cm->mbox_kind = kinds[i];
        return 0;
    }
    if (hipMalloc(&cm->mbox, bytes) != hipSuccess)
        return set_error(h, CWF_ERR_ALLOC, "failed to allocate the peer mailbox", "bytes=" + std::to_string(bytes));
    cm->mbox_kind = CWF_PEER_MAILBOX_DEVICE;
    return 0;
}

// attach of a PEER comm's member: the mailbox with this rank's receive layout in its header
int peer_attach(cwf_hip_system *h)
{
    cwf_hip_comm *cm = h->comm;
    const int n = cm->nranks;
    const uint64_t nghost = h->ds.N - h->ds.Nown;
    const size_t bytes = off_res(n, nghost) + 2 * res_par_bytes(n, nghost);
    if (int st = peer_alloc_mailbox(h, bytes))
        return st;
    cm->mbox_bytes = bytes;
    // the ticket (line 0) and the sticky error word (line 1), on lines of their own
    if (hipMalloc(reinterpret_cast<void **>(&cm->ticket), 256) != hipSuccess)
        return set_error(h, CWF_ERR_ALLOC, "failed to allocate device buffer");
    HIPTRY(h, hipMemset(cm->mbox, 0, bytes));
    HIPTRY(h, hipMemset(cm->ticket, 0, 256));
    MboxHeader hd{};
    hd.magic = kPeerMagic;
    hd.nranks = (uint64_t)n;
    hd.nghost = nghost;
    for (int p = 0; p < kMaxPeers; ++p)
        hd.recv_off[p] = ~0ull;
    for (size_t k = 0; k < h->nbr.size(); ++k)
    {
        hd.recv_off[h->nbr[k]] = h->recv_off[k];
        hd.recv_cnt[h->nbr[k]] = h->recv_off[k + 1] - h->recv_off[k];
    }
    if (hipDeviceGetPCIBusId(hd.bus, (int)sizeof hd.bus, cm->device) != hipSuccess)
    {
        (void)hipGetLastError();
        std::snprintf(hd.bus, sizeof hd.bus, "device-%d", cm->device);
    }
    hd.bus[sizeof hd.bus - 1] = 0;
    HIPTRY(h, hipMemcpy(cm->mbox, &hd, sizeof hd, hipMemcpyHostToDevice));
    cm->peer_member = h;
    return 0;
}

void peer_release(cwf_hip_comm *cm)
{
    for (void *p : cm->peer_mbox)
        if (p)
            (void)hipIpcCloseMemHandle(p);
    cm->peer_mbox.clear();
    if (cm->mbox)
        (void)hipFree(cm->mbox);
    if (cm->ticket)
        (void)hipFree(cm->ticket);
    cm->mbox = nullptr;
    cm->ticket = nullptr;
}

int peer_exchange(cwf_hip_system *h, std::initializer_list<Gather> gathers, const std::vector<float *> &vecs,
                  const PeerFold *fold)
{
    cwf_hip_comm *cm = h->comm;
    const int n = cm->nranks;
    if (cm->peer_mbox.size() != (size_t)n)
        return set_error(h, CWF_ERR_COMM, "peer communicator not connected (cwf_hip_comm_peer_connect)");
    if (gathers.size() > (size_t)kMaxPeerGathers)
        return set_error(h, CWF_ERR_UNSUPPORTED, "the peer communicator carries at most two scalar all-gathers a step");
    for (const Gather &q : gathers)
        if (q.count > kSlot)
            return set_error(h, CWF_ERR_UNSUPPORTED, "the peer communicator carries the FAST schedule only",
                             "PARITY's chunk-partial all-gathers need RCCL or LOCAL");
    constexpr uint64_t NTP = kPeerThreads;
    const uint32_t epoch = ++cm->epoch;
    const uint32_t par = epoch & 1u;
    PeerStep a{};
    a.send_idx = h->send_idx;
    a.nv = (uint32_t)vecs.size();
    for (size_t v = 0; v < vecs.size(); ++v)
        a.vec[v] = a.out[v] = vecs[v];
    a.nnbr = (uint32_t)h->nbr.size();
    for (uint32_t k = 0; k < a.nnbr; ++k)
    {
        const int q = h->nbr[k];
        const uint64_t qg = cm->peer_nghost[q], qoff = cm->peer_recv_off[q];
        char *base = static_cast<char *>(cm->peer_mbox[q]) + off_recv(n) + par * recv_bytes(qg);
        a.dst[k] = reinterpret_cast<float *>(base) + 3 * qoff;
        a.dst_vstride[k] = 3 * qg;
        a.src_off[k] = h->send_off[k];
        a.cnt[k] = h->send_off[k + 1] - h->send_off[k];
        a.total += a.cnt[k];
    }
    a.ng = 0;
    for (const Gather &q : gathers)
    {
        a.gcount[a.ng] = (uint32_t)q.count;
        a.gsrc[a.ng] = h->*(q.buf) + (size_t)h->rank * q.count;
        a.gbuf[a.ng] = h->*(q.buf);
        ++a.ng;
    }
    for (int p = 0; p < n; ++p)
    {
        char *pb = static_cast<char *>(p == h->rank ? cm->mbox : cm->peer_mbox[p]);
        a.gdst[p] = reinterpret_cast<double *>(pb + off_gath(n) + par * gath_bytes(n)) + (size_t)h->rank * kSlot;
        a.flag[p] = reinterpret_cast<uint32_t *>(pb + off_flags() + kFlagLine * (size_t)h->rank);
    }
    a.nranks = (uint32_t)n;
    a.rank = (uint32_t)h->rank;
    a.epoch = epoch;
    a.cnt_ticket = cm->ticket;
    a.sticky = cm->ticket + 32;
    a.flags = reinterpret_cast<const uint32_t *>(static_cast<char *>(cm->mbox) + off_flags());
    a.ctl = h->ctl;
    const uint64_t nghost = h->ds.N - h->ds.Nown;
    a.recv = reinterpret_cast<const float *>(static_cast<char *>(cm->mbox) + off_recv(n) + par * recv_bytes(nghost));
    a.nghost = nghost;
    a.ghost0 = h->ds.Nown;
    a.gath = reinterpret_cast<const double *>(static_cast<char *>(cm->mbox) + off_gath(n) + par * gath_bytes(n));
    if (fold && a.ng)
    {
        a.fa = fold->a;
        a.fb = fold->b;
        a.fn = fold->n;
        a.fk5 = fold->k5_stride;
    }
    // one workgroup per 1024 pushed nodes or 4096 unpacked floats, <= 64 (all resident: every one reaches its
    // ticket)
    const uint64_t work = std::max<uint64_t>((a.total * a.nv + NTP - 1) / NTP, (3 * nghost * a.nv + 4 * NTP - 1) / (4 * NTP));
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(work, 64));
    k_peer_step<<<grid, kPeerThreads, 0, h->stream>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(h, e, "peer exchange launch");
}

// ---- the fused lattice iteration's in-kernel exchange (lattice_fused.inc: fused_peer_wait / fused_peer_publish) ----
bool peer_fused_eligible(cwf_hip_system *h)
{
    cwf_hip_comm *cm = h->comm;
    const char *on = knob("CWF_PEER_FUSED");
    if (!cm || cm->kind != 2 || cm->nranks < 2 || (on && atoi(on) == 0) || !h->ds.t.lat || h->ds.Nown >= h->ds.N ||
        cm->peer_mbox.size() != (size_t)cm->nranks || h->nbr.size() > 2 || h->lat_plane.size() != h->ds.t.lnz)
        return false;
    // every send segment is one whole owned plane in plane order: row (i, j) of plane k is its 3 (j nx + i)-th float
    const uint64_t nsend = h->send_off.empty() ? 0 : h->send_off.back();
    std::vector<uint32_t> idx(nsend);
    if (nsend && hipMemcpy(idx.data(), h->send_idx, nsend * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return false;
    const uint32_t per = h->ds.t.lnx * h->ds.t.lny;
    h->px_send_k[0] = h->px_send_k[1] = -1;
    for (size_t k = 0; k < h->nbr.size(); ++k)
    {
        const uint64_t a = h->send_off[k], b = h->send_off[k + 1];
        if (b - a != per)
            return false;
        int32_t plane = -1;
        for (uint32_t q = 0; q < h->ds.t.lnz; ++q)
            if (h->lat_plane[q] == idx[a] && h->lat_plane[q] + per <= h->ds.Nown)
                plane = (int32_t)q;
        if (plane < 0)
            return false;
        for (uint64_t r = 0; r < per; ++r)
            if (idx[a + r] != idx[a] + r)
                return false;
        h->px_send_k[k] = plane;
    }
    // ranks on one device (a rehearsal; the mailbox headers' PCI bus ids): a rank's launch j waits, resident, for the
    // others' launch j - 1, so all the grids must fit together (two 436-workgroup C2 grids in 512 slots measured
    // slower than the exchange step: profiles/r05k_peer_rehearsal.txt)
    bool same = false;
    for (int p = 0; p < cm->nranks; ++p)
        same = same || (p != cm->rank && cm->peer_same_device[p] != 0);
    if (same && (uint64_t)h->fused_grid * (uint64_t)cm->nranks > pcg_lattice_resident_count(h->ds))
        return false;
    return true;
}

void peer_fused_args(const cwf_hip_system *h, unsigned j, FusedPeerArgs &pe, const double **gath_prev)
{
    const cwf_hip_comm *cm = h->comm;
    const int n = cm->nranks;
    const uint32_t epoch = h->px_ebase + j + 1u, par = epoch & 1u, prev = (epoch - 1u) & 1u;
    pe = FusedPeerArgs{};
    for (size_t k = 0; k < 2; ++k)
    {
        pe.send_k[k] = -1;
        if (k >= h->nbr.size() || h->px_send_k[k] < 0)
            continue;
        const int q = h->nbr[k];
        const uint64_t qg = cm->peer_nghost[q], qoff = cm->peer_recv_off[q];
        char *base = static_cast<char *>(cm->peer_mbox[q]) + off_recv(n) + par * recv_bytes(qg);
        pe.dst[k] = reinterpret_cast<float *>(base) + 3 * qoff;
        pe.dst_bytes[k] = (uint32_t)(12ull * (h->send_off[k + 1] - h->send_off[k]));
        pe.send_k[k] = h->px_send_k[k];
    }
    for (int p = 0; p < n; ++p)
    {
        char *pb = static_cast<char *>(p == h->rank ? cm->mbox : cm->peer_mbox[p]);
        pe.gdst[p] = reinterpret_cast<double *>(pb + off_gath(n) + par * gath_bytes(n)) + (size_t)h->rank * kSlot;
        pe.flag[p] = reinterpret_cast<uint32_t *>(pb + off_flags() + kFlagLine * (size_t)h->rank);
    }
    static_assert(kFlagLine == 64, "fused_peer_wait polls flags[16 p]");
    pe.flags = reinterpret_cast<const uint32_t *>(static_cast<char *>(cm->mbox) + off_flags());
    pe.ticket = cm->ticket + 16;
    pe.sticky = cm->ticket + 32;
    pe.done = cm->ticket + 48;
    const uint64_t nghost = h->ds.N - h->ds.Nown;
    pe.arecv = reinterpret_cast<const float *>(static_cast<char *>(cm->mbox) + off_recv(n) + prev * recv_bytes(nghost));
    pe.epoch = epoch;
    pe.nranks = (uint32_t)n;
    pe.rank = (uint32_t)h->rank;
    // gather 0 of the previous epoch: rank p's totals at [kSlot p]
    *gath_prev = reinterpret_cast<const double *>(static_cast<char *>(cm->mbox) + off_gath(n) + prev * gath_bytes(n));
}

size_t peer_resident_bytes(int nranks, uint64_t nghost) { return 2 * res_par_bytes(nranks, nghost); }

int peer_resident_clear(cwf_hip_system *h)
{
    const cwf_hip_comm *cm = h->comm;
    const uint64_t nghost = h->ds.N - h->ds.Nown;
    char *base = static_cast<char *>(cm->mbox) + off_res(cm->nranks, nghost);
    HIPTRY(h, hipMemset(base, 0, peer_resident_bytes(cm->nranks, nghost)));
    return 0;
}

void peer_resident_args(const cwf_hip_system *h, ResPeerArgs &pa)
{
    const cwf_hip_comm *cm = h->comm;
    const int n = cm->nranks;
    pa = ResPeerArgs{};
    pa.nranks = (uint32_t)n;
    pa.rank = (uint32_t)h->rank;
    const uint64_t nghost = h->ds.N - h->ds.Nown;
    for (size_t k = 0; k < 2 && k < h->nbr.size(); ++k)
    {
        const int q = h->nbr[k];
        const uint64_t qg = cm->peer_nghost[q], qoff = cm->peer_recv_off[q];
        for (uint32_t par = 0; par < 2; ++par)
        {
            char *base = static_cast<char *>(cm->peer_mbox[q]) + off_res(n, qg) + par * res_par_bytes(n, qg) +
                         res_tot_bytes(n);
            pa.rdst[k][par] = reinterpret_cast<float *>(base + 16ull * qoff);
        }
        pa.rdst_bytes[k] = (uint32_t)(16ull * (h->send_off[k + 1] - h->send_off[k]));
    }
    for (uint32_t par = 0; par < 2; ++par)
    {
        const char *mine = static_cast<const char *>(cm->mbox) + off_res(n, nghost) + par * res_par_bytes(n, nghost);
        pa.grecv[par] = reinterpret_cast<const float *>(mine + res_tot_bytes(n));
        pa.tot_mine[par] = reinterpret_cast<const uint32_t *>(mine);
        for (int p = 0; p < n; ++p)
        {
            const uint64_t pg = p == h->rank ? nghost : cm->peer_nghost[p];
            char *pb = static_cast<char *>(p == h->rank ? cm->mbox : cm->peer_mbox[p]);
            pa.tot[p][par] = reinterpret_cast<uint32_t *>(pb + off_res(n, pg) + par * res_par_bytes(n, pg));
        }
    }
    pa.grecv_bytes = (uint32_t)(16ull * nghost);
}

int peer_fused_begin(cwf_hip_system *h)
{
    cwf_hip_comm *cm = h->comm;
    h->px_ebase = cm->epoch;
    HIPTRY(h, hipMemsetAsync(cm->ticket + 16, 0, sizeof(uint32_t), h->stream));
    return 0;
}

int peer_fused_end(cwf_hip_system *h)
{
    cwf_hip_comm *cm = h->comm;
    uint32_t done = 0;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    HIPTRY(h, hipMemcpy(&done, cm->ticket + 48, sizeof done, hipMemcpyDeviceToHost));
    // launches that pushed: epochs ebase + 1 .. done (none: the solve ended at its prologue)
    if (done > h->px_ebase && done - h->px_ebase < (1u << 30))
        cm->epoch = done;
    return 0;
}

}  // namespace cwf

using namespace cwf;

extern "C" {

int cwf_hip_comm_create_peer(int32_t nranks, int32_t rank, int device, cwf_hip_comm **out)
{
    if (!out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    if (nranks < 1 || nranks > kMaxPeers || rank < 0 || rank >= nranks)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "rank out of range", "peer communicators hold <= 16 ranks");
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess)
        return hip_fail(nullptr, he, "hipSetDevice");
    cwf_hip_comm *cm = new (std::nothrow) cwf_hip_comm();
    if (!cm)
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    cm->kind = 2;
    cm->nranks = nranks;
    cm->rank = rank;
    cm->device = device;
    *out = cm;
    return 0;
}

int cwf_hip_comm_peer_handle(cwf_hip_comm *cm, uint8_t *handle)
{
    if (!cm || !handle || cm->kind != 2)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "not a peer communicator");
    if (!cm->mbox)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "attach the rank's handle first");
    (void)hipSetDevice(cm->device);
    hipIpcMemHandle_t m;
    const hipError_t e = hipIpcGetMemHandle(&m, cm->mbox);
    if (e != hipSuccess)
        return hip_fail(nullptr, e, "hipIpcGetMemHandle");
    static_assert(sizeof m <= CWF_IPC_HANDLE_BYTES, "ipc handle size");
    std::memset(handle, 0, CWF_IPC_HANDLE_BYTES);
    std::memcpy(handle, &m, sizeof m);
    return 0;
}

int cwf_hip_comm_peer_connect(cwf_hip_comm *cm, const uint8_t *handles)
{
    if (!cm || !handles || cm->kind != 2 || !cm->peer_member)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "attach the rank's handle to a peer communicator first");
    cwf_hip_system *h = cm->peer_member;
    (void)hipSetDevice(cm->device);
    const int n = cm->nranks;
    cm->peer_mbox.assign(n, nullptr);
    cm->peer_nghost.assign(n, 0);
    cm->peer_recv_off.assign(n, 0);
    cm->peer_same_device.assign(n, 1);
    MboxHeader mine{};
    HIPTRY(h, hipMemcpy(&mine, cm->mbox, sizeof mine, hipMemcpyDeviceToHost));
    for (int p = 0; p < n; ++p)
    {
        if (p == cm->rank)
            continue;
        hipIpcMemHandle_t m;
        std::memcpy(&m, handles + (size_t)p * CWF_IPC_HANDLE_BYTES, sizeof m);
        void *ptr = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&ptr, m, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess)
            return hip_fail(h, e, "hipIpcOpenMemHandle");
        cm->peer_mbox[p] = ptr;
        MboxHeader hd{};
        HIPTRY(h, hipMemcpy(&hd, ptr, sizeof hd, hipMemcpyDeviceToHost));
        if (hd.magic != kPeerMagic || hd.nranks != (uint64_t)n)
            return set_error(h, CWF_ERR_COMM, "peer mailbox does not match this communicator",
                             "peer=" + std::to_string(p));
        cm->peer_nghost[p] = hd.nghost;
        cm->peer_recv_off[p] = hd.recv_off[cm->rank];
        hd.bus[sizeof hd.bus - 1] = 0;
        cm->peer_same_device[p] = std::strncmp(hd.bus, mine.bus, sizeof hd.bus) == 0 ? 1 : 0;
    }
    // every neighbour expects exactly my send segment for it
    for (size_t k = 0; k < h->nbr.size(); ++k)
    {
        const int q = h->nbr[k];
        MboxHeader hd{};
        HIPTRY(h, hipMemcpy(&hd, cm->peer_mbox[q], sizeof hd, hipMemcpyDeviceToHost));
        if (hd.recv_off[cm->rank] == ~0ull || hd.recv_cnt[cm->rank] != h->send_off[k + 1] - h->send_off[k])
            return set_error(h, CWF_ERR_COMM, "halo plans disagree",
                             "rank=" + std::to_string(cm->rank) + "\npeer=" + std::to_string(q));
    }
    return 0;
}

// `steps` exchange steps shaped like the FAST iteration's second one (the {r.r, r.z} all-gather and the z halo;
// the first, p.Ap, has no halo) on h's stream, hipEvent-timed: the per-step latency the 8-GPU projection uses
// (every rank calls it). The untimed first step checks the halo's contents; z is clobbered (a solve recomputes it)
int cwf_hip_comm_time_exchange(cwf_hip_system *h, int32_t steps, double *us_per_step)
{
    if (!h || !us_per_step || steps < 1 || !h->sharded() || !h->comm)
        return set_error(h, CWF_ERR_ARGUMENT, "an attached handle and steps >= 1");
    if (h->comm->kind == 0 && h->nranks > 1)  // its exchange needs every member of the process (solve_pcg_group)
        return set_error(h, CWF_ERR_UNSUPPORTED, "time the exchange of a RCCL or PEER communicator");
    (void)hipSetDevice(h->device);
    hipEvent_t e0, e1;
    HIPTRY(h, hipEventCreate(&e0));
    HIPTRY(h, hipEventCreate(&e1));
    std::vector<cwf_hip_system *> g{h};
    std::vector<std::vector<float *>> vecs{{h->z}};
    // as the iteration runs it: with the fold of the update pass's shares (PEER folds them in the step itself)
    const PeerFold fold{h->part1, h->part2, fast_rrz_shares(h->ds, 0), 0};
    const auto step = [&]() {
        if (h->comm->kind == 2)
            return peer_exchange(h, {Gather{&cwf_hip_system::g_rrz, 2}}, {h->z}, &fold);
        fast_fold_rrz(h, 0, h->stream);
        return comm_exchange_vecs(g, {Gather{&cwf_hip_system::g_rrz, 2}}, vecs);
    };
    // the first (untimed) step carries a known pattern: every owned row of z = f(global id), the ghosts poisoned, and
    // afterwards every ghost row must hold its owner's f(global id). A transport that delivers stale or misplaced
    // rows (or none) fails the trial here instead of a solve later (bench.py --comm auto then takes RCCL)
    const uint64_t N = h->ds.N, Nown = h->ds.Nown;
    const bool check = h->node_gid.size() == N && N > Nown;
    const auto pat = [&](uint64_t n, int k) { return (float)((h->node_gid[n] * 3u + (uint64_t)k) % 4194304u + 1u); };
    std::vector<float> zh;
    if (check)
    {
        zh.assign(3 * N, std::nanf(""));
        for (uint64_t n = 0; n < Nown; ++n)
            for (int k = 0; k < 3; ++k)
                zh[3 * n + k] = pat(n, k);
        HIPTRY(h, hipMemcpyAsync(h->z, zh.data(), zh.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
    }
    // a step that timed out (a peer that never arrived, or a communicator already dead: its steps return at entry)
    // only shows in the control block: report it, then clear the solve fields so the next solve starts clean (the
    // communicator's sticky word stays set)
    const auto step_error = [&]() -> int {
        Ctl c{};
        HIPTRY(h, hipStreamSynchronize(h->stream));
        HIPTRY(h, hipMemcpy(&c, h->ctl, sizeof c, hipMemcpyDeviceToHost));
        if (!c.error)
            return 0;
        const int code = c.error, at = c.error_iter;
        c.error = 0;
        c.error_iter = 0;
        HIPTRY(h, hipMemcpy(h->ctl, &c, sizeof c, hipMemcpyHostToDevice));
        return set_error(h, code, code == CWF_ERR_COMM ? "peer exchange timed out" : "exchange step failed",
                         "step=" + std::to_string(at));
    };
    int st = step();  // warm
    if (!st)
        st = step_error();  // before the halo check: a timed-out step delivered nothing
    if (!st && check)
    {
        HIPTRY(h, hipStreamSynchronize(h->stream));
        HIPTRY(h, hipMemcpy(zh.data(), h->z, zh.size() * sizeof(float), hipMemcpyDeviceToHost));
        for (uint64_t n = Nown; n < N && !st; ++n)
            for (int k = 0; k < 3 && !st; ++k)
                if (!(zh[3 * n + k] == pat(n, k)))
                    st = set_error(h, CWF_ERR_COMM, "halo check failed",
                                   "ghost=" + std::to_string(n - Nown) + "\nglobal=" + std::to_string(h->node_gid[n]));
    }
    if (!st && hipEventRecord(e0, h->stream) != hipSuccess)
        st = set_error(h, CWF_ERR_HIP, "hipEventRecord");
    for (int i = 0; i < steps && !st; ++i)
        st = step();
    float ms = 0.f;
    if (!st && hipEventRecord(e1, h->stream) == hipSuccess && hipEventSynchronize(e1) == hipSuccess)
        (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *us_per_step = 1e3 * (double)ms / steps;
    if (st)
        return st;
    return step_error();
}

int cwf_hip_comm_peer_mailbox_kind(const cwf_hip_comm *cm, int *kind)
{
    if (!cm || !kind || cm->kind != 2)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "not a peer communicator");
    if (!cm->mbox)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "attach the rank's handle first");
    *kind = cm->mbox_kind;
    return 0;
}

}  // extern "C"

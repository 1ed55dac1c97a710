// comm.cpp -- communicators and the sharded FAST PCG schedule.
//
// Per PCG iteration a shard runs the same two kernels as one GPU, plus:
//   tiles -> fold p.Ap shares -> all-gather(1 f64/rank) -> update -> fold r.r / r.z shares
//         -> all-gather(2 f64/rank) -> halo(z)
// Every rank folds the gathered per-rank scalars in rank order, so alpha / beta / convergence are
// bitwise identical on all ranks and the control flow never diverges. Ghost rows are never
// reduced: their search direction is rebuilt locally from the exchanged z (p = z + beta p_old is
// the same fp32 expression on owner and ghost), so one halo of z per iteration suffices.
// RCCL is loaded with dlopen (torch's copy when already in the process, else /opt/rocm/lib); the
// LOCAL communicator runs all ranks of a decomposition in one process on one device (exchanges are
// device copies on one shared stream) and exists to test the decomposition on a single GPU.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only; the entry points are resolved at run time

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "cwf_internal.hpp"

namespace cwf
{
namespace
{

struct Rccl
{
    void *lib = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl *rccl(std::string *why)
{
    static Rccl r;
    static bool tried = false;
    static std::string err;
    if (!tried)
    {
        tried = true;
        void *lib = nullptr;
        if (const char *alt = knob("CWF_RCCL_LIB"))  // a test transport with the same entry points
        {
            lib = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
            if (!lib)
                err = std::string("dlopen ") + alt + " failed: " + dlerror();
        }
        else
        {
            lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // the process's RCCL (torch's), if any
            if (!lib)
                lib = dlopen("librccl.so.1", RTLD_NOW);
            if (!lib)
                lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
            if (!lib)
                err = std::string("dlopen librccl.so.1 failed: ") + dlerror();
        }
        if (lib)
        {
            bool ok = true;
            auto sym = [&](auto &fn, const char *name) {
                fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(lib, name));
                ok &= fn != nullptr;
            };
            sym(r.GetUniqueId, "ncclGetUniqueId");
            sym(r.CommInitRank, "ncclCommInitRank");
            sym(r.CommDestroy, "ncclCommDestroy");
            sym(r.AllGather, "ncclAllGather");
            sym(r.Send, "ncclSend");
            sym(r.Recv, "ncclRecv");
            sym(r.GroupStart, "ncclGroupStart");
            sym(r.GroupEnd, "ncclGroupEnd");
            sym(r.GetErrorString, "ncclGetErrorString");
            if (ok)
                r.lib = lib;
            else
                err = "librccl.so.1 lacks an expected entry point";
        }
    }
    if (!r.lib && why)
        *why = err;
    return r.lib ? &r : nullptr;
}

int nccl_fail(cwf_hip_system *h, ncclResult_t e, const char *what)
{
    const Rccl *r = rccl(nullptr);
    return set_error(h, CWF_ERR_COMM, std::string(what) + ": " + (r ? r->GetErrorString(e) : "rccl unavailable"),
                     "nccl=" + std::to_string((int)e));
}

#define NCCLTRY(h, expr)                                                                                       \
    do                                                                                                         \
    {                                                                                                          \
        ncclResult_t e__ = (expr);                                                                             \
        if (e__ != ncclSuccess)                                                                                \
            return nccl_fail((h), e__, #expr);                                                                 \
    } while (0)

#define HIPTRY(h, expr)                                                                                        \
    do                                                                                                         \
    {                                                                                                          \
        hipError_t e__ = (expr);                                                                               \
        if (e__ != hipSuccess)                                                                                 \
            return hip_fail((h), e__, #expr);                                                                  \
    } while (0)

}  // namespace

// One exchange step of a sharded solve: in-place all-gathers of per-rank double slots (slot r of buf is
// [r * count, (r + 1) * count)) and the halos of up to kMaxHaloVecs vectors (ghost rows <- the owners' values;
// vecs[m] lists member m's vectors, the same count for every member). Over RCCL every operation of the step is one
// ncclGroupStart/End, so the all-gathers and the halo send/recv pairs of an iteration go out as one launch.
int comm_exchange_vecs(const std::vector<cwf_hip_system *> &g, std::initializer_list<Gather> gathers,
                       const std::vector<std::vector<float *>> &vecs)
{
    cwf_hip_system *h0 = g[0];
    const size_t nv = vecs.empty() ? 0 : vecs[0].size();
    if (nv > kMaxHaloVecs)
        return set_error(h0, CWF_ERR_ARGUMENT, "too many halo vectors in one exchange");
    const bool gather = h0->nranks > 1;
    if (h0->comm && h0->comm->kind == 2)  // PEER: one launch that gathers its send rows from the vectors itself
        return (gather || nv) ? peer_exchange(h0, gathers, vecs.empty() ? std::vector<float *>{} : vecs[0]) : 0;
    for (size_t i = 0; i < g.size(); ++i)  // vector j's send segment at sendbuf + 3 nsend j
        for (size_t j = 0; j < nv; ++j)
            halo_pack(g[i], vecs[i][j], g[i]->stream, g[i]->sendbuf + 3 * g[i]->nsend * j);
    if (h0->comm && h0->comm->kind == 1)
    {
        if (!gather && !nv)
            return 0;
        const Rccl *r = rccl(nullptr);
        ncclComm_t c = static_cast<ncclComm_t>(h0->comm->nccl);
        NCCLTRY(h0, r->GroupStart());
        if (gather)
            for (const Gather &q : gathers)
            {
                double *b = h0->*(q.buf);
                NCCLTRY(h0, r->AllGather(b + (size_t)h0->rank * q.count, b, q.count, ncclFloat64, c, h0->stream));
            }
        for (size_t k = 0; k < h0->nbr.size(); ++k)
        {
            const size_t ns = h0->send_off[k + 1] - h0->send_off[k], nr = h0->recv_off[k + 1] - h0->recv_off[k];
            for (size_t j = 0; j < nv; ++j)
            {
                if (ns)
                    NCCLTRY(h0, r->Send(h0->sendbuf + 3 * (h0->nsend * j + h0->send_off[k]), 3 * ns, ncclFloat32,
                                        h0->nbr[k], c, h0->stream));
                if (nr)
                    NCCLTRY(h0, r->Recv(vecs[0][j] + 3 * ((size_t)h0->ds.Nown + h0->recv_off[k]), 3 * nr, ncclFloat32,
                                        h0->nbr[k], c, h0->stream));
            }
        }
        NCCLTRY(h0, r->GroupEnd());
        return 0;
    }
    // LOCAL (every rank in this process, one shared stream): device copies
    if (gather)
        for (const Gather &q : gathers)
            for (cwf_hip_system *dst : g)
                for (cwf_hip_system *src : g)
                    if (dst != src)
                        HIPTRY(dst, hipMemcpyAsync(dst->*(q.buf) + (size_t)src->rank * q.count,
                                                   src->*(q.buf) + (size_t)src->rank * q.count,
                                                   q.count * sizeof(double), hipMemcpyDeviceToDevice, dst->stream));
    if (!nv)
        return 0;
    // member m's ghosts from q = q's send segment for m
    for (size_t mi = 0; mi < g.size(); ++mi)
    {
        cwf_hip_system *m = g[mi];
        for (size_t k = 0; k < m->nbr.size(); ++k)
        {
            cwf_hip_system *q = g[m->nbr[k]];
            const auto it = std::find(q->nbr.begin(), q->nbr.end(), m->rank);
            if (it == q->nbr.end())
                return set_error(m, CWF_ERR_COMM, "halo plans disagree", "rank=" + std::to_string(m->rank));
            const size_t j = (size_t)(it - q->nbr.begin());
            const size_t nr = m->recv_off[k + 1] - m->recv_off[k], ns = q->send_off[j + 1] - q->send_off[j];
            if (nr != ns)
                return set_error(m, CWF_ERR_COMM, "halo plans disagree",
                                 "rank=" + std::to_string(m->rank) + "\npeer=" + std::to_string(q->rank));
            if (nr)
                for (size_t v = 0; v < nv; ++v)
                    HIPTRY(m, hipMemcpyAsync(vecs[mi][v] + 3 * ((size_t)m->ds.Nown + m->recv_off[k]),
                                             q->sendbuf + 3 * (q->nsend * v + q->send_off[j]), 3 * nr * sizeof(float),
                                             hipMemcpyDeviceToDevice, m->stream));
        }
    }
    return 0;
}

int comm_exchange(const std::vector<cwf_hip_system *> &g, std::initializer_list<Gather> gathers,
                  float *cwf_hip_system::*vec)
{
    std::vector<std::vector<float *>> vecs;
    if (vec)
        for (cwf_hip_system *h : g)
            vecs.push_back({h->*vec});
    return comm_exchange_vecs(g, gathers, vecs);
}

int comm_allgather(const std::vector<cwf_hip_system *> &g, double *cwf_hip_system::*buf, size_t count)
{
    return comm_exchange(g, {Gather{buf, count}}, nullptr);
}

int comm_halo(const std::vector<cwf_hip_system *> &g, float *cwf_hip_system::*vec)
{
    return comm_exchange(g, {}, vec);
}

// solve_pcg prologue (pcg.cpp:744-828) for a sharded system: owned-row dots, gathered scalars, halos
int sharded_pcg_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol)
{
    for (cwf_hip_system *h : g)
        fast_block_inverse(h, h->stream);
    if (int st = comm_halo(g, &cwf_hip_system::x))  // warm start: ghost x from the owners
        return st;
    for (size_t i = 0; i < g.size(); ++i)
    {
        cwf_hip_system *h = g[i];
        const uint32_t Down = 3u * h->ds.Nown;
        fast_keff(h, h->x, h->Ap, true, nullptr, nullptr, h->stream);
        launch_init_residual(h, rhs[i], h->stream);
        fast_dot(rhs[i], rhs[i], nullptr, Down, h->part0, nullptr, h->stream);
        fast_dot(h->r, h->r, nullptr, Down, h->part1, nullptr, h->stream);
        fold_pair(h->part0, h->part1, fast_dot_blocks(Down), h->g_init + 2 * h->rank, h->stream);
    }
    if (int st = comm_allgather(g, &cwf_hip_system::g_init, 2))
        return st;
    for (cwf_hip_system *h : g)
    {
        fast_init_scalars_strided(h, h->g_init, h->g_init + 1, (uint32_t)h->nranks, 2u, rel_tol, h->stream);
        launch_precond(h, h->ctl, h->stream);
    }
    if (int st = comm_halo(g, &cwf_hip_system::z))
        return st;
    for (cwf_hip_system *h : g)
    {
        const uint32_t Down = 3u * h->ds.Nown;
        fast_dot(h->r, h->z, nullptr, Down, h->part0, nullptr, h->stream);
        fold_pair(h->part0, nullptr, fast_dot_blocks(Down), h->g_rz0 + h->rank, h->stream);
    }
    if (int st = comm_allgather(g, &cwf_hip_system::g_rz0, 1))
        return st;
    for (cwf_hip_system *h : g)
    {
        fast_rho_from(h, h->g_rz0, (uint32_t)h->nranks, h->stream);
        launch_p_init(h, h->stream);
    }
    return 0;
}

// one FAST PCG iteration of every member (a single unsharded handle is the group {h} with one rank): two
// exchange steps, p.Ap after the tiles kernel and {r.r, r.z} + the z halo (one RCCL group) after the update
int fast_pcg_iteration_group(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs,
                             unsigned it, hipEvent_t e0, hipEvent_t e1)
{
    for (size_t i = 0; i < g.size(); ++i)  // member 0's launch carries the timing events
        fast_tiles_pcg(g[i], it, g[i]->stream, i ? nullptr : e0, i ? nullptr : e1);
    // PEER (one member per process): the exchange step folds the rank's shares itself, one launch fewer per step
    cwf_hip_system *h0 = g[0];
    if (h0->comm && h0->comm->kind == 2 && h0->nranks > 1)
    {
        const PeerFold fpap{h0->part0, nullptr, fast_tile_blocks(h0->ds)};
        if (int st = peer_exchange(h0, {Gather{&cwf_hip_system::g_pap, 1}}, {}, &fpap))
            return st;
        fast_update_pcg(h0, rhs[0], it, h0->stream);
        const PeerFold frrz{h0->part1, h0->part2, fast_rrz_shares(h0->ds, it)};
        return peer_exchange(h0, {Gather{&cwf_hip_system::g_rrz, 2}}, {h0->z}, &frrz);
    }
    for (cwf_hip_system *h : g)
        fast_fold_pap(h, h->stream);
    if (int st = comm_allgather(g, &cwf_hip_system::g_pap, 1))
        return st;
    for (size_t i = 0; i < g.size(); ++i)
    {
        fast_update_pcg(g[i], rhs[i], it, g[i]->stream);
        fast_fold_rrz(g[i], it, g[i]->stream);
    }
    return comm_exchange(g, {Gather{&cwf_hip_system::g_rrz, 2}}, g[0]->sharded() ? &cwf_hip_system::z : nullptr);
}

// ---- the sharded fused iteration (lattice_fused.inc on slab shards) ---------------------------------------------
// One launch and one exchange step per PCG iteration: launch j forms r_j, z_j, p_j, x_j for its owned rows and (from
// the received Ap_(j-1) rows and its own stored r_(j-1), p_(j-1)) the same r_j, p_j its neighbours form for its ghost
// rows, so only Ap_j's ghost rows and the five rank totals cross ranks: {rank totals} all-gather + Ap halo, ONE RCCL
// group or PEER step (against two per iteration in the two-kernel schedule above). Every rank folds the gathered
// totals in rank order, so every rank takes the same decisions.

// every member (and, through one all-gather, every rank) can run it: the decision is collective, taken at a handle's
// first sharded solve and kept (the shards' lattice plans do not change). 1 fused, 0 not, < 0 an error status
int group_fused(const std::vector<cwf_hip_system *> &g)
{
    cwf_hip_system *h0 = g[0];
    if (h0->fused_agreed >= 0)
        return h0->fused_agreed == 1;
    // a shard owning a single node plane keeps the two kernels: the fused launch's ghost-plane forms assume owned
    // planes on both sides of a brick's first and last plane (slabs one cell thick did not converge fused, LOCAL and
    // PEER alike; tests/test_gpu_lattice.py::test_thin_slab_shards_take_two_kernels)
    bool mine = true;
    for (cwf_hip_system *h : g)
        mine = mine && fast_fused(h) && h->ds.t.lat && h->ds.t.lk1 >= h->ds.t.lk0 + 2;
    // and the exchange inside the launches (PEER: one member per process); and the resident solve (PEER: every
    // iteration in one launch, resident.hip), whose tag base every rank then takes from the largest (the ranks'
    // granules must carry the same tags)
    const bool px = mine && g.size() == 1 && peer_fused_eligible(h0);
    const bool res = mine && g.size() == 1 && resident_shard_ready(h0);
    for (cwf_hip_system *h : g)
    {
        const double v[2] = {mine ? 1.0 : 0.0, (px ? 1.0 : 0.0) + (res ? 2.0 : 0.0) + 4.0 * (double)h->res.tag};
        HIPTRY(h, hipMemcpyAsync(h->g_init + 2 * h->rank, v, sizeof v, hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
    }
    // a rank that cannot learn the others' votes must not pick a schedule alone (its peers could agree on
    // the fused one and then wait for exchange steps it never runs): the solve fails instead, decided by nobody
    if (int st = comm_allgather(g, &cwf_hip_system::g_init, 2))
        return st < 0 ? st : set_error(h0, CWF_ERR_COMM, "schedule agreement all-gather failed");
    std::vector<double> f(2 * (size_t)h0->nranks, 0.0);
    HIPTRY(h0, hipStreamSynchronize(h0->stream));
    HIPTRY(h0, hipMemcpy(f.data(), h0->g_init, f.size() * sizeof(double), hipMemcpyDeviceToHost));
    bool all = true, all_px = true, all_res = true;
    uint64_t tag = 0;
    for (int r = 0; r < h0->nranks; ++r)
    {
        const uint64_t pv = (uint64_t)f[2 * (size_t)r + 1];
        all = all && f[2 * (size_t)r] == 1.0;
        all_px = all_px && (pv & 1u);
        all_res = all_res && (pv & 2u);
        tag = std::max<uint64_t>(tag, pv >> 2);
    }
    for (cwf_hip_system *h : g)
    {
        h->fused_agreed = all ? 1 : 0;
        h->px_agreed = all && all_px ? 1 : 0;
        h->res_agreed = all && all_res ? 1 : 0;
        if (h->res_agreed)
            h->res.tag = (uint32_t)tag;
    }
    return all ? 1 : 0;
}

namespace
{
// after launch j: the rank totals of its shares all-gathered into g_fsh, and Ap_j's ghost rows
int fused_exchange(const std::vector<cwf_hip_system *> &g, unsigned j)
{
    cwf_hip_system *h0 = g[0];
    if (h0->comm && h0->comm->kind == 2 && h0->nranks > 1)
    {
        unsigned stride = 0, count = 0;
        const double *sh = fast_fused_shares(h0, j, &stride, &count);
        PeerFold f{sh, nullptr, count, stride};
        return peer_exchange(h0, {Gather{&cwf_hip_system::g_fsh, kFusedSlotHost}}, {fast_fused_ap(h0, j)}, &f);
    }
    std::vector<std::vector<float *>> vecs;
    for (cwf_hip_system *h : g)
    {
        fast_fused_rank_totals(h, j, h->stream);
        vecs.push_back({fast_fused_ap(h, j)});
    }
    return comm_exchange_vecs(g, {Gather{&cwf_hip_system::g_fsh, kFusedSlotHost}}, vecs);
}
}  // namespace

namespace
{
// the fused and resident schedules' prologue: block inverse, the ghosts' global classes (once), ghost x, r_0 and the
// gathered norms, the tolerance, r_0's ghost rows (the first launch forms the ghosts' p_0 from them)
int sharded_fused_prologue(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs,
                           double rel_tol)
{
    for (cwf_hip_system *h : g)
        fast_block_inverse(h, h->stream);
    if (!g[0]->cls_global)  // the ghosts' classes from their owners, once per handle
    {
        for (cwf_hip_system *h : g)
            fast_fused_cls_out(h, h->stream);
        if (int st = comm_halo(g, &cwf_hip_system::tmp))
            return st;
        for (cwf_hip_system *h : g)
        {
            fast_fused_cls_in(h, h->stream);
            h->cls_global = true;
        }
    }
    if (int st = comm_halo(g, &cwf_hip_system::x))  // warm start: ghost x from the owners
        return st;
    for (size_t i = 0; i < g.size(); ++i)
    {
        cwf_hip_system *h = g[i];
        const uint32_t Down = 3u * h->ds.Nown;
        fast_keff(h, h->x, h->Ap, true, nullptr, nullptr, h->stream);
        launch_init_residual(h, rhs[i], h->stream);
        fast_dot(rhs[i], rhs[i], nullptr, Down, h->part0, nullptr, h->stream);
        fast_dot(h->r, h->r, nullptr, Down, h->part1, nullptr, h->stream);
        fold_pair(h->part0, h->part1, fast_dot_blocks(Down), h->g_init + 2 * h->rank, h->stream);
    }
    if (int st = comm_allgather(g, &cwf_hip_system::g_init, 2))
        return st;
    for (cwf_hip_system *h : g)
        fast_init_scalars_strided(h, h->g_init, h->g_init + 1, (uint32_t)h->nranks, 2u, rel_tol, h->stream);
    return comm_halo(g, &cwf_hip_system::r);
}
}  // namespace

int sharded_fused_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol)
{
    if (int st = sharded_fused_prologue(g, rhs, rel_tol))
        return st;
    if (g[0]->px_agreed == 1)  // the launches exchange themselves: epochs from here
        if (int st = peer_fused_begin(g[0]))
            return st;
    for (cwf_hip_system *h : g)
        fast_fused_launch0(h, h->stream);
    return g[0]->px_agreed == 1 ? 0 : fused_exchange(g, 0);
}

// the resident solve of PEER slab shards (resident.hip): the prologue only; the one launch then runs every
// iteration, its halo records and rank totals stored into the mailboxes by the kernel itself
int sharded_resident_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol)
{
    return sharded_fused_prologue(g, rhs, rel_tol);
}

int sharded_fused_iteration(const std::vector<cwf_hip_system *> &g, unsigned it, hipEvent_t e0, hipEvent_t e1)
{
    for (size_t i = 0; i < g.size(); ++i)
        fast_fused_iteration(g[i], it, g[i]->stream, i ? nullptr : e0, i ? nullptr : e1);
    return g[0]->px_agreed == 1 ? 0 : fused_exchange(g, it + 1u);
}

int sharded_fused_end(const std::vector<cwf_hip_system *> &g)
{
    return g[0]->px_agreed == 1 ? peer_fused_end(g[0]) : 0;
}

// ---- sharded PARITY (SURVEY.md 8e parity gate): the reference's fold orders across ranks --------------------
// Each rank's owned nodes are one contiguous range of global node ids, ascending by rank from node 0, and every
// rank but the last owns a whole number of reduction chunks (3 * owned % reduction_block == 0). Then a rank's
// k-th local chunk is global chunk (3 begin / B) + k, and the all-gathered per-rank chunk partials, folded
// rank after rank, are the global chunk partials folded in pcg.cpp:170-207 order (a rank's slot is padded with
// +0.0 past its own chunks; a sequential fp64 sum that starts at +0.0 is never -0.0, so adding +0.0 is exact).
// Owned K_eff / block-Jacobi rows are complete node gathers over the rank's elements in ascending global
// element order, bitwise the single-handle rows. Ghost rows of x / r / z are never read; p is refreshed on the
// ghosts by one halo after each p update. So every scalar, the residual history and every owned vector entry
// equal the single-handle PARITY solve bit for bit.
namespace
{
int parity_setup(const std::vector<cwf_hip_system *> &g)
{
    cwf_hip_system *h0 = g[0];
    const int n = h0->nranks;
    // (first global node, owned nodes) of every rank, gathered through the init-scalar slots
    for (cwf_hip_system *h : g)
    {
        const double v[2] = {(double)h->gbegin, (double)h->ds.Nown};
        HIPTRY(h, hipMemcpyAsync(h->g_init + 2 * h->rank, v, sizeof v, hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
    }
    if (int st = comm_allgather(g, &cwf_hip_system::g_init, 2))
        return st;
    std::vector<double> ranges(2 * (size_t)n);
    HIPTRY(h0, hipStreamSynchronize(h0->stream));
    HIPTRY(h0, hipMemcpy(ranges.data(), h0->g_init, ranges.size() * sizeof(double), hipMemcpyDeviceToHost));
    const uint64_t B = h0->reduction_block ? h0->reduction_block : 1;
    uint64_t next = 0, stride = 1;
    for (int r = 0; r < n; ++r)
    {
        const uint64_t begin = (uint64_t)ranges[2 * r], owned = (uint64_t)ranges[2 * r + 1];
        if (begin != next || (r + 1 < n && (3 * owned) % B != 0))
            return set_error(h0, CWF_ERR_UNSUPPORTED,
                             "sharded PARITY needs contiguous owned node ranges, ascending by rank from node 0, "
                             "each but the last a whole number of reduction blocks",
                             "rank=" + std::to_string(r) + "\nfirst_node=" + std::to_string(begin) +
                                 "\nowned_nodes=" + std::to_string(owned));
        next = begin + owned;
        stride = std::max<uint64_t>(stride, (3 * owned + B - 1) / B);
    }
    for (cwf_hip_system *h : g)
    {
        if (!h->owned_contiguous)
            return set_error(h, CWF_ERR_UNSUPPORTED, "sharded PARITY needs the rank's owned nodes in ascending "
                                                     "contiguous global order", "rank=" + std::to_string(h->rank));
        if (h->pstride == stride && h->gp0)
            continue;
        // (re)size the slot block: an attach resets pstride, so a re-attached handle reuses its block when it is
        // large enough and frees it otherwise (repeated attach / solve cycles do not grow device memory)
        const size_t bytes = 2 * (size_t)n * stride * sizeof(double);
        if (h->gp0 && h->gp_bytes < bytes)
        {
            (void)hipFree(h->gp0);
            h->owned.erase(std::remove(h->owned.begin(), h->owned.end(), static_cast<void *>(h->gp0)), h->owned.end());
            h->bytes -= h->gp_bytes;
            h->gp0 = h->gp1 = nullptr;
            h->gp_bytes = 0;
        }
        if (!h->gp0)
        {
            void *q = nullptr;
            if (hipMalloc(&q, bytes) != hipSuccess)
                return set_error(h, CWF_ERR_ALLOC, "failed to allocate device buffer", "bytes=" + std::to_string(bytes));
            h->owned.push_back(q);
            h->bytes += bytes;
            h->gp0 = static_cast<double *>(q);
            h->gp_bytes = bytes;
        }
        h->gp1 = h->gp0 + (size_t)n * stride;
        HIPTRY(h, hipMemset(h->gp0, 0, bytes));  // the +0.0 padding of every slot
        h->pstride = (uint32_t)stride;
    }
    return 0;
}

inline uint32_t owned_dofs(const cwf_hip_system *h) { return 3u * h->ds.Nown; }
inline uint32_t block_of(const cwf_hip_system *h) { return (uint32_t)(h->reduction_block ? h->reduction_block : 1); }
}  // namespace

int sharded_parity_init(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs, double rel_tol)
{
    if (int st = parity_setup(g))
        return st;
    const uint32_t S = g[0]->pstride, total = (uint32_t)g[0]->nranks * S;
    for (cwf_hip_system *h : g)
    {
        parity_block_jacobi(h, h->inv, h->stream);
        h->inv_fast = false;
    }
    if (int st = comm_halo(g, &cwf_hip_system::x))  // warm start: ghost x from the owners
        return st;
    for (size_t i = 0; i < g.size(); ++i)
    {
        cwf_hip_system *h = g[i];
        const size_t slot = (size_t)h->rank * S;
        parity_keff(h, h->x, h->Ap, true, nullptr, h->stream);
        launch_init_residual(h, rhs[i], h->stream);
        parity_dot_partials_n(owned_dofs(h), block_of(h), rhs[i], rhs[i], nullptr, h->gp0 + slot, nullptr, nullptr,
                              h->stream);
        parity_dot_partials_n(owned_dofs(h), block_of(h), h->r, h->r, nullptr, h->gp1 + slot, nullptr, nullptr,
                              h->stream);
    }
    if (int st = comm_exchange(g, {Gather{&cwf_hip_system::gp0, S}, Gather{&cwf_hip_system::gp1, S}}, nullptr))
        return st;
    for (cwf_hip_system *h : g)
    {
        parity_init_scalars(h, h->gp0, h->gp1, total, rel_tol, h->stream);
        launch_precond(h, h->ctl, h->stream);
        parity_dot_partials_n(owned_dofs(h), block_of(h), h->r, h->z, nullptr, h->gp0 + (size_t)h->rank * S, nullptr,
                              h->ctl, h->stream);
    }
    if (int st = comm_allgather(g, &cwf_hip_system::gp0, S))
        return st;
    for (cwf_hip_system *h : g)
    {
        parity_init_rho(h, h->gp0, total, h->stream);
        launch_p_init(h, h->stream);
    }
    return comm_halo(g, &cwf_hip_system::p);
}

int sharded_parity_iteration(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs,
                             hipEvent_t e0, hipEvent_t e1)
{
    const uint32_t S = g[0]->pstride, total = (uint32_t)g[0]->nranks * S;
    for (size_t i = 0; i < g.size(); ++i)
    {
        cwf_hip_system *h = g[i];
        if (i == 0 && e0)
            (void)hipEventRecord(e0, h->stream);
        parity_keff_dot(h, h->p, h->Ap, h->ctl, h->gp0 + (size_t)h->rank * S, h->stream);
        if (i == 0 && e1)
            (void)hipEventRecord(e1, h->stream);
    }
    if (int st = comm_allgather(g, &cwf_hip_system::gp0, S))
        return st;
    for (size_t i = 0; i < g.size(); ++i)
    {
        cwf_hip_system *h = g[i];
        const size_t slot = (size_t)h->rank * S;
        parity_alpha(h, h->gp0, total, h->stream);
        parity_update(h, rhs[i], h->gp0 + slot, h->gp1 + slot, h->stream);
    }
    if (int st = comm_exchange(g, {Gather{&cwf_hip_system::gp0, S}, Gather{&cwf_hip_system::gp1, S}}, nullptr))
        return st;
    for (cwf_hip_system *h : g)
    {
        parity_beta(h, h->gp0, h->gp1, total, h->stream);
        parity_p_update(h, h->stream);
    }
    return comm_halo(g, &cwf_hip_system::p);
}

}  // namespace cwf

using namespace cwf;

extern "C" {

int cwf_hip_comm_unique_id(uint8_t *id)
{
    if (!id)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    std::string why;
    const Rccl *r = rccl(&why);
    if (!r)
        return set_error(nullptr, CWF_ERR_COMM, why);
    ncclUniqueId u;
    NCCLTRY(nullptr, r->GetUniqueId(&u));
    std::memcpy(id, u.internal, CWF_COMM_ID_BYTES);
    return 0;
}

int cwf_hip_comm_create_rccl(int32_t nranks, int32_t rank, const uint8_t *id, int device, cwf_hip_comm **out)
{
    if (!id || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "rank out of range");
    std::string why;
    const Rccl *r = rccl(&why);
    if (!r)
        return set_error(nullptr, CWF_ERR_COMM, why);
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess)
        return hip_fail(nullptr, he, "hipSetDevice");
    ncclUniqueId u;
    std::memcpy(u.internal, id, CWF_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    NCCLTRY(nullptr, r->CommInitRank(&c, nranks, u, rank));
    cwf_hip_comm *cm = new (std::nothrow) cwf_hip_comm();
    if (!cm)
    {
        (void)r->CommDestroy(c);
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    }
    cm->kind = 1;
    cm->nranks = nranks;
    cm->device = device;
    cm->nccl = c;
    *out = cm;
    return 0;
}

int cwf_hip_comm_create_local(int32_t nranks, int device, cwf_hip_comm **out)
{
    if (!out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    if (nranks < 1)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "rank out of range");
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess)
        return hip_fail(nullptr, he, "hipSetDevice");
    cwf_hip_comm *cm = new (std::nothrow) cwf_hip_comm();
    if (!cm)
        return set_error(nullptr, CWF_ERR_ALLOC, "host allocation failed");
    cm->kind = 0;
    cm->nranks = nranks;
    cm->device = device;
    cm->members.assign(nranks, nullptr);
    if ((he = hipStreamCreateWithFlags(&cm->stream, hipStreamNonBlocking)) != hipSuccess)
    {
        delete cm;
        return hip_fail(nullptr, he, "hipStreamCreate");
    }
    *out = cm;
    return 0;
}

void cwf_hip_comm_destroy(cwf_hip_comm *cm)
{
    if (!cm)
        return;
    (void)hipSetDevice(cm->device);
    if (cm->kind == 1 && cm->nccl)
    {
        const Rccl *r = rccl(nullptr);
        if (r)
            (void)r->CommDestroy(static_cast<ncclComm_t>(cm->nccl));
    }
    for (cwf_hip_system *m : cm->members)
        if (m)
        {
            m->comm = nullptr;  // a still-attached handle falls back to its own stream
            if (m->own_stream)
            {
                m->stream = m->own_stream;
                m->own_stream = nullptr;
            }
        }
    if (cm->stream)
    {
        (void)hipStreamSynchronize(cm->stream);
        (void)hipStreamDestroy(cm->stream);
    }
    if (cm->kind == 2)
    {
        (void)hipDeviceSynchronize();
        peer_release(cm);
    }
    delete cm;
}

}  // extern "C"

extern "C" {

int cwf_hip_system_attach(cwf_hip_system *h, cwf_hip_comm *cm, int32_t rank, const cwf_shard_info *plan)
{
    if (!h || !cm || !plan)
        return set_error(h, CWF_ERR_ARGUMENT, "null pointer");
    if (h->comm)
        return set_error(h, CWF_ERR_ARGUMENT, "handle already attached");
    if (h->perm)
        return set_error(h, CWF_ERR_ARGUMENT, "shard handles keep their node order",
                         "create the handle with CWF_DESC_KEEP_NODE_ORDER (cwf_system_desc.reserved)");
    if (rank < 0 || rank >= cm->nranks || (cm->kind == 0 && cm->members[rank]))
        return set_error(h, CWF_ERR_ARGUMENT, "rank out of range or taken", "rank=" + std::to_string(rank));
    if (cm->device != h->device)
        return set_error(h, CWF_ERR_ARGUMENT, "communicator and handle are on different devices");
    // PEER: one member per process, checked before anything is allocated or attached (a failed attach
    // must not leave h->comm pointing at a communicator the caller then destroys)
    if (cm->kind == 2 && (cm->peer_member || rank != cm->rank))
        return set_error(h, CWF_ERR_ARGUMENT, "a peer communicator holds this process's rank only");
    if (plan->local_nodes != h->ds.N || plan->owned_nodes > h->ds.N)
        return set_error(h, CWF_ERR_SIZE, "halo plan does not match the handle",
                         "local_nodes=" + std::to_string(plan->local_nodes) + "\nhandle_nodes=" + std::to_string(h->ds.N));
    const uint32_t K = plan->neighbor_count;
    if (K && (!plan->neighbor_ranks || !plan->send_offsets || !plan->recv_offsets ||
              (plan->send_offsets[K] && !plan->send_nodes)))
        return set_error(h, CWF_ERR_ARGUMENT, "null halo plan array");
    for (uint32_t k = 0; k < K; ++k)
        if (plan->neighbor_ranks[k] < 0 || plan->neighbor_ranks[k] >= cm->nranks || plan->neighbor_ranks[k] == rank)
            return set_error(h, CWF_ERR_ARGUMENT, "bad neighbour rank", "k=" + std::to_string(k));
    if (K && plan->owned_nodes + plan->recv_offsets[K] != plan->local_nodes)
        return set_error(h, CWF_ERR_SIZE, "ghost ranges do not cover the ghost nodes");
    const uint64_t nsend = K ? plan->send_offsets[K] : 0;
    for (uint64_t i = 0; i < nsend; ++i)
        if (plan->send_nodes[i] >= plan->owned_nodes)
            return set_error(h, CWF_ERR_NODE_RANGE, "send list references a non-owned node", "i=" + std::to_string(i));
    if (int st = hipSetDevice(h->device); st != hipSuccess)
        return hip_fail(h, (hipError_t)st, "hipSetDevice");
    const int n = cm->nranks;
    auto alloc = [&](void **p, size_t bytes) -> int {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
        if (e != hipSuccess)
            return set_error(h, CWF_ERR_ALLOC, "failed to allocate device buffer", "bytes=" + std::to_string(bytes));
        h->owned.push_back(*p);
        h->bytes += std::max<size_t>(bytes, 16);
        return 0;
    };
    void *p = nullptr;
    if (int st = alloc(&p, 6 * (size_t)n * sizeof(double)))
        return st;
    h->g_pap = static_cast<double *>(p);
    h->g_rrz = h->g_pap + n;
    h->g_init = h->g_rrz + 2 * n;
    h->g_rz0 = h->g_init + 2 * n;
    HIPTRY(h, hipMemset(h->g_pap, 0, 6 * (size_t)n * sizeof(double)));
    if (int st = alloc(&p, nsend * sizeof(uint32_t)))
        return st;
    h->send_idx = static_cast<uint32_t *>(p);
    if (nsend)
        HIPTRY(h, hipMemcpy(h->send_idx, plan->send_nodes, nsend * sizeof(uint32_t), hipMemcpyHostToDevice));
    if (int st = alloc(&p, 3 * kMaxHaloVecs * nsend * sizeof(float)))  // one segment per halo vector of a step
        return st;
    h->sendbuf = static_cast<float *>(p);
    h->nsend = nsend;
    h->nbr.assign(plan->neighbor_ranks, plan->neighbor_ranks + K);
    h->send_off.assign(plan->send_offsets, plan->send_offsets + K + 1);
    h->recv_off.assign(plan->recv_offsets, plan->recv_offsets + K + 1);
    if (!K)
    {
        h->send_off.assign(1, 0);
        h->recv_off.assign(1, 0);
    }
    // from here on the handle's operator plan is the shard's: a failure leaves it unusable (not silently computing only
    // the owned rows of a partial plan as if it were unattached)
    const auto broken = [h](int st) {
        h->unusable = true;
        return st;
    };
    h->ds.Nown = (uint32_t)plan->owned_nodes;
    if (h->ds.t.lat)  // structured block: compute the rows of the planes holding owned nodes only
    {
        DevTiles &t = h->ds.t;
        uint32_t k0 = t.lnz, k1 = 0;
        for (uint32_t k = 0; k < t.lnz; ++k)
            if (h->lat_plane[k] < h->ds.Nown)
            {
                k0 = std::min(k0, k);
                k1 = std::max(k1, k + 1);
            }
        t.lk0 = k0 < k1 ? k0 : 0;
        t.lk1 = k0 < k1 ? k1 : 1;
        t.lzr = 0;  // the update pass stores z: the halo exchange carries z, and a ghost's class is a local one
        // a shard with ghosts takes the plane table even where its planes are affine (rank 0 of a slab stack: the
        // ghost plane stored right after the owned ones): the fused launch's ghost-plane stores of r_j / p_j are
        // instantiated on the plane-table kernels only
        if (h->ds.Nown < h->ds.N)
            t.lpstride = 0;
        lattice_plan(t);
        if (h->fsh)  // the fused iteration's shares for the shard's work items, its gathered rank totals
        {
            void *p = nullptr;
            if (int st = alloc(&p, 2ull * 5 * std::max<uint32_t>(t.lnwork, 1u) * sizeof(double)))
                return broken(st);
            h->fsh = static_cast<double *>(p);
            if (int st = alloc(&p, (size_t)kFusedSlotHost * n * sizeof(double)))
                return broken(st);
            h->g_fsh = static_cast<double *>(p);
            if (hipError_t e = hipMemset(h->g_fsh, 0, (size_t)kFusedSlotHost * n * sizeof(double)); e != hipSuccess)
                return broken(hip_fail(h, e, "hipMemset"));
        }
    }
    h->gbegin = plan->owned_nodes && plan->node_global ? plan->node_global[0] : 0;
    if (plan->node_global)
        h->node_gid.assign(plan->node_global, plan->node_global + plan->local_nodes);
    h->owned_contiguous = true;  // PARITY shards fold chunk partials in global order (comm.cpp parity_setup)
    if (plan->node_global)
        for (uint64_t i = 1; i < plan->owned_nodes; ++i)
            if (plan->node_global[i] != h->gbegin + i)
            {
                h->owned_contiguous = false;
                break;
            }
    h->pstride = 0;
    {  // a resident plan made before the attach is the whole block's: re-planned for the shard (its tags go on)
        const uint32_t tag = h->res.tag;
        h->res = cwf::ResidentPlan{};
        h->res.tag = tag;
    }
    h->comm = cm;
    h->rank = rank;
    h->nranks = n;
    if (cm->kind == 2)
        if (int st = peer_attach(h))
        {
            h->comm = nullptr;  // not attached: cwf_hip_system_destroy must not reach the communicator
            h->rank = 0;
            h->nranks = 1;
            return broken(st);
        }
    if (cm->kind == 0)
    {
        HIPTRY(h, hipStreamSynchronize(h->stream));
        h->own_stream = h->stream;
        h->stream = cm->stream;
        cm->members[rank] = h;
    }
    return 0;
}

}  // extern "C"

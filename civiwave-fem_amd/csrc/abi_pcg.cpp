// abi_pcg.cpp -- the PCG entry points of the C-ABI (include/cwf_hip.h; pcg.hpp:161-227): apply_keff, the block
// Jacobi inverse, dot, solve_pcg (single handle and LOCAL groups) and the residual history, over the device
// PCG driver run_pcg_group (the FAST / PARITY / sharded schedules, enqueued in batches with only
// the control block read back).
#include <cmath>
#include <cstring>

#include "abi_internal.hpp"
#include "blockinv_pack.hpp"

namespace cwf
{

std::string pcg_error_message(int code, int iter, std::string *ctx)
{
    if (code == CWF_ERR_DENOM_ZERO)
    {
        *ctx = "iteration=" + std::to_string(iter);
        return "CG denominator approached zero";  // pcg.cpp:846-849
    }
    if (code == CWF_ERR_COMM)  // a PEER exchange step's bounded wait (peer.hip): a peer never arrived
    {
        *ctx = "step=" + std::to_string(iter);
        return "peer exchange timed out";
    }
    if (code == CWF_ERR_HIP)  // resident.hip: a workgroup did not reach a phase within its bounded wait
    {
        *ctx = "phase=" + std::to_string(iter);
        return "resident solve: a workgroup missed the phase barrier";
    }
    if (code == CWF_ERR_RHO_ZERO && iter < 0)
    {
        *ctx = "rho~0";
        return "preconditioner produced near-zero rho";  // pcg.cpp:810-813
    }
    *ctx = "iteration=" + std::to_string(iter);
    return "CG rho approached zero";  // pcg.cpp:889-892
}

// the solve's telemetry and error from the control block read back last (every member's is identical)
int pcg_finish(const std::vector<cwf_hip_system *> &g, cwf_pcg_telemetry *tel)
{
    cwf_hip_system *h = g[0];
    const Ctl &c = *h->ctl_host;
    for (cwf_hip_system *m : g)
    {
        m->hist_count = c.iterations + 1;
        m->prev_iters = m->last_iters;
        m->last_iters = c.iterations;
    }
    if (tel)
    {
        tel->iterations = c.iterations;
        tel->residual_norm = c.res;
        tel->rhs_norm = c.rhs_norm_raw;
        tel->alpha_last = c.alpha_last;
        tel->beta_last = c.beta_last;
        tel->converged = c.converged;
        tel->reserved = 0;
    }
    if (c.error)
    {
        std::string ctx;
        std::string msg = pcg_error_message(c.error, c.error_iter, &ctx);
        for (size_t i = 1; i < g.size(); ++i)
            set_error(g[i], c.error, msg, ctx);
        return set_error(h, c.error, msg, ctx);
    }
    return 0;
}

// the resident solve: fast_fused_init (block inverse, r_0, norms, tolerance), then ONE launch that runs every
// iteration on chip (resident.hip) and leaves x, r and the control block; hipEvent-timed as a whole when timing is on
// (the handle's K_eff timing then counts its iterations: avg = the time per iteration). A PEER slab shard (one member
// per process): the sharded prologue instead of fast_fused_init, ghost x from the owners after the solve
int run_pcg_resident(cwf_hip_system *h, const float *rhs, const cwf_pcg_settings &set, cwf_pcg_telemetry *tel)
{
    hipStream_t st = h->stream;
    const bool shard = h->sharded();
    if (shard)
    {
        if (int e = sharded_resident_init({h}, {rhs}, set.relative_tolerance))
            return e;
    }
    else
        fast_fused_init(h, rhs, set.relative_tolerance, st, false);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->timing)
    {
        if (h->ev.size() < 2)
        {
            const size_t had = h->ev.size();
            h->ev.resize(2);
            for (size_t i = had; i < 2; ++i)
                HIPTRY(h, hipEventCreateWithFlags(&h->ev[i], hipEventDisableSystemFence));
        }
        e0 = h->ev[0];
        e1 = h->ev[1];
    }
    const uint32_t max_it = (uint32_t)std::min<uint64_t>(set.max_iterations, 1u << 24);
    launch_pcg_resident(h, max_it, st, e0, e1);
    // the next solve's tags start past every tag this one can publish (phases 0 .. max_it + 1)
    h->res.tag += max_it + 3u;
    HIPTRY(h, hipGetLastError());
    HIPTRY(h, hipMemcpyAsync(h->ctl_host, h->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st));
    HIPTRY(h, hipStreamSynchronize(st));
    if (shard && !h->ctl_host->error)  // ghost x <- owners (the stepper's node-wise updates read the ghost rows too)
    {
        if (int e = comm_halo({h}, &cwf_hip_system::x))
            return e;
        HIPTRY(h, hipStreamSynchronize(st));
    }
    if (e0 && h->ctl_host->iterations)
    {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess)
        {
            h->keff_ms += ms;
            h->keff_count += h->ctl_host->iterations;
        }
    }
    return pcg_finish({h}, tel);
}

// run solve_pcg on device buffers: rhs[i] and g[i]->x (holding the warm start) for every member of a
// group -- one handle, or every rank of a sharded system driven from this process (LOCAL comm).
int run_pcg_group(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs,
                  const cwf_pcg_settings &set, cwf_pcg_telemetry *tel)
{
    cwf_hip_system *h = g[0];
    if (set.max_iterations == 0)
        return set_error(h, CWF_ERR_MAX_ITERATIONS, "max_iterations must be >= 1", "max_iterations=0");
    const bool sharded = h->sharded();
    if (!sharded && g.size() != 1)
        return set_error(h, CWF_ERR_ARGUMENT, "a group needs attached shards");
    for (cwf_hip_system *m : g)
        if (m->mode != h->mode)
            return set_error(m, CWF_ERR_ARGUMENT, "every rank of a sharded solve runs in the same mode",
                             "rank=" + std::to_string(m->rank));
    for (cwf_hip_system *m : g)
        if (m->hist_cap < set.max_iterations + 1)
        {
            if (m->hist)
                (void)hipFree(m->hist);
            m->hist = nullptr;
            const uint64_t cap = std::max<uint64_t>(set.max_iterations + 1, 1024);
            if (hipMalloc(reinterpret_cast<void **>(&m->hist), cap * sizeof(double)) != hipSuccess)
                return set_error(m, CWF_ERR_ALLOC, "failed to grow matrix-free workspace buffers",
                                 "history=" + std::to_string(cap));
            m->hist_cap = cap;
        }
    hipStream_t st = h->stream;
    if (!set.warm_start)
        for (cwf_hip_system *m : g)
            HIPTRY(m, hipMemsetAsync(m->x, 0, m->ds.D * sizeof(float), m->stream));
    const bool fast = h->mode == CWF_MODE_FAST;
    // one launch per iteration (lattice_fused.inc); shards: one exchange per iteration, agreed by every rank
    int gf = 0;
    if (fast && sharded && (gf = group_fused(g)) < 0)
        return gf;
    const bool fused = fast && (sharded ? gf == 1 : fast_fused(h));
    // a block that fits on chip: the whole solve in one launch (resident.hip)
    if (fused && !sharded && set.max_iterations <= (1u << 24) && resident_ready(h))
        return run_pcg_resident(h, rhs[0], set, tel);
    if (fused && sharded && g.size() == 1 && h->res_agreed == 1 && set.max_iterations <= (1u << 24))
        return run_pcg_resident(h, rhs[0], set, tel);
    if (fused && sharded)
    {
        if (int e = sharded_fused_init(g, rhs, set.relative_tolerance))
            return e;
    }
    else if (fused)
        fast_fused_init(h, rhs[0], set.relative_tolerance, st);
    else if (sharded)
    {
        if (int e = fast ? sharded_pcg_init(g, rhs, set.relative_tolerance)
                         : sharded_parity_init(g, rhs, set.relative_tolerance))
            return e;
    }
    else if (fast)
        fast_pcg_init(h, rhs[0], set.relative_tolerance, st);
    else
        parity_pcg_init(h, rhs[0], set.relative_tolerance, st);
    HIPTRY(h, hipGetLastError());
    uint64_t enq = 0;
    constexpr uint64_t kMaxBatch = 64;
    uint64_t batch = set.check_interval > 0 ? std::min<uint64_t>((uint64_t)set.check_interval, kMaxBatch) : 4;
    // Batches end in a control-block read-back (a host round trip with the GPU idle) and overshoot the
    // converging iteration by up to a batch of no-op launches. Consecutive solves on one handle (warm-started
    // Newmark steps) take similar iteration counts, so with no check interval set and the handle's last two
    // solves within 25% of each other, the first batch runs up to 24 short of the smaller count and the
    // doubling restarts from 4 there: C2 steps ~17 read-backs and ~50 no-op iterations -> ~4 and <= 8. A
    // handle whose counts moved (its first solves, a static solve before Newmark steps, a changed tolerance)
    // doubles from 4, so a solve that converges early never waits on a long queue of no-op launches. Every
    // rank of a sharded solve has the same history (identical scalars), so their enqueued counts stay equal.
    uint64_t first = batch;
    const uint64_t lo = std::min(h->last_iters, h->prev_iters), hi = std::max(h->last_iters, h->prev_iters);
    if (set.check_interval <= 0 && lo > 40 && 4 * hi <= 5 * lo)
    {
        first = std::min<uint64_t>(lo - 24, kMaxFirstBatch);
        batch = 4;
    }
    if (h->timing && h->ev.size() < 2 * std::max(first, kMaxBatch))
    {
        const size_t had = h->ev.size();
        h->ev.resize(2 * std::max(first, kMaxBatch));
        for (size_t i = had; i < h->ev.size(); ++i)
            HIPTRY(h, hipEventCreateWithFlags(&h->ev[i], hipEventDisableSystemFence));  // no L2 write-back per timed launch
    }
    uint64_t prev_enq = 0, prev_nb = 0;
    for (;;)
    {
        // every member's control block is identical (rank-order folds); member 0's is polled
        HIPTRY(h, hipMemcpyAsync(h->ctl_host, h->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st));
        HIPTRY(h, hipStreamSynchronize(st));
        if (h->timing && prev_nb)
        {
            // only launches that did work: iteration index < completed iterations
            for (uint64_t i = 0; i < prev_nb; ++i)
            {
                if (prev_enq + i >= h->ctl_host->iterations)
                    break;
                if ((prev_enq + i) % (uint64_t)h->timing)
                    continue;
                float ms = 0.f;
                if (hipEventElapsedTime(&ms, h->ev[2 * i], h->ev[2 * i + 1]) == hipSuccess)
                {
                    h->keff_ms += ms;
                    ++h->keff_count;
                }
            }
            prev_nb = 0;
        }
        if (!h->ctl_host->active || enq >= set.max_iterations)
            break;
        const uint64_t nb = std::min<uint64_t>(enq ? batch : first, set.max_iterations - enq);
        for (uint64_t i = 0; i < nb; ++i)
        {
            const bool timed = h->timing && (enq + i) % (uint64_t)h->timing == 0;
            hipEvent_t e0 = timed ? h->ev[2 * i] : nullptr, e1 = timed ? h->ev[2 * i + 1] : nullptr;
            if (fused && sharded)
            {
                if (int e = sharded_fused_iteration(g, (unsigned)(enq + i), e0, e1))
                    return e;
            }
            else if (fused)
                fast_fused_iteration(h, (unsigned)(enq + i), st, e0, e1);
            else if (fast)
            {
                if (int e = fast_pcg_iteration_group(g, rhs, (unsigned)(enq + i), e0, e1))
                    return e;
            }
            else if (sharded)
            {
                if (int e = sharded_parity_iteration(g, rhs, e0, e1))
                    return e;
            }
            else
                parity_pcg_iteration(h, rhs[0], st, e0, e1);
        }
        if (fused)  // convergence of the batch's last launch (repeated idempotently by the next launch's start)
            for (cwf_hip_system *m : g)
                fast_fused_check(m, (unsigned)(enq + nb), m->stream);
        else if (fast)  // convergence of the batch's last update (repeated idempotently by the next tiles kernel)
            for (cwf_hip_system *m : g)
                fast_check_pcg(m, (unsigned)(enq + nb), m->stream);
        HIPTRY(h, hipGetLastError());
        prev_enq = enq;
        prev_nb = nb;
        enq += nb;
        if (set.check_interval <= 0)
            batch = std::min<uint64_t>(batch * 2, kMaxBatch);
    }
    if (fused)  // x is updated in every launch; the solve's r output is the last launch's
    {
        for (cwf_hip_system *m : g)
            fast_fused_finish(m, m->stream);
        if (sharded)
            if (int e = sharded_fused_end(g))
                return e;
    }
    else if (fast)  // x += alpha_j p_j of the iterations since the last lazy x update
        for (size_t i = 0; i < g.size(); ++i)
            fast_flush_x(g[i], rhs[i], g[i]->stream);
    if (sharded)  // ghost x <- owners, so node-wise stepper updates stay consistent on ghost rows
    {
        if (int e = comm_halo(g, &cwf_hip_system::x))
            return e;
        for (cwf_hip_system *m : g)
            HIPTRY(m, hipStreamSynchronize(m->stream));
    }
    return pcg_finish(g, tel);
}

int run_pcg(cwf_hip_system *h, const float *rhs_dev, const cwf_pcg_settings &set, cwf_pcg_telemetry *tel)
{
    if (h->comm && h->comm->kind == 0 && h->nranks > 1)
        return set_error(h, CWF_ERR_UNSUPPORTED, "a LOCAL-communicator shard solves through cwf_hip_solve_pcg_group");
    return run_pcg_group({h}, {rhs_dev}, set, tel);
}


}  // namespace cwf

using namespace cwf;

extern "C" {

int cwf_hip_apply_keff(cwf_hip_system *h, const float *x, float *y, uint64_t n, int kind)
{
    if (int st = check_ready(h))
        return st;
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "input/output span size mismatch",
                         "input=" + std::to_string(n) + "\ndofs=" + std::to_string(h->ds.D));
    const float *xin = nullptr;
    if (int st = stage_vec(h, x, h->tmp, kind, 3, &xin))
        return st;
    float *yout = kind == CWF_PTR_DEVICE && !h->perm ? y : h->Ap;
    if (h->mode == CWF_MODE_FAST)
        fast_keff(h, xin, yout, true, nullptr, nullptr, h->stream);
    else
        parity_keff(h, xin, yout, true, nullptr, h->stream);
    HIPTRY(h, hipGetLastError());
    if (int st = vec_out(h, yout, y, kind, 3))
        return st;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_hip_build_block_jacobi_inverse(cwf_hip_system *h, float *inv_out, uint64_t n, int kind)
{
    if (int st = check_ready(h))
        return st;
    const uint64_t req = 9ull * h->ds.N;
    if (n < req)
        return set_error(h, CWF_ERR_SIZE, "block inverse span too small",
                         "required=" + std::to_string(req) + "\navailable=" + std::to_string(n));
    float *dst = kind == CWF_PTR_DEVICE && !h->perm ? inv_out : h->inv;
    if (dst == h->inv)
        h->inv_fast = false;  // overwritten with the unsymmetrised reference inverse
    if (h->ds.hex)
        hex_block_jacobi(h, dst, h->stream);
    else
        parity_block_jacobi(h, dst, h->stream);
    HIPTRY(h, hipGetLastError());
    if (int st = vec_out(h, dst, inv_out, kind, 9))
        return st;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_hip_fast_block_inverse(cwf_hip_system *h, float *inv_out, uint64_t n, int kind, uint32_t *packed_out,
                               uint64_t *fallback_nodes)
{
    if (int st = check_ready(h))
        return st;
    const uint64_t N = h->ds.N, req = 9ull * N;
    if (n < req)
        return set_error(h, CWF_ERR_SIZE, "block inverse span too small",
                         "required=" + std::to_string(req) + "\navailable=" + std::to_string(n));
    if (h->mode != CWF_MODE_FAST)
        return set_error(h, CWF_ERR_ARGUMENT, "FAST-mode operator requested on a PARITY handle");
    fast_block_inverse(h, h->stream);
    HIPTRY(h, hipGetLastError());
    if (int st = vec_out(h, h->inv, inv_out, kind, 9))
        return st;
    if (packed_out || fallback_nodes)
    {
        std::vector<uint32_t> w(4 * N);
        if (N)
            HIPTRY(h, hipMemcpyAsync(w.data(), h->inv6, 16 * N, hipMemcpyDeviceToHost, h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
        std::vector<uint32_t> perm;  // caller's node of internal node i
        if (h->perm)
        {
            perm.resize(N);
            HIPTRY(h, hipMemcpy(perm.data(), h->perm, 4 * N, hipMemcpyDeviceToHost));
        }
        std::vector<uint32_t> out(4 * N);
        uint64_t nf = 0;
        for (uint64_t i = 0; i < N; ++i)
        {
            const uint64_t c = h->perm ? perm[i] : i;
            for (int k = 0; k < 4; ++k)
                out[4 * c + k] = w[4 * i + k];
            nf += (int32_t)w[4 * i] < 0;
        }
        if (packed_out)
            std::memcpy(packed_out, out.data(), out.size() * sizeof(uint32_t));
        if (fallback_nodes)
            *fallback_nodes = nf;
    }
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_pack_block_inverse(const float *v, uint32_t mask, uint32_t *w, float *d)
{
    if (!v || !w || !d)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    return cwf::pack_block_inverse(v, mask, w, d) ? 1 : 0;
}

int cwf_hip_dot(cwf_hip_system *h, const float *a, const float *b, uint64_t n, int kind, double *out,
                double *partials)
{
    if (int st = check_ready(h))
        return st;
    if (!out)
        return set_error(h, CWF_ERR_ARGUMENT, "null pointer");
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "dot product span size mismatch",
                         "lhs=" + std::to_string(n) + "\ndofs=" + std::to_string(h->ds.D));
    const float *da = nullptr, *db = nullptr;
    if (int st = stage_in(h, a, h->tmp, n, kind, &da))
        return st;
    if (int st = stage_in(h, b, h->Ap, n, kind, &db))
        return st;
    double *res = h->scal;
    uint32_t count;
    if (h->mode == CWF_MODE_FAST)
    {
        count = fast_dot_blocks(h->ds.D);
        fast_dot(da, db, nullptr, h->ds.D, h->part0, nullptr, h->stream);
        fast_fold(h->part0, count, res, h->stream);
    }
    else
    {
        count = parity_chunk_count(h);
        parity_dot_partials(h, da, db, nullptr, h->part0, nullptr, nullptr, h->stream);
        parity_fold(h->part0, count, res, h->stream);
    }
    HIPTRY(h, hipGetLastError());
    HIPTRY(h, hipMemcpyAsync(out, res, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (partials)
    {
        const uint64_t total = h->reduction_partials;
        const uint64_t ncopy = std::min<uint64_t>(count, total);
        if (kind == CWF_PTR_DEVICE)
        {
            HIPTRY(h, hipMemcpyAsync(partials, h->part0, ncopy * sizeof(double), hipMemcpyDeviceToDevice,
                                     h->stream));
            if (total > ncopy)
                HIPTRY(h, hipMemsetAsync(partials + ncopy, 0, (total - ncopy) * sizeof(double), h->stream));
        }
        else
        {
            HIPTRY(h, hipMemcpyAsync(partials, h->part0, ncopy * sizeof(double), hipMemcpyDeviceToHost, h->stream));
            HIPTRY(h, hipStreamSynchronize(h->stream));
            for (uint64_t c = ncopy; c < total; ++c)
                partials[c] = 0.0;
        }
    }
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_hip_solve_pcg(cwf_hip_system *h, const float *rhs, const cwf_pcg_settings *settings, float *x_inout,
                      float *residual_out, uint64_t n, int kind, cwf_pcg_telemetry *telemetry)
{
    if (int st = check_ready(h))
        return st;
    if (!rhs || !settings || !x_inout)
        return set_error(h, CWF_ERR_ARGUMENT, "null pointer");
    if (telemetry)
        std::memset(telemetry, 0, sizeof *telemetry);
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "rhs span size mismatch",
                         "rhs=" + std::to_string(n) + "\ndofs=" + std::to_string(h->ds.D));
    if (settings->max_iterations == 0)
        return set_error(h, CWF_ERR_MAX_ITERATIONS, "max_iterations must be >= 1", "max_iterations=0");
    const float *drhs = nullptr;
    if (int st = stage_vec(h, rhs, h->rhs, kind, 3, &drhs))
        return st;
    if (settings->warm_start)
        if (int st = vec_in(h, x_inout, h->x, kind, 3))
            return st;
    int st = run_pcg(h, drhs, *settings, telemetry);
    if (int e = vec_out(h, h->x, x_inout, kind, 3))
        return e;
    if (residual_out)
        if (int e = vec_out(h, h->r, residual_out, kind, 3))
            return e;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return st;
}

int cwf_hip_solve_pcg_group(cwf_hip_system *const *members, int32_t count, const float *const *rhs,
                            const cwf_pcg_settings *settings, float *const *x_inout, float *const *residual_out,
                            int kind, cwf_pcg_telemetry *telemetry)
{
    if (!members || count < 1 || !rhs || !settings || !x_inout)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    if (telemetry)
        std::memset(telemetry, 0, sizeof *telemetry);
    std::vector<cwf_hip_system *> g(members, members + count);
    cwf_hip_comm *cm = g[0] ? g[0]->comm : nullptr;
    for (int32_t i = 0; i < count; ++i)
    {
        if (int st = check_ready(g[i]))
            return st;
        if (!rhs[i] || !x_inout[i])
            return set_error(g[i], CWF_ERR_ARGUMENT, "null pointer");
        if (count > 1 && (!cm || cm->kind != 0 || g[i]->comm != cm || g[i]->rank != i || cm->nranks != count))
            return set_error(g[i], CWF_ERR_ARGUMENT, "members must be every rank of one LOCAL communicator, in rank order",
                             "member=" + std::to_string(i));
    }
    if (settings->max_iterations == 0)
        return set_error(g[0], CWF_ERR_MAX_ITERATIONS, "max_iterations must be >= 1", "max_iterations=0");
    std::vector<const float *> drhs(count);
    for (int32_t i = 0; i < count; ++i)
    {
        cwf_hip_system *h = g[i];
        if (int st = stage_in(h, rhs[i], h->rhs, h->ds.D, kind, &drhs[i]))
            return st;
        if (settings->warm_start)
            HIPTRY(h, hipMemcpyAsync(h->x, x_inout[i], h->ds.D * sizeof(float),
                                     kind == CWF_PTR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                     h->stream));
    }
    int st = run_pcg_group(g, drhs, *settings, telemetry);
    const hipMemcpyKind back = kind == CWF_PTR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    for (int32_t i = 0; i < count; ++i)
    {
        cwf_hip_system *h = g[i];
        HIPTRY(h, hipMemcpyAsync(x_inout[i], h->x, h->ds.D * sizeof(float), back, h->stream));
        if (residual_out && residual_out[i])
            HIPTRY(h, hipMemcpyAsync(residual_out[i], h->r, h->ds.D * sizeof(float), back, h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
    }
    return st;
}

int cwf_hip_residual_history(cwf_hip_system *h, double *out, uint64_t capacity, uint64_t *count)
{
    if (int st = check_ready(h))
        return st;
    const uint64_t c = std::min(capacity, h->hist_count);
    if (c && out)
        HIPTRY(h, hipMemcpy(out, h->hist, c * sizeof(double), hipMemcpyDeviceToHost));
    if (count)
        *count = c;
    return 0;
}

}  // extern "C"

// abi_stepper.cpp -- the device-resident Newmark Stepper of the C-ABI (newmark_stepper.cpp:1005-1379): create,
// step (predictor, RHS, Rayleigh damping product, Dirichlet clamp, PCG with warm start, corrector, adaptive dt),
// state access, external force and the harmonic load pattern.
#include <cfloat>
#include <cmath>
#include <cstring>

#include "abi_internal.hpp"

using namespace cwf;


// ------------------------------------------------------------------------------------------
// Stepper (newmark_stepper.cpp:1005-1379)
// ------------------------------------------------------------------------------------------

struct cwf_hip_stepper
{
    cwf_hip_system *sys = nullptr;
    cwf_stepper_desc d{};
    double dt = 1e-3, accumulated_time = 0.0, beta = 0.25, gamma = 0.5;
    uint64_t frame_index = 0;
    int warm_start = 1;
    float *u = nullptr, *v = nullptr, *a = nullptr, *up = nullptr, *vp = nullptr, *f = nullptr, *bcv = nullptr,
          *damp = nullptr, *kd = nullptr, *srhs = nullptr;
    double *lbase = nullptr, *lpat = nullptr;  // cwf_hip_stepper_set_load_pattern: f64 [3N] each (internal order)
    std::vector<void *> owned;
};

namespace
{
int st_alloc(cwf_hip_stepper *t, float **p, uint64_t n)
{
    void *q = nullptr;
    if (hipMalloc(&q, std::max<uint64_t>(n, 4) * sizeof(float)) != hipSuccess)
        return set_error(t->sys, CWF_ERR_ALLOC, "failed to allocate stepper buffers");
    t->owned.push_back(q);
    *p = static_cast<float *>(q);
    return 0;
}
}  // namespace

extern "C" {

void cwf_hip_stepper_destroy(cwf_hip_stepper *t)
{
    if (!t)
        return;
    (void)hipSetDevice(t->sys->device);
    (void)hipStreamSynchronize(t->sys->stream);
    for (void *p : t->owned)
        (void)hipFree(p);
    delete t;
}

int cwf_hip_stepper_create(cwf_hip_system *h, const cwf_stepper_desc *desc, cwf_hip_stepper **out)
{
    if (int st = check_ready(h))
        return st;
    if (!desc || !out)
        return set_error(h, CWF_ERR_ARGUMENT, "null pointer");
    *out = nullptr;
    auto *t = new (std::nothrow) cwf_hip_stepper();
    if (!t)
        return set_error(h, CWF_ERR_ALLOC, "host allocation failed");
    t->sys = h;
    t->d = *desc;
    t->d.external_force = nullptr;
    t->d.bc_value = nullptr;
    t->dt = desc->initial_dt > 0.0 ? desc->initial_dt : 1.0e-3;  // :1020
    t->warm_start = desc->warm_start;
    const uint64_t D = h->ds.D;
    for (float **p : {&t->u, &t->v, &t->a, &t->up, &t->vp, &t->f, &t->bcv, &t->damp, &t->kd, &t->srhs})
        if (int st = st_alloc(t, p, D))
        {
            cwf_hip_stepper_destroy(t);
            return st;
        }
    hipStream_t s = h->stream;
    for (float *p : {t->u, t->v, t->a, t->up, t->vp, t->f, t->bcv})
        (void)hipMemsetAsync(p, 0, D * sizeof(float), s);
    if (desc->external_force)
        (void)vec_in(h, desc->external_force, t->f, CWF_PTR_HOST, 3);
    if (desc->bc_value)
        (void)vec_in(h, desc->bc_value, t->bcv, CWF_PTR_HOST, 3);
    (void)hipMemsetAsync(h->x, 0, D * sizeof(float), s);  // solver.x starts at 0 (pack.cpp:214)
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess)
    {
        cwf_hip_stepper_destroy(t);
        return hip_fail(h, e, "stepper create");
    }
    *out = t;
    return 0;
}

int cwf_hip_stepper_step(cwf_hip_stepper *t, double sim_time, int paused, cwf_step_telemetry *tel)
{
    if (!t)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null handle");
    cwf_hip_system *h = t->sys;
    if (int st = check_ready(h))
        return st;
    hipStream_t s = h->stream;
    const uint32_t N = h->ds.N, D = h->ds.D;
    t->accumulated_time = sim_time;
    // refresh_coefficients + update_matrix_free_scalars (:1316-1326)
    const double b = t->beta, g = t->gamma, dt = t->dt;
    double c6[6];
    c6[0] = 1.0 / (b * dt * dt);
    c6[1] = g / (b * dt);
    c6[2] = 1.0 / (b * dt);
    c6[3] = (1.0 / (2.0 * b)) - 1.0;
    c6[4] = (g / b) - 1.0;
    c6[5] = dt * ((g / (2.0 * b)) - 1.0);
    const double inv_beta_dt2 = 1.0 / (b * dt * dt);
    const double gamma_over_beta_dt = g / (b * dt);
    const cwf::DevSys saved = h->ds;
    h->ds.sK = 1.0 + c6[1] * t->d.rayleigh_beta;
    h->ds.sM = c6[0] + c6[1] * t->d.rayleigh_alpha;
    stepper_predictor(D, t->u, t->v, t->a, t->up, t->vp, dt, b, g, s);
    stepper_assemble_rhs(N, h->ds.mass, t->u, t->v, t->a, t->f, t->srhs, t->damp, c6, t->d.rayleigh_alpha, s);
    if (std::fabs(t->d.rayleigh_beta) > DBL_EPSILON)
    {
        cwf::DevSys stiff = h->ds;  // stiffness_only_system_ (:1051-1053)
        stiff.sK = 1.0;
        stiff.sM = 0.0;
        if (h->mode == CWF_MODE_FAST)
            fast_keff_ds(stiff, t->damp, t->kd, true, nullptr, nullptr, s);
        else
            parity_keff_ds(stiff, t->damp, t->kd, true, nullptr, s);
        stepper_rhs_damping(D, t->srhs, t->kd, (float)t->d.rayleigh_beta, s);
    }
    stepper_clamp(N, h->ds.mask, t->bcv, t->u, t->srhs, s);
    const double tol = paused ? t->d.pause_tolerance : t->d.runtime_tolerance;
    cwf_pcg_settings ps{t->d.max_iterations, tol, t->warm_start, 0};
    cwf_pcg_telemetry pt{};
    int st = run_pcg(h, t->srhs, ps, &pt);
    h->ds.sK = saved.sK;
    h->ds.sM = saved.sM;
    if (st)
    {
        std::string inner = h->err;
        return set_error(h, st, "pcg solve failed", inner);  // :1130-1133
    }
    stepper_update(D, h->x, t->up, t->vp, t->u, t->v, t->a, (float)inv_beta_dt2, (float)gamma_over_beta_dt, s);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipStreamSynchronize(s);
    if (e != hipSuccess)
        return hip_fail(h, e, "stepper update");
    cwf_step_telemetry T{};
    T.simulation_time = sim_time;
    T.time_step = t->dt;
    T.applied_tolerance = tol;
    T.paused_mode = paused ? 1 : 0;
    T.pcg = pt;
    // adapt_timestep (:1328-1367)
    if (t->d.adaptive)
    {
        const double low = t->d.low_iteration_ratio * (double)t->d.max_iterations;
        if ((double)pt.iterations <= low)
        {
            t->dt *= t->d.increase_factor;
            T.dt_increased = 1;
        }
        else if (!pt.converged)
        {
            t->dt *= t->d.decrease_factor;
            T.dt_decreased = 1;
        }
        if (t->d.min_dt > 0.0 && t->dt <= t->d.min_dt)
        {
            t->dt = t->d.min_dt;
            T.dt_clamped_min = 1;
        }
        if (t->d.max_dt > 0.0 && t->dt >= t->d.max_dt)
        {
            t->dt = t->d.max_dt;
            T.dt_clamped_max = 1;
        }
    }
    ++t->frame_index;
    t->accumulated_time = sim_time + t->dt;
    if (tel)
        *tel = T;
    return 0;
}

int cwf_hip_stepper_get_state(cwf_hip_stepper *t, int which, float *out, uint64_t n, int kind)
{
    if (!t || !out)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    cwf_hip_system *h = t->sys;
    if (int st = check_ready(h))
        return st;
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "state span size mismatch");
    const float *src = which == 0   ? t->u
                       : which == 1 ? t->v
                       : which == 2 ? t->a
                       : which == 3 ? h->x
                       : which == 4 ? t->f  // nodes.external_force (after set_load_scale / set_external_force)
                                    : nullptr;
    if (!src)
        return set_error(h, CWF_ERR_ARGUMENT, "unknown state field");
    if (int st = vec_out(h, src, out, kind, 3))
        return st;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_hip_stepper_set_state(cwf_hip_stepper *t, int which, const float *in, uint64_t n, int kind)
{
    if (!t || !in)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    cwf_hip_system *h = t->sys;
    if (int st = check_ready(h))
        return st;
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "state span size mismatch");
    float *dst = which == 0 ? t->u : which == 1 ? t->v : which == 2 ? t->a : which == 3 ? h->x : nullptr;
    if (!dst)
        return set_error(h, CWF_ERR_ARGUMENT, "unknown state field");
    if (int st = vec_in(h, in, dst, kind, 3))
        return st;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_hip_stepper_set_external_force(cwf_hip_stepper *t, const float *f, uint64_t n, int kind)
{
    if (!t || !f)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    cwf_hip_system *h = t->sys;
    if (int st = check_ready(h))
        return st;
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "external force span size mismatch");
    if (int st = vec_in(h, f, t->f, kind, 3))
        return st;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_hip_stepper_set_load_pattern(cwf_hip_stepper *t, const double *base, const double *pattern, uint64_t n)
{
    if (!t || !base || !pattern)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null pointer");
    cwf_hip_system *h = t->sys;
    if (int st = check_ready(h))
        return st;
    if (n != h->ds.D)
        return set_error(h, CWF_ERR_SIZE, "load pattern span size mismatch",
                         "input=" + std::to_string(n) + "\ndofs=" + std::to_string(h->ds.D));
    if (!t->lbase)
    {
        void *q = nullptr;
        if (hipMalloc(&q, std::max<uint64_t>(2 * n, 2) * sizeof(double)) != hipSuccess)
            return set_error(h, CWF_ERR_ALLOC, "failed to allocate stepper buffers");
        t->owned.push_back(q);
        t->lbase = static_cast<double *>(q);
        t->lpat = t->lbase + n;
    }
    // a node's 3 f64 = 6 floats: the node-order conversion moves them as 6-float records
    if (int st = vec_in(h, reinterpret_cast<const float *>(base), reinterpret_cast<float *>(t->lbase), CWF_PTR_HOST, 6))
        return st;
    if (int st = vec_in(h, reinterpret_cast<const float *>(pattern), reinterpret_cast<float *>(t->lpat), CWF_PTR_HOST,
                        6))
        return st;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return 0;
}

int cwf_hip_stepper_set_load_scale(cwf_hip_stepper *t, double scale)
{
    if (!t)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null handle");
    cwf_hip_system *h = t->sys;
    if (int st = check_ready(h))
        return st;
    if (!t->lbase)
        return set_error(h, CWF_ERR_ARGUMENT, "no load pattern set", "cwf_hip_stepper_set_load_pattern");
    stepper_scaled_load(h->ds.D, t->lbase, t->lpat, scale, t->f, h->stream);  // ordered before the next step
    HIPTRY(h, hipGetLastError());
    return 0;
}

int cwf_hip_stepper_set_warm_start(cwf_hip_stepper *t, int enabled)
{
    if (!t)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null handle");
    t->warm_start = enabled ? 1 : 0;
    return 0;
}

int cwf_hip_stepper_time(const cwf_hip_stepper *t, double *current_time, double *time_step)
{
    if (!t)
        return set_error(nullptr, CWF_ERR_ARGUMENT, "null handle");
    if (current_time)
        *current_time = t->accumulated_time;
    if (time_step)
        *time_step = t->dt;
    return 0;
}

}  // extern "C"

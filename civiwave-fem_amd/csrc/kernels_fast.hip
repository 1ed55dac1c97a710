// kernels_fast.hip -- fast mode: fp32 element math, fp64 reductions fused into the producing
// kernels (deterministic: fixed block decomposition + fixed-order tree), tolerance-checked
// against the oracle instead of bit-checked.
#include "cwf_internal.hpp"

namespace cwf
{
namespace
{

constexpr int kBlock = 256;

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    return v;
}

// block of 256 threads -> one double (lane order fixed => deterministic)
__device__ __forceinline__ double block_sum(double v, double *lds4)
{
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        lds4[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        t = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    return t;
}

template <bool ISO>
__device__ __forceinline__ void stress_f32(const float *Dm, const float e[6], float s[6])
{
    if constexpr (ISO)
    {
#pragma unroll
        for (int r = 0; r < 3; ++r)
            s[r] = fmaf(Dm[3 * r + 2], e[2], fmaf(Dm[3 * r + 1], e[1], Dm[3 * r] * e[0]));
#pragma unroll
        for (int r = 3; r < 6; ++r)
            s[r] = Dm[6 + r] * e[r];
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 6; ++r)
        {
            float sum = 0.0f;
#pragma unroll
            for (int c = 0; c < 6; ++c)
                sum = fmaf(Dm[6 * r + c], e[c], sum);
            s[r] = sum;
        }
    }
}

// K_eff p in fp32, one thread per node over the ascending CSR; also writes the block's
// fp64 partial of p.Ap (the PCG denominator) so no separate dot pass is needed.
template <bool ISO, bool SANITIZE>
__global__ __launch_bounds__(kBlock) void k_keff_fast(DevSys s, const float *__restrict__ x,
                                                      float *__restrict__ y, const Ctl *__restrict__ ctl,
                                                      double *__restrict__ part)
{
    constexpr int kTab = ISO ? 12 : 36;
    constexpr int kMaxM = 16;
    __shared__ float dtab[kMaxM * 36];
    __shared__ double red[4];
    if (ctl && !ctl->active)
        return;
    const uint32_t nm = s.M < kMaxM ? s.M : kMaxM;
    for (uint32_t i = threadIdx.x; i < nm * kTab; i += kBlock)
    {
        const uint32_t m = i / kTab, t = i % kTab;
        const uint32_t src = ISO ? (t < 9 ? (t / 3) * 6 + (t % 3) : (t - 6) * 7) : t;
        dtab[i] = (float)s.dmat[36u * m + src];
    }
    __syncthreads();
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    double pap = 0.0;
    if (n < s.N)
    {
        float acc0 = 0.0f, acc1 = 0.0f, acc2 = 0.0f;
        const uint32_t jb = s.off[n], je = s.off[n + 1];
        const float sK = (float)s.sK;
        for (uint32_t j = jb; j < je; ++j)
        {
            const uint32_t inc = s.inc[j];
            const uint32_t e = inc >> 2, a = inc & 3u;
            const uint4 q0 = s.erec[4u * e + 0u];
            const uint4 q1 = s.erec[4u * e + 1u];
            const uint4 q2 = s.erec[4u * e + 2u];
            const uint4 q3 = s.erec[4u * e + 3u];
            const float g[12] = {__uint_as_float(q1.x), __uint_as_float(q1.y), __uint_as_float(q1.z),
                                 __uint_as_float(q1.w), __uint_as_float(q2.x), __uint_as_float(q2.y),
                                 __uint_as_float(q2.z), __uint_as_float(q2.w), __uint_as_float(q3.x),
                                 __uint_as_float(q3.y), __uint_as_float(q3.z), __uint_as_float(q3.w)};
            const uint32_t c[4] = {q0.x, q0.y, q0.z, q0.w};
            float eps[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 4; ++q)
            {
                const float *xp = x + 3u * c[q];
                float u0 = xp[0], u1 = xp[1], u2 = xp[2];
                if constexpr (SANITIZE)
                {
                    const uint32_t mk = s.mask[c[q]];
                    u0 = (mk & 1u) ? 0.f : u0;
                    u1 = (mk & 2u) ? 0.f : u1;
                    u2 = (mk & 4u) ? 0.f : u2;
                }
                const float gx = g[3 * q], gy = g[3 * q + 1], gz = g[3 * q + 2];
                eps[0] = fmaf(gx, u0, eps[0]);
                eps[1] = fmaf(gy, u1, eps[1]);
                eps[2] = fmaf(gz, u2, eps[2]);
                eps[3] = fmaf(gx, u1, fmaf(gy, u0, eps[3]));
                eps[4] = fmaf(gy, u2, fmaf(gz, u1, eps[4]));
                eps[5] = fmaf(gx, u2, fmaf(gz, u0, eps[5]));
            }
            const uint32_t mi = s.mat[e];
            float sig[6];
            if (mi < (uint32_t)kMaxM)
                stress_f32<ISO>(dtab + kTab * mi, eps, sig);
            else
            {
                float tab[36];
                for (int t = 0; t < kTab; ++t)
                    tab[t] = (float)s.dmat[36u * mi + (ISO ? (t < 9 ? (t / 3) * 6 + (t % 3) : (t - 6) * 7) : t)];
                stress_f32<ISO>(tab, eps, sig);
            }
            const float vol = s.vol[e] * sK;
            const float ax = a == 0 ? g[0] : a == 1 ? g[3] : a == 2 ? g[6] : g[9];
            const float ay = a == 0 ? g[1] : a == 1 ? g[4] : a == 2 ? g[7] : g[10];
            const float az = a == 0 ? g[2] : a == 1 ? g[5] : a == 2 ? g[8] : g[11];
            acc0 = fmaf(vol, fmaf(az, sig[5], fmaf(ay, sig[3], ax * sig[0])), acc0);
            acc1 = fmaf(vol, fmaf(az, sig[4], fmaf(ax, sig[3], ay * sig[1])), acc1);
            acc2 = fmaf(vol, fmaf(ax, sig[5], fmaf(ay, sig[4], az * sig[2])), acc2);
        }
        const uint32_t mk = s.mask[n];
        const float m = (float)((double)s.mass[n] * s.sM);
        const float x0 = x[3u * n + 0], x1 = x[3u * n + 1], x2 = x[3u * n + 2];
        float y0 = fmaf(m, (SANITIZE && (mk & 1u)) ? 0.f : x0, acc0);
        float y1 = fmaf(m, (SANITIZE && (mk & 2u)) ? 0.f : x1, acc1);
        float y2 = fmaf(m, (SANITIZE && (mk & 4u)) ? 0.f : x2, acc2);
        y0 = (mk & 1u) ? x0 : y0;
        y1 = (mk & 2u) ? x1 : y1;
        y2 = (mk & 4u) ? x2 : y2;
        y[3u * n + 0] = y0;
        y[3u * n + 1] = y1;
        y[3u * n + 2] = y2;
        pap = (double)x0 * (double)y0 + (double)x1 * (double)y1 + (double)x2 * (double)y2;
    }
    if (part)
    {
        const double t = block_sum(pap, red);
        if (threadIdx.x == 0)
            part[blockIdx.x] = t;
    }
}

// deterministic tree fold of `count` block partials by one 256-thread block
__device__ __forceinline__ double tree_fold(const double *__restrict__ p, uint32_t count, double *red)
{
    double v = 0.0;
    for (uint32_t i = threadIdx.x; i < count; i += kBlock)
        v += p[i];
    double t = block_sum(v, red);
    return t;  // valid in thread 0
}

__global__ __launch_bounds__(kBlock) void k_fold_fast(const double *__restrict__ p, uint32_t count,
                                                      double *__restrict__ out)
{
    __shared__ double red[4];
    const double t = tree_fold(p, count, red);
    if (threadIdx.x == 0)
        out[0] = t;
}

__global__ __launch_bounds__(kBlock) void k_dot_fast(const float *__restrict__ a, const float *__restrict__ b,
                                                     const float *__restrict__ c, uint32_t D,
                                                     double *__restrict__ pab, double *__restrict__ pac)
{
    __shared__ double red[4];
    double s0 = 0.0, s1 = 0.0;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < D; i += gridDim.x * kBlock)
    {
        const double av = (double)a[i];
        s0 += av * (double)b[i];
        if (c)
            s1 += av * (double)c[i];
    }
    const double t0 = block_sum(s0, red);
    if (threadIdx.x == 0)
        pab[blockIdx.x] = t0;
    if (c)
    {
        __syncthreads();
        const double t1 = block_sum(s1, red);
        if (threadIdx.x == 0)
            pac[blockIdx.x] = t1;
    }
}

__global__ __launch_bounds__(kBlock) void k_fast_init_scalars(Ctl *ctl, const double *__restrict__ p_rhs,
                                                              const double *__restrict__ p_rr, uint32_t count,
                                                              double rel_tol, double *__restrict__ hist)
{
    __shared__ double red[4];
    const double rhs_sq = tree_fold(p_rhs, count, red);
    __syncthreads();
    const double rr = tree_fold(p_rr, count, red);
    if (threadIdx.x != 0)
        return;
    double rhs_norm = sqrt(rhs_sq);
    if (rhs_norm < 1.0e-12)
        rhs_norm = 1.0;
    Ctl c{};
    c.res = sqrt(rr);
    c.rhs_norm = rhs_norm;
    c.rhs_norm_raw = sqrt(rhs_sq);
    c.tol = rel_tol * rhs_norm;
    c.converged = c.res <= c.tol ? 1 : 0;
    c.active = c.converged ? 0 : 1;
    hist[0] = c.res;
    *ctl = c;
}

__global__ __launch_bounds__(kBlock) void k_fast_rho(Ctl *ctl, const double *__restrict__ p_rz, uint32_t count)
{
    __shared__ double red[4];
    if (!ctl->active)
        return;
    const double rho = tree_fold(p_rz, count, red);
    if (threadIdx.x != 0)
        return;
    ctl->rho = rho;
    if (fabs(rho) < 1.0e-18)
    {
        ctl->error = CWF_ERR_RHO_ZERO;
        ctl->error_iter = -1;
        ctl->active = 0;
    }
}

__global__ __launch_bounds__(kBlock) void k_fast_alpha(Ctl *ctl, const double *__restrict__ p_pAp, uint32_t count)
{
    __shared__ double red[4];
    if (!ctl->active)
        return;
    const double denom = tree_fold(p_pAp, count, red);
    if (threadIdx.x != 0)
        return;
    ctl->denom = denom;
    if (fabs(denom) < 1.0e-18)
    {
        ctl->error = CWF_ERR_DENOM_ZERO;
        ctl->error_iter = (int)ctl->iterations;
        ctl->active = 0;
        return;
    }
    ctl->alpha = ctl->rho / denom;
    ctl->alpha_last = ctl->alpha;
}

__global__ __launch_bounds__(kBlock) void k_fast_beta(Ctl *ctl, const double *__restrict__ p_rr,
                                                      const double *__restrict__ p_rz, uint32_t count,
                                                      double *__restrict__ hist)
{
    __shared__ double red[4];
    if (!ctl->active)
        return;
    const double rr = tree_fold(p_rr, count, red);
    __syncthreads();
    const double rz = tree_fold(p_rz, count, red);
    if (threadIdx.x != 0)
        return;
    const double res = sqrt(rr);
    const unsigned long long it = ctl->iterations;
    ctl->res = res;
    ctl->iterations = it + 1;
    hist[it + 1] = res;
    if (res <= ctl->tol)
    {
        ctl->converged = 1;
        ctl->active = 0;
        return;
    }
    if (fabs(ctl->rho) < 1.0e-18)
    {
        ctl->error = CWF_ERR_RHO_ZERO;
        ctl->error_iter = (int)it;
        ctl->active = 0;
        return;
    }
    ctl->beta = rz / ctl->rho;
    ctl->beta_last = ctl->beta;
    ctl->rho = rz;
}

// x += alpha p; r -= alpha Ap; enforce; z = M^-1 r; block partials of r.r and r.z
__global__ __launch_bounds__(kBlock) void k_fast_update(DevSys s, const float *__restrict__ rhs,
                                                        const float *__restrict__ inv, const float *__restrict__ p,
                                                        const float *__restrict__ Ap, float *__restrict__ x,
                                                        float *__restrict__ r, float *__restrict__ z,
                                                        const Ctl *__restrict__ ctl, double *__restrict__ prr,
                                                        double *__restrict__ prz)
{
    __shared__ double red[4];
    if (!ctl->active)
        return;
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    double rr = 0.0, rz = 0.0;
    if (n < s.N)
    {
        const float alpha = (float)ctl->alpha;
        const uint32_t mk = s.mask[n];
        float rv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k)
        {
            const uint32_t d = 3u * n + k;
            float xv = fmaf(alpha, p[d], x[d]);
            float rw = fmaf(-alpha, Ap[d], r[d]);
            if (mk & (1u << k))
            {
                xv = rhs[d];
                rw = 0.0f;
            }
            x[d] = xv;
            r[d] = rw;
            rv[k] = rw;
        }
        const float *iv = inv + 9u * n;
#pragma unroll
        for (int k = 0; k < 3; ++k)
        {
            float zk = fmaf(iv[3 * k + 2], rv[2], fmaf(iv[3 * k + 1], rv[1], iv[3 * k] * rv[0]));
            zk = (mk & (1u << k)) ? 0.0f : zk;
            z[3u * n + k] = zk;
            rr += (double)rv[k] * (double)rv[k];
            rz += (double)rv[k] * (double)zk;
        }
    }
    const double t0 = block_sum(rr, red);
    if (threadIdx.x == 0)
        prr[blockIdx.x] = t0;
    __syncthreads();
    const double t1 = block_sum(rz, red);
    if (threadIdx.x == 0)
        prz[blockIdx.x] = t1;
}

__global__ __launch_bounds__(kBlock) void k_fast_p_update(DevSys s, const float *__restrict__ z,
                                                          float *__restrict__ p, const Ctl *__restrict__ ctl)
{
    if (!ctl->active)
        return;
    const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
    if (n >= s.N)
        return;
    const float beta = (float)ctl->beta;
    const uint32_t mk = s.mask[n];
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
        const uint32_t d = 3u * n + k;
        const float pv = fmaf(beta, p[d], z[d]);
        p[d] = (mk & (1u << k)) ? 0.0f : pv;
    }
}

inline unsigned grid_for(uint32_t n, uint32_t b) { return (n + b - 1) / b; }

}  // namespace

uint32_t fast_block_count(const cwf_hip_system *h) { return grid_for(h->ds.N, kBlock); }

void fast_keff(const cwf_hip_system *h, const float *x, float *y, bool sanitize, const Ctl *ctl, double *part,
               hipStream_t st)
{
    fast_keff_ds(h->ds, x, y, sanitize, ctl, part, st);
}

void fast_keff_ds(const DevSys &s, const float *x, float *y, bool sanitize, const Ctl *ctl, double *part,
                  hipStream_t st)
{
    if (s.N == 0)
        return;
    const dim3 g(grid_for(s.N, kBlock)), b(kBlock);
    if (s.iso)
    {
        if (sanitize)
            k_keff_fast<true, true><<<g, b, 0, st>>>(s, x, y, ctl, part);
        else
            k_keff_fast<true, false><<<g, b, 0, st>>>(s, x, y, ctl, part);
    }
    else
    {
        if (sanitize)
            k_keff_fast<false, true><<<g, b, 0, st>>>(s, x, y, ctl, part);
        else
            k_keff_fast<false, false><<<g, b, 0, st>>>(s, x, y, ctl, part);
    }
}

// dot over D dofs: one partial per 256-dof block (grid = ceil(D/256) capped) then fold
uint32_t fast_dot_blocks(uint32_t D) { return grid_for(D, kBlock) < 4096u ? grid_for(D, kBlock) : 4096u; }

void fast_dot(const float *a, const float *b, const float *c, uint32_t D, double *pab, double *pac, hipStream_t st)
{
    const uint32_t nb = fast_dot_blocks(D);
    if (nb)
        k_dot_fast<<<nb, kBlock, 0, st>>>(a, b, c, D, pab, pac);
}

void fast_fold(const double *part, uint32_t count, double *out, hipStream_t st)
{
    k_fold_fast<<<1, kBlock, 0, st>>>(part, count, out);
}

void fast_pcg_init(cwf_hip_system *h, const float *rhs, double rel_tol, hipStream_t st)
{
    const DevSys &s = h->ds;
    const uint32_t nbD = fast_dot_blocks(s.D);
    parity_block_jacobi(h, h->inv, st);
    fast_keff(h, h->x, h->Ap, true, nullptr, nullptr, st);
    launch_init_residual(h, rhs, st);  // r = rhs - Ap, enforce (pure f32 ops, shared with parity)
    fast_dot(rhs, rhs, nullptr, s.D, h->part0, nullptr, st);
    fast_dot(h->r, h->r, nullptr, s.D, h->part1, nullptr, st);
    k_fast_init_scalars<<<1, kBlock, 0, st>>>(h->ctl, h->part0, h->part1, nbD, rel_tol, h->hist);
    launch_precond(h, h->ctl, st);
    fast_dot(h->r, h->z, nullptr, s.D, h->part0, nullptr, st);
    k_fast_rho<<<1, kBlock, 0, st>>>(h->ctl, h->part0, nbD);
    launch_p_init(h, st);
}

void fast_pcg_iteration(cwf_hip_system *h, const float *rhs, hipStream_t st, hipEvent_t e0, hipEvent_t e1)
{
    const DevSys &s = h->ds;
    const uint32_t nb = fast_block_count(h);
    if (e0)
        (void)hipEventRecord(e0, st);
    fast_keff(h, h->p, h->Ap, false, h->ctl, h->part0, st);
    if (e1)
        (void)hipEventRecord(e1, st);
    k_fast_alpha<<<1, kBlock, 0, st>>>(h->ctl, h->part0, nb);
    k_fast_update<<<nb, kBlock, 0, st>>>(s, rhs, h->inv, h->p, h->Ap, h->x, h->r, h->z, h->ctl, h->part0,
                                         h->part1);
    k_fast_beta<<<1, kBlock, 0, st>>>(h->ctl, h->part0, h->part1, nb, h->hist);
    k_fast_p_update<<<nb, kBlock, 0, st>>>(s, h->z, h->p, h->ctl);
}

}  // namespace cwf

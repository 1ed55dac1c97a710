// kernels_fast.hip -- FAST-mode reductions and PCG orchestration: fp64 dots with a fixed
// decomposition (one partial per 256-DOF block, fixed-order tree fold) so results are
// deterministic run to run; tolerance-checked against the oracle instead of bit-checked.
// The per-iteration kernels (K_eff tiles with fused p-update/alpha, and the fused x/r/z/p
// update with beta) live in spmv_tiles.hip.
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

// block of 256 threads -> one double (lane order fixed => deterministic); valid in thread 0
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
    __syncthreads();
    return t;
}

// deterministic tree fold of `count` block partials by one 256-thread block
__device__ __forceinline__ double tree_fold(const double *__restrict__ p, uint32_t count, double *red,
                                            uint32_t stride = 1)
{
    double v = 0.0;
    for (uint32_t i = threadIdx.x; i < count; i += kBlock)
        v += p[(size_t)i * stride];
    return block_sum(v, red);
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
        const double t1 = block_sum(s1, red);
        if (threadIdx.x == 0)
            pac[blockIdx.x] = t1;
    }
}

// pcg.cpp:768-796 (norms, tolerance, early convergence)
__global__ __launch_bounds__(kBlock) void k_fast_init_scalars(Ctl *ctl, const double *__restrict__ p_rhs,
                                                              const double *__restrict__ p_rr, uint32_t count,
                                                              uint32_t stride, double rel_tol,
                                                              double *__restrict__ hist)
{
    __shared__ double red[4];
    const double rhs_sq = tree_fold(p_rhs, count, red, stride);
    const double rr = tree_fold(p_rr, count, red, stride);
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
    c.beta = 0.0;  // first search direction p = z + 0 * p
    hist[0] = c.res;
    *ctl = c;
}

// pcg.cpp:804-813
__global__ __launch_bounds__(kBlock) void k_fast_rho(Ctl *ctl, const double *__restrict__ p_rz, uint32_t count)
{
    __shared__ double red[4];
    if (!ctl->active)
        return;
    const double rho = tree_fold(p_rz, count, red);
    if (threadIdx.x != 0)
        return;
    ctl->rho = rho;
    ctl->rho2[0] = rho;
    if (fabs(rho) < 1.0e-18)
    {
        ctl->error = CWF_ERR_RHO_ZERO;
        ctl->error_iter = -1;
        ctl->active = 0;
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

// dot over D dofs: one partial per 256-dof block (grid = ceil(D/256) capped) then fold
__global__ __launch_bounds__(kBlock) void k_perm_copy(const uint32_t *__restrict__ perm, const float *__restrict__ src,
                                                      float *__restrict__ dst, uint32_t N, int w, int scatter)
{
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (uint64_t)N * w)
        return;
    const uint32_t i = (uint32_t)(t / w), k = (uint32_t)(t % w);
    const uint64_t ext = (uint64_t)perm[i] * w + k;
    if (scatter)
        dst[ext] = src[t];
    else
        dst[t] = src[ext];
}

// STREAM-like copy for the bandwidth probe: 16-B loads/stores per lane, four loads in flight per lane
// before their stores, nontemporal (each byte is touched once)
typedef float v4f __attribute__((ext_vector_type(4)));
// one 16-B element per thread, one pass (no grid stride): the fastest copy form measured on MI355X
// (tools/copy_probe.hip: 6.2-6.3 TB/s read + write; persistent grid-stride and blocked copies, plain or
// nontemporal, 4.4-5.3 TB/s; one-pass with 2 / 4 / 8 rows per workgroup 5.8 / 5.6 / 4.3 TB/s)
__global__ __launch_bounds__(256) void k_copy16(const v4f *__restrict__ a, v4f *__restrict__ b, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n)
        b[i] = a[i];
}

void copy16(const void *a, void *b, uint64_t bytes, hipStream_t st)
{
    const uint64_t n = bytes / 16;
    k_copy16<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(static_cast<const v4f *>(a), static_cast<v4f *>(b), n);
}

void perm_gather(const uint32_t *perm, const float *src, float *dst, uint32_t N, int w, hipStream_t st)
{
    const uint64_t n = (uint64_t)N * w;
    if (n)
        k_perm_copy<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, st>>>(perm, src, dst, N, w, 0);
}

void perm_scatter(const uint32_t *perm, const float *src, float *dst, uint32_t N, int w, hipStream_t st)
{
    const uint64_t n = (uint64_t)N * w;
    if (n)
        k_perm_copy<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, st>>>(perm, src, dst, N, w, 1);
}

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

// solve_pcg prologue (pcg.cpp:744-828) in FAST arithmetic
void fast_pcg_init(cwf_hip_system *h, const float *rhs, double rel_tol, hipStream_t st)
{
    const DevSys &s = h->ds;
    const uint32_t nbD = fast_dot_blocks(s.D);
    fast_block_inverse(h, st);
    fast_keff(h, h->x, h->Ap, true, nullptr, nullptr, st);
    launch_init_residual(h, rhs, st);  // r = rhs - Ap, enforce (pure f32 ops, shared with parity)
    fast_dot(rhs, rhs, nullptr, s.D, h->part0, nullptr, st);
    fast_dot(h->r, h->r, nullptr, s.D, h->part1, nullptr, st);
    k_fast_init_scalars<<<1, kBlock, 0, st>>>(h->ctl, h->part0, h->part1, nbD, 1u, rel_tol, h->hist);
    launch_precond(h, h->ctl, st);
    fast_dot(h->r, h->z, nullptr, s.D, h->part0, nullptr, st);
    k_fast_rho<<<1, kBlock, 0, st>>>(h->ctl, h->part0, nbD);
    launch_p_init(h, st);
}

// sharded prologue pieces (comm.cpp interleaves them with the all-gathers and halos)
void fast_init_scalars_strided(cwf_hip_system *h, const double *p_rhs, const double *p_rr, uint32_t count,
                               uint32_t stride, double rel_tol, hipStream_t st)
{
    k_fast_init_scalars<<<1, kBlock, 0, st>>>(h->ctl, p_rhs, p_rr, count, stride, rel_tol, h->hist);
}

void fast_rho_from(cwf_hip_system *h, const double *p_rz, uint32_t count, hipStream_t st)
{
    k_fast_rho<<<1, kBlock, 0, st>>>(h->ctl, p_rz, count);
}

}  // namespace cwf

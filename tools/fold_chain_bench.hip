// Microbenchmark: the latency floor of an ordered fp64 fold (total += partial[c] in chunk order) run by one
// thread, with its operands in registers, LDS (ds_read_b64 / b128) or global memory (L2-resident).
// hipcc --offload-arch=gfx950 -O3 -o fold_chain_bench fold_chain_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int N = 4096;

__global__ __launch_bounds__(256) void k_regs(const double *p, double *out, int reps)
{
    double v[16];
    for (int u = 0; u < 16; ++u)
        v[u] = p[u];
    double a = 0.0;
    if (threadIdx.x == 0)
        for (int r = 0; r < N / 16 * reps; ++r)
#pragma unroll
            for (int u = 0; u < 16; ++u)
                a += v[u];
    if (threadIdx.x == 0)
        out[0] = a;
}

template <int W>
__global__ __launch_bounds__(256) void k_lds(const double *p, double *out, int reps)
{
    __shared__ double buf[N];
    for (int i = threadIdx.x; i < N; i += 256)
        buf[i] = p[i];
    __syncthreads();
    double a = 0.0;
    if (threadIdx.x == 0)
        for (int r = 0; r < reps; ++r)
            for (int i = 0; i < N; i += W)
            {
                double q[W];
#pragma unroll
                for (int u = 0; u < W; ++u)
                    q[u] = buf[i + u];
#pragma unroll
                for (int u = 0; u < W; ++u)
                    a += q[u];
            }
    if (threadIdx.x == 0)
        out[0] = a;
}

// software pipelined: the next W values are loaded while the current W are added
template <int W>
__global__ __launch_bounds__(256) void k_lds_pipe(const double *p, double *out, int reps)
{
    __shared__ double buf[N + W];
    for (int i = threadIdx.x; i < N + W; i += 256)
        buf[i] = i < N ? p[i] : 0.0;
    __syncthreads();
    double a = 0.0;
    if (threadIdx.x == 0)
        for (int r = 0; r < reps; ++r)
        {
            double q[W], n[W];
#pragma unroll
            for (int u = 0; u < W; ++u)
                q[u] = buf[u];
            for (int i = W; i <= N; i += W)
            {
#pragma unroll
                for (int u = 0; u < W; ++u)
                    n[u] = buf[i + u];
#pragma unroll
                for (int u = 0; u < W; ++u)
                    a += q[u];
#pragma unroll
                for (int u = 0; u < W; ++u)
                    q[u] = n[u];
            }
        }
    if (threadIdx.x == 0)
        out[0] = a;
}

template <int W>
__global__ __launch_bounds__(64) void k_glob(const double *p, double *out, int reps)
{
    double a = 0.0;
    if (threadIdx.x == 0)
        for (int r = 0; r < reps; ++r)
            for (int i = 0; i < N; i += W)
            {
                double q[W];
#pragma unroll
                for (int u = 0; u < W; ++u)
                    q[u] = p[i + u];
#pragma unroll
                for (int u = 0; u < W; ++u)
                    a += q[u];
            }
    if (threadIdx.x == 0)
        out[0] = a;
}


// wave-uniform chain: wave 0 loads 64 partials per batch (one coalesced load per lane, PF batches ahead) and
// every lane adds them in order through readlane (SGPR operands), so no LDS and no divergence
__device__ __forceinline__ double lane_val(double v, int l)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int PF>
__global__ __launch_bounds__(256) void k_lane(const double *p, double *out, int reps)
{
    double a = 0.0;
    if (threadIdx.x < 64)
        for (int r = 0; r < reps; ++r)
        {
            double q[PF];
#pragma unroll
            for (int b = 0; b < PF; ++b)
                q[b] = p[64 * b + threadIdx.x];
            for (int base = 0; base < N; base += 64 * PF)
            {
#pragma unroll
                for (int b = 0; b < PF; ++b)
                {
                    const double v = q[b];
                    const int nb = base + 64 * (b + PF);
                    q[b] = nb < N ? p[nb + threadIdx.x] : 0.0;
#pragma unroll
                    for (int l = 0; l < 64; ++l)
                        a += lane_val(v, l);
                }
            }
        }
    if (threadIdx.x == 0)
        out[blockIdx.x] = a;
}

// ping-pong: two register sets of W doubles (read as W/2 16-B LDS reads); the next set's reads are issued before
// the current set's dependent adds, so the adds wait only for reads issued a batch earlier
template <int W>
__global__ __launch_bounds__(256) void k_lds_pp(const double *p, double *out, int reps)
{
    __shared__ double2 buf[(N + 2 * W) / 2];
    double *b = reinterpret_cast<double *>(buf);
    for (int i = threadIdx.x; i < N + 2 * W; i += 256)
        b[i] = i < N ? p[i] : 0.0;
    __syncthreads();
    double a = 0.0;
    if (threadIdx.x == 0)
        for (int r = 0; r < reps; ++r)
        {
            double2 A[W / 2], B[W / 2];
#pragma unroll
            for (int u = 0; u < W / 2; ++u)
                A[u] = buf[u];
            for (int i = 0; i < N; i += 2 * W)
            {
#pragma unroll
                for (int u = 0; u < W / 2; ++u)
                    B[u] = buf[(i + W) / 2 + u];
#pragma unroll
                for (int u = 0; u < W / 2; ++u)
                {
                    a += A[u].x;
                    a += A[u].y;
                }
#pragma unroll
                for (int u = 0; u < W / 2; ++u)
                    A[u] = buf[(i + 2 * W) / 2 + u];
#pragma unroll
                for (int u = 0; u < W / 2; ++u)
                {
                    a += B[u].x;
                    a += B[u].y;
                }
            }
        }
    if (threadIdx.x == 0)
        out[0] = a;
}

// plain batches read as 16-B LDS reads
template <int W>
__global__ __launch_bounds__(256) void k_lds128(const double *p, double *out, int reps)
{
    __shared__ double2 buf[N / 2];
    double *b = reinterpret_cast<double *>(buf);
    for (int i = threadIdx.x; i < N; i += 256)
        b[i] = p[i];
    __syncthreads();
    double a = 0.0;
    if (threadIdx.x == 0)
        for (int r = 0; r < reps; ++r)
            for (int i = 0; i < N / 2; i += W / 2)
            {
                double2 q[W / 2];
#pragma unroll
                for (int u = 0; u < W / 2; ++u)
                    q[u] = buf[i + u];
#pragma unroll
                for (int u = 0; u < W / 2; ++u)
                {
                    a += q[u].x;
                    a += q[u].y;
                }
            }
    if (threadIdx.x == 0)
        out[0] = a;
}

// the chain with wave 0's lanes all active on uniform addresses: the compiler turns the loads into scalar
// loads (SGPR operands of v_add_f64), one set of W requested ahead of the current set's adds
template <int W>
__global__ __launch_bounds__(64) void k_sgpr2(const double *__restrict__ p, double *out, int reps)
{
    double a = 0.0;
    for (int r = 0; r < reps; ++r)
    {
        double A[W], B[W];
#pragma unroll
        for (int u = 0; u < W; ++u)
            A[u] = p[u];
        for (int i = 0; i < N; i += 2 * W)
        {
#pragma unroll
            for (int u = 0; u < W; ++u)
                B[u] = p[i + W + u];
#pragma unroll
            for (int u = 0; u < W; ++u)
                a += A[u];
#pragma unroll
            for (int u = 0; u < W; ++u)
                A[u] = p[i + 2 * W + u];
#pragma unroll
            for (int u = 0; u < W; ++u)
                a += B[u];
        }
    }
    if (threadIdx.x == 0)
        out[0] = a;
}

template <typename K>
static void timeit(const char *name, K kern, int threads, const double *p, double *out, int grid = 1)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int reps : {1, 9})
    {
        kern<<<grid, threads>>>(p, out, reps);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        for (int k = 0; k < 20; ++k)
            kern<<<grid, threads>>>(p, out, reps);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("%-14s g%-5d reps %d: %8.2f us per launch, %6.2f ns per add\n", name, grid, reps, ms * 1e3 / 20,
               ms * 1e6 / 20 / (double)(N * reps));
    }
}

int main()
{
    std::vector<double> h(N + 128);
    for (int i = 0; i < N + 128; ++i)
        h[i] = 1.0 / (i + 1);
    double *p, *out;
    (void)hipMalloc(&p, (N + 128) * sizeof(double));
    (void)hipMalloc(&out, 8 * 4096);
    (void)hipMemcpy(p, h.data(), (N + 128) * sizeof(double), hipMemcpyHostToDevice);
    timeit("regs", k_regs, 256, p, out);
    timeit("lds W8", k_lds<8>, 256, p, out);
    timeit("lds W16", k_lds<16>, 256, p, out);
    timeit("lds W32", k_lds<32>, 256, p, out);
    timeit("lds_pipe W8", k_lds_pipe<8>, 256, p, out);
    timeit("lds_pipe W16", k_lds_pipe<16>, 256, p, out);
    timeit("glob W16", k_glob<16>, 64, p, out);
    timeit("glob W64", k_glob<64>, 64, p, out);
    timeit("lds_pp W8", k_lds_pp<8>, 256, p, out);
    timeit("lds_pp W16", k_lds_pp<16>, 256, p, out);
    timeit("lds_pp W24", k_lds_pp<24>, 256, p, out);
    timeit("lds128 W16", k_lds128<16>, 256, p, out);
    timeit("lds128 W32", k_lds128<32>, 256, p, out);
    timeit("sgpr2 W8", k_sgpr2<8>, 64, p, out);
    timeit("sgpr2 W16", k_sgpr2<16>, 64, p, out);
    timeit("sgpr2 W24", k_sgpr2<24>, 64, p, out);
    timeit("lane PF4", k_lane<4>, 256, p, out);
    timeit("lane PF8", k_lane<8>, 256, p, out);
    timeit("lane PF8", k_lane<8>, 256, p, out, 1024);
    timeit("lds W16", k_lds<16>, 256, p, out, 1024);
    h.resize(N);
    for (int i = 0; i < N; ++i)
        h[i] = 1.0 / (i + 1);
    double ref = 0.0;
    for (int i = 0; i < N; ++i)
        ref += h[i];
    double got = 0.0;
    k_lane<8><<<1, 256>>>(p, out, 1);
    (void)hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost);
    printf("lane fold == host sequential fold: %d\n", (int)(got == ref));
    k_lds_pp<16><<<1, 256>>>(p, out, 1);
    (void)hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost);
    printf("lds_pp fold == host sequential fold: %d\n", (int)(got == ref));
    k_sgpr2<16><<<1, 64>>>(p, out, 1);
    (void)hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost);
    printf("sgpr2 fold == host sequential fold: %d\n", (int)(got == ref));
    return 0;
}

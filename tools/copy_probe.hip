// HBM copy / read ceiling probe: variants of a 16-B-lane device copy over 2 GiB buffers, to calibrate
// the measured-copy figure bench.py reports beside the roofline (cwf_hip_bandwidth_probe).
// build: hipcc -O3 --offload-arch=gfx950 tools/copy_probe.hip -o tools/copy_probe ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_copy(const v4f *__restrict__ a, v4f *__restrict__ b, uint64_t n)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride)
    {
        v4f v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = NTL ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (NTS)
                __builtin_nontemporal_store(v[u], b + i + u * stride);
            else
                b[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride)
        b[i] = a[i];
}

// persistent, blocked: workgroup b copies the contiguous chunk [b n / g, (b + 1) n / g), U wave-wide 4-KB
// rows in flight per iteration (rows adjacent)
template <int U>
__global__ __launch_bounds__(256) void k_copy_blocked(const v4f *__restrict__ a, v4f *__restrict__ b, uint64_t n)
{
    const uint64_t lo = n * blockIdx.x / gridDim.x, hi = n * (blockIdx.x + 1) / gridDim.x;
    uint64_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 256 < hi; i += U * 256)
    {
        v4f v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = a[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u)
            b[i + u * 256] = v[u];
    }
    for (; i < hi; i += 256)
        b[i] = a[i];
}

// one pass, U adjacent rows per workgroup (grid = n / (256 U))
template <int U>
__global__ __launch_bounds__(256) void k_copy_pass(const v4f *__restrict__ a, v4f *__restrict__ b, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * 256 < n)
            v[u] = a[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * 256 < n)
            b[i + u * 256] = v[u];
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const v4f *__restrict__ a, float *__restrict__ out, uint64_t n)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    for (; i + (U - 1) * stride < n; i += U * stride)
    {
        v4f v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += v[u];
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f)
        out[0] = 1.f;
}

template <typename F>
double time_ms(F f, int reps)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    f();
    (void)hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; ++r)
        f();
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main()
{
    const uint64_t bytes = 2ull << 30, n = bytes / 16;
    v4f *a = nullptr, *b = nullptr;
    float *o = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&o, 16) != hipSuccess)
        return 1;
    (void)hipMemset(a, 0, bytes);
    (void)hipMemset(b, 0, bytes);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int reps = 10;
    const auto copy_line = [&](const char *name, auto kern, unsigned grid) {
        const double ms = time_ms([&] { kern<<<grid, 256>>>(a, b, n); }, reps);
        printf("%-34s grid %6u  %8.1f GB/s (read + write)\n", name, grid, 2.0 * bytes / (ms * 1e-3) / 1e9);
    };
    copy_line("copy nt/nt U4 (bench probe)", k_copy<4, true, true>, 256u * 8);
    copy_line("copy plain U4", k_copy<4, false, false>, 256u * 8);
    copy_line("copy plain U8", k_copy<8, false, false>, 256u * 8);
    copy_line("copy plain U4 grid CUs x 4", k_copy<4, false, false>, (unsigned)cus * 4);
    copy_line("copy plain U4 grid CUs x 32", k_copy<4, false, false>, (unsigned)cus * 32);
    copy_line("copy nt load / plain store U4", k_copy<4, true, false>, 256u * 8);
    copy_line("copy plain load / nt store U4", k_copy<4, false, true>, 256u * 8);
    copy_line("copy plain U1 one pass", k_copy<1, false, false>, (unsigned)((n + 255) / 256));
    copy_line("copy grid-stride U1", k_copy<1, false, false>, 256u * 8);
    copy_line("copy grid-stride U1 grid CUs x 8", k_copy<1, false, false>, (unsigned)cus * 8);
    copy_line("copy blocked U1", k_copy_blocked<1>, 256u * 8);
    copy_line("copy blocked U4", k_copy_blocked<4>, 256u * 8);
    copy_line("copy blocked U4 grid CUs x 4", k_copy_blocked<4>, (unsigned)cus * 4);
    copy_line("copy pass U2", k_copy_pass<2>, (unsigned)((n + 511) / 512));
    copy_line("copy pass U4", k_copy_pass<4>, (unsigned)((n + 1023) / 1024));
    copy_line("copy pass U8", k_copy_pass<8>, (unsigned)((n + 2047) / 2048));
    for (unsigned g : {256u * 8, (unsigned)cus * 16})
    {
        const double ms = time_ms([&] { k_read<8><<<g, 256>>>(a, o, n); }, reps);
        printf("%-34s grid %6u  %8.1f GB/s (read)\n", "read plain U8", g, bytes / (ms * 1e-3) / 1e9);
    }
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(o);
    return 0;
}

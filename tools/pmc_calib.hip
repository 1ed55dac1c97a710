// FETCH_SIZE / WRITE_SIZE calibration on known byte counts in the K_eff kernels' own access widths
// (MI355X_MICROARCH.md HBM section: FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read; other
// widths are uncalibrated). Each kernel touches a known number of bytes of 1 GiB+ buffers (far past the 256 MiB
// MALL, so no re-read is absorbed on-die); run under rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, and divide
// the per-launch counters (KiB) by the known bytes:
//   rd16   16-B lanes, coalesced stream              (the guide's calibrated case: FETCH x2)
//   rd12   12-B lanes (buffer_load_dwordx3), coalesced stream of node records
//   rd12g  12-B lanes gathered through a node permutation that is random inside 64-KiB windows (each record read
//          once; lines of a window are shared by gathers spread over one workgroup's lifetime)
//   rd12p  12-B lanes, the lattice brick pattern: a 34 x 10 tile of one plane of a 1024 x 1024 x nz node grid per
//          workgroup, tiles overlapping by one node (reads 340 / 256 x the 256 interior nodes' bytes)
//   wr12   12-B lanes (buffer_store_dwordx3), coalesced stream
//   wr16   16-B lanes, coalesced stream (the guide's calibrated WRITE case)
// build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib ; prints the known bytes per launch.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, -1, 0x00020000);
}

__global__ __launch_bounds__(256) void rd16(const v4f *__restrict__ a, uint64_t n, float *__restrict__ sink)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    float s = 0.f;
    if (i < n)
    {
        const v4f v = a[i];
        s = v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f)
        sink[0] = s;
}

__global__ __launch_bounds__(256) void rd12(const float *__restrict__ a, uint32_t n, float *__restrict__ sink)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const auto r = rsrc(a);
    float s = 0.f;
    if (i < n)
    {
        const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(r, 12u * i, 0, 0);
        s = __uint_as_float(w.x) + __uint_as_float(w.y) + __uint_as_float(w.z);
    }
    if (s == 12345.f)
        sink[0] = s;
}

__global__ __launch_bounds__(256) void rd12g(const float *__restrict__ a, const uint32_t *__restrict__ perm, uint32_t n,
                                             float *__restrict__ sink)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const auto r = rsrc(a);
    float s = 0.f;
    if (i < n)
    {
        const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(r, 12u * perm[i], 0, 0);
        s = __uint_as_float(w.x) + __uint_as_float(w.y) + __uint_as_float(w.z);
    }
    if (s == 12345.f)
        sink[0] = s;
}

// workgroup (bx, by, k): the 34 x 10 nodes (bx 32 - 1 .. bx 32 + 32, by 8 - 1 .. by 8 + 8) of plane k, two entries
// per thread (340 entries), 12 B each
__global__ __launch_bounds__(256) void rd12p(const float *__restrict__ a, uint32_t nx, uint32_t ny,
                                             float *__restrict__ sink)
{
    const uint32_t nbx = (nx - 2) / 32, nby = (ny - 2) / 8;
    const uint32_t bx = blockIdx.x % nbx, by = (blockIdx.x / nbx) % nby, k = blockIdx.x / (nbx * nby);
    const auto r = rsrc(a);
    float s = 0.f;
    for (uint32_t e = threadIdx.x; e < 340; e += 256)
    {
        const uint32_t i = bx * 32 + e % 34, j = by * 8 + e / 34;
        const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(r, 12u * ((k * ny + j) * nx + i), 0, 0);
        s += __uint_as_float(w.x) + __uint_as_float(w.y) + __uint_as_float(w.z);
    }
    if (s == 12345.f)
        sink[0] = s;
}

__global__ __launch_bounds__(256) void wr12(float *__restrict__ a, uint32_t n)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const auto r = rsrc(a);
    if (i < n)
    {
        const u32x3 v = {i, i + 1, i + 2};
        __builtin_amdgcn_raw_buffer_store_b96(v, r, 12u * i, 0, 0);
    }
}

__global__ __launch_bounds__(256) void wr16(v4f *__restrict__ a, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n)
        a[i] = v4f{(float)i, 1.f, 2.f, 3.f};
}

int main()
{
    const uint64_t bytes = 1536ull << 20;  // 1.5 GiB per buffer
    const uint32_t nodes = (uint32_t)(bytes / 12);
    float *a, *sink;
    uint32_t *perm;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 16) != hipSuccess ||
        hipMalloc(&perm, 4ull * nodes) != hipSuccess)
        return 1;
    (void)hipMemset(a, 0, bytes);
    std::vector<uint32_t> hp(nodes);
    const uint32_t win = 65536 / 12;  // records per 64-KiB window
    uint64_t st = 88172645463325252ull;
    for (uint32_t w0 = 0; w0 < nodes; w0 += win)
    {
        const uint32_t w1 = w0 + win < nodes ? w0 + win : nodes;
        for (uint32_t i = w0; i < w1; ++i)
            hp[i] = i;
        for (uint32_t i = w1 - 1; i > w0; --i)
        {
            st ^= st << 13;
            st ^= st >> 7;
            st ^= st << 17;
            const uint32_t j = w0 + (uint32_t)(st % (i - w0 + 1));
            const uint32_t t = hp[i];
            hp[i] = hp[j];
            hp[j] = t;
        }
    }
    (void)hipMemcpy(perm, hp.data(), 4ull * nodes, hipMemcpyHostToDevice);
    const uint64_t n16 = bytes / 16;
    const uint32_t nx = 1026, ny = 1026, nz = (uint32_t)(nodes / (nx * ny));
    const uint32_t tiles = ((nx - 2) / 32) * ((ny - 2) / 8) * nz;
    for (int rep = 0; rep < 3; ++rep)
    {
        rd16<<<(unsigned)((n16 + 255) / 256), 256>>>(reinterpret_cast<const v4f *>(a), n16, sink);
        rd12<<<(nodes + 255) / 256, 256>>>(a, nodes, sink);
        rd12g<<<(nodes + 255) / 256, 256>>>(a, perm, nodes, sink);
        rd12p<<<tiles, 256>>>(a, nx, ny, sink);
        wr12<<<(nodes + 255) / 256, 256>>>(a, nodes);
        wr16<<<(unsigned)((n16 + 255) / 256), 256>>>(reinterpret_cast<v4f *>(a), n16);
    }
    if (hipDeviceSynchronize() != hipSuccess)
        return 2;
    printf("{\"rd16\": %llu, \"rd12\": %llu, \"rd12g\": %llu, \"rd12g_perm\": %llu, \"rd12p\": %llu, "
           "\"rd12p_unique\": %llu, \"wr12\": %llu, \"wr16\": %llu}\n",
           (unsigned long long)bytes, 12ull * nodes, 12ull * nodes, 4ull * nodes, 12ull * 340 * tiles,
           12ull * (uint64_t)nx * ny * nz, 12ull * nodes, (unsigned long long)bytes);
    return 0;
}

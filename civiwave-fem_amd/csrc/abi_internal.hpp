// abi_internal.hpp -- what the C-ABI translation units (abi.cpp: handles, abi_pcg.cpp: apply_keff / block
// Jacobi / dot / solve_pcg, abi_stepper.cpp: the Stepper) share: the HIP error macro, device allocation and
// upload, vector staging between the caller's layout and the handle's, and the PCG driver.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "cwf_internal.hpp"

#define HIPTRY(h, expr)                                                                                        \
    do                                                                                                         \
    {                                                                                                          \
        hipError_t e__ = (expr);                                                                               \
        if (e__ != hipSuccess)                                                                                 \
            return hip_fail((h), e__, #expr);                                                                  \
    } while (0)


namespace cwf
{

template <class T> inline int dalloc(cwf_hip_system *h, T **p, size_t count)
{
    void *q = nullptr;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess)
        return set_error(h, CWF_ERR_ALLOC, "failed to allocate device buffer",
                         "bytes=" + std::to_string(bytes));
    h->owned.push_back(q);
    h->bytes += bytes;
    *p = static_cast<T *>(q);
    return 0;
}

// the Dirichlet mask can ride in node_part_off's top bits when the offsets leave them free
inline bool ht_off_mask_ok(const std::vector<uint32_t> &npo) { return npo.back() <= cwf::kPartOffBits; }

template <class T> inline int upload(cwf_hip_system *h, T **dst, const T *src, size_t count)
{
    if (int st = dalloc(h, dst, count))
        return st;
    if (count)
        HIPTRY(h, hipMemcpy(*dst, src, count * sizeof(T), hipMemcpyHostToDevice));
    return 0;
}

bool iso_pattern(const double *D);
int parity_incidence_slots(cwf_hip_system *h);
int parity_force_buffer(cwf_hip_system *h);
int check_ready(cwf_hip_system *h);
int stage_in(cwf_hip_system *h, const float *src, float *scratch, uint64_t n, int kind, const float **out);
int stage_vec(cwf_hip_system *h, const float *src, float *scratch, int kind, int w, const float **out);
int vec_in(cwf_hip_system *h, const float *src, float *dst, int kind, int w);
int vec_out(cwf_hip_system *h, const float *src, float *dst, int kind, int w);
std::vector<uint32_t> morton_node_order(const double *X, uint64_t N);
bool groups_enabled();
uint32_t group_lanes(uint64_t E);
std::string pcg_error_message(int code, int iter, std::string *ctx);
// solve_pcg on device buffers for a group (one handle, or every rank of a LOCAL sharded system)
int run_pcg_group(const std::vector<cwf_hip_system *> &g, const std::vector<const float *> &rhs,
                  const cwf_pcg_settings &set, cwf_pcg_telemetry *tel);
int run_pcg(cwf_hip_system *h, const float *rhs_dev, const cwf_pcg_settings &set, cwf_pcg_telemetry *tel);

}  // namespace cwf

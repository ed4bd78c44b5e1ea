// Internal helpers shared by the libmsl_hip.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <atomic>
#include "../../include/msl_hip.h"

#define MSL_ABI_VERSION 3

// Every kernel launch of the library goes through MSL_LAUNCH (r06): the block's thread
// count is checked against the kernel's own __launch_bounds__ (its code object's max flat workgroup size,
// hipFuncGetAttributes, queried once per launch site) before the launch, and an oversized block returns
// MSL_ERR_LAUNCH from the entry point instead of launching.  r05's kg2 experiment launched 256-thread
// helper kernels with a 512-thread block: an asynchronous "unspecified launch failure", not a status.
#define MSL_LAUNCH(K, GRID, BLOCK, SHM, ST, ...)                                                    \
  do {                                                                                              \
    static std::atomic<int> msl_bound_{0};                                                          \
    const int msl_e_ = ::msl::launch_guard(reinterpret_cast<const void*>(K), dim3(BLOCK), msl_bound_); \
    if (msl_e_ != MSL_OK) return msl_e_;                                                            \
    hipLaunchKernelGGL(K, GRID, BLOCK, SHM, ST, __VA_ARGS__);                                       \
  } while (0)

#define MSL_TRY(...)                 \
  do {                               \
    const int msl_t_ = (__VA_ARGS__); \
    if (msl_t_ != MSL_OK) return msl_t_; \
  } while (0)

#define MSL_CHECK_LAUNCH()                         \
  do {                                             \
    hipError_t e_ = hipGetLastError();             \
    if (e_ != hipSuccess) return (int)e_;          \
  } while (0)

namespace msl {

// MSL_OK if a block of `block` threads fits kernel k's launch bound (cached in `bound` after the first
// query), MSL_ERR_LAUNCH if not, the hipError_t if the query fails
static inline int launch_guard(const void* k, dim3 block, std::atomic<int>& bound) {
  int b = bound.load(std::memory_order_relaxed);
  if (b == 0) {
    hipFuncAttributes fa;
    const hipError_t e = hipFuncGetAttributes(&fa, k);
    if (e != hipSuccess) return (int)e;
    b = fa.maxThreadsPerBlock;
    bound.store(b, std::memory_order_relaxed);
  }
  return (long long)block.x * block.y * block.z > b ? MSL_ERR_LAUNCH : MSL_OK;
}

static inline hipStream_t as_stream(msl_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

__host__ __device__ static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// 64-lane wave reductions (CDNA wave = 64).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// absmax[r] = max |t[r][0..p)| for r < c (bn.hip; stream-ordered memset + one launch, integer
// atomicMax on the float bits: exact and order-independent).  The f16x3 convs' per-row partials.
int absmax_rows(const float* t, int c, int p, float* absmax, hipStream_t st);

// The kernel forms of a call (msl_forms, include/msl_hip.h): NULL = the defaults (f16x3, the hybrid
// stream-K schedule, one-launch packs, fused BN)
constexpr msl_forms kDefaultForms = {5, 1, 1, 1};
static inline const msl_forms& forms_of(const msl_forms* f) { return f ? *f : kDefaultForms; }
static inline bool forms_bad(const msl_forms* f) {
  return f && ((f->f32_form != 0 && f->f32_form != 2 && f->f32_form != 5) || (unsigned)f->sk_hybrid > 1u ||
               (unsigned)f->pack_form > 1u || (unsigned)f->bn_fused > 1u);
}

}  // namespace msl

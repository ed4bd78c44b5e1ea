// Internal helpers shared by the libmsl_hip.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include "../../include/msl_hip.h"

#define MSL_ABI_VERSION 2

#define MSL_CHECK_LAUNCH()                         \
  do {                                             \
    hipError_t e_ = hipGetLastError();             \
    if (e_ != hipSuccess) return (int)e_;          \
  } while (0)

namespace msl {

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

// 2^k with k = clamp(141 - biased exponent of mx, -100, 100): mx * 2^k in [2^14, 2^15) (fp16's
// largest finite value is 65504); a zero / fp32-subnormal maximum gives 2^100, inf / NaN 2^-100.
// `inv` = 2^-k.  Powers of two: scaling and unscaling are exact (the f16x3 operand scales).
__device__ __forceinline__ float pow2_scale(float mx, float& inv) {
  const int e = (int)((__float_as_uint(mx) >> 23) & 0xffu);
  const int k = min(100, max(-100, 141 - e));
  inv = __uint_as_float((unsigned)(127 - k) << 23);
  return __uint_as_float((unsigned)(127 + k) << 23);
}

// ---------------------------------------------------------------- stream-K output, folded
// The forward-form GEMMs (dconv_kernels.h fwd_sk_body) cut the (tile, K-step) space of their output
// into equal worker ranges: worker w covers iterations [sk_start(w), sk_start(w + 1)).  A tile whose
// iterations span several workers leaves one piece per worker (slot 1 for the tile's head piece, 0
// otherwise) that k_sk_reduce sums in worker order.  SkView lets a consumer of the output - the BN
// kernels (bn.hip, msl_bn_fwd_pend / msl_bn_bwd_pend) - do that sum itself while it reads the
// output, with k_sk_reduce's exact operation order, so the GEMM's output is not written, re-read
// and written again between the two launches.
__host__ __device__ __forceinline__ int sk_start(int w, int T, int NW) { return (int)((unsigned)(w * T) / (unsigned)NW); }
__host__ __device__ __forceinline__ int sk_worker_of(int i, int T, int NW) {
  return (int)((unsigned)((i + 1) * NW - 1) / (unsigned)T);
}
constexpr int kFoldMaxPieces = 4;  // pieces per split tile a folding consumer sums (unrolled)

struct SkView {
  const float* part;  // [NW][2][bm][bn] pieces
  float* out;         // [M][P] the GEMM's output: unsplit tiles final, split tiles (accum: the old values)
  int bm, bn, tiles_n, ks, nw, t, tdp, accum, P;
};

static inline SkView sk_view(const msl_sk_pending* p, float* out) {
  SkView v;
  v.part = p->part;
  v.out = out;
  v.bm = p->bm;
  v.bn = p->bn;
  v.tiles_n = p->tiles_n;
  v.ks = p->ks;
  v.nw = p->nw;
  v.t = p->t;
  v.tdp = p->tdp;
  v.accum = p->accum;
  v.P = p->p;
  return v;
}

// The fold of one output row m (one BN block = one channel = one GEMM row): a table of the row's
// tiles in LDS, {first worker, pieces} (pieces 0: the GEMM stored the tile itself), built once per
// block so each element costs a table read and its piece loads.  Worker w_lo's piece of a tile sits in
// slot 1 (its range reaches the tile's first K-step), every later worker's in slot 0 (k_sk_reduce:
// slot = sk_start(w) > tile start ? 0 : 1).
constexpr int kFoldBN = 128;          // pixel tile of the forward-form GEMMs (kSkBN)
constexpr int kFoldMaxTilesN = 1024;  // pixel tiles of a row a table holds

struct FoldTable {
  const int2* tab;
  __amdgpu_buffer_rsrc_t rout, rpart;
  __device__ __forceinline__ void build(const SkView& v, int m) {
    __shared__ int2 s_tab[kFoldMaxTilesN];
    const int tm = m / v.bm;
    for (int tn = threadIdx.x; tn < v.tiles_n; tn += blockDim.x) {
      const int t = tm * v.tiles_n + tn;
      int lo = 0, np = 0;
      if (t >= v.tdp) {
        const int tl = t - v.tdp;
        lo = sk_worker_of(tl * v.ks, v.t, v.nw);
        const int hi = sk_worker_of((tl + 1) * v.ks - 1, v.t, v.nw);
        if (hi > lo) np = hi - lo + 1;
      }
      s_tab[tn] = make_int2(lo, np);
    }
    rout = __builtin_amdgcn_make_buffer_rsrc((void*)v.out, (short)0, 0x7fffffff, 0x00020000);
    rpart = __builtin_amdgcn_make_buffer_rsrc((void*)v.part, (short)0, 0x7fffffff, 0x00020000);
    __syncthreads();
    tab = s_tab;
  }
};

// One element of a folded row in two phases, so that the loads of several elements are in flight
// together: issue() starts them (the ones a case does not need get an out-of-range offset: they return 0
// without a fetch), value() combines them into out[m][gp] as k_sk_reduce leaves it - a split tile is
// (accum ? old : 0) + (its FP or fewer pieces summed from 0 in worker order).
template <int FP>
struct FoldVal {
  float base, pc[FP];
  int np;
  __device__ __forceinline__ void issue(const FoldTable& ft, const SkView& v, int m, int gp, bool valid) {
    constexpr unsigned OOB = 0x80000000u;
    const int2 e = valid ? ft.tab[gp / kFoldBN] : make_int2(0, 0);
    np = e.y;
    const unsigned idx = (unsigned)m * (unsigned)v.P + (unsigned)gp;
    base = __uint_as_float(
        __builtin_amdgcn_raw_buffer_load_b32(ft.rout, (valid && (np == 0 || v.accum)) ? idx * 4u : OOB, 0, 0));
    const unsigned psz = (unsigned)(v.bm * kFoldBN * 4);
    const unsigned off = (unsigned)((m % v.bm) * kFoldBN + gp % kFoldBN) * 4u;
#pragma unroll
    for (int u = 0; u < FP; ++u)
      pc[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          ft.rpart, u < np ? (unsigned)((e.x + u) * 2 + (u == 0 ? 1 : 0)) * psz + off : OOB, 0, 0));
  }
  __device__ __forceinline__ float value(int accum) const {
    if (np == 0) return base;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < FP; ++u)
      if (u < np) acc += pc[u];
    return accum ? base + acc : acc;
  }
};

}  // namespace msl

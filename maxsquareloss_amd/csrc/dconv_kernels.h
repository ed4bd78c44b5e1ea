// Implicit-GEMM kernel templates for the dilated 3x3 conv (design notes in dconv.hip).
// Included by dconv.hip (libmsl_hip.so).
#pragma once
#include <type_traits>

#include "msl_internal.h"

namespace msl {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;  // buffer-op cache policy: sc1 (bypass L1, drop from L2 on store)

constexpr int kCB = 16;        // image channels per forward K-group (one tap, 16 channels)
constexpr int kPackPad = 128;  // packed-weight row padding (>= any BM)

struct FwdArgs {
  const float* A;     // packed weights [Kp][lda]
  const float* B;     // image [cimg][P]
  float* C;           // out [M][P] or slabs [S][M][P]
  const float* bias;  // [nbias][M] or null (only used when S == 1)
  int nbias;
  // H x W = one image; P = nimg * H * W pixels: a batch of images stacked along the pixel axis
  // ([C][nimg][H][W]), a tap's shifted read never crossing into the neighbouring image (its row
  // is validated modulo H)
  int M, lda, H, W, P, cimg, ncb, dil0, dil1, ksteps, kps;  // ksteps counts BK-deep steps
  int taps;           // 9 (3x3) or 1 (pointwise: dil0 = 0, so the single tap has no shift)
  long long slab;
  const void* Ax6;    // kMathX6P/PP: A split into bf16 planes [ks][plane][k half][lda][8] (k_split_pack)
  const void* Bx6;    // the BP form: the image operand's fp16 planes (k_split_img)
  int accum;          // stream-K forms: C = C_old + result (the fused residual-gradient sum)
  // r06, accum with accres != null: C = mask(accres) + result instead, mask(accres)[m][n] = accres[m][n] where bit
  // (n % hw) of row m * accni + n / hw of accmask is set, else 0 (hw = P / accni): the identity residual's
  // gradient of a bottleneck - its bn3 backward's ReLU-masked dy - formed in this epilogue from dy and the
  // forward's y > 0 bits, so the BN backward need not write it (msl_pconv_dgrad_resmask*)
  const float* accres;
  const unsigned long long* accmask;
  int accni;
  // kMathH3P: Ax6 holds A * sA as two fp16 planes [ks][plane][k half][lda][8]; ascale = {sA,
  // 1/sA} (written by the pack); bpart = the kNPart absmax partials of B (k_absmax)
  const float* ascale;
  const float* bpart;
  int bnpart;  // partials in bpart
};

// mask(accres)[m][n] of FwdArgs (r06): accres[m * P + n] if the forward's y > 0 bit of that element is set
__device__ __forceinline__ float acc_masked(const FwdArgs& a, int m, int n) {
  const int hw = a.P / a.accni;
  const int img = n / hw, px = n - img * hw;
  const unsigned long long w = a.accmask[(long long)(m * a.accni + img) * ((hw + 63) >> 6) + (px >> 6)];
  return ((w >> (px & 63)) & 1ull) ? a.accres[(long long)m * a.P + n] : 0.f;
}

struct WgradArgs {
  const float* dy;  // [M][P]
  const float* x;   // [N][P]
  float* C;         // dW [nbranch][M][N][taps] or slabs of that
  int M, N, H, W, P, dil0, dil1, ntap, ksteps, kps, accumulate;
  int taps;         // taps per branch: 9, or 1 for a pointwise conv (dil0 = 0)
  long long slab, cbranch;
};

// acc[i][j] += A_tile(kk..kk+BK) x B_tile over one LDS stage; A at As[k][m], B at Bs[k][n].
// All of the stage's operand reads are issued before the first MFMA, so the LDS latency of
// k-pair kk+1.. overlaps the MFMAs of k-pair kk (the compiler emits counted lgkmcnt waits).
template <int BK, int TM, int TN, int LDA_S, int LDB_S>
__device__ __forceinline__ void mfma_stage(const float* As, const float* Bs,
                                           int wm, int wn, int lane, f32x16 (&acc)[TM][TN]) {
  const int l32 = lane & 31, kh = lane >> 5;
  constexpr int KP = BK / 2;
  float av[KP][TM], bv[KP][TN];
#pragma unroll
  for (int kp = 0; kp < KP; ++kp) {
    const int kr = 2 * kp + kh;
#pragma unroll
    for (int i = 0; i < TM; ++i) av[kp][i] = As[kr * LDA_S + wm + i * 32 + l32];
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[kp][j] = Bs[kr * LDB_S + wn + j * 32 + l32];
  }
#pragma unroll
  for (int kp = 0; kp < KP; ++kp)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kp][i], bv[kp][j], acc[i][j], 0, 0, 0);
}

// Software-pipelined variant: the operands of k-pair kp+1 are read while the MFMAs of k-pair kp
// run (scheduling barriers keep the compiler from sinking the reads next to their use, which
// exposes the LDS latency once per k-pair), and `mid` - the next stage's DMA issue - is placed
// after the first k-pair so its address arithmetic overlaps the MFMA pipe.
template <int BK, int TM, int TN, int LDA_S, int LDB_S, typename F>
__device__ __forceinline__ void mfma_stage_pipe(const float* As, const float* Bs,
                                                int wm, int wn, int lane, f32x16 (&acc)[TM][TN], F&& mid) {
  const int l32 = lane & 31, kh = lane >> 5;
  constexpr int KP = BK / 2;
  float av[2][TM], bv[2][TN];
  auto load = [&](int kp, int buf) {
    const int kr = 2 * kp + kh;
#pragma unroll
    for (int i = 0; i < TM; ++i) av[buf][i] = As[kr * LDA_S + wm + i * 32 + l32];
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[buf][j] = Bs[kr * LDB_S + wn + j * 32 + l32];
  };
  load(0, 0);
#pragma unroll
  for (int kp = 0; kp < KP; ++kp) {
    const int cur = kp & 1;
    if (kp + 1 < KP) load(kp + 1, cur ^ 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][i], bv[cur][j], acc[i][j], 0, 0, 0);
    if (kp == 0) mid();
    __builtin_amdgcn_sched_barrier(0);
  }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// BF16 MFMA over one LDS stage of fp32 operands ([k][m] / [k][n] images, as the f32 stage):
// v_mfma_f32_32x32x16_bf16, lane (r = l&31, h = l>>5) takes A[m = r][k = 8h + j] and
// B[k = 8h + j][n = r], j = 0..7: eight conflict-free ds_read_b32 per operand (32 consecutive
// floats per half-wave), rounded to bf16 (RNE, v_cvt_pk_bf16_f32) in registers; fp32
// accumulation.  `mid` runs after the first 16-deep group.
template <int BK, int TM, int TN, int LDA_S, int LDB_S, typename F>
__device__ __forceinline__ void mfma_stage_bf16(const float* As, const float* Bs,
                                                int wm, int wn, int lane, f32x16 (&acc)[TM][TN], F&& mid) {
  const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < BK / 16; ++kk) {
    bf16x8 av[TM], bv[TN];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kr = kk * 16 + 8 * h + j;
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i][j] = (__bf16)As[kr * LDA_S + wm + i * 32 + l32];
#pragma unroll
      for (int t = 0; t < TN; ++t) bv[t][j] = (__bf16)Bs[kr * LDB_S + wn + t * 32 + l32];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[t], acc[i][t], 0, 0, 0);
    if (kk == 0) mid();
  }
}

// FP32 GEMM on the BF16 matrix cores ("x6"): each fp32 operand is split into three bf16 terms
// v = hi + mid + lo + e (RNE at each step, exact fp32 remainders: |mid| <= 2^-8 |v|,
// |lo| <= 2^-16 |v|, |e| <= 2^-24 |v|), and the six products down to 2^-16 relative are
// accumulated in fp32, smallest first: lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi (a bf16 x
// bf16 product is exact in fp32).  The dropped terms (mid*lo, lo*mid, lo*lo) and the residuals
// sit at the 2^-24 level of fp32's own rounding, so the result is fp32-accurate (checked against
// fp64 by the r01 tuning harness).  Six 32x32x16 bf16 MFMAs (6 x 32 cycles) replace eight
// 32x32x2 f32 MFMAs (8 x 64 cycles) for one 16-deep K slice.
struct Split3 {
  bf16x8 hi, mid, lo;
};

// matrix-core form of a conv kernel (template argument MT)
// kMathX6P: the x6 form with the A operand (packed weights) split once per call by
// k_split_pack instead of per read (fwd form only)
constexpr int kMathF32 = 0, kMathBf16 = 1, kMathX6 = 2, kMathX6P = 3;

__device__ __forceinline__ void split3_set(Split3& s, int j, float v) {
  const __bf16 h = (__bf16)v;
  const float r = v - (float)h;
  const __bf16 m = (__bf16)r;
  s.hi[j] = h;
  s.mid[j] = m;
  s.lo[j] = (__bf16)(r - (float)m);
}

__device__ __forceinline__ f32x16 mfma_x6(const Split3& a, const Split3& b, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.lo, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.lo, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.mid, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.mid, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.hi, c, 0, 0, 0);
}

// FP32 GEMM on the FP16 matrix cores ("f16x3", kMathH3P, r02): each operand tensor is scaled by
// a power of two s (its absolute maximum brought to [2^14, 2^15): k_absmax partials, pow2_scale)
// and split into two fp16 terms, v*s = hi + lo + e (RNE; the remainder v*s - hi is exact in fp32,
// |lo| <= 2^-11 |v*s|, |e| <= 2^-22 |v*s|).  The three products lo*hi, hi*lo, hi*hi go through
// v_mfma_f32_32x32x16_f16 (an fp16 x fp16 product is exact in fp32, fp32 accumulation); the
// dropped lo*lo and the residuals are <= 2^-22 of each product, random in sign, so over a K-deep
// dot product they stay below fp32 accumulation's own rounding (the same argument as 3xTF32:
// TF32 also carries 11 significant bits).  The result is multiplied by 1/(sA sB), exactly.  The
// per-tensor scale keeps both terms inside fp16's exponent range (weights ~1e-2 and gradients
// ~1e-7 would otherwise lose the lo term to subnormals).  Half the MFMAs of x6 per 16-deep slice.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int kMathH3P = 5;
// kMathH1P: the fp16 conv math (BASELINE config 5's fp16 MFMA path): the f16x3 operands' hi terms
// only - each operand tensor scaled by its power of two and rounded to fp16 once, one
// v_mfma_f32_32x32x16_f16 per 16-deep slice, fp32 sums, the result unscaled exactly.
constexpr int kMathH1P = 8;
constexpr int kNPart = 256;  // absmax partials per operand tensor (k_absmax blocks)

struct Split2h {
  f16x8 hi, lo;
};

__device__ __forceinline__ void split2h_set(Split2h& s, int j, float v) {  // v already scaled
  const _Float16 h = (_Float16)v;
  s.hi[j] = h;
  s.lo[j] = (_Float16)(v - (float)h);
}

// The f16x3 split of a pair (x0, x1) under the power-of-two scale s, packed: hi = fp16(x s),
// lo = fp16(x s - hi), two halves per register - the same values as the plain C form (x s is exact, so
// the fused product of v_fma_mix is too), in 4 VALU per pair: the compiler's form also rebuilt hi
// through an fp32 multiply and a pack beside the v_fma_mix that feeds lo (r05).
__device__ __forceinline__ void split2_mix(float x0, float x1, float s, unsigned& hi, unsigned& lo) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(x0), "v"(x1), "v"(s));
}

// split2h_set of eight values v[j] * sc (sc a power of two) through split2_mix: 2 VALU per value instead
// of the compiler's 3 (fp32 products, a pack, the hi plane widened back for the remainder) - r05
__device__ __forceinline__ void split2h_scaled(Split2h& out, const float (&v)[8], float sc) {
  union { unsigned u[4]; f16x8 h; } hi, lo;
#pragma unroll
  for (int q = 0; q < 4; ++q) split2_mix(v[2 * q], v[2 * q + 1], sc, hi.u[q], lo.u[q]);
  out.hi = hi.h;
  out.lo = lo.h;
}

// the plain image-operand map of the BD stage (x -> x * s): split through split2h_scaled
struct ScaleXf {
  float s;
  __device__ __forceinline__ float operator()(int, float v) const { return v * s; }
};

__device__ __forceinline__ f32x16 mfma_h3(const Split2h& a, const Split2h& b, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.lo, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.hi, b.lo, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a.hi, b.hi, c, 0, 0, 0);
}

// 2^k with k = clamp(141 - biased exponent of mx, -100, 100): mx * 2^k in [2^14, 2^15) (fp16's
// largest finite value is 65504); a zero / fp32-subnormal maximum gives 2^100, inf / NaN 2^-100.
// `inv` = 2^-k.  Powers of two: scaling and unscaling are exact.
__device__ __forceinline__ float pow2_scale(float mx, float& inv) {
  const int e = (int)((__float_as_uint(mx) >> 23) & 0xffu);
  const int k = min(100, max(-100, 141 - e));
  inv = __uint_as_float((unsigned)(127 - k) << 23);
  return __uint_as_float((unsigned)(127 + k) << 23);
}

// max over the n absmax partials of one tensor (kNPart from k_absmax, or one per channel from
// the BN kernels that produced it), by every wave on its own (wave-uniform): float4 loads, four
// in flight per lane (2048 partials: two rounds)
__device__ __forceinline__ float partials_max(const float* __restrict__ part, int n, int lane) {
  float m = 0.f;
  if ((n & 3) == 0 && ((uintptr_t)part & 15) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(part);
    const int n4 = n >> 2;
    for (int i = lane; i < n4; i += 256) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i + 64 * u < n4 ? p4[i + 64 * u] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 4; ++u) m = fmaxf(m, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
    }
  } else {
    for (int i = lane; i < n; i += 64) m = fmaxf(m, part[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  return __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(m)));
}

// Block b of kNPart writes max |x| over its share of nbranch rows of n floats (row r at
// x + r * stride) to part[b]: coalesced float loads, a block reduce through LDS.
__device__ __forceinline__ void absmax_block(const float* __restrict__ x, long long n, long long stride,
                                             int nbranch, int b, float* __restrict__ out) {
  __shared__ float red[4];
  constexpr long long NT = (long long)kNPart * 256;  // threads of the grid
  float m = 0.f;
  for (int r = 0; r < nbranch; ++r) {
    const float* row = x + r * stride;
    // float4 body with eight loads in flight per thread (one load at a time was latency-bound:
    // ~10 us for an 8.6 MB tensor), then the scalar tail (or all of a misaligned row)
    const long long n4 = ((uintptr_t)row & 15) == 0 ? n / 4 : 0;
    const float4* r4 = reinterpret_cast<const float4*>(row);
    for (long long i = (long long)b * 256 + threadIdx.x; i < n4; i += 8 * NT) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = i + u * NT < n4 ? r4[i + u * NT] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    for (long long i = n4 * 4 + (long long)b * 256 + threadIdx.x; i < n; i += NT) m = fmaxf(m, fabsf(row[i]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) *out = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__global__ void __launch_bounds__(256) k_absmax(const float* __restrict__ x, long long n, long long stride,
                                                int nbranch, float* __restrict__ part) {
  absmax_block(x, n, stride, nbranch, blockIdx.x, part + blockIdx.x);
}

// Operand fragment of a bf16 matrix-core form and its MFMA step (32x32x16: 8 k per lane).
template <int MT> struct MathFrag { typedef bf16x8 type; };
template <> struct MathFrag<kMathX6> { typedef Split3 type; };

template <int MT>
__device__ __forceinline__ void frag_set(typename MathFrag<MT>::type& f, int j, float v) {
  if constexpr (MT == kMathX6) split3_set(f, j, v);
  else f[j] = (__bf16)v;
}

template <int MT>
__device__ __forceinline__ f32x16 frag_mma(const typename MathFrag<MT>::type& a,
                                           const typename MathFrag<MT>::type& b, f32x16 c) {
  if constexpr (MT == kMathX6) return mfma_x6(a, b, c);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// One LDS stage of fp32 operands through mfma_x6 (same operand reads as mfma_stage_bf16).
template <int BK, int TM, int TN, int LDA_S, int LDB_S, typename F>
__device__ __forceinline__ void mfma_stage_x6(const float* As, const float* Bs,
                                              int wm, int wn, int lane, f32x16 (&acc)[TM][TN], F&& mid) {
  const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < BK / 16; ++kk) {
    Split3 av[TM], bv[TN];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kr = kk * 16 + 8 * h + j;
#pragma unroll
      for (int i = 0; i < TM; ++i) split3_set(av[i], j, As[kr * LDA_S + wm + i * 32 + l32]);
#pragma unroll
      for (int t = 0; t < TN; ++t) split3_set(bv[t], j, Bs[kr * LDB_S + wn + t * 32 + l32]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t) acc[i][t] = mfma_x6(av[i], bv[t], acc[i][t]);
    if (kk == 0) mid();
  }
}

// The fwd-form A operand [ks*16 + k][lda] fp32 split into its three bf16 terms, laid out for
// the x6 stage's operand reads: planes[((ks*3 + q)*2 + h)*lda + m][j] = term q of
// A[ks*16 + 8h + j][m] - one 16-B ds_read_b128 per (plane, fragment), 16-B rows per m so a
// 16-lane group of reads covers 64 distinct banks, and every 64 rows of one (ks, q, h) are one
// contiguous 1 KB LDS-DMA piece.
__global__ void __launch_bounds__(256) k_split_pack(const float* __restrict__ A, int ksteps, int lda,
                                                    __bf16* __restrict__ planes) {
  // one thread per (ks, half h, m): reads A[ks*16 + 8h + j][m], j < 8 (coalesced over m), writes
  // the three 16-B plane rows of that (ks, h, m) (coalesced over m)
  const long long n = (long long)ksteps * 2 * lda;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int m = (int)(e % lda);
    const long long kh = e / lda;
    const int h = (int)(kh & 1), ks = (int)(kh >> 1);
    Split3 sp;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_set(sp, j, A[((long long)ks * kCB + 8 * h + j) * lda + m]);
    bf16x8* out = reinterpret_cast<bf16x8*>(planes);
    const long long row = ((long long)(ks * 3) * 2 + h) * lda + m;  // plane 0
    out[row] = sp.hi;
    out[row + 2LL * lda] = sp.mid;
    out[row + 4LL * lda] = sp.lo;
  }
}

// x6 stage with the A fragments read as pre-split bf16 planes (one LDS stage = G K-steps of
// [plane][half][BM][8] bf16, 24*BM floats each) and the B fragments split as they are read.
template <int G, int TM, int TN, int BM, int LDB_S, typename F>
__device__ __forceinline__ void mfma_stage_x6p(const float* As, const float* Bs,
                                               int wm, int wn, int lane, f32x16 (&acc)[TM][TN], F&& mid) {
  const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < G; ++kk) {
    const bf16x8* Ab = reinterpret_cast<const bf16x8*>(As + kk * 24 * BM);
    Split3 av[TM], bv[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = wm + i * 32 + l32;
      av[i].hi = Ab[(0 * 2 + h) * BM + m];
      av[i].mid = Ab[(1 * 2 + h) * BM + m];
      av[i].lo = Ab[(2 * 2 + h) * BM + m];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kr = kk * 16 + 8 * h + j;
#pragma unroll
      for (int t = 0; t < TN; ++t) split3_set(bv[t], j, Bs[kr * LDB_S + wn + t * 32 + l32]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t) acc[i][t] = mfma_x6(av[i], bv[t], acc[i][t]);
    if (kk == 0) mid();
  }
}

// r06: s_setprio(1) around a wave's MFMA cluster (cdna_hip_programming.md T5): of a SIMD's two waves (two
// workgroups) the one in its MFMA phase wins the issue arbitration over the one reading fragments / splitting,
// so its cluster issues back to back.  BD f16x3 stages (kMfmaPrio): layer3 forward 83.0 -> 76.6 us, step
// -0.14 ms; the weight gradient's clusters too (kMfmaPrioWg, neutral to -0.05 ms); the LDS-form and fp16 stages
// (kMfmaPrioLds) measured neutral on configs 2 and 5 and stay off (profiles/r06_mfma_prio_ab.txt).
constexpr bool kMfmaPrio = true;
constexpr bool kMfmaPrioLds = false;
constexpr bool kMfmaPrioWg = true;
template <bool ON, int P>
__device__ __forceinline__ void mfma_prio() {
  if constexpr (ON) __builtin_amdgcn_s_setprio(P);
}

// f16x3 stage: A fragments from the pre-split fp16 planes (one LDS stage = G K-steps of
// [plane][half][BM][8] fp16, 16*BM floats each), B fragments scaled by sB and split as they are read.
template <int G, int TM, int TN, int BM, int LDB_S, typename F>
__device__ __forceinline__ void mfma_stage_h3p(const float* As, const float* Bs,
                                               int wm, int wn, int lane, f32x16 (&acc)[TM][TN], F&& mid,
                                               float sB) {
  const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < G; ++kk) {
    const f16x8* Ab = reinterpret_cast<const f16x8*>(As + kk * 16 * BM);
    if constexpr (TM * TN >= 8) {
      // the 256-row pointwise tiles (r06: 128 accumulator registers per lane): B read and split first, then
      // row block by row block, so only one A fragment's two planes are live at a time (all of them at once
      // spilled 74 VGPRs)
      Split2h bv[TN];
      float braw[TN][8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int t = 0; t < TN; ++t) braw[t][j] = Bs[(kk * 16 + 8 * h + j) * LDB_S + wn + t * 32 + l32];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int t = 0; t < TN; ++t) split2h_set(bv[t], j, braw[t][j] * sB);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        Split2h av;
        av.lo = Ab[(2 + h) * BM + wm + i * 32 + l32];
        av.hi = Ab[h * BM + wm + i * 32 + l32];
        mfma_prio<kMfmaPrioLds, 1>();
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av.lo, bv[t].hi, acc[i][t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av.hi, bv[t].lo, acc[i][t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av.hi, bv[t].hi, acc[i][t], 0, 0, 0);
        mfma_prio<kMfmaPrioLds, 0>();
      }
      if (kk == 0) mid();
      continue;
    }
    Split2h av[TM], bv[TN];
    float braw[TN][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int t = 0; t < TN; ++t) braw[t][j] = Bs[(kk * 16 + 8 * h + j) * LDB_S + wn + t * 32 + l32];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i].lo = Ab[(2 + h) * BM + wm + i * 32 + l32];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i].hi = Ab[h * BM + wm + i * 32 + l32];
    // every LDS read of the K-step issues before the B split's VALU work
    __builtin_amdgcn_sched_barrier(0);
    // (the plain C split here: split2h_scaled made the big pointwise GEMMs 3-4 % slower, r05)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int t = 0; t < TN; ++t) split2h_set(bv[t], j, braw[t][j] * sB);
    // product-major order: the TM*TN accumulators of one product are independent, so its MFMAs
    // issue back to back, and every A fragment is in registers before the first one
    mfma_prio<kMfmaPrioLds, 1>();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].lo, bv[t].hi, acc[i][t], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bv[t].lo, acc[i][t], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bv[t].hi, acc[i][t], 0, 0, 0);
    mfma_prio<kMfmaPrioLds, 0>();
    if (kk == 0) mid();
  }
}

// fp16 stage: A fragments from the pack's hi plane (G K-steps of [half][BM][8] fp16, 8*BM floats
// each), B fragments scaled by sB and rounded to fp16 as they are read.
template <int G, int TM, int TN, int BM, int LDB_S, typename F>
__device__ __forceinline__ void mfma_stage_h1p(const float* As, const float* Bs,
                                               int wm, int wn, int lane, f32x16 (&acc)[TM][TN], F&& mid,
                                               float sB) {
  const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < G; ++kk) {
    const f16x8* Ab = reinterpret_cast<const f16x8*>(As + kk * 8 * BM);
    f16x8 av[TM], bv[TN];
    float braw[TN][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int t = 0; t < TN; ++t) braw[t][j] = Bs[(kk * 16 + 8 * h + j) * LDB_S + wn + t * 32 + l32];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i] = Ab[h * BM + wm + i * 32 + l32];
    __builtin_amdgcn_sched_barrier(0);  // every LDS read of the K-step issues before the VALU work
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int t = 0; t < TN; ++t) bv[t][j] = (_Float16)(braw[t][j] * sB);
    mfma_prio<kMfmaPrioLds, 1>();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i], bv[t], acc[i][t], 0, 0, 0);
    mfma_prio<kMfmaPrioLds, 0>();
    if (kk == 0) mid();
  }
}

// f16x3 / fp16 stage with the B operand in registers (fwd_sk_body's BD form, r03): braw = this lane's
// 8 image values B[k = 8h .. 8h+7][n = its pixel] of the K-step, loaded from global memory a few
// K-steps ahead; A fragments from the LDS ring as in mfma_stage_h3p.  One K-step, one 32-pixel column
// per wave (1 x 4 waves).  xf(j, v) maps a loaded value to the scaled operand (v * sB).
template <int TM, int BM, bool HI_ONLY, typename F, typename X>
__device__ __forceinline__ void mfma_stage_hd(const float* As, int wm, int lane, f32x16 (&acc)[TM][1],
                                              F&& mid, X&& xf, const float (&braw)[8]) {
  const int l32 = lane & 31, h = lane >> 5;
  const f16x8* Ab = reinterpret_cast<const f16x8*>(As);
  if constexpr (HI_ONLY) {
    f16x8 av[TM], bv;
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i] = Ab[h * BM + wm + i * 32 + l32];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) bv[j] = (_Float16)xf(j, braw[j]);
    mfma_prio<kMfmaPrioLds, 1>();
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i], bv, acc[i][0], 0, 0, 0);
    mfma_prio<kMfmaPrioLds, 0>();
  } else {
    Split2h av[TM], bv;
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i].lo = Ab[(2 + h) * BM + wm + i * 32 + l32];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i].hi = Ab[h * BM + wm + i * 32 + l32];
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (std::is_same_v<std::decay_t<X>, ScaleXf>) {
      split2h_scaled(bv, braw, xf.s);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) split2h_set(bv, j, xf(j, braw[j]));
    }
    mfma_prio<kMfmaPrio, 1>();
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].lo, bv.hi, acc[i][0], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bv.lo, acc[i][0], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bv.hi, acc[i][0], 0, 0, 0);
    mfma_prio<kMfmaPrio, 0>();
  }
  mid();
}

// The BD stage with the image operand pre-split (k_split_img): braw[8 j ..] holds the lane's hi plane
// (floats 0..3 as 16 B) and lo plane (4..7) of pixel column j, already scaled; no split work in the loop.
// TN = 1: the 1 x 4 wave layout (128 rows x 32 pixels per wave); TN = 2: the 2 x 2 layout (r06, 64 rows x
// 64 pixels per wave: half the A-fragment LDS reads per MFMA).
template <int TM, int TN, int BM, bool HI_ONLY, typename F>
__device__ __forceinline__ void mfma_stage_hdp(const float* As, int wm, int lane, f32x16 (&acc)[TM][TN],
                                               F&& mid, const float (&braw)[8 * TN]) {
  const int l32 = lane & 31, h = lane >> 5;
  const f16x8* Ab = reinterpret_cast<const f16x8*>(As);
  union { float f[4]; f16x8 h; } bh[TN], bl[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[t].f[j] = braw[8 * t + j];
      bl[t].f[j] = braw[8 * t + 4 + j];
    }
  if constexpr (HI_ONLY) {
    f16x8 av[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i] = Ab[h * BM + wm + i * 32 + l32];
    mfma_prio<kMfmaPrioLds, 1>();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i], bh[t].h, acc[i][t], 0, 0, 0);
    mfma_prio<kMfmaPrioLds, 0>();
  } else {
    Split2h av[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i].lo = Ab[(2 + h) * BM + wm + i * 32 + l32];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[i].hi = Ab[h * BM + wm + i * 32 + l32];
    mfma_prio<kMfmaPrio, 1>();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].lo, bh[t].h, acc[i][t], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bl[t].h, acc[i][t], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bh[t].h, acc[i][t], 0, 0, 0);
    mfma_prio<kMfmaPrio, 0>();
  }
  mid();
}

// Forward form: C[m][p] = sum_k A[k][m] * B[k][p], BK = G * 16 (G tap-groups per K-step).
template <int BM, int BN, int BK, int WM, int WN>
__global__ void __launch_bounds__(256) k_igemm_fwd(FwdArgs a) {
  constexpr int G = BK / kCB;
  static_assert(BK % kCB == 0, "BK multiple of 16");
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves");
  constexpr int LDA_S = BM, LDB_S = BN;  // row reads are contiguous: no padding needed
  constexpr int A_STAGE = BK * LDA_S, STAGE = A_STAGE + BK * LDB_S;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid / WN) * (TM * 32), wn = (wid % WN) * (TN * 32);
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int split = blockIdx.z;
  const int s_begin = split * a.kps;
  const int s_end = min(a.ksteps, s_begin + a.kps);

  constexpr int BROWS = 256 / BN;        // B rows per pass
  constexpr int BPASS = kCB / BROWS;     // passes per tap-group
  const int bn = tid % BN, brow0 = tid / BN;
  const int p = n0 + bn;
  const int pq = p / a.W, px = p - pq * a.W, py = pq % a.H;  // row within its image
  const bool pin = p < a.P;

  constexpr int A_F4_ROW = BM / 4;
  constexpr int A_F4 = BK * A_F4_ROW;
  constexpr int APASS = (A_F4 + 255) / 256;

  float4 ra[APASS];
  float rb[G][BPASS];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int per_b = a.ncb * a.taps;
  auto gload = [&](int s) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int q = s * G + g;  // tap-group index
      const int b = q / per_b;
      const int rem = q - b * per_b;
      const int t = rem / a.ncb;
      const int cb = rem - t * a.ncb;
      const int d = b ? a.dil1 : a.dil0;
      const int dh = (t / 3 - 1) * d, dw = (t % 3 - 1) * d;
      const bool v = pin && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
      const int ci0 = cb * kCB + brow0;
      const float* src = a.B + (long long)ci0 * a.P + (p + dh * a.W + dw);
#pragma unroll
      for (int j = 0; j < BPASS; ++j) {
        const int ci = ci0 + j * BROWS;
        rb[g][j] = (v && ci < a.cimg) ? src[(long long)(j * BROWS) * a.P] : 0.f;
      }
    }
    const float* ab = a.A + (long long)s * BK * a.lda + m0;
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      const int idx = tid + i * 256;
      if (A_F4 % 256 == 0 || idx < A_F4) {
        const int r = idx / A_F4_ROW, c4 = idx - r * A_F4_ROW;
        ra[i] = *reinterpret_cast<const float4*>(ab + (long long)r * a.lda + c4 * 4);
      }
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * STAGE;
    float* Bs = As + A_STAGE;
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      const int idx = tid + i * 256;
      if (A_F4 % 256 == 0 || idx < A_F4) {
        const int r = idx / A_F4_ROW, c4 = idx - r * A_F4_ROW;
        *reinterpret_cast<float4*>(As + r * LDA_S + c4 * 4) = ra[i];
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < BPASS; ++j) Bs[(g * kCB + brow0 + j * BROWS) * LDB_S + bn] = rb[g][j];
  };

  if (s_begin < s_end) {
    gload(s_begin);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int s = s_begin; s < s_end; ++s) {
      const bool more = s + 1 < s_end;
      if (more) gload(s + 1);
      const float* As = smem + cur * STAGE;
      mfma_stage<BK, TM, TN, LDA_S, LDB_S>(As, As + A_STAGE, wm, wn, lane, acc);
      if (more) sstore(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  float* C = a.C + (long long)split * a.slab;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn + j * 32 + (lane & 31);
        if (m < a.M && n < a.P) {
          float v = acc[i][j][r];
          if (a.bias) {
            float bsum = a.bias[m];
            for (int b = 1; b < a.nbias; ++b) bsum += a.bias[b * a.M + m];
            v += bsum;
          }
          C[(long long)m * a.P + n] = v;
        }
      }
}

// Weight gradient: dW[m][n][tap] = sum_p dY[m][p] * X[n][p + shift(tap)], BK pixels per K-step.
template <int BM, int BN, int BK, int WM, int WN>
__global__ void __launch_bounds__(256) k_igemm_wgrad(WgradArgs a) {
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves");
  static_assert(BK == 32 || BK == 64, "BK");
  constexpr int LDA_S = BM + 1, LDB_S = BN + 1;  // odd strides: transposing writes are conflict-free
  constexpr int A_STAGE = BK * LDA_S, STAGE = A_STAGE + BK * LDB_S;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid / WN) * (TM * 32), wn = (wid % WN) * (TN * 32);
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int tapz = blockIdx.z % a.ntap;
  const int split = blockIdx.z / a.ntap;
  const int br = tapz / a.taps, t = tapz - br * a.taps;
  const int d = br ? a.dil1 : a.dil0;
  const int dh = (t / 3 - 1) * d, dw = (t % 3 - 1) * d;
  const int s_begin = split * a.kps;
  const int s_end = min(a.ksteps, s_begin + a.kps);

  constexpr int RSTEP = 256 / BK;  // rows covered per pass
  const int kl = tid % BK, r0 = tid / BK;
  constexpr int APASS = BM / RSTEP, BPASS = BN / RSTEP;
  float ra[APASS], rb[BPASS];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto gload = [&](int s) {
    const int p = s * BK + kl;
    const bool pv = p < a.P;
    const int pq = p / a.W, px = p - pq * a.W, py = pq % a.H;
    const bool vb = pv && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
    const int off = p + dh * a.W + dw;
#pragma unroll
    for (int j = 0; j < APASS; ++j) {
      const int m = m0 + r0 + RSTEP * j;
      ra[j] = (pv && m < a.M) ? a.dy[(long long)m * a.P + p] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < BPASS; ++j) {
      const int n = n0 + r0 + RSTEP * j;
      rb[j] = (vb && n < a.N) ? a.x[(long long)n * a.P + off] : 0.f;
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * STAGE;
    float* Bs = As + A_STAGE;
#pragma unroll
    for (int j = 0; j < APASS; ++j) As[kl * LDA_S + r0 + RSTEP * j] = ra[j];
#pragma unroll
    for (int j = 0; j < BPASS; ++j) Bs[kl * LDB_S + r0 + RSTEP * j] = rb[j];
  };

  if (s_begin < s_end) {
    gload(s_begin);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int s = s_begin; s < s_end; ++s) {
      const bool more = s + 1 < s_end;
      if (more) gload(s + 1);
      const float* As = smem + cur * STAGE;
      mfma_stage<BK, TM, TN, LDA_S, LDB_S>(As, As + A_STAGE, wm, wn, lane, acc);
      if (more) sstore(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  float* C = a.C + (long long)split * a.slab + (long long)br * a.cbranch;
  const long long ldc = (long long)a.N * a.taps;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn + j * 32 + (lane & 31);
        if (m < a.M && n < a.N) {
          const long long idx = (long long)m * ldc + (long long)n * a.taps + t;
          C[idx] = a.accumulate ? C[idx] + acc[i][j][r] : acc[i][j][r];
        }
      }
}


// ---------------------------------------------------------------------------------------------
// Forward form with an LDS-DMA ring (buffer_load ... lds): no register staging, STAGES-1 K-steps
// in flight across raw barriers with counted vmcnt waits.  The dilated halo is zero-filled by
// the buffer unit itself: a lane whose shifted pixel falls outside the image (or whose channel
// is padding) gets an out-of-range offset, which loads 0.
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma_b32(__amdgpu_buffer_rsrc_t r, float* lds_row, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_row, 4, voff, 0, 0, 0);
}
__device__ __forceinline__ void dma_b128(__amdgpu_buffer_rsrc_t r, float* lds_row, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_row, 16, voff, 0, 0, 0);
}

// The LDS base for the reads after a raw s_barrier: routed through an empty asm so the reads depend on
// it and stay below the barrier (r04: the compiler does not see the LDS-DMA builtins as stores to the
// array, treats its reads as movable, and may hoist a K-step's fragment reads above the barrier and the
// counted waits - a race with the other waves' DMA pieces of that stage).
typedef __attribute__((address_space(3))) float lds_f32;
__device__ __forceinline__ const float* lds_after_barrier(float* smem) {
  lds_f32* q = (lds_f32*)smem;
  asm volatile("" : "+v"(q));
  return (const float*)q;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// The forward-form image operand pre-split (variant bit 7, r03): planes[((cb*NP + q)*2 + h)*P + p] =
// 16 B = plane q of the 8 channels cb*16 + 8h .. +7 of pixel p, scaled by the tensor's power of two
// (0 past cimg).  NP = 2 (f16x3: hi, lo) or 1 (fp16: hi).  One thread per (cb, h, p): eight loads
// coalesced over p, one or two 16-B stores.
template <int NP>
__global__ void __launch_bounds__(256) k_split_img(const float* __restrict__ x, int cimg, int ncb, int P,
                                                   const float* __restrict__ part, int npart,
                                                   f16x8* __restrict__ planes) {
  float inv;
  const float sc = pow2_scale(partials_max(part, npart, threadIdx.x & 63), inv);
  const long long n = (long long)ncb * 2 * P;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int p = (int)(e % P);
    const int r = (int)(e / P);
    const int h = r & 1, cb = r >> 1;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cb * kCB + 8 * h + j;
      v[j] = c < cimg ? x[(long long)c * P + p] * sc : 0.f;
    }
    Split2h sp;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (NP == 1) sp.hi[j] = (_Float16)v[j];
      else split2h_set(sp, j, v[j]);
    }
    planes[((long long)(cb * NP) * 2 + h) * P + p] = sp.hi;
    if constexpr (NP == 2) planes[((long long)(cb * NP + 1) * 2 + h) * P + p] = sp.lo;
  }
}

// ---------------------------------------------------------------------------------------------
// Stream-K forward form.  The (tile, stage) iteration space of all output tiles is cut into NW
// equal ranges, one per persistent workgroup (NW = CUs x resident workgroups per CU), so every
// CU gets the same MFMA work whatever the tile count (65x129 maps give 132 or 264 tiles, which
// split-K can only spread over 256 CUs unevenly).  A tile cut by range boundaries leaves one
// piece per workgroup that touched it; k_sk_reduce (the next launch on the stream) sums them in
// worker order.  Nothing ever waits on another workgroup, so the kernel needs no co-residency
// and no dispatch-order assumption, and the sum order - hence the result - is fixed.
// Hybrid form (r02): when there are at least as many tiles as workers, the first tdp = R x grid
// tiles run data-parallel (worker w owns whole tiles w, w + grid, ...: no pieces, direct stores)
// and only the remaining tiles' iterations are cut into stream-K ranges over NW workers.  A
// 256->1024 pointwise forward (528 tiles) left ~1040 pieces (67 MB written and re-read) as pure
// stream-K and leaves 272 this way.  tdp = 0 is pure stream-K.
struct SkArgs {
  float* part;     // [NW][2][BM][BN] pieces of split tiles (row-major)
  int tiles_m, tiles_n, KS, NW;
  int T;           // stream-K iterations: (tiles - tdp) * KS  (T * NW < 2^31, checked by the planner)
  int tdp;         // leading tiles that run data-parallel (a multiple of the grid size)
  int gm;          // m-blocks per tile group (sk_tile): 1 = n fastest
  unsigned long long* prof;  // diagnostic builds only (fwd_sk_body PROF): per-wave cycle sums per loop phase
};

__device__ __forceinline__ int sk_start(int w, int T, int NW) { return (int)((unsigned)(w * T) / (unsigned)NW); }
// Tile t of the forward-form stream-K space -> (m-block, n-block).  gm <= 1: n fastest - consecutive
// tiles share an m-block, so the 64 workers of one XCD (consecutive ranges) read one or two m-blocks'
// weights and a contiguous pixel range (r02 layer3 fwd: 66 vs 154 MB fetched per launch with m
// fastest; profiles/r02_sk_tile_order.txt).  gm > 1: groups of gm m-blocks, m fastest inside a
// group - the gm tiles of one pixel block run on neighbouring workers, so the image block is
// fetched once (r04: the pointwise and layer4 GEMMs, dconv.hip launch_fwd_form).
__device__ __forceinline__ void sk_tile(int t, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  if (gm <= 1) {
    tm = t / tiles_n;
    tn = t - tm * tiles_n;
    return;
  }
  const int g = t / (gm * tiles_n), r = t - g * gm * tiles_n;
  const int m_in = min(gm, tiles_m - g * gm);  // m-blocks in this (possibly last, short) group
  tn = r / m_in;
  tm = g * gm + (r - tn * m_in);
}
__device__ __forceinline__ int sk_worker_of(int i, int T, int NW) {
  return (int)((unsigned)((i + 1) * NW - 1) / (unsigned)T);
}

// BD (r03, f16x3 / fp16, 1 x 4 waves, G = 1, STAGES = 4): the image operand skips LDS - each lane
// loads its own 8 values per K-step (B[8h .. 8h+7][its pixel], the shifted pixel zero-filled through an
// out-of-range offset) with plain buffer loads three K-steps ahead into a register ring, so the only
// LDS-DMA left per K-step is the two A-plane pieces (the 8 dword DMA pieces of B cost ~60 issue cycles
// each, more than the K-step's 12 MFMAs).  Every wave of the 1 x 4 layout reads its own 32 columns,
// so nothing is lost by not sharing B through LDS.
// PROF (diagnostic builds only, scripts/probe_sk.hip; 0 in the library), bit 0: s_memtime stamps around
// the BD loop's phases, summed per wave into sk.prof[wave][phase]: 0 the wait for the stage's A pieces,
// 1 the barrier, 2 fragment reads + split + MFMA issue + the next stage's issue, 3 the closing
// lgkmcnt(0), 4 the epilogue, 5 K-steps.  The stamps' own waits forbid overlaps the real kernel has: read
// the shares, not the length (cdna_hip_programming.md §7, In-kernel stamps).  Timing-only ablations
// (wrong results): bit 1 no image-operand loads (opaque zeros), bit 2 no A-plane LDS-DMA, bit 3 no
// K-step barrier.
__device__ __forceinline__ unsigned long long sk_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int BM, int BN, int G, int STAGES, int WM, int WN, bool PW = false, int MT = 0, bool ACC = false,
          bool BD = false, bool BP = false, int PROF = 0>
__device__ __forceinline__ void fwd_sk_body(FwdArgs a, SkArgs sk) {
  // one stream-K iteration = one LDS stage = G consecutive K-steps (16 channels of one tap each);
  // sk.KS counts stages per tile (a.ksteps / G).  PW: pointwise (one unshifted tap), so a B row
  // is 128 contiguous pixels and moves as dwordx4 (4 pixels per lane) instead of dwords.
  constexpr int BK = G * kCB;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves");
  static_assert(BN % 64 == 0 && BM % 32 == 0, "tiles");
  // r05: 256- and 384-row tiles of the LDS form computed wrong results from the first row on
  // (profiles/r05_aspp_384_tile_attempt.txt): the launch kept the workspace of 128-row pieces, and the larger
  // pieces ran past it (r06: dconv.hip fwd_piece_bytes).  Only the form validated since may be instantiated
  static_assert(BM <= 128 || (BM == 256 && PW && WM == 1 && WN == 4 && STAGES == 3),
                "fwd_sk_body: tiles over 128 rows are validated only as the 256-row pointwise form (r06)");
  constexpr bool H1 = MT == kMathH1P;                                 // fp16: the hi plane only
  constexpr bool H3 = MT == kMathH3P || H1;                           // f16x3: two fp16 planes
  constexpr bool APRE = MT == kMathX6P || H3;  // A from pre-split planes
  constexpr int NQ = H3 ? 4 : 6;  // (plane, k half) blocks of one pre-split K-step in the pack
  constexpr int NQL = H1 ? 2 : NQ;  // of them staged (fp16 math: plane 0's two halves)
  static_assert(!APRE || BM % 64 == 0, "pre-split A: 64-row DMA pieces");
  // BD: 1 x 4 waves (128 rows x 32 pixels each); the pre-split image (BP) also in 2 x 2 waves (64 x 64, r06)
  static_assert(!BD || (H3 && G == 1 && STAGES == 4 &&
                        ((WM == 1 && WN == 4 && TN == 1) || (BP && WM == 2 && WN == 2 && TM == 2 && TN == 2))),
                "BD form");
  constexpr int A_STAGE = APRE ? G * 4 * NQL * BM : BK * BM;
  constexpr int STAGE = A_STAGE + (BD ? 0 : BK * BN);
  constexpr int A_ROWS_PER_INST = 256 / BM;
  constexpr int A_INST = APRE ? G * NQL * (BM / 64) : BK / A_ROWS_PER_INST;
  // fp16 math on 64-row tiles (r04): a K-step's A is one plane's two 1-KB pieces; each wave issues
  // half a piece (its lane half of the 64 rows), so every wave still issues one A instruction
  constexpr bool AHALF = APRE && A_INST == 2;
  constexpr int A_INST_W = AHALF ? 1 : A_INST / 4;
  constexpr int NH = BN / 64;
  constexpr int BG_INST_W = PW ? kCB * BN / 256 / 4 : kCB * NH / 4;  // B DMAs per wave per K-step
  static_assert(!PW || BN == 128, "pointwise B rows: two rows of 128 pixels per dwordx4 instruction");
  static_assert(!BP || BD, "BP: the BD form with a pre-split image");
  constexpr int INST_W = A_INST_W + G * (BP ? (H1 ? 1 : 2) * TN : BD ? 8 : BG_INST_W);
  static_assert(AHALF || A_INST % 4 == 0, "A instructions split evenly over waves");
  static_assert(!AHALF || (G == 1 && BM == 64), "half-wave A pieces: one K-step of 64 rows per stage");
  static_assert((STAGES - 2) * INST_W < 64, "vmcnt range");
  // ONE __shared__ object: a second one (even a 4-byte flag) makes hipcc emit vmcnt(0) before the
  // first ds_read after every DMA issue, which drains the in-flight stage (cdna_hip_programming.md
  // §5, M = 256 item 4(a)).
  __shared__ __attribute__((aligned(16))) float smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wid / WN) * (TM * 32), wn = (wid % WN) * (TN * 32);
  // XCD-aware worker id: workgroups b, b+8, ... share an XCD and get consecutive ranges
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);  // a bijection for any nb
  // whole data-parallel tiles w, w + nb, ... below sk.tdp first, then this worker's stream-K
  // range of the remaining tiles' iterations (none for w >= sk.NW)
  int dp_t = w, it = 0, it_end = 0;
  // the stream-K worker index: w (XCD-aware: neighbouring ranges share an L2); for the remainder
  // after data-parallel rounds with fewer stream-K workers than workgroups, the block id, so those
  // workers spread over all XCDs instead of filling the first one
  const int sw = (sk.tdp > 0 && sk.NW < nb) ? b : w;
  if (sw < sk.NW) {
    it = sk.tdp * sk.KS + sk_start(sw, sk.T, sk.NW);
    it_end = sk.tdp * sk.KS + sk_start(sw + 1, sk.T, sk.NW);
  }

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.A, (short)0, (int)min(0x7fffffffLL, (long long)sk.KS * BK * a.lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.B, (short)0, (int)min(0x7fffffffLL, (long long)a.cimg * a.P * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Ax6, (short)0, (int)min(0x7fffffffLL, (long long)a.ksteps * NQ * a.lda * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rbx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Bx6, (short)0,
      (int)min(0x7fffffffLL, (long long)a.ncb * (H1 ? 2 : 4) * a.P * 16), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned chan_bytes = (unsigned)a.P * 4u;
  // f16x3: B's scale from its absmax partials, A's from the pack; the result is unscaled by both
  float sB = 1.f, iA = 1.f, iB = 1.f;
  if constexpr (H3) {
    sB = pow2_scale(partials_max(a.bpart, a.bnpart, lane), iB);
    iA = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(a.ascale[1])));
  }

  // PROF & 16 (timing only): a BN-apply + ReLU of the image operand in the BD split, per-channel
  // (alpha, beta) from an LDS table (alpha = sB, beta = 0: the identity on a non-negative image)
  const float* tabp = nullptr;
  if constexpr ((PROF & 16) != 0) {
    __shared__ float bn_tab[2 * 2048];
    for (int c = threadIdx.x; c < a.cimg; c += blockDim.x) {
      const int cb = c >> 4, hh = (c >> 3) & 1, j = c & 7;
      bn_tab[((cb * 2 + hh) * 2 + 0) * 8 + j] = sB;
      bn_tab[((cb * 2 + hh) * 2 + 1) * 8 + j] = 0.f;
    }
    __syncthreads();
    tabp = bn_tab;
  }
  f32x16 acc[TM][TN];
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};  // PROF: phase cycle sums (wave-uniform)
  unsigned long long te = 0;
  while (true) {
    if constexpr (PROF & 1) {
      if (te) ph[4] += sk_stamp() - te;  // the previous segment's epilogue (piece or output stores)
      te = 0;
    }
    int t, k_a, k_b;
    if (dp_t < sk.tdp) {
      t = dp_t;
      k_a = 0;
      k_b = sk.KS;
      dp_t += nb;
    } else if (it < it_end) {
      t = (unsigned)it / (unsigned)sk.KS;
      k_a = it - t * sk.KS;
      k_b = min(sk.KS, k_a + (it_end - it));
      it += k_b - k_a;
    } else {
      break;
    }
    const int nst = k_b - k_a;
    int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, sk.gm, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    // per-lane constants of this tile: A byte offsets (stage 0), pixel coordinates
    unsigned a_off[A_INST_W];
#pragma unroll
    for (int i = 0; i < A_INST_W; ++i) {
      const int inst = wid * A_INST_W + i;
      const int row = inst * A_ROWS_PER_INST + lane / (BM / 4);
      a_off[i] = (unsigned)((row * a.lda + m0 + (lane % (BM / 4)) * 4) * 4);
    }
    const unsigned a_stage_bytes = (unsigned)(BK * a.lda * 4);
    int py[NH], px[NH];
    bool pin[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int p = n0 + h * 64 + lane;
      pin[h] = p < a.P;
      const int pq = p / a.W;
      px[h] = p - pq * a.W;
      py[h] = pq % a.H;
    }
    // Issue cursor over the K-steps, in order (K is tap-major: ks = (branch*taps + tap)*ncb + cb):
    // the wave-uniform (tap, channel block) advances incrementally and the per-lane shifted pixel
    // offsets (OOB outside the image) are recomputed only when the tap changes.
    int c_cb, c_tap = -1;
    unsigned vrow[NH];
    unsigned vbd[TN];     // BD: this lane's shifted pixel byte offset per column (OOB outside the image)
    unsigned vbdh = OOB;  // BD (TN = 1), full channel blocks: + the lane's channel half (8 * (lane >> 5) rows)
    int pbd[TN], pxd[TN], pyd[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      vbd[j] = OOB;
      pbd[j] = n0 + wn + j * 32 + (lane & 31);
      const int pqd = pbd[j] / a.W;
      pxd[j] = pbd[j] - pqd * a.W;
      pyd[j] = pqd % a.H;
    }
    {
      // wave-uniform: the cursor lives in scalar registers (it feeds the scalar channel offsets)
      const int ks0 = __builtin_amdgcn_readfirstlane(k_a * G);
      const int tq = ks0 / a.ncb;  // branch*taps + tap
      c_cb = ks0 - tq * a.ncb;
      c_tap = tq;
    }
    auto set_tap = [&](int tq) {
      const int br = tq / a.taps;
      const int tp = tq - br * a.taps;
      const int d = br ? a.dil1 : a.dil0;
      const int dh = (tp / 3 - 1) * d, dw = (tp % 3 - 1) * d;
      const int shift = dh * a.W + dw;
      if constexpr (BD) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const bool v = pbd[j] < a.P && (unsigned)(pyd[j] + dh) < (unsigned)a.H &&
                         (unsigned)(pxd[j] + dw) < (unsigned)a.W;
          vbd[j] = v ? (unsigned)((pbd[j] + shift) * (BP ? 16 : 4)) : OOB;
        }
        vbdh = vbd[0] != OOB ? vbd[0] + (unsigned)(8 * (lane >> 5)) * chan_bytes : OOB;
      } else {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          const bool v = pin[h] && (unsigned)(py[h] + dh) < (unsigned)a.H && (unsigned)(px[h] + dw) < (unsigned)a.W;
          vrow[h] = v ? (unsigned)((n0 + h * 64 + lane + shift) * 4) : OOB;
        }
      }
    };
    set_tap(c_tap);
    float bdq[4][8 * TN];  // BD: the register ring of B values (K-step i in slot i % 4; 8 per column)
    float bdv[4];          // PROF & 16: the ring's pixel validity (+inf / 0) and channel blocks
    int bdc[4];
    // part 1: stage s's A pieces into LDS slot `slot`; part 2: its B operand (ring entry bq, or LDS),
    // advancing the cursor; 3: both
    auto issue = [&](int s, int slot, float (&bq)[8 * TN], float& bv, int& bc, int part = 3) {
      float* As = smem + slot * STAGE;
      float* Bs = As + A_STAGE;
      if (!(part & 1)) {
      } else if constexpr (AHALF) {
        // piece wid / 2 (= the k half of plane 0), rows 32 * (wid & 1) .. +31: the lanes of that half
        const int qh = wid >> 1;
        if ((lane >> 5) == (wid & 1))
          dma_b128(rx, As + qh * 256, (unsigned)(((s * NQ + qh) * a.lda + m0 + lane) * 16));
      } else if constexpr (APRE) {
        // piece inst = (g, plane*2 + half, 64-row block): planes row ((ks*NP+q)*2+h)*lda + m
#pragma unroll
        for (int i = 0; i < A_INST_W; ++i) {
          const int inst = wid * A_INST_W + i;
          const int g = inst / (NQL * (BM / 64)), r = inst % (NQL * (BM / 64));
          const int qh = r / (BM / 64), mb = (r % (BM / 64)) * 64;
          const int ks = s * G + g;
          if constexpr (!(PROF & 4))
            dma_b128(rx, As + inst * 256, (unsigned)(((ks * NQ + qh) * a.lda + m0 + mb + lane) * 16));
        }
      } else {
        const unsigned a_base = (unsigned)s * a_stage_bytes;
#pragma unroll
        for (int i = 0; i < A_INST_W; ++i) {
          const int inst = wid * A_INST_W + i;
          dma_b128(ra, As + inst * 256, a_off[i] + a_base);
        }
      }
#pragma unroll
      for (int g = 0; g < G && (part & 2); ++g) {
        const int cb16 = c_cb * kCB;
        if constexpr (BP) {
          // the pre-split planes: 16 B per plane of this lane's pixel (hi, then lo)
          constexpr int NPB = H1 ? 1 : 2;
          const unsigned pl_bytes = (unsigned)a.P * 16u;
#pragma unroll
          for (int q = 0; q < NPB; ++q) {
            const unsigned row = (unsigned)((c_cb * NPB + q) * 2 + (lane >> 5)) * pl_bytes;
#pragma unroll
            for (int t = 0; t < TN; ++t) {
              union { u32x4 u; float f[4]; } c;
              c.u = __builtin_amdgcn_raw_buffer_load_b128(rbx, vbd[t] + row, 0, 0);
#pragma unroll
              for (int j = 0; j < 4; ++j) bq[8 * t + 4 * q + j] = c.f[j];
            }
          }
        } else if constexpr (BD) {
          // channels cb16 + 8h + j of this lane's pixel.  The BD form runs only with every 16-channel
          // block full (cimg % 16 == 0, launch_sk): the channel offset is wave-uniform, so it rides in
          // the scalar soffset and the eight loads share one address VGPR (r04: a per-channel bound
          // check cost ~32 VALU per K-step, and a second load path made the compiler's wait counts
          // drain the queue); an out-of-image pixel's voffset >= 2^31 is out of range whatever the
          // soffset
          const unsigned sb = (unsigned)__builtin_amdgcn_readfirstlane(cb16) * chan_bytes;
          if constexpr ((PROF & 16) != 0) {
            bv = vbdh != OOB ? __builtin_inff() : 0.f;
            bc = __builtin_amdgcn_readfirstlane(c_cb);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if constexpr (PROF & 2)
              asm volatile("v_mov_b32 %0, 0" : "=v"(bq[j]));
            else
              bq[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vbdh, (int)(sb + j * chan_bytes), 0));
          }
        } else if constexpr (PW) {
          // lanes 0-31 -> row 2*inst, lanes 32-63 -> row 2*inst+1; 4 pixels per lane.  A chunk
          // that straddles P reads the next channel's first pixels: they only reach output
          // columns >= P, which are never stored.
          const int c4 = (lane & 31) * 4;
#pragma unroll
          for (int j = 0; j < BG_INST_W; ++j) {
            const int inst = wid * BG_INST_W + j;
            const int ci = cb16 + inst * 2 + (lane >> 5);
            const bool v = ci < a.cimg && n0 + c4 < a.P;
            const unsigned e = (unsigned)(ci * a.P + n0 + c4);
            dma_b128(rb, Bs + (g * kCB + inst * 2) * BN, v ? e * 4u : OOB);
          }
        } else {
#pragma unroll
          for (int j = 0; j < BG_INST_W; ++j) {
            const int inst = wid * BG_INST_W + j;
            const int r = inst / NH, h = inst % NH;  // wave-uniform
            const int ci = cb16 + r;
            const unsigned cofs = ci < a.cimg ? (unsigned)ci * chan_bytes : OOB;  // scalar
            dma_b32(rb, Bs + (g * kCB + r) * BN + h * 64, vrow[h] + cofs);
          }
        }
        if (++c_cb == a.ncb) {
          c_cb = 0;
          if (++c_tap * a.ncb < a.ksteps) set_tap(c_tap);  // (past the last K-step: nothing to set)
        }
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __builtin_amdgcn_s_barrier();  // the previous segment's LDS reads are complete in every wave
    if constexpr (BD) {
      // Every K-step issues a stage, also past the segment's end (K-steps >= nst: loads that land in a
      // ring slot and an LDS slot no later K-step reads, zero-filled out of range), so exactly two
      // stages are always younger than the one computed: one wait count, and the register ring's
      // loads are followed by the same number of loads on every path.  (With the issues conditional,
      // the compiler's wait-count analysis saw paths with no younger loads and drained the queue -
      // vmcnt(0) - before the split of every first and fourth K-step; r04.  Those drains had also
      // hidden the LDS-DMA ordering race described at the wait below.)
      issue(k_a, 0, bdq[0], bdv[0], bdc[0]);
      issue(k_a + 1, 1, bdq[1], bdv[1], bdc[1]);
      issue(k_a + 2, 2, bdq[2], bdv[2], bdc[2]);
      // K-step i: wait until stage i + 1 landed (only stage i + 2 younger), barrier (stage i + 1 is
      // complete in every wave's LDS pieces, and every wave has read slot i - 1's fragments, at step
      // i - 2), issue stage i + 3 into that slot and ring entry, read + split K-step i + 1's fragments,
      // and issue K-step i's MFMAs from the fragments read the step before
      // K-step i: wait until its A pieces landed, issue K-step i + 3's B loads into the ring entry
      // K-step i - 1 freed, barrier (the A slot refilled next was read by every wave at i - 1), compute
      // with K-step i + 3's A pieces issued into that slot after the MFMAs (r05: B ahead of the barrier,
      // -17 us on the ASPP classifier's forward, profiles/r05_bd_bsplit_ab.txt).
      // The count leaves only the two younger stages' LDS-DMA pieces in flight, not their B loads:
      // an LDS-DMA may land after register loads issued behind it (r04: with the B loads counted too -
      // vmcnt(2 * INST_W) - a wave now and then read a stage's A slot before another wave's DMA piece
      // had landed; scripts/dbg_det.py, profiles/r04_bd_wait_race.txt).  The B registers are waited
      // for by the compiler at their use.
      auto step = [&](int i, float (&cur)[8 * TN], float (&nxt)[8 * TN], float& curv, float& nxtv, int& curc,
                      int& nxtc) {
        unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
        if constexpr (PROF & 1) t0 = sk_stamp();
        wait_vmcnt<2 * A_INST_W>();
        if constexpr (PROF & 1) t1 = sk_stamp();
        // K-step i + 3's B loads right after the wait (their ring entry was read by this wave at i - 1;
        // no other wave is involved), before the barrier: the wait at i + 1 forces all but its four
        // youngest loads, so what it forces was issued a whole K-step earlier rather than after this
        // step's MFMAs.  The A pieces still go after the barrier (their LDS slot is shared).
        issue(k_a + i + STAGES - 1, 0, nxt, nxtv, nxtc, 2);
        if constexpr (!(PROF & 8)) __builtin_amdgcn_s_barrier();
        if constexpr (PROF & 1) t2 = sk_stamp();
        const float* As = lds_after_barrier(smem) + (i % STAGES) * STAGE;
        auto mid = [&] { issue(k_a + i + STAGES - 1, (i + STAGES - 1) % STAGES, nxt, nxtv, nxtc, 1); };
        if constexpr (BP) {
          mfma_stage_hdp<TM, TN, BM, H1>(As, wm, lane, acc, mid, cur);
        } else if constexpr ((PROF & 16) != 0) {
          const float4* tq = reinterpret_cast<const float4*>(tabp + (curc * 2 + (lane >> 5)) * 16);
          const float4 a0 = tq[0], a1 = tq[1], b0 = tq[2], b1 = tq[3];
          const float al[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
          const float be[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
          const float vm = curv;
          mfma_stage_hd<TM, BM, H1>(
              As, wm, lane, acc, mid,
              [&](int j, float v) { return __builtin_amdgcn_fmed3f(fmaf(v, al[j], be[j]), 0.f, vm); }, cur);
        } else {
          mfma_stage_hd<TM, BM, H1>(As, wm, lane, acc, mid, ScaleXf{sB}, cur);
        }
        if constexpr (PROF & 1) t3 = sk_stamp();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (PROF & 1) {
          const unsigned long long t4 = sk_stamp();
          ph[0] += t1 - t0;
          ph[1] += t2 - t1;
          ph[2] += t3 - t2;
          ph[3] += t4 - t3;
          ph[5] += 1;
        }
      };
      int i = 0;
      for (; i + 4 <= nst; i += 4) {
        step(i, bdq[0], bdq[3], bdv[0], bdv[3], bdc[0], bdc[3]);
        step(i + 1, bdq[1], bdq[0], bdv[1], bdv[0], bdc[1], bdc[0]);
        step(i + 2, bdq[2], bdq[1], bdv[2], bdv[1], bdc[2], bdc[1]);
        step(i + 3, bdq[3], bdq[2], bdv[3], bdv[2], bdc[3], bdc[2]);
      }
      if (i < nst) step(i, bdq[0], bdq[3], bdv[0], bdv[3], bdc[0], bdc[3]);
      if (i + 1 < nst) step(i + 1, bdq[1], bdq[0], bdv[1], bdv[0], bdc[1], bdc[0]);
      if (i + 2 < nst) step(i + 2, bdq[2], bdq[1], bdv[2], bdv[1], bdc[2], bdc[1]);
      wait_vmcnt<0>();  // the stages issued past the end land before the slots are reused
      if constexpr (PROF & 1) te = sk_stamp();
    } else {
      // as in the BD form: a stage issued every K-step, past the end too, so one wait count
#pragma unroll
    for (int k = 0; k < STAGES - 1; ++k) issue(k_a + k, k, bdq[0], bdv[0], bdc[0]);
    for (int i = 0; i < nst; ++i) {
      wait_vmcnt<(STAGES - 2) * INST_W>();
      __builtin_amdgcn_s_barrier();
      const float* As = lds_after_barrier(smem) + (i % STAGES) * STAGE;
      auto mid = [&] { issue(k_a + i + STAGES - 1, (i + STAGES - 1) % STAGES, bdq[0], bdv[0], bdc[0]); };
      if constexpr (MT == kMathBf16)
        mfma_stage_bf16<BK, TM, TN, BM, BN>(As, As + A_STAGE, wm, wn, lane, acc, mid);
      else if constexpr (MT == kMathX6)
        mfma_stage_x6<BK, TM, TN, BM, BN>(As, As + A_STAGE, wm, wn, lane, acc, mid);
      else if constexpr (MT == kMathX6P)
        mfma_stage_x6p<G, TM, TN, BM, BN>(As, As + A_STAGE, wm, wn, lane, acc, mid);
      else if constexpr (H1)
        mfma_stage_h1p<G, TM, TN, BM, BN>(As, As + A_STAGE, wm, wn, lane, acc, mid, sB);
      else if constexpr (H3)
        mfma_stage_h3p<G, TM, TN, BM, BN>(As, As + A_STAGE, wm, wn, lane, acc, mid, sB);
      else
        mfma_stage_pipe<BK, TM, TN, BM, BN>(As, As + A_STAGE, wm, wn, lane, acc, mid);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    wait_vmcnt<0>();  // the stages issued past the end land before the slots are reused
    }

    if constexpr (H3) {  // exact: both factors are powers of two
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * iA * iB;
    }
    constexpr int PSZ = BM * BN;
    if (k_a > 0 || k_b < sk.KS) {
      // A piece of a split tile: slot 0 = a piece that starts inside the tile (first segment of
      // the range), slot 1 = the tile's head piece (last segment of the range).  Stored row-major
      // [BM][BN] with plain stores (each half-wave writes 128 contiguous bytes per register) and
      // summed by k_sk_reduce after this launch: no flag, no fence, no wait.  (A last-arriver
      // fix-up inside the launch puts every tile's reduction at the very end of the kernel, where
      // all workgroups read pieces at once with nothing to overlap: 38 of 135 us on layer3.)
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)sk.part, (short)0, (int)min(0x7fffffffLL, (long long)sk.NW * 2 * PSZ * 4), 0x00020000);
      const unsigned pbase = (unsigned)((sw * 2 + (k_a > 0 ? 0 : 1)) * PSZ * 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nl = wn + j * 32 + (lane & 31);
          const int ml = wm + i * 32 + 4 * (lane >> 5);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ro = (r & 3) + 8 * (r >> 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                  pbase + (unsigned)(((ml + ro) * BN + nl) * 4), 0, 0);
          }
        }
      continue;
    }
    // sole worker of the tile: final output (+ the summed branch biases)
    // through a buffer resource; columns past P get an out-of-range offset, rows past M too.
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.C, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
    const bool full_m = m0 + BM <= a.M;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + j * 32 + (lane & 31);
        const int mrow = m0 + wm + i * 32 + 4 * (lane >> 5);
        const unsigned voff = n < a.P ? (unsigned)((mrow * a.P + n) * 4) : OOB;
        // ACC (msl_pconv_dgrad_acc, a compile-time form so the plain epilogue keeps its
        // registers): the fragment's 16 old values are loaded before its first store, so they are
        // in flight together (load-add-store per element serialised each load behind the
        // previous element's store: +30 us on a 2048 x 8385 output)
        float old[16];
        if constexpr (ACC) {
          if (a.accres) {  // r06: the masked residual gradient (acc_masked) instead of C's old values
            // the lane's column fixes the image, the mask word (32-bit half) and the bit once per
            // fragment; the 16 rows then differ by constant strides (buffer loads, OOB -> 0)
            const int hw = a.P / a.accni;
            const int img = n / hw, px = n - img * hw;
            const int w32 = ((hw + 63) >> 6) * 2;  // 32-bit mask words per (row, image)
            const unsigned mstride = (unsigned)(a.accni * w32 * 4);
            const unsigned moff = n < a.P ? (unsigned)(((mrow * a.accni + img) * w32 + (px >> 5)) * 4) : OOB;
            const int sh = px & 31;
            const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
                (void*)a.accres, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
            const __amdgpu_buffer_rsrc_t rmk = __builtin_amdgcn_make_buffer_rsrc(
                (void*)a.accmask, (short)0, (int)min(0x7fffffffLL, (long long)a.M * mstride), 0x00020000);
            unsigned mw[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int ro = (r & 3) + 8 * (r >> 2);
              const bool in = full_m || mrow + ro < a.M;
              old[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, in ? voff + ro * a.P * 4 : OOB, 0, 0));
              mw[r] = __builtin_amdgcn_raw_buffer_load_b32(rmk, in && n < a.P ? moff + ro * mstride : OOB, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) old[r] = ((mw[r] >> sh) & 1u) ? old[r] : 0.f;
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int ro = (r & 3) + 8 * (r >> 2);
              const unsigned off = full_m ? voff + ro * a.P * 4 : (mrow + ro < a.M ? voff + ro * a.P * 4 : OOB);
              old[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rc, off, 0, 0));
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          float v = acc[i][j][r];
          if (a.bias && mrow + ro < a.M) {
            float bsum = a.bias[mrow + ro];
            for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + mrow + ro];
            v += bsum;
          }
          const unsigned off = full_m ? voff + ro * a.P * 4 : (mrow + ro < a.M ? voff + ro * a.P * 4 : OOB);
          if constexpr (ACC) v = old[r] + v;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, off, 0, 0);
        }
      }
  }
  if constexpr (PROF & 1) {
    if (lane == 0) {  // vector stores of the wave-uniform sums (lane 0)
      const int gw = blockIdx.x * (blockDim.x >> 6) + wid;
#pragma unroll
      for (int k = 0; k < 6; ++k) sk.prof[gw * 8 + k] = ph[k];
    }
  }
}

template <int BM, int BN, int G, int STAGES, int WM, int WN, bool PW = false, int MT = 0, bool ACC = false>
__global__ void __launch_bounds__(256) k_igemm_fwd_sk(FwdArgs a, SkArgs sk) {
  fwd_sk_body<BM, BN, G, STAGES, WM, WN, PW, MT, ACC>(a, sk);
}

// The same kernel held to two waves per SIMD (<= 256 VGPRs + AGPRs): the f16x3 form, left to the
// compiler's default budget, takes 199 VGPRs + 64 AGPRs and one wave per SIMD.
template <int BM, int BN, int G, int STAGES, int WM, int WN, bool PW = false, int MT = 0, bool ACC = false,
          bool BD = false, bool BP = false, int PROF = 0>
__global__ void __launch_bounds__(256, 2) k_igemm_fwd_sk2(FwdArgs a, SkArgs sk) {
  fwd_sk_body<BM, BN, G, STAGES, WM, WN, PW, MT, ACC, BD, BP, PROF>(a, sk);
}

// sum of pieces w_lo..w_hi in that order (deterministic), eight loads in flight per step: a tile
// of the 132-tile layer3 GEMMs has 4-6 pieces, a chunked weight-gradient tile 7-14
template <typename F>
__device__ __forceinline__ float4 sum_pieces(int w_lo, int w_hi, F&& piece) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int wc = w_lo; wc <= w_hi; wc += 8) {
    float4 p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (wc + u <= w_hi) p[u] = piece(wc + u);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (wc + u <= w_hi) {
        acc.x += p[u].x;
        acc.y += p[u].y;
        acc.z += p[u].z;
        acc.w += p[u].w;
      }
  }
  return acc;
}

// Sum of the pieces of every split stream-K tile (worker order: deterministic), + the branch
// biases, into the output.  grid = (BM*BN / 1024 chunks, tiles - tdp: the stream-K tiles); blocks
// of unsplit tiles exit.  Pieces are row-major [BM][BN]: one float4 of 4 consecutive pixels per
// thread.
template <int BM, int BN>
__global__ void __launch_bounds__(256) k_sk_reduce(FwdArgs a, SkArgs sk) {
  constexpr int PSZ = BM * BN;
  const int tl = blockIdx.y, t = sk.tdp + tl;  // tile, and its index in the stream-K space
  const int w_lo = sk_worker_of(tl * sk.KS, sk.T, sk.NW);
  const int w_hi = sk_worker_of((tl + 1) * sk.KS - 1, sk.T, sk.NW);
  if (w_lo == w_hi) return;
  int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, sk.gm, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const float4* __restrict__ part = reinterpret_cast<const float4*>(sk.part);
  for (int g = blockIdx.x * 256 + threadIdx.x; g < PSZ / 4; g += gridDim.x * 256) {
    auto piece = [&](int wc) {
      const int slot = sk_start(wc, sk.T, sk.NW) > tl * sk.KS ? 0 : 1;
      return part[(long long)(wc * 2 + slot) * (PSZ / 4) + g];
    };
    const float4 acc = sum_pieces(w_lo, w_hi, piece);
    const int m = m0 + (g * 4) / BN, n = n0 + (g * 4) % BN;
    if (m >= a.M) continue;
    float bsum = 0.f;
    if (a.bias) {
      bsum = a.bias[m];
      for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + m];
    }
    float* dst = a.C + (long long)m * a.P + n;
    float vals[4] = {acc.x, acc.y, acc.z, acc.w};
    if (a.bias) {
#pragma unroll
      for (int c = 0; c < 4; ++c) vals[c] += bsum;
    }
    if (a.accum) {  // all four old values loaded before the first store
      float old[4];
      if (a.accres) {  // r06: the masked residual gradient (acc_masked)
#pragma unroll
        for (int c = 0; c < 4; ++c) old[c] = n + c < a.P ? acc_masked(a, m, n + c) : 0.f;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) old[c] = n + c < a.P ? dst[c] : 0.f;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) vals[c] = old[c] + vals[c];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (n + c < a.P) dst[c] = vals[c];
  }
}

// ---------------------------------------------------------------------------------------------
// Stream-K weight gradient.  dW[br][m][n][tap] = sum_p dY[m][p] * X[n][p + shift(br, tap)]:
// one GEMM tile (BM output channels x BN input channels) per (branch, tap, m-block, n-block),
// K = pixels in 64-pixel stages.  The (tile, stage) space is cut into NW equal worker ranges
// like k_igemm_fwd_sk; pieces of split tiles go to `part` and k_wsk_reduce sums them.
// Operands move by LDS-DMA, one 64-pixel row per wave-instruction (lane = pixel), into rows
// padded to 66 floats: the DMA of one row is lane-linear, and the MFMA operand reads - lane l32
// reads row l32 at two consecutive k (ds_read_b64) - hit 64 distinct banks.  A pixel outside the
// image (tap shift, row wrap) or past P gets an out-of-range offset, which the buffer unit
// zero-fills.  K is permuted inside a stage: half-wave kh takes pixels kh*32 .. kh*32+31, so a
// lane's two k of consecutive MFMAs are adjacent in LDS (any bijection of K is valid as long as
// both operands use it).
struct WskArgs {
  const float* dy;  // [M][P]
  const float* x;   // [N][P]
  float* dw;        // [nbranch][M][N][taps]
  float* part;      // [NW][slots][BM][BN]: worker w's piece of tile t in slot t - first_tile(w)
  int M, N, H, W, P, dil0, dil1, taps, accumulate, slots;  // H x W one image, P = nimg * H * W
  float invW, invH;
  int tiles_m, tiles_n, KS, NW, T;
  long long cbranch;  // M * N * taps
  const void* dyx6;   // k_wgrad_x6: dY split into bf16 planes by k_split_rows
  int lda;            // k_wgrad_x6: plane row length (M rounded up to kPackPad)
  // k_wgrad_x6 chunked split-K (nchunk > 0): work item i = (chunk c = i / ntiles, tile
  // t = i % ntiles) covers K-steps [c*kchunk, (c+1)*kchunk) of tile t and leaves one piece (slot
  // 0 of worker i); NW = ntiles * nchunk items.  Chunk-major items give the workgroups of one XCD
  // (consecutive items) the same pixel window of every tile: the window's dY and X rows stay in
  // that XCD's L2 across all tiles and taps.
  int nchunk, kchunk, ntiles;
  // pointwise (taps = 1) with the operands swapped (k_wgrad_x6 pre-splits the operand with fewer
  // rows): dy = the image [cin][P], x = dY [cout][P], M = cin, N = cout, so the tiles hold dW^T
  // and k_wsk_reduce writes them transposed into dw [cout][cin]
  int trans;
  // k_wgrad_x6<kMathH3P>: the kNPart absmax partials of the pre-split operand (dy) and of x
  const float* apart;
  const float* bpart;
  int anpart, bnpart;  // partials in apart / bpart
  // rowscale = 1: apart / bpart hold one maximum per row of their operand (anpart = M, bnpart = N),
  // and every row gets its own power-of-two scale: k_split_rows scales dY row m by s_m,
  // k_wgrad_x6 scales X row n by t_n, and k_wsk_reduce unscales dW[m][n] by 1/(s_m t_n) (exact).
  // Each dW element then keeps the full f16x3 precision of its own rows however far they sit below
  // the tensor's absolute maximum.  rowscale = 0: one scale per tensor (max over the partials).
  int rowscale;
};

constexpr int kWskBK = 64;

template <int BM, int BN, int STAGES, int WM, int WN, int MT = 0>
__global__ void __launch_bounds__(256) k_wgrad_sk(WskArgs a) {
  static_assert(WM * WN == 4, "4 waves");
  // row stride: 66 floats for the f32 b64 reads (64 distinct banks); 68 for the bf16 forms'
  // 16-B aligned b128 reads (4-dword chunks at 4*row: conflict-free per 16-lane group)
  constexpr int kWskLD = MT != kMathF32 ? 68 : 66;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(TM >= 1 && TN >= 1, "tiles");
  constexpr int A_STAGE = BM * kWskLD, STAGE = (BM + BN) * kWskLD;
  constexpr int AR_W = BM / 4, BR_W = BN / 4;  // rows (= DMA instructions) per wave and stage
  constexpr int INST_W = AR_W + BR_W;
  static_assert((STAGES - 2) * INST_W < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) float smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wid / WN) * (TM * 32), wn = (wid % WN) * (TN * 32);
  const int l32 = lane & 31, kh = lane >> 5;
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);
  const int it_begin = sk_start(w, a.T, a.NW), it_end = sk_start(w + 1, a.T, a.NW);

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.dy, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)min(0x7fffffffLL, (long long)a.N * a.P * 4), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned row_bytes = (unsigned)a.P * 4u;

  f32x16 acc[TM][TN];
  for (int it = it_begin; it < it_end;) {
    const int t = (unsigned)it / (unsigned)a.KS;
    const int k_a = it - t * a.KS;
    const int k_b = min(a.KS, k_a + (it_end - it));
    const int nst = k_b - k_a;
    it += nst;
    const int tm = t % a.tiles_m;
    const int t2 = t / a.tiles_m;
    const int tn = t2 % a.tiles_n;
    const int z = t2 / a.tiles_n;  // branch * taps + tap
    const int br = z / a.taps, tap = z - br * a.taps;
    const int m0 = tm * BM, n0 = tn * BN;
    const int d = br ? a.dil1 : a.dil0;
    const int dh = (tap / 3 - 1) * d, dw = (tap % 3 - 1) * d;
    const int shift = dh * a.W + dw;
    // scalar row offsets of this wave's rows (OOB past M / N)
    auto issue = [&](int s, int slot) {
      float* As = smem + slot * STAGE;
      float* Bs = As + A_STAGE;
      const int p = s * kWskBK + lane;
      const int pq = (int)(((float)p + 0.5f) * a.invW);
      const int px = p - pq * a.W;
      const int py = pq - a.H * (int)(((float)pq + 0.5f) * a.invH);  // row within its image
      const unsigned va = p < a.P ? (unsigned)p * 4u : OOB;
      const bool vb = p < a.P && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
      const unsigned vbo = vb ? (unsigned)(p + shift) * 4u : OOB;
#pragma unroll
      for (int i = 0; i < AR_W; ++i) {
        const int r = wid * AR_W + i;
        const unsigned ro = m0 + r < a.M ? (unsigned)(m0 + r) * row_bytes : OOB;
        dma_b32(rA, As + r * kWskLD, va + ro);
      }
#pragma unroll
      for (int i = 0; i < BR_W; ++i) {
        const int r = wid * BR_W + i;
        const unsigned ro = n0 + r < a.N ? (unsigned)(n0 + r) * row_bytes : OOB;
        dma_b32(rB, Bs + r * kWskLD, vbo + ro);
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int k = 0; k < STAGES - 1; ++k)
      if (k < nst) issue(k_a + k, k);
    for (int i = 0; i < nst; ++i) {
      const int younger = min(STAGES - 2, nst - 1 - i);
      if constexpr (STAGES >= 3) {
        if (younger >= 1) wait_vmcnt<INST_W>();
        else wait_vmcnt<0>();
      } else {
        wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      if (i + STAGES - 1 < nst) issue(k_a + i + STAGES - 1, (i + STAGES - 1) % STAGES);
      const float* As = lds_after_barrier(smem) + (i % STAGES) * STAGE;
      const float* Bs = As + A_STAGE;
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      if constexpr (MT != kMathF32) {
        // lane (r, h) of v_mfma_f32_32x32x16_bf16 takes pixels kk*16 + 8h .. +7 of row r
        typedef typename MathFrag<MT>::type Frag;
#pragma unroll
        for (int kk = 0; kk < kWskBK / 16; ++kk) {
          const int kc = kk * 16 + 8 * kh;
          Frag av[TM], bv[TN];
          auto rd8 = [&](Frag& f, const float* row) {
            const float4* src = reinterpret_cast<const float4*>(row + kc);
            const float4 u = src[0], v = src[1];
            frag_set<MT>(f, 0, u.x); frag_set<MT>(f, 1, u.y); frag_set<MT>(f, 2, u.z); frag_set<MT>(f, 3, u.w);
            frag_set<MT>(f, 4, v.x); frag_set<MT>(f, 5, v.y); frag_set<MT>(f, 6, v.z); frag_set<MT>(f, 7, v.w);
          };
#pragma unroll
          for (int ii = 0; ii < TM; ++ii) rd8(av[ii], As + (wm + ii * 32 + l32) * kWskLD);
#pragma unroll
          for (int jj = 0; jj < TN; ++jj) rd8(bv[jj], Bs + (wn + jj * 32 + l32) * kWskLD);
#pragma unroll
          for (int ii = 0; ii < TM; ++ii)
#pragma unroll
            for (int jj = 0; jj < TN; ++jj) acc[ii][jj] = frag_mma<MT>(av[ii], bv[jj], acc[ii][jj]);
        }
      } else {
#pragma unroll
      for (int kq = 0; kq < kWskBK / 4; ++kq) {
        const int kc = kh * 32 + 2 * kq;
        f32x2 av[TM], bv[TN];
#pragma unroll
        for (int ii = 0; ii < TM; ++ii)
          av[ii] = *reinterpret_cast<const f32x2*>(As + (wm + ii * 32 + l32) * kWskLD + kc);
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
          bv[jj] = *reinterpret_cast<const f32x2*>(Bs + (wn + jj * 32 + l32) * kWskLD + kc);
#pragma unroll
        for (int ii = 0; ii < TM; ++ii)
#pragma unroll
          for (int jj = 0; jj < TN; ++jj)
            acc[ii][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[ii].x, bv[jj].x, acc[ii][jj], 0, 0, 0);
#pragma unroll
        for (int ii = 0; ii < TM; ++ii)
#pragma unroll
          for (int jj = 0; jj < TN; ++jj)
            acc[ii][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[ii].y, bv[jj].y, acc[ii][jj], 0, 0, 0);
      }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // Every tile leaves its piece(s) in `part` (an unsplit tile: one slot-1 piece): dW is
    // [m][n][tap], so a tile's own stores would be 36-B strided; k_wsk_reduce writes all taps of
    // an (m, n) together.
    constexpr int PSZ = BM * BN;
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.part, (short)0, (int)min(0x7fffffffLL, (long long)a.NW * a.slots * PSZ * 4), 0x00020000);
    const int slot = t - it_begin / a.KS;
    const unsigned pbase = (unsigned)((w * a.slots + slot) * PSZ * 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn + j * 32 + l32;
        const int ml = wm + i * 32 + 4 * kh;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                pbase + (unsigned)(((ml + ro) * BN + nl) * 4), 0, 0);
        }
      }
  }
}

// dW (=|+=) the sum of every tile's pieces, in worker order.  One thread per (4 consecutive
// (m, n), tap) of an (m-block, n-block, branch) group, (m, n) fastest: the piece reads are float4
// and coalesced (consecutive threads, consecutive elements of one piece); the dW stores ([m][n]
// [tap]) are taps apart.  grid = (ceil(BM*BN / 4 * taps / 256), tiles_m * tiles_n * nbranch).
template <int BM, int BN>
__global__ void __launch_bounds__(256) k_wsk_reduce(WskArgs a) {
  constexpr int PSZ = BM * BN, P4 = PSZ / 4;
  static_assert(BN % 4 == 0, "float4 rows");
  const int gsz = a.tiles_m * a.tiles_n;
  const int br = blockIdx.y / gsz;
  const int rem = blockIdx.y - br * gsz;
  const int tn = rem / a.tiles_m, tm = rem - tn * a.tiles_m;
  if constexpr (BM == 128 && BN == 128) {
    if (a.trans) {
      // dW^T tile (pointwise, operands swapped; taps = nbranch = 1): block = one 32x32 sub-tile,
      // summed as float4 rows, transposed through LDS, written as 128-B runs of dw rows
      __shared__ float tt[32][33];
      const int sr = blockIdx.x >> 2, sc = blockIdx.x & 3;
      const int t = tn * a.tiles_m + tm;
      const int r = threadIdx.x >> 3, c4 = (threadIdx.x & 7) * 4;
      const int g4 = ((sr * 32 + r) * BN + sc * 32 + c4) / 4;
      const float4* __restrict__ part = reinterpret_cast<const float4*>(a.part);
      const int w_lo = a.nchunk > 0 ? 0 : sk_worker_of(t * a.KS, a.T, a.NW);
      const int w_hi = a.nchunk > 0 ? a.nchunk - 1 : sk_worker_of((t + 1) * a.KS - 1, a.T, a.NW);
      const float4 v = sum_pieces(w_lo, w_hi, [&](int wc) {
        if (a.nchunk > 0) return part[(long long)(wc * a.ntiles + t) * a.slots * P4 + g4];
        return part[(long long)(wc * a.slots + t - sk_start(wc, a.T, a.NW) / a.KS) * P4 + g4];
      });
      float sv[4] = {v.x, v.y, v.z, v.w};
      if (a.rowscale) {  // tile element (m, n): 1 / (s_m t_n), exact
        float ia, ib;
        pow2_scale(a.apart[min(a.M - 1, tm * BM + sr * 32 + r)], ia);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pow2_scale(a.bpart[min(a.N - 1, tn * BN + sc * 32 + c4 + q)], ib);
          sv[q] = sv[q] * ia * ib;
        }
      }
      tt[r][c4] = sv[0];
      tt[r][c4 + 1] = sv[1];
      tt[r][c4 + 2] = sv[2];
      tt[r][c4 + 3] = sv[3];
      __syncthreads();
      // thread -> dW row n = n0 + sc*32 + (tid >> 3) (a cout), columns m = m0 + sr*32 + rr .. + 3
      const int n = tn * BN + sc * 32 + (threadIdx.x >> 3), rr = (threadIdx.x & 7) * 4;
      if (n >= a.N) return;
      float* dst = a.dw + (long long)n * a.M + tm * BM + sr * 32 + rr;
      const int mm = a.M - (tm * BM + sr * 32 + rr);
      float vals[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) vals[q] = tt[rr + q][threadIdx.x >> 3];
      if (a.accumulate) {
        float old[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) old[q] = q < mm ? dst[q] : 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) vals[q] = old[q] + vals[q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < mm) dst[q] = vals[q];
      return;
    }
  }
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int tap = e / P4, g4 = e - tap * P4;
  if (tap >= a.taps) return;
  const int m = tm * BM + (g4 * 4) / BN, n = tn * BN + (g4 * 4) % BN;
  if (m >= a.M || n >= a.N) return;
  const int t = ((br * a.taps + tap) * a.tiles_n + tn) * a.tiles_m + tm;
  const float4* __restrict__ part = reinterpret_cast<const float4*>(a.part);
  // stream-K: the workers whose ranges touch tile t, in order; chunked: the items (c, t), c = 0..
  const int w_lo = a.nchunk > 0 ? 0 : sk_worker_of(t * a.KS, a.T, a.NW);
  const int w_hi = a.nchunk > 0 ? a.nchunk - 1 : sk_worker_of((t + 1) * a.KS - 1, a.T, a.NW);
  auto piece = [&](int wc) {
    if (a.nchunk > 0) return part[(long long)(wc * a.ntiles + t) * a.slots * P4 + g4];
    const int slot = t - sk_start(wc, a.T, a.NW) / a.KS;
    return part[(long long)(wc * a.slots + slot) * P4 + g4];
  };
  const float4 v = sum_pieces(w_lo, w_hi, piece);
  float* dst = a.dw + br * a.cbranch + ((long long)m * a.N + n) * a.taps + tap;
  float vals[4] = {v.x, v.y, v.z, v.w};
  const int nn = min(4, a.N - n);
  if (a.rowscale) {  // per-row f16x3 scales (k_wgrad_x6): dW[m][n] / (s_m t_n), exact
    float ia, ib;
    pow2_scale(a.apart[m], ia);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      pow2_scale(a.bpart[min(a.N - 1, n + c)], ib);
      vals[c] = vals[c] * ia * ib;
    }
  }
  if (a.accumulate) {  // all old values loaded before the first store
    float old[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) old[c] = c < nn ? dst[c * a.taps] : 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) vals[c] = old[c] + vals[c];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < nn) dst[c * a.taps] = vals[c];
}

// k_wsk_reduce's generic form for tiles with many pieces and few tiles (the 33k-px 1x1 weight
// gradients on 64x64 tiles: 4 tiles x ~128 pieces, 16 blocks of k_wsk_reduce, 27 us): S threads per
// float4 output, thread s summing pieces w_lo + s, w_lo + s + S, ... in order, the S partial sums
// then added in s order through LDS (deterministic; a different but fixed association).
// grid = (ceil(BM*BN/4 * taps / (256/S)), tiles_m * tiles_n * nbranch); stream-K pieces only.
template <int BM, int BN, int S>
__global__ void __launch_bounds__(256) k_wsk_reduce_wide(WskArgs a) {
  constexpr int PSZ = BM * BN, P4 = PSZ / 4, OPB = 256 / S;  // float4 outputs per block
  __shared__ float4 red[256];
  const int gsz = a.tiles_m * a.tiles_n;
  const int br = blockIdx.y / gsz;
  const int rem = blockIdx.y - br * gsz;
  const int tn = rem / a.tiles_m, tm = rem - tn * a.tiles_m;
  const int o = threadIdx.x / S, sl = threadIdx.x - o * S;
  const int e = blockIdx.x * OPB + o;
  const int tap = e / P4, g4 = e - tap * P4;
  const bool live = tap < a.taps;
  const int t = ((br * a.taps + (live ? tap : 0)) * a.tiles_n + tn) * a.tiles_m + tm;
  const float4* __restrict__ part = reinterpret_cast<const float4*>(a.part);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    const int w_lo = sk_worker_of(t * a.KS, a.T, a.NW);
    const int w_hi = sk_worker_of((t + 1) * a.KS - 1, a.T, a.NW);
    for (int wc = w_lo + sl; wc <= w_hi; wc += S) {
      const int slot = t - sk_start(wc, a.T, a.NW) / a.KS;
      const float4 v = part[(long long)(wc * a.slots + slot) * P4 + g4];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (sl != 0 || !live) return;
  float4 v = red[o * S];
#pragma unroll
  for (int q = 1; q < S; ++q) {
    const float4 u = red[o * S + q];
    v.x += u.x;
    v.y += u.y;
    v.z += u.z;
    v.w += u.w;
  }
  const int m = tm * BM + (g4 * 4) / BN, n = tn * BN + (g4 * 4) % BN;
  if (m >= a.M || n >= a.N) return;
  float* dst = a.dw + br * a.cbranch + ((long long)m * a.N + n) * a.taps + tap;
  float vals[4] = {v.x, v.y, v.z, v.w};
  const int nn = min(4, a.N - n);
  if (a.accumulate) {  // all old values loaded before the first store
    float old[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) old[c] = c < nn ? dst[c * a.taps] : 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) vals[c] = old[c] + vals[c];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < nn) dst[c * a.taps] = vals[c];
}

// r06: k_wsk_reduce's [m][n] (not transposed) form with S waves per block summing disjoint, interleaved subsets of
// a tile's pieces: wave s adds pieces w_lo + s, w_lo + s + S, ... in order for 64 consecutive float4 outputs
// (each load a coalesced 1-KB run of one piece), and wave 0 adds the S partial sums in s order (deterministic;
// a different, fixed association than k_wsk_reduce's single chain).  One chain per output put 8 loads in flight
// per thread at one 256-thread block per (tile, 64 outputs): the 1 x 1 1024 -> 256 reduce read its 32 MB of
// pieces at ~2.7 TB/s.  grid = (ceil(BM*BN/4 * taps / 64), tiles_m * tiles_n * nbranch), block 64 * S.
template <int BM, int BN, int S>
__global__ void __launch_bounds__(64 * S) k_wsk_reduce_split(WskArgs a) {
  static_assert(S >= 4, "the transposed form writes 256 values per block");
  constexpr int PSZ = BM * BN, P4 = PSZ / 4;
  __shared__ float4 red[64 * S];
  const int gsz = a.tiles_m * a.tiles_n;
  const int br = blockIdx.y / gsz;
  const int rem = blockIdx.y - br * gsz;
  const int tn = rem / a.tiles_m, tm = rem - tn * a.tiles_m;
  const int o = threadIdx.x & 63, sl = threadIdx.x >> 6;
  // trans (pointwise, operands swapped; taps = 1): block = an 8-row x 32-column sub-tile (64 float4), transposed
  // through LDS below; else 64 consecutive float4 of the [tap][m][n] piece layout
  const int sr = blockIdx.x >> 2, sc = blockIdx.x & 3;
  const int e = a.trans ? ((sr * 8 + (o >> 3)) * BN + sc * 32 + (o & 7) * 4) / 4 : blockIdx.x * 64 + o;
  const int tap = e / P4, g4 = e - tap * P4;
  const bool live = tap < a.taps;
  const int t = ((br * a.taps + (live ? tap : 0)) * a.tiles_n + tn) * a.tiles_m + tm;
  const float4* __restrict__ part = reinterpret_cast<const float4*>(a.part);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    const int w_lo = a.nchunk > 0 ? 0 : sk_worker_of(t * a.KS, a.T, a.NW);
    const int w_hi = a.nchunk > 0 ? a.nchunk - 1 : sk_worker_of((t + 1) * a.KS - 1, a.T, a.NW);
    auto piece = [&](int wc) {
      if (a.nchunk > 0) return part[(long long)(wc * a.ntiles + t) * a.slots * P4 + g4];
      return part[(long long)(wc * a.slots + t - sk_start(wc, a.T, a.NW) / a.KS) * P4 + g4];
    };
    for (int wc = w_lo + sl; wc <= w_hi; wc += 4 * S) {  // four loads in flight, added in order
      float4 p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (wc + u * S <= w_hi) p[u] = piece(wc + u * S);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (wc + u * S <= w_hi) {
          acc.x += p[u].x;
          acc.y += p[u].y;
          acc.z += p[u].z;
          acc.w += p[u].w;
        }
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  float4 v = red[o];
  if (sl == 0) {
#pragma unroll
    for (int q = 1; q < S; ++q) {
      const float4 u = red[q * 64 + o];
      v.x += u.x;
      v.y += u.y;
      v.z += u.z;
      v.w += u.w;
    }
  }
  const int m = tm * BM + (g4 * 4) / BN, n = tn * BN + (g4 * 4) % BN;
  if (a.trans) {  // dW^T: wave 0's sums (rowscaled) to LDS, then every thread writes one of 32 dW rows x 8 columns
    __shared__ float tt[8][33];
    if (sl == 0) {
      float sv[4] = {v.x, v.y, v.z, v.w};
      if (a.rowscale) {  // tile element (m, n): 1 / (s_m t_n), exact
        float ia, ib;
        pow2_scale(a.apart[min(a.M - 1, m)], ia);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pow2_scale(a.bpart[min(a.N - 1, n + q)], ib);
          sv[q] = sv[q] * ia * ib;
        }
      }
      const int r = o >> 3, c4 = (o & 7) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) tt[r][c4 + q] = sv[q];
    }
    __syncthreads();
    if (threadIdx.x >= 256) return;
    const int j = threadIdx.x >> 3, i = threadIdx.x & 7;  // dW row n0 + j (a cout), column m0 + i
    const int nr = tn * BN + sc * 32 + j, mc = tm * BM + sr * 8 + i;
    if (nr >= a.N || mc >= a.M) return;
    float* dst = a.dw + (long long)nr * a.M + mc;
    float val = tt[i][j];
    if (a.accumulate) val = *dst + val;
    *dst = val;
    return;
  }
  if (sl != 0 || !live) return;
  if (m >= a.M || n >= a.N) return;
  float* dst = a.dw + br * a.cbranch + ((long long)m * a.N + n) * a.taps + tap;
  float vals[4] = {v.x, v.y, v.z, v.w};
  const int nn = min(4, a.N - n);
  if (a.rowscale) {  // per-row f16x3 scales (k_wgrad_x6): dW[m][n] / (s_m t_n), exact
    float ia, ib;
    pow2_scale(a.apart[m], ia);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      pow2_scale(a.bpart[min(a.N - 1, n + c)], ib);
      vals[c] = vals[c] * ia * ib;
    }
  }
  if (a.accumulate) {  // all old values loaded before the first store
    float old[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) old[c] = c < nn ? dst[c * a.taps] : 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) vals[c] = old[c] + vals[c];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < nn) dst[c * a.taps] = vals[c];
}

// ---------------------------------------------------------------------------------------------
// bf16x6 weight gradient, register-staged (the layer2-4 and ASPP-free x6 path).
//
// k_wgrad_sk moves both fp32 operands by LDS-DMA, one 64-pixel row per wave-instruction (64 DMA
// issues per wave and stage at 128x128), and every wave splits the fp32 values of its own
// fragments into bf16 terms - each element twice, once per wave sharing its rows.  Here:
//   - dY is split once per call into bf16 planes (k_split_rows: [K-step = 16 pixels][plane]
//     [k half][row][8], zeros past P and M), read by each wave straight into registers (one 16-B
//     vector per lane and plane, one K-step ahead, like the forward's packed weights);
//   - X rows are loaded by threads in 4-pixel chunks (16-B loads; 8 lanes cover a row's 32
//     pixels of the stage, one 128-B line), masked, split once and written to LDS as 8-B quarters
//     of [plane][k half][n][8] rows - the forward kernels' B layout (ds_read_b128 fragments), with
//     32 B of padding per (plane, half) row block so both the 8-B stores and the fragment reads
//     are conflict-free;
//   - the image-border mask of a tap depends only on the pixel, so it is computed per K-step in
//     scalar registers (16 bits: row and column range tests of the K-step's pixel run) and each
//     lane tests its chunk's 4 bits;
//   - two K-steps per LDS stage, one barrier per 48 MFMAs per wave; pieces and k_wsk_reduce as
//     k_wgrad_sk (every tile leaves its pieces; the reduce writes dW taps-innermost).
// K-step = 16 pixels: KS = ceil(P / 16) per tile.  Needs W >= 16 (the mask handles one row wrap).
constexpr int kWx6BK = 16;

// planes[((ks*3 + q)*2 + h)*lda + m][j] = term q of src[m][ks*16 + 8h + j] (0 past P or M).
// Block = R = kSplitRowsR rows x 16 K-steps (256 pixels).  Each wave loads R / 4 rows, 16 B per lane and
// row (4 pixels: one coalesced 1-KB run per row and load; the r03 form's dword loads moved 256 B per
// instruction and ran at 3.3 TB/s), splits them and stores the 16-bit terms to LDS as [plane][row][pixel]
// rows padded to 528 B; the block then writes every (K-step, plane, half) as R consecutive rows of 16-B
// vectors (ds_read_b128 at a 528-B stride: conflict-free).  grid = (lda / R, ceil(KS / 16)).
// MT = kMathH3P: two fp16 planes of src * s, s = pow2_scale of src's absmax partials `part`.
// r05: R = 16 instead of 32 (twice the blocks, half the LDS each: more of them resident, so one block's
// load round trip overlaps another's transpose and stores)
constexpr int kSplitRowsR = 16;
template <int MT = kMathX6>
__global__ void __launch_bounds__(256) k_split_rows(const float* __restrict__ src, int M, int P, int KS, int lda,
                                                     bf16x8* __restrict__ planes, const float* __restrict__ part,
                                                     int npart, int rowscale = 0) {
  // LDS row stride (16-bit terms): 272 = 136 dwords, 8 mod 64, so the 16-B reads of a 16-lane group - rows r
  // of one k half and rows of the other, 16 B further - land on distinct bank slots (2r + h mod 16); r05 had
  // 264 (4 mod 64), where k half 1 of row r met row r + 1: 25 % of the kernel's LDS cycles were conflicts
  constexpr int R = kSplitRowsR, PX = 256, LDP = PX + 16;  // rows, pixels per block
  constexpr int KB = PX / kWx6BK;                // K-steps per block
  constexpr bool F16 = MT == kMathH3P || MT == kMathH1P;
  constexpr int NP = MT == kMathH1P ? 1 : F16 ? 2 : 3;
  __shared__ __attribute__((aligned(16))) unsigned short tile[NP * R * LDP];
  typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int m0 = blockIdx.x * R, ks0 = blockIdx.y * KB;
  const int p = ks0 * kWx6BK + 4 * lane;  // this lane's four pixels
  float sc = 1.f, inv;
  if constexpr (F16) {
    if (!rowscale) sc = pow2_scale(partials_max(part, npart, lane), inv);
  }
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)src, (short)0, (int)min(0x7fffffffLL, (long long)M * P * 4), 0x00020000);
  float v[R / 4][4];
#pragma unroll
  for (int i = 0; i < R / 4; ++i) {
    const int m = m0 + wv + 4 * i;
    union { u32x4 u; float f[4]; } c;
    if (p + 3 < P) {
      c.u = __builtin_amdgcn_raw_buffer_load_b128(rs, m < M ? (unsigned)(m * P + p) * 4u : 0x80000000u, 0, 0);
    } else {  // the block's last pixels: element by element, 0 past P
#pragma unroll
      for (int j = 0; j < 4; ++j)
        c.f[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rs, (m < M && p + j < P) ? (unsigned)(m * P + p + j) * 4u : 0x80000000u, 0, 0));
    }
    float s = sc;
    if constexpr (F16) {  // the row's own scale (its maximum: one partial per row)
      if (rowscale) s = m < M ? pow2_scale(part[m], inv) : 1.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[i][j] = F16 ? c.f[j] * s : c.f[j];
  }
#pragma unroll
  for (int i = 0; i < R / 4; ++i) {
    const int r = wv + 4 * i;
    u16x4 t0, t1, t2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = v[i][j];
      if constexpr (MT == kMathH1P) {
        t0[j] = __builtin_bit_cast(unsigned short, (_Float16)x);
      } else if constexpr (MT == kMathH3P) {
        const _Float16 h = (_Float16)x;
        t0[j] = __builtin_bit_cast(unsigned short, h);
        t1[j] = __builtin_bit_cast(unsigned short, (_Float16)(x - (float)h));
      } else {
        const __bf16 h = (__bf16)x;
        const float rem = x - (float)h;
        const __bf16 md = (__bf16)rem;
        t0[j] = __builtin_bit_cast(unsigned short, h);
        t1[j] = __builtin_bit_cast(unsigned short, md);
        t2[j] = __builtin_bit_cast(unsigned short, (__bf16)(rem - (float)md));
      }
    }
    *reinterpret_cast<u16x4*>(&tile[(0 * R + r) * LDP + 4 * lane]) = t0;
    if constexpr (NP > 1) *reinterpret_cast<u16x4*>(&tile[(1 * R + r) * LDP + 4 * lane]) = t1;
    if constexpr (NP > 2) *reinterpret_cast<u16x4*>(&tile[(2 * R + r) * LDP + 4 * lane]) = t2;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < KB * NP * 2 * R / 256; ++i) {  // (K-step, plane, half, row) vectors: 2*NP per K-step
    const int idx = tid + 256 * i;
    const int r = idx & (R - 1), u = idx / R;  // u = (ksl*NP + q)*2 + h
    const int h = u & 1, q = (u >> 1) % NP, ksl = u / (2 * NP);
    const int ks = ks0 + ksl;
    if (ks < KS)
      planes[(long long)((ks * NP + q) * 2 + h) * lda + m0 + r] =
          *reinterpret_cast<const bf16x8*>(&tile[(q * R + r) * LDP + ksl * kWx6BK + h * 8]);
  }
}

// k_wgrad_x6's per-segment border-mask table (K-steps): a segment up to this long reads its masks from
// LDS, computed by all threads at the segment's start, instead of the per-stage scalar cursor (r05)
constexpr int kWxMaskTab = 2048;

// MT = kMathH3P (f16x3): dY (the pre-split operand) as two fp16 planes scaled by k_split_rows<H3>,
// X scaled by its own pow2_scale (absmax partials bpart) and split into two fp16 planes; the
// pieces are unscaled by both before they are stored.
template <int MT = kMathX6>
__global__ void __launch_bounds__(256, 2) k_wgrad_x6(WskArgs a) {
  constexpr bool H1 = MT == kMathH1P;  // fp16 math: the hi planes only
  constexpr bool H3 = MT == kMathH3P || H1;
  constexpr int NP = H1 ? 1 : H3 ? 2 : 3;  // planes per operand
  constexpr int BM = 128, BN = 128, TM = 2, TN = 2;
  constexpr int RB = 128 * 16 + 32;   // bytes per (plane, k half) block of 128 rows, padded
  constexpr int KVB = 2 * NP * RB;    // one K-step's B planes
  // the second K-step of a stage starts 64 B past a multiple of 128 B (r06): a 16-lane group of the 8-B
  // plane stores holds both K-steps of two rows, and at f16x3's KVB (8320 B = 0 mod 128) the two K-steps
  // hit the same 16 banks - 2-way conflicts on every store, 34 % of the kernel's LDS cycles
  // (profiles/r05_wgrad_sq_final.txt); at 64 mod 128 they take the other 16
  constexpr int KVS = KVB + (192 - KVB % 128) % 128;
  constexpr int STAGEB = 2 * KVS;     // two K-steps
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  // + (r05) the segment's border-mask table: 16 bits per K-step, kWxMaskTab K-steps
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGEB + kWxMaskTab * 2];  // the only LDS object
  unsigned short* const mtab = reinterpret_cast<unsigned short*>(smem + 2 * STAGEB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const int l32 = lane & 31, kh = lane >> 5;
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);  // XCD-aware worker id
  int it_begin, it_end;
  if (a.nchunk > 0) {  // chunked split-K: one (chunk, tile) item per workgroup
    if (w >= a.NW) return;
    const int c = w / a.ntiles, t = w - c * a.ntiles;
    it_begin = t * a.KS + c * a.kchunk;
    it_end = t * a.KS + min(a.KS, (c + 1) * a.kchunk);
  } else {
    it_begin = sk_start(w, a.T, a.NW);
    it_end = sk_start(w + 1, a.T, a.NW);
  }

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.dyx6, (short)0, (int)min(0x7fffffffLL, (long long)a.KS * 2 * NP * a.lda * 16), 0x00020000);
  float sX = 1.f, iA = 1.f, iB = 1.f;
  if constexpr (H3) {
    if (!a.rowscale) {
      sX = pow2_scale(partials_max(a.bpart, a.bnpart, lane), iB);
      pow2_scale(partials_max(a.apart, a.anpart, lane), iA);
    }
  }
  float sXr[4] = {sX, sX, sX, sX};  // the scales of this thread's four B rows (per tile with rowscale)
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)min(0x7fffffffLL, (long long)a.N * a.P * 4), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned a_plane_bytes = (unsigned)a.lda * 16u;
  // this thread's B chunks: c = tid + 256 i -> row c / 8, chunk c % 8 (4 pixels) of the stage's 32
  const int cc = tid & 7;
  const int ck = cc >> 2, chh = (cc >> 1) & 1, cq = cc & 1;  // K-step, k half, quarter
  const int wofs = ck * KVS + chh * RB + (tid >> 3) * 16 + cq * 8;  // + q*2*RB + i*32*16

  f32x16 acc[TM][TN];
  for (int it = it_begin; it < it_end;) {
    const int t = (unsigned)it / (unsigned)a.KS;
    const int k_a = it - t * a.KS;
    const int k_b = min(a.KS, k_a + (it_end - it));
    const int nst = k_b - k_a;
    it += nst;
    const int tm = t % a.tiles_m;
    const int t2 = t / a.tiles_m;
    const int tn = t2 % a.tiles_n;
    const int z = t2 / a.tiles_n;  // branch * taps + tap
    const int br = z / a.taps, tap = z - br * a.taps;
    const int m0 = tm * BM, n0 = tn * BN;
    const int d = br ? a.dil1 : a.dil0;
    const int dh = (tap / 3 - 1) * d, dw = (tap % 3 - 1) * d;
    const int shift = dh * a.W + dw;
    // pixel cursor of the next K-step to load (scalar): ks*16 = cy*W + cx
    int ld_ks = k_a;
    int cy = (k_a * kWx6BK) / a.W, cx = k_a * kWx6BK - cy * a.W;  // cy: row within its image
    cy %= a.H;
    const int clo = max(0, -dw), chi = a.W - max(0, dw);  // valid source columns px + dw
    auto seg = [](int lo, int hi) -> unsigned {      // bits lo .. hi-1 of a 16-bit mask
      lo = max(lo, 0);
      hi = min(hi, 16);
      return hi > lo ? ((1u << hi) - (1u << lo)) : 0u;
    };
    // an unshifted tap (every pointwise gradient, the 3x3 centre tap): every pixel valid, no cursor
    // (r05: ~25 fewer scalar instructions per stage there)
    const bool unshifted = shift == 0;
    auto kmask = [&]() -> unsigned {  // valid pixels of K-step ld_ks; advances the cursor
      unsigned m16 = 0;
      if (ld_ks < k_b) {
        if (unshifted) {
          m16 = 0xffffu;
        } else {
          const int L1 = a.W - cx;  // pixels of the K-step left in row cy
          const int cy1 = cy + 1 == a.H ? 0 : cy + 1;  // the next row (of the next image after the last)
          if ((unsigned)(cy + dh) < (unsigned)a.H) m16 |= seg(clo - cx, min(L1, chi - cx));
          if ((unsigned)(cy1 + dh) < (unsigned)a.H) m16 |= seg(L1 + clo, L1 + chi);
        }
        const int left = a.P - ld_ks * kWx6BK;  // none past the last pixel
        if (left < kWx6BK) m16 &= (1u << max(left, 0)) - 1u;
      }
      ++ld_ks;
      if (!unshifted) {
        cx += kWx6BK;
        if (cx >= a.W) {
          cx -= a.W;
          if (++cy == a.H) cy = 0;
        }
      }
      return m16;
    };
    if constexpr (H3) {
      if (a.rowscale) {
        float iv;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = n0 + (tid >> 3) + 32 * i;
          sXr[i] = n < a.N ? pow2_scale(a.bpart[n], iv) : 1.f;
        }
      }
    }
    // per-row element offsets of this thread's four X rows at K-step 0 (+ the tap shift); a row past N
    // gets a sentinel that stays below -4 for every K-step (int32: N * P < 2^29, launch_wgrad)
    int rbase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nr = (tid >> 3) + 32 * i;
      rbase[i] = n0 + nr < a.N ? (n0 + nr) * a.P + 4 * cc + shift : (int)0xC0000000;
    }
    float rbv[16];
    unsigned rmb = 0, rsh = 0;
    // loads the stage's two K-steps (a missing second one is all-masked) into rv: exactly one 16-B load
    // per row, so every stage issues the same number of loads on every path (the compiler's wait
    // counts then keep the loads in flight across the MFMAs, r04).  The border mask is kept in mbo and
    // applied when the values are split (storeB), so nothing waits for the loads here; a run that
    // starts 1-3 pixels before X (row 0, negative shift) is loaded from X's start and shifted into
    // place there (sho: the shift per row, one byte each); one further before is masked whole.
    // the segment's masks from the LDS table (built below, before the prologue) when it fits: two
    // K-steps per 32-bit read at a wave-uniform address; else the scalar cursor
    const bool use_tab = nst + 3 <= kWxMaskTab;
    auto loadB = [&](float (&rv)[16], unsigned& mbo, unsigned& sho) {
      const int ks0 = ld_ks;
      unsigned m32;
      if (use_tab) {
        m32 = *reinterpret_cast<const unsigned*>(mtab + (ks0 - k_a));  // (ks0 - k_a even)
        ld_ks += 2;
      } else {
        const unsigned mk0 = kmask();  // (sequenced: both calls advance the cursor)
        m32 = mk0 | (kmask() << 16);
      }
      const unsigned mb = (m32 >> (4 * cc)) & 0xfu;
      mbo = mb;
      sho = 0;
      // a run that starts before X: only X's row 0 (tile n0 = 0, this thread's first row with
      // tid < 8) at the first K-steps of a negative shift - a wave-uniform test (r05: computed per row
      // and stage, it cost ~20 VALU per stage)
      if (n0 == 0 && ks0 * kWx6BK + shift < 0) {
        const int e0 = rbase[0] + ks0 * kWx6BK;
        sho = e0 < 0 && e0 > -4 ? (unsigned)(-e0) : 0u;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // branch-free (r05: the 64-bit form with nested conditions compiled to exec-mask branches,
        // ~15 instructions per row)
        const int e = rbase[i] + ks0 * kWx6BK;
        const unsigned off = e >= 0 ? (unsigned)e * 4u : (e > -4 ? 0u : OOB);
        union { u32x4 u; float f[4]; } c;
        c.u = __builtin_amdgcn_raw_buffer_load_b128(rB, off, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) rv[4 * i + j] = c.f[j];
      }
    };
    auto storeB = [&](int buf, const float (&rv0)[16], unsigned mbv, unsigned shv) {  // split once, NP 8-B plane quarters
      char* base = smem + buf * STAGEB + wofs;
      float rbv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) rbv[q] = rv0[q];
      if (shv) {  // rows loaded from X's start: element j of the run is element j - sh of the load
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned sh = (shv >> (8 * i)) & 0xffu;
#pragma unroll
          for (int j = 3; j >= 0; --j) {
            float v = 0.f;
#pragma unroll
            for (int k = 0; k < j; ++k) v = (unsigned)(j - k) == sh ? rv0[4 * i + k] : v;
            rbv[4 * i + j] = sh == 0 ? rv0[4 * i + j] : v;
          }
        }
      }
      if (__builtin_amdgcn_ballot_w64(mbv != 0xfu) != 0) {  // (r05: most waves' chunks are all valid)
#pragma unroll
        for (int q = 0; q < 16; ++q) rbv[q] = (mbv >> (q & 3)) & 1u ? rbv[q] : 0.f;
      }
      if constexpr (H1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f16x4 hi;
#pragma unroll
          for (int j = 0; j < 4; ++j) hi[j] = (_Float16)(rbv[4 * i + j] * sXr[i]);
          *reinterpret_cast<f16x4*>(base + i * 32 * 16) = hi;
        }
        return;
      } else if constexpr (H3) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint2 hi, lo;
          split2_mix(rbv[4 * i], rbv[4 * i + 1], sXr[i], hi.x, lo.x);
          split2_mix(rbv[4 * i + 2], rbv[4 * i + 3], sXr[i], hi.y, lo.y);
          char* dst = base + i * 32 * 16;
          *reinterpret_cast<uint2*>(dst) = hi;
          *reinterpret_cast<uint2*>(dst + 2 * RB) = lo;
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf16x4 hi, mid, lo;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = rbv[4 * i + j];
          const __bf16 h = (__bf16)v;
          const float r = v - (float)h;
          const __bf16 m = (__bf16)r;
          hi[j] = h;
          mid[j] = m;
          lo[j] = (__bf16)(r - (float)m);
        }
        char* dst = base + i * 32 * 16;
        *reinterpret_cast<bf16x4*>(dst) = hi;
        *reinterpret_cast<bf16x4*>(dst + 2 * RB) = mid;
        *reinterpret_cast<bf16x4*>(dst + 4 * RB) = lo;
      }
    };
    const unsigned a_voff = (unsigned)((kh * a.lda + m0 + wm + l32) * 16);
    u32x4 A0[TM][NP], A1[TM][NP];
    auto loadA = [&](u32x4 (&A)[TM][NP], int ks) {
#pragma unroll
      for (int ii = 0; ii < TM; ++ii)
#pragma unroll
        for (int q = 0; q < NP; ++q)
          A[ii][q] = __builtin_amdgcn_raw_buffer_load_b128(rA, a_voff + ii * 512,
                                                           (int)((unsigned)(ks * 2 * NP + 2 * q) * a_plane_bytes), 0);
    };
    auto compute = [&](const char* Bs, const u32x4 (&A)[TM][NP]) {
      if constexpr (H1) {
        f16x8 bv[TN];
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
          bv[jj] = *reinterpret_cast<const f16x8*>(Bs + kh * RB + (wn + jj * 32 + l32) * 16);
        mfma_prio<kMfmaPrioWg, 1>();
#pragma unroll
        for (int ii = 0; ii < TM; ++ii) {
          union { u32x4 u; f16x8 h; } c0;
          c0.u = A[ii][0];
#pragma unroll
          for (int jj = 0; jj < TN; ++jj)
            acc[ii][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(c0.h, bv[jj], acc[ii][jj], 0, 0, 0);
        }
        mfma_prio<kMfmaPrioWg, 0>();
        return;
      } else if constexpr (H3) {
        Split2h bv[TN];
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) {
          const char* src = Bs + kh * RB + (wn + jj * 32 + l32) * 16;
          bv[jj].hi = *reinterpret_cast<const f16x8*>(src);
          bv[jj].lo = *reinterpret_cast<const f16x8*>(src + 2 * RB);
        }
        mfma_prio<kMfmaPrioWg, 1>();
#pragma unroll
        for (int ii = 0; ii < TM; ++ii) {
          union { u32x4 u; f16x8 h; } c0, c1;
          c0.u = A[ii][0]; c1.u = A[ii][NP - 1];
          Split2h av;
          av.hi = c0.h; av.lo = c1.h;
#pragma unroll
          for (int jj = 0; jj < TN; ++jj) acc[ii][jj] = mfma_h3(av, bv[jj], acc[ii][jj]);
        }
        mfma_prio<kMfmaPrioWg, 0>();
        return;
      }
      Split3 bv[TN];
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        const char* src = Bs + kh * RB + (wn + jj * 32 + l32) * 16;
        bv[jj].hi = *reinterpret_cast<const bf16x8*>(src);
        bv[jj].mid = *reinterpret_cast<const bf16x8*>(src + 2 * RB);
        bv[jj].lo = *reinterpret_cast<const bf16x8*>(src + 4 * RB);
      }
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) {
        union { u32x4 u; bf16x8 h; } c0, c1, c2;
        c0.u = A[ii][0]; c1.u = A[ii][NP > 1 ? 1 : 0]; c2.u = A[ii][NP - 1];
        Split3 av;
        av.hi = c0.h; av.mid = c1.h; av.lo = c2.h;
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) acc[ii][jj] = mfma_x6(av, bv[jj], acc[ii][jj]);
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __syncthreads();  // the previous segment's LDS reads are complete in every wave
    if (use_tab) {
      // mask of K-step k_a + kc, as kmask computes it (0 past the segment's end, past P or outside the
      // image), one per thread at a time; kc up to nst + 2 (the loads issued past the end)
      for (int kc = tid; kc < nst + 3; kc += blockDim.x) {
        unsigned m16 = 0;
        if (kc < nst) {
          const int ks = k_a + kc;
          if (unshifted) {
            m16 = 0xffffu;
          } else {
            const int p = ks * kWx6BK;
            const int q = p / a.W;
            const int x = p - q * a.W, y = q % a.H;
            const int L1 = a.W - x;
            const int y1 = y + 1 == a.H ? 0 : y + 1;
            if ((unsigned)(y + dh) < (unsigned)a.H) m16 |= seg(clo - x, min(L1, chi - x));
            if ((unsigned)(y1 + dh) < (unsigned)a.H) m16 |= seg(L1 + clo, L1 + chi);
          }
          const int left = a.P - ks * kWx6BK;
          if (left < kWx6BK) m16 &= (1u << max(left, 0)) - 1u;
        }
        mtab[kc] = (unsigned short)m16;
      }
      __syncthreads();
    }
    loadB(rbv, rmb, rsh);
    loadA(A0, k_a);
    storeB(0, rbv, rmb, rsh);
    __syncthreads();
    // Every stage issues the same loads, past the segment's end too (A out of range reads 0, B past
    // the end is masked to 0, an odd segment's last K-step computes with zero B), so each wait
    // leaves the younger loads in flight: A for the next K-step and the next stage's B stay in
    // flight during the MFMAs.  (With the loads conditional, the compiler drained the queue -
    // vmcnt(0) - before every stage's first MFMA, waiting for the B loads just issued, r04.)
    // (r05: A a whole stage ahead in two more register sets was slower - 236 VGPRs, layer4 +15 us.)
    // The prefetch past a tile's last K-step reads up to two K-steps beyond the planes (the K-step
    // rides in the soffset, outside the range check): wgrad_planes_bytes reserves them.
    int ks = k_a;  // the K-step computed next
    for (int s = 0; 2 * s < nst; ++s) {
      const char* Bs = smem + (s & 1) * STAGEB;
      loadA(A1, ks + 1);
      loadB(rbv, rmb, rsh);  // the next stage: in flight during this stage's MFMAs
      __builtin_amdgcn_sched_barrier(0);  // (left to itself the compiler sinks a B load past the MFMAs)
      compute(Bs, A0);
      loadA(A0, ks + 2);
      compute(Bs + KVS, A1);
      ks += 2;
      storeB((s + 1) & 1, rbv, rmb, rsh);
      __syncthreads();
    }
    if (H3 && !a.rowscale) {  // exact: both factors are powers of two (rowscale: in k_wsk_reduce)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * iA * iB;
    }
    // every tile leaves its piece(s) in `part` (k_wsk_reduce<128, 128>, as k_wgrad_sk)
    constexpr int PSZ = BM * BN;
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.part, (short)0, (int)min(0x7fffffffLL, (long long)a.NW * a.slots * PSZ * 4), 0x00020000);
    const int slot = t - it_begin / a.KS;
    const unsigned pbase = (unsigned)((w * a.slots + slot) * PSZ * 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn + j * 32 + l32;
        const int ml = wm + i * 32 + 4 * kh;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                pbase + (unsigned)(((ml + ro) * BN + nl) * 4), 0, 0);
        }
      }
  }
}

}  // namespace msl

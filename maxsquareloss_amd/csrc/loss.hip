// Fused segmentation losses + bilinear upsampling on gfx950 (HBM/VALU-bound).
//
// Replaces, on the hot path of one UDA iteration (solve_gta5.py:178-235):
//   F.interpolate(.., align_corners=True)              deeplab_multi.py:124,128
//   F.softmax(pred, dim=1)                             solve_gta5.py:182-183
//   MaxSquareloss / IW_MaxSquareloss                   utils/loss.py:69-119
//   nn.CrossEntropyLoss(ignore_index=-1)               train_source.py:128
//   multi-level self-produced guidance label + CE      solve_gta5.py:206-213
//
// The losses read the LOW-resolution logits [C][Hi][Wi] (0.6 MB, L2 resident)
// and re-interpolate every hi-res pixel on the fly with torch-CPU's exact
// rounding (t = fma(x0, w0, x1*w1) per axis, width first), so the 40 MB hi-res
// logits are never re-read.  Forward: one pass, per-block partial records,
// deterministic finalize.  Backward: the loss/softmax gradient of a hi-res row
// is formed in LDS and folded straight into the low-res gradient with the
// transposed (separable) interpolation weights: rows -> T[C][Ho][Wi] ->
// d logits[C][Hi][Wi], a fixed-order gather (no atomics).
#include <math.h>
#include <cmath>

#include "msl_internal.h"

// No FMA contraction in this file: torch-CPU rounds s*o before subtracting floor(s*o), and
// the bilinear taps are exact fma(x0, w0, x1*w1) patterns written out explicitly below.
#pragma clang fp contract(off)

namespace msl {

enum LossKind { K_CE = 0, K_MS = 1, K_IW = 2, K_MULTI = 3, K_UPS = 4 };

constexpr int kStats = 64;       // floats in a stats record
constexpr int kFwdBlocks = 1024; // partial records per forward pass
constexpr int kMaxC = 32;

struct Geo {
  int C, Hi, Wi, Ho, Wo;
  float sh, sw;  // align_corners scales (in-1)/(out-1) in fp32, as torch computes them
};

struct Lin {
  int i0, i1;
  float w0, w1;
};

// area_pixel_compute_source_index + guard_index_and_lambda (align_corners=True)
__device__ __forceinline__ Lin lin(int o, float s, int n) {
  const float real = s * (float)o;
  int i0 = (int)floorf(real);
  i0 = min(i0, n - 1);
  const float lam = fminf(fmaxf(real - (float)i0, 0.f), 1.f);
  Lin r;
  r.i0 = i0;
  r.i1 = i0 + (i0 < n - 1 ? 1 : 0);
  r.w0 = 1.f - lam;
  r.w1 = lam;
  return r;
}

__device__ __forceinline__ float bilerp(const float* __restrict__ plane, int Wi, const Lin& ly,
                                        const Lin& lx) {
  const float* r0 = plane + ly.i0 * Wi;
  const float* r1 = plane + ly.i1 * Wi;
  const float t0 = __fmaf_rn(r0[lx.i0], lx.w0, __fmul_rn(r0[lx.i1], lx.w1));
  const float t1 = __fmaf_rn(r1[lx.i0], lx.w0, __fmul_rn(r1[lx.i1], lx.w1));
  return __fmaf_rn(t0, ly.w0, __fmul_rn(t1, ly.w1));
}

template <int CM>
__device__ __forceinline__ void up_logits(const float* __restrict__ L, const Geo& g, const Lin& ly,
                                          const Lin& lx, float (&v)[CM]) {
  const int hw = g.Hi * g.Wi;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < g.C) v[c] = bilerp(L + c * hw, g.Wi, ly, lx);
}

// softmax over C (max, exp(x - max), sequential sum, divide) + first-max argmax of p
template <int CM>
__device__ __forceinline__ void softmax(const float (&v)[CM], int C, float (&p)[CM], float& mx,
                                        float& sum) {
  mx = v[0];
#pragma unroll
  for (int c = 1; c < CM; ++c)
    if (c < C) mx = fmaxf(mx, v[c]);
  sum = 0.f;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) {
      p[c] = expf(v[c] - mx);
      sum += p[c];
    }
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) p[c] = p[c] / sum;
}

template <int CM>
__device__ __forceinline__ int argmax_first(const float (&p)[CM], int C, float& best) {
  best = p[0];
  int a = 0;
#pragma unroll
  for (int c = 1; c < CM; ++c)
    if (c < C && p[c] > best) {
      best = p[c];
      a = c;
    }
  return a;
}

// label2 of the multi-level guidance (solve_gta5.py:207-212)
template <int CM>
__device__ __forceinline__ int multi_label(const float (&P)[CM], const float (&P2)[CM], int C,
                                           float thr) {
  float m1, m2;
  argmax_first(P, C, m1);
  argmax_first(P2, C, m2);
  if (!(m1 > thr || m2 > thr)) return -1;
  float best = (P[0] + P2[0]) / 2.f;
  int a = 0;
#pragma unroll
  for (int c = 1; c < CM; ++c)
    if (c < C) {
      const float pc = (P[c] + P2[c]) / 2.f;
      if (pc > best) {
        best = pc;
        a = c;
      }
    }
  return a;
}

// Block-wide sum of one float (256 threads) -> returned to all threads.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// ---------------------------------------------------------------- forward
// Partial record layout per block (floats):
//   CE / MULTI: [0] = sum of -log p[y], [1] = n_valid
//   MS:         [0] = sum p^2
//   IW:         [0..C) = per-class sum of sum_k p_k^2 (by argmax class), [C..2C) = per-class count
template <int KIND, int CM>
__global__ void __launch_bounds__(256) k_loss_fwd(const float* __restrict__ L1,
                                                   const float* __restrict__ L2,
                                                   const int64_t* __restrict__ labels, Geo g,
                                                   float thr, float* __restrict__ part, int rec) {
  __shared__ float red[4];
  const int npx = g.Ho * g.Wo;
  float a0 = 0.f, a1 = 0.f;
  float cs[CM], cn[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) cs[c] = cn[c] = 0.f;

  for (int px = blockIdx.x * 256 + threadIdx.x; px < npx; px += gridDim.x * 256) {
    const int oy = px / g.Wo, ox = px - oy * g.Wo;
    const Lin ly = lin(oy, g.sh, g.Hi), lx = lin(ox, g.sw, g.Wi);
    float v[CM], p[CM], mx, sum;
    up_logits<CM>(L1, g, ly, lx, v);
    softmax<CM>(v, g.C, p, mx, sum);
    if (KIND == K_CE) {
      const int y = (int)labels[px];
      if (y >= 0 && y < g.C) {
        float vy = v[0];
#pragma unroll
        for (int c = 1; c < CM; ++c)
          if (c == y) vy = v[c];
        a0 += -((vy - mx) - logf(sum));
        a1 += 1.f;
      }
    } else if (KIND == K_MS) {
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < g.C) a0 += p[c] * p[c];
    } else if (KIND == K_IW) {
      float best;
      const int am = argmax_first<CM>(p, g.C, best);
      float s2 = 0.f;
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < g.C) s2 += p[c] * p[c];
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c == am) {
          cs[c] += s2;
          cn[c] += 1.f;
        }
    } else if (KIND == K_MULTI) {
      float v2[CM], P[CM], mx2, sum2;
      up_logits<CM>(L2, g, ly, lx, v2);
      softmax<CM>(v2, g.C, P, mx2, sum2);
      const int y = multi_label<CM>(P, p, g.C, thr);
      if (y >= 0) {
        float vy = v[0];
#pragma unroll
        for (int c = 1; c < CM; ++c)
          if (c == y) vy = v[c];
        a0 += -((vy - mx) - logf(sum));
        a1 += 1.f;
      }
    }
  }
  float* rp = part + (long long)blockIdx.x * rec;
  if (KIND == K_IW) {
    for (int c = 0; c < g.C; ++c) {
      float s = 0.f, n = 0.f;
#pragma unroll
      for (int k = 0; k < CM; ++k)
        if (k == c) {
          s = cs[k];
          n = cn[k];
        }
      s = block_sum(s, red);
      n = block_sum(n, red);
      if (threadIdx.x == 0) {
        rp[c] = s;
        rp[g.C + c] = n;
      }
    }
  } else {
    const float s0 = block_sum(a0, red);
    const float s1 = block_sum(a1, red);
    if (threadIdx.x == 0) {
      rp[0] = s0;
      rp[1] = s1;
    }
  }
}

// Deterministic finalize: one block sums the partial records in fixed order.
// stats: [0] loss, [1] n_valid (CE/MULTI) or H*W (MS/IW), [2..2+C) class weights (IW)
template <int KIND>
__global__ void __launch_bounds__(256) k_loss_finalize(const float* __restrict__ part, int nblk,
                                                        int rec, int C, int npx, float ratio,
                                                        float* __restrict__ out,
                                                        float* __restrict__ stats,
                                                        int32_t* __restrict__ hist,
                                                        float* __restrict__ weights) {
  __shared__ double sred[256];
  const int nvals = KIND == K_IW ? 2 * C : 2;
  __shared__ double vals[2 * kMaxC];
  for (int j = 0; j < nvals; ++j) {
    double s = 0.0;
    for (int b = threadIdx.x; b < nblk; b += 256) s += (double)part[(long long)b * rec + j];
    sred[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) sred[threadIdx.x] += sred[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) vals[j] = sred[0];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  for (int k = 0; k < kStats; ++k) stats[k] = 0.f;
  if (KIND == K_CE || KIND == K_MULTI) {
    const float n = (float)vals[1];
    const float loss = (float)(vals[0] / vals[1]);  // 0/0 -> nan, as the reference (quirk Q8)
    out[0] = loss;
    stats[0] = loss;
    stats[1] = n;
  } else if (KIND == K_MS) {
    const float loss = (float)(-vals[0] / (2.0 * (double)C * (double)npx));
    out[0] = loss;
    stats[0] = loss;
    stats[1] = (float)npx;
  } else if (KIND == K_IW) {
    // weight = 1 / max(hist^r * (sum hist)^(1-r), 1)   (loss.py:95), fp32 as the reference
    float tot = 0.f;
    for (int c = 0; c < C; ++c) tot += (float)vals[C + c];
    const float tp = powf(tot, 1.f - ratio);
    double l = 0.0;
    for (int c = 0; c < C; ++c) {
      const float h = (float)vals[C + c];
      const float w = 1.f / fmaxf(powf(h, ratio) * tp, 1.f);
      stats[2 + c] = w;
      if (weights) weights[c] = w;
      if (hist) hist[c] = (int32_t)vals[C + c];
      l += (double)w * vals[c];
    }
    const float loss = (float)(-l / (double)C);
    out[0] = loss;
    stats[0] = loss;
    stats[1] = (float)npx;
  }
}

// ---------------------------------------------------------------- backward
// Per-pixel hi-res gradient g[c] = dL/d logit_hi[c] for the loss KIND.
struct BwdScal {
  float a;  // CE/MULTI: gout / n_valid ; MS: -gout / (C*H*W) ; IW: -2*gout / C
};

template <int KIND, int CM>
__device__ __forceinline__ void pixel_grad(const float* __restrict__ L1, const float* __restrict__ L2,
                                           const int64_t* __restrict__ labels,
                                           const float* __restrict__ gin_hi, const Geo& g,
                                           const float* __restrict__ stats, float thr, float sc,
                                           int oy, int ox, const Lin& ly, float (&gr)[CM]) {
  if (KIND == K_UPS) {
    const long long hw = (long long)g.Ho * g.Wo;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < g.C) gr[c] = gin_hi[c * hw + (long long)oy * g.Wo + ox];
    return;
  }
  const Lin lx = lin(ox, g.sw, g.Wi);
  float v[CM], p[CM], mx, sum;
  up_logits<CM>(L1, g, ly, lx, v);
  softmax<CM>(v, g.C, p, mx, sum);
  if (KIND == K_CE || KIND == K_MULTI) {
    int y;
    if (KIND == K_CE) {
      y = (int)labels[(long long)oy * g.Wo + ox];
      if (y >= g.C) y = -1;
    } else {
      float v2[CM], P[CM], mx2, sum2;
      up_logits<CM>(L2, g, ly, lx, v2);
      softmax<CM>(v2, g.C, P, mx2, sum2);
      y = multi_label<CM>(P, p, g.C, thr);
    }
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < g.C) gr[c] = y < 0 ? 0.f : sc * (p[c] - (c == y ? 1.f : 0.f));
  } else {
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < g.C) s2 += p[c] * p[c];
    float a = sc;
    if (KIND == K_IW) {
      float best;
      const int am = argmax_first<CM>(p, g.C, best);
      float w = stats[2];
#pragma unroll
      for (int c = 1; c < CM; ++c)
        if (c == am) w = stats[2 + c];
      a = sc * w;
    }
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < g.C) gr[c] = a * p[c] * (p[c] - s2);
  }
}

// first ox with i0(ox) >= t (i0 is monotone in ox), searched in [lo, hi)
__device__ __forceinline__ int lb_ox(int t, int lo, int hi, const Geo& g) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (lin(mid, g.sw, g.Wi).i0 >= t) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// Block (oy, j): hi-res row oy, low-res columns ix in [ixa, ixb) (chunk j of gridDim.y).  The
// pixels that feed those columns, ox with i0(ox) in [ixa - 1, ixb), get their gradient G[c][ox]
// in LDS, then T[c][oy][ix] = sum_ox Wx[ox][ix] G[c][ox] in ascending ox (fp64).  Chunks of ~33
// columns (~280 pixels) instead of a whole row per block: 4x the blocks at a quarter of the LDS,
// so the latency-bound per-pixel softmax has 3-4x the waves in flight (r01: 130 us per loss).
// A pixel on a chunk border is computed by both neighbours: the same value, so T is unchanged.
template <int KIND, int CM>
__global__ void __launch_bounds__(256) k_bwd_rows(const float* __restrict__ L1,
                                                   const float* __restrict__ L2,
                                                   const int64_t* __restrict__ labels,
                                                   const float* __restrict__ gin_hi, Geo g, float thr,
                                                   const float* __restrict__ stats,
                                                   const float* __restrict__ gout,
                                                   float* __restrict__ T, int wmax) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* G = sm;                               // [C][wmax]
  float* wx0 = G + g.C * wmax;                 // [wmax]
  float* wx1 = wx0 + wmax;                     // [wmax]
  int* ix0 = reinterpret_cast<int*>(wx1 + wmax);  // [wmax]

  const int oy = blockIdx.x;
  const int nch = gridDim.y, per = (g.Wi + nch - 1) / nch;
  const int ixa = blockIdx.y * per, ixb = min(g.Wi, ixa + per);
  if (ixa >= ixb) return;
  const int ox_lo = lb_ox(ixa - 1, 0, g.Wo, g);
  const int ox_hi = ixb >= g.Wi ? g.Wo : lb_ox(ixb, ox_lo, g.Wo, g);
  const int nw = ox_hi - ox_lo;  // <= wmax (host bound)
  const Lin ly = lin(oy, g.sh, g.Hi);
  float sc = 0.f;
  if (KIND == K_CE || KIND == K_MULTI) sc = gout[0] / stats[1];
  else if (KIND == K_MS) sc = -gout[0] / ((float)g.C * stats[1]);
  else if (KIND == K_IW) sc = -2.f * gout[0] / (float)g.C;

  for (int k = threadIdx.x; k < nw; k += 256) {
    const int ox = ox_lo + k;
    const Lin lx = lin(ox, g.sw, g.Wi);
    wx0[k] = lx.w0;
    wx1[k] = lx.w1;
    ix0[k] = lx.i0;
    float gr[CM];
    pixel_grad<KIND, CM>(L1, L2, labels, gin_hi, g, stats, thr, sc, oy, ox, ly, gr);
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < g.C) G[c * wmax + k] = gr[c];
  }
  __syncthreads();
  auto bnd = [&](int t) {  // first chunk pixel with i0 >= t (t in [ixa - 1, ixb])
    int lo = 0, hi = nw;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ix0[mid] >= t) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  };
  const long long plane = (long long)g.Ho * g.Wi;
  const int ncol = ixb - ixa;
  for (int e = threadIdx.x; e < g.C * ncol; e += 256) {
    const int c = e / ncol, ix = ixa + (e - c * ncol);
    const int beg = bnd(ix > 0 ? ix - 1 : 0), end = ix + 1 <= g.Wi - 1 ? bnd(ix + 1) : nw;
    const float* Gc = G + c * wmax;
    double s = 0.0;  // ~2*Wo/Wi terms; fp64 keeps the gather at fp32-rounding accuracy
    for (int k = beg; k < end; ++k) {
      const int i0 = ix0[k];
      const int i1 = i0 + (i0 < g.Wi - 1 ? 1 : 0);
      float w = 0.f;
      if (i0 == ix) w += wx0[k];
      if (i1 == ix) w += wx1[k];
      s += (double)w * (double)Gc[k];
    }
    T[c * plane + (long long)oy * g.Wi + ix] = (float)s;
  }
}

// dlow[c][iy][ix] = sum_oy Wy[oy][iy] T[c][oy][ix]
__global__ void __launch_bounds__(256) k_bwd_cols(const float* __restrict__ T, Geo g,
                                                   float* __restrict__ dlow) {
  const int n = g.C * g.Hi * g.Wi;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int ix = e % g.Wi;
    const int r = e / g.Wi;
    const int iy = r % g.Hi;
    const int c = r / g.Hi;
    // oy range: i0(oy) in {iy-1, iy}
    auto lb = [&](int target) {
      int lo = 0, hi = g.Ho;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (lin(mid, g.sh, g.Hi).i0 >= target) hi = mid;
        else lo = mid + 1;
      }
      return lo;
    };
    const int beg = lb(iy > 0 ? iy - 1 : 0), end = lb(iy + 1);
    const float* Tc = T + (long long)c * g.Ho * g.Wi + ix;
    double s = 0.0;
    for (int oy = beg; oy < end; ++oy) {
      const Lin ly = lin(oy, g.sh, g.Hi);
      float w = 0.f;
      if (ly.i0 == iy) w += ly.w0;
      if (ly.i1 == iy) w += ly.w1;
      s += (double)w * (double)Tc[(long long)oy * g.Wi];
    }
    dlow[e] = (float)s;
  }
}

// ---------------------------------------------------------------- upsample forward
__global__ void __launch_bounds__(256) k_upsample_fwd(const float* __restrict__ in, Geo g,
                                                       float* __restrict__ out) {
  const unsigned wq = (g.Wo + 3) / 4;
  const unsigned n = (unsigned)g.C * g.Ho * wq;  // < 2^31 (msl_upsample_fwd checks): 32-bit decode
  const long long hwo = (long long)g.Ho * g.Wo;
  const bool vec = (g.Wo & 3) == 0;
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
    const int q = (int)(e % wq);
    const unsigned r = e / wq;
    const int oy = (int)(r % (unsigned)g.Ho);
    const int c = (int)(r / (unsigned)g.Ho);
    const Lin ly = lin(oy, g.sh, g.Hi);
    const float* plane = in + (long long)c * g.Hi * g.Wi;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int ox = min(q * 4 + k, g.Wo - 1);
      v[k] = bilerp(plane, g.Wi, ly, lin(ox, g.sw, g.Wi));
    }
    float* o = out + (long long)c * hwo + (long long)oy * g.Wo + q * 4;
    if (vec) {
      *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (q * 4 + k < g.Wo) o[k] = v[k];
    }
  }
}

// ---------------------------------------------------------------- prob-input losses
// record: [0] sum p^2 (MS) | IW: [0..C) class sums, [C..2C) class counts
template <int IW, int CM>
__global__ void __launch_bounds__(256) k_prob_fwd(const float* __restrict__ prob,
                                                   const int64_t* __restrict__ label, int C, int hw,
                                                   float* __restrict__ part, int rec) {
  __shared__ float red[4];
  float a0 = 0.f;
  float cs[CM], cn[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) cs[c] = cn[c] = 0.f;
  for (int px = blockIdx.x * 256 + threadIdx.x; px < hw; px += gridDim.x * 256) {
    float p[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) p[c] = prob[(long long)c * hw + px];
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) s2 += p[c] * p[c];
    if (!IW) {
      a0 += s2;
    } else {
      float best;
      const int am = argmax_first<CM>(p, C, best);
      const int lb = label ? (int)label[px] : am;
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c == am) cs[c] += s2;
        if (c == lb) cn[c] += 1.f;
      }
    }
  }
  float* rp = part + (long long)blockIdx.x * rec;
  if (IW) {
    for (int c = 0; c < C; ++c) {
      float s = 0.f, n = 0.f;
#pragma unroll
      for (int k = 0; k < CM; ++k)
        if (k == c) {
          s = cs[k];
          n = cn[k];
        }
      s = block_sum(s, red);
      n = block_sum(n, red);
      if (threadIdx.x == 0) {
        rp[c] = s;
        rp[C + c] = n;
      }
    }
  } else {
    const float s = block_sum(a0, red);
    if (threadIdx.x == 0) rp[0] = s;
  }
}

template <int IW, int CM>
__global__ void __launch_bounds__(256) k_prob_bwd(const float* __restrict__ prob, int C, int hw,
                                                   const float* __restrict__ weights,
                                                   const float* __restrict__ gout,
                                                   float* __restrict__ dprob) {
  const float g = gout[0];
  for (int px = blockIdx.x * 256 + threadIdx.x; px < hw; px += gridDim.x * 256) {
    float p[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) p[c] = prob[(long long)c * hw + px];
    float a;
    if (IW) {
      float best;
      const int am = argmax_first<CM>(p, C, best);
      a = -2.f * g * weights[am] / (float)C;
    } else {
      a = -g / ((float)C * (float)hw);
    }
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) dprob[(long long)c * hw + px] = a * p[c];
  }
}

// ---------------------------------------------------------------- label inspection
// The per-pixel decisions the fused losses take internally, written out: arg[px] = first-max
// argmax of softmax(up(L1)) (the IW histogram's class, loss.py:84-86), label2[px] = the
// multi-level guidance label with P = softmax(up(L2)), P2 = softmax(up(L1)) (solve_gta5.py:
// 206-212; -1 = ignored).  Same device functions as k_loss_fwd / pixel_grad.
template <int CM>
__global__ void __launch_bounds__(256) k_loss_labels(const float* __restrict__ L1,
                                                      const float* __restrict__ L2, Geo g,
                                                      float thr, int32_t* __restrict__ arg,
                                                      int32_t* __restrict__ label2) {
  const int npx = g.Ho * g.Wo;
  for (int px = blockIdx.x * 256 + threadIdx.x; px < npx; px += gridDim.x * 256) {
    const int oy = px / g.Wo, ox = px - oy * g.Wo;
    const Lin ly = lin(oy, g.sh, g.Hi), lx = lin(ox, g.sw, g.Wi);
    float v[CM], p[CM], mx, sum;
    up_logits<CM>(L1, g, ly, lx, v);
    softmax<CM>(v, g.C, p, mx, sum);
    if (arg) {
      float best;
      arg[px] = argmax_first<CM>(p, g.C, best);
    }
    if (label2) {
      float v2[CM], P[CM], mx2, sum2;
      up_logits<CM>(L2, g, ly, lx, v2);
      softmax<CM>(v2, g.C, P, mx2, sum2);
      label2[px] = multi_label<CM>(P, p, g.C, thr);
    }
  }
}

// ---------------------------------------------------------------- host helpers
static bool geo_ok(int c, int hi, int wi, int ho, int wo) {
  return c >= 1 && c <= kMaxC && hi >= 1 && wi >= 1 && ho >= 1 && wo >= 1 &&
         (long long)ho * wo < (1LL << 31);
}

static Geo make_geo(int c, int hi, int wi, int ho, int wo) {
  Geo g;
  g.C = c;
  g.Hi = hi;
  g.Wi = wi;
  g.Ho = ho;
  g.Wo = wo;
  g.sh = ho > 1 ? (float)(hi - 1) / (float)(ho - 1) : 0.f;
  g.sw = wo > 1 ? (float)(wi - 1) / (float)(wo - 1) : 0.f;
  return g;
}

static int rec_len(int C) { return 2 * C > 2 ? 2 * C : 2; }

// partial records + one trailing stats record (used by the prob-input forms)
static size_t part_bytes(int C) {
  return align_up(((size_t)kFwdBlocks * rec_len(C) + kStats) * 4, 256);
}

static size_t t_bytes(int c, int ho, int wi) { return align_up((size_t)c * ho * wi * 4, 256); }

// k_bwd_rows: column chunks per hi-res row, and the widest pixel range a chunk can need: the
// pixels whose i0 is one of the chunk's columns or the one before, at most ceil(1/sw) + 1 per
// column (sw = (Wi-1)/(Wo-1), fp32 as torch computes it), clamped to the row
static int rows_chunks(const Geo& g) { return std::max(1, std::min(8, g.Wi / 32)); }
static int rows_wmax(const Geo& g) {
  const int per = (g.Wi + rows_chunks(g) - 1) / rows_chunks(g);
  if (g.Wi < 2 || !(g.sw > 0.f)) return g.Wo;
  const long long each = (long long)std::ceil(1.0 / (double)g.sw) + 2;
  return (int)std::min<long long>(g.Wo, (per + 1) * each);
}
static size_t rows_lds(const Geo& g) { return (size_t)rows_wmax(g) * (g.C * 4 + 12); }

#define MSL_DISPATCH_C(C, CM, ...)      \
  do {                                  \
    if ((C) == 19) {                    \
      constexpr int CM = 19;            \
      __VA_ARGS__;                      \
    } else if ((C) == 16) {             \
      constexpr int CM = 16;            \
      __VA_ARGS__;                      \
    } else if ((C) == 13) {             \
      constexpr int CM = 13;            \
      __VA_ARGS__;                      \
    } else {                            \
      constexpr int CM = kMaxC;         \
      __VA_ARGS__;                      \
    }                                   \
  } while (0)

template <int KIND>
static int loss_fwd(const float* L1, const float* L2, const int64_t* labels, int c, int hi, int wi,
                    int ho, int wo, float thr, float ratio, float* out, float* stats,
                    int32_t* hist, float* weights, void* ws, size_t ws_bytes, msl_stream_t s) {
  if (!geo_ok(c, hi, wi, ho, wo) || !L1 || !out || !stats) return MSL_ERR_ARG;
  if (ws_bytes < part_bytes(c)) return MSL_ERR_WORKSPACE;
  const Geo g = make_geo(c, hi, wi, ho, wo);
  hipStream_t st = as_stream(s);
  float* part = (float*)ws;
  const int rec = rec_len(c);
  const int nblk = std::min(kFwdBlocks, cdiv((long long)ho * wo, 256));
  MSL_DISPATCH_C(c, CM,
                 MSL_LAUNCH((k_loss_fwd<KIND, CM>), dim3(nblk), dim3(256), 0, st, L1, L2,
                                    labels, g, thr, part, rec));
  MSL_CHECK_LAUNCH();
  MSL_LAUNCH((k_loss_finalize<KIND>), dim3(1), dim3(256), 0, st, part, nblk, rec, c,
                     ho * wo, ratio, out, stats, hist, weights);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

template <int KIND>
static int loss_bwd(const float* L1, const float* L2, const int64_t* labels, const float* gin_hi,
                    int c, int hi, int wi, int ho, int wo, float thr, const float* stats,
                    const float* gout, float* dlow, void* ws, size_t ws_bytes, msl_stream_t s) {
  if (!geo_ok(c, hi, wi, ho, wo) || !dlow) return MSL_ERR_ARG;
  if (ws_bytes < t_bytes(c, ho, wi)) return MSL_ERR_WORKSPACE;
  const Geo g = make_geo(c, hi, wi, ho, wo);
  const size_t lds = rows_lds(g);
  if (lds > 160 * 1024) return MSL_ERR_SHAPE;
  hipStream_t st = as_stream(s);
  float* T = (float*)ws;
  MSL_DISPATCH_C(c, CM, {
    auto kern = k_bwd_rows<KIND, CM>;
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    MSL_LAUNCH(kern, dim3(ho, rows_chunks(g)), dim3(256), lds, st, L1, L2, labels, gin_hi, g, thr,
                       stats, gout, T, rows_wmax(g));
  });
  MSL_CHECK_LAUNCH();
  const int n = c * hi * wi;
  MSL_LAUNCH(k_bwd_cols, dim3(std::min(cdiv(n, 256), 2048)), dim3(256), 0, st,
                     (const float*)T, g, dlow);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

}  // namespace msl

using namespace msl;

extern "C" {

size_t msl_loss_workspace(int c, int hi, int wi, int ho, int wo) {
  if (!geo_ok(c, hi, wi, ho, wo)) return 0;
  return std::max(part_bytes(c), t_bytes(c, ho, wi));
}

int msl_loss_stats_elems(void) { return kStats; }

int msl_upsample_fwd(const float* in, float* out, int c, int hi, int wi, int ho, int wo,
                     msl_stream_t stream) {
  if (c < 1 || hi < 1 || wi < 1 || ho < 1 || wo < 1 || !in || !out || (long long)c * ho * wo >= (1LL << 31))
    return MSL_ERR_ARG;
  const Geo g = make_geo(c, hi, wi, ho, wo);
  const long long n = (long long)c * ho * ((wo + 3) / 4);
  const int blocks = (int)std::min<long long>(cdiv(n, 256), 8192);
  MSL_LAUNCH(k_upsample_fwd, dim3(blocks), dim3(256), 0, as_stream(stream), in, g, out);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

size_t msl_upsample_bwd_workspace(int c, int hi, int wi, int ho, int wo) {
  return t_bytes(c, ho, wi);
}

int msl_upsample_bwd(const float* gout, float* gin, int c, int hi, int wi, int ho, int wo,
                     void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (!gout || c < 1 || c > kMaxC) return MSL_ERR_ARG;
  return loss_bwd<K_UPS>(nullptr, nullptr, nullptr, gout, c, hi, wi, ho, wo, 0.f, nullptr,
                         nullptr, gin, ws, ws_bytes, stream);
}

int msl_ce_up_fwd(const float* logits, const int64_t* labels, int c, int hi, int wi, int ho,
                  int wo, float* out, float* stats, void* ws, size_t ws_bytes,
                  msl_stream_t stream) {
  if (!labels) return MSL_ERR_ARG;
  return loss_fwd<K_CE>(logits, nullptr, labels, c, hi, wi, ho, wo, 0.f, 0.f, out, stats, nullptr,
                        nullptr, ws, ws_bytes, stream);
}

int msl_ce_up_bwd(const float* logits, const int64_t* labels, int c, int hi, int wi, int ho,
                  int wo, const float* stats, const float* gout, float* dlogits, void* ws,
                  size_t ws_bytes, msl_stream_t stream) {
  if (!logits || !labels || !stats || !gout) return MSL_ERR_ARG;
  return loss_bwd<K_CE>(logits, nullptr, labels, nullptr, c, hi, wi, ho, wo, 0.f, stats, gout,
                        dlogits, ws, ws_bytes, stream);
}

int msl_maxsquare_up_fwd(const float* logits, int c, int hi, int wi, int ho, int wo, float* out,
                         float* stats, void* ws, size_t ws_bytes, msl_stream_t stream) {
  return loss_fwd<K_MS>(logits, nullptr, nullptr, c, hi, wi, ho, wo, 0.f, 0.f, out, stats,
                        nullptr, nullptr, ws, ws_bytes, stream);
}

int msl_maxsquare_up_bwd(const float* logits, int c, int hi, int wi, int ho, int wo,
                         const float* stats, const float* gout, float* dlogits, void* ws,
                         size_t ws_bytes, msl_stream_t stream) {
  if (!logits || !stats || !gout) return MSL_ERR_ARG;
  return loss_bwd<K_MS>(logits, nullptr, nullptr, nullptr, c, hi, wi, ho, wo, 0.f, stats, gout,
                        dlogits, ws, ws_bytes, stream);
}

int msl_iw_maxsquare_up_fwd(const float* logits, int c, int hi, int wi, int ho, int wo,
                            float ratio, float* out, float* stats, int32_t* hist,
                            float* weights, void* ws, size_t ws_bytes, msl_stream_t stream) {
  return loss_fwd<K_IW>(logits, nullptr, nullptr, c, hi, wi, ho, wo, 0.f, ratio, out, stats, hist,
                        weights, ws, ws_bytes, stream);
}

int msl_iw_maxsquare_up_bwd(const float* logits, int c, int hi, int wi, int ho, int wo,
                            const float* stats, const float* gout, float* dlogits, void* ws,
                            size_t ws_bytes, msl_stream_t stream) {
  if (!logits || !stats || !gout) return MSL_ERR_ARG;
  return loss_bwd<K_IW>(logits, nullptr, nullptr, nullptr, c, hi, wi, ho, wo, 0.f, stats, gout,
                        dlogits, ws, ws_bytes, stream);
}

int msl_multi_ce_up_fwd(const float* logits1, const float* logits2, int c, int hi, int wi,
                        int ho, int wo, float thr, float* out, float* stats, void* ws,
                        size_t ws_bytes, msl_stream_t stream) {
  if (!logits2) return MSL_ERR_ARG;
  return loss_fwd<K_MULTI>(logits1, logits2, nullptr, c, hi, wi, ho, wo, thr, 0.f, out, stats,
                           nullptr, nullptr, ws, ws_bytes, stream);
}

int msl_multi_ce_up_bwd(const float* logits1, const float* logits2, int c, int hi, int wi,
                        int ho, int wo, float thr, const float* stats, const float* gout,
                        float* dlogits1, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (!logits1 || !logits2 || !stats || !gout) return MSL_ERR_ARG;
  return loss_bwd<K_MULTI>(logits1, logits2, nullptr, nullptr, c, hi, wi, ho, wo, thr, stats,
                           gout, dlogits1, ws, ws_bytes, stream);
}

int msl_loss_labels_up(const float* logits1, const float* logits2, int c, int hi, int wi, int ho,
                       int wo, float thr, int32_t* argmax1, int32_t* label2, msl_stream_t stream) {
  if (!geo_ok(c, hi, wi, ho, wo) || !logits1 || (label2 && !logits2)) return MSL_ERR_ARG;
  if (!argmax1 && !label2) return MSL_OK;
  const Geo g = make_geo(c, hi, wi, ho, wo);
  const int nblk = std::min(4096, cdiv((long long)ho * wo, 256));
  MSL_DISPATCH_C(c, CM,
                 MSL_LAUNCH((k_loss_labels<CM>), dim3(nblk), dim3(256), 0, as_stream(stream),
                                    logits1, logits2, g, thr, argmax1, label2));
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_maxsquare_prob_fwd(const float* prob, int c, int hw, float* out, void* ws,
                           size_t ws_bytes, msl_stream_t stream) {
  if (!prob || !out || c < 1 || c > kMaxC || hw < 1) return MSL_ERR_ARG;
  if (ws_bytes < part_bytes(c)) return MSL_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  const int nblk = std::min(kFwdBlocks, cdiv(hw, 256));
  const int rec = rec_len(c);
  float* part = (float*)ws;
  MSL_DISPATCH_C(c, CM,
                 MSL_LAUNCH((k_prob_fwd<0, CM>), dim3(nblk), dim3(256), 0, st, prob,
                                    (const int64_t*)nullptr, c, hw, part, rec));
  MSL_CHECK_LAUNCH();
  // MS finalize: -sum / (2*C*hw); stats scratch lives after the partials
  float* stats = part + (size_t)nblk * rec;
  MSL_LAUNCH((k_loss_finalize<K_MS>), dim3(1), dim3(256), 0, st, (const float*)part, nblk,
                     rec, c, hw, 0.f, out, stats, (int32_t*)nullptr, (float*)nullptr);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_maxsquare_prob_bwd(const float* prob, int c, int hw, const float* gout, float* dprob,
                           msl_stream_t stream) {
  if (!prob || !gout || !dprob || c < 1 || c > kMaxC || hw < 1) return MSL_ERR_ARG;
  MSL_DISPATCH_C(c, CM,
                 MSL_LAUNCH((k_prob_bwd<0, CM>), dim3(std::min(cdiv(hw, 256), 4096)),
                                    dim3(256), 0, as_stream(stream), prob, c, hw,
                                    (const float*)nullptr, gout, dprob));
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_iw_maxsquare_prob_fwd(const float* prob, const int64_t* label, int c, int hw,
                              float ratio, float* out, int32_t* hist, float* weights, void* ws,
                              size_t ws_bytes, msl_stream_t stream) {
  if (!prob || !out || !weights || c < 1 || c > kMaxC || hw < 1) return MSL_ERR_ARG;
  if (ws_bytes < part_bytes(c)) return MSL_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  const int nblk = std::min(kFwdBlocks, cdiv(hw, 256));
  const int rec = rec_len(c);
  float* part = (float*)ws;
  MSL_DISPATCH_C(c, CM,
                 MSL_LAUNCH((k_prob_fwd<1, CM>), dim3(nblk), dim3(256), 0, st, prob, label,
                                    c, hw, part, rec));
  MSL_CHECK_LAUNCH();
  float* stats = part + (size_t)nblk * rec;
  MSL_LAUNCH((k_loss_finalize<K_IW>), dim3(1), dim3(256), 0, st, (const float*)part, nblk,
                     rec, c, hw, ratio, out, stats, hist, weights);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_iw_maxsquare_prob_bwd(const float* prob, int c, int hw, const float* weights,
                              const float* gout, float* dprob, msl_stream_t stream) {
  if (!prob || !weights || !gout || !dprob || c < 1 || c > kMaxC || hw < 1) return MSL_ERR_ARG;
  MSL_DISPATCH_C(c, CM,
                 MSL_LAUNCH((k_prob_bwd<1, CM>), dim3(std::min(cdiv(hw, 256), 4096)),
                                    dim3(256), 0, as_stream(stream), prob, c, hw, weights, gout,
                                    dprob));
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

}  // extern "C"

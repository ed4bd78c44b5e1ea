// BatchNorm2d (train / eval) fused with the ReLU and residual-add of the Bottleneck
// (deeplab_multi.py:14-46, 75-79, 101): y = act(bn(x) [+ residual]), act = ReLU or identity.
//
// The reference runs BN in train mode at bs=1: statistics over one image's
// H*W pixels per channel.  MIOpen's train-mode BN uses a single-pass E[x^2]-E[x]^2 variance
// whose fp32 cancellation (1e-4 relative on a mean/std ~ 1/3 channel) compounds over the 104
// BN layers into O(1) logit differences; torch-CPU uses two passes.  Here each channel's
// statistics are accumulated in fp64 around a per-channel shift (its first element), which
// is at least as accurate as the CPU's two-pass fp32 sums.
//
// Layout [C][NI][P]: NI images (bs = 1 each: every image gets its own batch statistics, as the
// reference's separate source and target forwards do), P pixels per image; row r = c*NI + n holds
// channel c of image n.  Running statistics are updated image by image in order (n = 0 first),
// dgamma / dbeta summed image by image in order.  Train mode on layer1-4 maps: one fused launch per call (see
// k_bn_fwd_fused).  Otherwise: forward: stats kernel (grid C x S partial fp64 sums per channel) +
// a flat apply kernel over the whole tensor in float4s (each block folds the partials of the
// channels it touches).  Backward: per-channel reduce (sum g, sum g*xhat with g = dy masked by
// y > 0 when ReLU) + flat apply (dx, d residual, dgamma, dbeta).  HBM-bound: fwd reads x twice,
// writes y (+ reads the residual); bwd reads dy, x, y twice, writes dx (+ dres).
#include "msl_internal.h"

namespace msl {

constexpr int kBnMaxSplit = 16;
constexpr int kBnChunk = 8192;  // pixels per statistics block

static int bn_splits(int P) { return std::max(1, std::min(kBnMaxSplit, cdiv(P, kBnChunk))); }

// Elements per block of the flat (channel-crossing) apply kernels: a multiple of 4 small enough
// that a block touches at most 256 channels (their coefficients are staged in LDS).
static int bn_flat_chunk(int P) {
  int ch = 4096;
  while (ch > 4 && ch / P + 2 > 256) ch /= 2;
  return ch;
}

__device__ __forceinline__ void block_sum2_d(double& a, double& b, double* red) {
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  a = (red[0] + red[2]) + (red[4] + red[6]);
  b = (red[1] + red[3]) + (red[5] + red[7]);
}

// Visit elements [e0, e1) of a flat array: a 16-B-aligned float4 body shared over the block's
// threads plus a scalar head and tail (< 4 elements each).  f(e, v...) gets the element index.
template <bool VEC, typename F4, typename F1>
__device__ __forceinline__ void visit_range(long long e0, long long e1, F4&& f4, F1&& f1) {
  long long a0 = VEC ? ((e0 + 3) & ~3LL) : e1;
  long long a1 = VEC ? (e1 & ~3LL) : e1;
  if (a0 > a1) a0 = a1 = e1;
  for (long long e = e0 + threadIdx.x; e < a0; e += 256) f1(e);
  for (long long i = a0 / 4 + threadIdx.x; i < a1 / 4; i += 256) f4(i);
  for (long long e = a1 + threadIdx.x; e < e1; e += 256) f1(e);
}

// zero_am (the flat apply's absmax output, or null): zeroed here, one launch ahead of its atomicMax
template <bool VEC>
__global__ void __launch_bounds__(256) k_bn_stats(const float* __restrict__ x, int P, int S,
                                                   double* __restrict__ part, float* __restrict__ zero_am = nullptr,
                                                   int NI = 1) {
  __shared__ double red[8];
  const int c = blockIdx.x, s = blockIdx.y;
  if (zero_am && s == 0 && threadIdx.x == 0 && c % NI == 0) zero_am[c / NI] = 0.f;
  const long long base = (long long)c * P;
  const double shift = (double)x[base];
  const int chunk = cdiv(P, S);
  const int beg = s * chunk, end = min(P, beg + chunk);
  double s1 = 0.0, s2 = 0.0;
  auto acc = [&](float v) {
    const double d = (double)v - shift;
    s1 += d;
    s2 += d * d;
  };
  visit_range<VEC>(
      base + beg, base + end,
      [&](long long i) {
        const float4 v = reinterpret_cast<const float4*>(x)[i];
        acc(v.x); acc(v.y); acc(v.z); acc(v.w);
      },
      [&](long long e) { acc(x[e]); });
  block_sum2_d(s1, s2, red);
  if (threadIdx.x == 0) {
    part[((long long)c * S + s) * 2] = s1;
    part[((long long)c * S + s) * 2 + 1] = s2;
  }
}

struct BnArgs {
  const float* x;
  const float* gamma;
  const float* beta;
  const float* residual;
  float* y;
  float* running_mean;
  float* running_var;
  float* save_mean;
  float* save_invstd;
  long long* num_batches;
  const double* part;
  int C, NI, P, S, chunk, relu, training, update_running;  // C channels, NI images, P pixels per image
  float eps, momentum;
  float* absmax;  // [C] max |y| per channel (msl_bn_fwd_am: the next conv's f16x3 partials) or null
  unsigned long long* mask;  // msl_bn_fwd_mask: y > 0 as bits, [row][cdiv(P, 64)] words (fused form) or null
};

// Batch statistics of row r (channel r / NI of image r % NI) from the fp64 partial sums.
__device__ __forceinline__ void bn_row_stats(const BnArgs& a, int r, float& mean, float& invstd, double& var) {
  double s1 = 0.0, s2 = 0.0;
  for (int s = 0; s < a.S; ++s) {
    s1 += a.part[((long long)r * a.S + s) * 2];
    s2 += a.part[((long long)r * a.S + s) * 2 + 1];
  }
  const double n = (double)a.P;
  const double shift = (double)a.x[(long long)r * a.P];
  const double dm = s1 / n;
  var = s2 / n - dm * dm;
  if (var < 0.0) var = 0.0;
  mean = (float)(shift + dm);
  invstd = (float)(1.0 / sqrt(var + (double)a.eps));
}

// (1 - m) * old + m * v with every operation rounded on its own: whether the compiler contracts
// this into an fma depended on the kernel around it, so the pair, per-image and split forms rounded
// the running statistics differently (r03: the pair form's running_var 1 ulp off the per-image loop;
// r05: a two-image form's running_mean up to 4 ulps).  HIP's __fmul_rn / __fadd_rn are the plain
// operators (without OCML_BASIC_ROUNDED_OPERATIONS), which hipcc's -ffp-contract=fast may fuse; under
// contract(off) these operations carry no contract flag.
__device__ __forceinline__ float running_blend(float old, float m, float v) {
#pragma clang fp contract(off)
  return (1.f - m) * old + m * v;
}

// running statistics of channel c <- image n's batch statistics (one image after the other)
__device__ __forceinline__ void bn_running_update(const BnArgs& a, int c, float mean, double var) {
  const double n = (double)a.P;
  const float m = a.momentum;
  const float unbiased = (float)(a.P > 1 ? var * n / (n - 1.0) : var);
  a.running_mean[c] = running_blend(a.running_mean[c], m, mean);
  a.running_var[c] = running_blend(a.running_var[c], m, unbiased);
}

// The flat apply kernels' absmax output (r05): each thread keeps the max |v| of the row it is in (its
// elements come in increasing order, so the row only advances) and folds it into the block's per-row
// LDS maxima when the row changes; the block then folds those into absmax[channel] with an integer
// atomicMax on the float bits (|v| >= 0 orders as its bits; zeroed by the launch before).  Replaces a
// pass of its own over the output (absmax_rows) for the next conv's f16x3 / fp16 operand scale.
struct RowMax {
  int k = -1;
  float m = 0.f;
  __device__ __forceinline__ void add(unsigned* lds, int row, float v) {
    if (row != k) {
      flush(lds);
      k = row;
      m = 0.f;
    }
    m = fmaxf(m, fabsf(v));
  }
  __device__ __forceinline__ void flush(unsigned* lds) {
    if (k >= 0) atomicMax(lds + k, __float_as_uint(m));
  }
};

// Flat apply: block b covers elements [b*chunk, (b+1)*chunk) of the [C*NI][P] tensor (possibly
// several rows).  Each block derives the (alpha, beta') of the rows it touches from the fp64
// partial sums; the block holding a row's first element also publishes its saved statistics, and
// the one holding a channel's first row (image 0) updates its running statistics image by image.
template <bool VEC>
__global__ void __launch_bounds__(256) k_bn_apply(BnArgs a) {
  __shared__ float coef[2][256];
  __shared__ unsigned rmax[256];
  const long long N = (long long)a.C * a.NI * a.P;
  const long long start = (long long)blockIdx.x * a.chunk;
  const long long end = min(N, start + a.chunk);
  const int c0 = (int)(start / a.P);
  const int nch = (int)((end - 1) / a.P) - c0 + 1;
  if ((int)threadIdx.x < nch) {
    rmax[threadIdx.x] = 0u;
    const int r = c0 + threadIdx.x;  // row = (channel, image)
    const int c = r / a.NI;
    const bool owner = (long long)r * a.P >= start;  // this block holds the row's first element
    float mean, invstd;
    if (a.training) {
      double var;
      bn_row_stats(a, r, mean, invstd, var);
      if (owner && a.update_running && r % a.NI == 0) {
        for (int n = 0; n < a.NI; ++n) {
          float mn, is;
          double vn;
          bn_row_stats(a, r + n, mn, is, vn);
          bn_running_update(a, c, mn, vn);
        }
        if (c == 0 && a.num_batches) a.num_batches[0] += a.NI;
      }
    } else {
      mean = a.running_mean[c];
      invstd = 1.f / sqrtf(a.running_var[c] + a.eps);
    }
    if (owner) {
      a.save_mean[r] = mean;
      a.save_invstd[r] = invstd;
    }
    // y = x * alpha + beta'  (batch_norm_cpu_transform_input form)
    const float alpha = invstd * (a.gamma ? a.gamma[c] : 1.f);
    coef[0][threadIdx.x] = alpha;
    coef[1][threadIdx.x] = (a.beta ? a.beta[c] : 0.f) - mean * alpha;
  }
  __syncthreads();
  const long long cbound = (long long)(c0 + 1) * a.P;  // first element of channel c0+1
  RowMax rm;
  auto one = [&](long long e, float xv, float rv) {
    int k = 0;
    if (e >= cbound) k = (int)(e / a.P) - c0;
    float v = xv * coef[0][k] + coef[1][k];
    v += rv;
    v = a.relu ? fmaxf(v, 0.f) : v;
    if (a.absmax) rm.add(rmax, k, v);
    return v;
  };
  visit_range<VEC>(
      start, end,
      [&](long long i) {
        const float4 xv = reinterpret_cast<const float4*>(a.x)[i];
        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.residual) rv = reinterpret_cast<const float4*>(a.residual)[i];
        const long long e = 4 * i;
        float4 o;
        o.x = one(e, xv.x, rv.x);
        o.y = one(e + 1, xv.y, rv.y);
        o.z = one(e + 2, xv.z, rv.z);
        o.w = one(e + 3, xv.w, rv.w);
        reinterpret_cast<float4*>(a.y)[i] = o;
      },
      [&](long long e) { a.y[e] = one(e, a.x[e], a.residual ? a.residual[e] : 0.f); });
  if (a.absmax) {
    rm.flush(rmax);
    __syncthreads();
    if ((int)threadIdx.x < nch) atomicMax(reinterpret_cast<unsigned*>(a.absmax) + (c0 + threadIdx.x) / a.NI, rmax[threadIdx.x]);
  }
}

struct BnBwdArgs {
  const float* dy;
  const float* x;
  const float* y;  // output (for the ReLU mask) or null
  const float* gamma;
  const float* beta;  // fused form with relu and y = null: the mask recomputed from x (no residual)
  const float* save_mean;
  const float* save_invstd;
  float* dx;
  float* dres;
  float* dgamma;
  float* dbeta;
  double* part;
  int C, NI, P, S, chunk, relu, training, accumulate;
  float* absmax;  // [C] max |dx| per channel (msl_bn_bwd_am) or null
  const unsigned long long* mask;  // msl_bn_bwd_mask: the forward's y > 0 bits (fused form) instead of y
};

template <bool VEC>
__global__ void __launch_bounds__(256) k_bn_bwd_reduce(BnBwdArgs a) {
  __shared__ double red[8];
  const int c = blockIdx.x, s = blockIdx.y;
  // (c: the row; the apply launch after this one folds max |dx| into absmax[row / NI])
  if (a.absmax && s == 0 && threadIdx.x == 0 && c % a.NI == 0) a.absmax[c / a.NI] = 0.f;
  const long long base = (long long)c * a.P;
  const float mean = a.save_mean[c], invstd = a.save_invstd[c];
  const int chunk = cdiv(a.P, a.S);
  const int beg = s * chunk, end = min(a.P, beg + chunk);
  double sg = 0.0, sgx = 0.0;
  auto acc = [&](float g, float yv, float xv) {
    if (a.relu && !(yv > 0.f)) g = 0.f;
    const float xh = (xv - mean) * invstd;
    sg += (double)g;
    sgx += (double)g * (double)xh;
  };
  visit_range<VEC>(
      base + beg, base + end,
      [&](long long i) {
        const float4 g = reinterpret_cast<const float4*>(a.dy)[i];
        const float4 xv = reinterpret_cast<const float4*>(a.x)[i];
        float4 yv = make_float4(1.f, 1.f, 1.f, 1.f);
        if (a.relu) yv = reinterpret_cast<const float4*>(a.y)[i];
        acc(g.x, yv.x, xv.x); acc(g.y, yv.y, xv.y); acc(g.z, yv.z, xv.z); acc(g.w, yv.w, xv.w);
      },
      [&](long long e) { acc(a.dy[e], a.relu ? a.y[e] : 1.f, a.x[e]); });
  block_sum2_d(sg, sgx, red);
  if (threadIdx.x == 0) {
    a.part[((long long)c * a.S + s) * 2] = sg;
    a.part[((long long)c * a.S + s) * 2 + 1] = sgx;
  }
}

template <bool VEC>
__global__ void __launch_bounds__(256) k_bn_bwd_apply(BnBwdArgs a) {
  __shared__ float coef[5][256];
  __shared__ unsigned rmax[256];
  const long long N = (long long)a.C * a.NI * a.P;
  const long long start = (long long)blockIdx.x * a.chunk;
  const long long end = min(N, start + a.chunk);
  const int c0 = (int)(start / a.P);
  const int nch = (int)((end - 1) / a.P) - c0 + 1;
  auto sums = [&](int r, double& sg, double& sgx) {
    sg = sgx = 0.0;
    for (int s = 0; s < a.S; ++s) {
      sg += a.part[((long long)r * a.S + s) * 2];
      sgx += a.part[((long long)r * a.S + s) * 2 + 1];
    }
  };
  if ((int)threadIdx.x < nch) {
    rmax[threadIdx.x] = 0u;
    const int r = c0 + threadIdx.x;  // row = (channel, image)
    const int c = r / a.NI;
    double sg, sgx;
    sums(r, sg, sgx);
    if ((long long)r * a.P >= start && r % a.NI == 0) {  // the channel's parameter gradients, image by image
      float dg = sgx, db = sg;
      if (a.accumulate) {
        dg = a.dgamma ? a.dgamma[c] + (float)sgx : 0.f;
        db = a.dbeta ? a.dbeta[c] + (float)sg : 0.f;
      }
      for (int n = 1; n < a.NI; ++n) {
        double g1, g2;
        sums(r + n, g1, g2);
        dg += (float)g2;
        db += (float)g1;
      }
      if (a.dgamma) a.dgamma[c] = dg;
      if (a.dbeta) a.dbeta[c] = db;
    }
    const float w = a.gamma ? a.gamma[c] : 1.f;
    coef[0][threadIdx.x] = a.save_invstd[r] * w;  // invstd * gamma
    coef[1][threadIdx.x] = a.training ? (float)(sg / (double)a.P) : 0.f;
    coef[2][threadIdx.x] = a.training ? (float)(sgx / (double)a.P) : 0.f;
    coef[3][threadIdx.x] = a.save_mean[r];
    coef[4][threadIdx.x] = a.save_invstd[r];
  }
  __syncthreads();
  const long long cbound = (long long)(c0 + 1) * a.P;
  RowMax rm;
  // returns the masked upstream gradient g; dx through the reference's formula
  auto one = [&](long long e, float g, float yv, float xv, float& dxv) {
    int k = 0;
    if (e >= cbound) k = (int)(e / a.P) - c0;
    if (a.relu && !(yv > 0.f)) g = 0.f;
    const float xh = (xv - coef[3][k]) * coef[4][k];
    dxv = (g - coef[1][k] - xh * coef[2][k]) * coef[0][k];
    if (a.absmax) rm.add(rmax, k, dxv);
    return g;
  };
  visit_range<VEC>(
      start, end,
      [&](long long i) {
        const float4 g = reinterpret_cast<const float4*>(a.dy)[i];
        const float4 xv = reinterpret_cast<const float4*>(a.x)[i];
        float4 yv = make_float4(1.f, 1.f, 1.f, 1.f);
        if (a.relu) yv = reinterpret_cast<const float4*>(a.y)[i];
        const long long e = 4 * i;
        float4 gm, d;
        gm.x = one(e, g.x, yv.x, xv.x, d.x);
        gm.y = one(e + 1, g.y, yv.y, xv.y, d.y);
        gm.z = one(e + 2, g.z, yv.z, xv.z, d.z);
        gm.w = one(e + 3, g.w, yv.w, xv.w, d.w);
        if (a.dres) reinterpret_cast<float4*>(a.dres)[i] = gm;
        if (a.dx) reinterpret_cast<float4*>(a.dx)[i] = d;
      },
      [&](long long e) {
        float d;
        const float gm = one(e, a.dy[e], a.relu ? a.y[e] : 1.f, a.x[e], d);
        if (a.dres) a.dres[e] = gm;
        if (a.dx) a.dx[e] = d;
      });
  if (a.absmax) {
    rm.flush(rmax);
    __syncthreads();
    if ((int)threadIdx.x < nch) atomicMax(reinterpret_cast<unsigned*>(a.absmax) + (c0 + threadIdx.x) / a.NI, rmax[threadIdx.x]);
  }
}

// ---------------------------------------------------------------- fused one-block-per-channel form
// Train mode on maps of <= 16384 px (layers 2-4 at every BASELINE crop), or <= 33792 px with
// >= 128 channels (layer1's 256-channel maps at 1024x512): one 1024-thread block
// per channel keeps the channel's operands in registers (EPT elements per lane, lane-strided so
// every wave load is 256 contiguous bytes), reduces the fp64 sums in the block and applies in the
// same launch.  Forward: x (+ residual) read once, y written once — 2 (3) tensor passes instead
// of 3 (4) and one launch instead of two.  Backward: dy, x, y read once, dx (+ dres) written —
// 4 (5) passes instead of 7 (8).  Same per-element formulas as the flat kernels above.
constexpr int kBnFusedThreads = 1024;

// max over the block (kBnFusedThreads threads) of m, valid in thread 0
__device__ __forceinline__ float block_max16(float m, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < kBnFusedThreads / 64; ++i) r = fmaxf(r, red[i]);
  return r;
}

// absmax[c] = max |t[c][p]| over the channel (the split BN forms' absmax output; absmax zeroed
// beforehand): block (c, s) reduces 4096 elements of channel c (16 per thread, all loads in
// flight) and folds them in with an integer atomicMax on the float bits (|t| >= 0 orders as its
// bits).  One block per channel took 31 us for a 64-channel 33k-px map: 64 blocks.
constexpr int kAbsChunk = 4096;
__global__ void __launch_bounds__(256) k_absmax_rows(const float* __restrict__ t, int P, float* __restrict__ absmax) {
  __shared__ float red[4];
  const float* row = t + (long long)blockIdx.x * P;
  const int beg = blockIdx.y * kAbsChunk;
  float v[kAbsChunk / 256];
#pragma unroll
  for (int i = 0; i < kAbsChunk / 256; ++i) {
    const int e = beg + i * 256 + threadIdx.x;
    v[i] = e < P ? fabsf(row[e]) : 0.f;
  }
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < kAbsChunk / 256; ++i) m = fmaxf(m, v[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned*>(absmax) + blockIdx.x,
              __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

__global__ void __launch_bounds__(256) k_zero_rows(float* __restrict__ v, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = 0.f;
}

// The maxima are zeroed by a kernel, not hipMemsetAsync: inside a captured hipGraph (utils/graph.py)
// the memset node was not ordered against the atomicMax kernel that follows it - replays left stale
// or garbage maxima (up to 1e38) in the partials, i.e. wrong f16x3 operand scales (r03 pair-mode
// graph test).  Kernel nodes keep the stream order.
int absmax_rows(const float* t, int c, int p, float* absmax, hipStream_t st) {
  MSL_LAUNCH(k_zero_rows, dim3(cdiv(c, 256)), dim3(256), 0, st, absmax, c);
  MSL_CHECK_LAUNCH();
  MSL_LAUNCH(k_absmax_rows, dim3(c, cdiv(p, kAbsChunk)), dim3(256), 0, st, t, p, absmax);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}
constexpr int kBnRemaskMaxEpt = 16;  // msl_bn_bwd_am_beta's y = NULL: p <= 16 * 1024
constexpr int kBnFusedMaxP = 33 * kBnFusedThreads;  // layer1 at 1024x512: 257x129 = 33153 px
// forms.bn_fused (msl_forms, per call): the fused kernels where bn_fused_shape allows them
static bool bn_fused_enabled(const msl_forms* forms) { return forms_of(forms).bn_fused != 0; }
// beyond 16 elements per lane only with >= 128 channels: at 64 blocks (layer1's 64-channel
// maps) the split kernels' wider grids win the backward (profiles/r01_bn_forms.txt)
static bool bn_fused_shape(int c, int p) {
  return p <= 16 * kBnFusedThreads || (c >= 128 && p <= kBnFusedMaxP);
}

__device__ __forceinline__ void block_sum2_d16(double& a, double& b, double* red) {
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  a = 0.0;
  b = 0.0;
#pragma unroll
  for (int i = 0; i < kBnFusedThreads / 64; ++i) {  // fixed order: deterministic
    a += red[2 * i];
    b += red[2 * i + 1];
  }
}

// Row accesses of the fused kernels as buffer instructions: one 32-bit lane offset (t * 4) plus the
// element block j in the scalar offset, so the EPT loads and stores of a lane share one address VGPR
// (flat addressing held a 64-bit pointer per j: 80-103 VGPRs, one 1024-thread block per CU).  Lanes
// past the row are masked by the callers (no access is out of range).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bn_row(const float* p, int n) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, n * 4, 0x00020000);
}
__device__ __forceinline__ float bn_ld(__amdgpu_buffer_rsrc_t r, unsigned voff, int j) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, j * kBnFusedThreads * 4, 0));
}
__device__ __forceinline__ void bn_st(__amdgpu_buffer_rsrc_t r, unsigned voff, int j, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, j * kBnFusedThreads * 4, 0);
}
// r06: element block j's offset in the lane's VGPR offset (v + j * 4 KB), not in the scalar offset: the buffer range
// check covers the VGPR and immediate offsets only, so with the block offset there a lane past the row reads 0 and
// its store is dropped by the hardware - no per-element range test (and no branch) around the access
// (the add is an opaque asm statement, so each access computes its offset next to itself: as a plain add the
// compiler kept the EPT offsets live from the loads to the stores - 16 more VGPRs at EPT 16).  The backward's
// forms from kBnVoffMinEpt elements on (EPT 16: 14 -> 8 spilled VGPRs, 43 -> 8 SGPRs; EPT 33: 46 SGPRs -> none);
// the smaller ones keep the scalar block offset and explicit range tests, which they hold without spilling
__device__ __forceinline__ unsigned bn_voff(unsigned voff, int j) {
  if (j == 0) return voff;
  unsigned r;
  asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "i"(j * kBnFusedThreads * 4), "v"(voff));
  return r;
}
__device__ __forceinline__ float bn_ldv(__amdgpu_buffer_rsrc_t r, unsigned voff, int j) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, bn_voff(voff, j), 0, 0));
}
__device__ __forceinline__ void bn_stv(__amdgpu_buffer_rsrc_t r, unsigned voff, int j, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, bn_voff(voff, j), 0, 0);
}
constexpr int kBnVoffMinEpt = 16;
constexpr bool kBnOpaqueAll = false;  // the opaque thread index in the smaller forms too
constexpr int kBnTwoBlockEpt = 16;  // forms built for two blocks per CU (64 VGPRs)

// N fp64 sums over the block, each in block_sum2_d16's order (wave xor-shuffle, then the 16 waves in order):
// the joint two-image form below sums every value exactly as the one-image form does (red: N * 16 doubles)
template <int N>
__device__ __forceinline__ void block_sum_d16(double (&v)[N], double* red) {
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = wave_sum_d(v[k]);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) red[N * w + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = 0.0;
#pragma unroll
  for (int i = 0; i < kBnFusedThreads / 64; ++i) {  // fixed order: deterministic
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] += red[N * i + k];
  }
}

// NB images img0 .. img0 + NB - 1 of channel c, their loads, reductions and stores issued together (r06: with
// NB = 1 per image, a 256-channel pair BN - 256 blocks, one per CU - loaded, reduced and stored image 0 before
// image 1's loads: 12.2 us per forward at 2.8 TB/s, profiles/r06_bn_pair_ab.txt).  Every per-image value is
// computed with the one-image operations in the same order, so NB = 2 and two NB = 1 passes agree bit for bit;
// the running statistics and the batch counter are updated image by image, image 0 first, as before.
template <int EPT, int NB>
__device__ __forceinline__ void bn_fwd_rows(const BnArgs& a, int c, int img0, double* red, float& am) {
  constexpr bool VF = EPT >= kBnVoffMinEpt;  // (as bn_bwd_rows)
  int t = threadIdx.x;
  if constexpr (VF || kBnOpaqueAll) asm volatile("" : "+v"(t));
  const int P = a.P;
  const unsigned vo = (unsigned)t * 4u;
  float xv[NB][EPT];
  double sh[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const long long base = (long long)(c * a.NI + img0 + b) * P;
    const __amdgpu_buffer_rsrc_t rx = bn_row(a.x + base, P);
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      if constexpr (VF) {
        xv[b][j] = bn_ldv(rx, vo, j);
      } else {
        const int e = j * kBnFusedThreads + t;
        xv[b][j] = e < P ? bn_ld(rx, vo, j) : 0.f;
      }
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) sh[b] = (double)a.x[(long long)(c * a.NI + img0 + b) * P];
  double s[2 * NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      if (j * kBnFusedThreads + t < P) {
        const double d = (double)xv[b][j] - sh[b];
        s1 = __dadd_rn(s1, d);  // explicit roundings: the single-image and pair forms agree bit for bit
        s2 = __fma_rn(d, d, s2);
      }
    }
    s[2 * b] = s1;
    s[2 * b + 1] = s2;
  }
  block_sum_d16<2 * NB>(s, red);
  const double n = (double)P;
  float alpha[NB], bsh[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int r = c * a.NI + img0 + b;
    const double dm = s[2 * b] / n;
    double var = __fma_rn(-dm, dm, __ddiv_rn(s[2 * b + 1], n));
    if (var < 0.0) var = 0.0;
    const float mean = (float)(sh[b] + dm);
    const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
    if (t == 0) {
      if (a.update_running) {
        const float m = a.momentum;
        const float unbiased = (float)(P > 1 ? var * n / (n - 1.0) : var);
        a.running_mean[c] = running_blend(a.running_mean[c], m, mean);
        a.running_var[c] = running_blend(a.running_var[c], m, unbiased);
        if (c == 0 && a.num_batches) a.num_batches[0] += 1;
      }
      a.save_mean[r] = mean;
      a.save_invstd[r] = invstd;
    }
    alpha[b] = invstd * (a.gamma ? a.gamma[c] : 1.f);
    bsh[b] = __fmaf_rn(-mean, alpha[b], a.beta ? a.beta[c] : 0.f);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int r = c * a.NI + img0 + b;
    const long long base = (long long)r * P;
    const __amdgpu_buffer_rsrc_t ry = bn_row(a.y + base, P);
    // the residual is loaded after the statistics: not live across the reduction, so the EPT <= 16
    // forms fit 64 VGPRs (two 1024-thread blocks per CU)
    float rv[EPT];
    if (a.residual) {
      const __amdgpu_buffer_rsrc_t rr = bn_row(a.residual + base, P);
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        if constexpr (VF)
          rv[j] = bn_ldv(rr, vo, j);
        else
          rv[j] = j * kBnFusedThreads + t < P ? bn_ld(rr, vo, j) : 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) rv[j] = 0.f;
    }
    // r05: with a.mask, y > 0 of each wave's 64 consecutive pixels as one 64-bit word (a ballot): the
    // residual BN's backward then reads 1 bit per pixel for its ReLU mask instead of the 4-byte y
    // (lane j of the wave keeps block j's word, and the EPT words leave in one masked store after the loop)
    unsigned long long* mrow = a.mask ? a.mask + (long long)r * cdiv(P, 64) : nullptr;
    unsigned long long myword = 0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = j * kBnFusedThreads + t;
      bool pos = false;
      if constexpr (VF) {  // (stores past P dropped by bn_stv)
        float v = __fmaf_rn(xv[b][j], alpha[b], bsh[b]);
        v += rv[j];
        v = a.relu ? fmaxf(v, 0.f) : v;
        bn_stv(ry, vo, j, v);
        if (e < P) {
          am = fmaxf(am, fabsf(v));
          pos = v > 0.f;
        }
      } else if (e < P) {
        float v = __fmaf_rn(xv[b][j], alpha[b], bsh[b]);
        v += rv[j];
        v = a.relu ? fmaxf(v, 0.f) : v;
        bn_st(ry, vo, j, v);
        am = fmaxf(am, fabsf(v));
        pos = v > 0.f;
      }
      if (mrow) {
        const unsigned long long bits = __ballot(pos);
        if ((t & 63) == j) myword = bits;
      }
    }
    static_assert(EPT <= 64, "one mask word per lane");
    if (mrow && (t & 63) < EPT && (t & 63) * kBnFusedThreads + (t & ~63) < P)
      mrow[(t & 63) * (kBnFusedThreads / 64) + (t >> 6)] = myword;
  }
}

// JOINT: the two images of a pair together (launched for NI = 2, EPT <= 9) at one 1024-thread block per CU
// (128 VGPRs: the pair's registers); else image by image, two blocks per CU for EPT <= 16 (64 VGPRs)
template <int EPT, bool JOINT>
constexpr int bn_waves_per_eu() { return JOINT ? 4 : EPT <= kBnTwoBlockEpt ? 8 : 1; }

template <int EPT, bool JOINT = false>
__global__ void __launch_bounds__(kBnFusedThreads) __attribute__((amdgpu_waves_per_eu(bn_waves_per_eu<EPT, JOINT>()))) k_bn_fwd_fused(BnArgs a) {
  __shared__ double red[4 * kBnFusedThreads / 64];
  const int c = blockIdx.x;
  float am = 0.f;
  if constexpr (JOINT) {
    bn_fwd_rows<EPT, 2>(a, c, 0, red, am);
  } else {
    for (int img = 0; img < a.NI; ++img) {  // the channel's images one after the other
      if (img) __syncthreads();               // red[] is reused
      bn_fwd_rows<EPT, 1>(a, c, img, red, am);
    }
  }
  if (a.absmax) {
    __shared__ float redm[kBnFusedThreads / 64];
    am = block_max16(am, redm);
    if (threadIdx.x == 0) a.absmax[c] = am;
  }
}

// the backward's NB images of channel c (as bn_fwd_rows: joint loads and reductions, per-image arithmetic and
// the parameter gradients image by image, image 0 first)
template <int EPT, int NB>
__device__ __forceinline__ void bn_bwd_rows(const BnBwdArgs& a, int c, int img0, double* red, float& am, float& dg,
                                            float& db) {
  // t through an opaque register copy (r06): the image loop of the one-image form cannot hoist the EPT per-element
  // range tests out of the loop, where they were held across it (EPT = 16: 43 spilled SGPRs, 14 spilled VGPRs)
  constexpr bool VF = EPT >= kBnVoffMinEpt;
  int t = threadIdx.x;
  if constexpr (VF || kBnOpaqueAll) asm volatile("" : "+v"(t));
  const int P = a.P;
  const unsigned vo = (unsigned)t * 4u;
  float g[NB][EPT], xv[NB][EPT];
  float mean[NB], invstd[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int r = c * a.NI + img0 + b;
    const long long base = (long long)r * P;
    mean[b] = a.save_mean[r];
    invstd[b] = a.save_invstd[r];
    const __amdgpu_buffer_rsrc_t rdy = bn_row(a.dy + base, P), rx = bn_row(a.x + base, P);
#pragma unroll
    for (int j = 0; j < EPT; ++j) {  // 0 past P
      if constexpr (VF) {
        g[b][j] = bn_ldv(rdy, vo, j);
        xv[b][j] = bn_ldv(rx, vo, j);
      } else {
        const int e = j * kBnFusedThreads + t;
        g[b][j] = e < P ? bn_ld(rdy, vo, j) : 0.f;
        xv[b][j] = e < P ? bn_ld(rx, vo, j) : 0.f;
      }
    }
  }
  const float gm = a.gamma ? a.gamma[c] : 1.f;
  double s[2 * NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int r = c * a.NI + img0 + b;
    const float w = invstd[b] * gm;
    if (a.relu && a.mask) {  // the forward's y > 0 bits: one 8-byte word per wave and element block
      // r06: lane j of each wave loads element block j's word (the forward's store layout) and block j reads it
      // back with readlane (wave-uniform, scalar registers): one load per lane instead of EPT 64-bit vector
      // loads, which the compiler hoisted next to the row loads - 32 more VGPRs at EPT 16, 15 of them spilled
      const unsigned long long* mrow = a.mask + (long long)r * cdiv(P, 64);
      const int l = t & 63;
      unsigned long long mw = 0;
      if (l < EPT && l * kBnFusedThreads + (t & ~63) < P) mw = mrow[l * (kBnFusedThreads / 64) + (t >> 6)];
      const unsigned mlo = (unsigned)mw, mhi = (unsigned)(mw >> 32);
#pragma unroll
      for (int j = 0; j < EPT; ++j) {  // (g = 0 past P already)
        const unsigned half = l < 32 ? __builtin_amdgcn_readlane(mlo, j) : __builtin_amdgcn_readlane(mhi, j);
        if (!((half >> (l & 31)) & 1u)) g[b][j] = 0.f;
      }
    } else if (a.relu && a.y) {
      const __amdgpu_buffer_rsrc_t ryy = bn_row(a.y + (long long)r * P, P);
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        if constexpr (VF) {
          if (!(bn_ldv(ryy, vo, j) > 0.f)) g[b][j] = 0.f;
        } else {
          if (j * kBnFusedThreads + t < P && !(bn_ld(ryy, vo, j) > 0.f)) g[b][j] = 0.f;
        }
      }
    } else if (a.relu) {  // y > 0 recomputed with k_bn_fwd_fused's operations (its alpha, bsh)
      if constexpr (EPT <= kBnRemaskMaxEpt) {  // (the 33-element form spills twice as much with it)
        const float bsh = __fmaf_rn(-mean[b], w, a.beta ? a.beta[c] : 0.f);
#pragma unroll
        for (int j = 0; j < EPT; ++j)
          if (!(__fmaf_rn(xv[b][j], w, bsh) > 0.f)) g[b][j] = 0.f;
      }
    }
    double sg = 0.0, sgx = 0.0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const float xh = (xv[b][j] - mean[b]) * invstd[b];
      sg = __dadd_rn(sg, (double)g[b][j]);  // g = 0 past P
      sgx = __fma_rn((double)g[b][j], (double)xh, sgx);
    }
    s[2 * b] = sg;
    s[2 * b + 1] = sgx;
  }
  block_sum_d16<2 * NB>(s, red);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const double sg = s[2 * b], sgx = s[2 * b + 1];
    if (t == 0) {
      if (img0 + b == 0) {
        dg = (a.accumulate && a.dgamma) ? a.dgamma[c] + (float)sgx : (float)sgx;
        db = (a.accumulate && a.dbeta) ? a.dbeta[c] + (float)sg : (float)sg;
      } else {
        dg += (float)sgx;
        db += (float)sg;
      }
    }
    const float w = invstd[b] * gm;
    const float m1 = (float)(sg / (double)P), m2 = (float)(sgx / (double)P);
    const long long base = (long long)(c * a.NI + img0 + b) * P;
    const __amdgpu_buffer_rsrc_t rdres = bn_row(a.dres ? a.dres + base : nullptr, P);
    const __amdgpu_buffer_rsrc_t rdx = bn_row(a.dx ? a.dx + base : nullptr, P);
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = j * kBnFusedThreads + t;
      const float xh = (xv[b][j] - mean[b]) * invstd[b];
      const float d = __fmul_rn(__fmaf_rn(-xh, m2, __fsub_rn(g[b][j], m1)), w);
      if constexpr (VF) {  // (stores past P dropped by bn_stv)
        if (a.dres) bn_stv(rdres, vo, j, g[b][j]);
        if (a.dx) bn_stv(rdx, vo, j, d);
        if (e < P) am = fmaxf(am, fabsf(d));
      } else if (e < P) {
        if (a.dres) bn_st(rdres, vo, j, g[b][j]);
        if (a.dx) bn_st(rdx, vo, j, d);
        am = fmaxf(am, fabsf(d));
      }
    }
  }
}

template <int EPT, bool JOINT = false>
__global__ void __launch_bounds__(kBnFusedThreads) __attribute__((amdgpu_waves_per_eu(bn_waves_per_eu<EPT, JOINT>()))) k_bn_bwd_fused(BnBwdArgs a) {
  __shared__ double red[4 * kBnFusedThreads / 64];
  const int c = blockIdx.x;
  float am = 0.f;
  float dg = 0.f, db = 0.f;  // the parameter gradients, image by image (thread 0)
  if constexpr (JOINT) {
    bn_bwd_rows<EPT, 2>(a, c, 0, red, am, dg, db);
  } else {
    for (int img = 0; img < a.NI; ++img) {  // the channel's images one after the other
      if (img) __syncthreads();               // red[] is reused
      bn_bwd_rows<EPT, 1>(a, c, img, red, am, dg, db);
    }
  }
  if (threadIdx.x == 0) {
    if (a.dgamma) a.dgamma[c] = dg;
    if (a.dbeta) a.dbeta[c] = db;
  }
  if (a.absmax) {
    __shared__ float redm[kBnFusedThreads / 64];
    am = block_max16(am, redm);
    if (threadIdx.x == 0) a.absmax[c] = am;
  }
}


// r06: the pair (NI = 2) of <= kBnJointMaxC channels at EPT <= 9 runs the joint two-image kernels: there one round
// of <= 256 blocks leaves half of the CUs' block slots empty anyway, and the joint loads double what is in flight
// (256 ch fwd 11.7 vs 12.2 us, bwd 17.5 vs 19.0, bwd with the mask recomputed 12.1 vs 13.8).  From 512 channels the
// image-by-image kernel's two blocks per CU win (512 ch fwd 18.1 vs 23.3 us, 1024 ch + residual 37.5 vs 46.0;
// profiles/r06_bn_pair_ab.txt); at 16 elements the pair's registers spill.
constexpr int kBnJointPair = 1;
// r06: the joint forward at 16 elements too (128 VGPRs, one block per CU, no spill: config-5 256-channel maps 15.4 vs
// 17.1 us); the joint backward spills 33 VGPRs there and is slower (remask 28.6 vs 21.8 us; profiles/r06_bn_joint16_ab.txt)
constexpr bool kBnJoint16Fwd = true;
constexpr bool kBnJoint16Bwd = false;
constexpr int kBnJointMaxC = 256;
template <typename K, typename A>
static int bn_launch_fused(K k4, K k9, K k16, K k33, K j4, K j9, K j16, int c, int p, hipStream_t st, const A& a) {
  const bool joint = kBnJointPair && a.NI == 2 && c <= kBnJointMaxC;
  K k = p <= 4 * kBnFusedThreads ? (joint ? j4 : k4)
        : p <= 9 * kBnFusedThreads ? (joint ? j9 : k9)
        : p <= 16 * kBnFusedThreads ? (joint ? j16 : k16) : k33;
  MSL_LAUNCH(k, dim3(c), dim3(kBnFusedThreads), 0, st, a);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace msl

using namespace msl;

extern "C" {

int msl_bn_uses_fused(int c, int p, int training, const msl_forms* forms) {
  if (forms_bad(forms)) return MSL_ERR_ARG;
  return training && bn_fused_enabled(forms) && c >= 1 && p >= 1 && bn_fused_shape(c, p) ? 1 : 0;
}

size_t msl_bn_workspace(int c, int p, int nimg) {
  return align_up((size_t)c * std::max(nimg, 1) * bn_splits(p) * 2 * sizeof(double), 256);
}

int msl_bn_fwd(const float* x, const float* gamma, const float* beta, const float* residual,
               float* y, float* running_mean, float* running_var, long long* num_batches_tracked,
               float* save_mean, float* save_invstd, int c, int p, int nimg, int training,
               int update_running, float momentum, float eps, int relu, const msl_forms* forms, void* ws,
               size_t ws_bytes, msl_stream_t stream) {
  return msl_bn_fwd_am(x, gamma, beta, residual, y, running_mean, running_var, num_batches_tracked, save_mean,
                       save_invstd, c, p, nimg, training, update_running, momentum, eps, relu, forms, ws, ws_bytes, stream,
                       nullptr);
}

int msl_bn_fwd_am(const float* x, const float* gamma, const float* beta, const float* residual,
                  float* y, float* running_mean, float* running_var, long long* num_batches_tracked,
                  float* save_mean, float* save_invstd, int c, int p, int nimg, int training,
                  int update_running, float momentum, float eps, int relu, const msl_forms* forms, void* ws,
                  size_t ws_bytes, msl_stream_t stream, float* absmax) {
  return msl_bn_fwd_mask(x, gamma, beta, residual, y, running_mean, running_var, num_batches_tracked, save_mean,
                         save_invstd, c, p, nimg, training, update_running, momentum, eps, relu, forms, ws, ws_bytes,
                         stream, absmax, nullptr);
}

size_t msl_bn_relu_mask_bytes(int c, int p, int nimg) {
  if (c < 1 || p < 1 || nimg < 1) return 0;
  return (size_t)c * nimg * cdiv(p, 64) * sizeof(uint64_t);
}

int msl_bn_fwd_mask(const float* x, const float* gamma, const float* beta, const float* residual,
                    float* y, float* running_mean, float* running_var, long long* num_batches_tracked,
                    float* save_mean, float* save_invstd, int c, int p, int nimg, int training,
                    int update_running, float momentum, float eps, int relu, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream, float* absmax, uint64_t* relu_mask) {
  if (!x || !y || !save_mean || !save_invstd || c < 1 || p < 1 || nimg < 1 || (long long)c * nimg >= (1LL << 31))
    return MSL_ERR_ARG;
  if ((!training || update_running) && (!running_mean || !running_var)) return MSL_ERR_ARG;
  hipStream_t st = as_stream(stream);
  const int S = bn_splits(p);
  const int R = c * nimg;  // rows (channel, image)
  if (training && ws_bytes < msl_bn_workspace(c, p, nimg)) return MSL_ERR_WORKSPACE;
  double* part = (double*)ws;
  const bool vec = al16(x) && al16(y) && (!residual || al16(residual));
  if (forms_bad(forms)) return MSL_ERR_ARG;
  const bool fused = training && bn_fused_enabled(forms) && bn_fused_shape(c, p);
  if (relu_mask && !(fused && relu)) return MSL_ERR_ARG;  // the bits come from the fused kernels
  if (training && !fused) {
    if (vec)
      MSL_LAUNCH(k_bn_stats<true>, dim3(R, S), dim3(256), 0, st, x, p, S, part, absmax, nimg);
    else
      MSL_LAUNCH(k_bn_stats<false>, dim3(R, S), dim3(256), 0, st, x, p, S, part, absmax, nimg);
    MSL_CHECK_LAUNCH();
  } else if (!fused && absmax) {
    MSL_LAUNCH(k_zero_rows, dim3(cdiv(c, 256)), dim3(256), 0, st, absmax, c);
    MSL_CHECK_LAUNCH();
  }
  BnArgs a;
  a.x = x;
  a.gamma = gamma;
  a.beta = beta;
  a.residual = residual;
  a.y = y;
  a.running_mean = running_mean;
  a.running_var = running_var;
  a.save_mean = save_mean;
  a.save_invstd = save_invstd;
  a.num_batches = num_batches_tracked;
  a.part = part;
  a.C = c;
  a.NI = nimg;
  a.P = p;
  a.S = S;
  a.chunk = bn_flat_chunk(p);
  a.relu = relu;
  a.training = training;
  a.update_running = update_running;
  a.eps = eps;
  a.momentum = momentum;
  a.absmax = absmax;
  a.mask = reinterpret_cast<unsigned long long*>(relu_mask);
  if (fused) return bn_launch_fused(k_bn_fwd_fused<4>, k_bn_fwd_fused<9>, k_bn_fwd_fused<16>, k_bn_fwd_fused<33>,
                                        k_bn_fwd_fused<4, true>, k_bn_fwd_fused<9, true>, k_bn_fwd_fused<16, kBnJoint16Fwd>, c, p, st,
                                        a);
  const unsigned blocks = (unsigned)cdiv((long long)R * p, (long long)a.chunk);
  if (vec)
    MSL_LAUNCH(k_bn_apply<true>, dim3(blocks), dim3(256), 0, st, a);
  else
    MSL_LAUNCH(k_bn_apply<false>, dim3(blocks), dim3(256), 0, st, a);
  MSL_CHECK_LAUNCH();  // (absmax: folded in by k_bn_apply, zeroed by the launch before)
  return MSL_OK;
}

int msl_bn_bwd(const float* dy, const float* x, const float* y, const float* gamma,
               const float* save_mean, const float* save_invstd, float* dx, float* dres,
               float* dgamma, float* dbeta, int c, int p, int nimg, int training, int relu,
               int accumulate_params, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  return msl_bn_bwd_am(dy, x, y, gamma, save_mean, save_invstd, dx, dres, dgamma, dbeta, c, p, nimg, training, relu,
                       accumulate_params, forms, ws, ws_bytes, stream, nullptr);
}

int msl_bn_bwd_am(const float* dy, const float* x, const float* y, const float* gamma,
                  const float* save_mean, const float* save_invstd, float* dx, float* dres,
                  float* dgamma, float* dbeta, int c, int p, int nimg, int training, int relu,
                  int accumulate_params, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, float* absmax_dx) {
  if (relu && !y) return MSL_ERR_ARG;
  return msl_bn_bwd_am_beta(dy, x, y, gamma, nullptr, save_mean, save_invstd, dx, dres, dgamma, dbeta, c, p, nimg,
                            training, relu, accumulate_params, forms, ws, ws_bytes, stream, absmax_dx);
}

static int bn_bwd(const float* dy, const float* x, const float* y, const uint64_t* relu_mask, const float* gamma,
                  const float* beta, const float* save_mean, const float* save_invstd, float* dx, float* dres,
                  float* dgamma, float* dbeta, int c, int p, int nimg, int training, int relu, int accumulate_params,
                  const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, float* absmax_dx) {
  if (!dy || !x || !save_mean || !save_invstd || c < 1 || p < 1 || nimg < 1 || (long long)c * nimg >= (1LL << 31))
    return MSL_ERR_ARG;
  if (forms_bad(forms)) return MSL_ERR_ARG;
  const bool fused = training && bn_fused_enabled(forms) && bn_fused_shape(c, p);
  if (relu_mask && !(fused && relu)) return MSL_ERR_ARG;  // the bits are read by the fused kernels
  // the mask recompute is the fused kernels' alone, up to 16 elements per lane
  if (relu && !y && !relu_mask && !(fused && p <= kBnRemaskMaxEpt * kBnFusedThreads)) return MSL_ERR_ARG;
  if (absmax_dx && !dx) return MSL_ERR_ARG;
  if (ws_bytes < msl_bn_workspace(c, p, nimg)) return MSL_ERR_WORKSPACE;
  hipStream_t st = as_stream(stream);
  const int S = bn_splits(p);
  const int R = c * nimg;  // rows (channel, image)
  BnBwdArgs a;
  a.dy = dy;
  a.x = x;
  a.y = y;
  a.gamma = gamma;
  a.beta = beta;
  a.save_mean = save_mean;
  a.save_invstd = save_invstd;
  a.dx = dx;
  a.dres = dres;
  a.dgamma = dgamma;
  a.dbeta = dbeta;
  a.part = (double*)ws;
  a.C = c;
  a.NI = nimg;
  a.P = p;
  a.S = S;
  a.chunk = bn_flat_chunk(p);
  a.relu = relu;
  a.training = training;
  a.accumulate = accumulate_params;
  a.absmax = absmax_dx;
  a.mask = reinterpret_cast<const unsigned long long*>(relu_mask);
  if (fused)
    return bn_launch_fused(k_bn_bwd_fused<4>, k_bn_bwd_fused<9>, k_bn_bwd_fused<16>, k_bn_bwd_fused<33>,
                           k_bn_bwd_fused<4, true>, k_bn_bwd_fused<9, true>, k_bn_bwd_fused<16, kBnJoint16Bwd>, c, p, st, a);
  const bool vec = al16(dy) && al16(x) && (!relu || al16(y)) && (!dx || al16(dx)) && (!dres || al16(dres));
  const unsigned blocks = (unsigned)cdiv((long long)R * p, (long long)a.chunk);
  if (vec) {
    MSL_LAUNCH(k_bn_bwd_reduce<true>, dim3(R, S), dim3(256), 0, st, a);
    MSL_CHECK_LAUNCH();
    MSL_LAUNCH(k_bn_bwd_apply<true>, dim3(blocks), dim3(256), 0, st, a);
  } else {
    MSL_LAUNCH(k_bn_bwd_reduce<false>, dim3(R, S), dim3(256), 0, st, a);
    MSL_CHECK_LAUNCH();
    MSL_LAUNCH(k_bn_bwd_apply<false>, dim3(blocks), dim3(256), 0, st, a);
  }
  MSL_CHECK_LAUNCH();  // (absmax_dx: folded in by k_bn_bwd_apply, zeroed by k_bn_bwd_reduce)
  return MSL_OK;
}

int msl_bn_bwd_am_beta(const float* dy, const float* x, const float* y, const float* gamma, const float* beta,
                       const float* save_mean, const float* save_invstd, float* dx, float* dres,
                       float* dgamma, float* dbeta, int c, int p, int nimg, int training, int relu,
                       int accumulate_params, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream,
                       float* absmax_dx) {
  return bn_bwd(dy, x, y, nullptr, gamma, beta, save_mean, save_invstd, dx, dres, dgamma, dbeta, c, p, nimg, training,
                relu, accumulate_params, forms, ws, ws_bytes, stream, absmax_dx);
}

int msl_bn_bwd_mask(const float* dy, const float* x, const uint64_t* relu_mask, const float* gamma, const float* beta,
                    const float* save_mean, const float* save_invstd, float* dx, float* dres, float* dgamma,
                    float* dbeta, int c, int p, int nimg, int training, int relu, int accumulate_params,
                    const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, float* absmax_dx) {
  if (!relu_mask || !relu) return MSL_ERR_ARG;
  return bn_bwd(dy, x, nullptr, relu_mask, gamma, beta, save_mean, save_invstd, dx, dres, dgamma, dbeta, c, p, nimg,
                training, relu, accumulate_params, forms, ws, ws_bytes, stream, absmax_dx);
}

}  // extern "C"

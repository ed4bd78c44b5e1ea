// The stem and the strided glue of ResNetMulti on HIP, so the
// training step runs no library kernel and is bit-reproducible run to run:
//   - conv1 7x7 / stride 2 / pad 3 (deeplab_multi.py:73-74, 114): im2col into a [cin*49][P] column
//     matrix, then the pointwise GEMM kernels of dconv.hip (the 7x7 weight [64][3][7][7] is a
//     [64][147] pointwise weight as laid out); data gradient = pointwise dgrad + col2im (gather);
//   - maxpool 3x3 / stride 2 / pad 1 / ceil_mode (deeplab_multi.py:77, 114): first-max (NaN wins)
//     window scan in torch-CPU's order, the argmax index kept; backward as a gather over the
//     windows covering each input pixel, summed in torch-CPU's scatter order (bit-exact);
//   - x[:, :, ::s, ::s] for layer2.0's stride-2 1x1 conv1 and downsample (deeplab_multi.py:12-13,
//     96-99: Caffe-style, the stride sits on the 1x1 convs), and its transpose for the gradient.
// Every kernel is a plain gather: one thread per output element, no atomics, no float reordering;
// element indices in 32-bit arithmetic (the entry points keep the counts below 2^31).
#include "msl_internal.h"

namespace msl {

// col[(c*KH + i)*KW + j][n][oy*WO + ox] = x[c][n][oy*S - PAD + i*D][ox*S - PAD + j*D] (0 outside the
// image) for the NI images n of a [C][NI][H][W] batch.  Thread per (row k, image, output row oy, 4
// output columns): the 4 stores are one float4 when WO % 4 == 0.
__global__ void __launch_bounds__(256) k_im2col(const float* __restrict__ x, int H, int W, int NI, int KH, int KW,
                                                int S, int PAD, int D, int HO, int WO, int K,
                                                float* __restrict__ col) {
  const unsigned wq = (WO + 3) >> 2;
  const unsigned total = (unsigned)K * NI * HO * wq;  // < 2^31 (msl_im2col checks): 32-bit index math
  const long long P = (long long)NI * HO * WO;
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < total; e += gridDim.x * 256u) {
    const int q = (int)(e % wq);
    const unsigned r = e / wq;
    const int oy = (int)(r % (unsigned)HO);
    const unsigned r2 = r / (unsigned)HO;
    const int n = (int)(r2 % (unsigned)NI);
    const int k = (int)(r2 / (unsigned)NI);
    const int j = k % KW, i = (k / KW) % KH, c = k / (KW * KH);
    const int iy = oy * S - PAD + i * D;
    const bool rowok = (unsigned)iy < (unsigned)H;
    const float* src = x + (((long long)c * NI + n) * H + (rowok ? iy : 0)) * W;
    float v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ox = q * 4 + t;
      const int ix = ox * S - PAD + j * D;
      v[t] = (rowok && ox < WO && (unsigned)ix < (unsigned)W) ? src[ix] : 0.f;
    }
    float* dst = col + (long long)k * P + ((long long)n * HO + oy) * WO + q * 4;
    if ((WO & 3) == 0) {
      *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int t = 0; t < 4 && q * 4 + t < WO; ++t) dst[t] = v[t];
    }
  }
}

// x[c][n][y][xx] = sum over (i, j) (i-major) of col[(c*KH + i)*KW + j][n][oy][ox] for every window
// position that maps (oy, ox) onto (y, xx).
__global__ void __launch_bounds__(256) k_col2im(const float* __restrict__ col, int C, int H, int W, int NI, int KH,
                                                int KW, int S, int PAD, int D, int HO, int WO, float* __restrict__ x) {
  const unsigned total = (unsigned)C * NI * H * W;  // < 2^31 (checked by the entry point)
  const long long P = (long long)NI * HO * WO;
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < total; e += gridDim.x * 256u) {
    const int xx = (int)(e % (unsigned)W);
    const unsigned r = e / (unsigned)W;
    const int y = (int)(r % (unsigned)H);
    const unsigned r2 = r / (unsigned)H;
    const int n = (int)(r2 % (unsigned)NI);
    const int c = (int)(r2 / (unsigned)NI);
    float s = 0.f;
    for (int i = 0; i < KH; ++i) {
      const int ty = y + PAD - i * D;
      if (ty < 0 || ty % S) continue;
      const int oy = ty / S;
      if (oy >= HO) continue;
      for (int j = 0; j < KW; ++j) {
        const int tx = xx + PAD - j * D;
        if (tx < 0 || tx % S) continue;
        const int ox = tx / S;
        if (ox >= WO) continue;
        s += col[((long long)(c * KH + i) * KW + j) * P + ((long long)n * HO + oy) * WO + ox];
      }
    }
    x[e] = s;
  }
}

// torch-CPU max_pool2d (aten/native/cpu/MaxPoolKernel.cpp): window [oy*S - PAD, +K) clipped to the
// image, scanned row-major, `val > max || isnan(val)` replaces, max starts at -inf with the index
// of the window's first element.  idx = y*W + x within the channel.
__global__ void __launch_bounds__(256) k_maxpool_fwd(const float* __restrict__ x, int H, int W, int K, int S, int PAD,
                                                     int HO, int WO, long long total, float* __restrict__ y,
                                                     int32_t* __restrict__ idx) {
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < (unsigned)total; e += gridDim.x * 256u) {
    const int ox = (int)(e % (unsigned)WO);
    const unsigned r = e / (unsigned)WO;
    const int oy = (int)(r % (unsigned)HO);
    const long long c = r / (unsigned)HO;
    int y0 = oy * S - PAD, x0 = ox * S - PAD;
    const int y1 = min(y0 + K, H), x1 = min(x0 + K, W);
    y0 = max(y0, 0);
    x0 = max(x0, 0);
    const float* src = x + c * H * W;
    float best = -INFINITY;
    int bi = y0 * W + x0;
    for (int yy = y0; yy < y1; ++yy)
      for (int xx = x0; xx < x1; ++xx) {
        const float v = src[yy * W + xx];
        if (v > best || v != v) {
          best = v;
          bi = yy * W + xx;
        }
      }
    y[e] = best;
    idx[e] = bi;
  }
}

// dx[c][y][x] = sum of dy over the windows whose argmax is (y, x), in output scan order (oy, then
// ox, ascending) - the order torch-CPU's backward adds them in (bit-exact).
__global__ void __launch_bounds__(256) k_maxpool_bwd(const float* __restrict__ dy, const int32_t* __restrict__ idx,
                                                     int H, int W, int K, int S, int PAD, int HO, int WO,
                                                     long long total, float* __restrict__ dx) {
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < (unsigned)total; e += gridDim.x * 256u) {
    const int xx = (int)(e % (unsigned)W);
    const unsigned r = e / (unsigned)W;
    const int y = (int)(r % (unsigned)H);
    const long long c = r / (unsigned)H;
    const int me = y * W + xx;
    // windows covering y: oy*S - PAD <= y <= oy*S - PAD + K - 1
    const int ly = y + PAD - (K - 1), lx = xx + PAD - (K - 1);
    const int oy0 = ly <= 0 ? 0 : (ly + S - 1) / S, oy1 = min((y + PAD) / S, HO - 1);
    const int ox0 = lx <= 0 ? 0 : (lx + S - 1) / S, ox1 = min((xx + PAD) / S, WO - 1);
    const long long base = c * HO * WO;
    float s = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const long long o = base + (long long)oy * WO + ox;
        if (idx[o] == me) s += dy[o];
      }
    dx[e] = s;
  }
}

// r06: the ResNet stem's pools (K = 3, S = 2: at most 2 x 2 windows cover an input pixel, and a window has at most
// 3 x 3 taps) with every candidate loaded unconditionally from a clamped, valid address and masked afterwards, so
// all of a thread's loads are in flight together; the same scan orders as k_maxpool_fwd / k_maxpool_bwd (the
// same bits).  The generic kernels' loop bounds per thread left one or two dependent load chains per element:
// 105 us backward, 38 us forward for the 1024x512 pair (profiles/r06_step_breakdown.txt).
__global__ void __launch_bounds__(256) k_maxpool_fwd3(const float* __restrict__ x, int H, int W, int S, int PAD, int HO,
                                                      int WO, long long total, float* __restrict__ y,
                                                      int32_t* __restrict__ idx) {
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < (unsigned)total; e += gridDim.x * 256u) {
    const int ox = (int)(e % (unsigned)WO);
    const unsigned r = e / (unsigned)WO;
    const int oy = (int)(r % (unsigned)HO);
    const long long c = r / (unsigned)HO;
    const int y0 = oy * S - PAD, x0 = ox * S - PAD;
    const float* src = x + c * H * W;
    float v[9];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int yy = min(max(y0 + a, 0), H - 1), xx = min(max(x0 + b, 0), W - 1);
        v[3 * a + b] = src[yy * W + xx];
      }
    const int ya = max(y0, 0), xa = max(x0, 0);
    float best = -INFINITY;
    int bi = ya * W + xa;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int yy = y0 + a, xx = x0 + b;
        const float t = v[3 * a + b];
        if (yy >= 0 && yy < H && xx >= 0 && xx < W && (t > best || t != t)) {
          best = t;
          bi = yy * W + xx;
        }
      }
    y[e] = best;
    idx[e] = bi;
  }
}

__global__ void __launch_bounds__(256) k_maxpool_bwd22(const float* __restrict__ dy, const int32_t* __restrict__ idx,
                                                       int H, int W, int K, int S, int PAD, int HO, int WO,
                                                       long long total, float* __restrict__ dx) {
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < (unsigned)total; e += gridDim.x * 256u) {
    const int xx = (int)(e % (unsigned)W);
    const unsigned r = e / (unsigned)W;
    const int y = (int)(r % (unsigned)H);
    const long long c = r / (unsigned)H;
    const int me = y * W + xx;
    const int ly = y + PAD - (K - 1), lx = xx + PAD - (K - 1);
    const int oy0 = ly <= 0 ? 0 : (ly + S - 1) / S, oy1 = min((y + PAD) / S, HO - 1);
    const int ox0 = lx <= 0 ? 0 : (lx + S - 1) / S, ox1 = min((xx + PAD) / S, WO - 1);
    const long long base = c * HO * WO;
    int iv[4];
    float dv[4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const long long o = base + (long long)min(oy0 + a, HO - 1) * WO + min(ox0 + b, WO - 1);
        iv[2 * a + b] = idx[o];
        dv[2 * a + b] = dy[o];
      }
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        if (oy0 + a <= oy1 && ox0 + b <= ox1 && iv[2 * a + b] == me) s += dv[2 * a + b];
    dx[e] = s;
  }
}

// y[c][oy][ox] = x[c][oy*S][ox*S]   (fwd)      x[c][y][xx] = (y % S || xx % S) ? 0 : y'[..]  (bwd)
__global__ void __launch_bounds__(256) k_subsample(const float* __restrict__ x, int H, int W, int S, int HO, int WO,
                                                   long long total, float* __restrict__ y) {
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < (unsigned)total; e += gridDim.x * 256u) {
    const int ox = (int)(e % (unsigned)WO);
    const unsigned r = e / (unsigned)WO;
    const int oy = (int)(r % (unsigned)HO);
    const long long c = r / (unsigned)HO;
    y[e] = x[(c * H + (long long)oy * S) * W + (long long)ox * S];
  }
}

__global__ void __launch_bounds__(256) k_subsample_bwd(const float* __restrict__ dy, int H, int W, int S, int HO,
                                                       int WO, long long total, float* __restrict__ dx) {
  for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < (unsigned)total; e += gridDim.x * 256u) {
    const int xx = (int)(e % (unsigned)W);
    const unsigned r = e / (unsigned)W;
    const int y = (int)(r % (unsigned)H);
    const long long c = r / (unsigned)H;
    float v = 0.f;
    if (y % S == 0 && xx % S == 0 && y / S < HO && xx / S < WO) v = dy[(c * HO + y / S) * WO + xx / S];
    dx[e] = v;
  }
}

static unsigned grid_for(long long n) { return (unsigned)std::min<long long>((n + 255) / 256, 16384); }

// every kernel above decodes its element index in 32-bit arithmetic (a 64-bit division per element
// made the maxpool backward 5x slower than its bytes, r03): element counts stay below 2^31
static bool bad_geom(int c, int h, int w, int k, int s, int pad, int ho, int wo) {
  return c < 1 || h < 1 || w < 1 || k < 1 || s < 1 || pad < 0 || ho < 1 || wo < 1 ||
         (long long)c * h * w >= (1LL << 31) || (long long)c * ho * wo >= (1LL << 31);
}

}  // namespace msl

using namespace msl;

extern "C" {

int msl_im2col(const float* x, int c, int h, int w, int nimg, int kh, int kw, int stride, int pad, int dil, int ho,
               int wo, float* col, msl_stream_t stream) {
  if (!x || !col || nimg < 1 || bad_geom(c * nimg, h, w, std::max(kh, kw), stride, pad, ho, wo) || kh < 1 ||
      kw < 1 || dil < 1 || (long long)c * kh * kw * nimg * ho * wo >= (1LL << 31) ||
      (long long)nimg * ho * wo >= (1LL << 31))
    return MSL_ERR_ARG;
  const int K = c * kh * kw;
  const long long n = (long long)K * nimg * ho * ((wo + 3) / 4);
  MSL_LAUNCH(k_im2col, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, h, w, nimg, kh, kw, stride, pad,
                     dil, ho, wo, K, col);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_col2im(const float* col, int c, int h, int w, int nimg, int kh, int kw, int stride, int pad, int dil, int ho,
               int wo, float* x, msl_stream_t stream) {
  if (!x || !col || nimg < 1 || bad_geom(c * nimg, h, w, std::max(kh, kw), stride, pad, ho, wo) || kh < 1 ||
      kw < 1 || dil < 1 || (long long)nimg * ho * wo >= (1LL << 31))
    return MSL_ERR_ARG;
  const long long n = (long long)c * nimg * h * w;
  MSL_LAUNCH(k_col2im, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), col, c, h, w, nimg, kh, kw, stride,
                     pad, dil, ho, wo, x);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_maxpool_fwd(const float* x, int c, int h, int w, int k, int stride, int pad, int ho, int wo, float* y,
                    int32_t* idx, msl_stream_t stream) {
  if (!x || !y || !idx || bad_geom(c, h, w, k, stride, pad, ho, wo) || 2 * pad > k) return MSL_ERR_ARG;
  // every window must start inside the image (torch: the last window starts before h + pad)
  if ((long long)(ho - 1) * stride - pad >= h || (long long)(wo - 1) * stride - pad >= w) return MSL_ERR_SHAPE;
  const long long n = (long long)c * ho * wo;
  if (k == 3)
    MSL_LAUNCH(k_maxpool_fwd3, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, h, w, stride, pad, ho, wo, n, y,
               idx);
  else
    MSL_LAUNCH(k_maxpool_fwd, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, h, w, k, stride, pad, ho,
               wo, n, y, idx);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_maxpool_bwd(const float* dy, const int32_t* idx, int c, int h, int w, int k, int stride, int pad, int ho,
                    int wo, float* dx, msl_stream_t stream) {
  if (!dy || !idx || !dx || bad_geom(c, h, w, k, stride, pad, ho, wo) || 2 * pad > k) return MSL_ERR_ARG;
  const long long n = (long long)c * h * w;
  if (k <= 2 * stride)  // at most 2 x 2 windows per input pixel
    MSL_LAUNCH(k_maxpool_bwd22, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), dy, idx, h, w, k, stride, pad, ho,
               wo, n, dx);
  else
    MSL_LAUNCH(k_maxpool_bwd, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), dy, idx, h, w, k, stride,
               pad, ho, wo, n, dx);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_subsample(const float* x, int c, int h, int w, int stride, int ho, int wo, float* y, msl_stream_t stream) {
  if (!x || !y || bad_geom(c, h, w, 1, stride, 0, ho, wo) || (long long)(ho - 1) * stride >= h ||
      (long long)(wo - 1) * stride >= w)
    return MSL_ERR_ARG;
  const long long n = (long long)c * ho * wo;
  MSL_LAUNCH(k_subsample, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, h, w, stride, ho, wo, n, y);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_subsample_bwd(const float* dy, int c, int h, int w, int stride, int ho, int wo, float* dx,
                      msl_stream_t stream) {
  if (!dy || !dx || bad_geom(c, h, w, 1, stride, 0, ho, wo)) return MSL_ERR_ARG;
  const long long n = (long long)c * h * w;
  MSL_LAUNCH(k_subsample_bwd, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), dy, h, w, stride, ho, wo,
                     n, dx);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

}  // extern "C"

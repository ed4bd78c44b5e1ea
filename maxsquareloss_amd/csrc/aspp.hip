// ASPP heads as one pointwise GEMM plus shifts (Classifier_Module, deeplab_multi.py:51-66, 84-85;
// quirk Q1: only branches 0 and 1 - d = 6 and 12 - run, with their biases).
//
// A head maps cin = 1024 / 2048 channels to C = 19 (16) classes over two branches of nine dilated
// taps.  As a direct implicit GEMM its M = C fills a fraction of a 64-row tile and the 69-137 MB
// input is streamed once per tap (r03: ~0.5 ms forward and ~0.57 ms weight gradient per head call,
// 8x re-read traffic).  The head is linear in x, so the small operand is shifted instead:
//   forward:   Z[t*C + m][q] = sum_c W_b[m][c][k] x[c][q]           (t = b*9 + k: one pointwise
//              GEMM with M' = 18*C rows, x read once)
//              y[m][p] = sum_t valid_t(p) Z[t*C + m][p + off_t] + sum_b bias_b[m]
//   backward:  G[t*C + m][q] = valid_t(q - off_t) dY[m][q - off_t]  (the shifted, masked copies of dY)
//              dx = W'^T G   (pointwise data gradient, K = 18*C)
//              dW'[t*C + m][c] = sum_q G[t*C + m][q] x[c][q]        (pointwise weight gradient)
//              dW_b[m][c][k] = dW'[(b*9 + k)*C + m][c], dbias_b[m] = sum_p dY[m][p]
// with off_t = dh*W + dw for tap k = (dh/d + 1)*3 + (dw/d + 1) of branch b, and valid_t(p) = the
// tap's source pixel (row + dh, col + dw) lies inside p's own image (pixel axis = nimg images of
// h x w: a tap never reads the neighbouring image).  Exactly the conv's sums, in another fp32 order.
#include "msl_internal.h"

namespace msl {

// tap t of the two-branch head: (row, column) offset
__device__ __forceinline__ void aspp_tap(int t, int dil0, int dil1, int& dh, int& dw) {
  const int b = t / 9, k = t - b * 9;
  const int d = b ? dil1 : dil0;
  dh = (k / 3 - 1) * d;
  dw = (k % 3 - 1) * d;
}

// y[m][p] = sum_t valid Z[t*C + m][p + off_t] (taps in order, from 0) + (bias_0[m] + bias_1[m])
__global__ void __launch_bounds__(256) k_aspp_shift_add(const float* __restrict__ z, const float* __restrict__ bias,
                                                        float* __restrict__ y, int nt, int C, int H, int W, int P,
                                                        int dil0, int dil1) {
  const int p = blockIdx.x * 256 + threadIdx.x, m = blockIdx.y;
  if (p >= P) return;
  const int hw = H * W;
  const int r = p % hw, yy = r / W, xx = r - yy * W;
  float acc = 0.f;
  for (int t = 0; t < nt; ++t) {
    int dh, dw;
    aspp_tap(t, dil0, dil1, dh, dw);
    if ((unsigned)(yy + dh) < (unsigned)H && (unsigned)(xx + dw) < (unsigned)W)
      acc += z[(long long)(t * C + m) * P + p + dh * W + dw];
  }
  if (bias) {
    float bs = bias[m];
    for (int b = 1; b < nt / 9; ++b) bs += bias[b * C + m];
    acc += bs;
  }
  y[(long long)m * P + p] = acc;
}

// G[t*C + m][q] = dY[m][q - off_t] where that source pixel is inside q's image, else 0
__global__ void __launch_bounds__(256) k_aspp_shift_gather(const float* __restrict__ dy, float* __restrict__ g, int C,
                                                           int H, int W, int P, int dil0, int dil1) {
  const int q = blockIdx.x * 256 + threadIdx.x, row = blockIdx.y;  // row = t*C + m
  if (q >= P) return;
  const int t = row / C, m = row - t * C;
  int dh, dw;
  aspp_tap(t, dil0, dil1, dh, dw);
  const int r = q % (H * W), yy = r / W, xx = r - yy * W;
  float v = 0.f;
  if ((unsigned)(yy - dh) < (unsigned)H && (unsigned)(xx - dw) < (unsigned)W) v = dy[(long long)m * P + q - dh * W - dw];
  g[(long long)row * P + q] = v;
}

// dbias[b][m] = sum_p dY[m][p] for every branch b (one block per class; fixed order)
__global__ void __launch_bounds__(256) k_aspp_bias_grad(const float* __restrict__ dy, int P, float* __restrict__ db,
                                                        int C, int nbranch) {
  __shared__ float part[4];
  const int m = blockIdx.x;
  float s = 0.f;
  for (int p = threadIdx.x; p < P; p += 256) s += dy[(long long)m * P + p];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = (part[0] + part[1]) + (part[2] + part[3]);
    for (int b = 0; b < nbranch; ++b) db[b * C + m] = tot;
  }
}

// W'[(b*9 + k)*C + m][c] = W_b[m][c][k]  (W_b at w + b*branch_stride, [C][cin][3][3])
__global__ void __launch_bounds__(256) k_aspp_weight_layout(const float* __restrict__ w, long long branch_stride,
                                                            int nt, int C, int cin, float* __restrict__ wp) {
  const long long n = (long long)nt * C * cin;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int c = (int)(e % cin);
    const long long row = e / cin;
    const int t = (int)(row / C), m = (int)(row - (long long)t * C);
    const int b = t / 9, k = t - b * 9;
    wp[e] = w[b * branch_stride + ((long long)m * cin + c) * 9 + k];
  }
}

// dW_b[m][c][k] = dW'[(b*9 + k)*C + m][c]  (dw: [nbranch][C][cin][3][3])
__global__ void __launch_bounds__(256) k_aspp_weight_grad(const float* __restrict__ dwp, int nt, int C, int cin,
                                                          float* __restrict__ dw) {
  const long long n = (long long)nt * C * cin;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int k = (int)(e % 9);
    const long long q = e / 9;  // (b*C + m)*cin + c
    const int c = (int)(q % cin);
    const long long bm = q / cin;
    const int b = (int)(bm / C), m = (int)(bm - (long long)b * C);
    dw[e] = dwp[((long long)(b * 9 + k) * C + m) * cin + c];
  }
}

static bool aspp_bad(int nbranch, int c, int h, int w, int nimg, int dil0, int dil1) {
  return nbranch < 1 || nbranch > 2 || c < 1 || h < 1 || w < 1 || nimg < 1 || dil0 < 1 || (nbranch == 2 && dil1 < 1) ||
         (long long)nimg * h * w * 9 * nbranch * c >= (1LL << 31);
}

}  // namespace msl

using namespace msl;

extern "C" {

int msl_aspp_weight_layout(const float* w, long long branch_stride, int nbranch, int c, int cin, float* wp,
                           msl_stream_t stream) {
  if (!w || !wp || nbranch < 1 || nbranch > 2 || c < 1 || cin < 1) return MSL_ERR_ARG;
  const long long n = 9LL * nbranch * c * cin;
  MSL_LAUNCH(k_aspp_weight_layout, dim3((unsigned)std::min<long long>(cdiv(n, 256), 4096)), dim3(256), 0,
                     as_stream(stream), w, branch_stride, 9 * nbranch, c, cin, wp);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_aspp_weight_grad(const float* dwp, int nbranch, int c, int cin, float* dw, msl_stream_t stream) {
  if (!dwp || !dw || nbranch < 1 || nbranch > 2 || c < 1 || cin < 1) return MSL_ERR_ARG;
  const long long n = 9LL * nbranch * c * cin;
  MSL_LAUNCH(k_aspp_weight_grad, dim3((unsigned)std::min<long long>(cdiv(n, 256), 4096)), dim3(256), 0,
                     as_stream(stream), dwp, 9 * nbranch, c, cin, dw);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_aspp_shift_add(const float* z, const float* bias, float* y, int nbranch, int c, int h, int w, int nimg,
                       int dil0, int dil1, msl_stream_t stream) {
  if (!z || !y || aspp_bad(nbranch, c, h, w, nimg, dil0, dil1)) return MSL_ERR_ARG;
  const int P = nimg * h * w;
  MSL_LAUNCH(k_aspp_shift_add, dim3(cdiv(P, 256), c), dim3(256), 0, as_stream(stream), z, bias, y,
                     9 * nbranch, c, h, w, P, dil0, dil1);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_aspp_shift_gather(const float* dy, float* g, float* dbias, int nbranch, int c, int h, int w, int nimg,
                          int dil0, int dil1, msl_stream_t stream) {
  if (!dy || !g || aspp_bad(nbranch, c, h, w, nimg, dil0, dil1)) return MSL_ERR_ARG;
  const int P = nimg * h * w;
  hipStream_t st = as_stream(stream);
  MSL_LAUNCH(k_aspp_shift_gather, dim3(cdiv(P, 256), 9 * nbranch * c), dim3(256), 0, st, dy, g, c, h, w, P,
                     dil0, dil1);
  MSL_CHECK_LAUNCH();
  if (dbias) {
    MSL_LAUNCH(k_aspp_bias_grad, dim3(c), dim3(256), 0, st, dy, P, dbias, c, nbranch);
    MSL_CHECK_LAUNCH();
  }
  return MSL_OK;
}

}  // extern "C"

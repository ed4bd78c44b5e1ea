// Standalone tuning harness for the dilated-conv implicit-GEMM kernels (not part of the library).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I maxsquareloss_amd/csrc -I scripts scripts/tune_dconv.hip -o scripts/tune_dconv
// Times tile / depth / split variants at the layer3 (d=2) and layer4 (d=4) shapes in one process
// and checks every variant against the first one.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "dconv_kernels.h"
#include "tune_x6_variants.h"

using namespace msl;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_reduce(const float* ws, int S, long long n, float* out) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float v = ws[i];
    for (int s = 1; s < S; ++s) v += ws[(long long)s * n + i];
    out[i] = v;
  }
}

static void fill(std::vector<float>& v, unsigned seed, float scale) {
  unsigned s = seed;
  for (auto& x : v) {
    s = s * 1664525u + 1013904223u;
    x = ((s >> 8) / 16777216.0f - 0.5f) * scale;
  }
}

struct Shape { int cin, cout, h, w, dil; };

template <int BM, int BN, int BK, int WM, int WN>
float run_fwd(const Shape& sh, const float* x, const float* wp, float* y, float* ws, int S, int iters, int lda) {
  const int P = sh.h * sh.w;
  FwdArgs a{};
  a.A = wp; a.B = x; a.C = S > 1 ? ws : y; a.bias = nullptr; a.nbias = 0;
  a.M = sh.cout; a.lda = lda; a.H = sh.h; a.W = sh.w; a.P = P; a.cimg = sh.cin;
  a.ncb = (sh.cin + 15) / 16; a.dil0 = sh.dil; a.dil1 = 0;
  const int groups = a.ncb * 9;
  a.ksteps = groups / (BK / 16);
  a.kps = (a.ksteps + S - 1) / S;
  a.slab = (long long)sh.cout * P; a.taps = 9;
  dim3 grid((P + BN - 1) / BN, (sh.cout + BM - 1) / BM, S);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_igemm_fwd<BM, BN, BK, WM, WN>), grid, dim3(256), 0, 0, a);
    if (S > 1) hipLaunchKernelGGL(k_reduce, dim3(2048), dim3(256), 0, 0, (const float*)ws, S, a.slab, y);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int BM, int BN, int STAGES, int WM, int WN>
float run_fwd_dma(const Shape& sh, const float* x, const float* wp, float* y, float* ws, int S, int iters, int lda) {
  const int P = sh.h * sh.w;
  FwdArgs a{};
  a.A = wp; a.B = x; a.C = S > 1 ? ws : y; a.bias = nullptr; a.nbias = 0;
  a.M = sh.cout; a.lda = lda; a.H = sh.h; a.W = sh.w; a.P = P; a.cimg = sh.cin;
  a.ncb = (sh.cin + 15) / 16; a.dil0 = sh.dil; a.dil1 = 0;
  a.ksteps = a.ncb * 9;
  a.kps = (a.ksteps + S - 1) / S;
  a.slab = (long long)sh.cout * P; a.taps = 9;
  dim3 grid((P + BN - 1) / BN, (sh.cout + BM - 1) / BM, S);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_igemm_fwd_dma<BM, BN, STAGES, WM, WN>), grid, dim3(256), 0, 0, a);
    if (S > 1) hipLaunchKernelGGL(k_reduce, dim3(2048), dim3(256), 0, 0, (const float*)ws, S, a.slab, y);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int BM, int BN, int G, int STAGES, int WM, int WN, int MT = 0, bool PW = false>
float run_fwd_sk(const Shape& sh, const float* x, const float* wp, float* y, float* ws, int NW, int iters, int lda, int* flags) {
  const int P = sh.h * sh.w;
  const int taps = PW ? 1 : 9;
  FwdArgs a{};
  a.A = wp; a.B = x; a.C = y; a.bias = nullptr; a.nbias = 0;
  a.M = sh.cout; a.lda = lda; a.H = sh.h; a.W = sh.w; a.P = P; a.cimg = sh.cin;
  a.ncb = (sh.cin + 15) / 16; a.dil0 = PW ? 0 : sh.dil; a.dil1 = 0;
  a.ksteps = a.ncb * taps; a.kps = a.ksteps; a.slab = 0; a.taps = taps;
  SkArgs sk{};
  sk.part = ws; sk.flags = flags;
  sk.tiles_m = (sh.cout + BM - 1) / BM; sk.tiles_n = (P + BN - 1) / BN; sk.KS = a.ksteps / G; sk.NW = NW;
  sk.T = sk.tiles_m * sk.tiles_n * sk.KS;
  const int tiles = sk.tiles_m * sk.tiles_n;
  if (sk.T / NW > 2 * sk.KS) { printf("NW too small\n"); return 1e9f; }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipMemset(flags, 0, 1 << 20));
  if (MT == kMathX6P || MT == kMathX6PP) {  // the weight planes are split at pack time (once per SGD step)
    a.Ax6 = ws + (size_t)NW * 2 * BM * BN;
    hipLaunchKernelGGL(k_split_pack, dim3(2048), dim3(256), 0, 0, wp, a.ksteps, lda, (__bf16*)a.Ax6);
  }
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    if (MT == kMathX6PP) {
      a.Bx6 = ws + (size_t)NW * 2 * BM * BN + (size_t)a.ksteps * 6 * lda * 4;
      hipLaunchKernelGGL(k_split_act, dim3(2048), dim3(256), 0, 0, x, a.cimg, a.ncb, P, (__bf16*)a.Bx6);
    }
    hipLaunchKernelGGL((k_igemm_fwd_sk<BM, BN, G, STAGES, WM, WN, PW, MT>), dim3(NW), dim3(256), 0, 0, a, sk);
    hipLaunchKernelGGL((k_sk_reduce<BM, BN>), dim3(BM * BN / 1024, tiles), dim3(256), 0, 0, a, sk);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<int> fl(tiles);
  CK(hipMemcpy(fl.data(), flags, tiles * 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < tiles; ++i) if (fl[i]) { printf("COUNTER NOT RE-ARMED tile %d\n", i); break; }
  return ms / iters;
}

template <bool PW, int EXP = 0, int V = 0>
float run_x6reg(const Shape& sh, const float* x, const float* wp, float* y, float* ws, int NW, int iters, int lda,
                bool reduce = true) {
  const int P = sh.h * sh.w;
  const int taps = PW ? 1 : 9;
  FwdArgs a{};
  a.A = wp; a.B = x; a.C = y; a.bias = nullptr; a.nbias = 0;
  a.M = sh.cout; a.lda = lda; a.H = sh.h; a.W = sh.w; a.P = P; a.cimg = sh.cin;
  a.ncb = (sh.cin + 15) / 16; a.dil0 = PW ? 0 : sh.dil; a.dil1 = 0;
  a.ksteps = a.ncb * taps; a.kps = a.ksteps; a.slab = 0; a.taps = taps;
  SkArgs sk{};
  sk.part = ws; sk.flags = nullptr;
  sk.tiles_m = (sh.cout + 127) / 128; sk.tiles_n = (P + 127) / 128; sk.KS = a.ksteps;
  sk.T = sk.tiles_m * sk.tiles_n * sk.KS;
  sk.NW = std::min(NW, sk.T);
  if (sk.T / sk.NW > 2 * sk.KS) { printf("NW too small\n"); return 1e9f; }
  const int tiles = sk.tiles_m * sk.tiles_n;
  a.Ax6 = ws + (size_t)NW * 2 * 128 * 128;
  hipLaunchKernelGGL(k_split_pack, dim3(2048), dim3(256), 0, 0, wp, a.ksteps, lda, (__bf16*)a.Ax6);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    if (V == 1) hipLaunchKernelGGL(k_x6_sk2, dim3(sk.NW), dim3(256), 0, 0, a, sk);
    else if (V == 3) hipLaunchKernelGGL(k_x6_sk4, dim3(sk.NW), dim3(512), 0, 0, a, sk);
    else if (V == 4) hipLaunchKernelGGL(k_x6_sk5, dim3(sk.NW), dim3(512), 0, 0, a, sk);
    else if (V == 2) hipLaunchKernelGGL(k_x6_sk3, dim3(sk.NW), dim3(256), 0, 0, a, sk);
    else hipLaunchKernelGGL(k_x6_sk<EXP>, dim3(sk.NW), dim3(256), 0, 0, a, sk);
    if (reduce) hipLaunchKernelGGL((k_sk_reduce<128, 128>), dim3(128 * 128 / 1024, tiles), dim3(256), 0, 0, a, sk);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int BM, int MT>
float run_rg(const Shape& sh, const float* x, const float* wp, float* y, float* ws, int NW, int iters, int lda) {
  const int P = sh.h * sh.w;
  FwdArgs a{};
  a.A = wp; a.B = x; a.C = y; a.bias = nullptr; a.nbias = 0;
  a.M = sh.cout; a.lda = lda; a.H = sh.h; a.W = sh.w; a.P = P; a.cimg = sh.cin;
  a.ncb = (sh.cin + 15) / 16; a.dil0 = sh.dil; a.dil1 = 0;
  a.ksteps = a.ncb * 9; a.kps = a.ksteps; a.slab = 0; a.taps = 9;
  SkArgs sk{};
  sk.part = ws; sk.flags = nullptr;
  sk.tiles_m = (sh.cout + BM - 1) / BM; sk.tiles_n = (P + 127) / 128; sk.KS = a.ncb * 3;
  sk.T = sk.tiles_m * sk.tiles_n * sk.KS;
  sk.NW = std::min(NW, sk.T);
  const int tiles = sk.tiles_m * sk.tiles_n;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_conv_rg<BM, 128, 2, 2, MT>), dim3(sk.NW), dim3(256), 0, 0, a, sk);
    hipLaunchKernelGGL((k_sk_reduce<BM, 128>), dim3(BM * 128 / 1024, tiles), dim3(256), 0, 0, a, sk);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int BM, int BN, int BK, int WM, int WN>
float run_wgrad(const Shape& sh, const float* x, const float* dy, float* dw, float* ws, int S, int iters) {
  const int P = sh.h * sh.w;
  WgradArgs a;
  a.dy = dy; a.x = x; a.C = S > 1 ? ws : dw; a.M = sh.cout; a.N = sh.cin; a.H = sh.h; a.W = sh.w; a.P = P;
  a.dil0 = sh.dil; a.dil1 = 0; a.ntap = 9; a.ksteps = (P + BK - 1) / BK; a.kps = (a.ksteps + S - 1) / S;
  a.accumulate = 0; a.taps = 9; a.slab = (long long)sh.cout * sh.cin * 9; a.cbranch = a.slab;
  dim3 grid((sh.cin + BN - 1) / BN, (sh.cout + BM - 1) / BM, S * 9);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_igemm_wgrad<BM, BN, BK, WM, WN>), grid, dim3(256), 0, 0, a);
    if (S > 1) hipLaunchKernelGGL(k_reduce, dim3(2048), dim3(256), 0, 0, (const float*)ws, S, a.slab, dw);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

template <int BM, int BN, int ST, int MT = 0>
float run_wgrad_sk(const Shape& sh, const float* x, const float* dy, float* dw, float* ws, int NWmax, int iters) {
  const int P = sh.h * sh.w;
  WskArgs a{};
  a.dy = dy; a.x = x; a.dw = dw; a.part = ws; a.M = sh.cout; a.N = sh.cin; a.H = sh.h; a.W = sh.w; a.P = P;
  a.dil0 = sh.dil; a.dil1 = 0; a.taps = 9; a.accumulate = 0; a.invW = 1.0f / sh.w;
  a.tiles_m = (sh.cout + BM - 1) / BM; a.tiles_n = (sh.cin + BN - 1) / BN; a.KS = (P + kWskBK - 1) / kWskBK;
  const int tiles = a.tiles_m * a.tiles_n * 9;
  a.T = tiles * a.KS; a.NW = std::min(NWmax, a.T); a.cbranch = (long long)sh.cout * sh.cin * 9;
  a.slots = ((a.T + a.NW - 1) / a.NW + a.KS - 2) / a.KS + 1;
  a.nchunk = 0; a.kchunk = 0; a.ntiles = tiles; a.dyx6 = nullptr; a.lda = 0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_wgrad_sk<BM, BN, ST, (BM >= 64 ? 2 : 1), (BM >= 64 ? 2 : 4), MT>), dim3(a.NW), dim3(256), 0, 0, a);
    hipLaunchKernelGGL((k_wsk_reduce<BM, BN>), dim3((BM * BN / 4 * 9 + 255) / 256, a.tiles_m * a.tiles_n), dim3(256), 0, 0, a);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

// k_split_rows + k_wgrad_x6 + k_wsk_reduce<128, 128> (the library's x6 weight gradient at >= 128 ch)
float run_wgrad_x6(const Shape& sh, const float* x, const float* dy, float* dw, float* ws, int NWmax, int iters,
                   bool split_only = false, int chunks = 0) {
  const int P = sh.h * sh.w;
  WskArgs a{};
  a.dy = dy; a.x = x; a.dw = dw; a.part = ws; a.M = sh.cout; a.N = sh.cin; a.H = sh.h; a.W = sh.w; a.P = P;
  a.dil0 = sh.dil; a.dil1 = 0; a.taps = 9; a.accumulate = 0; a.invW = 1.0f / sh.w;
  a.tiles_m = (sh.cout + 127) / 128; a.tiles_n = (sh.cin + 127) / 128; a.KS = (P + kWx6BK - 1) / kWx6BK;
  const int tiles = a.tiles_m * a.tiles_n * 9;
  a.T = tiles * a.KS; a.NW = std::min(NWmax, a.T); a.cbranch = (long long)sh.cout * sh.cin * 9;
  a.slots = ((a.T + a.NW - 1) / a.NW + a.KS - 2) / a.KS + 1;
  a.lda = (sh.cout + 127) / 128 * 128;
  a.nchunk = 0; a.kchunk = 0; a.ntiles = tiles;
  if (chunks > 0) {  // chunked split-K: tiles x chunks items, one piece each
    a.kchunk = (a.KS + chunks - 1) / chunks;
    a.nchunk = (a.KS + a.kchunk - 1) / a.kchunk;
    a.NW = tiles * a.nchunk;
    a.slots = 1;
  }
  const size_t piece_bytes = (size_t)a.NW * a.slots * 128 * 128 * 4;
  bf16x8* planes = (bf16x8*)((char*)ws + piece_bytes);
  a.dyx6 = planes;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_split_rows<kMathX6>, dim3(a.lda / 64, (a.KS + 3) / 4), dim3(256), 0, 0, dy, a.M, P, a.KS, a.lda, planes, (const float*)nullptr);
    if (split_only) continue;
    hipLaunchKernelGGL(k_wgrad_x6<kMathX6>, dim3(a.NW), dim3(256), 0, 0, a);
    hipLaunchKernelGGL((k_wsk_reduce<128, 128>), dim3(128 * 128 / 4 * 9 / 256, a.tiles_m * a.tiles_n), dim3(256), 0, 0, a);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

static double maxdiff(const float* a, const float* b, size_t n, double* scale) {
  std::vector<float> ha(n), hb(n);
  CK(hipMemcpy(ha.data(), a, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost));
  double m = 0, s = 0;
  for (size_t i = 0; i < n; ++i) { m = std::max(m, (double)std::fabs(ha[i] - hb[i])); s = std::max(s, (double)std::fabs(hb[i])); }
  *scale = s;
  return m;
}

static unsigned lcg(unsigned& s) { s = s * 1664525u + 1013904223u; return s >> 8; }

// fp64 forward reference at sampled (cout, pixel) outputs.  Weights are the tap-major pack:
// row k = (tap * ncb + ci / 16) * 16 + ci % 16, column cout, stride lda.  Error relative to the
// sum of |terms| of that output.
static void err64_fwd(const Shape& sh, const std::vector<float>& hx, const std::vector<float>& hw, int lda,
                      const float* dev, double* mx, double* rms, int taps = 9) {
  const int P = sh.h * sh.w, ncb = (sh.cin + 15) / 16;
  std::vector<float> hy((size_t)sh.cout * P);
  CK(hipMemcpy(hy.data(), dev, hy.size() * 4, hipMemcpyDeviceToHost));
  unsigned s = 12345;
  double m = 0, q = 0;
  const int NS = 3000;
  for (int i = 0; i < NS; ++i) {
    const int co = lcg(s) % sh.cout, p = lcg(s) % P;
    const int py = p / sh.w, px = p % sh.w;
    double acc = 0, mag = 0;
    for (int t = 0; t < taps; ++t) {
      const int yy = taps == 1 ? py : py + (t / 3 - 1) * sh.dil, xx = taps == 1 ? px : px + (t % 3 - 1) * sh.dil;
      if (yy < 0 || yy >= sh.h || xx < 0 || xx >= sh.w) continue;
      for (int ci = 0; ci < sh.cin; ++ci) {
        const double v = (double)hw[((size_t)(t * ncb + ci / 16) * 16 + ci % 16) * lda + co] *
                         (double)hx[(size_t)ci * P + yy * sh.w + xx];
        acc += v;
        mag += std::fabs(v);
      }
    }
    const double e = std::fabs((double)hy[(size_t)co * P + p] - acc) / (mag > 0 ? mag : 1.0);
    m = std::max(m, e);
    q += e * e;
  }
  *mx = m;
  *rms = std::sqrt(q / NS);
}

// fp64 weight-gradient reference at sampled (cout, cin, tap): dW = sum_p dY[co][p] X[ci][p + shift]
static void err64_wgrad(const Shape& sh, const std::vector<float>& hx, const std::vector<float>& hdy,
                        const float* dev, double* mx, double* rms) {
  const int P = sh.h * sh.w;
  std::vector<float> hd((size_t)sh.cout * sh.cin * 9);
  CK(hipMemcpy(hd.data(), dev, hd.size() * 4, hipMemcpyDeviceToHost));
  unsigned s = 777;
  double m = 0, q = 0;
  const int NS = 600;
  for (int i = 0; i < NS; ++i) {
    const int co = lcg(s) % sh.cout, ci = lcg(s) % sh.cin, t = lcg(s) % 9;
    const int dh = (t / 3 - 1) * sh.dil, dw = (t % 3 - 1) * sh.dil;
    double acc = 0, mag = 0;
    for (int p = 0; p < P; ++p) {
      const int yy = p / sh.w + dh, xx = p % sh.w + dw;
      if (yy < 0 || yy >= sh.h || xx < 0 || xx >= sh.w) continue;
      const double v = (double)hdy[(size_t)co * P + p] * (double)hx[(size_t)ci * P + yy * sh.w + xx];
      acc += v;
      mag += std::fabs(v);
    }
    const double e = std::fabs((double)hd[((size_t)co * sh.cin + ci) * 9 + t] - acc) / (mag > 0 ? mag : 1.0);
    m = std::max(m, e);
    q += e * e;
  }
  *mx = m;
  *rms = std::sqrt(q / NS);
}

int main(int argc, char** argv) {
  // "sk": only the library's stream-K configuration on the layer3 shape (profiling runs)
  const bool sk_only = argc > 1 && std::string(argv[1]) == "sk";
  // "fsk": every stream-K row, nothing else
  const bool fsk_only = argc > 1 && std::string(argv[1]) == "fsk";
  // "wsks": the small weight gradients of layers 1-2 (64 / 128 channels) by worker count
  const bool wsks = argc > 1 && std::string(argv[1]) == "wsks";
  const bool wsk_only = (argc > 1 && std::string(argv[1]) == "wsk") || wsks;
  // "x6": the matrix-core forms (f32, bf16, bf16x6) of the stream-K kernels vs an fp64 reference
  const bool x6_mode = argc > 1 && std::string(argv[1]) == "x6";
  // "rg": the row-grouped forward kernel (k_conv_rg) vs the stream-K one, every form, vs fp64
  const bool rg_mode = argc > 1 && std::string(argv[1]) == "rg";
  // "big": 256-row x6 tiles (wave tile 128x64) vs the 128-row ones, vs fp64
  const bool big_mode = argc > 1 && std::string(argv[1]) == "big";
  // "pw": the pointwise (1x1) GEMMs of layer3 / layer4, x6 forms, vs fp64
  const bool pw_mode = argc > 1 && std::string(argv[1]) == "pw";
  // "reg": the register-staged x6 kernel (k_x6_sk) vs the LDS-DMA x6p one, 3x3 and pointwise
  const bool reg3 = argc > 1 && std::string(argv[1]) == "reg3";  // profiling: layer3 shape only
  // "abl": k_x6_sk alone (no reduce) and its timing ablations, layer3 / layer4
  const bool abl = argc > 1 && std::string(argv[1]) == "abl";
  // "reg2": k_x6_sk2 (A fragments in registers) vs k_x6_sk vs the LDS-DMA kernel, vs fp64
  const bool reg4 = argc > 1 && std::string(argv[1]) == "reg4";  // k_x6_sk4 (two K-groups, NW 256)
  const bool reg5 = argc > 1 && std::string(argv[1]) == "reg5";  // k_x6_sk5 (16x16x32, 8 waves, NW 256)
  const bool reg2 = (argc > 1 && std::string(argv[1]) == "reg2") || reg4 || reg5;
  const bool reg_mode = (argc > 1 && std::string(argv[1]) == "reg") || reg3 || abl || reg2;
  // "wx6": the register-staged x6 weight gradient (k_wgrad_x6) vs k_wgrad_sk's x6 form, vs fp64
  const bool wx6 = argc > 1 && std::string(argv[1]) == "wx6";
  const int iters = sk_only ? 5 : 20;
  std::vector<Shape> shapes = {{256, 256, 65, 129, 2}, {256, 128, 64, 256, 2}, {256, 256, 64, 128, 2}, {512, 512, 65, 129, 4}};
  if (wsks) shapes = {{128, 128, 65, 129, 1}, {64, 64, 129, 257, 1}};
  if (pw_mode) shapes = {{1024, 256, 65, 129, 0}, {256, 1024, 65, 129, 0}, {2048, 512, 65, 129, 0}, {512, 2048, 65, 129, 0}};
  if (reg_mode) shapes = {{256, 256, 65, 129, 2}, {512, 512, 65, 129, 4}, {1024, 256, 65, 129, 0}, {256, 1024, 65, 129, 0},
                          {2048, 512, 65, 129, 0}};
  if (reg3) shapes = {{256, 256, 65, 129, 2}};
  if (wx6) shapes = {{256, 256, 65, 129, 2}, {512, 512, 65, 129, 4}, {128, 128, 65, 129, 1}, {256, 256, 17, 33, 2}};
  if (abl) shapes = {{256, 256, 65, 129, 2}, {512, 512, 65, 129, 4}, {1024, 256, 65, 129, 0}};
  const bool pwx = pw_mode || reg_mode;
  for (const Shape& sh : shapes) {
    if ((x6_mode || rg_mode || big_mode) && (sh.cin != sh.cout || sh.h != 65)) continue;  // layer3 / layer4 shapes
    const int P = sh.h * sh.w;
    const int lda = (sh.cout + 255) / 256 * 256;
    const bool shape_pw = pwx && sh.dil == 0;
    const long long kp = (long long)((sh.cin + 15) / 16) * (shape_pw ? 1 : 9) * 16;
    std::vector<float> hx((size_t)sh.cin * P), hw((size_t)kp * lda), hdy((size_t)sh.cout * P);
    fill(hx, 1, 2.f); fill(hw, 2, 0.02f); fill(hdy, 3, 2.f);
    if (getenv("TUNE_ZERO")) {  // all-zero operands: the same instructions at a lower power draw (DVFS probe)
      std::fill(hx.begin(), hx.end(), 0.f); std::fill(hw.begin(), hw.end(), 0.f); std::fill(hdy.begin(), hdy.end(), 0.f);
    }
    float *x, *wp, *dy, *y, *yref, *ws, *dw, *dwref;
    int* flags; CK(hipMalloc(&flags, 1 << 20));
    CK(hipMalloc(&x, hx.size() * 4)); CK(hipMalloc(&wp, hw.size() * 4)); CK(hipMalloc(&dy, hdy.size() * 4));
    CK(hipMalloc(&y, (size_t)sh.cout * P * 4)); CK(hipMalloc(&yref, (size_t)sh.cout * P * 4));
    CK(hipMalloc(&ws, std::max((size_t)16 * std::max((size_t)sh.cout * P, (size_t)sh.cout * sh.cin * 9) * 4, (size_t)1024 * 4 * 128 * 128 * 4)));
    CK(hipMalloc(&dw, (size_t)sh.cout * sh.cin * 9 * 4)); CK(hipMalloc(&dwref, (size_t)sh.cout * sh.cin * 9 * 4));
    CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(wp, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dy, hdy.data(), hdy.size() * 4, hipMemcpyHostToDevice));
    const double gf = 2.0 * sh.cin * sh.cout * (shape_pw ? 1 : 9) * P / 1e9;
    printf("=== shape cin %d cout %d %dx%d d=%d : %.2f GFLOP per conv\n", sh.cin, sh.cout, sh.h, sh.w, sh.dil, gf);
    if (reg_mode) {
      double mx, rms;
#define REG(PW, NW) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_x6reg<PW>(sh, x, wp, y, ws, NW, iters, lda); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms, PW ? 1 : 9); \
      printf("reg  PW %d       NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", PW, NW, ms * 1e3, gf / ms, mx, rms); }
#define OLD(PW) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_fwd_sk<128, 128, 1, 4, 2, 2, 3, PW>(sh, x, wp, y, ws, 512, iters, lda, flags); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms, PW ? 1 : 9); \
      printf("x6p  PW %d ST 4  NW  512 : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", PW, ms * 1e3, gf / ms, mx, rms); }
#define REG2(PW, NW) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_x6reg<PW, 0, 1>(sh, x, wp, y, ws, NW, iters, lda); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms, PW ? 1 : 9); \
      printf("reg2 PW %d       NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", PW, NW, ms * 1e3, gf / ms, mx, rms); }
#define REG3(PW, NW) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_x6reg<PW, 0, 2>(sh, x, wp, y, ws, NW, iters, lda); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms, PW ? 1 : 9); \
      printf("reg3 PW %d       NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", PW, NW, ms * 1e3, gf / ms, mx, rms); }
#define REG4(PW, NW) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_x6reg<PW, 0, 3>(sh, x, wp, y, ws, NW, iters, lda); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms, PW ? 1 : 9); \
      printf("reg4 PW %d       NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", PW, NW, ms * 1e3, gf / ms, mx, rms); }
#define REG5(PW, NW) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_x6reg<PW, 0, 4>(sh, x, wp, y, ws, NW, iters, lda); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms, PW ? 1 : 9); \
      printf("reg5 PW %d       NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", PW, NW, ms * 1e3, gf / ms, mx, rms); }
      if (reg5) {
        if (shape_pw) { OLD(true) REG5(true, 256) }
        else { OLD(false) REG5(false, 256) }
      } else if (reg4) {
        if (shape_pw) { OLD(true) REG2(true, 512) REG4(true, 256) }
        else { OLD(false) REG2(false, 512) REG4(false, 256) }
      } else if (reg2) {
        if (shape_pw) { OLD(true) REG(true, 512) REG2(true, 512) REG3(true, 512) }
        else { OLD(false) REG(false, 512) REG2(false, 512) REG3(false, 512) }
      } else if (abl) {
#define ABL(PW, EXP, what) { float ms = run_x6reg<PW, EXP>(sh, x, wp, y, ws, 512, iters, lda, false); \
        printf("abl  %-34s : %8.1f us %7.1f TF\n", what, ms * 1e3, gf / ms); }
#define ABLS(PW) ABL(PW, 0, "kernel only") ABL(PW, 1, "loads of K-step 0 only") ABL(PW, 2, "no MFMA") \
        ABL(PW, 4, "no global loads") ABL(PW, 8, "no piece/output stores") ABL(PW, 16, "no split") \
        ABL(PW, 6, "no loads, no MFMA") ABL(PW, 12, "no loads, no stores") ABL(PW, 14, "no loads/MFMA/stores") \
        ABL(PW, 30, "no loads/MFMA/stores/split") ABL(PW, 96, "A bypasses LDS") ABL(PW, 104, "A bypasses LDS, no stores") \
        ABL(PW, 110, "A bypasses LDS, no loads/MFMA/stores")
        if (shape_pw) { ABLS(true) } else { ABLS(false) }
      } else if (reg3) {
        OLD(false) REG(false, 512)
      } else if (shape_pw) {
        OLD(true) REG(true, 512) REG(true, 384) REG(true, 256)
      } else {
        OLD(false) REG(false, 512) REG(false, 384) REG(false, 256)
      }
      continue;
    }
    if (pw_mode) {
      double mx, rms;  // (no taps=9 reference launch in this mode: the weights are 1x1-sized)
#define FSKP(BM, BN, G, ST, WM, WN, NW, MT) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_fwd_sk<BM, BN, G, ST, WM, WN, MT, true>(sh, x, wp, y, ws, NW, iters, lda, flags); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms, 1); \
      printf("pw   MT %d BM %3d BN %3d G %d ST %d NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", MT, BM, BN, G, ST, NW, ms * 1e3, gf / ms, mx, rms); }
      FSKP(128, 128, 1, 4, 2, 2, 512, 3)
      if (sh.cout >= 256) { FSKP(256, 128, 1, 3, 2, 2, 256, 3) FSKP(256, 128, 1, 4, 2, 2, 256, 3) FSKP(256, 128, 2, 2, 2, 2, 256, 3) }
      continue;
    }
    double sc;
#define FWD(BM, BN, BK, WM, WN, S) { float ms = run_fwd<BM, BN, BK, WM, WN>(sh, x, wp, y, ws, S, iters, lda); \
      double md = maxdiff(y, yref, (size_t)sh.cout * P, &sc); \
      printf("fwd   BM %3d BN %3d BK %2d W %dx%d S %d : %8.1f us %7.1f TF  maxdiff %.2e/%.2e\n", BM, BN, BK, WM, WN, S, ms * 1e3, gf / ms, md, sc); }
    run_fwd<64, 128, 16, 2, 2>(sh, x, wp, yref, ws, 1, 1, lda);
    FWD(64, 128, 16, 2, 2, 1) FWD(64, 128, 16, 2, 2, 2)
#define FDMA(BM, BN, ST, WM, WN, S) { float ms = run_fwd_dma<BM, BN, ST, WM, WN>(sh, x, wp, y, ws, S, iters, lda); \
      double md = maxdiff(y, yref, (size_t)sh.cout * P, &sc); \
      printf("fdma  BM %3d BN %3d ST %2d W %dx%d S %d grid %5d : %8.1f us %7.1f TF  maxdiff %.2e/%.2e\n", BM, BN, ST, WM, WN, S, \
             ((P + BN - 1) / BN) * ((sh.cout + BM - 1) / BM) * S, ms * 1e3, gf / ms, md, sc); }
#define FSK(BM, BN, G, ST, WM, WN, NW) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); float ms = run_fwd_sk<BM, BN, G, ST, WM, WN>(sh, x, wp, y, ws, NW, iters, lda, flags); \
      double md = maxdiff(y, yref, (size_t)sh.cout * P, &sc); \
      printf("fsk   BM %3d BN %3d G %d ST %2d W %dx%d NW %4d : %8.1f us %7.1f TF  maxdiff %.2e/%.2e\n", BM, BN, G, ST, WM, WN, NW, ms * 1e3, gf / ms, md, sc); }
#define WGR(BM, BN, BK, WM, WN, S) { float ms = run_wgrad<BM, BN, BK, WM, WN>(sh, x, dy, dw, ws, S, iters); \
      double md = maxdiff(dw, dwref, (size_t)sh.cout * sh.cin * 9, &sc); \
      printf("wgrad BM %3d BN %3d BK %2d W %dx%d S %2d : %8.1f us %7.1f TF  maxdiff %.2e/%.2e\n", BM, BN, BK, WM, WN, S, ms * 1e3, gf / ms, md, sc); }
#define WSK(BM, BN, ST, NW) { float ms = run_wgrad_sk<BM, BN, ST>(sh, x, dy, dw, ws, NW, iters); \
      double md = maxdiff(dw, dwref, (size_t)sh.cout * sh.cin * 9, &sc); \
      printf("wsk   BM %3d BN %3d ST %d NW %4d : %8.1f us %7.1f TF  maxdiff %.2e/%.2e\n", BM, BN, ST, NW, ms * 1e3, gf / ms, md, sc); }
#define FSKE(BM, BN, G, ST, WM, WN, NW, MT) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_fwd_sk<BM, BN, G, ST, WM, WN, MT>(sh, x, wp, y, ws, NW, iters, lda, flags); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms); \
      printf("fsk  MT %d BM %3d BN %3d G %d ST %d NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", MT, BM, BN, G, ST, NW, ms * 1e3, gf / ms, mx, rms); }
#define WSKE(BM, BN, ST, NW, MT) { float ms = run_wgrad_sk<BM, BN, ST, MT>(sh, x, dy, dw, ws, NW, iters); \
      err64_wgrad(sh, hx, hdy, dw, &mx, &rms); \
      printf("wsk  MT %d BM %3d BN %3d ST %d NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", MT, BM, BN, ST, NW, ms * 1e3, gf / ms, mx, rms); }
    if (wx6) {
      double mx, rms;
      WSKE(128, 128, 2, 256, 2)
#define WX6(NW) { CK(hipMemset(dw, 0, (size_t)sh.cout * sh.cin * 9 * 4)); \
      float ms = run_wgrad_x6(sh, x, dy, dw, ws, NW, iters); \
      err64_wgrad(sh, hx, hdy, dw, &mx, &rms); \
      printf("wx6  (split+kernel+reduce) NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", NW, ms * 1e3, gf / ms, mx, rms); }
      WX6(512)
#define WX6C(C) { CK(hipMemset(dw, 0, (size_t)sh.cout * sh.cin * 9 * 4)); \
      float ms = run_wgrad_x6(sh, x, dy, dw, ws, 512, iters, false, C); \
      err64_wgrad(sh, hx, hdy, dw, &mx, &rms); \
      printf("wx6  chunked split-K  chunks %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", C, ms * 1e3, gf / ms, mx, rms); }
      {
        const int tiles = ((sh.cout + 127) / 128) * ((sh.cin + 127) / 128) * 9;
        const int c1 = std::max(1, 512 / tiles), c2 = std::max(1, 1024 / tiles);
        WX6C(c1) WX6C(c2)
      }
      printf("k_split_rows alone: %.1f us\n", run_wgrad_x6(sh, x, dy, dw, ws, 512, iters, true) * 1e3);
      continue;
    }
    if (rg_mode) {
      double mx, rms;
#define RGE(BM, NW, MT) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_rg<BM, MT>(sh, x, wp, y, ws, NW, iters, lda); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms); \
      printf("rg   MT %d BM %3d         NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", MT, BM, NW, ms * 1e3, gf / ms, mx, rms); }
      FSKE(128, 128, 2, 2, 2, 2, 512, 0) FSKE(128, 128, 1, 3, 2, 2, 512, 2) FSKE(128, 128, 2, 2, 2, 2, 512, 1)
      RGE(128, 512, 0) RGE(128, 256, 0) RGE(128, 512, 2) RGE(128, 256, 2) RGE(128, 512, 1) RGE(64, 768, 0) RGE(64, 512, 2)
      continue;
    }
    if (big_mode) {
      double mx, rms;
#define FSKB(BM, BN, G, ST, WM, WN, NW, MT) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_fwd_sk<BM, BN, G, ST, WM, WN, MT>(sh, x, wp, y, ws, NW, iters, lda, flags); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms); \
      printf("fsk  MT %d BM %3d BN %3d G %d ST %d NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", MT, BM, BN, G, ST, NW, ms * 1e3, gf / ms, mx, rms); }
      FSKB(128, 128, 1, 4, 2, 2, 512, 3)
      FSKB(256, 128, 1, 3, 2, 2, 256, 3) FSKB(256, 128, 1, 4, 2, 2, 256, 3) FSKB(256, 128, 1, 2, 2, 2, 256, 3)
      FSKB(256, 128, 1, 3, 2, 2, 512, 3) FSKB(256, 128, 2, 2, 2, 2, 256, 3)
      continue;
    }
    if (x6_mode) {
      double mx, rms;
#define FSKE(BM, BN, G, ST, WM, WN, NW, MT) { CK(hipMemset(y, 0, (size_t)sh.cout * P * 4)); \
      float ms = run_fwd_sk<BM, BN, G, ST, WM, WN, MT>(sh, x, wp, y, ws, NW, iters, lda, flags); \
      err64_fwd(sh, hx, hw, lda, y, &mx, &rms); \
      printf("fsk  MT %d BM %3d BN %3d G %d ST %d NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", MT, BM, BN, G, ST, NW, ms * 1e3, gf / ms, mx, rms); }
#define WSKE(BM, BN, ST, NW, MT) { float ms = run_wgrad_sk<BM, BN, ST, MT>(sh, x, dy, dw, ws, NW, iters); \
      err64_wgrad(sh, hx, hdy, dw, &mx, &rms); \
      printf("wsk  MT %d BM %3d BN %3d ST %d NW %4d : %8.1f us %7.1f TF  err64 max %.2e rms %.2e\n", MT, BM, BN, ST, NW, ms * 1e3, gf / ms, mx, rms); }
      {  // the per-call activation split of the x6pp rows, alone
        __bf16* planes = (__bf16*)(ws + (size_t)32 * 1024 * 1024);  // 128 MB in: ws is >= 268 MB
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        for (int it = -2; it < iters; ++it) {
          if (it == 0) CK(hipEventRecord(e0));
          hipLaunchKernelGGL(k_split_act, dim3(2048), dim3(256), 0, 0, x, sh.cin, (sh.cin + 15) / 16, P, planes);
        }
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("k_split_act alone: %.1f us\n", ms * 1e3 / iters);
      }
      FSKE(128, 128, 1, 4, 2, 2, 512, 3) FSKE(128, 128, 1, 3, 2, 2, 512, 4) FSKE(128, 128, 1, 4, 2, 2, 512, 4)
      FSKE(128, 128, 1, 5, 2, 2, 256, 4) FSKE(128, 128, 2, 2, 2, 2, 512, 4) FSKE(128, 128, 2, 3, 2, 2, 256, 4)
      WSKE(64, 64, 2, 512, 0) WSKE(64, 64, 2, 512, 1) WSKE(64, 64, 2, 512, 2)
      WSKE(128, 128, 2, 256, 0) WSKE(128, 128, 2, 256, 2) WSKE(64, 128, 2, 512, 2)
      continue;
    }
    if (wsks) {
      run_wgrad<64, 128, 32, 2, 2>(sh, x, dy, dwref, ws, 1, 1);
      WSK(64, 64, 2, 512) WSK(64, 64, 2, 384) WSK(64, 64, 2, 256) WSK(64, 64, 2, 192) WSK(64, 64, 2, 128)
      WSK(64, 64, 3, 256) WSK(64, 64, 3, 128)
      continue;
    }
    if (wsk_only) {
      run_wgrad<64, 128, 32, 2, 2>(sh, x, dy, dwref, ws, 1, 1);
      WGR(64, 128, 32, 2, 2, 8)
      WSK(128, 128, 2, 256) WSK(64, 128, 2, 256) WSK(64, 128, 2, 512) WSK(64, 64, 2, 512) WSK(64, 64, 3, 256)
      WSK(128, 64, 2, 256)
      continue;
    }
    if (sk_only) {
      FSK(128, 128, 2, 2, 2, 2, 512)
      break;
    }
    FSK(128, 128, 1, 3, 2, 2, 256) FSK(128, 128, 1, 3, 2, 2, 512)
    FSK(128, 128, 1, 2, 2, 2, 512) FSK(128, 128, 2, 2, 2, 2, 512) FSK(128, 128, 2, 2, 2, 2, 256)
    FSK(128, 128, 2, 3, 2, 2, 256) FSK(128, 128, 4, 2, 2, 2, 256)
    FSK(64, 128, 1, 3, 2, 2, 768) FSK(64, 128, 2, 2, 2, 2, 768) FSK(64, 128, 2, 2, 2, 2, 512)
    if (fsk_only) continue;
    FDMA(128, 128, 3, 2, 2, 1) FDMA(128, 128, 3, 2, 2, 2) FDMA(128, 128, 3, 2, 2, 3) FDMA(128, 128, 3, 2, 2, 4)
    FDMA(128, 128, 3, 2, 2, 6) FDMA(128, 128, 3, 2, 2, 8)
    FDMA(64, 128, 3, 2, 2, 1) FDMA(64, 128, 3, 2, 2, 2) FDMA(64, 128, 3, 2, 2, 3) FDMA(64, 128, 3, 2, 2, 4)
    FDMA(64, 64, 3, 2, 2, 1) FDMA(64, 64, 3, 2, 2, 2) FDMA(64, 64, 3, 2, 2, 3)
    run_wgrad<64, 128, 32, 2, 2>(sh, x, dy, dwref, ws, 1, 1);
    WGR(64, 128, 32, 2, 2, 8)
    CK(hipFree(x)); CK(hipFree(wp)); CK(hipFree(dy)); CK(hipFree(y)); CK(hipFree(yref)); CK(hipFree(ws)); CK(hipFree(dw)); CK(hipFree(dwref));
  }
  return 0;
}

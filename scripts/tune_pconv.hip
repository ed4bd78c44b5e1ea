// Standalone tuning harness for the pointwise (1x1) convs on the forward-form GEMM kernels.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I maxsquareloss_amd/csrc scripts/tune_pconv.hip -o scripts/tune_pconv
// C[M][P] = A^T B with A = packed weights [cimg][lda], B = image [cimg][P]; checked against a
// naive fp64-accumulating kernel.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "dconv_kernels.h"

using namespace msl;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_naive(const float* A, const float* B, float* C, int M, int K, int P, int lda) {
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= (long long)M * P) return;
  const int m = (int)(i / P), p = (int)(i % P);
  double s = 0;
  for (int k = 0; k < K; ++k) s += (double)A[(long long)k * lda + m] * B[(long long)k * P + p];
  C[i] = (float)s;
}

static void fill(std::vector<float>& v, unsigned seed, float scale) {
  unsigned s = seed;
  for (auto& x : v) {
    s = s * 1664525u + 1013904223u;
    x = ((s >> 8) / 16777216.0f - 0.5f) * scale;
  }
}

static double maxdiff(const float* a, const float* b, size_t n, double* scale) {
  std::vector<float> ha(n), hb(n);
  CK(hipMemcpy(ha.data(), a, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost));
  double md = 0, sc = 0;
  for (size_t i = 0; i < n; ++i) { md = std::max(md, (double)std::fabs(ha[i] - hb[i])); sc = std::max(sc, (double)std::fabs(hb[i])); }
  *scale = sc;
  return md;
}

struct Shape { int cimg, M, P; };

template <int BM, int BN, int G, int STAGES, bool PW, int MT = 0>
float run_sk(const Shape& sh, const float* x, const float* wp, float* y, float* ws, int* flags, int NW, int iters, int lda) {
  FwdArgs a{};
  a.A = wp; a.B = x; a.C = y; a.bias = nullptr; a.nbias = 0;
  a.M = sh.M; a.lda = lda; a.H = 1; a.W = sh.P; a.P = sh.P; a.cimg = sh.cimg;
  a.ncb = (sh.cimg + 15) / 16; a.dil0 = 0; a.dil1 = 0;
  a.ksteps = a.ncb; a.kps = a.ksteps; a.slab = 0; a.taps = 1;
  if (a.ksteps % G) return 1e9f;
  SkArgs sk{};
  sk.part = ws; sk.flags = flags;
  sk.tiles_m = (sh.M + BM - 1) / BM; sk.tiles_n = (sh.P + BN - 1) / BN; sk.KS = a.ksteps / G;
  sk.T = sk.tiles_m * sk.tiles_n * sk.KS;
  sk.NW = std::min(NW, sk.T);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipMemset(flags, 0, 1 << 20));
  for (int it = -2; it < iters; ++it) {
    if (it == 0) CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_igemm_fwd_sk<BM, BN, G, STAGES, 2, 2, PW, MT>), dim3(sk.NW), dim3(256), 0, 0, a, sk);
    hipLaunchKernelGGL((k_sk_reduce<BM, BN>), dim3(BM * BN / 1024, sk.tiles_m * sk.tiles_n), dim3(256), 0, 0, a, sk);
  }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

int main(int argc, char** argv) {
  // "x6": the current library configuration (f32, G2 ST2 NW512) against the bf16x6 form
  const bool x6_mode = argc > 1 && std::string(argv[1]) == "x6";
  const bool big_only = argc > 1 && !x6_mode;
  const int iters = 20;
  // (cimg, M, P): fwd of conv1/conv3/downsample and the dgrad forms (cimg = cout, M = cin)
  Shape shapes[] = {{4096, 4096, 4096}, {1024, 256, 8385}, {256, 1024, 8385}, {512, 1024, 8385}, {2048, 512, 8385},
                    {512, 2048, 8385}, {1024, 2048, 8385}, {256, 64, 33153}, {64, 256, 33153}};
  for (const Shape& sh : shapes) {
    const int lda = (sh.M + 127) / 128 * 128;
    const int kp = (sh.cimg + 15) / 16 * 16;
    std::vector<float> hx((size_t)sh.cimg * sh.P), hw((size_t)kp * lda, 0.f);
    fill(hx, 1, 2.f);
    { std::vector<float> t((size_t)sh.cimg * lda); fill(t, 2, 0.05f); std::copy(t.begin(), t.end(), hw.begin()); }
    float *x, *wp, *y, *yref, *ws; int* flags;
    CK(hipMalloc(&x, hx.size() * 4)); CK(hipMalloc(&wp, hw.size() * 4));
    CK(hipMalloc(&y, (size_t)sh.M * sh.P * 4)); CK(hipMalloc(&yref, (size_t)sh.M * sh.P * 4));
    CK(hipMalloc(&ws, (size_t)1024 * 2 * 128 * 128 * 4)); CK(hipMalloc(&flags, 1 << 20));
    CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(wp, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_naive, dim3((unsigned)(((long long)sh.M * sh.P + 255) / 256)), dim3(256), 0, 0, wp, x, yref, sh.M, sh.cimg, sh.P, lda);
    CK(hipDeviceSynchronize());
    const double gf = 2.0 * sh.cimg * sh.M * sh.P / 1e9;
    printf("=== cimg %d M %d P %d : %.2f GFLOP\n", sh.cimg, sh.M, sh.P, gf);
    double sc;
#define SK(BM, BN, G, ST, PW, NW) { CK(hipMemset(y, 0, (size_t)sh.M * sh.P * 4)); \
      float ms = run_sk<BM, BN, G, ST, PW>(sh, x, wp, y, ws, flags, NW, iters, lda); \
      double md = maxdiff(y, yref, (size_t)sh.M * sh.P, &sc); \
      printf("sk BM %3d BN %3d G %d ST %d PW %d NW %4d : %8.1f us %7.1f TF  maxdiff %.2e/%.2e\n", BM, BN, G, ST, (int)PW, NW, ms * 1e3, gf / ms, md, sc); }
#define SKM(BM, G, ST, NW, MT) { CK(hipMemset(y, 0, (size_t)sh.M * sh.P * 4)); \
      float ms = run_sk<BM, 128, G, ST, false, MT>(sh, x, wp, y, ws, flags, NW, iters, lda); \
      double md = maxdiff(y, yref, (size_t)sh.M * sh.P, &sc); \
      printf("sk MT %d BM %3d G %d ST %d NW %4d : %8.1f us %7.1f TF  maxdiff %.2e/%.2e\n", MT, BM, G, ST, NW, ms * 1e3, gf / ms, md, sc); }
    if (x6_mode) {
      if (sh.P == 4096) continue;
      if (sh.M >= 128) {
        SKM(128, 2, 2, 512, 0) SKM(128, 1, 3, 512, 2) SKM(128, 1, 3, 256, 2) SKM(128, 2, 2, 512, 2) SKM(128, 1, 4, 512, 2)
      } else {
        SKM(64, 2, 2, 512, 0) SKM(64, 1, 3, 512, 2)
      }
      continue;
    }
    if (sh.M >= 128) {
      SK(128, 128, 2, 2, false, 512) SK(128, 128, 2, 2, true, 512) SK(128, 128, 2, 3, true, 256)
      SK(128, 128, 4, 2, true, 256) SK(128, 128, 2, 2, true, 256) SK(128, 128, 1, 3, true, 512)
      SK(128, 128, 1, 4, true, 512)
    }
    SK(64, 128, 2, 2, true, 512) SK(64, 128, 2, 3, true, 512) SK(64, 128, 1, 4, true, 768)
    CK(hipFree(x)); CK(hipFree(wp)); CK(hipFree(y)); CK(hipFree(yref)); CK(hipFree(ws)); CK(hipFree(flags));
    if (big_only) break;
  }
  return 0;
}

// Bare MFMA loops on register-resident random bf16 operands: v_mfma_f32_32x32x16_bf16 (4
// accumulators of 32x32, a 64x64 wave tile) vs v_mfma_f32_16x16x32_bf16 (16 accumulators of
// 16x16, the same tile and FLOPs), 512 workgroups x 4 waves, six products per step as in the
// bf16x6 form.  Times both (wall) to see which shape the chip sustains faster under its clock
// management (MI355X_MICROARCH.md, DVFS item 7).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/mfma_shape_probe.hip -o scripts/mfma_shape_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ bf16x8 rnd8(unsigned s) {
  bf16x8 v;
  for (int j = 0; j < 8; ++j) {
    s = s * 1664525u + 1013904223u;
    v[j] = (__bf16)((float)(s >> 8) * (1.0f / 16777216.0f) - 0.5f);
  }
  return v;
}

__global__ void __launch_bounds__(256, 2) k32(float* out, int iters) {
  const unsigned seed = blockIdx.x * 256 + threadIdx.x;
  bf16x8 a[2][3], b[2][3];
  for (int i = 0; i < 2; ++i)
    for (int q = 0; q < 3; ++q) { a[i][q] = rnd8(seed * 7 + i * 3 + q); b[i][q] = rnd8(seed * 11 + i * 3 + q + 100); }
  f32x16 acc[2][2] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);
      }
  }
  float s = 0.f;
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 2; ++j) for (int r = 0; r < 16; ++r) s += acc[i][j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// same FLOPs per iteration: 16 blocks x 6 MFMAs of 16x16x32 (K = 32 = two 32x32x16 K-steps' worth)
// -> run iters/2 iterations
__global__ void __launch_bounds__(256, 2) k16(float* out, int iters) {
  const unsigned seed = blockIdx.x * 256 + threadIdx.x;
  bf16x8 a[4][3], b[4][3];
  for (int i = 0; i < 4; ++i)
    for (int q = 0; q < 3; ++q) { a[i][q] = rnd8(seed * 7 + i * 3 + q); b[i][q] = rnd8(seed * 11 + i * 3 + q + 100); }
  f32x4 acc[4][4] = {};
  for (int it = 0; it < iters / 2; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][0], c, 0, 0, 0);
      }
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) for (int r = 0; r < 4; ++r) s += acc[i][j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 512 * 256 * 4);
  const int iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double flops = 512.0 * 4 * iters * 4 * 6 * 2.0 * 32 * 32 * 16;  // per launch
  for (int rep = 0; rep < 3; ++rep) {
    for (int v = 0; v < 2; ++v) {
      for (int w = 0; w < 2; ++w) {  // warm the clock state with one launch first
        if (v == 0) hipLaunchKernelGGL(k32, dim3(512), dim3(256), 0, 0, out, iters);
        else hipLaunchKernelGGL(k16, dim3(512), dim3(256), 0, 0, out, iters);
      }
      hipEventRecord(e0);
      for (int k = 0; k < 10; ++k) {
        if (v == 0) hipLaunchKernelGGL(k32, dim3(512), dim3(256), 0, 0, out, iters);
        else hipLaunchKernelGGL(k16, dim3(512), dim3(256), 0, 0, out, iters);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s  %8.3f ms/launch  %7.1f TF (bf16 MFMA)\n", v == 0 ? "32x32x16" : "16x16x32", ms / 10, flops / (ms / 10 * 1e-3) / 1e12);
    }
  }
  return 0;
}

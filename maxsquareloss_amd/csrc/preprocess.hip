// Input pipeline on the device (HBM-bound byte work): the last two host steps of the reference
// loaders, run after a uint8 H2D copy (4x fewer PCIe bytes than the fp32 image, 8x than int64):
//   _img_transform (numpy_transform): RGB uint8 HWC -> float32, [:, :, ::-1] (BGR), -= IMG_MEAN,
//       transpose to CHW                       datasets/cityscapes_Dataset.py:14, 245-251
//   _mask_transform / id2trainId: label ids -> trainIds through a 256-entry table (ignore = -1),
//       the dataset's id_to_trainid composed with the 16 / 13-class remaps
//                                              cityscapes_Dataset.py:124-155, 260-264;
//                                              gta5_Dataset.py:73-75; synthia_Dataset.py:56-62
// plus the optional horizontal mirror of the random_mirror augmentation (cityscapes_Dataset.py
// _train_sync_transform: Image.FLIP_LEFT_RIGHT on image and mask alike).
// Both outputs are bit-exact: uint8 -> fp32 is exact and x - mean is one RNE fp32 subtraction,
// exactly what numpy does on the float32 array.
#include "msl_internal.h"

namespace msl {

// One thread = 4 consecutive output pixels of one row (w % 4 == 0): three dword loads of the 12
// source bytes, three float4 stores (one per channel plane).
__global__ void __launch_bounds__(256) k_image_transform_x4(const uint8_t* __restrict__ rgb, int h, int w,
                                                             int mirror, float m0, float m1, float m2,
                                                             float* __restrict__ out) {
  const long long hw = (long long)h * w;
  const long long nq = hw / 4;
  for (long long q = blockIdx.x * 256LL + threadIdx.x; q < nq; q += (long long)gridDim.x * 256) {
    const long long p = q * 4;
    const int y = (int)(p / w), x = (int)(p - (long long)y * w);
    const int xs = mirror ? w - 4 - x : x;  // first source pixel of the 4 (reversed when mirrored)
    const uint32_t* src = reinterpret_cast<const uint32_t*>(rgb + ((long long)y * w + xs) * 3);
    const uint32_t u0 = src[0], u1 = src[1], u2 = src[2];
    uint8_t b[12];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      b[k] = (u0 >> (8 * k)) & 0xff;
      b[4 + k] = (u1 >> (8 * k)) & 0xff;
      b[8 + k] = (u2 >> (8 * k)) & 0xff;
    }
    float v[3][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = mirror ? 3 - j : j;  // source pixel of output pixel x + j
      v[0][j] = __fsub_rn((float)b[3 * s + 2], m0);  // B
      v[1][j] = __fsub_rn((float)b[3 * s + 1], m1);  // G
      v[2][j] = __fsub_rn((float)b[3 * s + 0], m2);  // R
    }
#pragma unroll
    for (int c = 0; c < 3; ++c)
      *reinterpret_cast<float4*>(out + c * hw + p) = make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
  }
}

__global__ void __launch_bounds__(256) k_image_transform(const uint8_t* __restrict__ rgb, int h, int w,
                                                          int mirror, float m0, float m1, float m2,
                                                          float* __restrict__ out) {
  const long long hw = (long long)h * w;
  for (long long p = blockIdx.x * 256LL + threadIdx.x; p < hw; p += (long long)gridDim.x * 256) {
    const int y = (int)(p / w), x = (int)(p - (long long)y * w);
    const uint8_t* s = rgb + ((long long)y * w + (mirror ? w - 1 - x : x)) * 3;
    out[p] = __fsub_rn((float)s[2], m0);
    out[hw + p] = __fsub_rn((float)s[1], m1);
    out[2 * hw + p] = __fsub_rn((float)s[0], m2);
  }
}

// One thread = 4 consecutive label pixels of one row (w % 4 == 0): one dword of ids, the table in
// LDS, two 16-B stores of int64 trainIds.
__global__ void __launch_bounds__(256) k_label_transform_x4(const uint8_t* __restrict__ ids, int h, int w,
                                                             int mirror, const int32_t* __restrict__ lut,
                                                             int64_t* __restrict__ out) {
  __shared__ int32_t t[256];
  t[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const long long nq = (long long)h * w / 4;
  for (long long q = blockIdx.x * 256LL + threadIdx.x; q < nq; q += (long long)gridDim.x * 256) {
    const long long p = q * 4;
    const int y = (int)(p / w), x = (int)(p - (long long)y * w);
    const int xs = mirror ? w - 4 - x : x;
    const uint32_t u = *reinterpret_cast<const uint32_t*>(ids + (long long)y * w + xs);
    long long v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = t[(u >> (8 * (mirror ? 3 - j : j))) & 0xff];
    longlong2* o = reinterpret_cast<longlong2*>(out + p);
    o[0] = make_longlong2(v[0], v[1]);
    o[1] = make_longlong2(v[2], v[3]);
  }
}

__global__ void __launch_bounds__(256) k_label_transform(const uint8_t* __restrict__ ids, int h, int w, int mirror,
                                                          const int32_t* __restrict__ lut,
                                                          int64_t* __restrict__ out) {
  const long long hw = (long long)h * w;
  for (long long p = blockIdx.x * 256LL + threadIdx.x; p < hw; p += (long long)gridDim.x * 256) {
    const int y = (int)(p / w), x = (int)(p - (long long)y * w);
    out[p] = lut[ids[(long long)y * w + (mirror ? w - 1 - x : x)]];
  }
}

static int blocks_for(long long n) { return (int)std::min<long long>(std::max<long long>(cdiv(n, 256), 1), 8192); }

}  // namespace msl

using namespace msl;

extern "C" {

int msl_image_transform(const uint8_t* rgb, int h, int w, int mirror, float mean_b, float mean_g,
                        float mean_r, float* out, msl_stream_t stream) {
  if (!rgb || !out || h < 1 || w < 1 || (long long)h * w >= (1LL << 40)) return MSL_ERR_ARG;
  const long long hw = (long long)h * w;
  const bool vec = (w % 4) == 0 && (reinterpret_cast<uintptr_t>(rgb) & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (vec)
    MSL_LAUNCH(k_image_transform_x4, dim3(blocks_for(hw / 4)), dim3(256), 0, as_stream(stream), rgb, h,
                       w, mirror ? 1 : 0, mean_b, mean_g, mean_r, out);
  else
    MSL_LAUNCH(k_image_transform, dim3(blocks_for(hw)), dim3(256), 0, as_stream(stream), rgb, h, w,
                       mirror ? 1 : 0, mean_b, mean_g, mean_r, out);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_label_transform(const uint8_t* ids, int h, int w, int mirror, const int32_t* lut256, int64_t* out,
                        msl_stream_t stream) {
  if (!ids || !lut256 || !out || h < 1 || w < 1 || (long long)h * w >= (1LL << 40)) return MSL_ERR_ARG;
  const long long hw = (long long)h * w;
  const bool vec = (w % 4) == 0 && (reinterpret_cast<uintptr_t>(ids) & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (vec)
    MSL_LAUNCH(k_label_transform_x4, dim3(blocks_for(hw / 4)), dim3(256), 0, as_stream(stream), ids, h,
                       w, mirror ? 1 : 0, lut256, out);
  else
    MSL_LAUNCH(k_label_transform, dim3(blocks_for(hw)), dim3(256), 0, as_stream(stream), ids, h, w,
                       mirror ? 1 : 0, lut256, out);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

}  // extern "C"

// Training-time evaluation: the argmax of the upsampled prediction and the
// class confusion matrix, on device.  The reference copies the 19 x H x W fp32 prediction and the
// label to the host every iteration, takes np.argmax over classes and bins
// num_class * gt + pred with np.bincount (tools/train_source.py:280-283, utils/eval.py:109-115).
//
// One thread per pixel: first-max argmax over the C class planes (np.argmax's tie rule: the
// lowest index wins; a NaN logit is taken as the maximum, as numpy does), then the (gt, pred)
// cell of a per-block LDS histogram; each block adds its non-zero cells to the int64 matrix
// with integer atomics.  Counts are order-independent, so the result is exact and deterministic.
#include "msl_internal.h"

namespace msl {

constexpr int kEvalMaxClasses = 64;  // LDS histogram of C*C ints

__global__ void __launch_bounds__(256) k_confusion(const float* __restrict__ pred,
                                                   const long long* __restrict__ label, int C, long long P,
                                                   unsigned long long* __restrict__ cm,
                                                   int* __restrict__ argmax_out) {
  __shared__ unsigned int h[kEvalMaxClasses * kEvalMaxClasses];
  for (int i = threadIdx.x; i < C * C; i += 256) h[i] = 0u;
  __syncthreads();
  for (long long p = blockIdx.x * 256LL + threadIdx.x; p < P; p += (long long)gridDim.x * 256) {
    int best = 0;
    float bv = pred[p];
    if (!(bv != bv)) {  // a NaN at class 0 is the answer already
      for (int c = 1; c < C; ++c) {
        const float v = pred[(long long)c * P + p];
        if (v != v) { best = c; break; }
        if (v > bv) { bv = v; best = c; }
      }
    }
    if (argmax_out) argmax_out[p] = best;
    const long long g = label[p];
    if (g >= 0 && g < C) atomicAdd(&h[(int)g * C + best], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * C; i += 256)
    if (h[i]) atomicAdd(&cm[i], (unsigned long long)h[i]);
}

}  // namespace msl

using namespace msl;

extern "C" {

int msl_confusion_accumulate(const float* pred, const long long* label, int c, long long p,
                             unsigned long long* confusion, int* argmax_out, msl_stream_t stream) {
  if (!pred || !label || !confusion || c < 1 || c > kEvalMaxClasses || p < 1) return MSL_ERR_ARG;
  const int blocks = (int)std::min<long long>((p + 255) / 256, 2048);
  MSL_LAUNCH(k_confusion, dim3(blocks), dim3(256), 0, as_stream(stream), pred, label, c, p,
                     confusion, argmax_out);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

}  // extern "C"

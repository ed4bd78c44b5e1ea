// One-launch SGD step over every parameter of the model (HBM-bound: read p, g,
// m; write p, m), reproducing torch.optim.SGD's single-tensor loop as the
// reference drives it (train_source.py:139-144, :382-383 of solve_gta5.py):
//
//   for each entry of optim_parameters()  (deeplab_multi.py:132-171)
//       d = g + wd * p                      (grad.add(param, alpha=wd) -> fma)
//       buf = d                  on the parameter's first step (new buffer per entry)
//       buf = momentum * buf + d otherwise
//       p  = p - lr * buf                   (param.add_(buf, alpha=-lr) -> fma)
//
// get_1x_lr_params_NOscale lists most backbone parameters 3 or 4 times
// (quirk Q2); those k entries run sequentially on one element, so one thread
// applies the k updates in registers.  Parameters whose grad is None are not
// in the table (torch skips them).
#include "msl_internal.h"

namespace msl {

constexpr int kSgdBlockElems = 4096;

// buf * momentum + d with the product rounded on its own, as torch-CPU's buf.mul_(momentum).add_(d)
// (train_source.py:139-144 through torch.optim.SGD): HIP's __fmul_rn / __fadd_rn are the plain
// operators, which hipcc's -ffp-contract=fast may fuse into an fma; under contract(off) they are not
__device__ __forceinline__ float momentum_blend(float b, float mom, float d) {
#pragma clang fp contract(off)
  return b * mom + d;
}

__global__ void __launch_bounds__(256) k_sgd(const msl_sgd_entry* __restrict__ entries,
                                              const int32_t* __restrict__ block_entry,
                                              const long long* __restrict__ block_offset,
                                              float lr0, float lr1, const float* __restrict__ lr_dev,
                                              float mom, float wd, float gscale) {
  const msl_sgd_entry e = entries[block_entry[blockIdx.x]];
  const long long base = block_offset[blockIdx.x];
  const long long end = base + kSgdBlockElems < e.numel ? base + kSgdBlockElems : e.numel;
  // the learning rates by value, or from device memory (a replayed hipGraph: the poly schedule
  // changes them every iteration, train_source.py:706-717)
  const float lr = lr_dev ? lr_dev[e.group ? 1 : 0] : (e.group ? lr1 : lr0);
  const float nlr = -lr;
  for (long long i = base + threadIdx.x; i < end; i += 256) {
    float p = e.param[i];
    const float g = gscale == 1.f ? e.grad[i] : e.grad[i] * gscale;
    float b = e.has_buf ? e.momentum[i] : 0.f;
    for (int r = 0; r < e.mult; ++r) {
      const float d = __fmaf_rn(p, wd, g);
      b = e.has_buf ? momentum_blend(b, mom, d) : d;
      p = __fmaf_rn(b, nlr, p);
    }
    e.param[i] = p;
    e.momentum[i] = b;
  }
}

}  // namespace msl

using namespace msl;

extern "C" {

int msl_sgd_block_elems(void) { return kSgdBlockElems; }

long long msl_sgd_plan(const long long* numels, int n_entries, int32_t* block_entry_host,
                       long long* block_offset_host, long long max_blocks) {
  long long nb = 0;
  for (int i = 0; i < n_entries; ++i) {
    for (long long off = 0; off < numels[i]; off += kSgdBlockElems) {
      if (block_entry_host && block_offset_host) {
        if (nb >= max_blocks) return -1;
        block_entry_host[nb] = i;
        block_offset_host[nb] = off;
      }
      ++nb;
    }
  }
  return nb;
}

int msl_sgd_step(const msl_sgd_entry* entries, const int32_t* block_entry,
                 const long long* block_offset, long long n_blocks, float lr0, float lr1,
                 float momentum, float weight_decay, float grad_scale, msl_stream_t stream) {
  if (!entries || !block_entry || !block_offset || n_blocks < 0 || n_blocks > 0x7fffffff)
    return MSL_ERR_ARG;
  if (n_blocks == 0) return MSL_OK;
  MSL_LAUNCH(k_sgd, dim3((unsigned)n_blocks), dim3(256), 0, as_stream(stream), entries,
                     block_entry, block_offset, lr0, lr1, (const float*)nullptr, momentum, weight_decay,
                     grad_scale);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

int msl_sgd_step_lr_dev(const msl_sgd_entry* entries, const int32_t* block_entry,
                        const long long* block_offset, long long n_blocks, const float* lr_dev,
                        float momentum, float weight_decay, float grad_scale, msl_stream_t stream) {
  if (!entries || !block_entry || !block_offset || !lr_dev || n_blocks < 0 || n_blocks > 0x7fffffff)
    return MSL_ERR_ARG;
  if (n_blocks == 0) return MSL_OK;
  MSL_LAUNCH(k_sgd, dim3((unsigned)n_blocks), dim3(256), 0, as_stream(stream), entries,
                     block_entry, block_offset, 0.f, 0.f, lr_dev, momentum, weight_decay, grad_scale);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

}  // extern "C"

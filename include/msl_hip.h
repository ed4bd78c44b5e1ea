/*
 * msl_hip.h — C-ABI of libmsl_hip.so, the MI355X (gfx950) kernels behind the
 * DeepLabv2/ResNet-101 MaxSquare domain-adaptation training step.
 *
 * The reference (shiyutang/MaxSquareLoss) has no native code and no FFI: its
 * boundary is the Python/nn.Module API.  Every entry point
 * below replaces one implicit ATen/cuDNN op of that API; the reference site it
 * stands in for is cited next to it (paths relative to the reference root).
 *
 * Conventions (all entry points):
 *   - Tensors are fp32 NCHW with N = 1 (bs = 1 per GPU), i.e.
 *     a [C][H][W] block; labels are int64 with -1 = ignore.
 *   - All pointers are caller-owned device pointers (the PyTorch caching
 *     allocator on the Python side).  The library allocates nothing; scratch
 *     comes from the caller's workspace, sized by the matching *_workspace()
 *     query, and no call leaves state that a later call reads.
 *   - No process state (ABI 3): the kernel FORMS of a call - which matrix-core
 *     form, schedule or BN kernel runs, not what the result means - come with
 *     the call as a const msl_forms* (NULL = the defaults), read on the host
 *     at launch time, so a captured hipGraph keeps the forms of its capture.
 *   - Work is enqueued on the given hipStream_t (passed as msl_stream_t) and
 *     is stream-ordered; no entry point synchronises the host, so every call
 *     is safe to capture in a hipGraph.
 *   - Return value: 0 = MSL_OK, < 0 = argument / shape / workspace / launch-bound error
 *     (see msl_status_string), > 0 = the hipError_t of a failed launch.
 */
#ifndef MSL_HIP_H
#define MSL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* msl_stream_t; /* a hipStream_t */

#define MSL_OK 0
#define MSL_ERR_SHAPE (-1)
#define MSL_ERR_WORKSPACE (-2)
#define MSL_ERR_ARG (-3)
/* a launch whose block exceeds the kernel's __launch_bounds__: refused on the host, before the launch (r06) */
#define MSL_ERR_LAUNCH (-4)

int msl_abi_version(void);
const char* msl_status_string(int status);

/* The kernel forms of a call (ABI 3: replaces ABI 2's process-wide setters msl_conv_set_f32_form,
 * msl_conv_set_pack_form, msl_conv_set_sk_hybrid, msl_bn_set_fused and the reserved int* counters
 * argument, which no kernel read).  Every conv, pack and BN entry point takes one; NULL = the
 * defaults {5, 1, 1, 1}.  A bad value is MSL_ERR_ARG.
 *   f32_form  matrix-core form of the fp32 conv entry points (msl_dconv_* / msl_pconv_* without
 *             _bf16 / _f16) and of the packs: 0 = v_mfma_f32_32x32x2_f32 (exact fmaf chain), 2 = each
 *             fp32 operand split into three bf16 terms, six products per 16-deep K slice on
 *             v_mfma_f32_32x32x16_bf16 with fp32 accumulation (fp32-accurate), 5 = each operand tensor
 *             scaled by a power of two (its absolute maximum brought to [2^14, 2^15)) and split into
 *             two fp16 terms, three products per slice on v_mfma_f32_32x32x16_f16 with fp32
 *             accumulation, the result unscaled exactly (fp32-accurate: the 3xTF32 scheme at fp16's
 *             11-bit significand; the default).  Packs are form-specific (form 5 writes fp16 planes
 *             and the weights' scale): a conv call must pass the f32_form its pack was made with; the
 *             _f16 entry points need packs made with form 5.  Replaces nothing in the reference (its
 *             convs are cuDNN fp32).
 *   sk_hybrid schedule of the forward-form kernels (fwd and data gradient; same results up to the
 *             fp32 summation order of split tiles): 1 = when the output tiles outnumber the 512
 *             workgroups, whole rounds of tiles run data-parallel and only the remainder is split
 *             stream-K (default); 0 = pure stream-K.
 *   pack_form weight-pack kernel (identical packed bytes either way): 1 = one LDS-transposing
 *             pack+split launch per pack call (default), 0 = element-wise gather + separate split.
 *   bn_fused  BN kernel form: 1 = train-mode layers with p <= 16384 (or p <= 33792 and c >= 128) run
 *             one fused statistics+apply launch per call (one block per channel, operands held in
 *             registers; default), 0 = the split statistics / flat-apply launches everywhere. */
typedef struct msl_forms {
  int f32_form;
  int sk_hybrid;
  int pack_form;
  int bn_fused;
} msl_forms;
int msl_forms_default(msl_forms* out);       /* writes the defaults */
int msl_forms_check(const msl_forms* forms); /* MSL_OK (NULL included) or MSL_ERR_ARG */

/* ------------------------------------------------------------------------
 * Dilated 3x3 convolution, stride 1, padding = dilation, as an FP32-MFMA
 * implicit GEMM.  One call covers either a single conv (nbranch = 1:
 * Bottleneck.conv2 of layer3 d=2 / layer4 d=4, deeplab_multi.py:17-18,82-83)
 * or the live part of an ASPP head (nbranch = 2: conv_d6(x) + conv_d12(x) with
 * biases, Classifier_Module.forward, deeplab_multi.py:62-66 incl. quirk Q1).
 * Weights of branch b start at w + b*branch_stride, shape [cout][cin][3][3].
 * Images: x / y / dy / dx hold nimg images of h x w as [channels][nimg][h][w] (nimg = 1: the
 * reference's bs = 1 NCHW layout).  Each image is convolved on its own (a tap never reads across
 * into the neighbouring image); the weight gradient sums over all of them.  The trainer runs the
 * source and target images of an iteration as one pair (nimg = 2).
 * ---------------------------------------------------------------------- */

/* Elements (fp32 units) of the packed operand produced by msl_dconv_pack (for_dgrad = 0:
 * forward layout, 1: transposed + tap-flipped layout for the data gradient): the fp32 K-major
 * pack followed by its bf16x6 planes (split once here, read by the bf16x6 fp32 form; with form 5,
 * the fp16 planes and a tail holding the weights' scale).  All
 * nbranch branches are packed by one call (branch b's weights at w + b*branch_stride floats). */
long long msl_dconv_packed_elems(int nbranch, int cin, int cout, int for_dgrad);
/* One weight pack of a batch: exactly what msl_dconv_pack (taps 9) / msl_pconv_pack (taps 1,
 * nbranch 1, branch_stride 0) would write into `packed`. */
typedef struct msl_pack_job {
  const float* w;
  long long branch_stride;
  float* packed;
  int nbranch, cin, cout, for_dgrad;
} msl_pack_job;
/* Blocks of one job in msl_conv_pack_many (-1 on bad arguments). */
long long msl_conv_pack_blocks(int nbranch, int taps, int cin, int cout, int for_dgrad);
/* Every job of `jobs` (device array, all with the same tap count) in one launch: job j runs blocks
 * block_start[j] .. block_start[j+1]-1 (device array of njobs+1 ascending offsets built with
 * msl_conv_pack_blocks; block_start[njobs] = total_blocks).  Byte-identical to the per-job calls;
 * replaces the ~120 per-conv pack launches of a training step by two. */
int msl_conv_pack_many(const msl_pack_job* jobs, const long long* block_start, int njobs, int taps,
                       long long total_blocks, const msl_forms* forms, msl_stream_t stream);
int msl_dconv_pack(const float* w, long long branch_stride, int nbranch, int cin, int cout,
                   int for_dgrad, float* packed, const msl_forms* forms, msl_stream_t stream);

/* y[cout][h][w] = sum_b conv3x3(x, W_b, dil_b) (+ sum_b bias[b][cout] if bias)
 * replaces nn.Conv2d.forward at deeplab_multi.py:35 (layer3/4) and :63-65 (ASPP). */
size_t msl_dconv_fwd_workspace(int nbranch, int cin, int cout, int h, int w, int nimg);
int msl_dconv_fwd(const float* x, const float* packed, const float* bias, float* y, int nbranch,
                  int cin, int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                  size_t ws_bytes, msl_stream_t stream);

/* dx[cin][h][w] = sum_b conv3x3^T(dy, W_b, dil_b)   (autograd of the same sites) */
size_t msl_dconv_dgrad_workspace(int nbranch, int cin, int cout, int h, int w, int nimg);
int msl_dconv_dgrad(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin,
                    int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream);

/* dw[b][cout][cin][3][3] (= or += when accumulate) and, if dbias != NULL,
 * dbias[b][cout] = sum_px dy (identical for both branches). */
size_t msl_dconv_wgrad_workspace(int nbranch, int cin, int cout, int h, int w, int nimg);
int msl_dconv_wgrad(const float* x, const float* dy, float* dw, float* dbias, int nbranch, int cin,
                    int cout, int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * Pointwise (1x1, stride 1, no bias) convolution: the same FP32-MFMA GEMM
 * kernels with one unshifted tap over the flat pixel axis p = h*w.  Replaces
 * Bottleneck.conv1 / conv3 (deeplab_multi.py:13, 20) and the downsample conv
 * (deeplab_multi.py:96-99)
 * wherever their stride is 1 (layer1, layer3, layer4 and layer2 blocks 2-4).
 * Weights [cout][cin] (= [cout][cin][1][1]).
 * ---------------------------------------------------------------------- */
long long msl_pconv_packed_elems(int cin, int cout, int for_dgrad);
int msl_pconv_pack(const float* w, int cin, int cout, int for_dgrad, float* packed, const msl_forms* forms,
                   msl_stream_t stream);

/* y[cout][p] = sum_ci W[cout][ci] x[ci][p] */
size_t msl_pconv_fwd_workspace(int cin, int cout, int p);
int msl_pconv_fwd(const float* x, const float* packed, float* y, int cin, int cout, int p,
                  const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);

/* dx[cin][p] = sum_co W[co][cin] dy[co][p] */
size_t msl_pconv_dgrad_workspace(int cin, int cout, int p);
int msl_pconv_dgrad(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                    const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);
/* msl_pconv_dgrad with accumulate = 1: dx += W^T dy (dx read and written by the GEMM's own
 * epilogue / piece reduce; the bottleneck's residual gradient summed without a separate add).
 * accumulate = 0 is msl_pconv_dgrad.  Replaces autograd's grad accumulation at the block input
 * (Bottleneck.forward, deeplab_multi.py:31-48: conv1(x) and the identity residual both read x). */
int msl_pconv_dgrad_acc(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                        int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);
/* msl_pconv_dgrad_acc's sum with the identity residual's gradient formed in the epilogue (r06):
 * dx = mask(res) + W^T dy, mask(res)[c][n] = res[c][n] where the forward's y > 0 bit of that element is set
 * (res_mask: msl_bn_fwd_mask's bits, rows c * nimg + image, cdiv(p / nimg, 64) words each), else 0.  dx is
 * written, not read.  The bottleneck's bn3 backward (msl_bn_bwd_mask with dres = NULL) then need not write
 * that gradient; replaces autograd's residual accumulation at deeplab_multi.py:31-48 (x feeds conv1 and
 * the identity residual).  Workspace: msl_pconv_dgrad_workspace.  _sc: the dy partials as in the _sc
 * entry points; _f16: the fp16 math as msl_pconv_dgrad_f16. */
int msl_pconv_dgrad_resmask_sc(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                               const float* res, const unsigned long long* res_mask, int nimg, const msl_forms* forms,
                               void* ws, size_t ws_bytes, msl_stream_t stream, const float* dy_part, int dy_npart);
int msl_pconv_dgrad_resmask_f16(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                                const float* res, const unsigned long long* res_mask, int nimg, const msl_forms* forms,
                                void* ws, size_t ws_bytes, msl_stream_t stream, const float* dy_part, int dy_npart);

/* dw[cout][cin] (= or += when accumulate) = sum_p dy[cout][p] x[cin][p] */
size_t msl_pconv_wgrad_workspace(int cin, int cout, int p);
int msl_pconv_wgrad(const float* x, const float* dy, float* dw, int cin, int cout, int p,
                    int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * The stem and the strided glue of ResNetMulti (csrc/stem.hip), all gather forms without atomics
 * (bit-reproducible).  Replaces the last library kernels of the training step:
 *   - conv1 7x7 / stride 2 / pad 3 (deeplab_multi.py:73-74, 114) = msl_im2col into a
 *     [c*kh*kw][ho*wo] column matrix + msl_pconv_fwd with the [cout][c*kh*kw] weight (the conv
 *     weight as laid out); its weight gradient msl_pconv_wgrad on the same columns; its data
 *     gradient msl_pconv_dgrad into columns + msl_col2im (sums the columns back, i-major, j-minor);
 *   - MaxPool2d(3, 2, 1, ceil_mode=True) (deeplab_multi.py:77, 114): window [o*s - pad, +k) clipped
 *     to the image, first max in row-major scan (a NaN replaces), idx = y*w + x of the max; the
 *     caller passes ho/wo (torch's ceil-mode output size); the backward sums dy over the windows
 *     whose idx is the pixel, in (oy, ox) order (torch-CPU's order: bit-exact);
 *   - x[:, :, ::s, ::s] (the stride of layer2.0's 1x1 conv1 and downsample, deeplab_multi.py:12-13,
 *     96-99) and its transpose (zeros elsewhere) for the gradient.
 * ---------------------------------------------------------------------- */
/* im2col / col2im over nimg images: x [c][nimg][h][w], col [c*kh*kw][nimg][ho][wo].  The pooling
 * and subsample entry points are per plane: call them with c = channels * nimg. */
int msl_im2col(const float* x, int c, int h, int w, int nimg, int kh, int kw, int stride, int pad, int dil, int ho,
               int wo, float* col, msl_stream_t stream);
int msl_col2im(const float* col, int c, int h, int w, int nimg, int kh, int kw, int stride, int pad, int dil, int ho,
               int wo, float* x, msl_stream_t stream);
int msl_maxpool_fwd(const float* x, int c, int h, int w, int k, int stride, int pad, int ho, int wo, float* y,
                    int32_t* idx, msl_stream_t stream);
int msl_maxpool_bwd(const float* dy, const int32_t* idx, int c, int h, int w, int k, int stride, int pad, int ho,
                    int wo, float* dx, msl_stream_t stream);
int msl_subsample(const float* x, int c, int h, int w, int stride, int ho, int wo, float* y, msl_stream_t stream);
int msl_subsample_bwd(const float* dy, int c, int h, int w, int stride, int ho, int wo, float* dx,
                      msl_stream_t stream);

/* ------------------------------------------------------------------------
 * Operand scales of the f16x3 form (msl_forms.f32_form 5).  Each GEMM operand is scaled by a
 * power of two derived from absolute maxima and split into two fp16 terms.  The maxima come as
 * PER-ROW partials: msl_absmax_partials writes part[r] = max |x[r][.]| for each of the `rows` rows
 * (channels) of a [rows][row_len] tensor, and msl_bn_fwd_am / msl_bn_bwd_am write the same per-
 * channel maxima for the tensor a BN kernel produced.  The plain fp32 entry points reduce them
 * themselves; the _sc variants below take them from the caller as (pointer, count), count = the
 * operand's rows (its channels; NULL = compute), so a tensor read by two GEMMs (x by the forward
 * and the weight gradient, dy by the data and the weight gradient) is reduced once, or not at all
 * when a BN kernel produced it.  The forward / data gradient scale the image operand by one
 * tensor-wide power of two (the maximum of the partials: its rows are the GEMM's K index); the
 * weight gradient scales every row of dY and of x by its own power of two (both are output
 * indices there), so each dW element keeps the form's full precision even for channels far
 * below the tensor's maximum.  Partials must describe exactly the tensor passed (same contents).
 * The other forms ignore them.
 * ---------------------------------------------------------------------- */
int msl_absmax_partials(const float* x, int rows, int row_len, float* part, msl_stream_t stream);
int msl_dconv_fwd_sc(const float* x, const float* packed, const float* bias, float* y, int nbranch,
                     int cin, int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                     size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart);
int msl_dconv_dgrad_sc(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin,
                       int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                       size_t ws_bytes, msl_stream_t stream, const float* dy_part, int dy_npart);
int msl_dconv_wgrad_sc(const float* x, const float* dy, float* dw, float* dbias, int nbranch, int cin,
                       int cout, int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms, void* ws,
                       size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart,
                       const float* dy_part, int dy_npart);
int msl_pconv_fwd_sc(const float* x, const float* packed, float* y, int cin, int cout, int p,
                     const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part,
                     int x_npart);
int msl_pconv_dgrad_acc_sc(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                           int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream,
                           const float* dy_part, int dy_npart);
int msl_pconv_wgrad_sc(const float* x, const float* dy, float* dw, int cin, int cout, int p,
                       int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part,
                       int x_npart, const float* dy_part, int dy_npart);

/* ------------------------------------------------------------------------
 * ASPP heads as a pointwise GEMM plus shifts (csrc/aspp.hip; Classifier_Module.forward,
 * deeplab_multi.py:51-66, 84-85, quirk Q1: branches 0 and 1 with their biases).  With nt = 9*nbranch
 * taps t = b*9 + k (k = (dh/d_b + 1)*3 + dw/d_b + 1) and W' = the [nt*c][cin] weight
 * W'[t*c + m][ci] = W_b[m][ci][k]:
 *   forward   Z = W' x (msl_pconv_fwd*, M = nt*c), y = msl_aspp_shift_add(Z): y[m][p] = sum over t
 *             (in order) of Z[t*c + m][p + off_t] where the tap's source pixel is inside p's image, plus
 *             bias_0[m] + bias_1[m] (bias nullable);
 *   backward  G = msl_aspp_shift_gather(dY): G[t*c + m][q] = dY[m][q - off_t] where that pixel is inside
 *             q's image (else 0), dbias[b][m] = sum_p dY[m][p] (nullable); dx = W'^T G
 *             (msl_pconv_dgrad*), dW' = G x^T (msl_pconv_wgrad*), msl_aspp_weight_grad(dW') ->
 *             dw [nbranch][c][cin][3][3].
 * x / y / dY hold nimg images of h x w ([channels][nimg][h][w]); W_b at w + b*branch_stride.
 * ---------------------------------------------------------------------- */
int msl_aspp_weight_layout(const float* w, long long branch_stride, int nbranch, int c, int cin, float* wp,
                           msl_stream_t stream);
int msl_aspp_weight_grad(const float* dwp, int nbranch, int c, int cin, float* dw, msl_stream_t stream);
int msl_aspp_shift_add(const float* z, const float* bias, float* y, int nbranch, int c, int h, int w, int nimg,
                       int dil0, int dil1, msl_stream_t stream);
int msl_aspp_shift_gather(const float* dy, float* g, float* dbias, int nbranch, int c, int h, int w, int nimg,
                          int dil0, int dil1, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * BF16-MFMA forms of the six conv calls above (BASELINE config 5, "fp16/bf16 MFMA
 * path"): identical arguments, workspaces and output layout; the fp32 operands are
 * rounded to bf16 (RNE) as they are read from LDS and multiplied by
 * v_mfma_f32_32x32x16_bf16 with fp32 accumulation.  Same reference sites.
 * ---------------------------------------------------------------------- */
int msl_dconv_fwd_bf16(const float* x, const float* packed, const float* bias, float* y, int nbranch,
                       int cin, int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                       size_t ws_bytes, msl_stream_t stream);
int msl_dconv_dgrad_bf16(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin,
                         int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                         size_t ws_bytes, msl_stream_t stream);
int msl_dconv_wgrad_bf16(const float* x, const float* dy, float* dw, float* dbias, int nbranch,
                         int cin, int cout, int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms,
                         void* ws, size_t ws_bytes, msl_stream_t stream);
int msl_pconv_fwd_bf16(const float* x, const float* packed, float* y, int cin, int cout, int p,
                       const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);
int msl_pconv_dgrad_bf16(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout,
                         int p, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);
int msl_pconv_wgrad_bf16(const float* x, const float* dy, float* dw, int cin, int cout, int p,
                         int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * FP16-MFMA forms (BASELINE config 5's fp16 MFMA path): each operand tensor scaled by a power of
 * two (its absolute maximum into [2^14, 2^15)) and rounded to fp16 once - the weights at pack
 * time, as the hi planes of the f16x3 packs, so the packs must be made in the f16x3 fp32 form
 * (forms.f32_form 5, the default; MSL_ERR_ARG for another f32_form) - then one
 * v_mfma_f32_32x32x16_f16 per 16-deep K slice with fp32 accumulation, the result unscaled
 * exactly (M <= 64: 64-row fp16 tiles, r04; the weight gradients with fewer than 128 channels on either
 * side keep exact f32 MFMA tiles).  Operand partials as in
 * the _sc entry points ((pointer, count), NULL = computed); msl_pconv_dgrad_f16 carries the
 * accumulate flag of msl_pconv_dgrad_acc.  Same workspaces and results layout.
 * ---------------------------------------------------------------------- */
int msl_dconv_fwd_f16(const float* x, const float* packed, const float* bias, float* y, int nbranch, int cin,
                      int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws, size_t ws_bytes,
                      msl_stream_t stream, const float* x_part, int x_npart);
int msl_dconv_dgrad_f16(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin, int cout,
                        int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws, size_t ws_bytes,
                        msl_stream_t stream, const float* dy_part, int dy_npart);
int msl_dconv_wgrad_f16(const float* x, const float* dy, float* dw, float* dbias, int nbranch, int cin, int cout,
                        int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes,
                        msl_stream_t stream, const float* x_part, int x_npart, const float* dy_part, int dy_npart);
int msl_pconv_fwd_f16(const float* x, const float* packed, float* y, int cin, int cout, int p, const msl_forms* forms,
                      void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart);
int msl_pconv_dgrad_f16(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                        int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream,
                        const float* dy_part, int dy_npart);
int msl_pconv_wgrad_f16(const float* x, const float* dy, float* dw, int cin, int cout, int p, int accumulate, const msl_forms* forms,
                        void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart,
                        const float* dy_part, int dy_npart);
/* 1 if the weight gradient of this conv (taps 9: msl_dconv_wgrad*, h x w maps of nimg images;
 * taps 1: msl_pconv_wgrad* with p = nimg*h*w) runs the split kernel - whose fp16 form rounds both
 * operands to fp16 (one power-of-two scale per row) - and 0 if it runs an fp32-accurate tile
 * kernel (fewer than 128 channels on a side, or too few tiles to fill the chip).  A plan query,
 * no work: the fp16-operand emulation of the tests (oracle conv_f16) asks it.  MSL_ERR_ARG on bad
 * dimensions. */
int msl_conv_wgrad_split(int nbranch, int taps, int cin, int cout, int h, int w, int nimg);

/* ------------------------------------------------------------------------
 * Bilinear upsample, align_corners=True (F.interpolate at deeplab_multi.py:124,
 * :128).  The forward reproduces torch-CPU's rounding bit for bit.
 * ---------------------------------------------------------------------- */
int msl_upsample_fwd(const float* in, float* out, int c, int hi, int wi, int ho, int wo,
                     msl_stream_t stream);
size_t msl_upsample_bwd_workspace(int c, int hi, int wi, int ho, int wo);
int msl_upsample_bwd(const float* gout, float* gin, int c, int hi, int wi, int ho, int wo,
                     void* ws, size_t ws_bytes, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * Fused losses on the *low-resolution* logits [c][hi][wi]: each kernel
 * re-interpolates (bit-exact bilinear) to [c][ho][wo] on the fly, applies the
 * softmax and the loss, and the backward returns the gradient w.r.t. the
 * low-res logits directly (loss backward + softmax backward + upsample
 * backward in one pass, deterministic gather form).  hi == ho, wi == wo is the
 * identity interpolation, i.e. the plain hi-res loss.
 *
 * Every *_fwd writes a small device "stats" record consumed by *_bwd and the
 * loss scalar to out[0]; gout is a device pointer to dL/d(loss).
 * ---------------------------------------------------------------------- */
size_t msl_loss_workspace(int c, int hi, int wi, int ho, int wo);
int msl_loss_stats_elems(void); /* floats in a stats record */

/* nn.CrossEntropyLoss(ignore_index=-1) (train_source.py:128, solve_gta5.py:226-231).
 * out[0] = mean CE over valid pixels (nan if none, quirk Q8), stats = {sum, n_valid}. */
int msl_ce_up_fwd(const float* logits, const int64_t* labels, int c, int hi, int wi, int ho,
                  int wo, float* out, float* stats, void* ws, size_t ws_bytes,
                  msl_stream_t stream);
int msl_ce_up_bwd(const float* logits, const int64_t* labels, int c, int hi, int wi, int ho,
                  int wo, const float* stats, const float* gout, float* dlogits, void* ws,
                  size_t ws_bytes, msl_stream_t stream);

/* MaxSquareloss (utils/loss.py:104-119): out[0] = -sum(p^2) / (2*C*H*W). */
int msl_maxsquare_up_fwd(const float* logits, int c, int hi, int wi, int ho, int wo, float* out,
                         float* stats, void* ws, size_t ws_bytes, msl_stream_t stream);
int msl_maxsquare_up_bwd(const float* logits, int c, int hi, int wi, int ho, int wo,
                         const float* stats, const float* gout, float* dlogits, void* ws,
                         size_t ws_bytes, msl_stream_t stream);

/* IW_MaxSquareloss (utils/loss.py:69-102): hist = per-class count of argmax p
 * (int32, bit-exact), weights = 1/max(hist^r * (HW)^(1-r), 1),
 * out[0] = -sum_px w[argmax] * sum_c p^2 / C.  hist/weights may be NULL. */
int msl_iw_maxsquare_up_fwd(const float* logits, int c, int hi, int wi, int ho, int wo,
                            float ratio, float* out, float* stats, int32_t* hist,
                            float* weights, void* ws, size_t ws_bytes, msl_stream_t stream);
int msl_iw_maxsquare_up_bwd(const float* logits, int c, int hi, int wi, int ho, int wo,
                            const float* stats, const float* gout, float* dlogits, void* ws,
                            size_t ws_bytes, msl_stream_t stream);

/* Multi-level self-produced guidance (solve_gta5.py:206-213): P = softmax(up(x2)),
 * P2 = softmax(up(x1)), label2 = (max P > thr | max P2 > thr) ? argmax((P+P2)/2) : -1,
 * out[0] = CE(up(x1), label2) (mean over valid, nan if none).  The backward
 * returns d/d x1 only (label2 is detached in the reference). */
int msl_multi_ce_up_fwd(const float* logits1, const float* logits2, int c, int hi, int wi,
                        int ho, int wo, float thr, float* out, float* stats, void* ws,
                        size_t ws_bytes, msl_stream_t stream);
int msl_multi_ce_up_bwd(const float* logits1, const float* logits2, int c, int hi, int wi,
                        int ho, int wo, float thr, const float* stats, const float* gout,
                        float* dlogits1, void* ws, size_t ws_bytes, msl_stream_t stream);

/* The per-pixel decisions inside the fused losses, written out (parity inspection; argmax1 and
 * label2 are int32 [ho*wo], either nullable): argmax1 = first-max argmax of softmax(up(logits1))
 * (torch.max at loss.py:84-86 / the IW histogram's class), label2 = the multi-level guidance
 * label of msl_multi_ce_up_fwd with logits1 = x1, logits2 = x2 (solve_gta5.py:206-212). */
int msl_loss_labels_up(const float* logits1, const float* logits2, int c, int hi, int wi, int ho,
                       int wo, float thr, int32_t* argmax1, int32_t* label2, msl_stream_t stream);

/* Probability-input forms, for callers that hand the loss an explicit prob
 * tensor exactly as the reference API does (loss.py:76, :110).
 * prob is [c][hw]; label (nullable) is int64 [hw]. */
int msl_maxsquare_prob_fwd(const float* prob, int c, int hw, float* out, void* ws,
                           size_t ws_bytes, msl_stream_t stream);
int msl_maxsquare_prob_bwd(const float* prob, int c, int hw, const float* gout, float* dprob,
                           msl_stream_t stream);
int msl_iw_maxsquare_prob_fwd(const float* prob, const int64_t* label, int c, int hw,
                              float ratio, float* out, int32_t* hist, float* weights, void* ws,
                              size_t ws_bytes, msl_stream_t stream);
int msl_iw_maxsquare_prob_bwd(const float* prob, int c, int hw, const float* weights,
                              const float* gout, float* dprob, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * BatchNorm2d fused with the Bottleneck's ReLU / residual add (deeplab_multi.py:31-46,
 * :115-117): y = act(bn(x) [+ residual]), act = ReLU if relu else identity.
 * Layout [c][nimg][p]: nimg images of p = H*W pixels each.
 * training = 1: batch statistics over the p pixels of each channel of each image on its own
 * (bs = 1, quirk Q9: the reference's source and target forwards are separate batches),
 * accumulated in fp64; running stats updated with momentum and the unbiased variance when
 * update_running, image by image in order (exactly nimg sequential bs=1 calls);
 * num_batches_tracked (nullable) += nimg.  training = 0: running statistics (model.eval() /
 * --freeze_bn).  save_mean / save_invstd [c][nimg] are outputs consumed by msl_bn_bwd, which sums
 * dgamma / dbeta image by image in order (as nimg accumulating calls would).
 * ---------------------------------------------------------------------- */
size_t msl_bn_workspace(int c, int p, int nimg);
int msl_bn_fwd(const float* x, const float* gamma, const float* beta, const float* residual,
               float* y, float* running_mean, float* running_var, long long* num_batches_tracked,
               float* save_mean, float* save_invstd, int c, int p, int nimg, int training,
               int update_running, float momentum, float eps, int relu, const msl_forms* forms, void* ws,
               size_t ws_bytes, msl_stream_t stream);
/* dx (nullable), dres = d residual (nullable), dgamma / dbeta (nullable, = or += when
 * accumulate_params: the training step accumulates straight into the flat gradient buffer);
 * y is the forward output (needed when relu). */
int msl_bn_bwd(const float* dy, const float* x, const float* y, const float* gamma,
               const float* save_mean, const float* save_invstd, float* dx, float* dres,
               float* dgamma, float* dbeta, int c, int p, int nimg, int training, int relu,
               int accumulate_params, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream);
/* msl_bn_fwd / msl_bn_bwd that also write absmax[c] = max |y[c][.]| (forward) or max |dx[c][.]|
 * (backward; dx required): the per-channel absmax partials (c of them) that the f16x3 conv
 * entry points (_sc) take for the tensor this BN produced - the next conv's input, or the
 * gradient of the conv before it - so those GEMMs need no absmax pass of their own.  The fused
 * kernels reduce it in registers, the split forms in their apply kernel (r05; before: a pass of its
 * own over the output). */
int msl_bn_fwd_am(const float* x, const float* gamma, const float* beta, const float* residual,
                  float* y, float* running_mean, float* running_var, long long* num_batches_tracked,
                  float* save_mean, float* save_invstd, int c, int p, int nimg, int training,
                  int update_running, float momentum, float eps, int relu, const msl_forms* forms, void* ws,
                  size_t ws_bytes, msl_stream_t stream, float* absmax);
int msl_bn_bwd_am(const float* dy, const float* x, const float* y, const float* gamma,
                  const float* save_mean, const float* save_invstd, float* dx, float* dres,
                  float* dgamma, float* dbeta, int c, int p, int nimg, int training, int relu,
                  int accumulate_params, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, float* absmax_dx);
/* msl_bn_bwd_am that may take y = NULL with relu for a BN WITHOUT a residual: the fused kernel
 * then recomputes the ReLU mask from x (y > 0 <=> fma(x, invstd*gamma, fma(-mean, invstd*gamma,
 * beta)) > 0, the forward's own float operations on the saved mean / invstd, so the mask is
 * identical) instead of reading y - one read of the map less.  beta = the forward's beta
 * (nullable = 0).  y = NULL needs msl_bn_uses_fused(c, p, training) and p <= 16384 (else
 * MSL_ERR_ARG); with y given it is msl_bn_bwd_am. */
int msl_bn_bwd_am_beta(const float* dy, const float* x, const float* y, const float* gamma,
                       const float* beta, const float* save_mean, const float* save_invstd, float* dx,
                       float* dres, float* dgamma, float* dbeta, int c, int p, int nimg, int training,
                       int relu, int accumulate_params, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream,
                       float* absmax_dx);
/* 1 if msl_bn_fwd / msl_bn_bwd run the fused one-block-per-channel kernels for this shape (else the
 * split stats / reduce + flat apply kernels). */
int msl_bn_uses_fused(int c, int p, int training, const msl_forms* forms);
/* The ReLU mask as bits (r05): msl_bn_fwd_mask is msl_bn_fwd_am that also writes y > 0 of every
 * pixel to relu_mask (bit e % 64 of word [row][e / 64], rows c * nimg + image, cdiv(p, 64) words per
 * row: msl_bn_relu_mask_bytes); msl_bn_bwd_mask is msl_bn_bwd_am_beta with relu_mask in place of y,
 * the same mask bit for bit.  For the residual BN + ReLU of a bottleneck (deeplab_multi.py:45-47)
 * the backward then reads 1 bit per pixel instead of the 4-byte block output.  Both need relu and
 * msl_bn_uses_fused(c, p, training, forms) (else MSL_ERR_ARG). */
size_t msl_bn_relu_mask_bytes(int c, int p, int nimg);
int msl_bn_fwd_mask(const float* x, const float* gamma, const float* beta, const float* residual,
                    float* y, float* running_mean, float* running_var, long long* num_batches_tracked,
                    float* save_mean, float* save_invstd, int c, int p, int nimg, int training,
                    int update_running, float momentum, float eps, int relu, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream, float* absmax, uint64_t* relu_mask);
int msl_bn_bwd_mask(const float* dy, const float* x, const uint64_t* relu_mask, const float* gamma,
                    const float* beta, const float* save_mean, const float* save_invstd, float* dx, float* dres,
                    float* dgamma, float* dbeta, int c, int p, int nimg, int training, int relu,
                    int accumulate_params, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream,
                    float* absmax_dx);

/* ------------------------------------------------------------------------
 * Training-time evaluation (tools/train_source.py:280-283 + utils/eval.py:109-118): for one
 * image's prediction pred[c][p] (fp32, the upsampled logits) and label[p] (int64, pixels outside
 * [0, c) ignored), confusion[gt * c + argmax] += 1 over the pixels, on the stream;
 * argmax = np.argmax over classes (lowest index on ties, NaN wins).  argmax_out [p] (int32,
 * nullable) receives the per-pixel argmax.  c <= 64.  Exact, deterministic counts.
 * ---------------------------------------------------------------------- */
int msl_confusion_accumulate(const float* pred, const long long* label, int c, long long p,
                             unsigned long long* confusion, int* argmax_out, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * Input pipeline (the loaders' last host steps, on the device after a uint8 H2D copy; byte-exact):
 *   msl_image_transform: out[c][y][x] = (float)rgb[y][xs][2 - c] - mean[c] (BGR order, mean =
 *     IMG_MEAN = {B, G, R}), xs = mirror ? w-1-x : x; rgb is uint8 HWC, out fp32 CHW
 *     (datasets/cityscapes_Dataset.py:14, 245-251 _img_transform with numpy_transform; the
 *     random_mirror FLIP_LEFT_RIGHT of _train_sync_transform);
 *   msl_label_transform: out[y][x] = lut256[ids[y][xs]] as int64 (trainId, -1 = ignore): the
 *     dataset's id_to_trainid composed with its 16/13-class remap (cityscapes_Dataset.py:124-155,
 *     260-264 id2trainId / _mask_transform; gta5_Dataset.py:73-75; synthia_Dataset.py:56-62).
 *     lut256 is a device int32[256] table.
 * ---------------------------------------------------------------------- */
int msl_image_transform(const uint8_t* rgb, int h, int w, int mirror, float mean_b, float mean_g,
                        float mean_r, float* out, msl_stream_t stream);
int msl_label_transform(const uint8_t* ids, int h, int w, int mirror, const int32_t* lut256,
                        int64_t* out, msl_stream_t stream);

/* ------------------------------------------------------------------------
 * SGD step with the reference's duplicated-parameter semantics (quirk Q2):
 * torch.optim.SGD(momentum, weight_decay) single-tensor loop over the
 * optim_parameters() groups (train_source.py:139-144, deeplab_multi.py:132-171),
 * where a parameter listed k times receives k sequential updates sharing one
 * momentum buffer.  One launch updates every entry.
 * ---------------------------------------------------------------------- */
typedef struct msl_sgd_entry {
  float* param;       /* updated in place */
  const float* grad;  /* read-only */
  float* momentum;    /* momentum buffer, updated in place */
  long long numel;
  int mult;           /* occurrences of this parameter in its group (1, 3 or 4) */
  int group;          /* 0: backbone (lr), 1: ASPP heads (10*lr) */
  int has_buf;        /* 0 on the parameter's first step (buffer created = d) */
  int pad_;
} msl_sgd_entry;

/* entries and block_entry live in device memory; block_entry[b] is the entry
 * processed by block b (chunks of msl_sgd_block_elems() elements), built by
 * msl_sgd_plan on the host. */
int msl_sgd_block_elems(void);
long long msl_sgd_plan(const long long* numels, int n_entries, int32_t* block_entry_host,
                       long long* block_offset_host, long long max_blocks);
int msl_sgd_step(const msl_sgd_entry* entries, const int32_t* block_entry,
                 const long long* block_offset, long long n_blocks, float lr0, float lr1,
                 float momentum, float weight_decay, float grad_scale, msl_stream_t stream);
/* The same step with the two group learning rates read from device memory (lr_dev[0] = group 0,
 * lr_dev[1] = group 1) when the kernel runs, so a captured hipGraph replays the poly schedule
 * (train_source.py:706-717) by updating lr_dev between replays. */
int msl_sgd_step_lr_dev(const msl_sgd_entry* entries, const int32_t* block_entry,
                        const long long* block_offset, long long n_blocks, const float* lr_dev,
                        float momentum, float weight_decay, float grad_scale, msl_stream_t stream);

/* Diagnostics (r06): the launch guard every entry point runs before each kernel launch (MSL_ERR_LAUNCH
 * when a block exceeds the kernel's __launch_bounds__).  Launches a 256-thread-bound probe kernel with
 * `threads` threads writing out[t] = t: MSL_OK (and out[0 .. threads) written) for 1 <= threads <= 256,
 * MSL_ERR_LAUNCH (nothing launched, out untouched) above.  Replaces nothing in the reference. */
int msl_launch_guard_probe(int threads, float* out, msl_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MSL_HIP_H */

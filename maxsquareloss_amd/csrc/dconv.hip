// Dilated 3x3 convolution (stride 1, padding = dilation) as FP32-MFMA implicit
// GEMMs on gfx950.  Replaces the cuDNN/oneDNN convolutions of
//   - Bottleneck.conv2 in layer3 (d=2) and layer4 (d=4)   deeplab_multi.py:17-18, 82-83
//   - the live ASPP branches conv_d6 + conv_d12 (+bias)    deeplab_multi.py:51-66, 84-85
// forward, data gradient and weight gradient.
//
// Layout: activations are [C][P] fp32 with P = H*W (N = 1, NCHW).  The pixel
// axis is tiled linearly (not in 2-D blocks): 65x129 maps do not tile in 2-D
// without ~20 % waste, while 128-pixel linear tiles waste < 1 %.  A dilated tap
// is then a constant shift of the linear pixel index plus a per-pixel validity
// test (row wrap / image border), evaluated once per K-step per thread.
//
// GEMM mapping (MFMA v_mfma_f32_32x32x2_f32: exact f32 FMA chains):
//   forward / dgrad:  C[m][p] = sum_k A[k][m] * B[k][p]
//       k = ((branch*9 + tap)*ncb + cb)*16 + ci_local  (one tap, 16 channels per K-step;
//       tap-major, so the shifted-pixel offsets change only every ncb K-steps)
//       A = packed weights [Kp][lda] (m contiguous; dgrad: transposed + tap-flipped)
//       B = image[cb*16 + ci_local][p + shift(tap)]  (zero outside the image)
//   wgrad (one GEMM per tap, batched over grid.z):
//       dW[m][n][tap] = sum_p dY[m][p] * X[n][p + shift(tap)]   (K = pixels)
// Both operands are staged through LDS ([k][m] / [k][n], so every MFMA operand
// read is a conflict-free ds_read_b32 of 32 consecutive floats), double
// buffered, one barrier per K-step.  Small GEMMs are split along K into fp32
// slabs that a reduce kernel sums deterministically (fixed order).
#include "dconv_kernels.h"

namespace msl {

// out[i] = (acc ? out[i] : 0) + sum_s ws[s*n + i] (+ sum_b bias[b*M + i/bias_div])
__global__ void __launch_bounds__(256) k_reduce_slabs(const float* __restrict__ ws, int S, long long n,
                                                       float* __restrict__ out, int accumulate,
                                                       const float* __restrict__ bias, int nbias,
                                                       int bias_M, int bias_div) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float v = ws[i];
    for (int s = 1; s < S; ++s) v += ws[(long long)s * n + i];
    if (bias) {
      const int m = (int)(i / bias_div);
      float bsum = bias[m];
      for (int b = 1; b < nbias; ++b) bsum += bias[b * bias_M + m];
      v += bsum;
    }
    out[i] = accumulate ? out[i] + v : v;
  }
}

// msl_launch_guard_probe's kernel: out[t] = t (a 256-thread bound, like most of the library's kernels)
__global__ void __launch_bounds__(256) k_guard_probe(float* __restrict__ out) { out[threadIdx.x] = (float)threadIdx.x; }

// dbias[b][m] (=|+=) sum_p dy[m][p], same value for every branch b.
__global__ void __launch_bounds__(256) k_bias_grad(const float* __restrict__ dy, int P,
                                                    float* __restrict__ db, int M, int nbranch,
                                                    int accumulate) {
  const int m = blockIdx.x;
  float s = 0.f;
  for (int p = threadIdx.x; p < P; p += 256) s += dy[(long long)m * P + p];
  s = wave_sum(s);
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = (part[0] + part[1]) + (part[2] + part[3]);
    for (int b = 0; b < nbranch; ++b) db[b * M + m] = accumulate ? db[b * M + m] + tot : tot;
  }
}

// Packed operand for the forward-form GEMM.
//   for_dgrad = 0: image = x (cin channels),  m = co: P[k][co] = W[co][ci][t]
//   for_dgrad = 1: image = dy (cout channels), m = ci: P[k][ci] = W[co][ci][8 - t]
// k = ((b*taps + t)*ncb + cb)*16 + c_local with c = cb*16 + c_local (image channel); taps = 9
// for the 3x3 convs, 1 for the pointwise ones.
__global__ void __launch_bounds__(256) k_pack(const float* __restrict__ w, long long branch_stride,
                                               int cin, int cout, int for_dgrad, int ncb, int lda,
                                               int taps, long long total, float* __restrict__ out) {
  const int cimg = for_dgrad ? cout : cin;
  const int mreal = for_dgrad ? cin : cout;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int m = (int)(e % lda);
    const long long k = e / lda;
    const int cl = (int)(k % kCB);
    const long long q = k / kCB;
    const int cb = (int)(q % ncb);
    const long long q2 = q / ncb;
    const int t = (int)(q2 % taps);
    const int b = (int)(q2 / taps);
    const int c = cb * kCB + cl;
    float v = 0.f;
    if (c < cimg && m < mreal) {
      const float* wb = w + (long long)b * branch_stride;
      if (!for_dgrad)
        v = wb[((long long)m * cin + c) * taps + t];
      else
        v = wb[((long long)c * cin + m) * taps + (taps - 1 - t)];
    }
    out[e] = v;
  }
}

// The same pack through LDS, with the bf16x6 planes split in the same launch: one block per
// (16-row m chunk, channel block cb, branch) - 256 blocks for a 256x256 conv.  Both weight
// layouts read as contiguous runs (fwd: W[m][cb*16..+16][taps] = 16*taps floats per m; dgrad:
// W[c][m0..m0+16][taps] = 16*taps floats per c), the tile is transposed in LDS, and the writes
// are 64-B fp32 row segments and 256-B plane runs.  k_pack's per-element gather (a 36-B or
// cin*36-B lane stride) took 6 us for a 256x256x9 weight; the split was a second 4.6-us launch.
// (64-row chunks: 64 blocks for that weight, 24 us - too few workgroups.)
constexpr int kPackTileM = 16;

// One (16-row m chunk, 16-channel block, branch) block of the pack + split; s = the block's LDS tile.
template <int TAPS>
__device__ __forceinline__ void pack_split_block(const float* __restrict__ w, long long branch_stride, int cin,
                                                 int cout, int for_dgrad, int ncb, int lda, int split,
                                                 float* __restrict__ out, __bf16* __restrict__ planes, int mx,
                                                 int cb, int b, float (*s)[kPackTileM + 1],
                                                 float* __restrict__ tail = nullptr) {
  const int m0 = mx * kPackTileM;
  const int cimg = for_dgrad ? cout : cin;
  const int mreal = for_dgrad ? cin : cout;
  const float* wb = w + (long long)b * branch_stride;
  constexpr int N = kCB * TAPS * kPackTileM;
  for (int i = threadIdx.x; i < N; i += 256) {
    int ml, cl, tm;  // tm = memory tap
    if (!for_dgrad) {  // i = (ml*16 + cl)*TAPS + tm: W[m][c][tm] contiguous over (cl, tm)
      tm = i % TAPS;
      cl = (i / TAPS) % kCB;
      ml = i / (TAPS * kCB);
    } else {  // i = (cl*16 + ml)*TAPS + tm: W[c][m][tm] contiguous over (ml, tm)
      tm = i % TAPS;
      ml = (i / TAPS) % kPackTileM;
      cl = i / (TAPS * kPackTileM);
    }
    const int m = m0 + ml, c = cb * kCB + cl;
    float v = 0.f;
    if (m < mreal && c < cimg)
      v = for_dgrad ? wb[((long long)c * cin + m) * TAPS + tm] : wb[((long long)m * cin + c) * TAPS + tm];
    const int t = for_dgrad ? TAPS - 1 - tm : tm;
    s[cl * TAPS + t][ml] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += 256) {  // i = (t*16 + cl)*16 + ml
    const int ml = i % kPackTileM, cl = (i / kPackTileM) % kCB, t = i / (kPackTileM * kCB);
    const long long k = ((long long)(b * TAPS + t) * ncb + cb) * kCB + cl;
    out[k * lda + m0 + ml] = s[cl * TAPS + t][ml];
  }
  if (!split) return;
  if (tail) {  // f16x3: two fp16 planes of W * sA; {sA, 1/sA} written by k_pack_scale* before this launch
    const float sc = tail[kNPart];
    f16x8* pl = reinterpret_cast<f16x8*>(planes);
    for (int i = threadIdx.x; i < TAPS * 2 * kPackTileM; i += 256) {
      const int ml = i % kPackTileM, h = (i / kPackTileM) & 1, t = i / (2 * kPackTileM);
      const long long ks = (long long)(b * TAPS + t) * ncb + cb;
      Split2h sp;
#pragma unroll
      for (int j = 0; j < 8; ++j) split2h_set(sp, j, s[(8 * h + j) * TAPS + t][ml] * sc);
      const long long row = ((ks * 2) * 2 + h) * lda + m0 + ml;  // plane 0
      pl[row] = sp.hi;
      pl[row + 2LL * lda] = sp.lo;
    }
    return;
  }
  bf16x8* pl = reinterpret_cast<bf16x8*>(planes);
  for (int i = threadIdx.x; i < TAPS * 2 * kPackTileM; i += 256) {  // i = (t*2 + h)*16 + ml
    const int ml = i % kPackTileM, h = (i / kPackTileM) & 1, t = i / (2 * kPackTileM);
    const long long ks = (long long)(b * TAPS + t) * ncb + cb;
    Split3 sp;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_set(sp, j, s[(8 * h + j) * TAPS + t][ml]);
    const long long row = ((ks * 3) * 2 + h) * lda + m0 + ml;  // plane 0 (k_split_pack layout)
    pl[row] = sp.hi;
    pl[row + 2LL * lda] = sp.mid;
    pl[row + 4LL * lda] = sp.lo;
  }
}

template <int TAPS>
__global__ void __launch_bounds__(256) k_pack_split(const float* __restrict__ w, long long branch_stride,
                                                    int cin, int cout, int for_dgrad, int ncb, int lda,
                                                    int split, float* __restrict__ out,
                                                    __bf16* __restrict__ planes, float* __restrict__ tail) {
  __shared__ float s[kCB * TAPS][kPackTileM + 1];  // [cl*TAPS + t][ml], t = packed tap index
  pack_split_block<TAPS>(w, branch_stride, cin, cout, for_dgrad, ncb, lda, split, out, planes, blockIdx.x,
                         blockIdx.y, blockIdx.z, s, tail);
}

// Packed-buffer tail (after the fp32 pack and its planes): the f16x3 form's kNPart absmax
// partials of the weights, then {sA, 1/sA}.
constexpr long long kPackTail = 320;
__host__ __device__ inline long long pack_tail_offset(long long f32_elems) { return f32_elems * 5 / 2; }

// f16x3 weight absmax of every job (grid = (kNPart, njobs)) into each job's pack tail
template <int TAPS>
__global__ void __launch_bounds__(256) k_absmax_jobs(const msl_pack_job* __restrict__ jobs) {
  const msl_pack_job jb = jobs[blockIdx.y];
  const int cimg = jb.for_dgrad ? jb.cout : jb.cin;
  const int m = jb.for_dgrad ? jb.cin : jb.cout;
  const long long f32 = (long long)jb.nbranch * ((cimg + kCB - 1) / kCB) * TAPS * kCB * ((m + kPackPad - 1) / kPackPad * kPackPad);
  absmax_block(jb.w, (long long)jb.cout * jb.cin * TAPS, jb.branch_stride, jb.nbranch, blockIdx.x,
               jb.packed + pack_tail_offset(f32) + blockIdx.x);
}

// {sA, 1/sA} of a pack from its kNPart weight absmax partials, once per pack (the pack blocks read
// sA: every one of them reducing the 256 partials itself read 4x its own 1-KB tile - 0.44 ms per
// step for the ~170k blocks of the step's packs, r03)
__device__ __forceinline__ void pack_scale(float* __restrict__ tail) {
  float inv;
  const float sc = pow2_scale(partials_max(tail, kNPart, threadIdx.x & 63), inv);
  if (threadIdx.x == 0) {
    tail[kNPart] = sc;
    tail[kNPart + 1] = inv;
  }
}
__global__ void __launch_bounds__(64) k_pack_scale(float* __restrict__ tail) { pack_scale(tail); }
template <int TAPS>
__global__ void __launch_bounds__(64) k_pack_scale_jobs(const msl_pack_job* __restrict__ jobs) {
  const msl_pack_job jb = jobs[blockIdx.x];
  const int cimg = jb.for_dgrad ? jb.cout : jb.cin;
  const int m = jb.for_dgrad ? jb.cin : jb.cout;
  const long long f32 = (long long)jb.nbranch * ((cimg + kCB - 1) / kCB) * TAPS * kCB * ((m + kPackPad - 1) / kPackPad * kPackPad);
  pack_scale(jb.packed + pack_tail_offset(f32));
}

// (m chunk, channel block) tiles per block of the batched pack: a pointwise tile is only 256 floats
// (one per thread), and the ~300k one-tile blocks of a step's pointwise packs took 288 us (r03)
template <int TAPS>
constexpr int kPackSub() { return TAPS == 1 ? 8 : 1; }

// Every weight pack of a step in one launch (per tap count): block b runs block b - start[j] of
// job j (start[] ascending, start[njobs] = the total), each job exactly as msl_*_pack would.
template <int TAPS>
__global__ void __launch_bounds__(256) k_pack_split_many(const msl_pack_job* __restrict__ jobs,
                                                         const long long* __restrict__ start, int njobs, int h3) {
  __shared__ float s[kCB * TAPS][kPackTileM + 1];
  const long long b = blockIdx.x;
  int lo = 0, hi = njobs - 1;  // the last job with start <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (start[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const msl_pack_job jb = jobs[lo];
  const int cimg = jb.for_dgrad ? jb.cout : jb.cin;
  const int m = jb.for_dgrad ? jb.cin : jb.cout;
  const int lda = (m + kPackPad - 1) / kPackPad * kPackPad;
  const int ncb = (cimg + kCB - 1) / kCB;
  const int nmx = lda / kPackTileM;
  const long long tiles = (long long)nmx * ncb * jb.nbranch;
  const long long f32 = (long long)jb.nbranch * ncb * TAPS * kCB * lda;
  constexpr int SUB = kPackSub<TAPS>();
#pragma unroll 1
  for (int sub = 0; sub < SUB; ++sub) {
    const long long local = (b - start[lo]) * SUB + sub;
    if (local >= tiles) break;  // block-uniform
    if (sub) __syncthreads();   // the previous tile's LDS reads are done
    const int mx = (int)(local % nmx);
    const long long rest = local / nmx;
    const int cb = (int)(rest % ncb), br = (int)(rest / ncb);
    pack_split_block<TAPS>(jb.w, jb.branch_stride, jb.cin, jb.cout, jb.for_dgrad, ncb, lda, m > 64 || h3, jb.packed,
                           reinterpret_cast<__bf16*>(jb.packed + f32), mx, cb, br, s,
                           h3 ? jb.packed + pack_tail_offset(f32) : nullptr);
  }
}

// ---------------------------------------------------------------- planning
// Forward form (fwd and dgrad) runs stream-K (k_igemm_fwd_sk): 128-pixel tiles of 128, 64 or
// 32 rows (by M: the ASPP forward has 19 classes), two K-steps per LDS stage, up to 512
// persistent workgroups (2 per CU), so every CU gets the same number of MFMA stages whatever
// the tile count.  The split-K tile kernel remains for an odd K-step count with M <= 32.
constexpr int kSkBN = 128, kSkNW = 512;
// The call's forms (msl_forms, r05: per call, no process state): sk_hybrid = the forward-form
// schedule (1: data-parallel rounds + stream-K remainder when the tiles outnumber the workers,
// SkArgs; 0: pure stream-K); f32_form = the matrix-core form of the fp32 entry points: kMathF32 runs
// v_mfma_f32_32x32x2_f32 (an exact fmaf chain), kMathX6 the three-way bf16 split on the BF16
// matrix cores (fp32-accurate, dconv_kernels.h; layer3 fwd 78 vs 102 us in the step, err vs fp64
// 4e-8 vs 6e-8 relative to sum|terms|), kMathH3P the scaled two-way fp16 split (three fp16
// MFMAs per slice; dconv_kernels.h Split2h); packs are form-specific.
static_assert(kMathF32 == 0 && kMathX6 == 2 && kMathH3P == 5, "msl_forms.f32_form values");

struct FwdPlan {
  bool sk;
  int G;  // stream-K: K-steps per stage
  int bm, bn, bk, tiles_m, tiles_n, ksteps, kps, S;
  int bmx;  // r06: the f16x3 pointwise GEMM's wide-tile rows (256; 0 = none), its pieces sized for them
};

// r06: f16x3 pointwise GEMMs with M a multiple of 256 from kPw256MinM on 256 x 128 tiles, 1 x 4 waves (each 256 rows
// x 32 pixels, its A fragments streamed row block by row block): the image operand read once per 256 rows.  Same box
// (profiles/r06_wide_tiles_ab.txt): 512 -> 2048 fwd 109 vs 118 us, 2048 -> 512 dgrad 120 vs 128; at M = 1024 even,
// at M <= 512 slower (fewer tiles than workers: 1024 -> 256 fwd 54 vs 48, 2048 -> 512 fwd 129 vs 107).  A 384-row
// tile for the ASPP heads (M = 342: the operand read once instead of three times) needs 192 accumulator registers
// per lane and spilled 96-188 VGPRs at one or two waves per SIMD: not built.
constexpr int kPw256MinM = 2048;
static int wide_rows(int taps, int M) { return taps == 1 && M % 256 == 0 && M >= kPw256MinM ? 256 : 0; }

static int pad_to(int v, int a) { return (v + a - 1) / a * a; }

static int choose_split(int tiles, int ksteps, int min_steps) {
  const int target = 512;  // 256 CUs x 2 resident workgroups
  if (tiles >= 384) return 1;
  int S = (target + tiles - 1) / tiles;
  S = std::max(1, std::min(S, ksteps / min_steps));
  return S;
}

static FwdPlan plan_fwd(int nbranch, int taps, int cimg, int M, int P, bool has_bias) {
  FwdPlan pl;
  const int groups = nbranch * cdiv(cimg, kCB) * taps;
  const int bm = M > 64 ? 128 : (M > 32 ? 64 : 32);
  pl.sk = groups % 2 == 0 || bm > 32;
  pl.bmx = pl.sk ? wide_rows(taps, M) : 0;
  if (pl.sk) {
    pl.G = groups % 2 == 0 ? 2 : 1;
    pl.bm = bm;
    pl.bn = kSkBN;
    pl.bk = pl.G * kCB;
    pl.tiles_m = cdiv(M, pl.bm);
    pl.tiles_n = cdiv(P, pl.bn);
    pl.ksteps = groups;
    pl.kps = groups / pl.G;  // stages per tile
    pl.S = 1;
    return pl;
  }
  pl.G = 1;
  pl.bm = 64;
  pl.bn = 128;
  pl.bk = 16;
  pl.tiles_m = cdiv(M, pl.bm);
  pl.tiles_n = cdiv(P, pl.bn);
  pl.ksteps = groups;
  int S = choose_split(pl.tiles_m * pl.tiles_n, pl.ksteps, 4);
  pl.kps = cdiv(pl.ksteps, S);
  pl.S = cdiv(pl.ksteps, pl.kps);
  return pl;
}

// Weight gradient: stream-K over (tile, 64-pixel stage) (k_wgrad_sk + k_wsk_reduce).  Tiles by
// shape (the r01 tuning harness, profiles/r01_tune_wsk*.txt): 128x128 at one workgroup per CU for the
// 512-channel layer4 convs, 64x64 at two per CU below, 32-row tiles for the 19-class ASPP.
struct WgradPlan {
  int bm, bn, nw, tiles_m, tiles_n, ntap, KS, slots;
  bool rx6;        // k_wgrad_x6 (register-staged bf16x6, dY pre-split) with 16-pixel K-steps
  int lda;         // rx6: dY plane row length
  int nchunk, kchunk;  // rx6: chunked split-K (items = tiles x nchunk, kchunk K-steps each)
  long long T;
};

// k_wgrad_x6 with chunked split-K: the chunk count whose (tile, chunk) items fill whole rounds of
// 512 resident workgroups best, at least 8 K-steps per item.  Returns the fill (0 if none).
static double plan_chunks(long long ntiles, int KS, int& nchunk, int& kchunk) {
  double best = 0.0;
  nchunk = kchunk = 0;
  for (int C = 1; C <= KS && ntiles * C <= 4096; ++C) {
    const int L = cdiv(KS, C);
    if (L < 8) break;
    const int Ce = cdiv(KS, L);
    const long long items = ntiles * Ce;
    const double eff = (double)items / (double)(cdiv(items, 512LL) * 512);
    if (eff > best + 0.01) {
      best = eff;
      nchunk = Ce;
      kchunk = L;
    }
  }
  return best;
}

static WgradPlan plan_wgrad(int nbranch, int taps, int cin, int cout, int P, bool x6 = false, int w = 0) {
  WgradPlan pl;
  pl.rx6 = false;
  pl.lda = 0;
  pl.nchunk = 0;
  pl.kchunk = 0;
  int bk = kWskBK;
  const int ntap = nbranch * taps;
  int nchunk = 0, kchunk = 0;
  const bool rx6_ok = x6 && cout >= 128 && cin >= 128 && w >= 16;
  const double fill = rx6_ok ? plan_chunks((long long)cdiv(cout, 128) * cdiv(cin, 128) * ntap, cdiv(P, kWx6BK),
                                           nchunk, kchunk) : 0.0;
  if (rx6_ok && (fill >= 0.75 || (cout >= 256 && cin >= 256))) {
    // x6, >= 128 channels: k_wgrad_x6 (dY split once, 16-pixel K-steps, two workgroups per CU),
    // chunked split-K when its items fill the resident slots (layer3 77.6 us, layer4 274,
    // layer2 38.8; stream-K 86.5 / 306 / 44.1; k_wgrad_sk 110 / 395 / 41.0 -
    // profiles/r02_wgrad_x6.txt), else stream-K over 512 workers
    pl.bm = 128; pl.bn = 128; pl.nw = 512;
    pl.rx6 = true;
    pl.lda = pad_to(cout, kPackPad);
    bk = kWx6BK;
    if (fill >= 0.75) {
      pl.nchunk = nchunk;
      pl.kchunk = kchunk;
    }
  } else if (x6 && cout >= 128 && cin >= 128) {
    pl.bm = 128; pl.bn = 128; pl.nw = 256;
  } else if (cout <= 32) {
    pl.bm = 32; pl.bn = 128; pl.nw = 256;
  } else if (cout >= 512 && cin >= 512) {
    pl.bm = 128; pl.bn = 128; pl.nw = 256;
  } else {
    // layers 1-2 (<= 128 channels): 256 workers, fewer pieces per tile for the reduce (layer2
    // 41.5 vs 44.3 us, layer1 44.1 vs 47.7; profiles/r01_tune_wsks.txt)
    pl.bm = 64; pl.bn = 64; pl.nw = (cout <= 128 && cin <= 128) ? 256 : 512;
  }
  pl.tiles_m = cdiv(cout, pl.bm);
  pl.tiles_n = cdiv(cin, pl.bn);
  pl.ntap = ntap;
  pl.KS = cdiv(P, bk);
  pl.T = (long long)pl.tiles_m * pl.tiles_n * pl.ntap * pl.KS;
  pl.nw = (int)std::min<long long>(pl.nw, pl.T);
  // tiles a worker range can touch: its length (<= ceil(T/NW) stages) starting anywhere in a tile
  pl.slots = (int)((cdiv(pl.T, (long long)pl.nw) + pl.KS - 2) / pl.KS + 1);
  if (pl.nchunk > 0) {  // one piece per (tile, chunk) item
    pl.nw = (int)((long long)pl.tiles_m * pl.tiles_n * pl.ntap * pl.nchunk);
    pl.slots = 1;
  }
  return pl;
}

static size_t wgrad_piece_bytes(const WgradPlan& pl) { return (size_t)pl.nw * pl.slots * pl.bm * pl.bn * sizeof(float); }
// (+ two K-steps: k_wgrad_x6's loads one stage ahead read up to K-step KS + 1, unused)
static size_t wgrad_planes_bytes(const WgradPlan& pl) { return pl.rx6 ? (size_t)(pl.KS + 2) * 6 * pl.lda * 16 : 0; }

// stream-K workspace: the published pieces, NW x 2 x BM*BN floats (summed by k_sk_reduce; no
// flags or other state survive a call).
// + (f16x3) the image's kNPart absmax partials at the end of the caller's workspace.
constexpr size_t kPartBytes = kNPart * sizeof(float);
// stream-K pieces, then (the BP form) the image operand's fp16 planes, then the partials at the end
static size_t fwd_piece_bytes(const FwdPlan& pl) {
  // (the <= 64-row f16x3 / fp16 3x3 tiles run 64 rows: room for those pieces whatever the form; the 256-row
  // pointwise tiles twice the 128-row pieces - r05's 256 / 384-row attempt kept the 128-row size, and its
  // pieces ran past the workspace into the image partials behind them)
  return align_up((size_t)kSkNW * 2 * std::max(pl.bmx, std::max(pl.bm, 64)) * pl.bn * sizeof(float), 256);
}
static size_t img_planes_bytes(int cimg, int P) { return align_up((size_t)cdiv(cimg, kCB) * kCB * P * 4, 256); }
// The f16x3 / fp16 forward-form GEMMs that read their image operand pre-split (k_split_img, BP form):
// the 3x3 ones with M >= 512 (profiles/r03_bp_ab.txt); fp16 math (one plane: a quarter of the loads'
// instructions, half their bytes) from M >= 128 (r05)
// r06: the 3x3 GEMMs with M >= kBqMinM read the pre-split image in the 2 x 2 wave layout (BQ: 64 rows x 64
// pixels per wave, half the A-fragment LDS reads per MFMA of the 1 x 4 layout, no split in the loop)
constexpr int kBqMinM = 1 << 30;
static bool bq_form(int taps, int M, bool small_f16) { return taps == 9 && !small_f16 && M >= kBqMinM; }

// The stream-K schedule of a forward-form launch over at most nw_max workers (see launch_fwd_form)
static SkArgs plan_sk(int tiles_m, int tiles_n, int KS, int nw_max, int hybrid, float* part) {
  SkArgs sk{};
  sk.part = part;
  sk.tiles_m = tiles_m;
  sk.tiles_n = tiles_n;
  sk.KS = KS;
  const long long tiles = (long long)tiles_m * tiles_n;
  sk.tdp = (hybrid && tiles >= nw_max) ? (int)(tiles / nw_max * nw_max) : 0;
  sk.gm = sk.tdp > 0 ? tiles_m : 1;
  const long long T = (tiles - sk.tdp) * KS;
  sk.NW = (int)std::min<long long>(nw_max, T);
  constexpr long long kSkMinIt = 8;
  if (sk.tdp > 0) sk.NW = (int)std::max<long long>(1, std::min<long long>(sk.NW, T / kSkMinIt));
  sk.T = (int)T;
  return sk;
}
static bool bp_form(int taps, int M, bool small_f16, bool h1 = false) {
  return taps == 9 && !small_f16 && (M >= 512 || (h1 && M >= 128) || bq_form(taps, M, small_f16));
}
static size_t fwd_ws_bytes(const FwdPlan& pl, int M, int P, int cimg, int taps) {
  // the planes only where the BP form can run (the stem / pointwise calls reserved them too).  The
  // query is form-independent (the forms come with the call, not with the query), so a 3x3 GEMM with
  // 128 <= M < 512 reserves the image planes that only the fp16 math's BP form reads (cimg x P x 4 bytes, e.g.
  // ~17 MB at layer2's pair shape) in every form: conservative, accepted
  if (pl.sk) return fwd_piece_bytes(pl) + (bp_form(taps, M, false, true) ? img_planes_bytes(cimg, P) : 0) + kPartBytes;
  return (pl.S > 1 ? (size_t)pl.S * M * P * sizeof(float) : 0) + kPartBytes;
}
static float* ws_partials(void* ws, size_t ws_bytes, int k) {  // k-th partials block from the end
  return reinterpret_cast<float*>((char*)ws + ((ws_bytes - (size_t)k * kPartBytes) & ~(size_t)15));
}

// The forward-form kernel, plain or with the accumulate epilogue (a template form of its own)
template <int BM, int G, int ST, int WM, int WN, int MT, bool PW = false>
static int launch_sk(int accum, dim3 grid, dim3 block, hipStream_t st, const FwdArgs& a, const SkArgs& sk,
                      bool bp = false) {
  if constexpr (MT == kMathH3P || MT == kMathH1P) {  // held to two waves per SIMD (k_igemm_fwd_sk2)
    if constexpr (!PW && BM == 128 && G == 1 && ST == 4 && WM == 2 && WN == 2) {
      // the 2 x 2 pre-split form (BQ, r06): 3x3 GEMMs only, never accumulating
      if (bp && !accum) {
        MSL_LAUNCH((k_igemm_fwd_sk2<BM, kSkBN, G, ST, WM, WN, PW, MT, false, true, true>), grid, block, 0, st,
                           a, sk);
        return MSL_OK;
      }
    }
    if constexpr (!PW && (BM == 128 || BM == 64) && G == 1 && ST == 4 && WM == 1 && WN == 4) {
      // (accumulating BD / BP forms at 64 rows only: the pointwise M <= 64 data gradients; no 3x3 call
      // accumulates, and the 128-row accumulating 3x3 forms are not instantiated)
      if (bp) {  // the image operand pre-split by k_split_img (never for the pointwise kernels: no BP / BD form)
        if constexpr (BM == 64) {
          if (accum) {
            MSL_LAUNCH((k_igemm_fwd_sk2<BM, kSkBN, G, ST, WM, WN, PW, MT, true, true, true>), grid, block, 0,
                               st, a, sk);
            return MSL_OK;
          }
        }
        if (!accum) {
          MSL_LAUNCH((k_igemm_fwd_sk2<BM, kSkBN, G, ST, WM, WN, PW, MT, false, true, true>), grid, block, 0,
                             st, a, sk);
          return MSL_OK;
        }
      }
      // the image operand straight to registers (BD form) for the shifted 3x3 rows (dword pieces);
      // the pointwise rows keep their two dwordx4 LDS-DMA pieces per wave and K-step (BD loses there:
      // 256 -> 1024 fwd 32.7 vs 31.0 us, 2048 -> 512 82.7 vs 75.1; layer3 3x3 fwd 52.4 vs 55.0,
      // layer4 172 vs 190; profiles/r03_fwd_forms_ab.txt)
      // (full 16-channel blocks only: the stem's 147-row im2col operand keeps the LDS form)
      if (a.cimg % kCB == 0) {
        if constexpr (BM == 64) {
          if (accum) {
            MSL_LAUNCH((k_igemm_fwd_sk2<BM, kSkBN, G, ST, WM, WN, PW, MT, true, true>), grid, block, 0, st, a,
                               sk);
            return MSL_OK;
          }
        }
        if (!accum) {
          MSL_LAUNCH((k_igemm_fwd_sk2<BM, kSkBN, G, ST, WM, WN, PW, MT, false, true>), grid, block, 0, st, a,
                             sk);
          return MSL_OK;
        }
      }
    }
    if (accum)
      MSL_LAUNCH((k_igemm_fwd_sk2<BM, kSkBN, G, ST, WM, WN, PW, MT, true>), grid, block, 0, st, a, sk);
    else
      MSL_LAUNCH((k_igemm_fwd_sk2<BM, kSkBN, G, ST, WM, WN, PW, MT, false>), grid, block, 0, st, a, sk);
  } else {
    if (accum)
      MSL_LAUNCH((k_igemm_fwd_sk<BM, kSkBN, G, ST, WM, WN, false, MT, true>), grid, block, 0, st, a, sk);
    else
      MSL_LAUNCH((k_igemm_fwd_sk<BM, kSkBN, G, ST, WM, WN, false, MT, false>), grid, block, 0, st, a, sk);
  }
  return MSL_OK;
}

template <int MT>
static int launch_fwd_form(const float* img, int cimg, const float* packed, int M, const float* bias,
                           int nbias, float* out, int nbranch, int taps, int h, int w, int nimg, int dil0,
                           int dil1, const msl_forms* forms, void* ws, size_t ws_bytes, hipStream_t st,
                           int accum = 0, const float* img_part = nullptr, int img_npart = 0,
                           const float* accres = nullptr, const unsigned long long* accmask = nullptr, int accni = 1) {
  if (forms_bad(forms)) return MSL_ERR_ARG;
  const int P = nimg * h * w;  // nimg images of h x w stacked along the pixel axis
  FwdPlan pl = plan_fwd(nbranch, taps, cimg, M, P, bias != nullptr);
  // The x6 form runs one K-step per stage, three stages deep (r01 tuning harness, layer3:
  // 87 us vs 115 with two K-steps per stage; f32 is indifferent); its 64- and 32-row tiles stay
  // on exact f32 MFMA (no gain measured there).
  // split forms (and the fp16 math, which reads the f16x3 packs' hi planes): 128-row tiles only
  constexpr bool F16 = MT == kMathH3P || MT == kMathH1P;
  constexpr bool X6L = MT == kMathX6 || F16;
  constexpr int MS = X6L ? kMathF32 : MT;
  constexpr int MB = F16 ? kMathX6 : MT;       // (not reached by the split forms)
  if (X6L && pl.sk && pl.bm == 128) {
    pl.G = 1;
    pl.bk = kCB;
    pl.kps = pl.ksteps;
  }
  // f16x3 / fp16 (r03): the 3x3 / ASPP GEMMs with M <= 64 (the 19-class ASPP forward, layer1's
  // 64-channel convs) on 64-row tiles of the same kernel (weights from the fp16 planes, the image
  // operand straight to registers) instead of exact-f32 32 / 64-row tiles: 3 fp16 MFMAs per 16-deep
  // slice at 64 rows cost 2.7x less matrix time than 8 f32 MFMAs at 32 rows.
  // (r03: also the pointwise / stem GEMMs with M <= 64 - layer1's 256 -> 64 convs, the 64-channel data
  // gradients, the stem's 147 -> 64 - through the same form with one unshifted tap)
  // r04: the fp16 math too (its single fp16 plane split into half-wave A pieces, fwd_sk_body AHALF)
  const bool small_f16 = F16 && pl.sk && pl.bm <= 64;
  if (small_f16) {
    pl.G = 1;
    pl.bm = 64;
    pl.bk = kCB;
    pl.tiles_m = cdiv(M, 64);
    pl.kps = pl.ksteps;
  }
  // fp16 pointwise GEMMs (r04): two K-steps per LDS stage, three stages (72 KB, two workgroups per
  // CU): one barrier per 8 MFMAs per wave instead of 4 (f16x3's two planes would need 96 KB)
  const bool pw2 = MT == kMathH1P && pl.sk && pl.bm == 128 && taps == 1 && dil0 == 0 && pl.ksteps % 2 == 0;
  if (pw2) {
    pl.G = 2;
    pl.bk = 2 * kCB;
    pl.kps = pl.ksteps / 2;
  }
  if (ws_bytes < fwd_ws_bytes(pl, M, P, cimg, taps)) return MSL_ERR_WORKSPACE;
  FwdArgs a{};
  a.Ax6 = nullptr;
  a.ascale = nullptr;
  a.bpart = nullptr;
  a.bnpart = 0;
  a.accum = accum;
  a.accres = accres;  // (r06: the masked residual gradient of msl_pconv_dgrad_resmask*; needs accum)
  a.accmask = accmask;
  a.accni = accni;
  if (accres && (!accum || !accmask || accni < 1 || P % accni != 0)) return MSL_ERR_ARG;
  a.A = packed;
  a.B = img;
  a.C = pl.S > 1 ? (float*)ws : out;
  a.bias = pl.S > 1 ? nullptr : bias;
  a.nbias = nbias;
  a.M = M;
  a.lda = pad_to(M, kPackPad);
  a.H = h;
  a.W = w;
  a.P = P;
  a.cimg = cimg;
  a.ncb = cdiv(cimg, kCB);
  a.dil0 = dil0;
  a.dil1 = dil1;
  a.ksteps = pl.ksteps;
  a.kps = pl.kps;
  a.taps = taps;
  a.slab = (long long)M * P;
  if (pl.sk) {
    SkArgs sk{};
    sk.part = (float*)ws;
    sk.tiles_m = pl.tiles_m;
    sk.tiles_n = pl.tiles_n;
    sk.KS = pl.kps;
    const long long tiles = (long long)pl.tiles_m * pl.tiles_n;
    if (tiles * sk.KS * kSkNW >= (1LL << 31) || (long long)cimg * P >= (1LL << 29) ||
        (long long)pl.ksteps * kCB * a.lda >= (1LL << 29))
      return MSL_ERR_SHAPE;  // 32-bit index arithmetic in the kernel
    // at least as many tiles as workers: whole rounds of tiles data-parallel, stream-K over the
    // rest (SkArgs); fewer: pure stream-K.  Every stream-K worker must own at least one iteration:
    // the piece count of a tile is the number of workgroups its iteration range touches.
    sk.tdp = (forms_of(forms).sk_hybrid && tiles >= kSkNW) ? (int)(tiles / kSkNW * kSkNW) : 0;
    // Tile order (r04): m fastest when whole rounds of tiles run data-parallel (hybrid): one XCD's
    // workers then hold every m-block of a few pixel blocks, so each image block is fetched once and
    // re-read from that L2 (same box: 256 -> 1024 fwd 42.7 vs 49.8 us, 2048 -> 512 dgrad 127 vs 141,
    // layer4 fwd 214 vs 226; profiles/r04_tile_order_ab.txt).  n fastest for pure stream-K: a worker's
    // range there is under one tile, the m-blocks of a pixel block run at staggered K offsets and get no
    // L2 reuse, and the shared weights of n fastest win (ASPP fwd, M = 342 over 128 K-steps: 134 vs
    // 101 us m fastest; layer3 fwd 79 vs 77.7; profiles/r04_aspp_tile_order.txt).
    sk.gm = sk.tdp > 0 ? pl.tiles_m : 1;
    const long long T = (tiles - sk.tdp) * sk.KS;
    sk.NW = (int)std::min<long long>(kSkNW, T);
    // the remainder after data-parallel rounds (e.g. 16 tiles x 16 K-steps of a 256 -> 1024 pointwise
    // GEMM): at one or two K-steps per worker every worker writes a whole 64-KB piece for almost no
    // work; at least kSkMinIt K-steps each (512 -> 2048 fwd 75.9 vs 82.2 us, 2048 -> 512 dgrad 85.6 vs
    // 90.0)
    constexpr long long kSkMinIt = 8;
    if (sk.tdp > 0) sk.NW = (int)std::max<long long>(1, std::min<long long>(sk.NW, T / kSkMinIt));
    sk.T = (int)T;
    a.C = out;
    a.bias = bias;
    const dim3 grid(sk.tdp > 0 ? kSkNW : sk.NW), block(256);
    const dim3 rgrid(pl.bm * kSkBN / 1024, (unsigned)(tiles - sk.tdp));
    const bool reduce = T > 0;
    if (X6L && (pl.bm == 128 || small_f16)) {
      // the x6 kernel stages its weights from the bf16 planes that pack() split once, behind
      // the fp32 part of the same buffer (M > 64 <=> 128-row tiles; f16x3: every M)
      const long long f32 = (long long)pl.ksteps * kCB * a.lda;
      a.Ax6 = reinterpret_cast<const __bf16*>(packed + f32);
      if constexpr (F16) {
        // f16x3 / fp16: the image's absmax partials, then the GEMM with the pack's {sA, 1/sA}
        if (img_part) {  // the caller's partials of this image (msl_absmax_partials, a BN kernel)
          a.bpart = img_part;
          a.bnpart = img_npart;
        } else {
          float* part = ws_partials(ws, ws_bytes, 1);
          MSL_LAUNCH(k_absmax, dim3(kNPart), block, 0, st, img, (long long)cimg * P, 0LL, 1, part);
          MSL_CHECK_LAUNCH();
          a.bpart = part;
          a.bnpart = kNPart;
        }
        a.ascale = packed + pack_tail_offset(f32) + kNPart;
        // the image operand pre-split once for the whole GEMM (BP form, behind the pieces): pays on
        // the layer4 3x3 GEMMs (M = 512: the split pass is shared by 4 row blocks and 9 taps), fwd
        // 162 vs 174 us, dgrad 172 vs 185; loses where the pass is a large share (pointwise 39 vs
        // 31 us, layer2 34 vs 31, ASPP 144 vs 135) - profiles/r03_bp_ab.txt
        const bool bp = bp_form(taps, M, small_f16, MT == kMathH1P);
        if (bp) {
          f16x8* planes = reinterpret_cast<f16x8*>((char*)ws + fwd_piece_bytes(pl));
          const long long n = (long long)a.ncb * 2 * P;
          const dim3 sgrid((unsigned)std::min<long long>(cdiv(n, 256), 8192));
          if constexpr (MT == kMathH1P)
            MSL_LAUNCH(k_split_img<1>, sgrid, block, 0, st, img, cimg, a.ncb, P, a.bpart, a.bnpart, planes);
          else
            MSL_LAUNCH(k_split_img<2>, sgrid, block, 0, st, img, cimg, a.ncb, P, a.bpart, a.bnpart, planes);
          MSL_CHECK_LAUNCH();
          a.Bx6 = planes;
        }
        // pointwise: B rows are unshifted, so they move as dwordx4 (4 pixels per lane: 2 DMAs per
        // wave and K-step instead of 8 dword ones): 1-4 us per call on the wide 1x1 GEMMs
        // (profiles/r02_f16x3_pw_dma.txt)
        // waves 1 x 4 (each 128 rows x 32 pixels): every wave splits only its own B columns
        // (2 x 2 waves split each column twice); step 40.5 vs 40.9 ms on one box
        // (profiles/r02_f16x3_waves.txt)
        if (small_f16) {
          MSL_TRY(launch_sk<64, 1, 4, 1, 4, MT>(accum, grid, block, st, a, sk, bp));
        } else if (taps == 1 && dil0 == 0 && MT == kMathH3P && pl.bmx > 0) {
          // wide tiles (r06): the plan, the grid and the reduce of that tile size
          if constexpr (MT == kMathH3P) {
            const int tm = cdiv(M, pl.bmx);
            const SkArgs s2 = plan_sk(tm, pl.tiles_n, pl.kps, kSkNW, forms_of(forms).sk_hybrid, (float*)ws);
            const dim3 g2(s2.tdp > 0 ? kSkNW : s2.NW);
            const dim3 r2(pl.bmx * kSkBN / 1024, (unsigned)((long long)tm * pl.tiles_n - s2.tdp));
            MSL_TRY(launch_sk<256, 1, 3, 1, 4, MT, true>(accum, g2, block, st, a, s2));
            MSL_CHECK_LAUNCH();
            if (s2.T > 0) MSL_LAUNCH((k_sk_reduce<256, kSkBN>), r2, block, 0, st, a, s2);
            MSL_CHECK_LAUNCH();
            return MSL_OK;
          }
        } else if (taps == 1 && dil0 == 0) {
          if constexpr (MT == kMathH1P) {
            if (pw2)
              MSL_TRY(launch_sk<128, 2, 3, 1, 4, MT, true>(accum, grid, block, st, a, sk, bp));
            else
              MSL_TRY(launch_sk<128, 1, 4, 1, 4, MT, true>(accum, grid, block, st, a, sk, bp));
          } else {
            MSL_TRY(launch_sk<128, 1, 4, 1, 4, MT, true>(accum, grid, block, st, a, sk, bp));
          }
        } else if (bp && !accum && bq_form(taps, M, small_f16)) {
          MSL_TRY(launch_sk<128, 1, 4, 2, 2, MT>(accum, grid, block, st, a, sk, bp));
        } else {
          MSL_TRY(launch_sk<128, 1, 4, 1, 4, MT>(accum, grid, block, st, a, sk, bp));
        }
      } else {
        MSL_TRY(launch_sk<128, 1, 4, 2, 2, kMathX6P>(accum, grid, block, st, a, sk));
      }
      MSL_CHECK_LAUNCH();
      if (reduce) {
        if (small_f16)
          MSL_LAUNCH((k_sk_reduce<64, kSkBN>), rgrid, block, 0, st, a, sk);
        else
          MSL_LAUNCH((k_sk_reduce<128, kSkBN>), rgrid, block, 0, st, a, sk);
      }
    } else if (pl.bm == 128) {
      if (pl.G == 2)
        MSL_TRY(launch_sk<128, 2, 2, 2, 2, MB>(accum, grid, block, st, a, sk));
      else
        MSL_TRY(launch_sk<128, 1, 3, 2, 2, MB>(accum, grid, block, st, a, sk));
      MSL_CHECK_LAUNCH();
      if (reduce) MSL_LAUNCH((k_sk_reduce<128, kSkBN>), rgrid, block, 0, st, a, sk);
    } else if (pl.bm == 64) {
      if (pl.G == 2)
        MSL_TRY(launch_sk<64, 2, 2, 2, 2, MS>(accum, grid, block, st, a, sk));
      else
        MSL_TRY(launch_sk<64, 1, 3, 2, 2, MS>(accum, grid, block, st, a, sk));
      MSL_CHECK_LAUNCH();
      if (reduce) MSL_LAUNCH((k_sk_reduce<64, kSkBN>), rgrid, block, 0, st, a, sk);
    } else {
      MSL_TRY(launch_sk<32, 2, 2, 1, 4, MS>(accum, grid, block, st, a, sk));
      MSL_CHECK_LAUNCH();
      if (reduce) MSL_LAUNCH((k_sk_reduce<32, kSkBN>), rgrid, block, 0, st, a, sk);
    }
    MSL_CHECK_LAUNCH();
    return MSL_OK;
  }
  // the split-K tile kernel (odd K-step count, M <= 32) has no bf16 form; x6 runs it in exact f32
  if (MT == kMathBf16 || accum) return MSL_ERR_SHAPE;
  dim3 grid(pl.tiles_n, pl.tiles_m, pl.S);
  MSL_LAUNCH((k_igemm_fwd<64, 128, 16, 2, 2>), grid, dim3(256), 0, st, a);
  MSL_CHECK_LAUNCH();
  if (pl.S > 1) {
    const long long n = (long long)M * P;
    const int blocks = (int)std::min<long long>(cdiv(n, 256), 4096);
    MSL_LAUNCH(k_reduce_slabs, dim3(blocks), dim3(256), 0, st, (const float*)ws, pl.S, n,
                       out, 0, bias, nbias, M, P);
    MSL_CHECK_LAUNCH();
  }
  return MSL_OK;
}

static bool bad_dims(int nbranch, int cin, int cout, int h, int w, int nimg = 1) {
  return nbranch < 1 || nbranch > 2 || cin < 1 || cout < 1 || h < 1 || w < 1 || nimg < 1 ||
         (long long)nimg * h * w > (1LL << 30);
}

// ---------------------------------------------------------------- shared by 3x3 and pointwise
// A packed operand is the fp32 K-major pack [ksteps*16][lda] followed by its bf16x6 planes
// [ks][plane][k half][lda][8] (k_split_pack; 1.5x the fp32 bytes).  The planes are written by
// pack() when M > 64 - the 128-row tiles of the x6 form, the only reader - so the split runs
// once per weight update instead of once per conv call.
static long long packed_f32_elems(int nbranch, int taps, int cin, int cout, int for_dgrad) {
  const int cimg = for_dgrad ? cout : cin;
  const int m = for_dgrad ? cin : cout;
  return (long long)nbranch * cdiv(cimg, kCB) * taps * kCB * pad_to(m, kPackPad);
}

static long long packed_elems(int nbranch, int taps, int cin, int cout, int for_dgrad) {
  return pack_tail_offset(packed_f32_elems(nbranch, taps, cin, cout, for_dgrad)) + kPackTail;
}

// forms.pack_form: 1 = k_pack_split, 0 = k_pack + k_split_pack
static int pack(const float* w, long long branch_stride, int nbranch, int taps, int cin, int cout,
                int for_dgrad, float* packed, const msl_forms* forms, hipStream_t st) {
  if (forms_bad(forms)) return MSL_ERR_ARG;
  const int cimg = for_dgrad ? cout : cin;
  const int m = for_dgrad ? cin : cout;
  const long long total = packed_f32_elems(nbranch, taps, cin, cout, for_dgrad);
  const int lda = pad_to(m, kPackPad);
  const int ncb = cdiv(cimg, kCB);
  __bf16* planes = reinterpret_cast<__bf16*>(packed + total);
  // f16x3: fp16 planes for every M (the <= 64-row 3x3 / ASPP tiles run f16x3 too since r03)
  const bool h3 = forms_of(forms).f32_form == kMathH3P;
  float* tail = h3 ? packed + pack_tail_offset(total) : nullptr;
  // M <= 64 has no planes to split, and its 128-row padding is mostly zeros, which k_pack's
  // fully coalesced rows write faster (ASPP fwd 2048 -> 19: 5.2 vs 9.5 us)
  if (!h3 && (forms_of(forms).pack_form == 0 || m <= 64)) {  // element-wise gather, then a separate split
    const int blocks = (int)std::min<long long>(cdiv(total, 256), 8192);
    MSL_LAUNCH(k_pack, dim3(blocks), dim3(256), 0, st, w, branch_stride, cin, cout, for_dgrad,
                       ncb, lda, taps, total, packed);
    MSL_CHECK_LAUNCH();
    if (m > 64) {
      const int ksteps = nbranch * ncb * taps;
      MSL_LAUNCH(k_split_pack, dim3((int)std::min<long long>(cdiv(total, 256), 4096)), dim3(256),
                         0, st, packed, ksteps, lda, planes);
      MSL_CHECK_LAUNCH();
    }
    return MSL_OK;
  }
  // lda is a multiple of kPackPad (128): the m chunks tile it exactly, zero rows included
  static_assert(kPackPad % kPackTileM == 0, "pack tiles must cover lda");
  const dim3 grid(lda / kPackTileM, ncb, nbranch);
  const int split = m > 64 || h3;
  if (taps != 9 && taps != 1) return MSL_ERR_ARG;
  if (h3) {
    MSL_LAUNCH(k_absmax, dim3(kNPart), dim3(256), 0, st, w, (long long)cout * cin * taps, branch_stride,
                       nbranch, tail);
    MSL_CHECK_LAUNCH();
    MSL_LAUNCH(k_pack_scale, dim3(1), dim3(64), 0, st, tail);
    MSL_CHECK_LAUNCH();
  }
  if (taps == 9)
    MSL_LAUNCH(k_pack_split<9>, grid, dim3(256), 0, st, w, branch_stride, cin, cout, for_dgrad, ncb,
                       lda, split, packed, planes, tail);
  else
    MSL_LAUNCH(k_pack_split<1>, grid, dim3(256), 0, st, w, branch_stride, cin, cout, for_dgrad, ncb,
                       lda, split, packed, planes, tail);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

// Pointwise weight gradients with more output than input channels run with the operands swapped
// (WskArgs::trans): k_wgrad_x6 pre-splits the operand with fewer rows - the image instead of dY
// (256 -> 1024: a 256-row split instead of a 1024-row one, ~10 vs ~20 us) - and the reduce writes
// the dW^T tiles transposed.
static bool wgrad_swaps(int nbranch, int taps, int cin, int cout) { return nbranch == 1 && taps == 1 && cout > cin; }
// k_wgrad_x6's piece reduce in the [m][n] orientation: waves per 64 outputs (1 = k_wsk_reduce's single chain)
constexpr int kWskSplit = 4, kWskSplitMinPieces = 16;

static size_t wgrad_core_bytes(int nbranch, int taps, int cin, int cout, int P, int w) {
  // large enough for either fp32 form and orientation: pieces, then (k_wgrad_x6) the split planes
  size_t b = 0;
  for (int x6 = 0; x6 < 2; ++x6)
    for (int sw = 0; sw < 2; ++sw) {
      WgradPlan pl = sw ? plan_wgrad(nbranch, taps, cout, cin, P, x6 != 0, w)
                        : plan_wgrad(nbranch, taps, cin, cout, P, x6 != 0, w);
      b = std::max(b, wgrad_piece_bytes(pl) + wgrad_planes_bytes(pl));
    }
  return align_up(b, 16);
}

static size_t wgrad_ws_bytes(int nbranch, int taps, int cin, int cout, int P, int w) {
  // + (f16x3) both operands' per-row absmax partials when the caller passes none
  return wgrad_core_bytes(nbranch, taps, cin, cout, P, w) + align_up((size_t)(cin + cout) * 4, 16) + 16;
}

template <int MT>
static int launch_wgrad(const float* x, const float* dy, float* dw, float* dbias, int nbranch,
                        int taps, int cin, int cout, int h, int w, int nimg, int dil0, int dil1,
                        int accumulate, void* ws, size_t ws_bytes, hipStream_t st,
                        const float* x_part = nullptr, int x_npart = 0, const float* dy_part = nullptr,
                        int dy_npart = 0) {
  const int P = nimg * h * w;
  constexpr bool F16 = MT == kMathH3P || MT == kMathH1P;
  constexpr bool X6L = MT == kMathX6 || F16;
  constexpr int MS = X6L ? kMathF32 : MT;  // the split forms only on 128x128 tiles (plan_wgrad)
  constexpr int MB = F16 ? kMathX6 : MT;   // k_wgrad_sk has no f16 form: x6 there
  if (ws_bytes < wgrad_ws_bytes(nbranch, taps, cin, cout, P, w)) return MSL_ERR_WORKSPACE;
  WgradPlan pl = plan_wgrad(nbranch, taps, cin, cout, P, X6L, w);
  bool trans = false;
  if (X6L && wgrad_swaps(nbranch, taps, cin, cout) && !dbias) {
    WgradPlan ps = plan_wgrad(nbranch, taps, cout, cin, P, true, w);
    if (ps.rx6) {  // dW^T = image . dY^T: M = cin (pre-split), N = cout
      pl = ps;
      trans = true;
      std::swap(x, dy);
      std::swap(x_part, dy_part);
      std::swap(x_npart, dy_npart);
      std::swap(cin, cout);
    }
  }
  if (pl.T * pl.nw >= (1LL << 31) || (long long)pl.nw * pl.slots * pl.bm * pl.bn * 4 >= (1LL << 31) || (long long)std::max(cin, cout) * P >= (1LL << 29) ||
      (long long)P + kWskBK >= (1LL << 22))
    return MSL_ERR_SHAPE;  // 32-bit index arithmetic, float pixel-row division in the kernel
  WskArgs a{};
  a.dy = dy;
  a.x = x;
  a.dw = dw;
  a.part = (float*)ws;
  a.M = cout;
  a.N = cin;
  a.H = h;
  a.W = w;
  a.P = P;
  a.dil0 = dil0;
  a.dil1 = dil1;
  a.taps = taps;
  a.accumulate = accumulate;
  a.slots = pl.slots;
  a.invW = 1.0f / (float)w;
  a.invH = 1.0f / (float)h;
  a.tiles_m = pl.tiles_m;
  a.tiles_n = pl.tiles_n;
  a.KS = pl.KS;
  a.NW = pl.nw;
  a.T = (int)pl.T;
  a.cbranch = (long long)cout * cin * taps;
  a.dyx6 = nullptr;
  a.lda = pl.lda;
  a.nchunk = pl.nchunk;
  a.kchunk = pl.kchunk;
  a.ntiles = pl.tiles_m * pl.tiles_n * pl.ntap;
  a.trans = trans ? 1 : 0;
  a.apart = nullptr;
  a.bpart = nullptr;
  a.anpart = a.bnpart = 0;
  const dim3 grid(pl.nw), block(256);
  const dim3 rgrid(cdiv((long long)pl.bm * pl.bn / 4 * taps, 256), pl.tiles_m * pl.tiles_n * nbranch), rblock(256);
  if (pl.rx6) {
    bf16x8* planes = reinterpret_cast<bf16x8*>((char*)ws + wgrad_piece_bytes(pl));
    a.dyx6 = planes;
    if constexpr (F16) {  // both operands' per-row absmax partials, then the per-row scaled split
      const float* ap = dy_part;
      const float* bp = x_part;
      int an = dy_npart, bn = x_npart;
      // the caller's partials are one maximum per row (msl_absmax_partials, the BN kernels' per-
      // channel outputs); none given: reduce them here (after a swap the operands traded places)
      float* rp = reinterpret_cast<float*>((char*)ws + wgrad_core_bytes(nbranch, taps, cin, cout, P, w));
      if (!ap) {
        const int e = absmax_rows(dy, cout, P, rp, st);
        if (e != MSL_OK) return e;
        ap = rp;
        an = cout;
      }
      if (!bp) {
        float* r2 = rp + align_up((size_t)cout, 4);
        const int e = absmax_rows(x, cin, P, r2, st);
        if (e != MSL_OK) return e;
        bp = r2;
        bn = cin;
      }
      a.apart = ap;
      a.bpart = bp;
      a.anpart = an;
      a.bnpart = bn;
      a.rowscale = (an == cout && bn == cin) ? 1 : 0;
      MSL_LAUNCH(k_split_rows<MT>, dim3(pl.lda / kSplitRowsR, cdiv(pl.KS, 16)), dim3(256), 0, st, dy, cout, P,
                         pl.KS, pl.lda, planes, ap, an, a.rowscale);
      MSL_CHECK_LAUNCH();
      MSL_LAUNCH((k_wgrad_x6<MT>), grid, block, 0, st, a);
    } else {
      MSL_LAUNCH(k_split_rows<kMathX6>, dim3(pl.lda / kSplitRowsR, cdiv(pl.KS, 16)), dim3(256), 0, st, dy, cout, P,
                         pl.KS, pl.lda, planes, (const float*)nullptr, 0);
      MSL_CHECK_LAUNCH();
      MSL_LAUNCH(k_wgrad_x6<kMathX6>, grid, block, 0, st, a);
    }
    MSL_CHECK_LAUNCH();
    // r06: S waves per 64 outputs, each summing every S-th piece (k_wsk_reduce_split), where a tile has >= 16 pieces
    // (the 16- and 9-tile layer3 1x1 / layer2 3x3 gradients: 32-56 chunks; at 8 pieces, 512 -> 2048, it lost 4 us)
    const long long tile_pieces = pl.nchunk > 0 ? pl.nchunk : cdiv((long long)pl.nw, (long long)a.ntiles);
    if (kWskSplit > 1 && tile_pieces >= kWskSplitMinPieces)
      MSL_LAUNCH((k_wsk_reduce_split<128, 128, kWskSplit>), dim3(cdiv(128LL * 128 / 4 * taps, 64), rgrid.y),
                 dim3(64 * kWskSplit), 0, st, a);
    else
      MSL_LAUNCH((k_wsk_reduce<128, 128>), rgrid, rblock, 0, st, a);
  } else if (pl.bm == 128) {
    MSL_LAUNCH((k_wgrad_sk<128, 128, 2, 2, 2, MB>), grid, block, 0, st, a);
    MSL_CHECK_LAUNCH();
    MSL_LAUNCH((k_wsk_reduce<128, 128>), rgrid, rblock, 0, st, a);
  } else if (pl.bm == 64) {
    MSL_LAUNCH((k_wgrad_sk<64, 64, 2, 2, 2, MS>), grid, block, 0, st, a);
    MSL_CHECK_LAUNCH();
    // few tiles with many pieces each (the 33k-px 1x1 gradients: 4 tiles x ~128 pieces): 8 threads
    // per output float4 (k_wsk_reduce_wide) instead of one serial chain of every piece
    const long long pieces = cdiv((long long)pl.nw, std::max(1LL, pl.T / pl.KS));  // per (tile, tap)
    if ((long long)rgrid.x * rgrid.y < 256 && pieces >= 16)
      MSL_LAUNCH((k_wsk_reduce_wide<64, 64, 8>), dim3(cdiv((long long)64 * 64 / 4 * taps, 32), rgrid.y), rblock,
                         0, st, a);
    else
      MSL_LAUNCH((k_wsk_reduce<64, 64>), rgrid, rblock, 0, st, a);
  } else {
    MSL_LAUNCH((k_wgrad_sk<32, 128, 2, 1, 4, MS>), grid, block, 0, st, a);
    MSL_CHECK_LAUNCH();
    MSL_LAUNCH((k_wsk_reduce<32, 128>), rgrid, rblock, 0, st, a);
  }
  MSL_CHECK_LAUNCH();
  if (dbias) {
    MSL_LAUNCH(k_bias_grad, dim3(cout), dim3(256), 0, st, dy, P, dbias, cout, nbranch,
                       accumulate);
    MSL_CHECK_LAUNCH();
  }
  return MSL_OK;
}

// the fp32 entry points: the kernel template of the call's f32 form
template <typename... Args>
static int fwd_f32(const msl_forms* forms, Args... args) {
  if (forms_bad(forms)) return MSL_ERR_ARG;
  const int form = forms_of(forms).f32_form;
  if (form == kMathH3P) return launch_fwd_form<kMathH3P>(args...);
  return form == kMathX6 ? launch_fwd_form<kMathX6>(args...) : launch_fwd_form<kMathF32>(args...);
}

template <typename... Args>
static int wgrad_f32(const msl_forms* forms, Args... args) {
  if (forms_bad(forms)) return MSL_ERR_ARG;
  const int form = forms_of(forms).f32_form;
  if (form == kMathH3P) return launch_wgrad<kMathH3P>(args...);
  return form == kMathX6 ? launch_wgrad<kMathX6>(args...) : launch_wgrad<kMathF32>(args...);
}

}  // namespace msl

using namespace msl;

extern "C" {

int msl_abi_version(void) { return MSL_ABI_VERSION; }

int msl_forms_default(msl_forms* out) {
  if (!out) return MSL_ERR_ARG;
  *out = kDefaultForms;
  return MSL_OK;
}

int msl_forms_check(const msl_forms* forms) { return forms_bad(forms) ? MSL_ERR_ARG : MSL_OK; }

int msl_launch_guard_probe(int threads, float* out, msl_stream_t stream) {
  if (threads < 1 || !out) return MSL_ERR_ARG;
  MSL_LAUNCH(k_guard_probe, dim3(1), dim3(threads), 0, as_stream(stream), out);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

const char* msl_status_string(int status) {
  switch (status) {
    case MSL_OK: return "ok";
    case MSL_ERR_SHAPE: return "invalid shape";
    case MSL_ERR_WORKSPACE: return "workspace too small";
    case MSL_ERR_ARG: return "invalid argument";
    case MSL_ERR_LAUNCH: return "block exceeds the kernel's launch bounds";
    default: return status > 0 ? hipGetErrorString((hipError_t)status) : "unknown error";
  }
}

// ------------------------------------------------------------------ dilated 3x3
long long msl_dconv_packed_elems(int nbranch, int cin, int cout, int for_dgrad) {
  return packed_elems(nbranch, 9, cin, cout, for_dgrad);
}

int msl_dconv_pack(const float* w, long long branch_stride, int nbranch, int cin, int cout,
                   int for_dgrad, float* packed, const msl_forms* forms, msl_stream_t stream) {
  if (bad_dims(nbranch, cin, cout, 1, 1) || !w || !packed) return MSL_ERR_ARG;
  return pack(w, branch_stride, nbranch, 9, cin, cout, for_dgrad, packed, forms, as_stream(stream));
}

long long msl_conv_pack_blocks(int nbranch, int taps, int cin, int cout, int for_dgrad) {
  if (bad_dims(nbranch, cin, cout, 1, 1) || (taps != 1 && taps != 9)) return -1;
  const int cimg = for_dgrad ? cout : cin;
  const int m = for_dgrad ? cin : cout;
  const long long tiles = (long long)(pad_to(m, kPackPad) / kPackTileM) * cdiv(cimg, kCB) * nbranch;
  return taps == 1 ? cdiv(tiles, (long long)kPackSub<1>()) : tiles;  // blocks of msl_conv_pack_many
}

int msl_conv_pack_many(const msl_pack_job* jobs, const long long* block_start, int njobs, int taps,
                       long long total_blocks, const msl_forms* forms, msl_stream_t stream) {
  if (!jobs || !block_start || njobs < 1 || total_blocks < 1 || total_blocks >= (1LL << 31) ||
      (taps != 1 && taps != 9) || forms_bad(forms))
    return MSL_ERR_ARG;
  hipStream_t st = as_stream(stream);
  const int h3 = forms_of(forms).f32_form == kMathH3P;
  if (h3) {  // the weights' absmax partials first (jobs with M > 64: the split packs)
    if (taps == 9)
      MSL_LAUNCH(k_absmax_jobs<9>, dim3(kNPart, (unsigned)njobs), dim3(256), 0, st, jobs);
    else
      MSL_LAUNCH(k_absmax_jobs<1>, dim3(kNPart, (unsigned)njobs), dim3(256), 0, st, jobs);
    MSL_CHECK_LAUNCH();
    if (taps == 9)
      MSL_LAUNCH(k_pack_scale_jobs<9>, dim3((unsigned)njobs), dim3(64), 0, st, jobs);
    else
      MSL_LAUNCH(k_pack_scale_jobs<1>, dim3((unsigned)njobs), dim3(64), 0, st, jobs);
    MSL_CHECK_LAUNCH();
  }
  if (taps == 9)
    MSL_LAUNCH(k_pack_split_many<9>, dim3((unsigned)total_blocks), dim3(256), 0, st, jobs, block_start, njobs,
                       h3);
  else
    MSL_LAUNCH(k_pack_split_many<1>, dim3((unsigned)total_blocks), dim3(256), 0, st, jobs, block_start, njobs,
                       h3);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

size_t msl_dconv_fwd_workspace(int nbranch, int cin, int cout, int h, int w, int nimg) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg)) return 0;
  const int P = nimg * h * w;
  // large enough with or without a bias (the plan depends on it)
  return std::max(fwd_ws_bytes(plan_fwd(nbranch, 9, cin, cout, P, false), cout, P, cin, 9),
                  fwd_ws_bytes(plan_fwd(nbranch, 9, cin, cout, P, true), cout, P, cin, 9));
}

int msl_dconv_fwd(const float* x, const float* packed, const float* bias, float* y, int nbranch,
                  int cin, int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                  size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !packed || !y || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return fwd_f32(forms, x, cin, packed, cout, bias, nbranch, y, nbranch, 9, h, w, nimg, dil0, dil1,
                         forms, ws, ws_bytes, as_stream(stream));
}

size_t msl_dconv_dgrad_workspace(int nbranch, int cin, int cout, int h, int w, int nimg) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg)) return 0;
  const int P = nimg * h * w;
  return fwd_ws_bytes(plan_fwd(nbranch, 9, cout, cin, P, false), cin, P, cout, 9);
}

int msl_dconv_dgrad(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin,
                    int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !dy || !packed_dgrad || !dx || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return fwd_f32(forms, dy, cout, packed_dgrad, cin, nullptr, 0, dx, nbranch, 9, h, w, nimg, dil0, dil1,
                         forms, ws, ws_bytes, as_stream(stream));
}

size_t msl_dconv_wgrad_workspace(int nbranch, int cin, int cout, int h, int w, int nimg) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg)) return 0;
  const int P = nimg * h * w;
  return wgrad_ws_bytes(nbranch, 9, cin, cout, P, w);
}

int msl_dconv_wgrad(const float* x, const float* dy, float* dw, float* dbias, int nbranch, int cin,
                    int cout, int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !dy || !dw || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return wgrad_f32(forms, x, dy, dw, dbias, nbranch, 9, cin, cout, h, w, nimg, dil0, dil1, accumulate, ws,
                      ws_bytes, as_stream(stream));
}

// ------------------------------------------------------------------ pointwise (1x1, stride 1)
// A pointwise conv is the same GEMM with one unshifted tap (dilation 0) over the flat pixel axis.
long long msl_pconv_packed_elems(int cin, int cout, int for_dgrad) {
  return packed_elems(1, 1, cin, cout, for_dgrad);
}

int msl_pconv_pack(const float* w, int cin, int cout, int for_dgrad, float* packed, const msl_forms* forms,
                   msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, 1) || !w || !packed) return MSL_ERR_ARG;
  return pack(w, 0, 1, 1, cin, cout, for_dgrad, packed, forms, as_stream(stream));
}

size_t msl_pconv_fwd_workspace(int cin, int cout, int p) {
  if (bad_dims(1, cin, cout, 1, p)) return 0;
  return fwd_ws_bytes(plan_fwd(1, 1, cin, cout, p, false), cout, p, cin, 1);
}

int msl_pconv_fwd(const float* x, const float* packed, float* y, int cin, int cout, int p,
                  const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, p) || !x || !packed || !y) return MSL_ERR_ARG;
  return fwd_f32(forms, x, cin, packed, cout, nullptr, 0, y, 1, 1, 1, p, 1, 0, 0, forms, ws,
                         ws_bytes, as_stream(stream));
}

size_t msl_pconv_dgrad_workspace(int cin, int cout, int p) {
  if (bad_dims(1, cin, cout, 1, p)) return 0;
  return fwd_ws_bytes(plan_fwd(1, 1, cout, cin, p, false), cin, p, cout, 1);
}

int msl_pconv_dgrad(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                    const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, p) || !dy || !packed_dgrad || !dx) return MSL_ERR_ARG;
  return fwd_f32(forms, dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms,
                         ws, ws_bytes, as_stream(stream));
}

int msl_pconv_dgrad_acc(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                        int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, p) || !dy || !packed_dgrad || !dx) return MSL_ERR_ARG;
  if (!accumulate)
    return fwd_f32(forms, dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms, ws, ws_bytes,
                   as_stream(stream));
  return fwd_f32(forms, dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms, ws, ws_bytes,
                 as_stream(stream), 1);
}

static bool bad_parts(const float* p, int n) { return p && n < 1; }

int msl_conv_wgrad_split(int nbranch, int taps, int cin, int cout, int h, int w, int nimg) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || (taps != 1 && taps != 9)) return MSL_ERR_ARG;
  const int P = nimg * h * w;
  const int wr = taps == 1 ? P : w;  // a pointwise call passes one flat row (msl_pconv_wgrad*)
  if (wgrad_swaps(nbranch, taps, cin, cout) && plan_wgrad(nbranch, taps, cout, cin, P, true, wr).rx6) return 1;
  return plan_wgrad(nbranch, taps, cin, cout, P, true, wr).rx6 ? 1 : 0;
}

int msl_absmax_partials(const float* x, int rows, int row_len, float* part, msl_stream_t stream) {
  if (!x || !part || rows < 1 || row_len < 1) return MSL_ERR_ARG;
  return absmax_rows(x, rows, row_len, part, as_stream(stream));
}

int msl_dconv_fwd_sc(const float* x, const float* packed, const float* bias, float* y, int nbranch,
                     int cin, int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                     size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart) {
  if (bad_parts(x_part, x_npart)) return MSL_ERR_ARG;
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !packed || !y || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return fwd_f32(forms, x, cin, packed, cout, bias, nbranch, y, nbranch, 9, h, w, nimg, dil0, dil1, forms, ws, ws_bytes,
                 as_stream(stream), 0, x_part, x_npart);
}

int msl_dconv_dgrad_sc(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin,
                       int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                       size_t ws_bytes, msl_stream_t stream, const float* dy_part, int dy_npart) {
  if (bad_parts(dy_part, dy_npart)) return MSL_ERR_ARG;
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !dy || !packed_dgrad || !dx || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return fwd_f32(forms, dy, cout, packed_dgrad, cin, nullptr, 0, dx, nbranch, 9, h, w, nimg, dil0, dil1, forms, ws,
                 ws_bytes, as_stream(stream), 0, dy_part, dy_npart);
}

int msl_dconv_wgrad_sc(const float* x, const float* dy, float* dw, float* dbias, int nbranch, int cin,
                       int cout, int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms, void* ws,
                       size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart,
                       const float* dy_part, int dy_npart) {
  if (bad_parts(x_part, x_npart) || bad_parts(dy_part, dy_npart)) return MSL_ERR_ARG;
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !dy || !dw || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return wgrad_f32(forms, x, dy, dw, dbias, nbranch, 9, cin, cout, h, w, nimg, dil0, dil1, accumulate, ws, ws_bytes,
                   as_stream(stream), x_part, x_npart, dy_part, dy_npart);
}

int msl_pconv_fwd_sc(const float* x, const float* packed, float* y, int cin, int cout, int p,
                     const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part,
                     int x_npart) {
  if (bad_parts(x_part, x_npart)) return MSL_ERR_ARG;
  if (bad_dims(1, cin, cout, 1, p) || !x || !packed || !y) return MSL_ERR_ARG;
  return fwd_f32(forms, x, cin, packed, cout, nullptr, 0, y, 1, 1, 1, p, 1, 0, 0, forms, ws, ws_bytes,
                 as_stream(stream), 0, x_part, x_npart);
}

int msl_pconv_dgrad_acc_sc(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                           int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream,
                           const float* dy_part, int dy_npart) {
  if (bad_parts(dy_part, dy_npart)) return MSL_ERR_ARG;
  if (bad_dims(1, cin, cout, 1, p) || !dy || !packed_dgrad || !dx) return MSL_ERR_ARG;
  return fwd_f32(forms, dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms, ws, ws_bytes,
                 as_stream(stream), accumulate ? 1 : 0, dy_part, dy_npart);
}

int msl_pconv_dgrad_resmask_sc(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                               const float* res, const unsigned long long* res_mask, int nimg, const msl_forms* forms,
                               void* ws, size_t ws_bytes, msl_stream_t stream, const float* dy_part, int dy_npart) {
  if (bad_parts(dy_part, dy_npart)) return MSL_ERR_ARG;
  if (bad_dims(1, cin, cout, 1, p) || !dy || !packed_dgrad || !dx || !res || !res_mask || nimg < 1 || p % nimg)
    return MSL_ERR_ARG;
  return fwd_f32(forms, dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms, ws, ws_bytes,
                 as_stream(stream), 1, dy_part, dy_npart, res, res_mask, nimg);
}

int msl_pconv_wgrad_sc(const float* x, const float* dy, float* dw, int cin, int cout, int p,
                       int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part,
                       int x_npart, const float* dy_part, int dy_npart) {
  if (bad_parts(x_part, x_npart) || bad_parts(dy_part, dy_npart)) return MSL_ERR_ARG;
  if (bad_dims(1, cin, cout, 1, p) || !x || !dy || !dw) return MSL_ERR_ARG;
  return wgrad_f32(forms, x, dy, dw, nullptr, 1, 1, cin, cout, 1, p, 1, 0, 0, accumulate, ws, ws_bytes, as_stream(stream),
                   x_part, x_npart, dy_part, dy_npart);
}

size_t msl_pconv_wgrad_workspace(int cin, int cout, int p) {
  if (bad_dims(1, cin, cout, 1, p)) return 0;
  return wgrad_ws_bytes(1, 1, cin, cout, p, p);
}

int msl_pconv_wgrad(const float* x, const float* dy, float* dw, int cin, int cout, int p,
                    int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, p) || !x || !dy || !dw) return MSL_ERR_ARG;
  return wgrad_f32(forms, x, dy, dw, nullptr, 1, 1, cin, cout, 1, p, 1, 0, 0, accumulate, ws, ws_bytes,
                      as_stream(stream));
}


// ------------------------------------------------------------------ BF16-MFMA forms
// Same operands, workspaces and results layout; products in bf16 (RNE from the fp32 operands),
// sums in fp32 (BASELINE config 5's fp16/bf16 MFMA path).
int msl_dconv_fwd_bf16(const float* x, const float* packed, const float* bias, float* y, int nbranch,
                  int cin, int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                  size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !packed || !y || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return launch_fwd_form<kMathBf16>(x, cin, packed, cout, bias, nbranch, y, nbranch, 9, h, w, nimg, dil0, dil1,
                         forms, ws, ws_bytes, as_stream(stream));
}

int msl_dconv_dgrad_bf16(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin,
                    int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !dy || !packed_dgrad || !dx || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return launch_fwd_form<kMathBf16>(dy, cout, packed_dgrad, cin, nullptr, 0, dx, nbranch, 9, h, w, nimg, dil0, dil1,
                         forms, ws, ws_bytes, as_stream(stream));
}

int msl_dconv_wgrad_bf16(const float* x, const float* dy, float* dw, float* dbias, int nbranch, int cin,
                    int cout, int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms, void* ws,
                    size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !dy || !dw || dil0 < 1 ||
      (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  if (forms_bad(forms)) return MSL_ERR_ARG;
  return launch_wgrad<kMathBf16>(x, dy, dw, dbias, nbranch, 9, cin, cout, h, w, nimg, dil0, dil1, accumulate, ws,
                      ws_bytes, as_stream(stream));
}

int msl_pconv_fwd_bf16(const float* x, const float* packed, float* y, int cin, int cout, int p,
                  const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, p) || !x || !packed || !y) return MSL_ERR_ARG;
  return launch_fwd_form<kMathBf16>(x, cin, packed, cout, nullptr, 0, y, 1, 1, 1, p, 1, 0, 0, forms, ws,
                         ws_bytes, as_stream(stream));
}

int msl_pconv_dgrad_bf16(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                    const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, p) || !dy || !packed_dgrad || !dx) return MSL_ERR_ARG;
  return launch_fwd_form<kMathBf16>(dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms,
                         ws, ws_bytes, as_stream(stream));
}

int msl_pconv_wgrad_bf16(const float* x, const float* dy, float* dw, int cin, int cout, int p,
                    int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream) {
  if (bad_dims(1, cin, cout, 1, p) || !x || !dy || !dw || forms_bad(forms)) return MSL_ERR_ARG;
  return launch_wgrad<kMathBf16>(x, dy, dw, nullptr, 1, 1, cin, cout, 1, p, 1, 0, 0, accumulate, ws, ws_bytes,
                      as_stream(stream));
}

// ------------------------------------------------------------------ FP16-MFMA forms
// BASELINE config 5's fp16 MFMA path on the f16x3 machinery: each operand tensor scaled by its
// power of two and rounded to fp16 once (the weights at pack time: the f16x3 packs' hi planes,
// so packs must be made in the f16x3 fp32 form, the default), one v_mfma_f32_32x32x16_f16 per
// 16-deep slice, fp32 sums, the result unscaled exactly.  The 64- / 32-row tiles (M <= 64) run
// exact f32 MFMA.  Partials as in the _sc entry points ((pointer, count), NULL = computed).
static bool f16_ready(const msl_forms* forms) { return !forms_bad(forms) && forms_of(forms).f32_form == kMathH3P; }

int msl_dconv_fwd_f16(const float* x, const float* packed, const float* bias, float* y, int nbranch, int cin,
                      int cout, int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws, size_t ws_bytes,
                      msl_stream_t stream, const float* x_part, int x_npart) {
  if (!f16_ready(forms) || bad_parts(x_part, x_npart) || bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !packed || !y ||
      dil0 < 1 || (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return launch_fwd_form<kMathH1P>(x, cin, packed, cout, bias, nbranch, y, nbranch, 9, h, w, nimg, dil0, dil1, forms,
                                   ws, ws_bytes, as_stream(stream), 0, x_part, x_npart);
}

int msl_dconv_dgrad_f16(const float* dy, const float* packed_dgrad, float* dx, int nbranch, int cin, int cout,
                        int h, int w, int nimg, int dil0, int dil1, const msl_forms* forms, void* ws, size_t ws_bytes,
                        msl_stream_t stream, const float* dy_part, int dy_npart) {
  if (!f16_ready(forms) || bad_parts(dy_part, dy_npart) || bad_dims(nbranch, cin, cout, h, w, nimg) || !dy || !packed_dgrad ||
      !dx || dil0 < 1 || (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return launch_fwd_form<kMathH1P>(dy, cout, packed_dgrad, cin, nullptr, 0, dx, nbranch, 9, h, w, nimg, dil0, dil1,
                                   forms, ws, ws_bytes, as_stream(stream), 0, dy_part, dy_npart);
}

int msl_dconv_wgrad_f16(const float* x, const float* dy, float* dw, float* dbias, int nbranch, int cin, int cout,
                        int h, int w, int nimg, int dil0, int dil1, int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes,
                        msl_stream_t stream, const float* x_part, int x_npart, const float* dy_part, int dy_npart) {
  if (!f16_ready(forms) || bad_parts(x_part, x_npart) || bad_parts(dy_part, dy_npart) ||
      bad_dims(nbranch, cin, cout, h, w, nimg) || !x || !dy || !dw || dil0 < 1 || (nbranch == 2 && dil1 < 1))
    return MSL_ERR_ARG;
  return launch_wgrad<kMathH1P>(x, dy, dw, dbias, nbranch, 9, cin, cout, h, w, nimg, dil0, dil1, accumulate, ws, ws_bytes,
                                as_stream(stream), x_part, x_npart, dy_part, dy_npart);
}

int msl_pconv_fwd_f16(const float* x, const float* packed, float* y, int cin, int cout, int p, const msl_forms* forms,
                      void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart) {
  if (!f16_ready(forms) || bad_parts(x_part, x_npart) || bad_dims(1, cin, cout, 1, p) || !x || !packed || !y)
    return MSL_ERR_ARG;
  return launch_fwd_form<kMathH1P>(x, cin, packed, cout, nullptr, 0, y, 1, 1, 1, p, 1, 0, 0, forms, ws, ws_bytes,
                                   as_stream(stream), 0, x_part, x_npart);
}

int msl_pconv_dgrad_f16(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                        int accumulate, const msl_forms* forms, void* ws, size_t ws_bytes, msl_stream_t stream,
                        const float* dy_part, int dy_npart) {
  if (!f16_ready(forms) || bad_parts(dy_part, dy_npart) || bad_dims(1, cin, cout, 1, p) || !dy || !packed_dgrad || !dx)
    return MSL_ERR_ARG;
  return launch_fwd_form<kMathH1P>(dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms, ws,
                                   ws_bytes, as_stream(stream), accumulate ? 1 : 0, dy_part, dy_npart);
}

int msl_pconv_dgrad_resmask_f16(const float* dy, const float* packed_dgrad, float* dx, int cin, int cout, int p,
                                const float* res, const unsigned long long* res_mask, int nimg, const msl_forms* forms,
                                void* ws, size_t ws_bytes, msl_stream_t stream, const float* dy_part, int dy_npart) {
  if (!f16_ready(forms) || bad_parts(dy_part, dy_npart) || bad_dims(1, cin, cout, 1, p) || !dy || !packed_dgrad || !dx ||
      !res || !res_mask || nimg < 1 || p % nimg)
    return MSL_ERR_ARG;
  return launch_fwd_form<kMathH1P>(dy, cout, packed_dgrad, cin, nullptr, 0, dx, 1, 1, 1, p, 1, 0, 0, forms, ws,
                                   ws_bytes, as_stream(stream), 1, dy_part, dy_npart, res, res_mask, nimg);
}

int msl_pconv_wgrad_f16(const float* x, const float* dy, float* dw, int cin, int cout, int p, int accumulate, const msl_forms* forms,
                        void* ws, size_t ws_bytes, msl_stream_t stream, const float* x_part, int x_npart,
                        const float* dy_part, int dy_npart) {
  if (!f16_ready(forms) || bad_parts(x_part, x_npart) || bad_parts(dy_part, dy_npart) || bad_dims(1, cin, cout, 1, p) ||
      !x || !dy || !dw)
    return MSL_ERR_ARG;
  return launch_wgrad<kMathH1P>(x, dy, dw, nullptr, 1, 1, cin, cout, 1, p, 1, 0, 0, accumulate, ws, ws_bytes,
                                as_stream(stream), x_part, x_npart, dy_part, dy_npart);
}

}  // extern "C"

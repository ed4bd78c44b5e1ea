// Experimental bf16x6 stream-K forward kernels, timed against the library's LDS-DMA kernel
// (k_igemm_fwd_sk<.., kMathX6P>) by scripts/tune_dconv.hip modes reg / reg2 / abl; not part of
// the library.  Results: profiles/r02_fwd_kernel_variants.txt, DESIGN.md section 4.
#pragma once
#include "dconv_kernels.h"

namespace msl {

// ---------------------------------------------------------------------------------------------
// Register-staged bf16x6 stream-K forward form (fwd / dgrad of the dilated 3x3 convs and the
// pointwise convs, 128x128 tiles, 4 waves of 64x64).  k_igemm_fwd_sk<.., kMathX6P> moves its B
// operand (fp32 image rows, one shifted pixel per lane) by LDS-DMA - one dword per lane, 8 of those
// ~60-cycle issues per wave and stage beside 3 for A - and every wave then splits the fp32 values
// of its own B fragments into bf16 planes, so each B element is split by both waves that share its
// pixel columns.  Here the operands go through registers instead:
//   - each thread loads one pixel x 8 channels of the stage's B tile (eight coalesced dword buffer
//     loads; out-of-image / padding channels come back 0 from the buffer unit), splits them once
//     into the three bf16 planes and writes three 16-B vectors, and loads three 16-B vectors of the
//     pre-split A planes (k_pack_split layout) and writes them;
//   - LDS holds both operands as [plane][k half][128][8] bf16, so every fragment is one
//     conflict-free ds_read_b128 per plane and the MFMA loop has no split work left;
//   - stage s+1 is loaded into registers before the MFMAs of stage s and written after them
//     (issue early / write late), double-buffered LDS, one barrier per stage.
// Same iteration space, pieces, reduce (k_sk_reduce<128, 128>) and results as the DMA kernel.
// EXP != 0 are timing ablations for the tuning harness (wrong results), a bit mask: 1 = every
// stage loads K-step 0 (cache-resident operands), 2 = no MFMAs, 4 = no global operand loads,
// 8 = no piece / output stores, 16 = no split (B's fp32 bits written as the planes), 32 = A not
// written to LDS, 64 = A fragments from the thread's own loaded registers (no A LDS reads).
template <int EXP = 0>
__global__ void __launch_bounds__(256, 2) k_x6_sk(FwdArgs a, SkArgs sk) {
  constexpr int BM = 128, BN = 128, TM = 2, TN = 2;
  constexpr int VEC = 6 * 128;                   // 16-B vectors per operand per stage
  constexpr int STAGE = 2 * VEC;                 // A then B
  __shared__ __attribute__((aligned(16))) bf16x8 smem[2 * STAGE];  // 48 KB: the only LDS object

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const int l32 = lane & 31, kh = lane >> 5;
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);  // XCD-aware worker id
  const int T = sk.T;
  const int it_begin = sk_start(w, T, sk.NW), it_end = sk_start(w + 1, T, sk.NW);

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Ax6, (short)0, (int)min(0x7fffffffLL, (long long)a.ksteps * 6 * a.lda * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.B, (short)0, (int)min(0x7fffffffLL, (long long)a.cimg * a.P * 4), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned chan_bytes = (unsigned)a.P * 4u;
  const int bn = tid & 127, bh = tid >> 7;  // this thread's B pixel column and channel half

  f32x16 acc[TM][TN];
  for (int it = it_begin; it < it_end;) {
    const int t = (unsigned)it / (unsigned)sk.KS;
    const int k_a = it - t * sk.KS;
    const int k_b = min(sk.KS, k_a + (it_end - it));
    const int nst = k_b - k_a;
    it += nst;
    int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const int p = n0 + bn;
    const bool pin = p < a.P;
    const int py = p / a.W, px = p - py * a.W;
    // K cursor: ks = (branch*taps + tap)*ncb + cb; the shifted pixel offset changes with the tap
    int c_cb, c_tap, ks = k_a;
    {
      const int tq = k_a / a.ncb;
      c_cb = k_a - tq * a.ncb;
      c_tap = tq;
    }
    unsigned vrow = OOB;
    auto set_tap = [&](int tq) {
      const int br = tq / a.taps;
      const int tp = tq - br * a.taps;
      const int d = br ? a.dil1 : a.dil0;
      const int dh = (tp / 3 - 1) * d, dw = (tp % 3 - 1) * d;
      const bool v = pin && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
      vrow = v ? (unsigned)((p + dh * a.W + dw) * 4) : OOB;
    };
    set_tap(c_tap);
    u32x4 ra[3], ra_keep[3];
    float rbv[8];
    // per-thread parts of the load offsets (VGPRs, fixed for the segment); the K-step, plane and
    // channel parts go in the scalar offset, so a stage's loads cost no vector ALU work
    const unsigned a_voff = (unsigned)((((tid >> 7) * a.lda) + m0 + (tid & 127)) * 16);
    const unsigned a_plane_bytes = (unsigned)a.lda * 16u;
    const bool full_cb = (a.cimg & (kCB - 1)) == 0;  // no padding channel in any block
    auto load = [&]() {  // the operands of K-step ks into registers; advances the cursor
#pragma unroll
      for (int i = 0; i < 3; ++i)  // vectors tid + 256 i: (plane*2 + half) = tid/128 + 2i, m = tid % 128
        if constexpr (EXP & 4) ra[i] = u32x4{(unsigned)tid, (unsigned)i, (unsigned)ks, 0u};
        else ra[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, a_voff,
                                                           (int)((unsigned)((EXP & 1 ? 0 : ks) * 6 + 2 * i) * a_plane_bytes), 0);
      const int c0 = (EXP & 1 ? 0 : c_cb) * kCB + 8 * bh;
      if constexpr (EXP & 4) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rbv[j] = (float)(tid + j + ks);
      } else if (full_cb) {
        const unsigned vb = vrow + (unsigned)c0 * chan_bytes;  // OOB stays out of range
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rbv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vb, (int)(j * chan_bytes), 0));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned cofs = c0 + j < a.cimg ? (unsigned)(c0 + j) * chan_bytes : OOB;
          rbv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vrow + cofs, 0, 0));
        }
      }
      ++ks;
      if (++c_cb == a.ncb) {
        c_cb = 0;
        if (++c_tap * a.ncb < a.ksteps) set_tap(c_tap);
      }
    };
    auto store = [&](int buf) {  // split B once, write both operands' planes
      bf16x8* As = smem + buf * STAGE;
      bf16x8* Bs = As + VEC;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        union { u32x4 u; bf16x8 h; } cv;
        cv.u = ra[i];
        if constexpr (EXP & 64) ra_keep[i] = ra[i];
        if constexpr (!(EXP & 32)) As[tid + 256 * i] = cv.h;
      }
      Split3 sp;
      if constexpr (EXP & 16) {
        union { float f[8]; bf16x8 h[2]; } raw;
#pragma unroll
        for (int j = 0; j < 8; ++j) raw.f[j] = rbv[j];
        sp.hi = raw.h[0];
        sp.mid = raw.h[1];
        sp.lo = raw.h[0];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) split3_set(sp, j, rbv[j]);
      }
      Bs[bh * 128 + bn] = sp.hi;
      Bs[(2 + bh) * 128 + bn] = sp.mid;
      Bs[(4 + bh) * 128 + bn] = sp.lo;
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __syncthreads();  // the previous segment's LDS reads are complete in every wave
    load();
    store(0);
    __syncthreads();
    for (int i = 0; i < nst; ++i) {
      const bool more = i + 1 < nst;
      if (more) load();  // stage i+1: in flight during this stage's MFMAs
      const bf16x8* As = smem + (i & 1) * STAGE;
      const bf16x8* Bs = As + VEC;
      Split3 av[TM], bv[TN];
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) {
        const int m = wm + ii * 32 + l32;
        if constexpr (EXP & 64) {
          union { u32x4 u; bf16x8 h; } c0, c1, c2;
          c0.u = ra_keep[0]; c1.u = ra_keep[1]; c2.u = ra_keep[2];
          av[ii].hi = c0.h; av[ii].mid = c1.h; av[ii].lo = c2.h;
        } else {
          av[ii].hi = As[kh * 128 + m];
          av[ii].mid = As[(2 + kh) * 128 + m];
          av[ii].lo = As[(4 + kh) * 128 + m];
        }
      }
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        const int n = wn + jj * 32 + l32;
        bv[jj].hi = Bs[kh * 128 + n];
        bv[jj].mid = Bs[(2 + kh) * 128 + n];
        bv[jj].lo = Bs[(4 + kh) * 128 + n];
      }
      if constexpr (EXP & 2) {  // keep the fragment reads live
#pragma unroll
        for (int ii = 0; ii < TM; ++ii)
          acc[ii][0][0] += (float)av[ii].hi[0] + (float)av[ii].mid[0] + (float)av[ii].lo[0];
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
          acc[0][jj][1] += (float)bv[jj].hi[0] + (float)bv[jj].mid[0] + (float)bv[jj].lo[0];
      } else {
#pragma unroll
        for (int ii = 0; ii < TM; ++ii)
#pragma unroll
          for (int jj = 0; jj < TN; ++jj) acc[ii][jj] = mfma_x6(av[ii], bv[jj], acc[ii][jj]);
      }
      if (more) store((i + 1) & 1);
      __syncthreads();
    }

    constexpr int PSZ = BM * BN;
    if constexpr (EXP & 8) {
      const float live = acc[0][0][0] + acc[0][1][0] + acc[1][0][0] + acc[1][1][0];  // every MFMA chain live
      if (live == 1.2345f) a.C[tid] = live;
      continue;
    }
    if (k_a > 0 || k_b < sk.KS) {  // a piece of a split tile (as k_igemm_fwd_sk)
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)sk.part, (short)0, (int)min(0x7fffffffLL, (long long)sk.NW * 2 * PSZ * 4), 0x00020000);
      const unsigned pbase = (unsigned)((w * 2 + (k_a > 0 ? 0 : 1)) * PSZ * 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nl = wn + j * 32 + l32;
          const int ml = wm + i * 32 + 4 * kh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ro = (r & 3) + 8 * (r >> 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                  pbase + (unsigned)(((ml + ro) * BN + nl) * 4), 0, 0);
          }
        }
      continue;
    }
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.C, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + j * 32 + l32;
        const int mrow = m0 + wm + i * 32 + 4 * kh;
        const unsigned voff = n < a.P ? (unsigned)((mrow * a.P + n) * 4) : OOB;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          float v = acc[i][j][r];
          if (a.bias && mrow + ro < a.M) {
            float bsum = a.bias[mrow + ro];
            for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + mrow + ro];
            v += bsum;
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc,
                                                mrow + ro < a.M ? voff + ro * a.P * 4 : OOB, 0, 0);
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
// k_x6_sk with the A operand kept out of LDS: every wave loads its own fragments of the pre-split
// weight planes (k_pack_split layout: one 16-B vector per lane and plane, the row of the lane, the
// k half of the half-wave) straight into registers one K-step ahead, and the LDS holds only B
// (split once per element).  Two K-steps per LDS stage: per 48 MFMAs per wave, 6 16-B LDS stores
// per thread, 12 16-B fragment reads per wave and one barrier (k_x6_sk: twice the stores and reads
// and two barriers).  Same iteration space, pieces, reduce and results as k_x6_sk.
__global__ void __launch_bounds__(256, 2) k_x6_sk2(FwdArgs a, SkArgs sk) {
  constexpr int BM = 128, BN = 128, TM = 2, TN = 2;
  constexpr int KV = 6 * 128;     // 16-B vectors of one K-step's B planes [plane][k half][128]
  constexpr int STAGE = 2 * KV;   // two K-steps
  __shared__ __attribute__((aligned(16))) bf16x8 smem[2 * STAGE];  // 48 KB: the only LDS object

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const int l32 = lane & 31, kh = lane >> 5;
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);  // XCD-aware worker id
  const int T = sk.T;
  const int it_begin = sk_start(w, T, sk.NW), it_end = sk_start(w + 1, T, sk.NW);

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Ax6, (short)0, (int)min(0x7fffffffLL, (long long)a.ksteps * 6 * a.lda * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.B, (short)0, (int)min(0x7fffffffLL, (long long)a.cimg * a.P * 4), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned chan_bytes = (unsigned)a.P * 4u;
  const unsigned a_plane_bytes = (unsigned)a.lda * 16u;
  const bool full_cb = (a.cimg & (kCB - 1)) == 0;  // no padding channel in any block
  const int bn = tid & 127, bh = tid >> 7;          // this thread's B pixel column and channel half

  f32x16 acc[TM][TN];
  for (int it = it_begin; it < it_end;) {
    const int t = (unsigned)it / (unsigned)sk.KS;
    const int k_a = it - t * sk.KS;
    const int k_b = min(sk.KS, k_a + (it_end - it));
    const int nst = k_b - k_a;
    it += nst;
    int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const int p = n0 + bn;
    const bool pin = p < a.P;
    const int py = p / a.W, px = p - py * a.W;
    int c_cb, c_tap;  // B cursor: ks = (branch*taps + tap)*ncb + cb
    {
      const int tq = k_a / a.ncb;
      c_cb = k_a - tq * a.ncb;
      c_tap = tq;
    }
    unsigned vrow = OOB;
    auto set_tap = [&](int tq) {
      const int br = tq / a.taps;
      const int tp = tq - br * a.taps;
      const int d = br ? a.dil1 : a.dil0;
      const int dh = (tp / 3 - 1) * d, dw = (tp % 3 - 1) * d;
      const bool v = pin && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
      vrow = v ? (unsigned)((p + dh * a.W + dw) * 4) : OOB;
    };
    set_tap(c_tap);
    float rbv[16];
    auto loadB = [&](int j0) {  // one K-step of this thread's B column into rbv[j0 .. j0+7]
      const int c0 = c_cb * kCB + 8 * bh;
      if (full_cb) {
        const unsigned vb = vrow + (unsigned)c0 * chan_bytes;  // OOB stays out of range
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rbv[j0 + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vb, (int)(j * chan_bytes), 0));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned cofs = c0 + j < a.cimg ? (unsigned)(c0 + j) * chan_bytes : OOB;
          rbv[j0 + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vrow + cofs, 0, 0));
        }
      }
      if (++c_cb == a.ncb) {
        c_cb = 0;
        if (++c_tap * a.ncb < a.ksteps) set_tap(c_tap);
      }
    };
    auto storeB = [&](int buf, int j0, int kk) {  // split once, three 16-B plane vectors
      Split3 sp;
#pragma unroll
      for (int j = 0; j < 8; ++j) split3_set(sp, j, rbv[j0 + j]);
      bf16x8* Bs = smem + buf * STAGE + kk * KV;
      Bs[bh * 128 + bn] = sp.hi;
      Bs[(2 + bh) * 128 + bn] = sp.mid;
      Bs[(4 + bh) * 128 + bn] = sp.lo;
    };
    // this wave's A fragment rows; K-step and plane in the scalar offset
    const unsigned a_voff = (unsigned)((kh * a.lda + m0 + wm + l32) * 16);
    u32x4 A0[TM][3], A1[TM][3];
    auto loadA = [&](u32x4 (&A)[TM][3], int ks) {
#pragma unroll
      for (int ii = 0; ii < TM; ++ii)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          A[ii][q] = __builtin_amdgcn_raw_buffer_load_b128(rx, a_voff + ii * 512,
                                                           (int)((unsigned)(ks * 6 + 2 * q) * a_plane_bytes), 0);
    };
    auto compute = [&](const bf16x8* Bs, const u32x4 (&A)[TM][3]) {
      Split3 bv[TN];
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        const int n = wn + jj * 32 + l32;
        bv[jj].hi = Bs[kh * 128 + n];
        bv[jj].mid = Bs[(2 + kh) * 128 + n];
        bv[jj].lo = Bs[(4 + kh) * 128 + n];
      }
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) {
        union { u32x4 u; bf16x8 h; } c0, c1, c2;
        c0.u = A[ii][0]; c1.u = A[ii][1]; c2.u = A[ii][2];
        Split3 av;
        av.hi = c0.h; av.mid = c1.h; av.lo = c2.h;
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) acc[ii][jj] = mfma_x6(av, bv[jj], acc[ii][jj]);
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __syncthreads();  // the previous segment's LDS reads are complete in every wave
    const bool two0 = nst > 1;
    loadB(0);
    if (two0) loadB(8);
    loadA(A0, k_a);
    storeB(0, 0, 0);
    if (two0) storeB(0, 8, 1);
    __syncthreads();
    int ks = k_a;  // the K-step computed next
    for (int s = 0; 2 * s < nst; ++s) {
      const int left = nst - 2 * s;   // K-steps from this stage on
      const int nxt = left - 2;       // K-steps of the next stage (<= 0: none)
      if (nxt > 0) {                  // next stage's B: in flight during this stage's MFMAs
        loadB(0);
        if (nxt > 1) loadB(8);
      }
      const bf16x8* Bs = smem + (s & 1) * STAGE;
      if (ks + 1 < k_b) loadA(A1, ks + 1);
      compute(Bs, A0);
      ++ks;
      if (left > 1) {
        if (ks + 1 < k_b) loadA(A0, ks + 1);
        compute(Bs + KV, A1);
        ++ks;
      }
      if (nxt > 0) {
        storeB((s + 1) & 1, 0, 0);
        if (nxt > 1) storeB((s + 1) & 1, 8, 1);
      }
      __syncthreads();
    }

    constexpr int PSZ = BM * BN;
    if (k_a > 0 || k_b < sk.KS) {  // a piece of a split tile (as k_igemm_fwd_sk)
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)sk.part, (short)0, (int)min(0x7fffffffLL, (long long)sk.NW * 2 * PSZ * 4), 0x00020000);
      const unsigned pbase = (unsigned)((w * 2 + (k_a > 0 ? 0 : 1)) * PSZ * 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nl = wn + j * 32 + l32;
          const int ml = wm + i * 32 + 4 * kh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ro = (r & 3) + 8 * (r >> 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                  pbase + (unsigned)(((ml + ro) * BN + nl) * 4), 0, 0);
          }
        }
      continue;
    }
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.C, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + j * 32 + l32;
        const int mrow = m0 + wm + i * 32 + 4 * kh;
        const unsigned voff = n < a.P ? (unsigned)((mrow * a.P + n) * 4) : OOB;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          float v = acc[i][j][r];
          if (a.bias && mrow + ro < a.M) {
            float bsum = a.bias[mrow + ro];
            for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + mrow + ro];
            v += bsum;
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc,
                                                mrow + ro < a.M ? voff + ro * a.P * 4 : OOB, 0, 0);
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
// k_x6_sk2 on v_mfma_f32_16x16x32_bf16: the same operands, LDS layout and stream-K structure, a
// 64x64 wave tile as 4x4 blocks of 16x16 with K = 32 (one LDS stage = two K-steps) per MFMA.
// Both MFMA shapes have the same cycles per FLOP, but on an MFMA-dense loop the chip holds a
// higher clock for the 16x16 shape (MI355X_MICROARCH.md, DVFS item 7).  Lane (l16, g = lane/16)
// of an operand takes K-step g/2, k half g%2 of the stage.  A: one 16-B vector per lane and plane
// from the pre-split planes, each row block refilled right after its last MFMA of a stage (a
// full stage of cover before its next use).
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16_x6(const Split3& a, const Split3& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.mid, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.mid, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, c, 0, 0, 0);
}

__global__ void __launch_bounds__(256, 2) k_x6_sk3(FwdArgs a, SkArgs sk) {
  constexpr int BM = 128, BN = 128, TB = 4;  // 4x4 blocks of 16x16 per wave
  constexpr int KV = 6 * 128;
  constexpr int STAGE = 2 * KV;
  __shared__ __attribute__((aligned(16))) bf16x8 smem[2 * STAGE];  // 48 KB: the only LDS object

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const int l16 = lane & 15, g = lane >> 4;
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);  // XCD-aware worker id
  const int T = sk.T;
  const int it_begin = sk_start(w, T, sk.NW), it_end = sk_start(w + 1, T, sk.NW);

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Ax6, (short)0, (int)min(0x7fffffffLL, (long long)a.ksteps * 6 * a.lda * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.B, (short)0, (int)min(0x7fffffffLL, (long long)a.cimg * a.P * 4), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned chan_bytes = (unsigned)a.P * 4u;
  const unsigned a_plane_bytes = (unsigned)a.lda * 16u;
  const bool full_cb = (a.cimg & (kCB - 1)) == 0;
  const int bn = tid & 127, bh = tid >> 7;

  f32x4 acc[TB][TB];
  for (int it = it_begin; it < it_end;) {
    const int t = (unsigned)it / (unsigned)sk.KS;
    const int k_a = it - t * sk.KS;
    const int k_b = min(sk.KS, k_a + (it_end - it));
    const int nst = k_b - k_a;
    it += nst;
    int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const int p = n0 + bn;
    const bool pin = p < a.P;
    const int py = p / a.W, px = p - py * a.W;
    int c_cb, c_tap;
    {
      const int tq = k_a / a.ncb;
      c_cb = k_a - tq * a.ncb;
      c_tap = tq;
    }
    unsigned vrow = OOB;
    auto set_tap = [&](int tq) {
      const int br = tq / a.taps;
      const int tp = tq - br * a.taps;
      const int d = br ? a.dil1 : a.dil0;
      const int dh = (tp / 3 - 1) * d, dw = (tp % 3 - 1) * d;
      const bool v = pin && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
      vrow = v ? (unsigned)((p + dh * a.W + dw) * 4) : OOB;
    };
    set_tap(c_tap);
    float rbv[16];
    auto loadB = [&](int j0) {
      const int c0 = c_cb * kCB + 8 * bh;
      if (full_cb) {
        const unsigned vb = vrow + (unsigned)c0 * chan_bytes;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rbv[j0 + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vb, (int)(j * chan_bytes), 0));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned cofs = c0 + j < a.cimg ? (unsigned)(c0 + j) * chan_bytes : OOB;
          rbv[j0 + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vrow + cofs, 0, 0));
        }
      }
      if (++c_cb == a.ncb) {
        c_cb = 0;
        if (++c_tap * a.ncb < a.ksteps) set_tap(c_tap);
      }
    };
    auto storeB = [&](int buf, int j0, int kk) {
      Split3 sp;
#pragma unroll
      for (int j = 0; j < 8; ++j) split3_set(sp, j, rbv[j0 + j]);
      bf16x8* Bs = smem + buf * STAGE + kk * KV;
      Bs[bh * 128 + bn] = sp.hi;
      Bs[(2 + bh) * 128 + bn] = sp.mid;
      Bs[(4 + bh) * 128 + bn] = sp.lo;
    };
    // A: lane (l16, g) reads plane row ((ks + g/2)*3 + q)*2 + g%2 of column m0 + wm + 16*ii + l16;
    // a stage's second K-step must exist (else the lane reads zeros past the planes' end)
    const unsigned a_voff = (unsigned)((((g >> 1) * 6 + (g & 1)) * a.lda + m0 + wm + l16) * 16);
    u32x4 A[TB][3];
    auto loadA = [&](int ii, int ks, bool two) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
        A[ii][q] = __builtin_amdgcn_raw_buffer_load_b128(
            rx, (two || g < 2) ? a_voff + ii * 256 : OOB, (int)((unsigned)(ks * 6 + 2 * q) * a_plane_bytes), 0);
    };
#pragma unroll
    for (int i = 0; i < TB; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const bool two0 = nst > 1;
    loadB(0);
    if (two0) loadB(8);
#pragma unroll
    for (int ii = 0; ii < TB; ++ii) loadA(ii, k_a, two0);
    storeB(0, 0, 0);
    if (two0) storeB(0, 8, 1);
    else {  // a lone K-step: the second half of the stage reads zeros
      bf16x8* Bs = smem + KV;
      const bf16x8 z = {};
      Bs[bh * 128 + bn] = z; Bs[(2 + bh) * 128 + bn] = z; Bs[(4 + bh) * 128 + bn] = z;
    }
    __syncthreads();
    int ks = k_a;  // first K-step of the stage being computed
    for (int s = 0; 2 * s < nst; ++s) {
      const int left = nst - 2 * s;
      const int nxt = left - 2;  // K-steps of the next stage
      const bf16x8* Bs = smem + (s & 1) * STAGE;
      Split3 bv[TB];
#pragma unroll
      for (int jj = 0; jj < TB; ++jj) {
        const int n = wn + jj * 16 + l16;
        const bf16x8* src = Bs + (g >> 1) * KV + (g & 1) * 128 + n;
        bv[jj].hi = src[0];
        bv[jj].mid = src[256];
        bv[jj].lo = src[512];
      }
#pragma unroll
      for (int ii = 0; ii < TB; ++ii) {
        Split3 av;
        union { u32x4 u; bf16x8 h; } c0, c1, c2;
        c0.u = A[ii][0]; c1.u = A[ii][1]; c2.u = A[ii][2];
        av.hi = c0.h; av.mid = c1.h; av.lo = c2.h;
#pragma unroll
        for (int jj = 0; jj < TB; ++jj) acc[ii][jj] = mfma16_x6(av, bv[jj], acc[ii][jj]);
        if (nxt > 0) loadA(ii, ks + 2, nxt > 1);  // this row block of the next stage
        if (ii == 1 && nxt > 0) {  // next stage's B (issued here: fewer registers live at the stage head)
          loadB(0);
          if (nxt > 1) loadB(8);
        }
      }
      if (nxt > 0) {
        storeB((s + 1) & 1, 0, 0);
        if (nxt > 1) storeB((s + 1) & 1, 8, 1);
        else {
          bf16x8* Bz = smem + ((s + 1) & 1) * STAGE + KV;
          const bf16x8 z = {};
          Bz[bh * 128 + bn] = z; Bz[(2 + bh) * 128 + bn] = z; Bz[(4 + bh) * 128 + bn] = z;
        }
      }
      ks += 2;
      __syncthreads();
    }

    constexpr int PSZ = BM * BN;
    if (k_a > 0 || k_b < sk.KS) {  // a piece of a split tile, row-major [BM][BN] (k_sk_reduce<128, 128>)
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)sk.part, (short)0, (int)min(0x7fffffffLL, (long long)sk.NW * 2 * PSZ * 4), 0x00020000);
      const unsigned pbase = (unsigned)((w * 2 + (k_a > 0 ? 0 : 1)) * PSZ * 4);
#pragma unroll
      for (int i = 0; i < TB; ++i)
#pragma unroll
        for (int j = 0; j < TB; ++j) {
          const int nl = wn + j * 16 + l16;
          const int ml = wm + i * 16 + 4 * g;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                  pbase + (unsigned)(((ml + r) * BN + nl) * 4), 0, 0);
        }
      continue;
    }
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.C, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < TB; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) {
        const int n = n0 + wn + j * 16 + l16;
        const int mrow = m0 + wm + i * 16 + 4 * g;
        const unsigned voff = n < a.P ? (unsigned)((mrow * a.P + n) * 4) : OOB;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r];
          if (a.bias && mrow + r < a.M) {
            float bsum = a.bias[mrow + r];
            for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + mrow + r];
            v += bsum;
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc,
                                                mrow + r < a.M ? voff + r * a.P * 4 : OOB, 0, 0);
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
// k_x6_sk2 with two K-groups per workgroup: 512 threads, one workgroup per CU (NW = 256), waves
// 0-3 and 4-7 each run the k_x6_sk2 loop on one half of the worker's K range of a tile, with
// LDS rings of their own (2 x 48 KB), and the two partial tiles are summed through LDS before the
// piece / output store.  Stream-K leaves ~NW + tiles pieces: half the workers, half the piece
// bytes (and reduce reads) of the 512-worker kernels at the same occupancy.
__global__ void __launch_bounds__(512, 1) k_x6_sk4(FwdArgs a, SkArgs sk) {
  constexpr int BM = 128, BN = 128, TM = 2, TN = 2;
  constexpr int KV = 6 * 128;
  constexpr int STAGE = 2 * KV;
  __shared__ __attribute__((aligned(16))) bf16x8 smem[2 * 2 * STAGE];  // 96 KB: the only LDS object

  const int tid = threadIdx.x, lane = tid & 63;
  const int grp = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gt = tid & 255;
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = (gw >> 1) * 64, wn = (gw & 1) * 64;
  const int l32 = lane & 31, kh = lane >> 5;
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);
  const int T = sk.T;
  const int it_begin = sk_start(w, T, sk.NW), it_end = sk_start(w + 1, T, sk.NW);

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Ax6, (short)0, (int)min(0x7fffffffLL, (long long)a.ksteps * 6 * a.lda * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.B, (short)0, (int)min(0x7fffffffLL, (long long)a.cimg * a.P * 4), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned chan_bytes = (unsigned)a.P * 4u;
  const unsigned a_plane_bytes = (unsigned)a.lda * 16u;
  const bool full_cb = (a.cimg & (kCB - 1)) == 0;
  const int bn = gt & 127, bh = gt >> 7;
  bf16x8* gsm = smem + grp * 2 * STAGE;  // this group's ring

  f32x16 acc[TM][TN];
  for (int it = it_begin; it < it_end;) {
    const int t = (unsigned)it / (unsigned)sk.KS;
    const int k_a = it - t * sk.KS;
    const int k_b = min(sk.KS, k_a + (it_end - it));
    const int nst = k_b - k_a;
    it += nst;
    int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    // this group's K-steps: group 0 the first ceil(nst/2), group 1 the rest
    const int h0 = (nst + 1) >> 1;
    const int g_a = grp ? k_a + h0 : k_a;
    const int g_n = grp ? nst - h0 : h0;
    const int g_b = g_a + g_n;
    const int nstages = (h0 + 1) >> 1;  // both groups run as many barriers as group 0
    const int p = n0 + bn;
    const bool pin = p < a.P;
    const int py = p / a.W, px = p - py * a.W;
    int c_cb, c_tap;
    {
      const int tq = g_a / a.ncb;
      c_cb = g_a - tq * a.ncb;
      c_tap = tq;
    }
    unsigned vrow = OOB;
    auto set_tap = [&](int tq) {
      const int br = tq / a.taps;
      const int tp = tq - br * a.taps;
      const int d = br ? a.dil1 : a.dil0;
      const int dh = (tp / 3 - 1) * d, dw = (tp % 3 - 1) * d;
      const bool v = pin && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
      vrow = v ? (unsigned)((p + dh * a.W + dw) * 4) : OOB;
    };
    if (g_n > 0) set_tap(c_tap);
    float rbv[16];
    auto loadB = [&](int j0) {
      const int c0 = c_cb * kCB + 8 * bh;
      if (full_cb) {
        const unsigned vb = vrow + (unsigned)c0 * chan_bytes;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rbv[j0 + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vb, (int)(j * chan_bytes), 0));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned cofs = c0 + j < a.cimg ? (unsigned)(c0 + j) * chan_bytes : OOB;
          rbv[j0 + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vrow + cofs, 0, 0));
        }
      }
      if (++c_cb == a.ncb) {
        c_cb = 0;
        if (++c_tap * a.ncb < a.ksteps) set_tap(c_tap);
      }
    };
    auto storeB = [&](int buf, int j0, int kk) {
      Split3 sp;
#pragma unroll
      for (int j = 0; j < 8; ++j) split3_set(sp, j, rbv[j0 + j]);
      bf16x8* Bs = gsm + buf * STAGE + kk * KV;
      Bs[bh * 128 + bn] = sp.hi;
      Bs[(2 + bh) * 128 + bn] = sp.mid;
      Bs[(4 + bh) * 128 + bn] = sp.lo;
    };
    const unsigned a_voff = (unsigned)((kh * a.lda + m0 + wm + l32) * 16);
    u32x4 A0[TM][3], A1[TM][3];
    auto loadA = [&](u32x4 (&A)[TM][3], int ks) {
#pragma unroll
      for (int ii = 0; ii < TM; ++ii)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          A[ii][q] = __builtin_amdgcn_raw_buffer_load_b128(rx, a_voff + ii * 512,
                                                           (int)((unsigned)(ks * 6 + 2 * q) * a_plane_bytes), 0);
    };
    auto compute = [&](const bf16x8* Bs, const u32x4 (&A)[TM][3]) {
      Split3 bv[TN];
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        const int n = wn + jj * 32 + l32;
        bv[jj].hi = Bs[kh * 128 + n];
        bv[jj].mid = Bs[(2 + kh) * 128 + n];
        bv[jj].lo = Bs[(4 + kh) * 128 + n];
      }
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) {
        union { u32x4 u; bf16x8 h; } c0, c1, c2;
        c0.u = A[ii][0]; c1.u = A[ii][1]; c2.u = A[ii][2];
        Split3 av;
        av.hi = c0.h; av.mid = c1.h; av.lo = c2.h;
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) acc[ii][jj] = mfma_x6(av, bv[jj], acc[ii][jj]);
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __syncthreads();  // the previous segment's LDS reads (and the partial-sum exchange) are done
    if (g_n > 0) {
      loadB(0);
      if (g_n > 1) loadB(8);
      loadA(A0, g_a);
      storeB(0, 0, 0);
      if (g_n > 1) storeB(0, 8, 1);
    }
    __syncthreads();
    int ks = g_a;
    for (int s = 0; s < nstages; ++s) {
      const int left = g_n - 2 * s;  // this group's K-steps from this stage on (<= 0: idle)
      const int nxt = left - 2;
      if (nxt > 0) {
        loadB(0);
        if (nxt > 1) loadB(8);
      }
      const bf16x8* Bs = gsm + (s & 1) * STAGE;
      if (left > 0) {
        if (ks + 1 < g_b) loadA(A1, ks + 1);
        compute(Bs, A0);
        ++ks;
        if (left > 1) {
          if (ks + 1 < g_b) loadA(A0, ks + 1);
          compute(Bs + KV, A1);
          ++ks;
        }
      }
      if (nxt > 0) {
        storeB((s + 1) & 1, 0, 0);
        if (nxt > 1) storeB((s + 1) & 1, 8, 1);
      }
      __syncthreads();
    }
    // group 1's partial tile -> LDS (each wave its 64x64 quadrant, lane-linear), group 0 adds it
    float* xs = reinterpret_cast<float*>(smem);
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) xs[((gw * 4 + i * 2 + j) * 16 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (grp == 1) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] += xs[((gw * 4 + i * 2 + j) * 16 + r) * 64 + lane];

    constexpr int PSZ = BM * BN;
    if (k_a > 0 || k_b < sk.KS) {
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)sk.part, (short)0, (int)min(0x7fffffffLL, (long long)sk.NW * 2 * PSZ * 4), 0x00020000);
      const unsigned pbase = (unsigned)((w * 2 + (k_a > 0 ? 0 : 1)) * PSZ * 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nl = wn + j * 32 + l32;
          const int ml = wm + i * 32 + 4 * kh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ro = (r & 3) + 8 * (r >> 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                  pbase + (unsigned)(((ml + ro) * BN + nl) * 4), 0, 0);
          }
        }
      continue;
    }
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.C, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + j * 32 + l32;
        const int mrow = m0 + wm + i * 32 + 4 * kh;
        const unsigned voff = n < a.P ? (unsigned)((mrow * a.P + n) * 4) : OOB;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          float v = acc[i][j][r];
          if (a.bias && mrow + ro < a.M) {
            float bsum = a.bias[mrow + ro];
            for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + mrow + ro];
            v += bsum;
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc,
                                                mrow + ro < a.M ? voff + ro * a.P * 4 : OOB, 0, 0);
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
// 16x16x32 form for the clock: 512 threads (8 waves of 32x64, one workgroup per CU, NW = 256),
// A fragments straight from the planes into registers (a stage = two K-steps = one K = 32 MFMA
// slab), B split once into LDS by all 512 threads.  Per wave and stage: 2 row blocks x 4 column
// blocks x 6 products of v_mfma_f32_16x16x32_bf16 (the same FLOPs per SIMD as two 32x32x16
// waves of 64x64), 24 A + 48 B fragment registers, 32 accumulators.
__global__ void __launch_bounds__(512, 1) k_x6_sk5(FwdArgs a, SkArgs sk) {
  constexpr int BM = 128, BN = 128, TI = 2, TJ = 4;
  constexpr int KV = 6 * 128;
  constexpr int STAGE = 2 * KV;
  __shared__ __attribute__((aligned(16))) bf16x8 smem[2 * STAGE];  // 48 KB: the only LDS object

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int l16 = lane & 15, g = lane >> 4;
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);
  const int T = sk.T;
  const int it_begin = sk_start(w, T, sk.NW), it_end = sk_start(w + 1, T, sk.NW);

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Ax6, (short)0, (int)min(0x7fffffffLL, (long long)a.ksteps * 6 * a.lda * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.B, (short)0, (int)min(0x7fffffffLL, (long long)a.cimg * a.P * 4), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned chan_bytes = (unsigned)a.P * 4u;
  const unsigned a_plane_bytes = (unsigned)a.lda * 16u;
  const bool full_cb = (a.cimg & (kCB - 1)) == 0;
  // B staging: thread -> pixel column bn, K-step kk of the stage, channel half bh
  const int bn = tid & 127, bkk = (tid >> 7) & 1, bh = tid >> 8;

  f32x4 acc[TI][TJ];
  for (int it = it_begin; it < it_end;) {
    const int t = (unsigned)it / (unsigned)sk.KS;
    const int k_a = it - t * sk.KS;
    const int k_b = min(sk.KS, k_a + (it_end - it));
    const int nst = k_b - k_a;
    it += nst;
    int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const int p = n0 + bn;
    const bool pin = p < a.P;
    const int py = p / a.W, px = p - py * a.W;
    // this thread's B cursor runs over the K-steps k_a + bkk, k_a + bkk + 2, ...
    auto vrow_of = [&](int ks) -> unsigned {
      const int tq = ks / a.ncb;
      const int br = tq / a.taps;
      const int tp = tq - br * a.taps;
      const int d = br ? a.dil1 : a.dil0;
      const int dh = (tp / 3 - 1) * d, dw = (tp % 3 - 1) * d;
      const bool v = pin && (unsigned)(py + dh) < (unsigned)a.H && (unsigned)(px + dw) < (unsigned)a.W;
      return v ? (unsigned)((p + dh * a.W + dw) * 4) : OOB;
    };
    float rbv[8];
    auto loadB = [&](int ks) {  // K-step ks (this thread's half of it), zeros past k_b
      if (ks >= k_b) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rbv[j] = 0.f;
        return;
      }
      const unsigned vrow = vrow_of(ks);
      const int c0 = (ks - (ks / a.ncb) * a.ncb) * kCB + 8 * bh;
      if (full_cb) {
        const unsigned vb = vrow + (unsigned)c0 * chan_bytes;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rbv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vb, (int)(j * chan_bytes), 0));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned cofs = c0 + j < a.cimg ? (unsigned)(c0 + j) * chan_bytes : OOB;
          rbv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, vrow + cofs, 0, 0));
        }
      }
    };
    auto storeB = [&](int buf) {
      Split3 sp;
#pragma unroll
      for (int j = 0; j < 8; ++j) split3_set(sp, j, rbv[j]);
      bf16x8* Bs = smem + buf * STAGE + bkk * KV;
      Bs[bh * 128 + bn] = sp.hi;
      Bs[(2 + bh) * 128 + bn] = sp.mid;
      Bs[(4 + bh) * 128 + bn] = sp.lo;
    };
    const unsigned a_voff = (unsigned)((((g >> 1) * 6 + (g & 1)) * a.lda + m0 + wr * 32 + l16) * 16);
    u32x4 A0[TI][3], A1[TI][3];
    auto loadA = [&](u32x4 (&A)[TI][3], int ks) {  // the stage starting at K-step ks
      const bool two = ks + 1 < k_b;
#pragma unroll
      for (int ii = 0; ii < TI; ++ii)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          A[ii][q] = __builtin_amdgcn_raw_buffer_load_b128(
              rx, (two || g < 2) ? a_voff + ii * 256 : OOB, (int)((unsigned)(ks * 6 + 2 * q) * a_plane_bytes), 0);
    };
    auto compute = [&](const bf16x8* Bs, const u32x4 (&A)[TI][3]) {
      Split3 bv[TJ];
#pragma unroll
      for (int jj = 0; jj < TJ; ++jj) {
        const bf16x8* src = Bs + (g >> 1) * KV + (g & 1) * 128 + wc * 64 + jj * 16 + l16;
        bv[jj].hi = src[0];
        bv[jj].mid = src[256];
        bv[jj].lo = src[512];
      }
#pragma unroll
      for (int ii = 0; ii < TI; ++ii) {
        union { u32x4 u; bf16x8 h; } c0, c1, c2;
        c0.u = A[ii][0]; c1.u = A[ii][1]; c2.u = A[ii][2];
        Split3 av;
        av.hi = c0.h; av.mid = c1.h; av.lo = c2.h;
#pragma unroll
        for (int jj = 0; jj < TJ; ++jj) acc[ii][jj] = mfma16_x6(av, bv[jj], acc[ii][jj]);
      }
    };
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    loadB(k_a + bkk);
    loadA(A0, k_a);
    storeB(0);
    __syncthreads();
    const int nstg = (nst + 1) >> 1;
    for (int s = 0; s < nstg; ++s) {
      const int ks = k_a + 2 * s;
      const bool more = s + 1 < nstg;
      if (more) loadB(ks + 2 + bkk);
      const bf16x8* Bs = smem + (s & 1) * STAGE;
      if (s & 1) {
        if (more) loadA(A0, ks + 2);
        compute(Bs, A1);
      } else {
        if (more) loadA(A1, ks + 2);
        compute(Bs, A0);
      }
      if (more) storeB((s + 1) & 1);
      __syncthreads();
    }

    constexpr int PSZ = BM * BN;
    if (k_a > 0 || k_b < sk.KS) {
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)sk.part, (short)0, (int)min(0x7fffffffLL, (long long)sk.NW * 2 * PSZ * 4), 0x00020000);
      const unsigned pbase = (unsigned)((w * 2 + (k_a > 0 ? 0 : 1)) * PSZ * 4);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int nl = wc * 64 + j * 16 + l16;
          const int ml = wr * 32 + i * 16 + 4 * g;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rp,
                                                  pbase + (unsigned)(((ml + r) * BN + nl) * 4), 0, 0);
        }
      continue;
    }
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.C, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int n = n0 + wc * 64 + j * 16 + l16;
        const int mrow = m0 + wr * 32 + i * 16 + 4 * g;
        const unsigned voff = n < a.P ? (unsigned)((mrow * a.P + n) * 4) : OOB;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r];
          if (a.bias && mrow + r < a.M) {
            float bsum = a.bias[mrow + r];
            for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + mrow + r];
            v += bsum;
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc,
                                                mrow + r < a.M ? voff + r * a.P * 4 : OOB, 0, 0);
        }
      }
  }
}

}  // namespace msl

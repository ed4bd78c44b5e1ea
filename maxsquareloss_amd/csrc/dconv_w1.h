// The W1 form of the 3x3 forward-form GEMM (r06; included by dconv.hip after dconv_kernels.h).
#pragma once
#include "dconv_kernels.h"

namespace msl {

// W1 (r06): the f16x3 / fp16 3x3 forward and data-gradient GEMM at ONE wave per SIMD with twice the
// matrix work per wave and K-step.  The BD form (fwd_sk_body) runs 128 x 32 pixels per wave, 12 MFMAs per
// wave-K-step, two waves per SIMD; its counters (profiles/r05_fwd_sq_late.txt) put MFMA busy at 0.37 with
// half of the wave time waiting to issue.  Here:
//   - a workgroup of 4 waves owns 128 rows x 256 pixels; each wave 128 rows x 64 pixels (TM = 4, TN = 2),
//     24 MFMAs per K-step (f16x3), one wave per SIMD, 256 workgroups (one per CU);
//   - EVERY operand moves by LDS-DMA: the A pieces (shared by the 4 waves) and each wave's own image
//     operand, read from the pre-split fp16 planes (k_split_img: 16 B = 8 channels of one plane per lane
//     and column, so a wave's 1-KB piece lands exactly as its MFMA B fragments, lane by lane).  With only
//     DMA in the loop the vmcnt count is exact (an LDS-DMA may land after register loads issued behind it,
//     r04), so STAGES - 2 K-steps stay in flight across each wait instead of one: a first W1 build with
//     the image loaded to registers (BD) waited on them every K-step and ran layer3 at 99.5 vs 78 us;
//   - the fragments of K-step i + 1 (A and B) are read from LDS during K-step i's MFMAs (two register sets);
//   - stream-K over 256 workers, pieces of 128 x 256 summed by k_sk_reduce<128, 256>.
// Per K-step i: wait until K-step i + 1's pieces landed, barrier (every wave's pieces of i + 1 are in LDS,
// every wave has consumed the fragments of slot i - 1... i + 2 - STAGES), issue K-step i + STAGES - 1's
// pieces into the slot of i - 1, read K-step i + 1's fragments, run K-step i's MFMAs.  Every K-step issues
// the same pieces, also past the segment's end (zero-filled out of range or never read), so the wait count
// is the same on every path.
constexpr int kW1BM = 128, kW1BN = 256, kW1NW = 256, kW1Stages = 5;

template <int MT>
__global__ void __launch_bounds__(256, 1) k_igemm_fwd_w1(FwdArgs a, SkArgs sk) {
  constexpr int BM = kW1BM, BN = kW1BN, TM = 4, TN = 2, STAGES = kW1Stages;
  constexpr bool H1 = MT == kMathH1P;
  static_assert(MT == kMathH3P || H1, "W1: the f16x3 / fp16 forms");
  constexpr int NQ = 4;                          // (plane, k half) blocks of one K-step in the pack
  constexpr int NQL = H1 ? 2 : 4;                // of them staged (fp16: the hi plane's two halves)
  constexpr int NPB = H1 ? 1 : 2;                // image planes
  constexpr int A_FL = NQL * BM * 4;             // floats of a slot's A part: NQL blocks of BM 16-B rows
  constexpr int B_FL = 4 * NPB * TN * 256;       // floats of its B part: a 1-KB piece per (wave, plane, column)
  constexpr int SLOT = A_FL + B_FL;
  constexpr int A_INST_W = NQL * (BM / 64) / 4;  // A pieces per wave and K-step
  constexpr int B_INST_W = NPB * TN;             // B pieces per wave and K-step
  constexpr int INST_W = A_INST_W + B_INST_W;
  static_assert(A_INST_W >= 1 && (STAGES - 2) * INST_W < 64, "pieces per wave, vmcnt range");
  static_assert(STAGES * SLOT * 4 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) float smem[STAGES * SLOT];  // the only LDS object

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid * (TN * 32);
  // XCD-aware worker id, data-parallel tiles first, then the stream-K range (as fwd_sk_body)
  const int nb = gridDim.x, b = blockIdx.x;
  const int w = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);
  int dp_t = w, it = 0, it_end = 0;
  const int sw = (sk.tdp > 0 && sk.NW < nb) ? b : w;
  if (sw < sk.NW) {
    it = sk.tdp * sk.KS + sk_start(sw, sk.T, sk.NW);
    it_end = sk.tdp * sk.KS + sk_start(sw + 1, sk.T, sk.NW);
  }
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Ax6, (short)0, (int)min(0x7fffffffLL, (long long)a.ksteps * NQ * a.lda * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rbx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Bx6, (short)0, (int)min(0x7fffffffLL, (long long)a.ncb * NPB * 2 * a.P * 16), 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  const unsigned plane_bytes = (unsigned)a.P * 16u;
  float iB;
  pow2_scale(partials_max(a.bpart, a.bnpart, lane), iB);  // (the planes were scaled by k_split_img)
  const float iA = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(a.ascale[1])));

  typedef typename std::conditional<H1, f16x8, Split2h>::type Frag;
  f32x16 acc[TM][TN];
  while (true) {
    int t, k_a, k_b;
    if (dp_t < sk.tdp) {
      t = dp_t;
      k_a = 0;
      k_b = sk.KS;
      dp_t += nb;
    } else if (it < it_end) {
      t = (unsigned)it / (unsigned)sk.KS;
      k_a = it - t * sk.KS;
      k_b = min(sk.KS, k_a + (it_end - it));
      it += k_b - k_a;
    } else {
      break;
    }
    const int nst = k_b - k_a;
    int tm, tn;
    sk_tile(t, sk.tiles_m, sk.tiles_n, sk.gm, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    // this lane's two pixel columns (n0 + wn + 32 j + l32) and their image coordinates
    int pc[TN], pcx[TN], pcy[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      pc[j] = n0 + wn + j * 32 + l32;
      const int q = pc[j] / a.W;
      pcx[j] = pc[j] - q * a.W;
      pcy[j] = q % a.H;
    }
    // issue cursor (wave-uniform, tap-major K: ks = (branch * taps + tap) * ncb + cb)
    int c_cb, c_tap;
    {
      const int ks0 = __builtin_amdgcn_readfirstlane(k_a);
      c_tap = ks0 / a.ncb;
      c_cb = ks0 - c_tap * a.ncb;
    }
    unsigned vb[TN];  // per column: the lane's shifted pixel in its k half's plane rows, OOB outside the image
    auto set_tap = [&](int tq) {
      const int br = tq / a.taps;
      const int tp = tq - br * a.taps;
      const int d = br ? a.dil1 : a.dil0;
      const int dh = (tp / 3 - 1) * d, dw = (tp % 3 - 1) * d;
      const int shift = dh * a.W + dw;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bool v = pc[j] < a.P && (unsigned)(pcy[j] + dh) < (unsigned)a.H && (unsigned)(pcx[j] + dw) < (unsigned)a.W;
        vb[j] = v ? (unsigned)(pc[j] + shift) * 16u + (unsigned)hh * plane_bytes : OOB;
      }
    };
    set_tap(c_tap);
    // K-step s's pieces into slot `slot`: the A pieces (64 rows of one (plane, k half) block each), then this
    // wave's image pieces (plane q, column j: its lanes' 16 B at the cursor's channel block); advances the cursor
    auto issue = [&](int s, int slot) {
      float* As = smem + slot * SLOT;
#pragma unroll
      for (int i = 0; i < A_INST_W; ++i) {
        const int inst = wid * A_INST_W + i;
        const int qh = inst / (BM / 64), mb = (inst % (BM / 64)) * 64;
        dma_b128(rx, As + inst * 256, (unsigned)(((s * NQ + qh) * a.lda + m0 + mb + lane) * 16));
      }
      float* Bw = As + A_FL + wid * (B_INST_W * 256);
#pragma unroll
      for (int q = 0; q < NPB; ++q) {
        const int so = __builtin_amdgcn_readfirstlane((c_cb * NPB + q) * 2) * (int)plane_bytes;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rbx, (lds_void*)(Bw + (q * TN + j) * 256), 16, vb[j], so, 0, 0);
      }
      if (++c_cb == a.ncb) {
        c_cb = 0;
        if (++c_tap * a.ncb < a.ksteps) set_tap(c_tap);  // (past the last K-step: nothing to set)
      }
    };
    // K-step fragments from a slot: A rows i * 32 + l32 of the lane's k half; B: the lane's own 16 B per piece
    auto read = [&](const float* Sl, Frag (&av)[TM], Frag (&bv)[TN]) {
      const f16x8* Ab = reinterpret_cast<const f16x8*>(Sl);
      const f16x8* Bb = reinterpret_cast<const f16x8*>(Sl + A_FL + wid * (B_INST_W * 256));
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (H1) {
          bv[j] = Bb[j * 64 + lane];
        } else {
          bv[j].hi = Bb[(0 * TN + j) * 64 + lane];
          bv[j].lo = Bb[(1 * TN + j) * 64 + lane];
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (H1) {
          av[i] = Ab[hh * BM + i * 32 + l32];
        } else {
          av[i].hi = Ab[hh * BM + i * 32 + l32];
          av[i].lo = Ab[(2 + hh) * BM + i * 32 + l32];
        }
      }
    };
    auto compute = [&](const Frag (&av)[TM], const Frag (&bv)[TN]) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (H1) {
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i], bv[j], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].lo, bv[j].hi, acc[i][j], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bv[j].lo, acc[i][j], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i].hi, bv[j].hi, acc[i][j], 0, 0, 0);
        }
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    Frag av0[TM], bv0[TN], av1[TM], bv1[TN];
    __builtin_amdgcn_s_barrier();  // the previous segment's LDS reads are complete in every wave
#pragma unroll
    for (int k = 0; k < STAGES - 1; ++k) issue(k_a + k, k);
    wait_vmcnt<(STAGES - 2) * INST_W>();  // K-step k_a landed (only k_a + 1 .. + STAGES - 2 younger)
    __builtin_amdgcn_s_barrier();
    read(lds_after_barrier(smem), av0, bv0);
    auto step = [&](int i, const Frag (&avc)[TM], const Frag (&bvc)[TN], Frag (&avn)[TM], Frag (&bvn)[TN]) {
      wait_vmcnt<(STAGES - 3) * INST_W>();  // K-step i + 1 landed (only i + 2 .. i + STAGES - 2 younger)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);  // one scheduling region per K-step: nothing drifts across the barrier
      issue(k_a + i + STAGES - 1, (i + STAGES - 1) % STAGES);  // the slot of i - 1: consumed at i - 1 by all
      read(lds_after_barrier(smem) + ((i + 1) % STAGES) * SLOT, avn, bvn);
      compute(avc, bvc);
      // the interleave: each DMA piece (~60 issue cycles) and pair of fragment reads between MFMAs, so the
      // matrix pipe is never left idle behind a run of them (left alone, the compiler issues the six pieces
      // back to back after the barrier and sinks the reads behind the MFMAs)
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
#pragma unroll
      for (int g = 0; g < INST_W; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (the LDS-DMA piece)
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      // this K-step's fragment reads complete before the next barrier (the BD form's rule: the compiler lets
      // MFMAs, and with them its own waits for the reads, drift across a raw barrier, and past a barrier any
      // wave may refill a slot that the barrier released)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    int i = 0;
    for (; i + 2 <= nst; i += 2) {
      step(i, av0, bv0, av1, bv1);
      step(i + 1, av1, bv1, av0, bv0);
    }
    if (i < nst) step(i, av0, bv0, av1, bv1);
    wait_vmcnt<0>();  // the stages issued past the end land before the slots are reused

#pragma unroll
    for (int ii = 0; ii < TM; ++ii)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[ii][j][r] = acc[ii][j][r] * iA * iB;  // exact: powers of two
    constexpr int PSZ = BM * BN;
    if (k_a > 0 || k_b < sk.KS) {
      // a piece of a split tile (slot 0: starts inside the tile, slot 1: the tile's head), row-major
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)sk.part, (short)0, (int)min(0x7fffffffLL, (long long)sk.NW * 2 * PSZ * 4), 0x00020000);
      const unsigned pbase = (unsigned)((sw * 2 + (k_a > 0 ? 0 : 1)) * PSZ * 4);
#pragma unroll
      for (int ii = 0; ii < TM; ++ii)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nl = wn + j * 32 + l32;
          const int ml = ii * 32 + 4 * hh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ro = (r & 3) + 8 * (r >> 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[ii][j][r]), rp,
                                                  pbase + (unsigned)(((ml + ro) * BN + nl) * 4), 0, 0);
          }
        }
      continue;
    }
    // sole worker of the tile: the output (+ the summed branch biases); columns past P / rows past M OOB
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.C, (short)0, (int)min(0x7fffffffLL, (long long)a.M * a.P * 4), 0x00020000);
#pragma unroll
    for (int ii = 0; ii < TM; ++ii)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + j * 32 + l32;
        const int mrow = m0 + ii * 32 + 4 * hh;
        const unsigned voff = n < a.P ? (unsigned)((mrow * a.P + n) * 4) : OOB;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          float v = acc[ii][j][r];
          if (a.bias && mrow + ro < a.M) {
            float bsum = a.bias[mrow + ro];
            for (int b2 = 1; b2 < a.nbias; ++b2) bsum += a.bias[b2 * a.M + mrow + ro];
            v += bsum;
          }
          const unsigned off = mrow + ro < a.M ? voff + ro * a.P * 4 : OOB;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, off, 0, 0);
        }
      }
  }
}

}  // namespace msl

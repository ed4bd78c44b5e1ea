// Diagnostic build (r05): the layer3-shaped f16x3 BD forward (k_igemm_fwd_sk2) with in-kernel s_memtime
// stamps (fwd_sk_body PROF) - where a K-step of the loop spends its cycles.  Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 scripts/probe_sk.hip maxsquareloss_amd/csrc/bn.hip \
//         -o scripts/probe_sk.so
// driven by scripts/probe_sk.py.  The launch restates launch_fwd_form's BD f16x3 path (dconv.hip).
#include "../maxsquareloss_amd/csrc/dconv.hip"

extern "C" int probe_bd_fwd(const float* x, const float* packed, float* y, int cin, int cout, int h, int w, int nimg,
                            int dil, const float* x_part, int x_npart, void* ws, size_t ws_bytes,
                            unsigned long long* prof, int with_prof, msl_stream_t stream) {
  hipStream_t st = as_stream(stream);
  const int P = nimg * h * w;
  FwdPlan pl = plan_fwd(1, 9, cin, cout, P, false);
  if (!pl.sk || pl.bm != 128 || cin % kCB) return MSL_ERR_SHAPE;
  pl.G = 1;
  pl.bk = kCB;
  pl.kps = pl.ksteps;
  FwdArgs a{};
  a.A = packed;
  a.B = x;
  a.C = y;
  a.M = cout;
  a.lda = pad_to(cout, kPackPad);
  a.H = h;
  a.W = w;
  a.P = P;
  a.cimg = cin;
  a.ncb = cdiv(cin, kCB);
  a.dil0 = dil;
  a.ksteps = pl.ksteps;
  a.kps = pl.kps;
  a.taps = 9;
  a.slab = (long long)cout * P;
  const long long f32 = (long long)pl.ksteps * kCB * a.lda;
  a.Ax6 = reinterpret_cast<const __bf16*>(packed + f32);
  a.bpart = x_part;
  a.bnpart = x_npart;
  a.ascale = packed + pack_tail_offset(f32) + kNPart;
  SkArgs sk{};
  sk.part = (float*)ws;
  sk.tiles_m = pl.tiles_m;
  sk.tiles_n = pl.tiles_n;
  sk.KS = pl.kps;
  const long long tiles = (long long)pl.tiles_m * pl.tiles_n;
  const int nwk = kSkNW;
  if (ws_bytes < (size_t)nwk * 2 * 128 * kSkBN * 4) return MSL_ERR_WORKSPACE;
  sk.tdp = tiles >= nwk ? (int)(tiles / nwk * nwk) : 0;
  sk.gm = sk.tdp > 0 ? pl.tiles_m : 1;
  const long long T = (tiles - sk.tdp) * sk.KS;
  sk.NW = (int)std::min<long long>(nwk, T);
  if (sk.tdp > 0) sk.NW = (int)std::max<long long>(1, std::min<long long>(sk.NW, T / 8));
  sk.T = (int)T;
  sk.prof = prof;
  const dim3 grid(sk.tdp > 0 ? nwk : sk.NW), block(256);
  // with_prof: 1 stamps; 2, 4, 8, 6, 14 timing-only ablations, 16 a BN-apply of the image operand
  // (dconv_kernels.h fwd_sk_body PROF)
#define PROBE_CASE(V)                                                                                              \
  case V:                                                                                                          \
    hipLaunchKernelGGL((k_igemm_fwd_sk2<128, kSkBN, 1, 4, 1, 4, false, kMathH3P, false, true, false, V>), grid,     \
                       block, 0, st, a, sk);                                                                       \
    break;
  switch (with_prof) {
    PROBE_CASE(0)
    PROBE_CASE(1)
    PROBE_CASE(2)
    PROBE_CASE(4)
    PROBE_CASE(6)
    PROBE_CASE(8)
    PROBE_CASE(14)
    PROBE_CASE(16)

    default: return MSL_ERR_ARG;
  }
  MSL_CHECK_LAUNCH();
  if (T > 0)
    hipLaunchKernelGGL((k_sk_reduce<128, kSkBN>), dim3(128 * kSkBN / 1024, (unsigned)(tiles - sk.tdp)), block, 0, st,
                       a, sk);
  MSL_CHECK_LAUNCH();
  return MSL_OK;
}

extern "C" int probe_workers(int cin, int cout, int h, int w, int nimg) {
  const int P = nimg * h * w;
  FwdPlan pl = plan_fwd(1, 9, cin, cout, P, false);
  const long long tiles = (long long)pl.tiles_m * pl.tiles_n;
  return tiles >= kSkNW ? kSkNW : (int)std::min<long long>(kSkNW, tiles * pl.ksteps);
}

// MFMA implicit-GEMM kernel family for gfx950 (v2): plain / batched GEMM in any
// operand orientation, and convolution forward, data-gradient and
// weight-gradient, bf16 inputs with fp32 accumulation on
// v_mfma_f32_16x16x32_bf16.
//
// Replaces the reference's per-sample im2col + sgemm convolution
// (ConvolutionLayer, src/worker/layer.cc:63-123: unpack_patch2col F3,
// pack_col2patch F4, gW += dot(grad, col.T()) F5) and the DotEngine GEMMs
// (include/mshadow/tensor_expr_engine-inl.hpp:339-383): no column buffer is
// materialised; operand loaders gather im2col tiles from NHWC tensors.
//
//   C[m][n] (=|+=) alpha * sum_k A(m, k) * B(n, k)  (+ bias[n]) (ReLU)
//
// Structure: BM x BN x 64 tiles (BM, BN in {64, 128}), 256 threads = 2x2
// waves, each wave (BM/2)x(BN/2) of 16x16x32 MFMA tiles.  Operands are staged
// global -> registers -> double-buffered LDS, one barrier per K-tile, with the
// next tile's global loads issued before the current tile's MFMAs (T14).
// Kernel arguments are never written (a v1 that patched its by-value argument
// struct had it spilled to scratch and every operand load degraded to flat_*).
// Loads are branch-free: out-of-range / padding vectors read a clamped, valid
// address and are zeroed with a select.  LDS images:
//   KMAJOR  [rows][64 k]: 128-B rows, fragment = ds_read_b128, chunk XOR
//           (row>>1)&7 (conflict-free for the b128 lane groups);
//   KOUTER  [64 k][rows]: fragment = 2 x ds_read_b64_tr_b16 (hardware
//           transpose), chunk XOR chosen per row width (T10).
// Convolution specifics:
//   * K is ordered (tap, channel) with channel fastest; when the per-tap
//     channel count is a multiple of 64 the tap of a K-tile is wave-uniform
//     (scalar math only), otherwise each lane splits its own index.
//   * dgrad with stride > 1 is split into stride_h*stride_w phases
//     (blockIdx.z): each phase is a dense problem over the output pixels of
//     that phase and only the taps that reach them -- no masked work; phases
//     with no taps write zeros.
//   * dgrad reads the weights [K][R][S][C] directly as a K-outer operand (the
//     (k, c) slice of one tap is row-major): no transposed copy.
//   * wgrad splits the pixel reduction across workgroups (blockIdx.z) and
//     accumulates fp32 partial tiles atomically into the [K][R][S][C]
//     gradient (the layout of the flat gradient buffer).
#include <stdio.h>
#include <stdlib.h>

#include <stdexcept>
#include <type_traits>

#include "igemm_kern.h"

namespace sg {

// wdot[c] += sign * sum_rows W[row][c] * dW[row][c] over a [rows][C] weight
// (rows = K*R*S of a KRSC filter): the <W, dW> input-channel sums of the
// identity-sum BN backward (batchnorm.hip, bn_bwd_finalize_wdot_k).  Block =
// 64 channels x 4 row lanes, WDOT_RB rows per block, one atomic per channel.
constexpr int WDOT_RB = 64;
__global__ void __launch_bounds__(256) wdot_colsum_k(const bf16* __restrict__ w, const float* __restrict__ dw,
                                                     int rows, int C, float sign, float* __restrict__ wdot,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float tau, int* __restrict__ flag) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (gamma != nullptr && blockIdx.y == 0 && lane == 0 && c < C) {
    // the producer BN's gate (bn_bwd_finalize_wdot_k): the recovered xhat
    // carries y's bf16 rounding times |xhat| + |beta / gamma|
    const float g = fabsf(gamma[c]);
    if (!(g >= tau && fabsf(beta[c]) <= 4.f * g)) *flag = 1;  // (NaN raises it too)
  }
  const int r0 = blockIdx.y * WDOT_RB;
  float a = 0.f;
  if (c < C) {
    const int r1 = min(rows, r0 + WDOT_RB);
    for (int r = r0 + lane; r < r1; r += 4) a += (float)w[(int64_t)r * C + c] * dw[(int64_t)r * C + c];
  }
  red[lane][cl] = a;
  __syncthreads();
  if (lane == 0 && c < C) atomicAdd(wdot + c, sign * (red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]));
}

// WT[t][c][k] = W[k][t][c] (bf16): per-tap [K][C] -> [C][K] through a 64x64
// LDS tile (+1 column pad against bank conflicts), 256 threads.
__global__ void __launch_bounds__(256) wt_transpose_k(const bf16* __restrict__ w, bf16* __restrict__ wt, int K,
                                                      int T, int C) {
  __shared__ bf16 tile[64][65];
  const int c0 = blockIdx.x * 64, k0 = blockIdx.y * 64, t = blockIdx.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int k = k0 + r, c = c0 + tx;
    tile[r][tx] = (k < K && c < C) ? w[((int64_t)k * T + t) * C + c] : (bf16)0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, k = k0 + tx;
    if (c < C && k < K) wt[((int64_t)t * C + c) * K + k] = tile[tx][r];
  }
}

// Every conv weight of a backward pass transposed in ONE launch (instead of
// one small launch in front of each dgrad).  desc[i] = {src, dst, K, T, C,
// first tile}; workgroup b takes tile b of the descriptor whose range holds
// it (tiles of a weight ordered like wt_transpose_k's grid: c-block fastest).
struct WtDesc {
  const bf16* src;
  bf16* dst;
  int K, T, C, tile0;
};
__global__ void __launch_bounds__(256) wt_transpose_batched_k(const WtDesc* __restrict__ desc, int n) {
  __shared__ bf16 tile[64][65];
  int d = 0;
  while (d + 1 < n && desc[d + 1].tile0 <= (int)blockIdx.x) ++d;  // n is small (one entry per conv)
  const WtDesc w = desc[d];
  const int lt = blockIdx.x - w.tile0;
  const int cb = (w.C + 63) / 64, kbn = (w.K + 63) / 64;
  const int c0 = (lt % cb) * 64, k0 = ((lt / cb) % kbn) * 64, t = lt / (cb * kbn);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int k = k0 + r, c = c0 + tx;
    tile[r][tx] = (k < w.K && c < w.C) ? w.src[((int64_t)k * w.T + t) * w.C + c] : (bf16)0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, k = k0 + tx;
    if (c < w.C && k < w.K) w.dst[((int64_t)t * w.C + c) * w.K + k] = tile[tx][r];
  }
}

}  // namespace sg

using namespace sg;

static void init_phase_identity(ConvGeom& g) {
  for (int i = 0; i < 16; ++i) {
    g.phs[i].dns = FastDiv(1);
    g.phs[i].dWp = FastDiv(1);
    g.phs[i].dHpWp = FastDiv(1);
  }
}

static ConvGeom make_geom(int N, int H, int W, int C, int K, int R, int S, int Ho, int Wo, int sh, int sw, int ph,
                          int pw, int dh, int dw) {
  ConvGeom g{};
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S; g.Ho = Ho; g.Wo = Wo;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dw;
  g.dC = FastDiv(C); g.dS = FastDiv(S); g.dK = FastDiv(K); g.dWo = FastDiv(Wo); g.dHoWo = FastDiv(Ho * Wo);
  g.bq_n = BK / (Ho * Wo);
  g.bq_h = (BK % (Ho * Wo)) / Wo;
  g.bq_w = BK % Wo;
  init_phase_identity(g);
  return g;
}

// dgrad phases (dilation 1).  Returns the number of phases (sh*sw <= 16).
static int make_phases(ConvGeom& g) {
  int np = 0;
  for (int a = 0; a < g.sh; ++a)
    for (int b = 0; b < g.sw; ++b) {
      Phase& P = g.phs[np++];
      P.a = a; P.b = b;
      P.r0 = (a + g.ph) % g.sh;
      P.s0 = (b + g.pw) % g.sw;
      P.nr = P.r0 < g.R ? (g.R - P.r0 + g.sh - 1) / g.sh : 0;
      P.ns = P.s0 < g.S ? (g.S - P.s0 + g.sw - 1) / g.sw : 0;
      P.offh = (a + g.ph - P.r0) / g.sh;
      P.offw = (b + g.pw - P.s0) / g.sw;
      P.Hp = a < g.H ? (g.H - a + g.sh - 1) / g.sh : 0;
      P.Wp = b < g.W ? (g.W - b + g.sw - 1) / g.sw : 0;
      P.dns = FastDiv(P.ns > 0 ? P.ns : 1);
      P.dWp = FastDiv(P.Wp > 0 ? P.Wp : 1);
      P.dHpWp = FastDiv(P.Hp * P.Wp > 0 ? P.Hp * P.Wp : 1);
    }
  return np;
}

// Tuning knobs (sg_set_tuning): 0 = wgrad tile/split policy, 1 = LDS-staged
// bf16 epilogue, 2 = K-slice-major XCD mapping of split-K launches, 3 = wgrad
// split-count scale (2^v), 4 = forced tile shape (5/6/7: the 8-wave variants
// of pick_big at any size), 5 = 8-wave tiles for non-split launches (pick_big),
// 6 = single-stage short-K variant for GEMMs of at most this many K-tiles
// (round 3: 8 measured +0.3..0.6 % over 4 and 2, profiles/r3/ab_short_k_threshold.jsonl; round 5, after the
// persistent and algebraic paths took the K <= 128 tails: 2 is +0.38 % over 8 and 0 +0.2 %, the stage-3/4
// K = 256 / 512 forwards and gsum data gradients run faster on the 8-wave two-workgroup tile,
// profiles/r5/ab_short_k_cap_r6w.jsonl)
// (0 = off), 7 = early DMA issue in the 2-stage loop (measured -3.5 % conv time)
// 8 = non-temporal output stores in the LDS-staged bf16 epilogue, 9 = persistent
// short-K kernel for the 1x1-conv GEMM shapes (sk_gemm_k)
// key 10: workgroup target of the 8-wave split-K weight gradient (0: 1024 with taps, 512 for 1x1)
// key 11: 1 = strided data gradients never take the single-stage short-K kernel (A/B)
// key 12: > 0 forces the split count of the 8-wave weight gradient (sweeps);
// key 13: split policy of that kernel: 1 = quantisation-aware (default), 0 = powers of 2 to the target
// key 14: the 4-wave three-stage ring for the plain (K-major / K-outer) GEMMs of the generic tile path:
//         0 = auto (under-filled launches of 8-64 K-tiles), 3 = always, -1 = never
// key 15: 1 = the 8-wave weight gradient on 256 x 128 tiles (64 x 64 wave tiles, three-stage ring) when K >= 256
//         (ResNet-50 b1024 step +0.33 %, three alternating pairs on one box: profiles/r5/ab_wgrad_256x128.jsonl)
// key 16: 256 x 128 three-stage tiles in place of the 8-wave 128 x 128 ones (1 conv fwd, 2 + dgrad, 3 all)
// key 17: 1 = 128 x 256 three-stage weight-gradient tiles for K_out < 256 (with key 15)
// key 18: 1 = the persistent streaming GEMM (st_gemm_k) for the 1x1-conv shapes with K >= 256
//         (plain bf16 output, optional BN statistics)
// key 19: 1 = __syncthreads (vmcnt(0) drain of the output stores) at the staged epilogue's barriers
//         after its global stores; 0 = LDS-only barriers (default)
extern "C" int sg_bn_deterministic();  // batchnorm.hip: deterministic-reduction mode
static int g_tune[20] = {5, 1, 1, 0, 0, 1, 2, 1, 0, 1, 0, 0, 0, 1, 0, 1, 0, 0, 1, 0};
// one-shot: the next dgrad's wt scratch is already transposed.  Per OS
// thread: the runtime's executor threads (hogwild / aggregated replicas)
// each set and consume their own flag, so one thread's set can never be
// taken by another thread's dgrad
static thread_local int g_wt_ready = 0;
// one-shot (per OS thread): the next dgrad adds this masked residual gradient
static thread_local const bf16* g_res_g = nullptr;
static thread_local int g_res_s = 1, g_res_Ho = 0, g_res_Wo = 0;  // (compact strided res_g, sg_conv_dgrad_gsum)
static thread_local const uint8_t* g_res_mask = nullptr;
// one-shot (per OS thread): the next dgrad with a mask-only BN producer writes
// its output masked (stats_mode 4, the algebraic residual-BN backward's g~)
static thread_local int g_mask_out = 0;

// SG_GEMM_LOG=1: one stderr line per GEMM launch (operand modes, shape,
// epilogue features) -- the per-shape breakdown behind a kernel profile
static int gemm_log() {
  static int on = [] {
    const char* e = getenv("SG_GEMM_LOG");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return on;
}

constexpr int stages_c(int BM, int BN, int STAGES) { return STAGES * (BM + BN) * BK * 2; }

template <int BM, int BN, int AM, int BMODE, int OUT, int NTH = NT, int WM = 2, int WN = 2, int STAGES = 2,
          int FLAGS = 0>
static void launch_t(const GemmArgs& p_in, int tiles, int ydim, int zdim, hipStream_t s) {
  GemmArgs p = p_in;
  p.lds_epilogue = g_tune[1];
  p.epi_fence = g_tune[19];
  p.early_issue = g_tune[7];
  p.nt_store = g_tune[8];
  p.xcd_split = (OUT == OUT_F32_ATOMIC && g_tune[2] && ydim == 1 && zdim >= 8 && (zdim & 7) == 0) ? 1 : 0;
  dim3 grid(tiles, ydim, zdim), block(NTH);
  constexpr int stages = STAGES * (BM + BN) * BK * 2;
  constexpr int rch = (STAGES == 1 || BM * (BN + 4) * 4 <= 152 * 1024) ? BM : BM / 4;  // epilogue row chunk
  constexpr int etile = STAGES == 1 ? (OUT == OUT_BF16 ? BM * (BN + 8) * 2 : BM * (BN + 4) * 4)  // bf16 staging
                        : OUT == OUT_BF16 ? rch * (BN + 4) * 4                                  // fp32 epilogue tile
                        : OUT == OUT_F32_ATOMIC ? BM * (BN + 4) * 4 : 0;
  constexpr int ered = (OUT == OUT_BF16) ? NTH * 16 * 4 : 0;  // BN-stats reduction scratch
  static_assert(STAGES != 1 || (OUT == OUT_BF16 && ered <= (etile > stages_c(BM, BN, STAGES) ? etile : stages_c(BM, BN, STAGES))),
                "single-stage variant: bf16 output only");
  constexpr int lds = stages > etile ? stages : etile;
  static_assert(lds <= 160 * 1024, "LDS budget");
  auto* kern = igemm_k<BM, BN, AM, BMODE, OUT, NTH, WM, WN, STAGES, FLAGS>;
  if (gemm_log())
    fprintf(stderr, "SG_GEMM_L igemm_k<%d,%d,%d,%d,%d,%d,%d,%d,%d,%d> grid %d %d %d\n", BM, BN, AM, BMODE, OUT, NTH, WM,
            WN, STAGES, FLAGS, tiles, ydim, zdim);
  if constexpr (lds > 65536) {
    static bool attr = [kern] {
      return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    }();
    (void)attr;
  }
  hipLaunchKernelGGL(kern, grid, block, lds, s, p);
}

template <int OUT, int FLAGS = 0>
static void launch_pp(const GemmArgs& p_in, int tiles, int ydim, hipStream_t s) {
  GemmArgs p = p_in;
  p.lds_epilogue = g_tune[1];
  p.epi_fence = g_tune[19];
  p.nt_store = g_tune[8];
  constexpr int lds = 2 * PP_BUF;
  auto* kern = pp_gemm_k<OUT, FLAGS>;
  if (gemm_log()) fprintf(stderr, "SG_GEMM_L pp_gemm_k<%d,%d> grid %d %d 1\n", OUT, FLAGS, tiles, ydim);
  static bool attr = [kern] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(tiles, ydim, 1), dim3(512), lds, s, p);
}

// persistent short-K launch: one workgroup per CU (the device's CU count),
// gridDim.x a multiple of 8 (the workgroups of every column slice that share
// an M-tile sit on one XCD); M-tiles from a dynamic queue per column slice
template <int KT, int EPI = 0, int AM = LM_KMAJOR>
static void launch_sk(const GemmArgs& p, int tiles_m, int tiles_n, hipStream_t s) {
  constexpr int lds = sk_lds(KT);
  auto* kern = sk_gemm_k<KT, EPI, AM>;
  static bool attr = [kern] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  (void)attr;
  const int cus = sg_cu_count();
  int g = (cus + tiles_n - 1) / tiles_n;
  g = (g + 7) / 8 * 8;
  if (g > tiles_m) g = tiles_m >= 8 ? tiles_m / 8 * 8 : 8;  // (a multiple of 8: the per-XCD tile partition)
  GemmArgs q = p;
  q.wq = 8 * tiles_n <= QMAX ? sg_workq_slot() : nullptr;
  if (gemm_log())
    fprintf(stderr, "SG_GEMM_L sk_gemm_k<%d,%d,%d> grid %d %d 1 M=%d N=%d K=%d\n", KT, EPI, AM, g, tiles_n, p.M, p.N,
            p.K);
  hipLaunchKernelGGL(kern, dim3(g, tiles_n, 1), dim3(256), lds, s, q);
}

// persistent streaming launch (st_gemm_k): one workgroup per CU as launch_sk,
// A and B both streamed through the K-tile ring
static void launch_st(const GemmArgs& p, int tiles_m, int tiles_n, hipStream_t s) {
  auto* kern = st_gemm_k<0>;
  static bool attr = [kern] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ST_LDS) == hipSuccess;
  }();
  (void)attr;
  const int cus = sg_cu_count();
  int g = (cus + tiles_n - 1) / tiles_n;
  g = (g + 7) / 8 * 8;
  if (g > tiles_m) g = tiles_m >= 8 ? tiles_m / 8 * 8 : 8;
  GemmArgs q = p;
  q.wq = 8 * tiles_n <= QMAX ? sg_workq_slot() : nullptr;
  if (gemm_log())
    fprintf(stderr, "SG_GEMM_L st_gemm_k<0> grid %d %d 1 M=%d N=%d K=%d\n", g, tiles_n, p.M, p.N, p.K);
  hipLaunchKernelGGL(kern, dim3(g, tiles_n, 1), dim3(256), ST_LDS, s, q);
}

// 8-wave (512-thread) tiles.  Returns 0 (the 4-wave v2 tiles) or
//   1: 128 x 128, waves 2 x 4 of 64 x 32, 2 stages, two workgroups per CU
//      (measured on ResNet-50 b1024: equal or up to 10 % faster than the
//      4-wave 128 x 128 tile when N >= 128);
//   2: 256 x 64, waves 4 x 2 of 64 x 32, 4-stage ring (the whole 160 KB),
//      one workgroup per CU;
//   3: 256 x 128, waves 4 x 2 of 64 x 64, 3-stage ring, one workgroup per CU.
// 2 and 3 keep two K-tiles in flight but lose to two independent workgroups
// per CU on every ResNet-50 conv (the waves of one workgroup reach each
// barrier together, nothing else covers the MFMA pipe): tests only.
//   4: the ping-pong 256 x 256 kernel (pp_gemm_k; plain K-major GEMMs).
//      (256 x 256 and 256 x 128 tiles in igemm_k's own early-issue loop
//      were measured slower than its 128 x 128 tile on every ResNet-50
//      1x1-conv GEMM shape and only 8-12 % faster at 8192^3:
//      profiles/r3/gemm_ceiling_256tiles.jsonl.)
static int pick_big(int M, int N) {
  if (g_tune[4] == 5) return 1;  // tests: force a variant at any size
  if (g_tune[4] == 6) return 2;
  if (g_tune[4] == 7) return 3;
  if (g_tune[4] == 8) return 4;
  if (!g_tune[5] || g_tune[4] != 0) return 0;
  auto wg = [&](int bm, int bn) { return (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (N >= 128 && !((N % 128) != 0 && (N % 128) <= 64) && wg(128, 128) >= 512) return 1;
  return 0;
}
static int big_bm(int big) { return big == 1 ? 128 : 256; }

// pick the tile: avoid wasting half a 128-tile on 64-wide problems; prefer
// 64-row tiles when 128-row ones leave the 256 CUs under-filled
static void pick_tile(int M, int N, int& BM, int& BN) {
  auto wg = [&](int bm, int bn) { return (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  BM = 128;
  BN = N <= 64 ? 64 : 128;
  if (BN == 128 && (N % 128) != 0 && (N % 128) <= 64) BN = 64;
  if (wg(BM, BN) < 256 && M > 64) BM = 64;
  if (wg(BM, BN) < 256 && BN == 128) BN = 64;
}

template <int AM, int BMODE, int OUT>
static void launch_tile(const GemmArgs& p, int M, int BM, int BN, int splits, hipStream_t s, int batch, int zdim) {
  const int tiles = ((M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int z = zdim > 0 ? zdim : splits;
  if (BM == 128 && BN == 128) launch_t<128, 128, AM, BMODE, OUT>(p, tiles, batch, z, s);
  else if (BM == 128 && BN == 64) launch_t<128, 64, AM, BMODE, OUT>(p, tiles, batch, z, s);
  else if (BM == 64 && BN == 128) launch_t<64, 128, AM, BMODE, OUT>(p, tiles, batch, z, s);
  else launch_t<64, 64, AM, BMODE, OUT>(p, tiles, batch, z, s);
}

// wgrad: the reduction (output pixels) is huge and M x N small, so
// parallelism comes from split-K; use the largest tile that fits (operand
// reuse -> arithmetic intensity) and only as many splits as fill the chip.
static void pick_wgrad(int M, int N, int K, int mode, int& BM, int& BN, int& splits) {
  const int nkt = (K + BK - 1) / BK;
  // measured (tools/tune_conv.py, b256): bigger tiles win when the pixel
  // reduction dwarfs the output (early, narrow layers); 64x64 + many splits
  // elsewhere
  if (mode == 4) mode = ((long)K >= 8L * M * N) ? 1 : 0;
  if (mode == 0) {
    pick_tile(M, N, BM, BN);
    const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    splits = 1;
    while (tiles * splits < 768 && splits * 2 <= nkt / 4) splits *= 2;
    return;
  }
  auto fit = [](int d) { return (d >= 128 && !((d % 128) != 0 && (d % 128) <= 64)) ? 128 : 64; };
  BM = fit(M);
  BN = fit(N);
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int target = mode == 1 ? 512 : mode == 2 ? 1024 : 768;
  const int min_kt = mode == 2 ? 4 : 8;
  splits = 1;
  while (tiles * splits < target && (splits * 2) * min_kt <= nkt) splits *= 2;
}

template <int AM, int BMODE, int OUT, int FLAGS = 0>
static void launch(const GemmArgs& p, int M, int splits, hipStream_t s, int batch, int zdim) {
  int BM, BN;
  if (gemm_log())
    fprintf(stderr, "SG_GEMM am=%d bm=%d out=%d flags=%d M=%d N=%d K=%d splits=%d batch=%d z=%d beta=%g stats=%d "
                    "smode=%d det=%d res=%d bias=%d relu=%d act=%d phase=%d R=%d S=%d C=%d sh=%d\n",
            AM, BMODE, OUT, FLAGS, M, p.N, p.K, splits, batch, zdim, p.beta, p.stats != nullptr, p.stats_mode,
            p.stats_det, p.res_g != nullptr, p.bias != nullptr, p.relu, p.act, p.out_phase, p.g.R, p.g.S, p.g.C,
            p.g.sh);
  if constexpr (OUT != OUT_F32_ATOMIC) {
    {
      const int z = zdim > 0 ? zdim : 1;
      // persistent short-K kernel (knob 9): 1x1-conv forward / data-gradient shapes
      if (FLAGS == 0 && OUT == OUT_BF16 && AM == LM_KMAJOR && BMODE == LM_KMAJOR && g_tune[9] && g_tune[4] == 0 &&
          !p.out_phase && zdim <= 1 && batch == 1 && p.K <= 128 && (p.N & 127) == 0 && !p.bias && !p.relu &&
          p.alpha == 1.f && p.stats_mode == 0 && !(p.stats && p.stats_det) && g_tune[1] && !p.res_g &&
          (p.ldc & 7) == 0 && (long)((M + 127) / 128) * (p.N / 128) >= 2048) {
        const int tiles_m = (M + 127) / 128;
        if (p.K <= 64) launch_sk<1>(p, tiles_m, p.N / 128, s);
        else launch_sk<2>(p, tiles_m, p.N / 128, s);
        return;
      }
      // persistent streaming kernel (knob 18; 1: where it measured faster --
      // K = 256, and K = 512 with one column slice -- 2: every K >= 256):
      // tools/bench_1x1.py, profiles/r6/bench_1x1_stream.jsonl: -11..-13 % on
      // 200704 x 1024 x 256, 802816 x 512 x 256, 3211264 x 128 x 256, -4 % on
      // 802816 x 128 x 512, +9..+19 % on the K >= 512 wide-N shapes
      if (FLAGS == 0 && OUT == OUT_BF16 && AM == LM_KMAJOR && BMODE == LM_KMAJOR && g_tune[18] && g_tune[4] == 0 &&
          (g_tune[18] >= 2 || p.K == 256 || (p.K == 512 && p.N == 128)) &&
          !p.out_phase && zdim <= 1 && batch == 1 && p.K >= 256 && (p.K & 63) == 0 && (p.N & 127) == 0 &&
          !p.bias && !p.relu && p.act == 0 && p.act_bwd == 0 && p.alpha == 1.f && p.beta == 0.f &&
          p.stats_mode == 0 && !(p.stats && p.stats_det) && !p.res_g && g_tune[1] && (p.ldc & 7) == 0 &&
          (p.lda & 7) == 0 && (p.ldb & 7) == 0 && (long)((M + 127) / 128) * (p.N / 128) >= 2048) {
        launch_st(p, (M + 127) / 128, p.N / 128, s);
        return;
      }
      // (a strided dgrad's phases each reduce over their own taps only: the
      // longest phase decides -- the stride-2 3x3 data gradients, 1-4 taps)
      int kmax = p.K;
      if (p.out_phase) {
        kmax = 0;
        for (int i = 0; i < z; ++i) kmax = max(kmax, p.g.phs[i].nr * p.g.phs[i].ns * p.g.K);
      }
      if (OUT == OUT_BF16 && g_tune[6] > 0 && g_tune[4] == 0 && p.beta == 0.f &&
          (kmax + BK - 1) / BK <= g_tune[6] && p.N >= 128 && !((p.N % 128) != 0 && (p.N % 128) <= 64) &&
          (long)((M + 127) / 128) * ((p.N + 127) / 128) >= 1024 && (g_tune[11] == 0 || !p.out_phase)) {
        const int tiles = ((M + 127) / 128) * ((p.N + 127) / 128);
        launch_t<128, 128, AM, BMODE, OUT_BF16, 256, 2, 2, 1, FLAGS>(p, tiles, batch, z, s);
        return;
      }
      int big = pick_big(M, p.N);
      // the ping-pong 256 x 256 kernel: plain K-major GEMMs (1x1 convs, dgrad
      // of 1x1 convs) with long K and enough 256 x 256 tiles for the chip
      // (measured: +8..28 % at K >= 2048, slower on short K --
      // profiles/r3/gemm_ceiling_pp.jsonl); never with deterministic BN
      // statistics (their row count assumes igemm_k's tile rows)
      const bool pp_ok = AM == LM_KMAJOR && BMODE == LM_KMAJOR && !p.out_phase && zdim <= 1 &&
                         !(p.stats && p.stats_det);
      if (big == 0 && g_tune[4] == 0 && g_tune[5] && pp_ok && p.K >= 2048 &&
          (long)((M + 255) / 256) * ((p.N + 255) / 256) >= 256)
        big = 4;
      if (big == 4) {
        if (pp_ok) {
          launch_pp<OUT, FLAGS>(p, ((M + 255) / 256) * ((p.N + 255) / 256), batch, s);
          return;
        }
        big = 1;
      }
      // knob 16 (A/B): the 256 x 128 three-stage tiles (64 x 64 wave tiles) for
      // 1: 3x3 / 7x7 conv forwards, 2: also data gradients, 3: every 8-wave GEMM
      if (big == 1 && g_tune[16] > 0 && !sg_bn_deterministic() && M >= 256 &&
          (g_tune[16] >= 3 || AM == LM_CONV_FWD || (g_tune[16] == 2 && AM == LM_DGRAD_A)))
        big = 3;
      if (big == 1) {
        const int tiles = ((M + 127) / 128) * ((p.N + 127) / 128);
        launch_t<128, 128, AM, BMODE, OUT, 512, 2, 4, 2, FLAGS>(p, tiles, batch, z, s);
        return;
      }
      if (big == 2) {
        const int tiles = ((M + 255) / 256) * ((p.N + 63) / 64);
        launch_t<256, 64, AM, BMODE, OUT, 512, 4, 2, 4, FLAGS>(p, tiles, batch, z, s);
        return;
      }
      if (big == 3) {
        const int tiles = ((M + 255) / 256) * ((p.N + 127) / 128);
        launch_t<256, 128, AM, BMODE, OUT, 512, 4, 2, 3, FLAGS>(p, tiles, batch, z, s);
        return;
      }
    }
  }
  pick_tile(M, p.N, BM, BN);
  if (g_tune[4] > 0 && g_tune[4] < 5) {  // tuning: force a tile shape (1: 128x64, 2: 64x128, 3: 64x64, 4: 128x128)
    BM = (g_tune[4] == 2 || g_tune[4] == 3) ? 64 : 128;
    BN = (g_tune[4] == 1 || g_tune[4] == 3) ? 64 : 128;
  }
  const int tiles = ((M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int z = zdim > 0 ? zdim : splits;
  // three-stage ring for plain GEMMs that leave the chip under-filled (at most
  // four workgroups per CU) with 8-64 K-tiles each: the Linear layers of a
  // BERT-sized batch, where each workgroup's K loop ran at the DMA latency.
  // Measured (profiles/r5/ab_bert_three_stage_ring.jsonl, bert_tiles_r6n.jsonl):
  // BERT-base 3 780 -> 3 905 seq/s, sonnx-BERT 3 608 -> 3 714; ResNet-50 and
  // AlexNet within noise when forced everywhere.  Knob 14: 0 auto, 3 always, -1 never.
  if constexpr ((AM == LM_KMAJOR || AM == LM_KOUTER) && (BMODE == LM_KMAJOR || BMODE == LM_KOUTER) && FLAGS == 0) {
    const long wgs = (long)tiles * (batch > 0 ? batch : 1) * (z > 0 ? z : 1);
    const int nkt = ((z > 1 ? p.k_per_split : p.K) + BK - 1) / BK;
    const bool ring = g_tune[14] == 3 || (g_tune[14] == 0 && wgs <= 4L * sg_cu_count() && nkt >= 8 && nkt <= 64);
    if (ring && !p.out_phase) {
      if (BM == 128 && BN == 128) launch_t<128, 128, AM, BMODE, OUT, NT, 2, 2, 3>(p, tiles, batch, z, s);
      else if (BM == 128 && BN == 64) launch_t<128, 64, AM, BMODE, OUT, NT, 2, 2, 3>(p, tiles, batch, z, s);
      else if (BM == 64 && BN == 128) launch_t<64, 128, AM, BMODE, OUT, NT, 2, 2, 3>(p, tiles, batch, z, s);
      else launch_t<64, 64, AM, BMODE, OUT, NT, 2, 2, 3>(p, tiles, batch, z, s);
      return;
    }
  }
  if (BM == 128 && BN == 128) launch_t<128, 128, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
  else if (BM == 128 && BN == 64) launch_t<128, 64, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
  else if (BM == 64 && BN == 128) launch_t<64, 128, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
  else launch_t<64, 64, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
}

// split-K of a plain fp32-atomic GEMM (a Linear's weight gradient): double
// the splits only while the grid stays within two workgroups per CU and each
// split keeps >= 32 K-tiles -- every split adds a full atomic pass over the
// output.  Measured on BERT-base's four weight gradients (K = 4096 tokens,
// tools/bert_gemm_sweep.py, profiles/r5/bert_gemm_sweep*.jsonl): the old
// target of 768 workgroups (4 splits) ran 10-25 % slower than this rule.
static int pick_splits(int M, int N, int K, int want) {
  if (want > 0) return want;
  int BM, BN;
  pick_tile(M, N, BM, BN);
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = 1;
  const int nkt = (K + BK - 1) / BK;
  const int cap = 2 * sg_cu_count();
  while (tiles * splits * 2 <= cap && nkt / (splits * 2) >= 32) splits *= 2;
  if (tiles < cap / 8)  // (a tiny output: split-K is the only parallelism left)
    while (tiles * splits < cap && nkt / (splits * 2) >= 4) splits *= 2;
  return splits;
}

static inline int kps(int K, int splits) {
  const int nkt = (K + BK - 1) / BK;
  return ((nkt + splits - 1) / splits) * BK;
}

static unsigned extent_bytes(int64_t elems) {
  if (elems * 2 >= (int64_t)1 << 31)
    throw std::runtime_error("igemm: operand exceeds 2 GiB (32-bit buffer offsets); split the batch");
  return (unsigned)(elems * 2);
}

extern "C" {

int sg_bn_deterministic();  // batchnorm.hip: deterministic-reduction mode
int sg_ws_prezeroed();      // batchnorm.hip: one-shot 'workspace pre-zeroed' flag (per-step arena)
// conv3x3.hip: persistent 3x3/s1/p1 64->64-channel, 56-wide convolution
int sg_conv3x3_ok(int N, int H, int W, int C, int K);
int sg_conv3x3_64(const void* x, const void* w, int wmode, void* y, void* stats, const void* mask, int N, int H,
                  int W, int C, int K, hipStream_t s);

// Plain GEMM: C[M][N] = alpha * sum_k A(m,k) B(n,k) (+ beta*C) ... with
//   a_kouter = 0: A stored [M][K] (lda), 1: A stored [K][M]
//   b_kouter = 0: B stored [N][K] (ldb), 1: B stored [K][N]
// out_mode 0 bf16, 1 f32, 2 f32 atomic (split-K, C pre-initialised).
void sg_gemm_heads(const void* a, int64_t lda, int a_kouter, const void* b, int64_t ldb, int b_kouter, void* c,
                   int64_t ldc, int M, int N, int K, float alpha, float beta, const void* bias, int relu,
                   int out_mode, int splits, int batch, int64_t sa, int64_t sb, int64_t sc, int bh, int64_t sa2,
                   int64_t sb2, int64_t sc2, hipStream_t s);

void sg_gemm(const void* a, int64_t lda, int a_kouter, const void* b, int64_t ldb, int b_kouter, void* c,
             int64_t ldc, int M, int N, int K, float alpha, float beta, const void* bias, int relu, int out_mode,
             int splits, int batch, int64_t sa, int64_t sb, int64_t sc, hipStream_t s) {
  sg_gemm_heads(a, lda, a_kouter, b, ldb, b_kouter, c, ldc, M, N, K, alpha, beta, bias, relu, out_mode, splits,
                batch, sa, sb, sc, 0, 0, 0, 0, s);
}

// sg_gemm with a fused activation (bf16 output through the LDS-staged
// epilogue): act (codes in GemmArgs) with the pre-activation also written to
// aux when given, or act_bwd: out *= act'(act_x) -- then optionally also
// colsum[n] += sum_m out[m][n] (fp32 atomics).  Returns 0 (nothing launched)
// when the shape cannot take the staged epilogue.
int sg_gemm_act(const void* a, int64_t lda, int a_kouter, const void* b, int64_t ldb, int b_kouter, void* c,
                int64_t ldc, int M, int N, int K, float alpha, const void* bias, int batch, int64_t sa, int64_t sb,
                int64_t sc, int act, void* aux, int act_bwd, const void* act_x, float* colsum, hipStream_t s) {
  if ((N & 7) != 0 || (ldc & 7) != 0 || !g_tune[1] || g_tune[4] != 0 || (act == 0) == (act_x == nullptr) ||
      M <= 0 || K <= 0 || batch != 1 || (colsum && (act != 0 || sg_bn_deterministic())))
    return 0;
  GemmArgs p{};
  init_phase_identity(p.g);
  p.sa = sa; p.sb = sb; p.sc = sc;
  p.M = M; p.N = N; p.K = K; p.a = (const bf16*)a; p.lda = lda; p.b = (const bf16*)b; p.ldb = ldb;
  p.c = c; p.ldc = ldc; p.alpha = alpha; p.beta = 0.f; p.bias = (const float*)bias; p.relu = 0;
  p.act = act; p.aux = (bf16*)aux; p.act_x = (const bf16*)act_x; p.act_bwd = act_bwd;
  if (colsum) {  // += column sums of the output (the producer's bias gradient), summed in the staged epilogue
    p.stats = colsum;
    p.stats_mode = 5;
    p.stats_det = 0;
  }
  p.k_per_split = kps(K, 1);
  p.a_bytes = extent_bytes(a_kouter ? (int64_t)(K - 1) * lda + M : (int64_t)(M - 1) * lda + K);
  p.b_bytes = extent_bytes(b_kouter ? (int64_t)(K - 1) * ldb + N : (int64_t)(N - 1) * ldb + K);
  // the GELU derivative alone (BERT's fc2 data gradient, K-major operands):
  // its own instantiation with the activation fixed at compile time (FLAGS
  // bit 1; the runtime dispatch multiplied the epilogue's SALU / VALU work,
  // profiles/r6/pmc_actgrad_epilogue.txt)
  if (act == 0 && act_bwd == 5 && !a_kouter && !b_kouter) {
    launch<LM_KMAJOR, LM_KMAJOR, OUT_BF16, 3>(p, M, 1, s, batch, 0);
    return 1;
  }
  if (!a_kouter && !b_kouter) launch<LM_KMAJOR, LM_KMAJOR, OUT_BF16, 1>(p, M, 1, s, batch, 0);
  else if (!a_kouter && b_kouter) launch<LM_KMAJOR, LM_KOUTER, OUT_BF16, 1>(p, M, 1, s, batch, 0);
  else if (a_kouter && !b_kouter) launch<LM_KOUTER, LM_KMAJOR, OUT_BF16, 1>(p, M, 1, s, batch, 0);
  else launch<LM_KOUTER, LM_KOUTER, OUT_BF16, 1>(p, M, 1, s, batch, 0);
  return 1;
}

// sg_gemm with a two-level batch: batch index y -> (y / bh, y % bh) with
// strides (sa, sa2), (sb, sb2), (sc, sc2); bh = 0 is the plain batched GEMM.
void sg_gemm_heads(const void* a, int64_t lda, int a_kouter, const void* b, int64_t ldb, int b_kouter, void* c,
                   int64_t ldc, int M, int N, int K, float alpha, float beta, const void* bias, int relu,
                   int out_mode, int splits, int batch, int64_t sa, int64_t sb, int64_t sc, int bh, int64_t sa2,
                   int64_t sb2, int64_t sc2, hipStream_t s) {
  GemmArgs p{};
  init_phase_identity(p.g);
  p.sa = sa; p.sb = sb; p.sc = sc;
  p.bh = bh; p.sa2 = sa2; p.sb2 = sb2; p.sc2 = sc2;
  p.M = M; p.N = N; p.K = K; p.a = (const bf16*)a; p.lda = lda; p.b = (const bf16*)b; p.ldb = ldb;
  p.c = c; p.ldc = ldc; p.alpha = alpha; p.beta = beta; p.bias = (const float*)bias; p.relu = relu;
  splits = (out_mode == OUT_F32_ATOMIC) ? pick_splits(M, N, K, splits) : 1;
  p.k_per_split = kps(K, splits);
  p.a_bytes = extent_bytes(a_kouter ? (int64_t)(K - 1) * lda + M : (int64_t)(M - 1) * lda + K);
  p.b_bytes = extent_bytes(b_kouter ? (int64_t)(K - 1) * ldb + N : (int64_t)(N - 1) * ldb + K);
#define GO(AM, BMD)                                                                  \
  {                                                                                  \
    if (out_mode == OUT_BF16) launch<AM, BMD, OUT_BF16>(p, M, splits, s, batch, 0);  \
    else if (out_mode == OUT_F32) launch<AM, BMD, OUT_F32>(p, M, splits, s, batch, 0); \
    else launch<AM, BMD, OUT_F32_ATOMIC>(p, M, splits, s, batch, 0);                \
  }
  if (!a_kouter && !b_kouter) GO(LM_KMAJOR, LM_KMAJOR)
  else if (!a_kouter && b_kouter) GO(LM_KMAJOR, LM_KOUTER)
  else if (a_kouter && !b_kouter) GO(LM_KOUTER, LM_KMAJOR)
  else GO(LM_KOUTER, LM_KOUTER)
#undef GO
}

// conv forward: x NHWC bf16, w [K][R][S][C] bf16 -> y [N*Ho*Wo][K]
void sg_conv_fwd(const void* x, const void* w, void* y, const void* bias, int N, int H, int W, int C, int K, int R,
                 int S, int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int relu, int out_mode,
                 void* stats, hipStream_t s) {
  GemmArgs p{};
  p.stats = (out_mode == OUT_BF16 && (K & 7) == 0 && g_tune[1]) ? (float*)stats : nullptr;
  p.stats_det = sg_bn_deterministic();
  if (p.stats && !p.stats_det && !sg_ws_prezeroed())  // (consumes the one-shot pre-zeroed flag)
    sg_zero_async(p.stats, sizeof(float) * 32 * 2 * K, s);  // atomic slot rows
  const bool k3s1 = R == 3 && S == 3 && sh == 1 && sw == 1 && ph == 1 && pw == 1 && dh == 1 && dw == 1 &&
                   Ho == H && Wo == W;
  if (k3s1 && out_mode == OUT_BF16 && !bias && !relu && !(p.stats && p.stats_det) &&
      sg_conv3x3_ok(N, H, W, C, K)) {
    sg_conv3x3_64(x, w, 0, y, p.stats, nullptr, N, H, W, C, K, s);
    return;
  }
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw);
  p.M = N * Ho * Wo; p.N = K; p.K = R * S * C;
  p.a = (const bf16*)x; p.lda = 0; p.b = (const bf16*)w; p.ldb = R * S * C;
  p.c = y; p.ldc = K; p.alpha = 1.f; p.beta = 0.f; p.bias = (const float*)bias; p.relu = relu;
  p.k_per_split = kps(p.K, 1);
  p.a_bytes = extent_bytes((int64_t)N * H * W * C);
  p.b_bytes = extent_bytes((int64_t)K * R * S * C);
  if (R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0) {
    // 1x1 stride-1 conv: the NHWC input IS the [pixels][C] operand -- a plain
    // K-major GEMM (no im2col gather state: these one/two-K-tile GEMMs are
    // dominated by their per-tile setup and epilogue)
    p.lda = C;
    if (out_mode == OUT_F32) launch<LM_KMAJOR, LM_KMAJOR, OUT_F32>(p, p.M, 1, s, 1, 0);
    else launch<LM_KMAJOR, LM_KMAJOR, OUT_BF16>(p, p.M, 1, s, 1, 0);
    return;
  }
  if (out_mode == OUT_F32) launch<LM_CONV_FWD, LM_KMAJOR, OUT_F32>(p, p.M, 1, s, 1, 0);
  else launch<LM_CONV_FWD, LM_KMAJOR, OUT_BF16>(p, p.M, 1, s, 1, 0);
}

// The fused residual tail's forward with its 1x1-conv output recomputed
// instead of stored (autograd.ConvBNAddReLU): pass 0 runs the persistent
// short-K GEMM for the BN statistics only (stats: 32 atomic slot rows
// [32][2][N]; no output written), pass 1 runs it again with the BN affine,
// the residual add, the ReLU and the mask bits in the epilogue (out, mask
// [M][N/8]).  On the stage-1/2 tails (K <= 128: the GEMM reads 64-128 bf16 per
// output row of 256-512) the second GEMM pass costs far less HBM traffic than
// writing and re-reading the conv output.  sg_sk_tail_ok: the shape takes the
// persistent kernel (else the caller runs the unfused conv + BN apply).
int sg_sk_tail_ok(int M, int N, int K) {
  return g_tune[9] && g_tune[4] == 0 && g_tune[1] && !sg_bn_deterministic() && K <= 128 && (K & 7) == 0 &&
         (N & 127) == 0 && (long)((M + 127) / 128) * (N / 128) >= 2048;
}

int sg_sk_tail(const void* a, const void* w, void* out, void* stats, const void* scale, const void* shift,
               const void* res, void* mask, int M, int N, int K, int pass, hipStream_t s) {
  if (!sg_sk_tail_ok(M, N, K)) return 0;
  GemmArgs p{};
  p.M = M; p.N = N; p.K = K;
  p.a = (const bf16*)a; p.lda = K; p.b = (const bf16*)w; p.ldb = K;
  p.ldc = N; p.alpha = 1.f; p.beta = 0.f;
  p.k_per_split = kps(K, 1);
  p.a_bytes = extent_bytes((int64_t)M * K);
  p.b_bytes = extent_bytes((int64_t)N * K);
  const int tiles_m = (M + 127) / 128;
  if (pass == 0) {
    p.stats = (float*)stats;
    if (!sg_ws_prezeroed()) sg_zero_async(p.stats, sizeof(float) * 32 * 2 * N, s);
    if (K <= 64) launch_sk<1, 0>(p, tiles_m, N / 128, s);
    else launch_sk<2, 0>(p, tiles_m, N / 128, s);
  } else {
    extent_bytes((int64_t)M * N);  // (output and residual within 32-bit buffer offsets)
    p.c = out;
    p.ep_scale = (const float*)scale; p.ep_shift = (const float*)shift;
    p.ep_res = (const bf16*)res; p.ep_mask = (uint8_t*)mask;
    if (K <= 64) launch_sk<1, 1>(p, tiles_m, N / 128, s);
    else launch_sk<2, 1>(p, tiles_m, N / 128, s);
  }
  return 1;
}

// The two-branch (downsample) tail's recomputed apply pass: out = relu(bf16([y | x] .
// wf^T) + shift) and its mask, K = K1 + K2 <= 128 (K1 % 64 == 0): wf [N][K1 + K2]
// holds both branches' weights with their BN scales folded in (bnres.hip
// fold_k), shift the sum of both BN shifts.  Returns 0 when the persistent
// kernel does not take the shape.
int sg_sk_tail2(const void* y, const void* x, const void* wf, const void* shift, const void* ones, void* out,
                void* mask, int M, int N, int K1, int K2, hipStream_t s) {
  const int K = K1 + K2;
  if (!sg_sk_tail_ok(M, N, K) || (K1 & 63) != 0 || K1 <= 0 || K2 <= 0) return 0;
  GemmArgs p{};
  p.M = M; p.N = N; p.K = K;
  p.a = (const bf16*)y; p.lda = K1; p.a2 = (const bf16*)x; p.lda2 = K2; p.a2_split = K1;
  p.b = (const bf16*)wf; p.ldb = K;
  p.ldc = N; p.alpha = 1.f; p.beta = 0.f;
  p.k_per_split = kps(K, 1);
  p.a_bytes = extent_bytes((int64_t)M * K1);
  p.a2_bytes = extent_bytes((int64_t)M * K2);
  p.b_bytes = extent_bytes((int64_t)N * K);
  extent_bytes((int64_t)M * N);
  p.c = out;
  p.ep_scale = (const float*)ones; p.ep_shift = (const float*)shift;
  p.ep_res = nullptr; p.ep_mask = (uint8_t*)mask;
  launch_sk<2, 1, LM_KMAJOR2>(p, (M + 127) / 128, N / 128, s);
  return 1;
}

// conv data gradient: dy [N*Ho*Wo][K] bf16, w [K][R][S][C] bf16 -> dx [N*H*W][C]
// (dilation 1; stride phases on blockIdx.z).  beta != 0 accumulates into dx
// (dx = dgrad + beta*dx: the gradient of a tensor with several consumers is
// summed in the epilogue instead of by a separate add pass; phases without
// taps then leave beta*dx).  wt (optional, K*R*S*C bf16 scratch, used when
// K % 64 == 0): the weights are transposed into it and read K-major.
void sg_conv_dgrad_bn(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S,
                      int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, float beta,
                      void* wt, void* bn_ws, const void* bn_x, const void* bn_mean, const void* bn_invstd,
                      const void* bn_scale, const void* bn_shift, hipStream_t s);

void sg_conv_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S, int Ho,
                   int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, float beta, void* wt,
                   hipStream_t s) {
  sg_conv_dgrad_bn(dy, w, dx, N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, out_mode, beta, wt, nullptr,
                   nullptr, nullptr, nullptr, nullptr, nullptr, s);
}

// As sg_conv_dgrad; with bn_ws != nullptr (bf16 out, beta == 0, C % 8 == 0,
// non-deterministic mode) the epilogue also writes the BatchNorm(+ReLU)
// backward partial sums of the producer BN into 32 atomic slot rows
// bn_ws[32][2][C] (zeroed here unless the one-shot pre-zeroed flag is set).
void sg_conv_dgrad_bn_ex(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S,
                         int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, float beta,
                         void* wt, void* bn_ws, const void* bn_x, const void* bn_mean, const void* bn_invstd,
                         const void* bn_scale, const void* bn_shift, const void* bn_mask, hipStream_t s);

void sg_conv_dgrad_bn(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S,
                      int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, float beta,
                      void* wt, void* bn_ws, const void* bn_x, const void* bn_mean, const void* bn_invstd,
                      const void* bn_scale, const void* bn_shift, hipStream_t s) {
  sg_conv_dgrad_bn_ex(dy, w, dx, N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, out_mode, beta, wt, bn_ws, bn_x,
                      bn_mean, bn_invstd, bn_scale, bn_shift, nullptr, s);
}

// dx = dgrad(dy, w) + res_g * bit(res_mask) (bf16, fresh dx: no beta
// read): the data gradient of a residual block's input, with the masked
// output gradient of the block's residual BN(+ReLU) -- the shortcut path's
// gradient -- added in the epilogue instead of being written by the BN
// backward and read back.  Returns 0 (nothing launched) when the shape does
// not take the LDS-staged epilogue (C % 8, stride 1 only): the caller then
// materialises the residual gradient itself.
int sg_conv_dgrad_res(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S,
                      int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, void* wt, const void* res_g,
                      const void* res_mask, hipStream_t s) {
  if ((C & 7) != 0 || !g_tune[1] || sh != 1 || sw != 1 || dh != 1 || dw != 1) {
    g_wt_ready = 0;
    return 0;
  }
  g_res_g = (const bf16*)res_g;
  g_res_mask = (const uint8_t*)res_mask;
  sg_conv_dgrad_bn_ex(dy, w, dx, N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, OUT_BF16, 0.f, wt, nullptr,
                      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, s);
  return 1;
}

// dx = (dgrad(dy, w) + acc) * bit(mask) (bf16, fresh dx), sum of dx per
// channel into bn_ws[32][2][C] (first half; zeroed here unless pre-zeroed):
// the gradient of a fused residual tail's output (autograd.ConvBNAddReLU)
// completed by this dgrad, masked and summed in the epilogue (stats_mode 4);
// the other consumers' gradient `acc` (bf16, or nullptr) is added from its
// own buffer like the lazy residual gradient (so the single-stage short-K
// variant, beta == 0, still applies).
// acc_s > 1 (1x1 stride-1 convs only): acc is compact, [N][acc_Ho][acc_Wo][C] at every
// acc_s-th pixel (a strided shortcut's input gradient, never placed on the full grid)
void sg_conv_dgrad_gsum(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S,
                        int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, void* wt, const void* acc,
                        void* bn_ws, const void* mask, int acc_s, int acc_Ho, int acc_Wo, hipStream_t s) {
  if (acc_s > 1 && (R != 1 || S != 1 || sh != 1 || sw != 1 || ph != 0 || pw != 0 || !acc))
    throw std::runtime_error("conv_dgrad_gsum: a strided accumulator needs a 1x1 stride-1 conv");
  g_res_g = (const bf16*)acc;
  g_res_mask = nullptr;
  g_mask_out = 1;
  g_res_s = acc_s > 1 ? acc_s : 1;
  g_res_Ho = acc_Ho;
  g_res_Wo = acc_Wo;
  sg_conv_dgrad_bn_ex(dy, w, dx, N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, OUT_BF16, 0.f, wt, bn_ws,
                      nullptr, nullptr, nullptr, nullptr, nullptr, mask, s);
}

// bn_mask != nullptr and bn_x == nullptr: the epilogue sums only the
// ReLU-masked gradient (stats_mode 3, the identity-sum BN backward).
// bn_mask != nullptr: the producer BN is a residual BN(+ReLU) whose ReLU mask
// is its 1-bit map; beta may then be 1 (dx accumulates the other consumers'
// gradient and the epilogue sums the partials of the FINAL value)
void sg_conv_dgrad_bn_ex(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S,
                         int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, float beta,
                         void* wt, void* bn_ws, const void* bn_x, const void* bn_mean, const void* bn_invstd,
                         const void* bn_scale, const void* bn_shift, const void* bn_mask, hipStream_t s) {
  const bool wt_ready = g_wt_ready;  // one-shot: wt already holds the K-major weights (batched pre-pass)
  g_wt_ready = 0;
  const bool mask_out = g_mask_out;
  g_mask_out = 0;
  GemmArgs p{};
  p.res_g = g_res_g;  // one-shot residual-gradient source (sg_conv_dgrad_res)
  p.res_mask = g_res_mask;
  p.res_s = g_res_s;
  if (p.res_s > 1) {
    p.res_H = H; p.res_W = W; p.res_Ho = g_res_Ho; p.res_Wo = g_res_Wo;
    p.res_dW = FastDiv((uint32_t)W);
    p.res_dH = FastDiv((uint32_t)H);
  }
  g_res_g = nullptr;
  g_res_mask = nullptr;
  g_res_s = 1;
  if (bn_ws && out_mode == OUT_BF16 && (beta == 0.f || bn_mask) && (C & 7) == 0 && g_tune[1] &&
      !sg_bn_deterministic()) {
    p.stats = (float*)bn_ws;
    p.stats_mode = bn_mask ? (bn_x ? 2 : (mask_out ? 4 : 3)) : 1;
    p.bnb_mask = (const uint8_t*)bn_mask;
    p.bnb_x = (const bf16*)bn_x;
    p.bnb_mean = (const float*)bn_mean; p.bnb_invstd = (const float*)bn_invstd;
    p.bnb_scale = (const float*)bn_scale; p.bnb_shift = (const float*)bn_shift;
    if (!sg_ws_prezeroed()) sg_zero_async(bn_ws, sizeof(float) * 32 * 2 * C, s);
  }
  if (R == 3 && S == 3 && sh == 1 && sw == 1 && ph == 1 && pw == 1 && dh == 1 && dw == 1 && Ho == H && Wo == W &&
      out_mode == OUT_BF16 && beta == 0.f && !p.res_g && (!p.stats || p.stats_mode == 3) && wt && (K & 63) == 0 &&
      sg_conv3x3_ok(N, H, W, C, K)) {
    // the persistent 64-channel kernel over the flipped K-major weights
    if (!wt_ready)
      hipLaunchKernelGGL(wt_transpose_k, dim3((C + 63) / 64, (K + 63) / 64, R * S), dim3(256), 0, s, (const bf16*)w,
                         (bf16*)wt, K, R * S, C);
    sg_conv3x3_64(dy, wt, 1, dx, p.stats, p.bnb_mask, N, H, W, C, K, s);
    return;
  }
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw);
  if (R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0) {
    // 1x1 stride-1: dx[M][C] = dy[M][K] W[K][C], a plain GEMM (dy K-major;
    // W K-outer, or K-major through the transposed copy)
    p.M = N * H * W; p.N = C; p.K = K;
    p.a = (const bf16*)dy; p.lda = K;
    p.c = dx; p.ldc = C; p.alpha = 1.f; p.beta = beta; p.bias = nullptr; p.relu = 0;
    p.k_per_split = kps(p.K, 1);
    p.a_bytes = extent_bytes((int64_t)p.M * K);
    p.b_bytes = extent_bytes((int64_t)K * C);
    if (wt && (K & 63) == 0) {
      if (!wt_ready)
        hipLaunchKernelGGL(wt_transpose_k, dim3((C + 63) / 64, (K + 63) / 64, 1), dim3(256), 0, s, (const bf16*)w,
                           (bf16*)wt, K, 1, C);
      p.b = (const bf16*)wt; p.ldb = K;
      // a fused tail's output gradient (stats_mode 4) on a short-K shape: the
      // persistent kernel with the masked-sum epilogue (sk_gemm_k EPI 2; the
      // compact strided accumulator stays on the generic kernel)
      if (p.stats && p.stats_mode == 4 && p.res_s <= 1 && out_mode == OUT_BF16 && beta == 0.f && g_tune[9] &&
          g_tune[4] == 0 && K <= 128 && (C & 127) == 0 && (long)((p.M + 127) / 128) * (C / 128) >= 2048) {
        GemmArgs q = p;
        q.ep_res = p.res_g;
        q.ep_mask = (uint8_t*)p.bnb_mask;
        q.res_g = nullptr;
        if (K <= 64) launch_sk<1, 2>(q, (p.M + 127) / 128, C / 128, s);
        else launch_sk<2, 2>(q, (p.M + 127) / 128, C / 128, s);
        return;
      }
      if (out_mode == OUT_F32) launch<LM_KMAJOR, LM_KMAJOR, OUT_F32>(p, p.M, 1, s, 1, 0);
      else launch<LM_KMAJOR, LM_KMAJOR, OUT_BF16>(p, p.M, 1, s, 1, 0);
    } else {
      p.b = (const bf16*)w; p.ldb = C;
      if (out_mode == OUT_F32) launch<LM_KMAJOR, LM_KOUTER, OUT_F32>(p, p.M, 1, s, 1, 0);
      else launch<LM_KMAJOR, LM_KOUTER, OUT_BF16>(p, p.M, 1, s, 1, 0);
    }
    return;
  }
  const int np = make_phases(p.g);
  int Mmax = 0;
  for (int i = 0; i < np; ++i) Mmax = Mmax > N * p.g.phs[i].Hp * p.g.phs[i].Wp ? Mmax : N * p.g.phs[i].Hp * p.g.phs[i].Wp;
  p.M = Mmax; p.N = C; p.K = R * S * K;
  p.a = (const bf16*)dy; p.lda = 0; p.b = (const bf16*)w; p.ldb = 0;
  p.c = dx; p.ldc = C; p.alpha = 1.f; p.beta = beta; p.bias = nullptr; p.relu = 0;
  p.out_phase = 1;
  p.k_per_split = kps(p.K, 1);
  p.a_bytes = extent_bytes((int64_t)N * Ho * Wo * K);
  p.b_bytes = extent_bytes((int64_t)K * R * S * C);
  extent_bytes((int64_t)N * H * W * C);
  if (wt && (K & 63) == 0) {
    // K-major weights: transpose once per call (weights are small), then the
    // B operand is read with ds_read_b128 like the forward's, not transposed
    // through LDS
    if (!wt_ready)
      hipLaunchKernelGGL(wt_transpose_k, dim3((C + 63) / 64, (K + 63) / 64, R * S), dim3(256), 0, s, (const bf16*)w,
                         (bf16*)wt, K, R * S, C);
    p.b = (const bf16*)wt;
    if (out_mode == OUT_F32) launch<LM_DGRAD_A, LM_DGRAD_BT, OUT_F32>(p, Mmax, 1, s, 1, np);
    else launch<LM_DGRAD_A, LM_DGRAD_BT, OUT_BF16>(p, Mmax, 1, s, 1, np);
    return;
  }
  if (out_mode == OUT_F32) launch<LM_DGRAD_A, LM_DGRAD_B, OUT_F32>(p, Mmax, 1, s, 1, np);
  else launch<LM_DGRAD_A, LM_DGRAD_B, OUT_BF16>(p, Mmax, 1, s, 1, np);
}

// Split count of the 8-wave split-K weight gradient, quantisation-aware:
// two of these workgroups run per CU, so the launch runs in waves of 2 x CUs
// workgroups and a partial last wave costs a whole one -- 1152 workgroups (36
// tiles x 32 splits) are 2.25 waves.  Among split counts with >= 16 K-tiles
// per split and at most twice the power-of-2 choice `sp0`, take the one
// minimising ceil(tiles * sp / slots) * (ceil(nkt / sp) + e), e the atomic
// epilogue in K-tile units; ties go to fewer splits (fewer atomic passes over
// the output).  Measured on the ResNet-50 b1024 shapes (tools/wgrad_sweep.py,
// profiles/r5/wgrad_sweep.jsonl): stage-2/3/4 3x3 weight gradients 368 / 300 /
// 293 us -> 263 / 266 / 255 us (splits 56 / 14 / 7).
static int wgrad_splits_q(int tiles, int nkt, int sp0, int per_cu = 2) {
  const int slots = per_cu * sg_cu_count();
  constexpr int e = 6;
  int best = sp0;
  long best_cost = (long)((tiles * sp0 + slots - 1) / slots) * ((nkt + sp0 - 1) / sp0 + e);
  for (int sp = 1; sp <= 2 * sp0 && nkt / sp >= 16; ++sp) {
    const long cost = (long)((tiles * sp + slots - 1) / slots) * ((nkt + sp - 1) / sp + e);
    if (cost < best_cost || (cost == best_cost && sp < best)) {
      best = sp;
      best_cost = cost;
    }
  }
  return best;
}

// conv weight gradient: dW[K][R*S*C] (fp32, accumulated atomically: the caller
// zeroes it unless accumulating) += dy^T * im2col(x)
void sg_conv_wgrad(const void* x, const void* dy, void* dw_out, int N, int H, int W, int C, int K, int R, int S,
                   int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int splits, hipStream_t s) {
  GemmArgs p{};
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw);
  p.M = K; p.N = R * S * C; p.K = N * Ho * Wo;
  p.a = (const bf16*)dy; p.lda = K; p.b = (const bf16*)x; p.ldb = 0;
  p.c = dw_out; p.ldc = R * S * C; p.alpha = 1.f; p.beta = 0.f; p.bias = nullptr; p.relu = 0;
  p.a_bytes = extent_bytes((int64_t)N * Ho * Wo * K);
  p.b_bytes = extent_bytes((int64_t)N * H * W * C);
  int BM, BN, sp;
  int mode = g_tune[0], extra = g_tune[3];
  if (mode == 5) {
    // measured per-shape policy (tools/tune_conv.py, ResNet-50 b256, after the
    // LDS-staged atomic epilogue and the K-slice-major XCD mapping):
    //  * filters with taps (3x3, 7x7): 2x / 4x more K-slices than the base
    //    policy (narrow outputs need more) -- -10..-25 %;
    //  * 1x1 with stride 2, or halving the channels (a stage's entry conv):
    //    128x128 tiles, fewer slices (mode 1) -- -5..-30 %;
    //  * other 1x1: base policy.
    if (R * S > 1) {
      mode = 4;
      extra += K <= 128 ? 2 : 1;
    } else {
      mode = (sh > 1 || sw > 1 || C == 2 * K) ? 1 : 4;
    }
  }
  pick_wgrad(p.M, p.N, p.K, mode, BM, BN, sp);
  if (extra > 0) {  // scale the split count (bounded by the K-tiles)
    const int nkt = (p.K + BK - 1) / BK;
    for (int i = 0; i < extra && sp * 2 <= nkt; ++i) sp *= 2;
  }
  // 8-wave 128x128 tiles (two workgroups per CU) once both output dims fill
  // them; split-K up to ~1024 workgroups for filters with taps, ~512 for 1x1
  // (measured, ResNet-50 b1024: -12..-40 % on every such layer vs the 4-wave
  // policy; 64-wide outputs and the stem keep it)
  const bool big = g_tune[5] && p.M >= 128 && p.N >= 128 && splits <= 0 && !sg_bn_deterministic();
  if (big) {
    const int tiles = ((p.M + 127) / 128) * ((p.N + 127) / 128);
    const int nkt = (p.K + BK - 1) / BK;
    const int target = g_tune[10] > 0 ? g_tune[10] : R * S > 1 ? 1024 : 512;
    sp = 1;
    while (tiles * sp < target && sp * 2 * 4 <= nkt) sp *= 2;
    if (g_tune[13] && g_tune[10] <= 0) sp = wgrad_splits_q(tiles, nkt, sp);
    if (g_tune[12] > 0) sp = g_tune[12];
    if (g_tune[15] == 1 && p.M >= 256 && (p.M & 255) == 0) {  // (M = 384: a half-empty second row of tiles, AlexNet -2 %)
      // 256 x 128 tiles of 64 x 64 wave tiles (half the LDS fragment traffic
      // per MFMA of the 64 x 32 wave tiles), three-stage ring, one per CU
      const int t2 = ((p.M + 255) / 256) * ((p.N + 127) / 128);
      int sp2 = 1;
      while (t2 * sp2 < target && sp2 * 2 * 4 <= nkt) sp2 *= 2;
      // (one workgroup per CU: its 144 KB ring; the model's picks match the
      // best measured split of every eligible ResNet-50 layer,
      // profiles/r5/wgrad_sweep_256x128_on.jsonl)
      if (g_tune[13] && g_tune[10] <= 0) sp2 = wgrad_splits_q(t2, nkt, sp2, 1);
      if (g_tune[12] > 0) sp2 = g_tune[12];
      p.k_per_split = kps(p.K, sp2);
      launch_t<256, 128, LM_KOUTER, LM_WGRAD_B, OUT_F32_ATOMIC, 512, 4, 2, 3>(p, t2, 1, sp2, s);
      return;
    }
    if (g_tune[15] == 1 && g_tune[17] == 1 && p.M < 256 && p.N >= 256) {
      // K_out = 128 (stage 2): 128 x 256 tiles, waves 2 x 4 of 64 x 64 (A/B: knob 17)
      const int t2 = ((p.M + 127) / 128) * ((p.N + 255) / 256);
      int sp2 = 1;
      while (t2 * sp2 < target && sp2 * 2 * 4 <= nkt) sp2 *= 2;
      if (g_tune[13] && g_tune[10] <= 0) sp2 = wgrad_splits_q(t2, nkt, sp2, 1);
      if (g_tune[12] > 0) sp2 = g_tune[12];
      p.k_per_split = kps(p.K, sp2);
      launch_t<128, 256, LM_KOUTER, LM_WGRAD_B, OUT_F32_ATOMIC, 512, 2, 4, 3>(p, t2, 1, sp2, s);
      return;
    }
    p.k_per_split = kps(p.K, sp);
    launch_t<128, 128, LM_KOUTER, LM_WGRAD_B, OUT_F32_ATOMIC, 512, 2, 4, 2>(p, tiles, 1, sp, s);
    return;
  }
  if (splits > 0) sp = splits;
  if (sg_bn_deterministic()) sp = 1;  // one writer per gradient element: reproducible
  p.k_per_split = kps(p.K, sp);
  launch_tile<LM_KOUTER, LM_WGRAD_B, OUT_F32_ATOMIC>(p, p.M, BM, BN, sp, s, 1, 0);
}

// rows of the fused-BN-statistics workspace a conv forward writes
// ([rows][2][K]: tiles_m in deterministic mode, else 32 atomic slot rows that
// the caller zeroes); 0 if that conv cannot produce them
int sg_conv_stats_rows(int M, int N) {
  if ((N & 7) != 0 || !g_tune[1]) return 0;
  if (!sg_bn_deterministic()) return 32;
  if (int big = pick_big(M, N)) {
    if (big == 4) big = 1;  // the ping-pong kernel is not used with deterministic statistics
    return (M + big_bm(big) - 1) / big_bm(big);
  }
  int BM, BN;
  pick_tile(M, N, BM, BN);
  return (M + BM - 1) / BM;
}

void sg_set_wt_ready(int on) { g_wt_ready = on; }
void sg_set_dgrad_mask_out(int on) { g_mask_out = on; }
// wdot[c] += sign * sum_rows W[row][c] dW[row][c] (zeroes wdot first unless the
// one-shot pre-zeroed flag is set and sign > 0 ... callers pass zero_first)
// gamma != nullptr: also raise the int flag stored at wdot + C (zeroed with
// wdot) when the producer BN's |gamma| / |beta| fail the recovery gate
void sg_wdot_colsum(const void* w, const void* dw, int rows, int C, float sign, void* wdot, int zero_first,
                    const void* gamma, const void* beta, float tau, hipStream_t s) {
  if (zero_first && !sg_ws_prezeroed()) sg_zero_async(wdot, sizeof(float) * (C + 1), s);
  hipLaunchKernelGGL(wdot_colsum_k, dim3((C + 63) / 64, (rows + WDOT_RB - 1) / WDOT_RB), dim3(256), 0, s,
                     (const bf16*)w, (const float*)dw, rows, C, sign, (float*)wdot, (const float*)gamma,
                     (const float*)beta, tau, (int*)((float*)wdot + C));
}
// desc: n WtDesc entries in device memory (32 bytes each), total = sum of tiles
void sg_wt_transpose_batched(const void* desc, int n, int total, hipStream_t s) {
  static_assert(sizeof(WtDesc) == 32, "descriptor layout shared with the Python packer");
  if (n > 0 && total > 0)
    hipLaunchKernelGGL(wt_transpose_batched_k, dim3(total), dim3(256), 0, s, (const WtDesc*)desc, n);
}
void sg_set_tuning(int key, int value) {
  if (key >= 0 && key < 20) g_tune[key] = value;
}
int sg_get_tuning(int key) { return key >= 0 && key < 20 ? g_tune[key] : 0; }

}  // extern "C"

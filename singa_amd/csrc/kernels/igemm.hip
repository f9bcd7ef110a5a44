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
#include <stdexcept>
#include <type_traits>

#include "common.h"

namespace sg {

constexpr int BK = 64, NT = 256;

enum LoadMode : int {
  LM_KMAJOR = 0,   // plain [rows][K] (ld)
  LM_KOUTER = 1,   // plain [K][rows] (ld)
  LM_CONV_FWD = 2, // A of fwd: im2col of x NHWC, K = (r, s, c)
  LM_DGRAD_A = 3,  // A of dgrad: gather of dy NHWC over the phase taps, K = (tap, k)
  LM_WGRAD_B = 4,  // B of wgrad: x gathered, rows = (r, s, c), K = output pixels
  LM_DGRAD_B = 5,  // B of dgrad: W [K][R][S][C] as K-outer, rows = c, K = (tap, k)
  LM_DGRAD_BT = 6, // B of dgrad from the transposed copy WT [R][S][C][K]: K-major rows c, K = (tap, k)
};
enum OutMode : int { OUT_BF16 = 0, OUT_F32 = 1, OUT_F32_ATOMIC = 2 };

struct Phase {
  int a, b;            // output pixel phase (h % sh == a, w % sw == b)
  int r0, s0, nr, ns;  // taps r = r0 + sh*j (j < nr), s = s0 + sw*i (i < ns)
  int offh, offw;      // oh = hh + offh - j, ow = ww + offw - i
  int Hp, Wp;          // phase grid size
  FastDiv dns, dWp, dHpWp;
};

struct ConvGeom {
  int N, H, W, C;  // input (NHWC)
  int K, R, S;     // filters [K][R][S][C]
  int Ho, Wo;      // output
  int sh, sw, ph, pw, dh, dw;
  int bq_n, bq_h, bq_w;  // BK output pixels = bq_n images + bq_h rows + bq_w columns (mixed radix)
  FastDiv dC, dS, dK, dWo, dHoWo;
  Phase phs[16];
};

struct GemmArgs {
  int M, N, K;
  const bf16* a;
  int64_t lda;
  const bf16* b;
  int64_t ldb;
  void* c;
  int64_t ldc;
  float alpha, beta;
  const float* bias;
  int relu;
  int k_per_split;     // multiple of BK
  int64_t sa, sb, sc;  // batch strides (elements), blockIdx.y = batch
  // two-level batch (attention heads read in place from a [B][S][3][H][D]
  // projection): with bh > 0, batch y -> (y / bh) * s? + (y % bh) * s?2
  int bh;
  int64_t sa2, sb2, sc2;
  int out_phase;       // dgrad: output rows map through the phase grid
  int lds_epilogue;    // stage bf16 output tiles through LDS (16-byte stores)
  unsigned a_bytes, b_bytes;  // operand extents (buffer-resource ranges; per batch slice)
  float* stats;        // optional BN statistics of the bf16 output: ws[row][2][N] (sum, sum of squares)
  int stats_det;       // 1: row = tile row, plain stores (deterministic); 0: row = tile row % 32, atomics
  int xcd_split;       // split-K: K-slice-major XCD mapping (gridDim.z % 8 == 0, gridDim.y == 1)
  int early_issue;     // 2-stage loop: issue tile kt+1 before waiting for tile kt (two barriers per tile)
  int nt_store;        // LDS-staged bf16 epilogue: non-temporal 16-byte output stores
  // stats_mode 1 (dgrad feeding a BN(+ReLU) backward): with g = out * [x*scale+shift > 0]
  // and xhat = (x - mean) * invstd, the epilogue sums (g, g*xhat) per channel
  // into `stats` -- the BN backward's reduction pass, fused
  // stats_mode 2: the same sums for a residual BN(+ReLU) whose ReLU mask is
  // the 1-bit map bnb_mask [rows][C/8] written by its forward apply
  // stats_mode 3: only sum(g) over the mask bits (the identity-sum BN backward)
  int stats_mode;
  // residual-gradient accumulate (bf16 LDS-staged epilogue, beta == 0, no
  // stats): out += res_g * bit(res_mask) -- the gradient a residual
  // BN(+ReLU) passes to its shortcut input is its masked output gradient;
  // the consuming conv's dgrad adds it from (dy, 1-bit mask) directly, so
  // the BN backward never writes it as a tensor
  const bf16* res_g;
  const uint8_t* res_mask;
  const uint8_t* bnb_mask;
  const bf16* bnb_x;
  const float *bnb_mean, *bnb_invstd, *bnb_scale, *bnb_shift;
  ConvGeom g;
  // (kept after g: every other kernel's argument layout is unchanged)
  // fused activation of the bf16 output (LDS-staged epilogue, host-checked):
  // codes 1 relu, 2 sigmoid, 3 tanh, 4 stanh, 5 gelu (erf), 6 gelu (tanh);
  // aux (optional): the pre-activation z (bf16, laid out like C)
  int act;
  bf16* aux;
  // fused activation backward: out = bf16(out) * act'(act_x), act_x the
  // activation's output (codes 1-4) or its input z (5, 6), laid out like C
  // (beta == 0: it is read up front in place of the accumulate source)
  const bf16* act_x;
  int act_bwd;
};

// the fused activations: the formulas of elementwise.hip's unary_f / unary_b,
// so a fused epilogue rounds exactly like the separate kernels did
__device__ __forceinline__ float ep_act(int a, float x) {
  switch (a) {
    case 1: return fmaxf(x, 0.f);
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: return tanhf(x);
    case 4: return 1.7159047f * tanhf(0.66666667f * x);
    case 5: return 0.5f * x * (1.f + erff(x * 0.70710678118f));
    case 6: return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x)));
    default: return x;
  }
}
// derivative from the output y (codes 1-4) or the input x (5, 6)
__device__ __forceinline__ float ep_dact(int a, float t) {
  switch (a) {
    case 1: return t > 0.f ? 1.f : 0.f;
    case 2: return t * (1.f - t);
    case 3: return 1.f - t * t;
    case 4: return 0.66666667f * 1.7159047f - 0.66666667f / 1.7159047f * t * t;
    case 5: return 0.5f * (1.f + erff(t * 0.70710678118f)) + t * 0.3989422804f * __expf(-0.5f * t * t);
    case 6: {
      const float u = 0.7978845608f * (t + 0.044715f * t * t * t), th = tanhf(u);
      const float du = 0.7978845608f * (1.f + 3.f * 0.044715f * t * t);
      return 0.5f * (1.f + th) + 0.5f * t * (1.f - th * th) * du;
    }
    default: return 1.f;
  }
}

__device__ __forceinline__ int kmajor_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
template <int ROWS>
__device__ __forceinline__ int kouter_swz(int krow, int chunk) {
  if constexpr (ROWS >= 128) return chunk ^ (((krow & 3) << 2) | ((krow >> 2) & 3));
  else return chunk ^ ((((krow >> 1) & 1) << 1) | (((krow >> 3) & 1) << 2));
}

// byte distance between k-halves of a K-outer LDS image with ROWS columns
template <int ROWS>
constexpr int kk_off(int kk) { return kk * 32 * ROWS * 2; }

__device__ __forceinline__ uint4 sel(bool ok, uint4 v) { return ok ? v : make_uint4(0, 0, 0, 0); }

// ------------------------------------------------------------------------------
// Operand loader: ROWS = tile rows of this operand, VPT 16-byte vectors/thread,
// staged global -> LDS directly with global_load_lds_dwordx4 (no registers,
// no ds_write, no zero-select: out-of-range / padding vectors read a zero
// page).  One wave-instruction fills 1 KB of LDS at (wave-uniform base +
// lane*16), so each operand image is laid out lane-linearly and the XOR
// swizzle is applied to the SOURCE chunk each lane fetches:
//   KMAJOR kinds: thread t owns rows (t>>3)+32v, LDS slot t&7 holds k-chunk
//                 (t&7) ^ swz(row)           (a wave = 8 rows x 128 B)
//   KOUTER kinds: thread t owns k-rows t/CPR + (256/CPR)v, LDS slot t%CPR
//                 holds column chunk (t%CPR) ^ swz(k-row)
// Conv gathers cache each vector's row pointer for the current filter tap and
// recompute it only when the (wave-uniform) tap changes.
// ------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// 16-byte buffer load straight into LDS (buffer_load_dwordx4 ... offen lds):
// 32-bit byte offsets against a buffer resource; an offset past num_records
// returns zeros, which implements padding / out-of-range rows for free.
// Operands are < 2 GiB (host-checked), so a masked-off vector keeps its
// per-lane offset biased by BIAS: any non-negative scalar advance (< 2 GiB)
// added later still lands past num_records.  The K loop therefore costs one
// v_add per 16-byte vector (per-lane part + scalar K advance) plus the SALU
// write of the wave-uniform LDS destination into M0.
constexpr unsigned OOB = 0xFFFFFFF0u;
constexpr unsigned BIAS = 0x80000000u;
__device__ __forceinline__ void bld16(__amdgpu_buffer_rsrc_t rsrc, unsigned off, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)lds_wave_base, 16, off, 0, 0, 0);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int ROWS, int MODE, int NTH = NT>
struct Loader {
  static constexpr int VPT = ROWS * 8 / NTH;  // 16-byte vectors (= LDS-DMA wave-instructions) per thread per K-tile
  static constexpr bool KOUT = (MODE == LM_KOUTER || MODE == LM_WGRAD_B || MODE == LM_DGRAD_B);
  static constexpr int CPR = ROWS / 8;   // KOUTER: chunks per k-row
  static constexpr int KRP = NTH / CPR;  // KOUTER: k-rows per pass
  static constexpr int RPV = NTH / 8;    // KMAJOR: rows per pass
  static_assert(VPT >= 1 && CPR <= 64, "tile too small for the thread count");
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned voff[VPT];  // per-lane byte offsets (BIAS-ed when masked); see issue()
  int pbase[VPT];      // conv gathers: element offset of this row's pixel at tap 0 (may lie in the padding)
  int i0[VPT], j0[VPT];
  bool ok[VPT];
  int64_t ld;
  int wv;                     // wave id (wave-uniform, SGPR)
  int lchunk;                 // KMAJOR: the k-chunk this lane fetches (swizzled)
  int kr0;                    // KOUTER: this lane's k-row within a pass
  int cr, cs, cc;             // WGRAD_B: fixed column decomposition
  bool cok;
  // WGRAD_B pixel walk (general conv): per vector the input coordinates of
  // this lane's tap at its current pixel and the byte offset of that element,
  // advanced by BK pixels per K-tile with mixed-radix carries (adds and
  // selects only: the per-tile divisions and 32-bit multiplies it replaces
  // are quarter-rate and made the weight gradient VALU-bound)
  int wih[VPT], wiw[VPT], wpo[VPT];
  int ihl, iwl;               // wrap limits (ow >= Wo <=> iw >= iwl; oh >= Ho <=> ih >= ihl)
  int tap_cached;             // conv gathers: tap of the cached row offsets
  bool uni;                   // conv gathers: channels per tap % 64 == 0 (whole K-tile in one tap)

  __device__ __forceinline__ void init(const GemmArgs& p, int row0, int nrows, const Phase& P, int64_t ld_,
                                       const bf16* src, unsigned bytes) {
    const int t = threadIdx.x;
    wv = __builtin_amdgcn_readfirstlane(t >> 6);
    ld = ld_;
    tap_cached = -1;
    rsrc = make_rsrc(src, bytes);
    if constexpr (!KOUT) {
      const int row_l = t >> 3;  // (row >> 1) & 7 is the same for every v (RPV*v keeps bits 1-3)
      lchunk = (t & 7) ^ ((row_l >> 1) & 7);
      if constexpr (MODE == LM_CONV_FWD) uni = (p.g.C & 63) == 0;
      if constexpr (MODE == LM_DGRAD_A) uni = (p.g.K & 63) == 0;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int row = row0 + row_l + RPV * v;
        ok[v] = row < nrows;
        const int rr = ok[v] ? row : 0;
        if constexpr (MODE == LM_KMAJOR) {
          voff[v] = ok[v] ? (unsigned)(rr * (int)ld + lchunk * 8) * 2u : BIAS;
        } else if constexpr (MODE == LM_CONV_FWD) {
          const ConvGeom& g = p.g;
          const int n = g.dHoWo.div(rr);
          const int rem = rr - n * g.Ho * g.Wo;
          const int oh = g.dWo.div(rem);
          const int ow = rem - oh * g.Wo;
          i0[v] = oh * g.sh - g.ph;
          j0[v] = ow * g.sw - g.pw;
          pbase[v] = n * g.H * g.W * g.C + (i0[v] * g.W + j0[v]) * g.C;
        } else if constexpr (MODE == LM_DGRAD_BT) {
          voff[v] = ok[v] ? (unsigned)(rr * p.g.K + lchunk * 8) * 2u : BIAS;  // row c of a tap slab [C][K]
        } else {  // LM_DGRAD_A: row = (n, hh, ww) of the phase grid
          const ConvGeom& g = p.g;
          const int n = P.dHpWp.div(rr);
          const int rem = rr - n * P.Hp * P.Wp;
          const int hh = P.dWp.div(rem);
          const int ww = rem - hh * P.Wp;
          i0[v] = hh + P.offh;
          j0[v] = ww + P.offw;
          pbase[v] = n * g.Ho * g.Wo * g.K + (i0[v] * g.Wo + j0[v]) * g.K;
        }
      }
    } else {
      kr0 = t / CPR;
      const int col = row0 + (((t % CPR) ^ kouter_swz<ROWS>(kr0, 0)) * 8);  // swz(kr) same for every v
      cok = col < nrows;
      if constexpr (MODE == LM_KOUTER) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) voff[v] = cok ? (unsigned)((kr0 + KRP * v) * (int)ld + col) * 2u : BIAS;
      } else if constexpr (MODE == LM_WGRAD_B) {
        const ConvGeom& g = p.g;
        const int c2 = cok ? col : 0;
        const int rs = g.dC.div(c2);
        cc = c2 - rs * g.C;
        cr = g.dS.div(rs);
        cs = rs - cr * g.S;
        ihl = g.Ho * g.sh + cr * g.dh - g.ph;
        iwl = g.Wo * g.sw + cs * g.dw - g.pw;
#pragma unroll
        for (int v = 0; v < VPT; ++v) voff[v] = cok ? (unsigned)((kr0 + KRP * v) * g.C + cc) * 2u : BIAS;
      } else {  // LM_DGRAD_B
        cc = col;
      }
    }
  }

  // WGRAD_B: position the pixel walk at the first K-tile (k0 = kbeg)
  __device__ __forceinline__ void start(const GemmArgs& p, int k0) {
    if constexpr (MODE == LM_WGRAD_B) {
      const ConvGeom& g = p.g;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int pix = k0 + kr0 + KRP * v;
        const int pp = pix < p.K ? pix : 0;
        const int n = g.dHoWo.div(pp);
        const int rem = pp - n * g.Ho * g.Wo;
        const int oh = g.dWo.div(rem);
        const int ow = rem - oh * g.Wo;
        wih[v] = oh * g.sh - g.ph + cr * g.dh;
        wiw[v] = ow * g.sw - g.pw + cs * g.dw;
        wpo[v] = (((n * g.H + wih[v]) * g.W + wiw[v]) * g.C + cc) * 2;
      }
    }
  }
  __device__ __forceinline__ void wadvance(const ConvGeom& g) {
    const int C2 = g.C * 2;
    const int dw_ = g.bq_w * g.sw, dh_ = g.bq_h * g.sh;
    const int dP = C2 * (dw_ + g.W * dh_ + g.bq_n * g.H * g.W);
    const int dRow = C2 * (g.sh * g.W - g.Wo * g.sw), dImg = C2 * (g.H * g.W - g.Ho * g.sh * g.W);
    const int wrapw = g.Wo * g.sw, wraph = g.Ho * g.sh;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      int iw = wiw[v] + dw_;
      const bool c1 = iw >= iwl;
      iw -= c1 ? wrapw : 0;
      int ih = wih[v] + dh_ + (c1 ? g.sh : 0);
      const bool c2 = ih >= ihl;
      ih -= c2 ? wraph : 0;
      wiw[v] = iw;
      wih[v] = ih;
      wpo[v] += dP + (c1 ? dRow : 0) + (c2 ? dImg : 0);
    }
  }

  // Issue the K-tile starting at k0 (absolute) into the LDS stage `lds`.
  // live == false: a dummy tile (past the end of K) that only keeps the
  // per-tile DMA count uniform -- every vector goes through a null resource
  // (num_records 0: no memory traffic, zeros into a stage nobody reads).
  __device__ __forceinline__ void issue(const GemmArgs& p, int row0, int nrows, int k0, int kend, const Phase& P,
                                        char* lds, bool live = true) {
    const __amdgpu_buffer_rsrc_t rs = live ? rsrc : make_rsrc(nullptr, 0);
    const bool full = kend - k0 >= BK;  // wave-uniform: no per-lane K bound inside this tile
    if constexpr (MODE == LM_KMAJOR) {
      const bool kin = full || (k0 + lchunk * 8 < kend);
#pragma unroll
      for (int v = 0; v < VPT; ++v)
        bld16(rs, kin ? voff[v] + (unsigned)k0 * 2u : OOB, lds + (8 * wv + RPV * v) * 128);
    } else if constexpr (MODE == LM_DGRAD_BT) {
      // K-tile = one tap (g.K % 64 == 0, host-checked): scalar tap math, then
      // a plain K-major row fetch from that tap's [C][K] slab
      const ConvGeom& g = p.g;
      const int tap = g.dK.div(k0);
      const int j = P.dns.div(tap), i = tap - j * P.ns;
      const int r = P.r0 + g.sh * j, sc = P.s0 + g.sw * i;
      const unsigned adv = (unsigned)((r * g.S + sc) * g.C * g.K + k0 - tap * g.K) * 2u;
#pragma unroll
      for (int v = 0; v < VPT; ++v) bld16(rs, voff[v] + adv, lds + (8 * wv + RPV * v) * 128);
    } else if constexpr (MODE == LM_CONV_FWD || MODE == LM_DGRAD_A) {
      const ConvGeom& g = p.g;
      const int CH = MODE == LM_CONV_FWD ? g.C : g.K;
      const FastDiv& dch = MODE == LM_CONV_FWD ? g.dC : g.dK;
      const int HH = MODE == LM_CONV_FWD ? g.H : g.Ho, WW = MODE == LM_CONV_FWD ? g.W : g.Wo;
      if (uni) {  // the whole K-tile is one tap (K % 64 == 0 too): row offsets cached per tap
        const int tap = dch.div(k0);
        if (tap != tap_cached) {
          tap_cached = tap;
          int dr, ds;
          if constexpr (MODE == LM_CONV_FWD) {
            const int r = g.dS.div(tap), s = tap - r * g.S;
            dr = r * g.dh;
            ds = s * g.dw;
          } else {
            const int j = P.dns.div(tap), i = tap - j * P.ns;
            dr = -j;
            ds = -i;
          }
          // the tap moves every row of the tile by the same (scalar) offset:
          // only the bounds test is per lane (no per-lane multiplies)
          const int tdelta = (dr * WW + ds) * CH + lchunk * 8;
#pragma unroll
          for (int v = 0; v < VPT; ++v) {
            const int ih = i0[v] + dr, iw = j0[v] + ds;
            const bool o = ok[v] && (unsigned)ih < (unsigned)HH && (unsigned)iw < (unsigned)WW;
            voff[v] = o ? (unsigned)(pbase[v] + tdelta) * 2u : BIAS;
          }
        }
        const unsigned adv = (unsigned)(k0 - tap * CH) * 2u;
#pragma unroll
        for (int v = 0; v < VPT; ++v) bld16(rs, voff[v] + adv, lds + (8 * wv + RPV * v) * 128);
      } else {  // per-lane tap (channel counts not a multiple of 64, e.g. the padded stem)
        int kk = k0 + lchunk * 8;
        const bool kin = kk < kend;
        kk = kin ? kk : 0;
        const int tap = dch.div(kk);
        const int c0 = kk - tap * CH;
        int dr, ds;
        if constexpr (MODE == LM_CONV_FWD) {
          const int r = g.dS.div(tap), s = tap - r * g.S;
          dr = r * g.dh;
          ds = s * g.dw;
        } else {
          const int j = P.dns.div(tap), i = tap - j * P.ns;
          dr = -j;
          ds = -i;
        }
        const int tdelta = (dr * WW + ds) * CH + c0;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
          const int ih = i0[v] + dr, iw = j0[v] + ds;
          const bool o = ok[v] && kin && (unsigned)ih < (unsigned)HH && (unsigned)iw < (unsigned)WW;
          const int off = pbase[v] + tdelta;
          bld16(rs, o ? (unsigned)off * 2u : OOB, lds + (8 * wv + RPV * v) * 128);
        }
      }
    } else if constexpr (MODE == LM_KOUTER) {
      const unsigned adv = (unsigned)k0 * (unsigned)ld * 2u;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const bool o = full || (k0 + kr0 + KRP * v < kend);
        bld16(rs, o ? voff[v] + adv : OOB, lds + (wv * (64 / CPR) + KRP * v) * (ROWS * 2));
      }
    } else if constexpr (MODE == LM_DGRAD_B) {
      // B(n = c, kk = (tap, k)) = W[k][r][s][c]; rows c contiguous per (k, tap)
      const ConvGeom& g = p.g;
      const int col = cc;
      const bool cin = cok;
      const int RSC = g.R * g.S * g.C;
      const bool uk = (g.K & 63) == 0;
      const int tapu = g.dK.div(k0);
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        int kk = k0 + kr0 + KRP * v;
        const bool kin = kk < kend;
        kk = kin ? kk : 0;
        const int tap = uk ? tapu : (int)g.dK.div(kk);
        const int k = kk - tap * g.K;
        const int j = P.dns.div(tap), i = tap - j * P.ns;
        const int r = P.r0 + g.sh * j, s = P.s0 + g.sw * i;
        const bool o = cin && kin;
        const int off = k * RSC + (r * g.S + s) * g.C + col;
        bld16(rs, o ? (unsigned)off * 2u : OOB, lds + (wv * (64 / CPR) + KRP * v) * (ROWS * 2));
      }
    } else if constexpr (MODE == LM_WGRAD_B) {
      const ConvGeom& g = p.g;
      if (g.R == 1 && g.S == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0) {
        // 1x1 stride-1 conv: input pixel == output pixel, no bounds
        const unsigned adv = (unsigned)k0 * (unsigned)g.C * 2u;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
          const bool o = full || (k0 + kr0 + KRP * v < kend);
          bld16(rs, o ? voff[v] + adv : OOB, lds + (wv * (64 / CPR) + KRP * v) * (ROWS * 2));
        }
      } else {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
          const bool o = cok && (full || k0 + kr0 + KRP * v < kend) && (unsigned)wih[v] < (unsigned)g.H &&
                         (unsigned)wiw[v] < (unsigned)g.W;
          bld16(rs, o ? (unsigned)wpo[v] : OOB, lds + (wv * (64 / CPR) + KRP * v) * (ROWS * 2));
        }
        wadvance(g);  // the K-tiles are issued in order: position the walk at k0 + BK
      }
    }
  }

  // 16x32 fragment (rows r0..r0+15, k = kk*32..+31) for MFMA lane l: the
  // per-lane byte offsets inside a stage image are loop-invariant, so the
  // kernel computes them once (frag_offsets) and the K loop only adds the
  // stage base (frag_at) -- the swizzle math used to cost ~10 VALU per MFMA.
  __device__ __forceinline__ void frag_offsets(int r0, int kk, int& o0, int& o1) const {
    const int l = threadIdx.x & 63;
    if constexpr (KOUT) {
      const int g = l >> 4, i = l & 15;
      const int q = i >> 2, pp = i & 3;
      const int col = r0 + 4 * pp;
      const int ch = col >> 3, within = (col & 7) * 2;
      const int kb0 = kk * 32 + 8 * g + q, kb1 = kb0 + 4;
      o0 = kb0 * (ROWS * 2) + kouter_swz<ROWS>(kb0, ch) * 16 + within;
      o1 = kb1 * (ROWS * 2) + kouter_swz<ROWS>(kb1, ch) * 16 + within;
    } else {
      const int row = r0 + (l & 15);
      const int ch = kk * 4 + (l >> 4);
      o0 = row * 128 + kmajor_swz(row, ch) * 16;
      o1 = 0;
    }
  }

  // The same fragment at a compile-time LDS offset OFF (stage base) from
  // byte address base + o.  KOUT: ds_read_b64_tr_b16 as inline asm -- the
  // builtin makes the compiler put s_waitcnt vmcnt(0) in front of it (it
  // cannot tell the read from the LDS-DMA still in flight into the OTHER
  // stage), which serialised every K-outer kernel's next-tile DMA with its
  // MFMAs.  The caller waits for the reads itself (lds_fence).
  template <int OFF>
  __device__ __forceinline__ bf16x8 frag_c(unsigned base, int o0, int o1) const {
    if constexpr (KOUT) {
      typedef short v4s __attribute__((ext_vector_type(4)));
      v4s x0, x1;
      if constexpr (OFF + 1024 * 1024 < 0) {
      } else if constexpr (OFF <= 65535 - 2048) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x0) : "v"(base + o0), "i"(OFF));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x1) : "v"(base + o1), "i"(OFF));
      } else {
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(x0) : "v"(base + OFF + o0));
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(x1) : "v"(base + OFF + o1));
      }
      i16x8 r;
      r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
      r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
      return __builtin_bit_cast(bf16x8, r);
    } else {
      return *(const bf16x8*)((const __attribute__((address_space(3))) char*)(size_t)base + OFF + o0);
    }
  }

  __device__ __forceinline__ bf16x8 frag_at(const char* lds, int o0, int o1) const {
    if constexpr (KOUT) {
      typedef short v4s __attribute__((ext_vector_type(4)));
      v4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + o0));
      v4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + o1));
      i16x8 r;
      r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
      r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
      return __builtin_bit_cast(bf16x8, r);
    } else {
      return *(const bf16x8*)(lds + o0);
    }
  }
};

// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] at [15:14]).  The
// builtin (not inline asm) keeps the compiler's own waitcnt bookkeeping exact.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
// Raw workgroup barrier: unlike __syncthreads() it does not drain the LDS-DMA
// still in flight (the fence of __syncthreads() makes the compiler emit
// vmcnt(0)); the empty asm statements keep the compiler from moving memory
// operations across it.
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}


// NTH threads = WM x WN waves, each owning a (BM/WM) x (BN/WN) block of 16x16
// MFMA tiles.  STAGES == 2: the v2 loop (one __syncthreads per K-tile, the
// next tile's DMA overlapping this tile's MFMAs, two workgroups per CU hide
// the rest).  STAGES >= 3 (the 8-wave big-tile variant, one workgroup per
// CU): a ring of STAGES LDS stages with STAGES-1 K-tiles in flight; each
// K-tile starts with a COUNTED vmcnt (this wave's DMA for the tile retired,
// the younger tiles still in flight) and a raw barrier (every wave's DMA
// retired, every wave done reading the stage about to be refilled).
// FLAGS bit 0: the fused-activation epilogue (sg_gemm_act) -- a separate
// instantiation, so every other kernel compiles exactly as without it
template <int BM, int BN, int AM, int BMODE, int OUT, int NTH = NT, int WM = 2, int WN = 2, int STAGES = 2,
          int FLAGS = 0>
__global__ void __launch_bounds__(NTH, STAGES == 1 ? 3 : (NTH == 512 && STAGES == 2 && BM * BN <= 128 * 128) ? 4 : 2)
    igemm_k(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;  // 16x16 MFMA tiles per wave
  static_assert(WM * WN * 64 == NTH, "wave grid");

  const int64_t yb = p.bh > 0 ? (int64_t)(blockIdx.y / p.bh) : (int64_t)blockIdx.y;
  const int64_t yh = p.bh > 0 ? (int64_t)(blockIdx.y % p.bh) : 0;
  const bf16* __restrict__ pa = p.a + yb * p.sa + yh * p.sa2;
  const bf16* __restrict__ pb = p.b + yb * p.sb + yh * p.sb2;
  char* pc = (char*)p.c + (yb * p.sc + yh * p.sc2) * (OUT == OUT_BF16 ? 2 : 4);
  // dgrad: phase from blockIdx.z (the output rows are that phase's pixels)
  const int phase = p.out_phase ? (int)blockIdx.z : 0;
  const Phase& P = p.g.phs[phase];
  const int M = p.out_phase ? p.g.N * P.Hp * P.Wp : p.M;
  const int K = p.out_phase ? P.nr * P.ns * p.g.K : p.K;

  // XCD-aware bijective remap, then bands of 8 tile-rows for L2 reuse of B
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  int split = blockIdx.z;
  if (bid >= nwg) return;
  if (OUT == OUT_F32_ATOMIC && p.xcd_split) {
    // split-K with splits % 8 == 0 (host-checked), gridDim.y == 1: workgroups
    // are dispatched round-robin over the 8 XCDs in linear-id order, so give
    // each XCD whole K-slices with ALL their tiles, tile index fastest: the
    // workgroups resident on one XCD then stream the same K window (pixels)
    // of both operands and share it through that XCD's L2, instead of every
    // XCD holding several K windows of a tile subset.
    const int L = blockIdx.x + (int)gridDim.x * (int)blockIdx.z;
    const int xcd = L & 7, loc = L >> 3;
    split = xcd * ((int)gridDim.z >> 3) + loc / nwg;
    bid = loc % nwg;
  } else if (nwg >= 8) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int band = 8;
  const int group = bid / (band * tiles_n);
  const int first_m = group * band;
  const int gm = min(tiles_m - first_m, band);
  const int tm = first_m + (bid % (band * tiles_n)) % gm;
  const int tn = (bid % (band * tiles_n)) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = p.out_phase ? 0 : split * p.k_per_split;
  const int kend = p.out_phase ? K : min(K, kbeg + p.k_per_split);
  if (OUT == OUT_F32_ATOMIC && kbeg >= kend) return;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  Loader<BM, AM, NTH> la;
  Loader<BN, BMODE, NTH> lb;
  la.init(p, m0, M, P, p.lda, pa, p.a_bytes);
  lb.init(p, n0, p.N, P, p.ldb, pb, p.b_bytes);
  lb.start(p, kbeg);

  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // loop-invariant fragment offsets (per lane) for every (tile, k-half)
  int oa0[TM][BK / 32], oa1[TM][BK / 32], ob0[TN][BK / 32], ob1[TN][BK / 32];
#pragma unroll
  for (int kk = 0; kk < BK / 32; ++kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i) la.frag_offsets(wm * WTM + i * 16, kk, oa0[i][kk], oa1[i][kk]);
#pragma unroll
    for (int j = 0; j < TN; ++j) lb.frag_offsets(wn * WTN + j * 16, kk, ob0[j][kk], ob1[j][kk]);
  }

  auto compute = [&](const char* sa) {
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = la.frag_at(sa, oa0[i][kk], oa1[i][kk]);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = lb.frag_at(sb, ob0[j][kk], ob1[j][kk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  // compile-time stage variant (the 2-stage loops): asm tr-reads + one
  // explicit LDS wait per k-half, tied to the fragments so the MFMAs stay after it
  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  auto compute_c = [&](auto stage) {
    constexpr int SA = decltype(stage)::value * STAGE;
    constexpr bool ANY_TR = Loader<BM, AM, NTH>::KOUT || Loader<BN, BMODE, NTH>::KOUT;
    static_assert(BK == 64, "two k-halves");
    auto half = [&](auto kkc) {
      constexpr int kk = decltype(kkc)::value;
      bf16x8 fa[TM], fb[TN];
      // K-outer images: k-half kk sits 32 k-rows further with the same
      // swizzle (it depends on k-row bits 0-3 only), so its offsets are the
      // kk = 0 ones plus an immediate -- 2 fewer VGPRs per fragment
      constexpr int KA = Loader<BM, AM, NTH>::KOUT ? 1 : 0, KB = Loader<BN, BMODE, NTH>::KOUT ? 1 : 0;
      constexpr int OA = SA + KA * kk_off<BM>(kk), OB = SA + A_BYTES + KB * kk_off<BN>(kk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = la.template frag_c<OA>(lds_base, oa0[i][KA ? 0 : kk], oa1[i][KA ? 0 : kk]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = lb.template frag_c<OB>(lds_base, ob0[j][KB ? 0 : kk], ob1[j][KB ? 0 : kk]);
      if constexpr (ANY_TR) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(fb[j]));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    };
    half(std::integral_constant<int, 0>{});
    half(std::integral_constant<int, 1>{});
  };

  if constexpr (STAGES == 1) {
    // single stage (the short-K variant: one or two K-tiles, four workgroups
    // per CU hide each other's load latency instead of double buffering)
    for (int kt = 0; kt < nk; ++kt) {
      if (kt > 0) __syncthreads();  // every wave done reading the stage
      la.issue(p, m0, M, kbeg + kt * BK, kend, P, smem);
      lb.issue(p, n0, p.N, kbeg + kt * BK, kend, P, smem + A_BYTES);
      __syncthreads();  // (drains this wave's DMA: vmcnt(0)) ... and every wave's
      compute_c(std::integral_constant<int, 0>{});
    }
  } else if (STAGES == 2 && p.early_issue) {
    // two barriers per K-tile: the DMA of tile kt+1 is issued as soon as
    // every wave has finished reading its stage (tile kt-1), BEFORE waiting
    // for tile kt -- two tiles in flight across that wait
    constexpr int LPT = Loader<BM, AM, NTH>::VPT + Loader<BN, BMODE, NTH>::VPT;
    // unrolled by two so the stage of every tile is a compile-time constant:
    // the fragment reads then carry it in their immediate offset (no per-tile
    // VALU re-basing of the loop-invariant fragment offsets)
    auto step = [&](auto stage, int kt) {
      constexpr int cur = decltype(stage)::value;
      if (kt > 0) raw_barrier();  // every wave done reading stage cur^1 (tile kt-1)
      char* nxt = smem + (cur ^ 1) * STAGE;
      const bool live = kt + 1 < nk;
      la.issue(p, m0, M, kbeg + (kt + 1) * BK, kend, P, nxt, live);
      lb.issue(p, n0, p.N, kbeg + (kt + 1) * BK, kend, P, nxt + A_BYTES, live);
      wait_vmcnt<LPT>();  // this wave's DMA for tile kt landed
      raw_barrier();      // ... every wave's
      compute_c(stage);
    };
    if (nk > 0) {
      la.issue(p, m0, M, kbeg, kend, P, smem);
      lb.issue(p, n0, p.N, kbeg, kend, P, smem + A_BYTES);
      for (int kt = 0; kt < nk; kt += 2) {
        step(std::integral_constant<int, 0>{}, kt);
        if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
      }
    }
  } else if constexpr (STAGES == 2) {
    auto step = [&](auto stage, int kt) {
      constexpr int cur = decltype(stage)::value;
      // this wave's DMA for tile kt retired (vmcnt(0)), then every wave's has,
      // and every wave finished reading the other stage (tile kt-1)
      __syncthreads();
      // next tile (a null-resource dummy after the last one: the DMA issue
      // stays in the MFMA block, so it interleaves with the MFMAs)
      char* nxt = smem + (cur ^ 1) * STAGE;
      const bool live = kt + 1 < nk;
      la.issue(p, m0, M, kbeg + (kt + 1) * BK, kend, P, nxt, live);
      lb.issue(p, n0, p.N, kbeg + (kt + 1) * BK, kend, P, nxt + A_BYTES, live);
      compute_c(stage);
    };
    if (nk > 0) {
      la.issue(p, m0, M, kbeg, kend, P, smem);
      lb.issue(p, n0, p.N, kbeg, kend, P, smem + A_BYTES);
      for (int kt = 0; kt < nk; kt += 2) {  // unrolled by two: compile-time stage offsets
        step(std::integral_constant<int, 0>{}, kt);
        if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
      }
    }
  } else {
    // LDS-DMA wave-instructions per K-tile (every thread issues all of them
    // unconditionally: out-of-range vectors read the zero-returning OOB
    // offset, tiles past the end go through a null resource), so the count
    // of in-flight tiles -- and the vmcnt -- is the same every iteration
    constexpr int LPT = Loader<BM, AM, NTH>::VPT + Loader<BN, BMODE, NTH>::VPT;
    constexpr int D = STAGES - 1;  // K-tiles in flight ahead of the one computed
    static_assert(D * LPT < 64, "vmcnt range");
#pragma unroll
    for (int s = 0; s < D; ++s) {
      la.issue(p, m0, M, kbeg + s * BK, kend, P, smem + s * STAGE, s < nk);
      lb.issue(p, n0, p.N, kbeg + s * BK, kend, P, smem + s * STAGE + A_BYTES, s < nk);
    }
    int cur = 0;   // stage of tile kt
    int fill = D;  // stage that tile kt + D goes to
    for (int kt = 0; kt < nk; ++kt) {
      wait_vmcnt<(D - 1) * LPT>();  // this wave's DMA for tile kt landed
      raw_barrier();                // ... every wave's; stage `fill` is no longer read
      char* st = smem + fill * STAGE;
      const bool live = kt + D < nk;
      la.issue(p, m0, M, kbeg + (kt + D) * BK, kend, P, st, live);
      lb.issue(p, n0, p.N, kbeg + (kt + D) * BK, kend, P, st + A_BYTES, live);
      compute(smem + cur * STAGE);
      cur = cur + 1 == STAGES ? 0 : cur + 1;
      fill = fill + 1 == STAGES ? 0 : fill + 1;
    }
  }
  wait_vmcnt<0>();  // the dummy DMA too, before the epilogue reuses the LDS
  wait_vmcnt<0>();  // the dummy DMA too, before the epilogue reuses the LDS
#include "igemm_epilogue.inc"
}

// ------------------------------------------------------------------------------
// Ping-pong 256 x 256 x 64 GEMM (K-major A [M][K] and B [N][K]), 512 threads.
//
// igemm_k's loop -- every wave loads fragments, waits at the barrier, runs its
// MFMAs, waits again -- leaves the MFMA pipe idle whenever all waves of a
// workgroup sit at the same barrier; its 128 x 128 tile tops out near 0.9 PF on
// large GEMMs (and a 256 x 256 tile in the same loop is no better).  Here the
// eight waves form two groups (wave row wr = 0 / 1, one wave of each group per
// SIMD) that run one barrier apart: while one group issues its LDS fragment
// reads and the next half-tile's LDS-DMA, the other group's MFMAs (at raised
// priority) own the SIMD, then they swap.  Each K-tile is 4 phases, one per
// 64 x 32 quadrant (mi, ni) of the wave's 128 x 64 output: (0,0) (0,1) (1,1)
// (1,0), 16 MFMAs each.
//
// LDS: 2 buffers x 4 half-tiles of 16 KB (A-h0, A-h1, B-h0, B-h1).  Half-tile
// A-h(mi) holds the 64 rows of quadrant row mi of BOTH wave rows, B-h(ni) the
// 32 columns of quadrant column ni of all four wave columns, so a half-tile is
// dead after the phase that reads it into registers and can be refilled with
// a later K-tile's while this K-tile's other quadrants still compute.  Each
// phase issues one half-tile and waits with a COUNTED vmcnt for the one the
// next phase reads, four half-tiles staying in flight (never vmcnt(0) in the
// loop; schedule below).  Measured (profiles/r3/gemm_ceiling_pp.jsonl,
// random bf16): 8192^3 1234 TF vs 1029 for igemm_k's best tile; +12..28 % on
// K = 2304..4608, +8 % at K = 2048; slower than igemm_k on short K (<= 1024),
// where the tile's prologue and epilogue dominate.
// ------------------------------------------------------------------------------
constexpr int PP_HALF = 128 * BK * 2;  // one half-tile image (16 KB)
constexpr int PP_BUF = 4 * PP_HALF;    // one K-tile (64 KB)

template <int OUT, int FLAGS = 0>
__global__ void __launch_bounds__(512, 2) pp_gemm_k(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = 256, BN = 256;
  const int64_t yb = p.bh > 0 ? (int64_t)(blockIdx.y / p.bh) : (int64_t)blockIdx.y;
  const int64_t yh = p.bh > 0 ? (int64_t)(blockIdx.y % p.bh) : 0;
  const bf16* __restrict__ pa = p.a + yb * p.sa + yh * p.sa2;
  const bf16* __restrict__ pb = p.b + yb * p.sb + yh * p.sb2;
  char* pc = (char*)p.c + (yb * p.sc + yh * p.sc2) * (OUT == OUT_BF16 ? 2 : 4);
  const Phase& P = p.g.phs[0];
  const int M = p.M, N = p.N, K = p.K;

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  if (bid >= nwg) return;
  if (nwg >= 8) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int band = 8;
  const int group = bid / (band * tiles_n);
  const int first_m = group * band;
  const int gm = min(tiles_m - first_m, band);
  const int tm = first_m + (bid % (band * tiles_n)) % gm;
  const int tn = (bid % (band * tiles_n)) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + BK - 1) / BK;

  const int t = threadIdx.x, l = t & 63;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wv >> 2, wc = wv & 3;

  // LDS-DMA sources: thread t fetches local rows rl and rl + 64 of a half-tile
  // image (one wave-instruction = 8 rows x 128 B), k-chunk (t & 7) ^ swz(row)
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(pa, p.a_bytes), rb = make_rsrc(pb, p.b_bytes);
  const int rl = t >> 3;
  const int lchunk = (t & 7) ^ ((rl >> 1) & 7);
  unsigned va[2][2], vb[2][2];  // [half][v] byte offsets (BIAS-ed past the extent when out of range)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int m = m0 + v * 128 + h * 64 + rl;
      va[h][v] = m < M ? (unsigned)(m * (int)p.lda + lchunk * 8) * 2u : BIAS;
      const int lr = rl + 64 * v;
      const int n = n0 + (lr >> 5) * 64 + h * 32 + (lr & 31);
      vb[h][v] = n < N ? (unsigned)(n * (int)p.ldb + lchunk * 8) * 2u : BIAS;
    }
  // half-tile q (0 A-h0, 1 B-h0, 2 B-h1, 3 A-h1) of K-tile kt into buffer kt & 1
  auto issue = [&](auto qc, int kt) {
    constexpr int q = decltype(qc)::value;
    constexpr bool isA = q == 0 || q == 3;
    constexpr int h = q == 0 ? 0 : q == 1 ? 0 : q == 2 ? 1 : 1;
    constexpr int slot = isA ? h : 2 + h;  // image position inside the buffer
    const int k0 = kt * BK;
    const bool live = kt < nk;
    const __amdgpu_buffer_rsrc_t rs = live ? (isA ? ra : rb) : make_rsrc(nullptr, 0);
    const bool kin = K - k0 >= BK || k0 + lchunk * 8 < K;
    char* dst = smem + (kt & 1) * PP_BUF + slot * PP_HALF + (8 * wv) * 128;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      unsigned off = kin ? (isA ? va[h][v] : vb[h][v]) + (unsigned)k0 * 2u : OOB;
      asm volatile("" : "+v"(off));  // materialise the select (else hipcc splits the load into two branches)
      bld16(rs, off, dst + 64 * v * 128);
    }
  };

  // fragment offsets inside a half-tile image (same layout for every image)
  int oa[4][2], ob[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int ch = kk * 4 + (l >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wr * 64 + i * 16 + (l & 15);
      oa[i][kk] = r * 128 + kmajor_swz(r, ch) * 16;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = wc * 32 + j * 16 + (l & 15);
      ob[j][kk] = r * 128 + kmajor_swz(r, ch) * 16;
    }
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];  // A of the current quadrant row; B of both quadrant columns
  typedef const __attribute__((address_space(3))) char* lds_cp;
  const lds_cp lbase = (lds_cp)(__attribute__((address_space(3))) char*)smem;

  // one phase: [fragment reads + DMA of half-tile Q of K-tile kt + KT +
  // counted wait] barrier [16 MFMAs of quadrant (MI, NI) at priority 1] barrier
  auto phase = [&](auto mic, auto nic, auto rac, auto rbc, auto qc, auto ktc, int kt) {
    constexpr int MI = decltype(mic)::value, NI = decltype(nic)::value;
    const lds_cp buf = lbase + (kt & 1) * PP_BUF;
    auto& fb = NI == 0 ? fb0 : fb1;
    if constexpr (decltype(rbc)::value) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fb[j][kk] = *(const bf16x8*)(buf + (2 + NI) * PP_HALF + ob[j][kk]);
    }
    if constexpr (decltype(rac)::value) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fa[i][kk] = *(const bf16x8*)(buf + MI * PP_HALF + oa[i][kk]);
    }
    issue(qc, kt + decltype(ktc)::value);
    wait_vmcnt<8>();  // four half-tiles stay in flight
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[MI * 4 + i][NI * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk], fa[i][kk], acc[MI * 4 + i][NI * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using T = std::true_type;
  using F = std::false_type;

  // Half-tile schedule (q: 0 A-h0, 1 B-h0, 2 B-h1, 3 A-h1).  Last reads of
  // K-tile t: A-h0, B-h0 in phase 1 (B-h0's fragments stay in registers for
  // phase 4), B-h1 in 2, A-h1 in 3.  Refills, each >= 2 phases after the read
  // of the image it overwrites (same buffer, K-tile t+2 or t+1):
  //   phase 1: B-h1(t+1)  2: A-h1(t+1)  3: A-h0(t+2)  4: B-h0(t+2)
  // so every half-tile is issued 5-6 phases before the phase that reads it
  // and every wait can leave the four youngest half-tiles in flight.
  if (nk > 0) {
    issue(I0{}, 0);
    issue(I1{}, 0);
    issue(I2{}, 0);
    issue(I3{}, 0);
    issue(I0{}, 1);
    issue(I1{}, 1);
    wait_vmcnt<8>();  // A-h0 and B-h0 of K-tile 0 (this wave's share)
    raw_barrier();    // ... every wave's
    if (wr == 1) __builtin_amdgcn_s_barrier();  // the second group runs one barrier behind
    for (int kt = 0; kt < nk; ++kt) {
      phase(I0{}, I0{}, T{}, T{}, I2{}, I1{}, kt);  // (0,0): reads A-h0, B-h0
      phase(I0{}, I1{}, F{}, T{}, I3{}, I1{}, kt);  // (0,1): reads B-h1
      phase(I1{}, I1{}, T{}, F{}, I0{}, I2{}, kt);  // (1,1): reads A-h1
      phase(I1{}, I0{}, F{}, F{}, I1{}, I2{}, kt);  // (1,0): registers only
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // rebalance the barrier count
  }
  wait_vmcnt<0>();  // the dummy DMA of K-tile nk too, before the epilogue reuses the LDS
  {
    constexpr int NTH = 512, STAGES = 2, WTM = 128, WTN = 64, TM = 8, TN = 4;
    const int wm = wr, wn = wc;
#include "igemm_epilogue.inc"
  }
}

// ------------------------------------------------------------------------------
// Persistent short-K GEMM for the 1x1-conv shapes (K <= 128, K-major A [M][K]
// and B [N][K], bf16 output): C[M][N] = A B^T (+ beta C), optional fused BN
// statistics.  igemm_k spends most of such a tile in its fixed parts (address
// setup, the first operand fetch, the epilogue and the per-tile statistics
// reduction: 7.2 VALU per MFMA, profiles/r3/pmc_gemm_200704x256x1024.txt).
// Here one workgroup per CU keeps its 128-column slice of B resident in LDS and
// walks the M-tiles tm = blockIdx.x, + gridDim.x, ...: the next tile's A is
// DMA'd into the other ring slot while this tile computes, the tile's output is
// staged as bf16 through LDS into 16-byte row stores whose completion overlaps
// the next tile's MFMAs, and the BN statistics stay in registers across all of
// the workgroup's tiles (one LDS reduction and one atomic per column at the end).
// Measured in round 3 (profiles/r3/sk_check.log, ab_persistent_short_k.jsonl):
// -5..+4 % per shape and neutral on the step, so it was opt-in; on the round-4
// step (native activation pool, persistent stem / stage-1 3x3 kernels, block
// pooling) the same switch is +2.0 % (profiles/r4/ab_sk_default.jsonl: 14.17k
// vs 13.90k img/s, three alternating rounds), so tuning knob 9 is on by default.
// ------------------------------------------------------------------------------
constexpr int SK_TILE = 128 * BK * 2;             // one 128-row K-tile image (16 KB)
constexpr int SK_LDT = 128 + 8;                   // bf16 staging row stride (+16 B)
constexpr int SK_STG = 128 * SK_LDT * 2;          // output staging image
constexpr int sk_lds(int kt) { return 3 * kt * SK_TILE + SK_STG; }

template <int KT>
__global__ void __launch_bounds__(256, 1) sk_gemm_k(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = 128, BN = 128, NTH = 256, WN = 2, WTM = 64, WTN = 64, TM = 4, TN = 4;
  char* sB = smem;
  char* sA = smem + KT * SK_TILE;
  bf16* sC = (bf16*)(smem + 3 * KT * SK_TILE);
  const int M = p.M, N = p.N, K = p.K;
  const int tiles_m = (M + BM - 1) / BM;
  const int n0 = blockIdx.y * BN;
  int tm = blockIdx.x;
  if (tm >= tiles_m) return;
  const Phase& P = p.g.phs[0];
  const int l = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;

  Loader<BM, LM_KMAJOR, NTH> la;
  Loader<BN, LM_KMAJOR, NTH> lb;
  lb.init(p, n0, N, P, p.ldb, p.b, p.b_bytes);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) lb.issue(p, n0, N, kt * BK, K, P, sB + kt * SK_TILE);
  la.init(p, tm * BM, M, P, p.lda, p.a, p.a_bytes);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) la.issue(p, tm * BM, M, kt * BK, K, P, sA + kt * SK_TILE);

  int oa0[TM][2], oa1[TM][2], ob0[TN][2], ob1[TN][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i) la.frag_offsets(wm * WTM + i * 16, kk, oa0[i][kk], oa1[i][kk]);
#pragma unroll
    for (int j = 0; j < TN; ++j) lb.frag_offsets(wn * WTN + j * 16, kk, ob0[j][kk], ob1[j][kk]);
  }

  // epilogue geometry: thread owns 8 columns (chunk ch) of rows r0 + 16 * pass
  constexpr int CPRW = BN / 8, RPP = NTH / CPRW, NPS = BM / RPP;
  const int ch = threadIdx.x % CPRW, r0 = threadIdx.x / CPRW;
  const int n = n0 + ch * 8;
  float st_s[8], st_q[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) { st_s[r] = 0.f; st_q[r] = 0.f; }

  // Pipeline (per thread, in issue order): ... DMA A(it) | stores(it-2) |
  // DMA A(it+1) | stores(it-1) ...; vector-memory operations retire in issue
  // order, so "A(it) landed" is a counted wait that leaves the two younger
  // tiles' stores and the next DMA in flight.  Every per-tile count is
  // uniform: out-of-range rows go through buffer stores / loads that the
  // resource drops, tiles past the end are DMA'd from a null resource.
  constexpr int D = KT * Loader<BM, LM_KMAJOR, NTH>::VPT;  // DMA instructions per tile
  const bool has_beta = p.beta != 0.f;
  const __amdgpu_buffer_rsrc_t rnull = make_rsrc(nullptr, 0);
  // the ring: A(it) lives in slot it & 1; the prologue issued A(0), A(1) follows
  {
    const int t1 = tm + (int)gridDim.x;
    const bool live = t1 < tiles_m;
    la.init(p, (live ? t1 : tm) * BM, M, P, p.lda, p.a, p.a_bytes);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) la.issue(p, t1 * BM, M, kt * BK, K, P, sA + (KT + kt) * SK_TILE, live);
  }
  for (int it = 0;; ++it) {
    const int buf = it & 1;
    if (it == 0) wait_vmcnt<D>();
    else if (it == 1) {
      if (has_beta) wait_vmcnt<2 * NPS + D>(); else wait_vmcnt<NPS + D>();
    } else {
      if (has_beta) wait_vmcnt<4 * NPS + D>(); else wait_vmcnt<2 * NPS + D>();
    }
    raw_barrier();  // A(it) landed for every wave; every wave is done with tile it-1
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const char* a_img = sA + (buf * KT + kt) * SK_TILE;
      const char* b_img = sB + kt * SK_TILE;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = la.frag_at(a_img, oa0[i][kk], oa1[i][kk]);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = lb.frag_at(b_img, ob0[j][kk], ob1[j][kk]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    }
    // acc -> bf16 staging
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * WTM + i * 16 + (l & 15);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn * WTN + j * 16 + (l >> 4) * 4;
        bf16x4 o;
        o[0] = (bf16)acc[i][j][0]; o[1] = (bf16)acc[i][j][1]; o[2] = (bf16)acc[i][j][2]; o[3] = (bf16)acc[i][j][3];
        *(bf16x4*)(sC + ml * SK_LDT + nl) = o;
      }
    }
    raw_barrier();  // staging complete; every wave is done reading A(it)'s slot
    // A(it+2) into the slot A(it) just left (null resource past the end)
    const int t2 = tm + 2 * (int)gridDim.x;
    {
      const bool live = t2 < tiles_m;
      la.init(p, (live ? t2 : tm) * BM, M, P, p.lda, p.a, p.a_bytes);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) la.issue(p, t2 * BM, M, kt * BK, K, P, sA + (buf * KT + kt) * SK_TILE, live);
    }
    // staging -> global: 16-byte buffer stores against this tile's row range
    const int m0 = tm * BM;
    const int rows = min(BM, M - m0);
    const __amdgpu_buffer_rsrc_t rc =
        n < N ? make_rsrc((const bf16*)p.c + (int64_t)m0 * p.ldc, (unsigned)((int64_t)rows * p.ldc * 2)) : rnull;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 old[NPS];
    if (has_beta) {
#pragma unroll
      for (int pass = 0; pass < NPS; ++pass)
        old[pass] = __builtin_amdgcn_raw_buffer_load_b128(rc, (unsigned)(((r0 + pass * RPP) * (int)p.ldc + n) * 2), 0, 0);
    }
#pragma unroll
    for (int pass = 0; pass < NPS; ++pass) {
      const int ml = r0 + pass * RPP;
      bf16x8 o = *(const bf16x8*)(sC + ml * SK_LDT + ch * 8);
      if (has_beta) {
        const bf16x8 ob = __builtin_bit_cast(bf16x8, old[pass]);
#pragma unroll
        for (int r = 0; r < 8; ++r) o[r] = (bf16)((float)o[r] + p.beta * (float)ob[r]);
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rc, (unsigned)((ml * (int)p.ldc + n) * 2),
                                             0, 0);
      if (p.stats && ml < rows) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float f = (float)o[r];
          st_s[r] += f;
          st_q[r] += f * f;
        }
      }
    }
    tm += (int)gridDim.x;
    if (tm >= tiles_m) break;
  }
  wait_vmcnt<0>();
  if (p.stats) {
    // once per workgroup: the RPP row-threads of each 8-column chunk through
    // LDS, then one atomic per column value into slot row blockIdx.x & 31
    __syncthreads();
    float* red = (float*)smem;  // [NTH][16]
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      red[threadIdx.x * 16 + r] = st_s[r];
      red[threadIdx.x * 16 + 8 + r] = st_q[r];
    }
    __syncthreads();
    if (threadIdx.x < CPRW * 16) {
      const int c = threadIdx.x >> 4, r = threadIdx.x & 15;
      const int nn = n0 + c * 8;
      if (nn < N) {
        float a = red[c * 16 + r];
        for (int k = 1; k < RPP; ++k) a += red[(k * CPRW + c) * 16 + r];
        const int col = r < 8 ? nn + r : N + nn + (r - 8);
        atomicAdd(p.stats + (int64_t)(blockIdx.x & 31) * 2 * N + col, a);
      }
    }
  }
}

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
// (8: measured +0.3..0.6 % over 4 and 2 on the ResNet-50 step, profiles/r3/ab_short_k_threshold.jsonl)
// (0 = off), 7 = early DMA issue in the 2-stage loop (measured -3.5 % conv time)
// 8 = non-temporal output stores in the LDS-staged bf16 epilogue, 9 = persistent
// short-K kernel for the 1x1-conv GEMM shapes (sk_gemm_k)
// key 10: workgroup target of the 8-wave split-K weight gradient (0: 1024 with taps, 512 for 1x1)
// key 11: 1 = strided data gradients never take the single-stage short-K kernel (A/B)
static int g_tune[12] = {5, 1, 1, 0, 0, 1, 8, 1, 0, 1, 0, 0};
// one-shot: the next dgrad's wt scratch is already transposed.  Per OS
// thread: the runtime's executor threads (hogwild / aggregated replicas)
// each set and consume their own flag, so one thread's set can never be
// taken by another thread's dgrad
static thread_local int g_wt_ready = 0;
// one-shot (per OS thread): the next dgrad adds this masked residual gradient
static thread_local const bf16* g_res_g = nullptr;
static thread_local const uint8_t* g_res_mask = nullptr;

constexpr int stages_c(int BM, int BN, int STAGES) { return STAGES * (BM + BN) * BK * 2; }

template <int BM, int BN, int AM, int BMODE, int OUT, int NTH = NT, int WM = 2, int WN = 2, int STAGES = 2,
          int FLAGS = 0>
static void launch_t(const GemmArgs& p_in, int tiles, int ydim, int zdim, hipStream_t s) {
  GemmArgs p = p_in;
  p.lds_epilogue = g_tune[1];
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
  p.nt_store = g_tune[8];
  constexpr int lds = 2 * PP_BUF;
  auto* kern = pp_gemm_k<OUT, FLAGS>;
  static bool attr = [kern] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(tiles, ydim, 1), dim3(512), lds, s, p);
}

// persistent short-K launch: one workgroup per CU, gridDim.x a multiple of 8
// (the workgroups of every column slice that share an M-tile sit on one XCD)
template <int KT>
static void launch_sk(const GemmArgs& p, int tiles_m, int tiles_n, hipStream_t s) {
  constexpr int lds = sk_lds(KT);
  auto* kern = sk_gemm_k<KT>;
  static bool attr = [kern] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  (void)attr;
  int g = (256 + tiles_n - 1) / tiles_n;
  g = (g + 7) / 8 * 8;
  if (g > tiles_m) g = tiles_m;
  hipLaunchKernelGGL(kern, dim3(g, tiles_n, 1), dim3(256), lds, s, p);
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
  if (BM == 128 && BN == 128) launch_t<128, 128, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
  else if (BM == 128 && BN == 64) launch_t<128, 64, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
  else if (BM == 64 && BN == 128) launch_t<64, 128, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
  else launch_t<64, 64, AM, BMODE, OUT, NT, 2, 2, 2, FLAGS>(p, tiles, batch, z, s);
}

static int pick_splits(int M, int N, int K, int want) {
  if (want > 0) return want;
  int BM, BN;
  pick_tile(M, N, BM, BN);
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = 1;
  const int nkt = (K + BK - 1) / BK;
  while (tiles * splits < 768 && splits * 2 <= nkt / 4) splits *= 2;
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
// aux when given, or act_bwd: out *= act'(act_x).  Returns 0 (nothing
// launched) when the shape cannot take the staged epilogue.
int sg_gemm_act(const void* a, int64_t lda, int a_kouter, const void* b, int64_t ldb, int b_kouter, void* c,
                int64_t ldc, int M, int N, int K, float alpha, const void* bias, int batch, int64_t sa, int64_t sb,
                int64_t sc, int act, void* aux, int act_bwd, const void* act_x, hipStream_t s) {
  if ((N & 7) != 0 || (ldc & 7) != 0 || !g_tune[1] || g_tune[4] != 0 || (act == 0) == (act_x == nullptr) ||
      M <= 0 || K <= 0 || batch != 1)
    return 0;
  GemmArgs p{};
  init_phase_identity(p.g);
  p.sa = sa; p.sb = sb; p.sc = sc;
  p.M = M; p.N = N; p.K = K; p.a = (const bf16*)a; p.lda = lda; p.b = (const bf16*)b; p.ldb = ldb;
  p.c = c; p.ldc = ldc; p.alpha = alpha; p.beta = 0.f; p.bias = (const float*)bias; p.relu = 0;
  p.act = act; p.aux = (bf16*)aux; p.act_x = (const bf16*)act_x; p.act_bwd = act_bwd;
  p.k_per_split = kps(K, 1);
  p.a_bytes = extent_bytes(a_kouter ? (int64_t)(K - 1) * lda + M : (int64_t)(M - 1) * lda + K);
  p.b_bytes = extent_bytes(b_kouter ? (int64_t)(K - 1) * ldb + N : (int64_t)(N - 1) * ldb + K);
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
  GemmArgs p{};
  p.res_g = g_res_g;  // one-shot residual-gradient source (sg_conv_dgrad_res)
  p.res_mask = g_res_mask;
  g_res_g = nullptr;
  g_res_mask = nullptr;
  if (bn_ws && out_mode == OUT_BF16 && (beta == 0.f || bn_mask) && (C & 7) == 0 && g_tune[1] &&
      !sg_bn_deterministic()) {
    p.stats = (float*)bn_ws;
    p.stats_mode = bn_mask ? (bn_x ? 2 : 3) : 1;
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
  if (key >= 0 && key < 12) g_tune[key] = value;
}

}  // extern "C"

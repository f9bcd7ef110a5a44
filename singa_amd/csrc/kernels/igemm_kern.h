// Device side of the MFMA implicit-GEMM kernel family (igemm.hip): operand
// loaders, igemm_k, pp_gemm_k, sk_gemm_k and helpers.  A header so other
// translation units (bnres.hip) can instantiate the same kernels for their
// own operand modes in parallel with igemm.hip's build.
#pragma once
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
  // two-source A operands (GemmArgs::a2): the algebraic residual-BN backward
  // (bnres.hip) runs GEMMs over [g | y] without materialising the concatenation
  LM_KMAJOR2 = 7,  // [rows][K]: k < a2_split from a (lda), k >= a2_split from a2 (lda2), K-tiles never straddle
  LM_KOUTER2 = 8,  // [K][rows]: rows < a2_split from a (lda), rows >= a2_split from a2 (lda2), tiles never straddle
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
  int epi_fence;       // 1: the staged epilogue's barriers after output stores are __syncthreads (knob 19 A/B)
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
  // stats_mode 5 (gemm_act only): stats is an fp32 [N] vector += the column
  // sums of the bf16 output (atomics; the staged epilogue of igemm_k / pp_gemm_k)
  int stats_mode;
  // residual-gradient accumulate (bf16 LDS-staged epilogue, beta == 0, no
  // stats): out += res_g * bit(res_mask) -- the gradient a residual
  // BN(+ReLU) passes to its shortcut input is its masked output gradient;
  // the consuming conv's dgrad adds it from (dy, 1-bit mask) directly, so
  // the BN backward never writes it as a tensor
  const bf16* res_g;
  const uint8_t* res_mask;
  // res_s > 1: res_g is COMPACT -- the gradient of a strided 1x1 shortcut's
  // input, [N][Ho][Wo][C] at every res_s-th pixel of this output's H x W grid
  // (rows = pixels, 1x1 stride-1 data gradient); the other pixels add nothing
  int res_s, res_H, res_W, res_Ho, res_Wo;
  FastDiv res_dW, res_dH;
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
  // persistent kernels (sk_gemm_k): dynamic work-queue slot (common.h), one
  // counter per (column slice, XCD); nullptr = static blockIdx partition
  int* wq;
  // two-source A (LM_KMAJOR2 / LM_KOUTER2): the second source and where it starts
  const bf16* a2;
  int64_t lda2;
  unsigned a2_bytes;
  int a2_split;
  // sk_gemm_k<KT, 1> (a fused residual tail's recomputed forward): the output
  // is relu(bf16(acc) * ep_scale[n] + ep_shift[n] + ep_res) and its ReLU mask
  // bits ep_mask [M][N / 8] -- the conv output itself is never stored
  const float* ep_scale;
  const float* ep_shift;
  const bf16* ep_res;
  uint8_t* ep_mask;
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

// 8-wide forms of the fused activations, NOT inlined: the staged epilogue's
// unrolled passes would otherwise carry 32 inlined copies of every
// activation's math (erf, exp, tanh), and that code growth made the fused
// kernels slow whatever the activation (tools/bench_actgrad.py: relu ~ gelu)
struct F8 {
  float x[8];
};
__device__ __attribute__((noinline)) bf16x8 ep_act8(int a, bf16x8 z) {
  bf16x8 o;
#pragma unroll
  for (int r = 0; r < 8; ++r) o[r] = (bf16)ep_act(a, (float)z[r]);
  return o;
}
__device__ __attribute__((noinline)) bf16x8 ep_dact8(int a, F8 v, bf16x8 t) {
  bf16x8 o;
#pragma unroll
  for (int r = 0; r < 8; ++r) o[r] = (bf16)((float)(bf16)v.x[r] * ep_dact(a, (float)t[r]));
  return o;
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
  static constexpr bool KOUT = (MODE == LM_KOUTER || MODE == LM_WGRAD_B || MODE == LM_DGRAD_B || MODE == LM_KOUTER2);
  static constexpr int CPR = ROWS / 8;   // KOUTER: chunks per k-row
  static constexpr int KRP = NTH / CPR;  // KOUTER: k-rows per pass
  static constexpr int RPV = NTH / 8;    // KMAJOR: rows per pass
  static_assert(VPT >= 1 && CPR <= 64, "tile too small for the thread count");
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned voff[VPT];  // per-lane byte offsets (BIAS-ed when masked); see issue()
  __amdgpu_buffer_rsrc_t rsrc2;  // LM_KMAJOR2: the second source (k >= ksplit)
  unsigned voff2[VPT];
  int ksplit;
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
    if constexpr (MODE == LM_KMAJOR2) {
      rsrc2 = make_rsrc(p.a2, p.a2_bytes);
      ksplit = p.a2_split;
    }
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
        } else if constexpr (MODE == LM_KMAJOR2) {
          voff[v] = ok[v] ? (unsigned)(rr * (int)ld + lchunk * 8) * 2u : BIAS;
          voff2[v] = ok[v] ? (unsigned)(rr * (int)p.lda2 + lchunk * 8) * 2u : BIAS;
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
      } else if constexpr (MODE == LM_KOUTER2) {
        // the whole tile comes from one source (row0 is tile-uniform, the split tile-aligned)
        const bool second = row0 >= p.a2_split;
        if (second) {
          rsrc = make_rsrc(p.a2, p.a2_bytes);
          ld = p.lda2;
        }
        const int colx = second ? col - p.a2_split : col;
        const bool ok2 = cok && (second || col < p.a2_split);
#pragma unroll
        for (int v = 0; v < VPT; ++v) voff[v] = ok2 ? (unsigned)((kr0 + KRP * v) * (int)ld + colx) * 2u : BIAS;
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
    } else if constexpr (MODE == LM_KMAJOR2) {
      // K-tile from the first or the second source (k0 is wave-uniform)
      const bool kin = full || (k0 + lchunk * 8 < kend);
      if (k0 >= ksplit) {
        const __amdgpu_buffer_rsrc_t rs2 = live ? rsrc2 : make_rsrc(nullptr, 0);
        const unsigned adv = (unsigned)(k0 - ksplit) * 2u;
#pragma unroll
        for (int v = 0; v < VPT; ++v) bld16(rs2, kin ? voff2[v] + adv : OOB, lds + (8 * wv + RPV * v) * 128);
      } else {
#pragma unroll
        for (int v = 0; v < VPT; ++v)
          bld16(rs, kin ? voff[v] + (unsigned)k0 * 2u : OOB, lds + (8 * wv + RPV * v) * 128);
      }
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
    } else if constexpr (MODE == LM_KOUTER || MODE == LM_KOUTER2) {
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
// Barrier ordering LDS accesses only (this wave's LDS operations complete,
// then the raw barrier): an epilogue barrier after global stores.  With
// __syncthreads() the compiler emits s_waitcnt vmcnt(0) first, so every wave
// of the workgroup would wait for its output stores to land before the BN
// statistics reduction (fence = 1: that behaviour, tuning knob 19 for A/B).
__device__ __forceinline__ void lds_barrier(int fence) {
  if (fence) {
    __syncthreads();
  } else {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    raw_barrier();
  }
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
  } else if constexpr (STAGES == 3) {
    // Three-stage ring with compile-time stages.  4 waves: for SHORT workgroups (BERT-sized GEMMs: a few
    // hundred tiles of 12-48 K-tiles, 1-2 workgroups per CU): two K-tiles in
    // flight while the third multiplies.  The 2-stage loops keep one in
    // flight, and a 64-wide K-tile is only ~250 MFMA cycles per wave, so their
    // K loop ran at the DMA latency.  8 waves (the 256 x 128 tile of 64 x 64
    // wave tiles, one workgroup per CU): the weight-gradient variant of knob 15.
    // Unrolled by three: every stage offset is
    // a compile-time constant (the fragment reads carry it as an immediate and
    // the compiler can tell them from the DMA into the other stages).
    constexpr int LPT = Loader<BM, AM, NTH>::VPT + Loader<BN, BMODE, NTH>::VPT;
    static_assert(LPT < 64, "vmcnt range");
    auto step = [&](auto stage, int kt) {
      constexpr int cur = decltype(stage)::value;
      constexpr int fill = (cur + 2) % 3;
      wait_vmcnt<LPT>();  // this wave's DMA for tile kt landed (tile kt+1 may still fly)
      raw_barrier();      // ... every wave's; every wave done reading stage `fill` (tile kt-1)
      const bool live = kt + 2 < nk;
      la.issue(p, m0, M, kbeg + (kt + 2) * BK, kend, P, smem + fill * STAGE, live);
      lb.issue(p, n0, p.N, kbeg + (kt + 2) * BK, kend, P, smem + fill * STAGE + A_BYTES, live);
      compute_c(stage);
    };
    if (nk > 0) {
      la.issue(p, m0, M, kbeg, kend, P, smem);
      lb.issue(p, n0, p.N, kbeg, kend, P, smem + A_BYTES);
      la.issue(p, m0, M, kbeg + BK, kend, P, smem + STAGE, nk > 1);
      lb.issue(p, n0, p.N, kbeg + BK, kend, P, smem + STAGE + A_BYTES, nk > 1);
      for (int kt = 0; kt < nk; kt += 3) {
        step(std::integral_constant<int, 0>{}, kt);
        if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
        if (kt + 2 < nk) step(std::integral_constant<int, 2>{}, kt + 2);
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

// EPI 0: C = A B^T (+ beta C), optional BN statistics; with p.c == nullptr
//        only the statistics (the stores go to a null resource: the first
//        pass of a recomputed fused tail).
// EPI 1: the fused residual tail's second pass: out = relu(bf16(A B^T) *
//        scale + shift + res) and its ReLU mask bits (GemmArgs::ep_*).
// EPI 2: a 1x1 conv's data gradient completing a fused tail's output
//        gradient: out = bf16(bf16(A B^T) + res) * bit(ep_mask) (res: the other
//        consumers' gradient, or none) and its column sums into p.stats
//        (stats_mode 4 of the generic kernels: the tail's g~ and sum g~).
// AM: LM_KMAJOR, or LM_KMAJOR2 -- A from two sources split at p.a2_split
// (a multiple of 64): the two-branch tail [y | x] . [W3' | Wd']^T
template <int KT, int EPI = 0, int AM = LM_KMAJOR>
__global__ void __launch_bounds__(256, 1) sk_gemm_k(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = 128, BN = 128, NTH = 256, WN = 2, WTM = 64, WTN = 64, TM = 4, TN = 4;
  char* sB = smem;
  char* sA = smem + KT * SK_TILE;
  bf16* sC = (bf16*)(smem + 3 * KT * SK_TILE);
  int* sQ = (int*)(smem + sk_lds(KT) - 16);  // ticket broadcast (the staging image leaves its last 16 B unused)
  const int M = p.M, N = p.N, K = p.K;
  const int tiles_m = (M + BM - 1) / BM;
  const int n0 = blockIdx.y * BN;
  // this workgroup's M-tiles.  Workgroups are dispatched round-robin over
  // the 8 XCDs, so bx & 7 is this workgroup's XCD (gridDim.x % 8 == 0, and
  // every column slice's workgroup bx sits on the same XCD): the M-tiles
  // m = xcd + 8 i belong to that XCD, where every column slice reads the same
  // A tiles through one L2.  Local index j = bx >> 3 of G8 = G / 8 per XCD:
  // i = j, j + G8, j + 2 G8, then (with a queue, one counter per (slice,
  // XCD)) i = 3 G8 + ticket, tickets taken three tiles ahead; (without)
  // i = j + k G8 -- the static partition.  Increasing per workgroup.
  const int G = (int)gridDim.x, G8 = G >> 3, xcd = blockIdx.x & 7;
  const int qid = blockIdx.y * 8 + xcd;
  int tm = xcd + 8 * (blockIdx.x >> 3);
  int t1 = tm + 8 * G8, t2 = tm + 16 * G8;
  const Phase& P = p.g.phs[0];
  const int l = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  if (tm >= tiles_m) {
    if (p.wq && threadIdx.x == 0) wq_done(p.wq, 8 * (int)gridDim.y);
    return;
  }
  // EPI 1: this thread's 8 columns of the BN affine, loaded (and waited
  // for) before the first DMA so no wait for them lands inside the loop
  float esc[8], esf[8];
  if constexpr (EPI == 1) {
    const int nn = n0 + (threadIdx.x % (BN / 8)) * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      esc[r] = p.ep_scale[nn + r];
      esf[r] = p.ep_shift[nn + r];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) asm volatile("" ::"v"(esc[r]), "v"(esf[r]));
  }

  Loader<BM, AM, NTH> la;
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

  // Pipeline (per wave, in issue order): ... Q(it-1) | DMA A(it+1) |
  // [loads(it-1)] stores(it-1) | Q(it) | DMA A(it+2) | ...; vector-memory
  // operations retire in issue order, so "A(it) landed" is a counted wait that
  // leaves the younger tiles' stores, the queue op and the next DMA in flight.
  // Q(it) is ONE vector-memory op per wave: wave 0 takes the ticket of tile
  // it+3 (lane 0, agent-scope atomic), the other waves store to a null
  // resource (dropped) -- every wave's count stays uniform.  Every per-tile
  // count is uniform: out-of-range rows go through buffer stores / loads that
  // the resource drops, tiles past the end are DMA'd from a null resource.
  constexpr int D = KT * Loader<BM, AM, NTH>::VPT;  // DMA instructions per tile
  const bool has_beta = p.beta != 0.f;
  const __amdgpu_buffer_rsrc_t rnull = make_rsrc(nullptr, 0);
  int ticket = 0;  // wave 0 lane 0: the last queue op's result
  auto queue_op = [&]() {
    if (wid == 0 && p.wq) {
      if (l == 0) ticket = wq_take(p.wq, qid);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(0u, rnull, 0u, 0, 0);
    }
  };
  // the ring: A(it) lives in slot it & 1; the prologue issued A(0), A(1) follows
  {
    const bool live = t1 < tiles_m;
    la.init(p, (live ? t1 : tm) * BM, M, P, p.lda, p.a, p.a_bytes);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) la.issue(p, t1 * BM, M, kt * BK, K, P, sA + (KT + kt) * SK_TILE, live);
  }
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  // EPI 1: the residual rows of the NEXT tile, loaded one tile ahead (right
  // after this tile's stores) so their latency hides behind a tile of work;
  // ldc == N, host-checked -- residual and output share the row stride
  u32x4 rres[NPS];
  unsigned mres[NPS];  // EPI 2: the next tile's mask bytes, prefetched with its residual
  auto load_res = [&](int t) {
    const int mt = t < tiles_m ? t : 0;
    const int trows = min(BM, M - mt * BM);
    const __amdgpu_buffer_rsrc_t rr =  // (no residual: loads of zeros, the count stays uniform)
        t < tiles_m && p.ep_res
            ? make_rsrc(p.ep_res + (int64_t)mt * BM * p.ldc, (unsigned)((int64_t)trows * p.ldc * 2))
            : rnull;
#pragma unroll
    for (int pass = 0; pass < NPS; ++pass)
      rres[pass] = __builtin_amdgcn_raw_buffer_load_b128(rr, (unsigned)(((r0 + pass * RPP) * (int)p.ldc + n) * 2), 0, 0);
    if constexpr (EPI == 2) {
      const __amdgpu_buffer_rsrc_t rm =
          t < tiles_m ? make_rsrc(p.ep_mask + (int64_t)mt * BM * (N >> 3), (unsigned)(trows * (N >> 3))) : rnull;
#pragma unroll
      for (int pass = 0; pass < NPS; ++pass)
        mres[pass] = __builtin_amdgcn_raw_buffer_load_b8(rm, (unsigned)((r0 + pass * RPP) * (N >> 3) + (n >> 3)), 0, 0);
    }
  };
  if constexpr (EPI >= 1) load_res(tm);
  for (int it = 0;; ++it) {
    const int buf = it & 1;
    // A(it) landed (younger: [loads] stores(it-2), Q(it-1), A(it+1), [loads] stores(it-1);
    // it == 1: Q(0), A(2), [loads] stores(0))
    // (per-tile epilogue ops E: NPS stores, + NPS loads with beta; EPI 1: NPS
    // output stores, NPS mask-byte stores and the next tile's NPS residual
    // loads -- after the prologue's residual loads (NPS) of tile 0)
    // (EPI 2: NPS output stores, then the next tile's NPS residual and NPS
    // mask-byte loads -- after the prologue's 2 NPS loads of tile 0)
    if (it == 0) {
      if constexpr (EPI == 1) wait_vmcnt<NPS + D>();
      else if constexpr (EPI == 2) wait_vmcnt<2 * NPS + D>();
      else wait_vmcnt<D>();
    } else if (it == 1) {
      if constexpr (EPI == 1) wait_vmcnt<4 * NPS + D + 1>();
      else if constexpr (EPI == 2) wait_vmcnt<5 * NPS + D + 1>();
      else if (has_beta) wait_vmcnt<2 * NPS + D + 1>(); else wait_vmcnt<NPS + D + 1>();
    } else {
      if constexpr (EPI >= 1) wait_vmcnt<6 * NPS + D + 1>();
      else if (has_beta) wait_vmcnt<4 * NPS + D + 1>(); else wait_vmcnt<2 * NPS + D + 1>();
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
    if (it > 0 && wid == 0 && l == 0) {
      // Q(it-1) (the ticket of tile it+2) retired: younger are A(it+1) and [loads] stores(it-1)
      if constexpr (EPI >= 1) wait_vmcnt<3 * NPS + D>();
      else if (has_beta) wait_vmcnt<2 * NPS + D>(); else wait_vmcnt<NPS + D>();
      *sQ =p.wq ? xcd + 8 * (3 * G8 + ticket) : tm + 16 * G8;
    }
    // this wave's LDS writes (staging, ticket) complete before the barrier: a
    // raw s_barrier does not wait for them, and a ds_write issued just before
    // it can still be in flight when another wave's ds_read after it runs
    // (the ticket written last was read stale now and then: waves then
    // disagreed on the next tile -- tests/test_workq_gpu.py stress test)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt / expcnt untouched
    raw_barrier();  // staging complete; every wave is done reading A(it)'s slot; the ticket is in
    if (it > 0) t2 = __builtin_amdgcn_readfirstlane(*sQ);  // (wave-uniform: scalar tile math below)
    // A(it+2) into the slot A(it) just left (null resource past the end)
    queue_op();  // Q(it): the ticket of tile it+3
    {
      const bool live = t2 < tiles_m;
      la.init(p, (live ? t2 : tm) * BM, M, P, p.lda, p.a, p.a_bytes);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) la.issue(p, t2 * BM, M, kt * BK, K, P, sA + (buf * KT + kt) * SK_TILE, live);
    }
    // staging -> global: 16-byte buffer stores against this tile's row range
    const int m0 = tm * BM;
    const int rows = min(BM, M - m0);
    // (N % 128 == 0, host-checked: every column chunk is in range, and the
    // resource stays wave-uniform -- no waterfall loop around the stores)
    const __amdgpu_buffer_rsrc_t rc =
        p.c ? make_rsrc((const bf16*)p.c + (int64_t)m0 * p.ldc, (unsigned)((int64_t)rows * p.ldc * 2)) : rnull;
    u32x4 old[NPS];
    if constexpr (EPI == 1) {
      const __amdgpu_buffer_rsrc_t rmk = make_rsrc(p.ep_mask + (int64_t)m0 * (N >> 3), (unsigned)(rows * (N >> 3)));
#pragma unroll
      for (int pass = 0; pass < NPS; ++pass) {
        const int ml = r0 + pass * RPP;
        bf16x8 o = *(const bf16x8*)(sC + ml * SK_LDT + ch * 8);
        const bf16x8 rb = __builtin_bit_cast(bf16x8, rres[pass]);
        unsigned b = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          // the unfused path's arithmetic: the bf16 conv output, BN affine, + residual, ReLU
          o[r] = (bf16)fmaxf((float)o[r] * esc[r] + esf[r] + (float)rb[r], 0.f);
          b |= ((float)o[r] > 0.f ? 1u : 0u) << r;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rc, (unsigned)((ml * (int)p.ldc + n) * 2),
                                               0, 0);
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)b, rmk, (unsigned)(ml * (N >> 3) + (n >> 3)), 0, 0);
      }
      load_res(t1);  // the next tile's residual (null resource past the end)
    } else if constexpr (EPI == 2) {
#pragma unroll
      for (int pass = 0; pass < NPS; ++pass) {
        const int ml = r0 + pass * RPP;
        bf16x8 o = *(const bf16x8*)(sC + ml * SK_LDT + ch * 8);
        const bf16x8 rb = __builtin_bit_cast(bf16x8, rres[pass]);
#pragma unroll
        for (int r = 0; r < 8; ++r)
          o[r] = ((mres[pass] >> r) & 1u) != 0 ? (bf16)((float)o[r] + (float)rb[r]) : (bf16)0.f;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rc, (unsigned)((ml * (int)p.ldc + n) * 2),
                                               0, 0);
        if (ml < rows) {
#pragma unroll
          for (int r = 0; r < 8; ++r) st_s[r] += (float)o[r];
        }
      }
      load_res(t1);
    } else {
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
    }
    tm = t1;
    t1 = t2;
    if (tm >= tiles_m) break;
  }
  wait_vmcnt<0>();
  if (p.wq && threadIdx.x == 0) wq_done(p.wq, 8 * (int)gridDim.y);  // every ticket of this workgroup is taken
  if (EPI != 1 && p.stats) {
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

// ------------------------------------------------------------------------------
// Persistent streaming GEMM for the memory-bound 1x1-conv shapes with longer K
// (K = 256 .. 2048 in 64-wide K-tiles, K-major A [M][K] and B [N][K], bf16
// output, optional fused BN statistics).  igemm_k's two workgroups per CU keep
// ONE K-tile in flight each and stop streaming at every tile's prologue and
// epilogue: the wide-N shapes (N = 512 .. 2048, two thirds of their bytes are
// output) ran at 1.3-2.3 TB/s (tools/bench_1x1.py, tools/gemm_shapes.py).  The
// sk_gemm_k design (one workgroup per CU walking the M-tiles of one 128-column
// slice, M-tiles from per-(slice, XCD) work queues, statistics in registers,
// the tile staged through LDS into 16-byte stores that retire behind the next
// tile's work) cannot keep B resident at these K, so here A and B both stream
// through a three-stage ring of K-tiles that runs CONTINUOUSLY across tiles:
// the DMA of the next tile's first two K-tiles is in flight while this tile
// finishes and writes its output.  Every wave issues the same vector-memory
// ops per K-tile (DMA; past the last tile from a null resource) and per tile
// (its stores and one queue op), so each K-tile's wait is a counted vmcnt.
// ------------------------------------------------------------------------------
constexpr int ST_STAGE = 2 * SK_TILE;                    // A and B K-tile images (32 KB)

// wq_take without the wait: through the builtin, the atomic optimizer turns
// the one-lane atomic into a wave scan that needs the returned value at once
// (s_waitcnt vmcnt(0) right after it -- wave 0 would drain every DMA in flight
// once per tile).  The result is read only after an explicit counted wait
// that retires this op (st_gemm_k's wait before the ticket broadcast).
__device__ __forceinline__ int wq_take_nowait(int* slot, int q) {
  int v;
  int* addr = slot + q * QSTRIDE;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(v) : "v"(addr), "v"(1) : "memory");
  return v;
}
constexpr int ST_LDS = 3 * ST_STAGE + SK_STG;             // ring + output staging (130 KB)

template <int EPI = 0>
__global__ void __launch_bounds__(256, 1) st_gemm_k(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = 128, BN = 128, NTH = 256, WN = 2, WTM = 64, WTN = 64, TM = 4, TN = 4;
  static_assert(EPI == 0, "plain output with optional BN statistics");
  bf16* sC = (bf16*)(smem + 3 * ST_STAGE);
  int* sQ = (int*)(smem + ST_LDS - 16);  // ticket broadcast (the staging image leaves its last 16 B unused)
  const int M = p.M, N = p.N, K = p.K;
  const int KT = K / BK;  // >= 2, host-checked (K % 64 == 0)
  const int tiles_m = (M + BM - 1) / BM;
  const int n0 = blockIdx.y * BN;
  // tiles as sk_gemm_k: XCD xcd = bx & 7 owns M-tiles m = xcd + 8 i; this
  // workgroup's i = j, j + G8, j + 2 G8, then 3 G8 + ticket (queue) or j + k G8
  const int G = (int)gridDim.x, G8 = G >> 3, xcd = blockIdx.x & 7;
  const int qid = blockIdx.y * 8 + xcd;
  int tm = xcd + 8 * (blockIdx.x >> 3);
  int t1 = tm + 8 * G8, t2 = tm + 16 * G8;
  const Phase& P = p.g.phs[0];
  const int l = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  if (tm >= tiles_m) {
    if (p.wq && threadIdx.x == 0) wq_done(p.wq, 8 * (int)gridDim.y);
    return;
  }
  Loader<BM, LM_KMAJOR, NTH> la, la1;  // this tile's A loader and the next tile's
  Loader<BN, LM_KMAJOR, NTH> lb;
  lb.init(p, n0, N, P, p.ldb, p.b, p.b_bytes);
  la.init(p, tm * BM, M, P, p.lda, p.a, p.a_bytes);
  la1.init(p, (t1 < tiles_m ? t1 : tm) * BM, M, P, p.lda, p.a, p.a_bytes);
  constexpr int LPT = Loader<BM, LM_KMAJOR, NTH>::VPT + Loader<BN, LM_KMAJOR, NTH>::VPT;  // DMA ops per K-tile
  // epilogue geometry: thread owns 8 columns (chunk ch) of rows r0 + RPP * pass
  constexpr int CPRW = BN / 8, RPP = NTH / CPRW, NPS = BM / RPP;
  constexpr int E_OPS = NPS + 1;  // per tile: NPS output stores and one queue op
  static_assert(2 * LPT + E_OPS < 64, "vmcnt range");
  // DMA of K-tile kt of tile t (live: t in range) into ring stage st
  auto issue = [&](Loader<BM, LM_KMAJOR, NTH>& a, int t, int kt, int st) {
    char* base = smem + st * ST_STAGE;
    const bool live = t < tiles_m;
    a.issue(p, t * BM, M, kt * BK, K, P, base, live);
    lb.issue(p, n0, N, kt * BK, K, P, base + SK_TILE, live);
  };
  issue(la, tm, 0, 0);
  issue(la, tm, 1, 1);

  int oa0[TM][2], oa1[TM][2], ob0[TN][2], ob1[TN][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i) la.frag_offsets(wm * WTM + i * 16, kk, oa0[i][kk], oa1[i][kk]);
#pragma unroll
    for (int j = 0; j < TN; ++j) lb.frag_offsets(wn * WTN + j * 16, kk, ob0[j][kk], ob1[j][kk]);
  }
  const int ch = threadIdx.x % CPRW, r0 = threadIdx.x / CPRW;
  const int n = n0 + ch * 8;
  float st_s[8], st_q[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) { st_s[r] = 0.f; st_q[r] = 0.f; }
  const __amdgpu_buffer_rsrc_t rnull = make_rsrc(nullptr, 0);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  int ticket = 0;  // wave 0 lane 0: the last queue op's result
  int stage = 0;   // ring stage of the K-tile being computed
  for (int it = 0;; ++it) {
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < KT; ++kt) {
      // K-tile (it, kt) landed: younger are the next K-tile's DMA and, for the
      // first two K-tiles of a tile after the first, the previous tile's
      // epilogue ops (stores + queue op) -- issued between those DMAs
      if (it > 0 && kt < 2) wait_vmcnt<LPT + E_OPS>();
      else wait_vmcnt<LPT>();
      raw_barrier();  // ... for every wave; every wave is done reading the stage refilled below
      {
        const int fill = stage == 0 ? 2 : stage - 1;  // (stage + 2) % 3
        if (kt + 2 < KT) issue(la, tm, kt + 2, fill);
        else issue(la1, t1, kt + 2 - KT, fill);
      }
      const char* a_img = smem + stage * ST_STAGE;
      const char* b_img = a_img + SK_TILE;
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
      stage = stage == 2 ? 0 : stage + 1;
    }
    // ---- epilogue of tile tm: acc -> bf16 staging
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
    if (it > 0 && wid == 0 && l == 0) {
      // Q(it-1) -- the ticket of tile it+2 -- retired: only this tile's last
      // two DMAs (the next tile's first K-tiles) may still be younger
      wait_vmcnt<2 * LPT>();
      *sQ = p.wq ? xcd + 8 * (3 * G8 + ticket) : tm + 16 * G8;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): staging / ticket writes complete before the barrier
    raw_barrier();  // staging complete; the ticket is in
    if (it > 0) t2 = __builtin_amdgcn_readfirstlane(*sQ);
    // Q(it): the ticket of tile it+3 (one op per wave: the others store to a null resource)
    if (wid == 0 && p.wq) {
      if (l == 0) ticket = wq_take_nowait(p.wq, qid);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(0u, rnull, 0u, 0, 0);
    }
    // staging -> global: 16-byte buffer stores against this tile's row range
    const int m0 = tm * BM;
    const int rows = min(BM, M - m0);
    const __amdgpu_buffer_rsrc_t rc =
        make_rsrc((const bf16*)p.c + (int64_t)m0 * p.ldc, (unsigned)((int64_t)rows * p.ldc * 2));
#pragma unroll
    for (int pass = 0; pass < NPS; ++pass) {
      const int ml = r0 + pass * RPP;
      const bf16x8 o = *(const bf16x8*)(sC + ml * SK_LDT + ch * 8);
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
    // (the staging image is rewritten only after the next tile's K loop: its
    // barriers order these reads before those writes)
    tm = t1;
    t1 = t2;
    if (tm >= tiles_m) break;
    la = la1;
    la1.init(p, (t1 < tiles_m ? t1 : tm) * BM, M, P, p.lda, p.a, p.a_bytes);
  }
  wait_vmcnt<0>();
  if (p.wq && threadIdx.x == 0) wq_done(p.wq, 8 * (int)gridDim.y);  // every ticket of this workgroup is taken
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

}  // namespace sg

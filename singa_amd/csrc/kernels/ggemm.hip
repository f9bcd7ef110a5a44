// Generic MFMA GEMM / implicit-GEMM convolution for gfx950: any shape, any
// stride, groups and dilation, fp32 OR bf16 operands.
//
// The reference computes every InnerProduct and convolution in fp32 sgemm
// (DotEngine, include/mshadow/tensor_expr_engine-inl.hpp:272-298,339-383;
// ConvolutionLayer / InnerProductLayer, src/worker/layer.cc:63-123,193-211).
// This is that precision on the matrix cores:
//   * fp32 operands: v_mfma_f32_16x16x4_f32 -- exact f32 (a k-ordered fmaf
//     chain), 157 TF on MI355X (gfx950 has no xf32/TF32 form, and no
//     downcast happens here);
//   * bf16 operands: v_mfma_f32_16x16x32_bf16, for the shapes the tuned
//     bf16 kernel (igemm.hip: LDS-DMA staging, K-multiple-of-8 rows) does not
//     take -- ragged dimensions, grouped / dilated convolutions.
//
//   C[m][n] (=|+=) alpha * sum_k A(m, k) * B(n, k) (+ bias[n]) (ReLU)
//
// Structure: BM x BN x 32 tiles (64 or 128 square), 256 threads = 2 x 2 waves.
// Operands are staged global -> registers -> LDS (two stages, one barrier per
// K-tile; the next tile's global loads are in flight during this tile's
// MFMAs).  Every operand element is loaded through a "unit" of 4 elements
// that are contiguous in memory when the shapes allow (one 16-byte fp32 / 8-
// byte bf16 vector load), or 4 bounds-checked scalar loads otherwise, so no
// dimension needs padding.  LDS images are [rows][32 k]: each MFMA lane reads
// its 4 (fp32) or 8 (bf16) consecutive k of one row with a single
// ds_read_b128 -- the k order inside an MFMA step is permuted identically for
// A and B, which leaves the sum unchanged.
//   fp32: unpadded 128-B rows, the 16-B chunk c of row r stored at chunk
//         c ^ swz(r), swz(r) = (r ^ r >> 2) & 7: 8 consecutive rows (one
//         b128 read phase) hit 8 distinct chunks, and so do the 8 row-quads
//         a K-outer loader scatters its scalar stores over (an 8-way bank
//         conflict with a padded [rows][36] image);
//   bf16: rows padded by 16 bytes (80-B stride), conflict-free b128 reads.
// fp32 tiles of 128 x 128 run v_mfma_f32_32x32x2_f32 (each wave 64 x 64 as
// 2 x 2 blocks, lane halves reading alternate k-chunks); 64 x 64 tiles run
// v_mfma_f32_16x16x4_f32.
//
// Operand modes (the loader gathers the implicit-GEMM operands itself):
//   KMAJ    plain [rows][K] (ld)                     k-contiguous units
//   KOUT    plain [K][rows] (ld)                     row-contiguous units
//   CFWD_A  conv fwd A: im2col of x NHWC, rows = output pixels, k = (r, s, c)
//   DGRAD_A conv dgrad A: dy NHWC gathered per input pixel, k = (r, s, k_out),
//           taps that do not land on the stride grid are zero
//   DGRAD_B conv dgrad B: W [K][R][S][Cg], rows = c, k = (r, s, k_out)
//   WGRAD_B conv wgrad B: x gathered, rows = (r, s, c), k = output pixels
// A group of a grouped convolution is one batch index (blockIdx.y): every
// operand and the output advance by their per-group batch stride.
#include <stdlib.h>

#include <stdexcept>
#include <string>
#include <type_traits>

#include "common.h"

namespace sg {
namespace gg {

constexpr int BK = 32, NT = 256;
enum Mode : int { KMAJ = 0, KOUT = 1, CFWD_A = 2, DGRAD_A = 3, DGRAD_B = 4, WGRAD_B = 5 };
enum Out : int { O_BF16 = 0, O_F32 = 1, O_F32_ATOMIC = 2 };

struct Geom {
  int N, H, W, C, K;    // input NHWC (C total channels), K total filters
  int Cg, Kg, R, S;     // per-group channels / filters; filter taps
  int Ho, Wo, sh, sw, ph, pw, dh, dw;
  FastDiv dCg, dKg, dS, dWo, dHoWo, dW, dHW, dsh, dsw;
};

struct Args {
  int M, N, K;
  const void* a;
  int64_t lda, sa;  // leading dim, batch (group) stride in elements
  const void* b;
  int64_t ldb, sb;
  void* c;
  int64_t ldc, sc;
  float alpha, beta;
  const float* bias;
  int64_t sbias;
  int relu, out_mode;
  int k_per_split;   // multiple of BK
  int vec_a, vec_b;  // 4-element units are contiguous + aligned (vector loads)
  float* csum;       // optional: csum[n] += sum_k B(n, k) (the bias gradient of a weight-gradient GEMM)
  const void* act_x; // optional: C[m][n] *= act'(X[m][n]), X the activation OUTPUT laid out like C (ldc)
  int act_bwd;       // activation of act_x (Act codes)
  void* aux;         // optional: the pre-activation z of a fused activation (laid out like C)
  Geom g;
};

// fused activations (the relu field of Args; act_bwd): codes 0 none, 1 relu,
// 2 sigmoid, 3 tanh, 4 stanh -- the formulas of elementwise.hip's unary_f /
// unary_b, derivatives from the activation's output.  (The GELUs, codes 5 / 6,
// live in the tuned bf16 kernel's epilogue only: inlined into every
// instantiation here they doubled this file's code.)
enum Act : int { A_NONE = 0, A_RELU = 1, A_SIGMOID = 2, A_TANH = 3, A_STANH = 4 };
__device__ __forceinline__ float act_f(int a, float v) {
  switch (a) {
    case A_RELU: return fmaxf(v, 0.f);
    case A_SIGMOID: return 1.f / (1.f + __expf(-v));
    case A_TANH: return tanhf(v);
    case A_STANH: return 1.7159047f * tanhf(0.66666667f * v);
    default: return v;
  }
}
__device__ __forceinline__ float dact_y(int a, float t) {
  switch (a) {
    case A_RELU: return t > 0.f ? 1.f : 0.f;
    case A_SIGMOID: return t * (1.f - t);
    case A_TANH: return 1.f - t * t;
    case A_STANH: return 0.66666667f * 1.7159047f - 0.66666667f / 1.7159047f * t * t;
    default: return 1.f;
  }
}

template <typename T> struct V4;
template <> struct V4<float> { typedef f32x4 t; };
template <> struct V4<bf16> { typedef bf16x4 t; };

template <typename T> constexpr int pad_of() { return sizeof(T) == 4 ? 0 : 8; }
template <typename T> constexpr int ld_of() { return BK + pad_of<T>(); }
// fp32 LDS image: element offset of (row, k) -- 16-byte chunk XOR swizzle
__device__ __forceinline__ int swz(int r) { return (r ^ (r >> 2)) & 7; }
__device__ __forceinline__ int f32_pos(int row, int k) { return row * BK + 4 * (((k >> 2) ^ swz(row))) + (k & 3); }

// One operand's loader: ROWS tile rows x BK k, U units of 4 elements / thread.
template <typename T, int ROWS, int MODE>
struct Ld {
  static constexpr bool RC = (MODE == KOUT || MODE == DGRAD_B || MODE == WGRAD_B);
  static constexpr int U = ROWS * BK / 4 / NT;
  static constexpr int RQ = ROWS / 4;   // RC: row quads per k-row
  static constexpr int KS = NT / RQ;    // RC: k-rows per pass
  static_assert(U >= 1, "tile too small");
  typedef typename V4<T>::t VT;
  VT v[U];
  const T* base;
  int64_t ld;
  int nrows;
  bool vec;
  // k-contiguous modes: per unit row info; RC modes: per element column info
  int ri0[U], ri1[U], ri2[U];
  bool rok[U];
  int ci0[4], ci1[4], ci2[4];
  bool cok[4];

  __device__ __forceinline__ void init(const Args& p, const T* src, int64_t ld_, int row0, int nrows_, bool vec_) {
    base = src;
    ld = ld_;
    nrows = nrows_;
    vec = vec_;
    const int t = threadIdx.x;
    const Geom& g = p.g;
    if constexpr (!RC) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = row0 + (t >> 3) + 32 * u;
        rok[u] = row < nrows;
        const int rr = rok[u] ? row : 0;
        if constexpr (MODE == KMAJ) {
          ri0[u] = rr;
        } else if constexpr (MODE == CFWD_A) {
          const int n = g.dHoWo.div(rr);
          const int rem = rr - n * g.Ho * g.Wo;
          const int oh = g.dWo.div(rem);
          const int ow = rem - oh * g.Wo;
          ri0[u] = n;
          ri1[u] = oh * g.sh - g.ph;
          ri2[u] = ow * g.sw - g.pw;
        } else {  // DGRAD_A: rows are input pixels (n, h, w)
          const int n = g.dHW.div(rr);
          const int rem = rr - n * g.H * g.W;
          const int h = g.dW.div(rem);
          const int w = rem - h * g.W;
          ri0[u] = n;
          ri1[u] = h + g.ph;
          ri2[u] = w + g.pw;
        }
      }
    } else {
      const int r4 = row0 + 4 * (t % RQ);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = r4 + e;
        cok[e] = col < nrows;
        const int cc = cok[e] ? col : 0;
        if constexpr (MODE == KOUT || MODE == DGRAD_B) {
          ci0[e] = cc;
        } else {  // WGRAD_B: col = (r, s, c)
          const int rs = g.dCg.div(cc);
          const int c = cc - rs * g.Cg;
          const int r = g.dS.div(rs);
          const int s = rs - r * g.S;
          ci0[e] = r * g.dh - g.ph;
          ci1[e] = s * g.dw - g.pw;
          ci2[e] = c;
        }
      }
    }
  }

  // element offset + validity of (row info u / column e, absolute k)
  __device__ __forceinline__ bool at_k(const Geom& g, int u, int k, int64_t& off) const {
    if constexpr (MODE == KMAJ) {
      off = (int64_t)ri0[u] * ld + k;
      return rok[u];
    } else if constexpr (MODE == CFWD_A) {
      const int rs = g.dCg.div(k);
      const int c = k - rs * g.Cg;
      const int r = g.dS.div(rs);
      const int s = rs - r * g.S;
      const int ih = ri1[u] + r * g.dh, iw = ri2[u] + s * g.dw;
      off = (((int64_t)ri0[u] * g.H + ih) * g.W + iw) * g.C + c;
      return rok[u] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
    } else {  // DGRAD_A: k = (r, s, ko)
      const int rs = g.dKg.div(k);
      const int ko = k - rs * g.Kg;
      const int r = g.dS.div(rs);
      const int s = rs - r * g.S;
      const int th = ri1[u] - r * g.dh, tw = ri2[u] - s * g.dw;
      const int oh = g.dsh.div((unsigned)(th < 0 ? 0 : th)), ow = g.dsw.div((unsigned)(tw < 0 ? 0 : tw));
      const bool ok = th >= 0 && tw >= 0 && oh * g.sh == th && ow * g.sw == tw && oh < g.Ho && ow < g.Wo;
      off = (((int64_t)ri0[u] * g.Ho + oh) * g.Wo + ow) * g.K + ko;
      return rok[u] && ok;
    }
  }
  __device__ __forceinline__ bool at_col(const Geom& g, int e, int k, int64_t& off) const {
    if constexpr (MODE == KOUT) {
      off = (int64_t)k * ld + ci0[e];
      return cok[e];
    } else if constexpr (MODE == DGRAD_B) {  // W [Kg][R][S][Cg] (group base in src), k = (r, s, ko)
      const int rs = g.dKg.div(k);
      const int ko = k - rs * g.Kg;
      off = ((int64_t)ko * g.R * g.S + rs) * g.Cg + ci0[e];
      return cok[e];
    } else {  // WGRAD_B: k = output pixel
      const int n = g.dHoWo.div(k);
      const int rem = k - n * g.Ho * g.Wo;
      const int oh = g.dWo.div(rem);
      const int ow = rem - oh * g.Wo;
      const int ih = oh * g.sh + ci0[e], iw = ow * g.sw + ci1[e];
      off = (((int64_t)n * g.H + ih) * g.W + iw) * g.C + ci2[e];
      return cok[e] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
    }
  }

  // global -> registers for the K-tile at k0 (k < kend valid)
  __device__ __forceinline__ void load(const Geom& g, int k0, int kend) {
    const int t = threadIdx.x;
    if constexpr (!RC) {
      const int kb = k0 + 4 * (t & 7);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (vec) {
          int64_t off;
          const bool ok = kb < kend && at_k(g, u, kb, off);
          v[u] = ok ? *(const VT*)(base + off) : VT{};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            int64_t off;
            const bool ok = kb + e < kend && at_k(g, u, kb + e, off);
            v[u][e] = ok ? base[off] : (T)0.f;
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + t / RQ + KS * u;
        const bool kin = k < kend;
        const int kk = kin ? k : 0;
        if (vec) {
          int64_t off;
          const bool ok = kin && at_col(g, 0, kk, off);
          v[u] = ok ? *(const VT*)(base + off) : VT{};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            int64_t off;
            const bool ok = kin && at_col(g, e, kk, off);
            v[u][e] = ok ? base[off] : (T)0.f;
          }
        }
      }
    }
  }

  // registers -> LDS image [ROWS][BK + pad]
  __device__ __forceinline__ void store(T* lds) const {
    constexpr int LD = ld_of<T>();
    const int t = threadIdx.x;
    if constexpr (sizeof(T) == 4) {  // swizzled unpadded image
      if constexpr (!RC) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int row = (t >> 3) + 32 * u;
          *(VT*)(lds + f32_pos(row, 4 * (t & 7))) = v[u];
        }
      } else {
        const int r4 = 4 * (t % RQ);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = t / RQ + KS * u;
#pragma unroll
          for (int e = 0; e < 4; ++e) lds[f32_pos(r4 + e, k)] = v[u][e];
        }
      }
    } else if constexpr (!RC) {
#pragma unroll
      for (int u = 0; u < U; ++u) *(VT*)(lds + ((t >> 3) + 32 * u) * LD + 4 * (t & 7)) = v[u];
    } else {
      const int r4 = 4 * (t % RQ);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = t / RQ + KS * u;
#pragma unroll
        for (int e = 0; e < 4; ++e) lds[(r4 + e) * LD + k] = v[u][e];
      }
    }
  }
};

template <typename T, int BM, int BN, int AM, int BMODE, bool M32V = true>
__global__ void __launch_bounds__(NT, 2) ggemm_k(const Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int LD = ld_of<T>();
  constexpr int A_EL = BM * LD, STAGE_EL = (BM + BN) * LD;
  // fp32 128x128: 32x32x2 MFMA blocks (each wave 2 x 2 of them) unless M32V
  // is off (16x16x4 blocks, 4 x 4 per wave)
  constexpr bool M32 = sizeof(T) == 4 && BM == 128 && BN == 128 && M32V;
  constexpr int MB = M32 ? 32 : 16;
  constexpr int WTM = BM / 2, WTN = BN / 2, TM = WTM / MB, TN = WTN / MB;
  typedef typename std::conditional<M32, f32x16, f32x4>::type AccT;
  T* lds = (T*)smem;

  const int64_t y = blockIdx.y;
  const T* pa = (const T*)p.a + y * p.sa;
  const T* pb = (const T*)p.b + y * p.sb;
  const float* bias = p.bias ? p.bias + y * p.sbias : nullptr;

  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  if (bid >= nwg) return;
  if (nwg >= 8) {  // XCD-aware bijective remap: consecutive tiles share an XCD's L2
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

  const int kbeg = blockIdx.z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  if (p.out_mode == O_F32_ATOMIC && kbeg >= kend) return;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  Ld<T, BM, AM> la;
  Ld<T, BN, BMODE> lb;
  la.init(p, pa, p.lda, m0, p.M, p.vec_a);
  lb.init(p, pb, p.ldb, n0, p.N, p.vec_b);

  const int l = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  AccT acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = AccT{};

  const int g4 = l >> 4;
  auto compute = [&](const T* sa_) {
    const T* sb_ = sa_ + A_EL;
    if constexpr (M32) {
      // lane half h = l >> 5 reads k-chunk 2q + h of rows (l & 31): element e
      // of the float4 feeds the MFMA over the k pair {8q + e, 8q + 4 + e}
      const int h = l >> 5;
#pragma unroll
      for (int q = 0; q < BK / 8; ++q) {
        float4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = *(const float4*)(sa_ + f32_pos(wm * WTM + 32 * i + (l & 31), 8 * q + 4 * h));
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = *(const float4*)(sb_ + f32_pos(wn * WTN + 32 * j + (l & 31), 8 * q + 4 * h));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[j].x, fa[i].x, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[j].y, fa[i].y, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[j].z, fa[i].z, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[j].w, fa[i].w, acc[i][j], 0, 0, 0);
          }
      }
    } else if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int c = 0; c < BK / 16; ++c) {
        float4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = *(const float4*)(sa_ + f32_pos(wm * WTM + 16 * i + (l & 15), 16 * c + 4 * g4));
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = *(const float4*)(sb_ + f32_pos(wn * WTN + 16 * j + (l & 15), 16 * c + 4 * g4));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j].x, fa[i].x, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j].y, fa[i].y, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j].z, fa[i].z, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j].w, fa[i].w, acc[i][j], 0, 0, 0);
          }
      }
    } else {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = *(const bf16x8*)(sa_ + (wm * WTM + 16 * i + (l & 15)) * LD + 8 * g4);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = *(const bf16x8*)(sb_ + (wn * WTN + 16 * j + (l & 15)) * LD + 8 * g4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  // fused column sums of B (workgroups of the first M tile): thread t sums
  // column n = t % BN over its k slice of every K-tile image
  const bool do_cs = p.csum != nullptr && tm == 0;
  constexpr int CS_G = NT / BN, CS_K = BK / CS_G;
  float cs_acc = 0.f;
  auto colsum_tile = [&](const T* sb_) {
    const int n = threadIdx.x % BN, k0 = (threadIdx.x / BN) * CS_K;
#pragma unroll
    for (int k = 0; k < CS_K; ++k) {
      if constexpr (sizeof(T) == 4) cs_acc += (float)sb_[f32_pos(n, k0 + k)];
      else cs_acc += (float)sb_[n * LD + k0 + k];
    }
  };

  if (nk > 0) {
    la.load(p.g, kbeg, kend);
    lb.load(p.g, kbeg, kend);
    la.store(lds);
    lb.store(lds + A_EL);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) {  // next tile's global loads in flight during this tile's MFMAs
        la.load(p.g, kbeg + (kt + 1) * BK, kend);
        lb.load(p.g, kbeg + (kt + 1) * BK, kend);
      }
      compute(lds + cur * STAGE_EL);
      if (do_cs) colsum_tile(lds + cur * STAGE_EL + A_EL);
      if (more) {
        T* nx = lds + (cur ^ 1) * STAGE_EL;
        la.store(nx);
        lb.store(nx + A_EL);
      }
      __syncthreads();
    }
  }

  if (do_cs) {  // (workgroup-uniform) the CS_G partials of a column in a fixed order, one atomic per column
    float* red = (float*)smem;
    __syncthreads();  // every wave done with the last stage
    red[threadIdx.x] = cs_acc;
    __syncthreads();
    if ((int)threadIdx.x < BN && n0 + (int)threadIdx.x < p.N) {
      float sum = 0.f;
#pragma unroll
      for (int g = 0; g < CS_G; ++g) sum += red[g * BN + threadIdx.x];
      atomicAdd(p.csum + n0 + threadIdx.x, sum);
    }
    __syncthreads();  // the epilogue may reuse the LDS
  }

  constexpr int EPI_LDS = 2 * STAGE_EL * (int)sizeof(T);
#include "ggemm_epilogue.inc"
}

// ------------------------------------------------------------------------------
// fp32 plain GEMM with LDS-DMA staging (f32d_k): the same C = alpha A B^T
// (+ epilogue) as ggemm_k<float> for K-major / K-outer operands whose 4-float
// units are contiguous and 16-byte aligned, but the operands go global -> LDS
// with buffer_load_dwordx4 ... lds (no registers, no ds_write) through a ring
// of three K-tile stages: two K-tiles stay in flight while the third is
// multiplied, each K-tile starting with a COUNTED vmcnt and one barrier.
// ggemm_k's register staging holds one K-tile in flight, and a 64 x 64 x 32
// fp32 K-tile is only ~1000 MFMA cycles per wave: the load latency was exposed
// every K-tile (MFMA pipe ~55 % busy on the mlp.conf shapes,
// profiles/ggemm_r4/pmc_f32.txt).
//
// LDS images (fp32, BK = 32 k per stage):
//   K-major operand  [rows][32 k], 16-byte chunk c of row r at c ^ swz(r)
//                    (f32_pos, as ggemm_k's image); lane (r = t>>3, slot t&7)
//                    fetches chunk slot ^ swz(r), so one wave-instruction
//                    fills 8 rows = 1 KB lane-linearly;
//   K-outer operand  [32 k][rows], chunk c of k-row kr at c ^ (4 ((kr>>2)&3))
//                    (kout_pos): the MFMA lanes of one k-step read k-rows
//                    kr, kr+4, kr+8, kr+12 (lane groups l>>4) of 16
//                    consecutive rows, and the XOR puts the four groups on
//                    disjoint 16-bank sets -- ds_read_b32 conflict-free.
// A lane of a 16x16x4 MFMA step q of k-chunk c holds k = 16c + 4(l>>4) + q for
// both operands (float4 reads from K-major images, four scalar reads from
// K-outer ones), i.e. ggemm_k's k order: the sum is the same fmaf chain.
// Reference: DotEngine's fp32 sgemm, include/mshadow/tensor_expr_engine-inl.hpp:272-298.
// ------------------------------------------------------------------------------
constexpr unsigned D_OOB = 0xFFFFFFF0u;  // an offset past any extent: the load returns zeros
constexpr unsigned D_BIAS = 0x80000000u; // masked lanes keep a biased offset (see igemm_kern.h)
// The DMA is inline asm (M0 = the wave's LDS destination): issued through the
// builtin, the compiler puts s_waitcnt vmcnt(0) in front of every LDS read it
// cannot prove disjoint from the DMA in flight (here: every fragment read of
// the runtime-indexed ring), serialising the ring.  The K loop waits for the
// DMA itself with counted vmcnts; the compiler tracks the fragment reads.
typedef int d_i32x4 __attribute__((ext_vector_type(4)));
// (M0 is listed as clobbered: the compiler keeps nothing in it in these
// kernels -- it is the LDS-DMA destination register and the asm sets it first)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(d_i32x4 r, unsigned off, unsigned lds_wave_base) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds_wave_base), "v"(off), "s"(r)
               : "memory", "m0");
}
#pragma clang diagnostic pop
// buffer resource: base, stride 0, num_records = bytes (0: a null resource)
__device__ __forceinline__ d_i32x4 rsrc_of(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  return d_i32x4{(int)(unsigned)a, (int)((unsigned)(a >> 32) & 0xFFFFu), (int)bytes, 0x00020000};
}
template <int N>
__device__ __forceinline__ void d_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
template <int ROWS>
__device__ __forceinline__ int kout_pos(int row, int k) {
  return k * ROWS + 4 * ((row >> 2) ^ (((k >> 2) & 3) << 2)) + (row & 3);
}

template <int ROWS, int MODE>
struct DLd {
  static constexpr bool RC = MODE == KOUT;
  static constexpr int VPT = ROWS * BK / 4 / NT;  // 16-byte vectors per thread per K-tile
  static constexpr int CPR = ROWS / 4;            // K-outer: chunks per k-row
  static constexpr int KRP = NT / CPR;            // K-outer: k-rows per pass
  static_assert(VPT >= 1 && (!RC || ROWS >= 64), "K-outer images need >= 64 rows (16 chunks per k-row)");
  d_i32x4 rsrc;
  unsigned voff[VPT];
  unsigned ldb4;  // K-outer: bytes per k-row of the source
  int wv, lk;     // wave; K-major: this lane's k within a tile, K-outer: its k-row within a pass

  __device__ __forceinline__ void init(const float* src, unsigned bytes, int64_t ld, int row0, int nrows) {
    const int t = threadIdx.x;
    wv = __builtin_amdgcn_readfirstlane(t >> 6);
    rsrc = rsrc_of(src, bytes);
    if constexpr (!RC) {
      const int rl = t >> 3;
      lk = 4 * ((t & 7) ^ swz(rl));  // swz(rl + 32 v) == swz(rl)
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int row = row0 + rl + 32 * v;
        voff[v] = row < nrows ? (unsigned)(row * (int)ld + lk) * 4u : D_BIAS;
      }
    } else {
      ldb4 = (unsigned)ld * 4u;
      lk = t / CPR;
      const int slot = t % CPR;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int kr = lk + KRP * v;
        const int col = row0 + 4 * (slot ^ (((kr >> 2) & 3) << 2));
        voff[v] = col < nrows ? (unsigned)(kr * (int)ld + col) * 4u : D_BIAS;
      }
    }
  }
  // the K-tile at k0 into the stage image at `img`; live == false: a dummy
  // through a null resource (keeps the per-tile DMA count uniform)
  __device__ __forceinline__ void issue(int k0, int kend, unsigned img, bool live) const {
    d_i32x4 rs = rsrc;
    if (!live) rs[2] = 0;
    const bool full = kend - k0 >= BK;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      unsigned off;
      if constexpr (!RC) {
        off = (full || k0 + lk < kend) ? voff[v] + (unsigned)k0 * 4u : D_OOB;
      } else {
        off = (full || k0 + lk + KRP * v < kend) ? voff[v] + (unsigned)k0 * ldb4 : D_OOB;
      }
      dma16(rs, off, img + 1024u * wv + 4096u * v);
    }
  }
};

template <int BM, int BN, int AM, int BMODE>
__global__ void __launch_bounds__(NT, 2) f32d_k(const Args p) {
  using T = float;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGES = 3, D = STAGES - 1;
  constexpr int A_B = BM * BK * 4, STAGE = (BM + BN) * BK * 4;
  constexpr bool M32 = false;
  constexpr int WTM = BM / 2, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  typedef f32x4 AccT;

  const int64_t y = blockIdx.y;
  const float* pa = (const float*)p.a + y * p.sa;
  const float* pb = (const float*)p.b + y * p.sb;
  const float* bias = p.bias ? p.bias + y * p.sbias : nullptr;

  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
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

  const int kbeg = blockIdx.z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  if (p.out_mode == O_F32_ATOMIC && kbeg >= kend) return;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // operand extents (bytes) for the buffer resources: host-checked < 2^31
  auto extent = [&](int mode, int rows, int64_t ld) -> unsigned {
    return mode == KOUT ? (unsigned)(((int64_t)(p.K - 1) * ld + rows) * 4) : (unsigned)(((int64_t)(rows - 1) * ld + p.K) * 4);
  };
  DLd<BM, AM> la;
  DLd<BN, BMODE> lb;
  la.init(pa, extent(AM, p.M, p.lda), p.lda, m0, p.M);
  lb.init(pb, extent(BMODE, p.N, p.ldb), p.ldb, n0, p.N);

  const int l = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int g4 = l >> 4;
  AccT acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = AccT{};

  auto compute = [&](const char* st) {
    const float* sa_ = (const float*)st;
    const float* sb_ = (const float*)(st + A_B);
#pragma unroll
    for (int c = 0; c < BK / 16; ++c) {
      const int k = 16 * c + 4 * g4;
      float fa[TM][4], fb[TN][4];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + 16 * i + (l & 15);
        if constexpr (AM == KOUT) {
#pragma unroll
          for (int q = 0; q < 4; ++q) fa[i][q] = sa_[kout_pos<BM>(r, k + q)];
        } else {
          const float4 v = *(const float4*)(sa_ + f32_pos(r, k));
          fa[i][0] = v.x; fa[i][1] = v.y; fa[i][2] = v.z; fa[i][3] = v.w;
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WTN + 16 * j + (l & 15);
        if constexpr (BMODE == KOUT) {
#pragma unroll
          for (int q = 0; q < 4; ++q) fb[j][q] = sb_[kout_pos<BN>(r, k + q)];
        } else {
          const float4 v = *(const float4*)(sb_ + f32_pos(r, k));
          fb[j][0] = v.x; fb[j][1] = v.y; fb[j][2] = v.z; fb[j][3] = v.w;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j][q], fa[i][q], acc[i][j], 0, 0, 0);
    }
  };

  // fused column sums of B (workgroups of the first M tile), as in ggemm_k
  const bool do_cs = p.csum != nullptr && tm == 0;
  constexpr int CS_G = NT / BN, CS_K = BK / CS_G;
  float cs_acc = 0.f;
  auto colsum_tile = [&](const char* st) {
    const float* sb_ = (const float*)(st + A_B);
    const int n = threadIdx.x % BN, k0 = (threadIdx.x / BN) * CS_K;
#pragma unroll
    for (int k = 0; k < CS_K; ++k) {
      if constexpr (BMODE == KOUT) cs_acc += sb_[kout_pos<BN>(n, k0 + k)];
      else cs_acc += sb_[f32_pos(n, k0 + k)];
    }
  };

  if (nk > 0) {
    constexpr int LPT = DLd<BM, AM>::VPT + DLd<BN, BMODE>::VPT;
    static_assert(D * LPT < 64, "vmcnt range");
    const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
#pragma unroll
    for (int s = 0; s < D; ++s) {
      la.issue(kbeg + s * BK, kend, lds0 + s * STAGE, s < nk);
      lb.issue(kbeg + s * BK, kend, lds0 + s * STAGE + A_B, s < nk);
    }
    int cur = 0, fill = D;
    for (int kt = 0; kt < nk; ++kt) {
      d_wait_vmcnt<(D - 1) * LPT>();  // this wave's DMA of K-tile kt landed
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();   // ... every wave's; stage `fill` is no longer read
      asm volatile("" ::: "memory");
      const unsigned st = lds0 + (unsigned)(fill * STAGE);
      const bool live = kt + D < nk;
      la.issue(kbeg + (kt + D) * BK, kend, st, live);
      lb.issue(kbeg + (kt + D) * BK, kend, st + A_B, live);
      compute(smem + cur * STAGE);
      if (do_cs) colsum_tile(smem + cur * STAGE);
      cur = cur + 1 == STAGES ? 0 : cur + 1;
      fill = fill + 1 == STAGES ? 0 : fill + 1;
    }
  }
  d_wait_vmcnt<0>();  // the dummy DMAs too, before the LDS is reused
  __syncthreads();

  if (do_cs) {
    float* red = (float*)smem;
    red[threadIdx.x] = cs_acc;
    __syncthreads();
    if ((int)threadIdx.x < BN && n0 + (int)threadIdx.x < p.N) {
      float sum = 0.f;
#pragma unroll
      for (int g = 0; g < CS_G; ++g) sum += red[g * BN + threadIdx.x];
      atomicAdd(p.csum + n0 + threadIdx.x, sum);
    }
    __syncthreads();
  }
  constexpr int EPI_LDS = STAGES * STAGE;
#include "ggemm_epilogue.inc"
}

template <int BM, int BN, int AM, int BMODE>
static void launch_d(const Args& p, int batch, int splits, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  constexpr int lds = 3 * (BM + BN) * BK * 4;
  auto* kern = f32d_k<BM, BN, AM, BMODE>;
  if constexpr (lds > 65536) {
    static bool attr = [kern] {
      return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    }();
    (void)attr;
  }
  hipLaunchKernelGGL(kern, dim3(tiles, batch, splits), dim3(NT), lds, s, p);
}

template <typename T, int BM, int BN, int AM, int BMODE, bool M32V = true>
static void launch_t(const Args& p, int batch, int splits, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  constexpr int lds = 2 * (BM + BN) * ld_of<T>() * (int)sizeof(T);
  auto* kern = ggemm_k<T, BM, BN, AM, BMODE, M32V>;
  if constexpr (lds > 65536) {
    static bool attr = [kern] {
      return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    }();
    (void)attr;
  }
  hipLaunchKernelGGL(kern, dim3(tiles, batch, splits), dim3(NT), lds, s, p);
}

// minimum 128x128 tile count for the big tile (fp32 / bf16); SG_GG_T128_F32 /
// SG_GG_T128 override (A/B tuning)
static long t128_min(bool f32) {
  static const long v32 = [] {
    // measured (mlp_gpu, MI355X): 64x64 16x16x4 tiles everywhere 749k samples/s,
    // 128x128 32x32x2 tiles from 96 tiles up 352k -- the big fp32 tile stays opt-in
    const char* e = getenv("SG_GG_T128_F32");
    return e ? atol(e) : (1L << 40);
  }();
  static const long v16 = [] {
    const char* e = getenv("SG_GG_T128");
    return e ? atol(e) : 192L;
  }();
  return f32 ? v32 : v16;
}

static bool big_tile(int M, int N, bool f32 = false) {
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
  return M >= 128 && N >= 128 && t128 >= t128_min(f32);
}

template <typename T, int AM, int BMODE>
static void launch(const Args& p, int batch, int splits, hipStream_t s) {
  if (big_tile(p.M, p.N, sizeof(T) == 4)) launch_t<T, 128, 128, AM, BMODE>(p, batch, splits, s);
  else launch_t<T, 64, 64, AM, BMODE>(p, batch, splits, s);
}

// split-K count for atomic outputs: fill ~512 workgroups, >= 4 K-tiles each
static int pick_splits(int M, int N, int K, int batch, int want, int bm, int bn) {
  if (want > 0) return want;
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * (batch > 0 ? batch : 1);
  const int nkt = (K + BK - 1) / BK;
  int sp = 1;
  while (tiles * sp < 512 && sp * 2 * 4 <= nkt && sp < 4096) sp *= 2;
  return sp;
}

// fp32 GEMM tuning (sg_ggemm_tune): key 0 = tile (0 auto, 1 64x64, 2 128x128
// on 32x32x2, 3 128x64, 4 64x128, 5 128x128 on 16x16x4, 6 64x32, 7 32x64,
// 8 32x32); key 1 = split-K (0 auto, -1 never, n > 1 forced; a plain fp32
// output split over K is zeroed -- or kept,
// beta = 1 -- and the splits add into it with atomics, split 0 adding the bias).
// (Measured and dropped: a 2-deep register prefetch of the global loads --
// no gain at any MLP shape, +36 VGPRs.)
// key 2 = the LDS-DMA fp32 kernel f32d_k (0 on where it applies, the tile
// choice restricted to its tiles; 1 on, unrestricted choice; -1 never).
static int g_gg[3] = {0, 0, 0};

static void tile_dims(int t, int& bm, int& bn) {
  bm = (t == 2 || t == 3 || t == 5) ? 128 : (t == 7 || t == 8) ? 32 : 64;
  bn = (t == 2 || t == 4 || t == 5) ? 128 : (t == 6 || t == 8) ? 32 : 64;
}

__global__ void zero_rows_k(float* c, int64_t ldc, int64_t sc, int N) {
  float* r = c + blockIdx.y * sc + (int64_t)blockIdx.x * ldc;
  for (int n = threadIdx.x; n < N; n += blockDim.x) r[n] = 0.f;
}

// fp32 tile / split-K choice: the configuration with the least modelled
// time.  A CU runs ceil(workgroups / 256) tiles concurrently, so the time is
// that many tiles' MACs over the CU rate scaled by the tile's relative
// efficiency (measured, tools/bench_ggemm_f32.py: 64x64 1.0; 32x64 / 128x64 /
// 64x128 0.9; 64x32 / 32x32 0.85; one tile per CU loses another 40 %), plus
// for split-K the extra output traffic (zeroing + one fp32 atomic per split
// per element at ~4 TB/s).  On the mlp.conf shapes its picks are within 2.5 %
// of the best configuration of the sweep (profiles/ggemm_r4/).
// With operands the LDS-DMA kernel takes (dma: 0 no, else 1 + 2 a_kouter +
// 4 b_kouter), only the tiles it runs are candidates: f32d_k beat ggemm_k at
// every such (shape, tile, splits) of the mlp.conf sweep
// (profiles/r5/ggemm_f32_dma_sweep.jsonl); 32-row tiles need that operand K-major.
static void pick_f32(int M, int N, int K, int batch, bool can_split, bool zero_first, int& tile, int& splits,
                     int dma = 0) {
  static const int cand[] = {1, 7, 3, 4, 6, 8};
  static const double eff[] = {0, 1.0, 0, 0.9, 0.9, 0, 0.85, 0.9, 0.85};
  static const int sps[] = {1, 2, 3, 4, 8};
  const int nkt = (K + BK - 1) / BK;
  double best = 1e300;
  tile = 1;
  splits = 1;
  for (int t : cand) {
    int bm, bn;
    tile_dims(t, bm, bn);
    // (small outputs keep the 32-row tiles: more workgroups beat the DMA ring there)
    if (dma && (long)M * N * batch > (1L << 18) && ((bm < 64 && (dma & 2)) || (bn < 64 && (dma & 4)))) continue;
    const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch;
    for (int sp : sps) {
      if (sp > 1 && (!can_split || nkt < 2 * sp)) continue;
      const long per_cu = (tiles * sp + 255) / 256;
      const long kk = (long)((nkt + sp - 1) / sp) * BK;
      const double e = eff[t] * (per_cu == 1 ? 0.6 : 1.0);
      double cost = (double)per_cu * bm * bn * kk / e;  // MACs at unit efficiency
      // split-K output traffic in MAC-equivalents: bytes / 4 TB/s * (128 MAC/clk * 2.2 GHz * 0.58)
      if (sp > 1) cost += (double)(sp + (zero_first ? 1 : 0)) * M * N * 4.0 * batch / 4e12 * (128 * 2.2e9 * 0.58);
      if (cost < best * 0.999) {
        best = cost;
        tile = t;
        splits = sp;
      }
    }
  }
}

template <int AM, int BMODE>
static void launch_f32(const Args& p, int batch, int splits, int tile, hipStream_t s) {
  switch (tile) {
    case 2: launch_t<float, 128, 128, AM, BMODE, true>(p, batch, splits, s); break;
    case 3: launch_t<float, 128, 64, AM, BMODE>(p, batch, splits, s); break;
    case 4: launch_t<float, 64, 128, AM, BMODE>(p, batch, splits, s); break;
    case 5: launch_t<float, 128, 128, AM, BMODE, false>(p, batch, splits, s); break;
    case 6: launch_t<float, 64, 32, AM, BMODE>(p, batch, splits, s); break;
    case 7: launch_t<float, 32, 64, AM, BMODE>(p, batch, splits, s); break;
    case 8: launch_t<float, 32, 32, AM, BMODE>(p, batch, splits, s); break;
    default: launch_t<float, 64, 64, AM, BMODE>(p, batch, splits, s); break;
  }
}

// the LDS-DMA fp32 kernel for tile t when its constraints hold: both
// operands in 16-byte units (vec), K-outer operands >= 64 tile rows, operand
// extents < 2 GiB (32-bit buffer offsets)
template <int AM, int BMODE>
static bool launch_dma_t(const Args& p, int batch, int splits, int tile, hipStream_t s) {
  switch (tile) {
    case 1: launch_d<64, 64, AM, BMODE>(p, batch, splits, s); return true;
    case 3: launch_d<128, 64, AM, BMODE>(p, batch, splits, s); return true;
    case 4: launch_d<64, 128, AM, BMODE>(p, batch, splits, s); return true;
    case 5: launch_d<128, 128, AM, BMODE>(p, batch, splits, s); return true;
    default: break;
  }
  if constexpr (AM == KMAJ) {
    if (tile == 7) { launch_d<32, 64, AM, BMODE>(p, batch, splits, s); return true; }
    if constexpr (BMODE == KMAJ) {
      if (tile == 8) { launch_d<32, 32, AM, BMODE>(p, batch, splits, s); return true; }
    }
  }
  if constexpr (BMODE == KMAJ) {
    if (tile == 6) { launch_d<64, 32, AM, BMODE>(p, batch, splits, s); return true; }
  }
  return false;
}

static int g_last_dma = 0;  // the last fp32 sg_ggemm ran f32d_k (tests)
static bool try_dma(const Args& p, int a_kouter, int b_kouter, int batch, int splits, int tile, hipStream_t s) {
  g_last_dma = 0;
  if (g_gg[2] < 0 || !p.vec_a || !p.vec_b || p.K <= 0) return false;
  auto ext = [&](bool kout, int rows, int64_t ld, int64_t sb) {
    return ((kout ? (int64_t)(p.K - 1) * ld + rows : (int64_t)(rows - 1) * ld + p.K) + sb * (batch - 1)) * 4;
  };
  if (ext(a_kouter, p.M, p.lda, p.sa) >= ((int64_t)1 << 31) || ext(b_kouter, p.N, p.ldb, p.sb) >= ((int64_t)1 << 31))
    return false;
  bool ok;
  if (!a_kouter && !b_kouter) ok = launch_dma_t<KMAJ, KMAJ>(p, batch, splits, tile, s);
  else if (!a_kouter && b_kouter) ok = launch_dma_t<KMAJ, KOUT>(p, batch, splits, tile, s);
  else if (a_kouter && !b_kouter) ok = launch_dma_t<KOUT, KMAJ>(p, batch, splits, tile, s);
  else ok = launch_dma_t<KOUT, KOUT>(p, batch, splits, tile, s);
  g_last_dma = ok ? 1 : 0;
  return ok;
}

static inline int kps(int K, int splits) {
  const int nkt = (K + BK - 1) / BK;
  return ((nkt + splits - 1) / splits) * BK;
}

static Geom make_geom(int N, int H, int W, int C, int K, int R, int S, int Ho, int Wo, int sh, int sw, int ph, int pw,
                      int dh, int dw, int groups) {
  Geom g{};
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S; g.Ho = Ho; g.Wo = Wo;
  g.Cg = C / groups; g.Kg = K / groups;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dw;
  g.dCg = FastDiv(g.Cg > 0 ? g.Cg : 1); g.dKg = FastDiv(g.Kg > 0 ? g.Kg : 1); g.dS = FastDiv(S);
  g.dWo = FastDiv(Wo > 0 ? Wo : 1); g.dHoWo = FastDiv(Ho * Wo > 0 ? Ho * Wo : 1);
  g.dW = FastDiv(W > 0 ? W : 1); g.dHW = FastDiv(H * W > 0 ? H * W : 1);
  g.dsh = FastDiv(sh); g.dsw = FastDiv(sw);
  return g;
}

static void check_int(int64_t v, const char* what) {
  if (v >= ((int64_t)1 << 31)) throw std::runtime_error(std::string("ggemm: ") + what + " exceeds 2^31");
}

template <typename T>
static bool aligned(const void* p, int64_t a, int64_t b = 0, int64_t c = 0) {
  return ((uintptr_t)p % (4 * sizeof(T))) == 0 && a % 4 == 0 && b % 4 == 0 && c % 4 == 0;
}

}  // namespace gg
}  // namespace sg

using namespace sg::gg;

extern "C" {
int sg_bn_deterministic();

void sg_ggemm_tune(int key, int value) {
  if (key >= 0 && key < 3) g_gg[key] = value;
}
int sg_ggemm_last_dma() { return g_last_dma; }

// Generic GEMM (dt 0: fp32 operands, 1: bf16 operands):
//   C[batch][M][N] = alpha * A(m, k) B(n, k) (+ beta C) (+ bias[n]) (ReLU)
//   csum (optional, batch 1): csum[n] += sum_k B(n, k) -- a weight-gradient
//   GEMM's bias gradient from the dy tiles it already stages (no extra pass)
//   relu: fused activation of the output (Act codes: 1 relu, 2 sigmoid, 3 tanh,
//   4 stanh); act_x (optional): C *= act'(X), X = the activation output of
//   code act_bwd laid out like C -- a data-gradient GEMM that also takes the
//   producer's activation backward
//   a_kouter = 0: A stored [M][K] (lda), 1: [K][M]; b_kouter = 0: B stored [N][K], 1: [K][N]
//   out_mode 0 bf16, 1 fp32, 2 fp32 atomic (split-K, C pre-initialised)
void sg_ggemm(int dt, const void* a, int64_t lda, int a_kouter, int64_t sa, const void* b, int64_t ldb, int b_kouter,
              int64_t sb, void* c, int64_t ldc, int64_t sc, int M, int N, int K, float alpha, float beta,
              const void* bias, int relu, int out_mode, int splits, int batch, float* csum, int act_bwd,
              const void* act_x, void* aux, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return;
  if (csum && batch != 1) throw std::runtime_error("ggemm: fused column sums need batch 1");
  check_int((int64_t)M * N, "M*N");
  Args p{};
  p.M = M; p.N = N; p.K = K;
  p.a = a; p.lda = lda; p.sa = sa; p.b = b; p.ldb = ldb; p.sb = sb;
  p.c = c; p.ldc = ldc; p.sc = sc; p.alpha = alpha; p.beta = beta; p.bias = (const float*)bias; p.sbias = 0;
  p.relu = relu; p.out_mode = out_mode; p.csum = csum; p.act_x = act_x; p.act_bwd = act_bwd; p.aux = aux;
  const bool f = dt == 0;
  int tile = 0;
  if (f) {
    // plain fp32 output split over K: C zeroed (beta 0) or kept (beta 1) and accumulated atomically
    const bool plain_ok = out_mode == O_F32 && !relu && !act_x && !aux && (beta == 0.f || beta == 1.f);
    const bool can_split = out_mode == O_F32_ATOMIC || plain_ok;
    int sp = 1;
    const bool dma_ops = g_gg[2] >= 0 && aligned<float>(a, lda, sa, a_kouter ? M : K) &&
                         aligned<float>(b, ldb, sb, b_kouter ? N : K);
    pick_f32(M, N, K, batch, can_split, out_mode == O_F32 && beta == 0.f, tile, sp,
             dma_ops && g_gg[2] == 0 ? 1 + (a_kouter ? 2 : 0) + (b_kouter ? 4 : 0) : 0);
    if (g_gg[0] > 0) tile = g_gg[0];
    if (sg_bn_deterministic()) sp = 1;  // split-K atomics add in arbitrary order
    if (g_gg[1] != 0) sp = g_gg[1] > 1 && K >= 2 * BK * g_gg[1] ? g_gg[1] : 1;
    if (out_mode == O_F32_ATOMIC && splits > 0) sp = splits;  // caller's explicit count
    if (!can_split) sp = 1;
    if (out_mode == O_F32 && sp > 1) {
      if (beta == 0.f) hipLaunchKernelGGL(zero_rows_k, dim3(M, batch), dim3(256), 0, s, (float*)c, ldc, sc, N);
      out_mode = p.out_mode = O_F32_ATOMIC;
    }
    splits = sp;
  } else if (out_mode == O_F32_ATOMIC) {
    const int bm = big_tile(M, N) ? 128 : 64;
    splits = pick_splits(M, N, K, batch, splits, bm, bm);
  } else {
    splits = 1;
  }
  p.k_per_split = kps(K > 0 ? K : 1, splits);
  if (out_mode == O_F32_ATOMIC && splits == 1) {
    // one writer per output element: accumulate with a plain read-add-store
    // (C = alpha AB + 1 * C) instead of scattered fp32 atomics
    p.out_mode = O_F32;
    p.beta = 1.f;
  }
  p.g = make_geom(1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 1);
  p.vec_a = f ? aligned<float>(a, lda, sa, a_kouter ? M : K) : aligned<sg::bf16>(a, lda, sa, a_kouter ? M : K);
  p.vec_b = f ? aligned<float>(b, ldb, sb, b_kouter ? N : K) : aligned<sg::bf16>(b, ldb, sb, b_kouter ? N : K);
  if (f && try_dma(p, a_kouter, b_kouter, batch, splits, tile, s)) return;
  if (f) {
    if (!a_kouter && !b_kouter) launch_f32<KMAJ, KMAJ>(p, batch, splits, tile, s);
    else if (!a_kouter && b_kouter) launch_f32<KMAJ, KOUT>(p, batch, splits, tile, s);
    else if (a_kouter && !b_kouter) launch_f32<KOUT, KMAJ>(p, batch, splits, tile, s);
    else launch_f32<KOUT, KOUT>(p, batch, splits, tile, s);
  } else {
    if (!a_kouter && !b_kouter) launch<sg::bf16, KMAJ, KMAJ>(p, batch, splits, s);
    else if (!a_kouter && b_kouter) launch<sg::bf16, KMAJ, KOUT>(p, batch, splits, s);
    else if (a_kouter && !b_kouter) launch<sg::bf16, KOUT, KMAJ>(p, batch, splits, s);
    else launch<sg::bf16, KOUT, KOUT>(p, batch, splits, s);
  }
}

// Convolution forward, NHWC activations, weights [K][R][S][C/groups]:
//   y[N*Ho*Wo][K] = conv(x, w) (+ bias) (ReLU); out_mode 0 bf16 / 1 fp32
void sg_gconv_fwd(int dt, const void* x, const void* w, void* y, const void* bias, int N, int H, int W, int C, int K,
                  int R, int S, int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int relu,
                  int out_mode, hipStream_t s) {
  Args p{};
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups);
  const Geom& g = p.g;
  check_int((int64_t)N * H * W * C, "input");
  check_int((int64_t)N * Ho * Wo * K, "output");
  p.M = N * Ho * Wo; p.N = g.Kg; p.K = R * S * g.Cg;
  p.a = x; p.lda = 0; p.sa = g.Cg;  // group g reads channels [g*Cg, (g+1)*Cg)
  p.b = w; p.ldb = (int64_t)R * S * g.Cg; p.sb = (int64_t)g.Kg * R * S * g.Cg;
  p.c = y; p.ldc = K; p.sc = g.Kg;
  p.alpha = 1.f; p.beta = 0.f; p.bias = (const float*)bias; p.sbias = g.Kg; p.relu = relu; p.out_mode = out_mode;
  p.k_per_split = kps(p.K > 0 ? p.K : 1, 1);
  const bool f = dt == 0;
  p.vec_a = (f ? aligned<float>(x, C, g.Cg) : aligned<sg::bf16>(x, C, g.Cg)) ? 1 : 0;
  p.vec_b = (f ? aligned<float>(w, p.ldb, p.sb, p.K) : aligned<sg::bf16>(w, p.ldb, p.sb, p.K)) ? 1 : 0;
  if (f) launch<float, CFWD_A, KMAJ>(p, groups, 1, s);
  else launch<sg::bf16, CFWD_A, KMAJ>(p, groups, 1, s);
}

// Convolution data gradient: dx[N*H*W][C] (= | += beta *) dgrad(dy[N*Ho*Wo][K], w)
void sg_gconv_dgrad(int dt, const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S,
                    int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int out_mode,
                    float beta, hipStream_t s) {
  Args p{};
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups);
  const Geom& g = p.g;
  check_int((int64_t)N * H * W * C, "input");
  check_int((int64_t)N * Ho * Wo * K, "output");
  p.M = N * H * W; p.N = g.Cg; p.K = R * S * g.Kg;
  p.a = dy; p.lda = 0; p.sa = g.Kg;
  p.b = w; p.ldb = 0; p.sb = (int64_t)g.Kg * R * S * g.Cg;
  p.c = dx; p.ldc = C; p.sc = g.Cg;
  p.alpha = 1.f; p.beta = beta; p.bias = nullptr; p.relu = 0; p.out_mode = out_mode;
  p.k_per_split = kps(p.K > 0 ? p.K : 1, 1);
  const bool f = dt == 0;
  p.vec_a = (f ? aligned<float>(dy, K, g.Kg) : aligned<sg::bf16>(dy, K, g.Kg)) ? 1 : 0;
  p.vec_b = (f ? aligned<float>(w, g.Cg, p.sb) : aligned<sg::bf16>(w, g.Cg, p.sb)) ? 1 : 0;
  if (f) launch<float, DGRAD_A, DGRAD_B>(p, groups, 1, s);
  else launch<sg::bf16, DGRAD_A, DGRAD_B>(p, groups, 1, s);
}

// Convolution weight gradient: dw[K][R][S][C/groups] (fp32) += dy^T im2col(x)
// (split over the pixel reduction with fp32 atomics; the caller zeroes dw
// unless accumulating)
void sg_gconv_wgrad(int dt, const void* x, const void* dy, void* dw_out, int N, int H, int W, int C, int K, int R,
                    int S, int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int splits,
                    hipStream_t s) {
  Args p{};
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups);
  const Geom& g = p.g;
  check_int((int64_t)N * H * W * C, "input");
  check_int((int64_t)N * Ho * Wo * K, "output");
  p.M = g.Kg; p.N = R * S * g.Cg; p.K = N * Ho * Wo;
  p.a = dy; p.lda = K; p.sa = g.Kg;  // A(row = ko, k = pixel) = dy[pixel][g*Kg + ko]: K-outer
  p.b = x; p.ldb = 0; p.sb = g.Cg;
  p.c = dw_out; p.ldc = (int64_t)R * S * g.Cg; p.sc = (int64_t)g.Kg * R * S * g.Cg;
  p.alpha = 1.f; p.beta = 0.f; p.bias = nullptr; p.relu = 0; p.out_mode = O_F32_ATOMIC;
  {
    const int bm = big_tile(p.M, p.N, dt == 0) ? 128 : 64;
    splits = pick_splits(p.M, p.N, p.K, groups, splits, bm, bm);
  }
  p.k_per_split = kps(p.K > 0 ? p.K : 1, splits);
  if (splits == 1) {  // single writer: read-add-store accumulation (see sg_ggemm)
    p.out_mode = O_F32;
    p.beta = 1.f;
  }
  const bool f = dt == 0;
  p.vec_a = (f ? aligned<float>(dy, K, g.Kg, p.M) : aligned<sg::bf16>(dy, K, g.Kg, p.M)) ? 1 : 0;
  p.vec_b = (f ? aligned<float>(x, C, g.Cg) : aligned<sg::bf16>(x, C, g.Cg)) ? 1 : 0;
  if (f) launch<float, KOUT, WGRAD_B>(p, groups, splits, s);
  else launch<sg::bf16, KOUT, WGRAD_B>(p, groups, splits, s);
}

}  // extern "C"

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
  int out_phase;       // dgrad: output rows map through the phase grid
  ConvGeom g;
};

__device__ __forceinline__ int kmajor_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
template <int ROWS>
__device__ __forceinline__ int kouter_swz(int krow, int chunk) {
  if constexpr (ROWS == 128) return chunk ^ (((krow & 3) << 2) | ((krow >> 2) & 3));
  else return chunk ^ ((((krow >> 1) & 1) << 1) | (((krow >> 3) & 1) << 2));
}

__device__ __forceinline__ uint4 sel(bool ok, uint4 v) { return ok ? v : make_uint4(0, 0, 0, 0); }

// ------------------------------------------------------------------------------
// Operand loader: ROWS = tile rows of this operand, VPT 16-byte vectors/thread.
// KMAJOR kinds: thread t owns rows (t>>3)+32v, k-chunk t&7.
// KOUTER kinds: thread t owns k-rows t/CPR + (256/CPR)v, col chunk t%CPR.
// ------------------------------------------------------------------------------
template <int ROWS, int MODE>
struct Loader {
  static constexpr int VPT = ROWS / 32;
  static constexpr bool KOUT = (MODE == LM_KOUTER || MODE == LM_WGRAD_B || MODE == LM_DGRAD_B);
  static constexpr int CPR = ROWS / 8;  // KOUTER: chunks per k-row
  static constexpr int KRP = NT / CPR;  // KOUTER: k-rows per pass
  int64_t base[VPT];
  int i0[VPT], j0[VPT];
  bool ok[VPT];
  int64_t ld;
  int cr, cs, cc;  // WGRAD_B: fixed column decomposition
  bool cok;

  __device__ __forceinline__ void init(const GemmArgs& p, int row0, int nrows, const Phase& P, int64_t ld_) {
    const int t = threadIdx.x;
    ld = ld_;
    if constexpr (!KOUT) {
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int row = row0 + (t >> 3) + 32 * v;
        ok[v] = row < nrows;
        const int rr = ok[v] ? row : 0;
        if constexpr (MODE == LM_KMAJOR) {
          base[v] = (int64_t)rr * ld;
        } else if constexpr (MODE == LM_CONV_FWD) {
          const ConvGeom& g = p.g;
          const int n = g.dHoWo.div(rr);
          const int rem = rr - n * g.Ho * g.Wo;
          const int oh = g.dWo.div(rem);
          const int ow = rem - oh * g.Wo;
          base[v] = (int64_t)n * g.H * g.W * g.C;
          i0[v] = oh * g.sh - g.ph;
          j0[v] = ow * g.sw - g.pw;
        } else {  // LM_DGRAD_A: row = (n, hh, ww) of the phase grid
          const ConvGeom& g = p.g;
          const int n = P.dHpWp.div(rr);
          const int rem = rr - n * P.Hp * P.Wp;
          const int hh = P.dWp.div(rem);
          const int ww = rem - hh * P.Wp;
          base[v] = (int64_t)n * g.Ho * g.Wo * g.K;
          i0[v] = hh + P.offh;
          j0[v] = ww + P.offw;
        }
      }
    } else if constexpr (MODE == LM_WGRAD_B) {
      const ConvGeom& g = p.g;
      const int col = row0 + (t % CPR) * 8;  // gemm column n = (r, s, c)
      cok = col < nrows;
      const int c2 = cok ? col : 0;
      const int rs = g.dC.div(c2);
      cc = c2 - rs * g.C;
      cr = g.dS.div(rs);
      cs = rs - cr * g.S;
    }
  }

  // Fetch the K-tile starting at k0 (absolute) into registers.
  __device__ __forceinline__ void fetch(uint4 (&rg)[VPT], const GemmArgs& p, const bf16* __restrict__ src,
                                        int row0, int nrows, int k0, int kend, const Phase& P) const {
    const int t = threadIdx.x;
    if constexpr (MODE == LM_KMAJOR) {
      const int kk = k0 + (t & 7) * 8;
      const bool kin = kk < kend;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const bool o = ok[v] && kin;
        rg[v] = sel(o, *(const uint4*)(src + (o ? base[v] + kk : 0)));
      }
    } else if constexpr (MODE == LM_CONV_FWD) {
      const ConvGeom& g = p.g;
      int kk = k0 + (t & 7) * 8;
      const bool kin = kk < kend;
      kk = kin ? kk : 0;
      int tap, c0;
      if ((g.C & 63) == 0) {  // wave-uniform tap
        tap = g.dC.div(k0);
        c0 = kk - tap * g.C;
      } else {
        tap = g.dC.div(kk);
        c0 = kk - tap * g.C;
      }
      const int r = g.dS.div(tap), s = tap - r * g.S;
      const int dr = r * g.dh, ds = s * g.dw;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int ih = i0[v] + dr, iw = j0[v] + ds;
        const bool o = ok[v] && kin && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const int64_t off = base[v] + ((int64_t)ih * g.W + iw) * g.C + c0;
        rg[v] = sel(o, *(const uint4*)(src + (o ? off : 0)));
      }
    } else if constexpr (MODE == LM_DGRAD_A) {
      const ConvGeom& g = p.g;
      int kk = k0 + (t & 7) * 8;
      const bool kin = kk < kend;
      kk = kin ? kk : 0;
      int tap, k;
      if ((g.K & 63) == 0) {
        tap = g.dK.div(k0);
        k = kk - tap * g.K;
      } else {
        tap = g.dK.div(kk);
        k = kk - tap * g.K;
      }
      const int j = P.dns.div(tap), i = tap - j * P.ns;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int oh = i0[v] - j, ow = j0[v] - i;
        const bool o = ok[v] && kin && (unsigned)oh < (unsigned)g.Ho && (unsigned)ow < (unsigned)g.Wo;
        const int64_t off = base[v] + ((int64_t)oh * g.Wo + ow) * g.K + k;
        rg[v] = sel(o, *(const uint4*)(src + (o ? off : 0)));
      }
    } else if constexpr (MODE == LM_KOUTER) {
      const int col = row0 + (t % CPR) * 8;
      const bool cin = col < nrows;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int kr = k0 + t / CPR + KRP * v;
        const bool o = cin && kr < kend;
        rg[v] = sel(o, *(const uint4*)(src + (o ? (int64_t)kr * ld + col : 0)));
      }
    } else if constexpr (MODE == LM_DGRAD_B) {
      // B(n = c, kk = (tap, k)) = W[k][r][s][c]; rows c contiguous per (k, tap)
      const ConvGeom& g = p.g;
      const int col = row0 + (t % CPR) * 8;
      const bool cin = col < nrows;
      const int RSC = g.R * g.S * g.C;
      const bool uni = (g.K & 63) == 0;
      const int tapu = g.dK.div(k0);
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        int kk = k0 + t / CPR + KRP * v;
        const bool kin = kk < kend;
        kk = kin ? kk : 0;
        const int tap = uni ? tapu : (int)g.dK.div(kk);
        const int k = kk - tap * g.K;
        const int j = P.dns.div(tap), i = tap - j * P.ns;
        const int r = P.r0 + g.sh * j, s = P.s0 + g.sw * i;
        const bool o = cin && kin;
        const int64_t off = (int64_t)k * RSC + (r * g.S + s) * g.C + col;
        rg[v] = sel(o, *(const uint4*)(src + (o ? off : 0)));
      }
    } else if constexpr (MODE == LM_WGRAD_B) {
      const ConvGeom& g = p.g;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int pix = k0 + t / CPR + KRP * v;  // output pixel (n, oh, ow)
        bool o = cok && pix < kend;
        const int pp = o ? pix : 0;
        const int n = g.dHoWo.div(pp);
        const int rem = pp - n * g.Ho * g.Wo;
        const int oh = g.dWo.div(rem);
        const int ow = rem - oh * g.Wo;
        const int ih = oh * g.sh - g.ph + cr * g.dh;
        const int iw = ow * g.sw - g.pw + cs * g.dw;
        o = o && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const int64_t off = (((int64_t)n * g.H + ih) * g.W + iw) * g.C + cc;
        rg[v] = sel(o, *(const uint4*)(src + (o ? off : 0)));
      }
    }
  }

  __device__ __forceinline__ void store(const uint4 (&rg)[VPT], char* lds) const {
    const int t = threadIdx.x;
    if constexpr (KOUT) {
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int kr = t / CPR + KRP * v, ch = t % CPR;
        *(uint4*)(lds + kr * (ROWS * 2) + kouter_swz<ROWS>(kr, ch) * 16) = rg[v];
      }
    } else {
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const int row = (t >> 3) + 32 * v, ch = t & 7;
        *(uint4*)(lds + row * 128 + kmajor_swz(row, ch) * 16) = rg[v];
      }
    }
  }

  // 16x32 fragment (rows r0..r0+15, k = kk*32..+31) for MFMA lane l
  __device__ __forceinline__ bf16x8 frag(const char* lds, int r0, int kk) const {
    const int l = threadIdx.x & 63;
    if constexpr (KOUT) {
      const int g = l >> 4, i = l & 15;
      const int q = i >> 2, pp = i & 3;
      const int col = r0 + 4 * pp;
      const int ch = col >> 3, within = (col & 7) * 2;
      const int kb0 = kk * 32 + 8 * g + q, kb1 = kb0 + 4;
      typedef short v4s __attribute__((ext_vector_type(4)));
      const char* a0 = lds + kb0 * (ROWS * 2) + kouter_swz<ROWS>(kb0, ch) * 16 + within;
      const char* a1 = lds + kb1 * (ROWS * 2) + kouter_swz<ROWS>(kb1, ch) * 16 + within;
      v4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a0));
      v4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a1));
      i16x8 r;
      r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
      r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
      return __builtin_bit_cast(bf16x8, r);
    } else {
      const int row = r0 + (l & 15);
      const int ch = kk * 4 + (l >> 4);
      return *(const bf16x8*)(lds + row * 128 + kmajor_swz(row, ch) * 16);
    }
  }
};

template <int BM, int BN, int AM, int BMODE, int OUT>
__global__ void __launch_bounds__(NT, 2) igemm_k(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 MFMA tiles per wave

  const bf16* __restrict__ pa = p.a + (int64_t)blockIdx.y * p.sa;
  const bf16* __restrict__ pb = p.b + (int64_t)blockIdx.y * p.sb;
  char* pc = (char*)p.c + (int64_t)blockIdx.y * p.sc * (OUT == OUT_BF16 ? 2 : 4);
  // dgrad: phase from blockIdx.z (the output rows are that phase's pixels)
  const int phase = p.out_phase ? (int)blockIdx.z : 0;
  const Phase& P = p.g.phs[phase];
  const int M = p.out_phase ? p.g.N * P.Hp * P.Wp : p.M;
  const int K = p.out_phase ? P.nr * P.ns * p.g.K : p.K;

  // XCD-aware bijective remap, then bands of 8 tile-rows for L2 reuse of B
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
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

  const int kbeg = p.out_phase ? 0 : (int)blockIdx.z * p.k_per_split;
  const int kend = p.out_phase ? K : min(K, kbeg + p.k_per_split);
  if (OUT == OUT_F32_ATOMIC && kbeg >= kend) return;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  Loader<BM, AM> la;
  Loader<BN, BMODE> lb;
  la.init(p, m0, M, P, p.lda);
  lb.init(p, n0, p.N, P, p.ldb);

  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    uint4 ra[Loader<BM, AM>::VPT], rb[Loader<BN, BMODE>::VPT];
    la.fetch(ra, p, pa, m0, M, kbeg, kend, P);
    lb.fetch(rb, p, pb, n0, p.N, kbeg, kend, P);
    la.store(ra, smem);
    lb.store(rb, smem + A_BYTES);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) {
        la.fetch(ra, p, pa, m0, M, kbeg + (kt + 1) * BK, kend, P);
        lb.fetch(rb, p, pb, n0, p.N, kbeg + (kt + 1) * BK, kend, P);
      }
      const char* sa = smem + cur * STAGE;
      const char* sb = sa + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = la.frag(sa, wm * (BM / 2) + i * 16, kk);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = lb.frag(sb, wn * (BN / 2) + j * 16, kk);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
      if (more) {
        char* nxt = smem + (cur ^ 1) * STAGE;
        la.store(ra, nxt);
        lb.store(rb, nxt + A_BYTES);
      }
      __syncthreads();
    }
  }

  // Epilogue.  acc[i][j] = D[n][m]: lane col m = l&15, rows n = (l>>4)*4+r.
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / 2) + i * 16 + (l & 15);
    if (m >= M) continue;
    int64_t rowoff;
    if (p.out_phase) {
      const ConvGeom& g = p.g;
      const int n = P.dHpWp.div(m);
      const int rem = m - n * P.Hp * P.Wp;
      const int hh = P.dWp.div(rem);
      const int ww = rem - hh * P.Wp;
      rowoff = (((int64_t)n * g.H + P.a + g.sh * hh) * g.W + P.b + g.sw * ww) * p.ldc;
    } else {
      rowoff = (int64_t)m * p.ldc;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + (l >> 4) * 4;
      if (n >= p.N) continue;
      float v[4] = {acc[i][j][0] * p.alpha, acc[i][j][1] * p.alpha, acc[i][j][2] * p.alpha,
                    acc[i][j][3] * p.alpha};
      const bool full = n + 3 < p.N;
      if (OUT == OUT_F32_ATOMIC) {
        float* c = (float*)pc + rowoff + n;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (full || n + r < p.N) atomicAdd(c + r, v[r]);
        continue;
      }
      if (p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (full || n + r < p.N) ? p.bias[n + r] : 0.f;
      }
      if (OUT == OUT_F32) {
        float* c = (float*)pc + rowoff + n;
        if (p.beta != 0.f) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (full || n + r < p.N) v[r] += p.beta * c[r];
        }
        if (p.relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (full && ((p.ldc & 3) == 0)) *(float4*)c = make_float4(v[0], v[1], v[2], v[3]);
        else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) c[r] = v[r];
        }
      } else {
        bf16* c = (bf16*)pc + rowoff + n;
        if (p.beta != 0.f) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (full || n + r < p.N) v[r] += p.beta * (float)c[r];
        }
        if (p.relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (full && ((p.ldc & 3) == 0)) {
          bf16x4 o;
          o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
          *(bf16x4*)c = o;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) c[r] = (bf16)v[r];
        }
      }
    }
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

template <int BM, int BN, int AM, int BMODE, int OUT>
static void launch_t(const GemmArgs& p, int tiles, int ydim, int zdim, hipStream_t s) {
  dim3 grid(tiles, ydim, zdim), block(NT);
  constexpr int lds = 2 * (BM + BN) * BK * 2;
  hipLaunchKernelGGL((igemm_k<BM, BN, AM, BMODE, OUT>), grid, block, lds, s, p);
}

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
static void launch(const GemmArgs& p, int M, int splits, hipStream_t s, int batch, int zdim) {
  int BM, BN;
  pick_tile(M, p.N, BM, BN);
  const int tiles = ((M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int z = zdim > 0 ? zdim : splits;
  if (BM == 128 && BN == 128) launch_t<128, 128, AM, BMODE, OUT>(p, tiles, batch, z, s);
  else if (BM == 128 && BN == 64) launch_t<128, 64, AM, BMODE, OUT>(p, tiles, batch, z, s);
  else if (BM == 64 && BN == 128) launch_t<64, 128, AM, BMODE, OUT>(p, tiles, batch, z, s);
  else launch_t<64, 64, AM, BMODE, OUT>(p, tiles, batch, z, s);
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

extern "C" {

// Plain GEMM: C[M][N] = alpha * sum_k A(m,k) B(n,k) (+ beta*C) ... with
//   a_kouter = 0: A stored [M][K] (lda), 1: A stored [K][M]
//   b_kouter = 0: B stored [N][K] (ldb), 1: B stored [K][N]
// out_mode 0 bf16, 1 f32, 2 f32 atomic (split-K, C pre-initialised).
void sg_gemm(const void* a, int64_t lda, int a_kouter, const void* b, int64_t ldb, int b_kouter, void* c,
             int64_t ldc, int M, int N, int K, float alpha, float beta, const void* bias, int relu, int out_mode,
             int splits, int batch, int64_t sa, int64_t sb, int64_t sc, hipStream_t s) {
  GemmArgs p{};
  init_phase_identity(p.g);
  p.sa = sa; p.sb = sb; p.sc = sc;
  p.M = M; p.N = N; p.K = K; p.a = (const bf16*)a; p.lda = lda; p.b = (const bf16*)b; p.ldb = ldb;
  p.c = c; p.ldc = ldc; p.alpha = alpha; p.beta = beta; p.bias = (const float*)bias; p.relu = relu;
  splits = (out_mode == OUT_F32_ATOMIC) ? pick_splits(M, N, K, splits) : 1;
  p.k_per_split = kps(K, splits);
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
                 hipStream_t s) {
  GemmArgs p{};
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw);
  p.M = N * Ho * Wo; p.N = K; p.K = R * S * C;
  p.a = (const bf16*)x; p.lda = 0; p.b = (const bf16*)w; p.ldb = R * S * C;
  p.c = y; p.ldc = K; p.alpha = 1.f; p.beta = 0.f; p.bias = (const float*)bias; p.relu = relu;
  p.k_per_split = kps(p.K, 1);
  if (out_mode == OUT_F32) launch<LM_CONV_FWD, LM_KMAJOR, OUT_F32>(p, p.M, 1, s, 1, 0);
  else launch<LM_CONV_FWD, LM_KMAJOR, OUT_BF16>(p, p.M, 1, s, 1, 0);
}

// conv data gradient: dy [N*Ho*Wo][K] bf16, w [K][R][S][C] bf16 -> dx [N*H*W][C]
// (dilation 1; stride phases on blockIdx.z)
void sg_conv_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int K, int R, int S, int Ho,
                   int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, hipStream_t s) {
  GemmArgs p{};
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw);
  const int np = make_phases(p.g);
  int Mmax = 0;
  for (int i = 0; i < np; ++i) Mmax = Mmax > N * p.g.phs[i].Hp * p.g.phs[i].Wp ? Mmax : N * p.g.phs[i].Hp * p.g.phs[i].Wp;
  p.M = Mmax; p.N = C; p.K = R * S * K;
  p.a = (const bf16*)dy; p.lda = 0; p.b = (const bf16*)w; p.ldb = 0;
  p.c = dx; p.ldc = C; p.alpha = 1.f; p.beta = 0.f; p.bias = nullptr; p.relu = 0;
  p.out_phase = 1;
  p.k_per_split = kps(p.K, 1);
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
  splits = pick_splits(p.M, p.N, p.K, splits);
  p.k_per_split = kps(p.K, splits);
  launch<LM_KOUTER, LM_WGRAD_B, OUT_F32_ATOMIC>(p, p.M, splits, s, 1, 0);
}

}  // extern "C"

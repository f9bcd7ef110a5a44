// MFMA implicit-GEMM kernel family for gfx950: plain GEMM (any operand
// orientation), convolution forward, data-gradient and weight-gradient, all
// bf16 inputs with fp32 accumulation on v_mfma_f32_16x16x32_bf16.
//
// Replaces the reference's per-sample im2col + sgemm convolution
// (ConvolutionLayer, src/worker/layer.cc:63-123: unpack_patch2col F3,
// pack_col2patch F4, gW += dot(grad, col.T()) F5) and the DotEngine GEMMs
// (include/mshadow/tensor_expr_engine-inl.hpp:339-383): no column buffer is
// materialised; the operand loaders gather im2col tiles straight from the
// NHWC activation tensor into LDS.
//
//   C[m][n] (=|+=) alpha * sum_k A(m, k) * B(n, k)  (+ bias[n]) (ReLU)
//
// Tile 128x128x64, 256 threads = 4 waves in a 2x2 arrangement, each wave a
// 64x64 sub-tile of 4x4 MFMA 16x16x32 tiles.  Operands are staged through
// registers into a double-buffered LDS image (one barrier per K-tile, global
// loads for tile k+1 issued before the MFMAs of tile k: cdna_hip_programming
// T14).  Each operand is one of two LDS image kinds:
//   KMAJOR  [rows][64 k], 128-B rows, fragment = one ds_read_b128, chunk
//           XOR-swizzled with (row>>1)&7 (conflict-free for the b128 lane
//           groups);
//   KOUTER  [64 k][128 rows], 256-B rows, fragment = two ds_read_b64_tr_b16
//           (hardware transpose), chunk XOR-swizzled with T10 pattern (b).
// The MFMA is issued with the B fragment as its A operand so each lane ends
// with 4 consecutive n-columns of one output row: 8/16-byte epilogue stores.
#include "common.h"

namespace sg {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;

enum LoadMode : int { LM_KMAJOR = 0, LM_KOUTER = 1, LM_CONV_FWD = 2, LM_CONV_DGRAD = 3, LM_CONV_WGRAD = 4 };
enum OutMode : int { OUT_BF16 = 0, OUT_F32 = 1, OUT_F32_ATOMIC = 2 };

struct ConvGeom {
  int N, H, W, C;      // input (NHWC)
  int K, R, S;         // filters [K][R][S][C]
  int Ho, Wo;          // output
  int sh, sw, ph, pw, dh, dw;
  FastDiv dC, dS, dK, dWo, dHoWo, dW, dHW;
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
  int k_per_split;  // multiple of BK
  int64_t sa, sb, sc;  // batch strides (elements), blockIdx.y = batch
  ConvGeom g;
};

__device__ __forceinline__ int kmajor_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
__device__ __forceinline__ int kouter_swz(int krow, int chunk) {
  return chunk ^ (((krow & 3) << 2) | ((krow >> 2) & 3));
}

// ---- per-thread loader state -------------------------------------------------
// KMAJOR-kind loaders: thread t owns rows (t>>3) + 32*v, k-chunk (t&7).
// KOUTER-kind loaders: thread t owns k-rows (t>>4) + 16*v, col-chunk (t&15).
struct LoadState {
  int64_t base[4];  // per-row base offset (elements) or image offset
  int i0[4], j0[4]; // conv: ih0/iw0 (fwd), h+ph / w+pw (dgrad)
  bool ok[4];
  // KOUTER conv (wgrad) column info
  int cr, cs, cc;
  bool cok;
};

template <int MODE>
__device__ __forceinline__ void loader_init(LoadState& st, const GemmArgs& p, int tile_row0, int nrows) {
  const int t = threadIdx.x;
  if constexpr (MODE == LM_KMAJOR || MODE == LM_CONV_FWD || MODE == LM_CONV_DGRAD) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = tile_row0 + (t >> 3) + 32 * v;
      st.ok[v] = row < nrows;
      const int rr = st.ok[v] ? row : 0;
      if constexpr (MODE == LM_KMAJOR) {
        st.base[v] = (int64_t)rr;
      } else if constexpr (MODE == LM_CONV_FWD) {
        const ConvGeom& g = p.g;
        int n = g.dHoWo.div(rr);
        int rem = rr - n * g.Ho * g.Wo;
        int oh = g.dWo.div(rem);
        int ow = rem - oh * g.Wo;
        st.base[v] = (int64_t)n * g.H * g.W * g.C;
        st.i0[v] = oh * g.sh - g.ph;
        st.j0[v] = ow * g.sw - g.pw;
      } else {  // CONV_DGRAD: row = (n, h, w) of dx
        const ConvGeom& g = p.g;
        int n = g.dHW.div(rr);
        int rem = rr - n * g.H * g.W;
        int h = g.dW.div(rem);
        int w = rem - h * g.W;
        st.base[v] = (int64_t)n * g.Ho * g.Wo * g.K;
        st.i0[v] = h + g.ph;
        st.j0[v] = w + g.pw;
      }
    }
  } else if constexpr (MODE == LM_CONV_WGRAD) {
    const ConvGeom& g = p.g;
    const int col = tile_row0 + (t & 15) * 8;  // gemm column n = (r, s, c)
    st.cok = col < nrows;
    const int cc = st.cok ? col : 0;
    int rs = g.dC.div(cc);
    st.cc = cc - rs * g.C;
    st.cr = g.dS.div(rs);
    st.cs = rs - st.cr * g.S;
  }
}

// Load the 4 16-byte vectors of K-tile starting at k0 into regs.
template <int MODE>
__device__ __forceinline__ void loader_fetch(uint4 (&rg)[4], const LoadState& st, const GemmArgs& p,
                                             const bf16* __restrict__ src, int64_t ld, int tile_row0, int nrows,
                                             int k0, int kend) {
  const int t = threadIdx.x;
  const uint4 z = make_uint4(0, 0, 0, 0);
  if constexpr (MODE == LM_KMAJOR) {
    const int kk = k0 + (t & 7) * 8;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      rg[v] = (st.ok[v] && kk < kend) ? *(const uint4*)(src + st.base[v] * ld + kk) : z;
    }
  } else if constexpr (MODE == LM_CONV_FWD) {
    const ConvGeom& g = p.g;
    const int kk = k0 + (t & 7) * 8;
    const bool kin = kk < kend;
    int rs = g.dC.div(kin ? kk : 0);
    int c0 = (kin ? kk : 0) - rs * g.C;
    int r = g.dS.div(rs);
    int s = rs - r * g.S;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      int ih = st.i0[v] + r * g.dh, iw = st.j0[v] + s * g.dw;
      bool ok = st.ok[v] && kin && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      rg[v] = ok ? *(const uint4*)(src + st.base[v] + ((int64_t)ih * g.W + iw) * g.C + c0) : z;
    }
  } else if constexpr (MODE == LM_CONV_DGRAD) {
    const ConvGeom& g = p.g;
    const int kk = k0 + (t & 7) * 8;  // (r, s, k) with k fastest
    const bool kin = kk < kend;
    int rs = g.dK.div(kin ? kk : 0);
    int k = (kin ? kk : 0) - rs * g.K;
    int r = g.dS.div(rs);
    int s = rs - r * g.S;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      int hn = st.i0[v] - r * g.dh, wn = st.j0[v] - s * g.dw;
      int oh = hn / g.sh, ow = wn / g.sw;
      bool ok = st.ok[v] && kin && hn >= 0 && wn >= 0 && oh * g.sh == hn && ow * g.sw == wn && oh < g.Ho &&
                ow < g.Wo;
      rg[v] = ok ? *(const uint4*)(src + st.base[v] + ((int64_t)oh * g.Wo + ow) * g.K + k) : z;
    }
  } else if constexpr (MODE == LM_KOUTER) {
    const int col = tile_row0 + (t & 15) * 8;
    const bool cok = col < nrows;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int kr = k0 + (t >> 4) + 16 * v;
      rg[v] = (cok && kr < kend) ? *(const uint4*)(src + (int64_t)kr * ld + col) : z;
    }
  } else if constexpr (MODE == LM_CONV_WGRAD) {
    const ConvGeom& g = p.g;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int pix = k0 + (t >> 4) + 16 * v;  // output pixel (n, oh, ow)
      bool ok = st.cok && pix < kend;
      const int pp = ok ? pix : 0;
      int n = g.dHoWo.div(pp);
      int rem = pp - n * g.Ho * g.Wo;
      int oh = g.dWo.div(rem);
      int ow = rem - oh * g.Wo;
      int ih = oh * g.sh - g.ph + st.cr * g.dh;
      int iw = ow * g.sw - g.pw + st.cs * g.dw;
      ok = ok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      rg[v] = ok ? *(const uint4*)(src + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + st.cc) : z;
    }
  }
}

template <int MODE>
__device__ __forceinline__ void loader_store(const uint4 (&rg)[4], char* lds) {
  const int t = threadIdx.x;
  if constexpr (MODE == LM_KOUTER || MODE == LM_CONV_WGRAD) {
    // [64 k][128 rows] bf16: 256 B per k-row, 16 chunks
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int kr = (t >> 4) + 16 * v, ch = t & 15;
      *(uint4*)(lds + kr * 256 + kouter_swz(kr, ch) * 16) = rg[v];
    }
  } else {
    // [128 rows][64 k] bf16: 128 B per row, 8 chunks
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = (t >> 3) + 32 * v, ch = t & 7;
      *(uint4*)(lds + row * 128 + kmajor_swz(row, ch) * 16) = rg[v];
    }
  }
}

// Read the 16x32 fragment (rows r0..r0+15, k = kk*32 .. +31) for MFMA lane l.
template <int MODE>
__device__ __forceinline__ bf16x8 frag_read(const char* lds, int r0, int kk) {
  const int l = threadIdx.x & 63;
  if constexpr (MODE == LM_KOUTER || MODE == LM_CONV_WGRAD) {
    const int g = l >> 4, i = l & 15;
    const int q = i >> 2, pp = i & 3;
    // lane 4q+p supplies row (k) kb+q, columns col0 + 4p .. +3
    const int col = r0 + 4 * pp;
    const int ch = col >> 3, within = (col & 7) * 2;
    const int kb0 = kk * 32 + 8 * g + q, kb1 = kb0 + 4;
    typedef short v4s __attribute__((ext_vector_type(4)));
    const char* a0 = lds + kb0 * 256 + kouter_swz(kb0, ch) * 16 + within;
    const char* a1 = lds + kb1 * 256 + kouter_swz(kb1, ch) * 16 + within;
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

template <int AM, int BMODE, int OUT>
__global__ void __launch_bounds__(NT, 2) igemm_k(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (blockIdx.y) {
    p.a += blockIdx.y * p.sa;
    p.b += blockIdx.y * p.sb;
    p.c = (char*)p.c + blockIdx.y * p.sc * (OUT == OUT_BF16 ? 2 : 4);
  }
  constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand per stage
  // stage s: A at smem + s*2*TILE, B at smem + s*2*TILE + TILE
#define LA(st) (smem + (st) * 2 * TILE_BYTES)
#define LB(st) (smem + (st) * 2 * TILE_BYTES + TILE_BYTES)

  // XCD-aware remap of the (m, n) tile grid: consecutive logical tiles land on
  // the same XCD (blocks b and b+8 share one under round-robin dispatch).
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    bid = base + (bid >> 3);
  }
  // group tiles along m in bands of 8 for L2 reuse of B
  const int band = 8;
  const int group = bid / (band * tiles_n);
  const int first_m = group * band;
  const int gm = min(tiles_m - first_m, band);
  const int tm = first_m + (bid % (band * tiles_n)) % gm;
  const int tn = (bid % (band * tiles_n)) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = blockIdx.z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  if (kbeg >= kend) return;
  const int nk = (kend - kbeg + BK - 1) / BK;

  LoadState sa, sb;
  loader_init<AM>(sa, p, m0, p.M);
  loader_init<BMODE>(sb, p, n0, p.N);

  uint4 ra[4], rb[4];
  loader_fetch<AM>(ra, sa, p, p.a, p.lda, m0, p.M, kbeg, kend);
  loader_fetch<BMODE>(rb, sb, p, p.b, p.ldb, n0, p.N, kbeg, kend);
  loader_store<AM>(ra, LA(0));
  loader_store<BMODE>(rb, LB(0));
  __syncthreads();

  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      loader_fetch<AM>(ra, sa, p, p.a, p.lda, m0, p.M, kbeg + (kt + 1) * BK, kend);
      loader_fetch<BMODE>(rb, sb, p, p.b, p.ldb, n0, p.N, kbeg + (kt + 1) * BK, kend);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_read<AM>(LA(cur), wm * 64 + i * 16, kk);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_read<BMODE>(LB(cur), wn * 64 + j * 16, kk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      loader_store<AM>(ra, LA(cur ^ 1));
      loader_store<BMODE>(rb, LB(cur ^ 1));
    }
    __syncthreads();
  }

#undef LA
#undef LB
  // Epilogue.  acc[i][j] = D[n][m] with lane col m = l&15, rows n = (l>>4)*4+r.
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (l & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (l >> 4) * 4;
      if (n >= p.N) continue;
      float v[4] = {acc[i][j][0] * p.alpha, acc[i][j][1] * p.alpha, acc[i][j][2] * p.alpha, acc[i][j][3] * p.alpha};
      const bool full = n + 3 < p.N;
      if (OUT == OUT_F32_ATOMIC) {
        float* c = (float*)p.c + (int64_t)m * p.ldc + n;
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
        float* c = (float*)p.c + (int64_t)m * p.ldc + n;
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
        bf16* c = (bf16*)p.c + (int64_t)m * p.ldc + n;
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

// W [K][R][S][C] -> Wt [C][R][S][K]  (dgrad B operand), bf16
__global__ void wt_transpose_k(const bf16* __restrict__ w, bf16* __restrict__ wt, int K, int RS, int C) {
  const int64_t total = (int64_t)K * RS * C;
  SG_GRID_STRIDE(i, total) {
    int c = (int)(i % C);
    int64_t t = i / C;
    int rs = (int)(t % RS);
    int k = (int)(t / RS);
    wt[((int64_t)c * RS + rs) * K + k] = w[i];
  }
}

}  // namespace sg

using namespace sg;

static ConvGeom make_geom(int N, int H, int W, int C, int K, int R, int S, int Ho, int Wo, int sh, int sw, int ph,
                          int pw, int dh, int dw) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S; g.Ho = Ho; g.Wo = Wo;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dw;
  g.dC = FastDiv(C); g.dS = FastDiv(S); g.dK = FastDiv(K); g.dWo = FastDiv(Wo); g.dHoWo = FastDiv(Ho * Wo);
  g.dW = FastDiv(W); g.dHW = FastDiv(H * W);
  return g;
}

template <int AM, int BMODE, int OUT>
static void launch(const GemmArgs& p, int splits, hipStream_t s, int batch = 1) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles, batch, splits), block(NT);
  hipLaunchKernelGGL((igemm_k<AM, BMODE, OUT>), grid, block, 4 * BM * BK * 2, s, p);
}

// choose split-K so that the grid has >= ~2 waves of workgroups
static int pick_splits(int M, int N, int K, int want) {
  if (want > 0) return want;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = 1;
  const int nkt = (K + BK - 1) / BK;
  while (tiles * splits < 512 && splits * 2 <= nkt / 2) splits *= 2;
  return splits;
}

static inline int kps(int K, int splits) {
  int nkt = (K + BK - 1) / BK;
  return ((nkt + splits - 1) / splits) * BK;
}

extern "C" {

// Plain GEMM: C[M][N] = alpha * op(A) op(B)^T ...  with
//   a_kouter = 0: A stored [M][K] (lda), 1: A stored [K][M]
//   b_kouter = 0: B stored [N][K] (ldb), 1: B stored [K][N]
// out_mode 0 bf16, 1 f32, 2 f32 atomic (split-K, C pre-initialised).
void sg_gemm(const void* a, int64_t lda, int a_kouter, const void* b, int64_t ldb, int b_kouter, void* c,
             int64_t ldc, int M, int N, int K, float alpha, float beta, const void* bias, int relu, int out_mode,
             int splits, int batch, int64_t sa, int64_t sb, int64_t sc, hipStream_t s) {
  GemmArgs p{};
  p.sa = sa; p.sb = sb; p.sc = sc;
  p.M = M; p.N = N; p.K = K; p.a = (const bf16*)a; p.lda = lda; p.b = (const bf16*)b; p.ldb = ldb;
  p.c = c; p.ldc = ldc; p.alpha = alpha; p.beta = beta; p.bias = (const float*)bias; p.relu = relu;
  if (out_mode == OUT_F32_ATOMIC) splits = pick_splits(M, N, K, splits);
  else splits = 1;
  p.k_per_split = kps(K, splits);
#define G(AM, BMD, OUT) launch<AM, BMD, OUT>(p, splits, s, batch)
#define GO(AM, BMD)                       \
  if (out_mode == OUT_BF16) G(AM, BMD, OUT_BF16); \
  else if (out_mode == OUT_F32) G(AM, BMD, OUT_F32); \
  else G(AM, BMD, OUT_F32_ATOMIC);
  if (!a_kouter && !b_kouter) { GO(LM_KMAJOR, LM_KMAJOR) }
  else if (!a_kouter && b_kouter) { GO(LM_KMAJOR, LM_KOUTER) }
  else if (a_kouter && !b_kouter) { GO(LM_KOUTER, LM_KMAJOR) }
  else { GO(LM_KOUTER, LM_KOUTER) }
#undef GO
#undef G
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
  if (out_mode == OUT_F32) launch<LM_CONV_FWD, LM_KMAJOR, OUT_F32>(p, 1, s);
  else launch<LM_CONV_FWD, LM_KMAJOR, OUT_BF16>(p, 1, s);
}

// conv data gradient: dy [N*Ho*Wo][K] bf16, wt [C][R][S][K] bf16 -> dx [N*H*W][C]
void sg_conv_dgrad(const void* dy, const void* wt, void* dx, int N, int H, int W, int C, int K, int R, int S, int Ho,
                   int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, hipStream_t s) {
  GemmArgs p{};
  p.g = make_geom(N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw);
  p.M = N * H * W; p.N = C; p.K = R * S * K;
  p.a = (const bf16*)dy; p.lda = 0; p.b = (const bf16*)wt; p.ldb = R * S * K;
  p.c = dx; p.ldc = C; p.alpha = 1.f; p.beta = 0.f; p.bias = nullptr; p.relu = 0;
  p.k_per_split = kps(p.K, 1);
  if (out_mode == OUT_F32) launch<LM_CONV_DGRAD, LM_KMAJOR, OUT_F32>(p, 1, s);
  else launch<LM_CONV_DGRAD, LM_KMAJOR, OUT_BF16>(p, 1, s);
}

// conv weight gradient: dW[K][R*S*C] (fp32, accumulated atomically: caller
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
  launch<LM_KOUTER, LM_CONV_WGRAD, OUT_F32_ATOMIC>(p, splits, s);
}

void sg_wt_transpose(const void* w, void* wt, int K, int RS, int C, hipStream_t s) {
  hipLaunchKernelGGL(wt_transpose_k, dim3(sg_grid((int64_t)K * RS * C)), dim3(256), 0, s, (const bf16*)w, (bf16*)wt,
                     K, RS, C);
}

}  // extern "C"

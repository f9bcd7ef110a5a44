// Algebraic backward of a ResNet bottleneck's residual tail
//
//   c3 = W y2 (1x1 conv, W [K4][C]),  out = relu(BN(c3) + res)
//
// without any pass over c3 or its gradient.  The residual BN(+ReLU)
// backward normally reads (dy, mask, c3) twice -- a reduction for
// (sum g~, sum g~ x^) and an apply writing dc3 -- and the conv then reads dc3
// for its data and weight gradients (~12 ms of the ResNet-50 b1024 step,
// profiles/r5/r50_b1024_kernel_stats_r5a_round_start.txt).  With g~ = dy *
// mask (written masked by the upstream conv's dgrad epilogue, stats_mode 4,
// which also sums it), s = gamma invstd, a = mean g~, b = mean(g~ x^),
// u = s b invstd, v = u mu - s a:
//
//   dc3 = s g~ - u c3 + v                          (per output channel k)
//   dW  = diag(s) G - diag(u) W Gram(y2) + v (x) colsum(y2),  G = g~^T y2
//   dy2 = [g~ | y2] Bd^T + bias,  Bd = [W^T diag(s) | -W^T diag(u) W],  bias = W^T v
//   sum g~ c3[k] = <W[k], G[k]>  (the BN's second reduction, from G)
//
// so the backward is one two-source weight-gradient GEMM ([g~ | y2]^T y2 ->
// G and Gram, igemm_kern.h LM_KOUTER2), two small fp32 GEMMs (W Gram and
// W^T diag(u) W, ggemm.hip), the coefficient / combination kernels below,
// and one two-source data-gradient GEMM (K = K4 + C, LM_KMAJOR2) whose
// epilogue still serves the producer BN's identity-sum backward.  Extra
// MFMA work: +C/K4 (25 %) on both GEMMs; bytes saved: two full passes over
// the K4-channel tensor.
//
// Reference: the conv backward of src/worker/layer.cc:99-123 (F5 weight
// gradient, col2im data gradient); BatchNorm / residual blocks are
// north-star additions.
#include <algorithm>
#include <stdexcept>

#include "igemm_kern.h"

namespace sg {
namespace bnres {

// Per output channel k (one wave per row): sg = <W[k], G[k]>, gs = sum g~
// (the 32 atomic slot rows of the upstream epilogue), the BN parameter
// gradients, the coefficients (s, u, v), and the fp32 copies W[k] / u W[k]
// for the small GEMMs.
__global__ void __launch_bounds__(256) coef_k(const float* __restrict__ G, const bf16* __restrict__ w,
                                              const float* __restrict__ gws, const float* __restrict__ mean,
                                              const float* __restrict__ invstd, const float* __restrict__ gamma,
                                              float inv_p, int K4, int C, float* __restrict__ coef,
                                              float* __restrict__ wf, float* __restrict__ wu, float* __restrict__ dg,
                                              float* __restrict__ db) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= K4) return;
  const bf16* wr = w + (int64_t)k * C;
  const float* gr = G + (int64_t)k * C;
  float sgc = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float wv = (float)wr[c];
    sgc += wv * gr[c];
    wf[(int64_t)k * C + c] = wv;
  }
  sgc = wave_sum(sgc);
  float gs = lane < 32 ? gws[(int64_t)lane * 2 * K4 + k] : 0.f;
  gs = wave_sum(gs);
  const float mu = mean[k], is = invstd[k];
  const float m1 = sgc - mu * gs;  // sum g~ (c3 - mu)
  const float dgam = is * m1;      // sum g~ x^
  const float a = gs * inv_p, b = dgam * inv_p;
  const float s = gamma[k] * is, u = s * b * is, v = u * mu - s * a;
  if (lane == 0) {
    dg[k] += dgam;
    db[k] += gs;
    coef[k] = s;
    coef[K4 + k] = u;
    coef[2 * K4 + k] = v;
  }
  for (int c = lane; c < C; c += 64) wu[(int64_t)k * C + c] = u * (float)wr[c];
}

// grid (C / 64, K4 / 16 + C / 64), 256 threads.  Blocks by < K4 / 16: the
// 16 x 64 tile (k, c) of dW = s G - u T + v cs (T = W Gram) added into the
// weight gradient, its <W, dW> column sums (the producer BN's identity-sum
// input) and W^T v column sums (the data gradient's bias), and the
// transposed Bd[c][k] = s_k W[k][c].  Blocks by >= K4 / 16: Bd[c][K4 + j] =
// -M[c][j].  Block (cb, 0) also evaluates the producer BN's identity-sum gate
// on gamma2 / beta2 (as wdot_colsum_k: the int flag at wdot + C).
__global__ void __launch_bounds__(256) combine_k(const float* __restrict__ G, const float* __restrict__ T,
                                                 const float* __restrict__ Mm, const float* __restrict__ cs,
                                                 const float* __restrict__ coef, const bf16* __restrict__ w, int K4,
                                                 int C, float* __restrict__ dw, bf16* __restrict__ bd,
                                                 float* __restrict__ bias, float* __restrict__ wdot,
                                                 const float* __restrict__ gamma2, const float* __restrict__ beta2,
                                                 float tau, int cs_rows) {
  // main part: 16 k-rows per block (a stage-1 tail has K4 = 256, C = 64: 64-row
  // blocks gave 5 workgroups, each thread walking 16 dependent rows -- ~18 us of
  // latency per call; 16-row blocks quadruple the grid)
  constexpr int KB = 16;
  __shared__ bf16 tile[KB][66];
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int cb = blockIdx.x, kb = blockIdx.y;
  const int c = cb * 64 + cl;
  const int ldb = K4 + C;
  const int nkb = K4 / KB;
  if (kb >= nkb) {  // the -M part of Bd
    const int j = (kb - nkb) * 64 + cl;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int cc = cb * 64 + rg + 4 * i;
      bd[(int64_t)cc * ldb + K4 + j] = (bf16)(-Mm[(int64_t)cc * C + j]);
    }
    return;
  }
  if (kb == 0 && rg == 0 && gamma2 != nullptr) {
    const float g2 = fabsf(gamma2[c]);
    if (!(g2 >= tau && fabsf(beta2[c]) <= 4.f * g2)) *(int*)(wdot + C) = 1;  // (NaN raises it too)
  }
  float csv = 0.f;  // column sums of y: cs_rows slot rows [cs_rows][C]
  for (int r = 0; r < cs_rows; ++r) csv += cs[(int64_t)r * C + c];
  float wd = 0.f, bs = 0.f;
#pragma unroll
  for (int i = 0; i < KB / 4; ++i) {
    const int kl = rg + 4 * i;
    const int k = kb * KB + kl;
    const int64_t o = (int64_t)k * C + c;
    const float s = coef[k], u = coef[K4 + k], v = coef[2 * K4 + k];
    const float wv = (float)w[o];
    const float d = s * G[o] - u * T[o] + v * csv;
    dw[o] += d;
    wd += wv * d;
    bs += wv * v;
    tile[kl][cl] = (bf16)(s * wv);
  }
  red[0][rg][cl] = wd;
  red[1][rg][cl] = bs;
  __syncthreads();
  if (rg == 0) {
    atomicAdd(wdot + c, red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl]);
    atomicAdd(bias + c, red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl]);
  }
  // Bd[c][k] = tile[k][c]: rows c of this block, KB consecutive k per row
  const int kk = threadIdx.x & (KB - 1), cq = threadIdx.x / KB;  // 16 rows c per pass
#pragma unroll
  for (int i = 0; i < 64 * KB / 256; ++i) {
    const int ccl = cq + (256 / KB) * i;
    bd[(int64_t)(cb * 64 + ccl) * ldb + kb * KB + kk] = tile[kk][ccl];
  }
}

// g~ = dy * bit(mask) written out, sum g~ per channel into 32 atomic slot rows
// ws[slot][2][C] (first half).  The fallback when no upstream dgrad epilogue
// produced g~ (a block feeding the global pooling).  Thread = 8 channels x a
// row lane; grid (bands, C / (8 * CT)).
__global__ void __launch_bounds__(256) masksum_k(const bf16* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                 bf16* __restrict__ g, float* __restrict__ ws, int64_t R, int C,
                                                 int rows_per_band) {
  __shared__ float red[256 * 8];
  const int chunks = C / 8;
  const int CT = chunks < 64 ? chunks : 64;
  const int RT = 256 / CT;
  const int tx = threadIdx.x % CT, ty = threadIdx.x / CT;
  const int c0 = (blockIdx.y * CT + tx) * 8;
  const bool cok = ty < RT && c0 < C;
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_band;
  const int64_t r1 = min(R, r0 + rows_per_band);
  if (cok) {
    for (int64_t r = r0 + ty; r < r1; r += RT) {
      const bf16x8 d = __builtin_nontemporal_load((const bf16x8*)(dy + r * C + c0));
      const unsigned m = mask[(r * C + c0) >> 3];
      bf16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        o[i] = ((m >> i) & 1u) != 0 ? d[i] : (bf16)0.f;
        a[i] += (float)o[i];
      }
      *(bf16x8*)(g + r * C + c0) = o;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[threadIdx.x * 8 + i] = cok ? a[i] : 0.f;
  __syncthreads();
  const int CW = CT * 8;
  for (int j = threadIdx.x; j < CW; j += 256) {
    const int cc = blockIdx.y * CW + j;
    if (cc >= C) break;
    float sum = 0.f;
    for (int k = 0; k < RT; ++k) sum += red[(k * CT + j / 8) * 8 + (j & 7)];
    atomicAdd(ws + (int64_t)(blockIdx.x & 31) * 2 * C + cc, sum);
  }
}

// A downsample tail's strided 1x1 shortcut conv reads only every s-th pixel:
// pick_k gathers those pixels into a dense NHWC tensor (the shortcut then is
// a plain GEMM, and its algebraic backward a dense two-source GEMM), place_k
// writes the input gradient back to the full grid (zeros between).  16-byte
// vectors, one per thread per iteration; 32-bit indices (host-checked).
__global__ void __launch_bounds__(256) pick_k(const uint4* __restrict__ x, uint4* __restrict__ y, unsigned total,
                                             unsigned CV, unsigned Wo, unsigned Ho, unsigned W, unsigned H,
                                             unsigned st) {
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const unsigned c = i % CV, p = i / CV;
    const unsigned j = p % Wo, t = p / Wo;
    const unsigned r = t % Ho, n = t / Ho;
    y[i] = x[((n * H + st * r) * W + st * j) * CV + c];
  }
}

__global__ void __launch_bounds__(256) place_k(const uint4* __restrict__ xs, uint4* __restrict__ dx, unsigned total,
                                              unsigned CV, unsigned W, unsigned H, unsigned Wo, unsigned Ho,
                                              unsigned st) {
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const unsigned c = i % CV, p = i / CV;
    const unsigned w = p % W, t = p / W;
    const unsigned h = t % H, n = t / H;
    uint4 v = {0u, 0u, 0u, 0u};
    if (h % st == 0 && w % st == 0 && h / st < Ho && w / st < Wo) v = xs[((n * Ho + h / st) * Wo + w / st) * CV + c];
    dx[i] = v;
  }
}

// The two-branch tail's folded weights: wf[n] = [bf16(s3[n] W3[n]) | bf16(sd[n] Wd[n])],
// shift[n] = f3[n] + fd[n], ones[n] = 1 (the apply pass's unit scale)
__global__ void __launch_bounds__(256) fold_k(const bf16* __restrict__ w3, const bf16* __restrict__ wd,
                                             const float* __restrict__ s3, const float* __restrict__ f3,
                                             const float* __restrict__ sd, const float* __restrict__ fd, int N,
                                             int K1, int K2, bf16* __restrict__ wf, float* __restrict__ shift,
                                             float* __restrict__ ones) {
  const int n = blockIdx.x;
  const int K = K1 + K2;
  for (int k = threadIdx.x; k < K; k += 256)
    wf[(int64_t)n * K + k] = k < K1 ? (bf16)(s3[n] * (float)w3[(int64_t)n * K1 + k])
                                    : (bf16)(sd[n] * (float)wd[(int64_t)n * K2 + k - K1]);
  if (threadIdx.x == 0) {
    shift[n] = f3[n] + fd[n];
    ones[n] = 1.f;
  }
}

// BN statistics of c = y W^T without c: sum_k = W[k] . colsum(y) and
// sumsq_k = W[k]^T Gram(y) W[k] (Gram = y^T y, fp32 [C][C]; colsum as cs_rows
// slot rows [cs_rows][C]) -> ws[0][2][K4] (sum | sumsq), the layout
// bn_fwd_from_ws reads with rows = 1.  One workgroup per output channel.
__global__ void __launch_bounds__(256) gram_stats_k(const bf16* __restrict__ w, const float* __restrict__ gram,
                                                   const float* __restrict__ cs, int cs_rows, int K4, int C,
                                                   float* __restrict__ ws) {
  __shared__ float sh[8];
  const int k = blockIdx.x;
  const bf16* wk = w + (int64_t)k * C;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < C; i += 256) {
    const float* gi = gram + (int64_t)i * C;
    float t = 0.f;
    for (int j = 0; j < C; ++j) t += gi[j] * (float)wk[j];
    float ci = 0.f;
    for (int r = 0; r < cs_rows; ++r) ci += cs[(int64_t)r * C + i];
    const float wi = (float)wk[i];
    s1 += wi * ci;
    s2 += wi * t;
  }
  s1 = block_sum(s1, sh);
  s2 = block_sum(s2, sh);
  if (threadIdx.x == 0) {
    ws[k] = s1;
    ws[K4 + k] = s2;
  }
}

template <int BM, int BN, int AM, int BMODE, int OUT, int NTH, int WM, int WN, int STAGES>
void go(const GemmArgs& p, int tiles, int zdim, hipStream_t s) {
  constexpr int stages = STAGES * (BM + BN) * BK * 2;
  constexpr int rch = (STAGES == 1 || BM * (BN + 4) * 4 <= 152 * 1024) ? BM : BM / 4;
  constexpr int etile = OUT == OUT_BF16 ? rch * (BN + 4) * 4 : OUT == OUT_F32_ATOMIC ? BM * (BN + 4) * 4 : 0;
  constexpr int lds = stages > etile ? stages : etile;
  static_assert(lds <= 160 * 1024, "LDS budget");
  auto* kern = igemm_k<BM, BN, AM, BMODE, OUT, NTH, WM, WN, STAGES, 0>;
  if constexpr (lds > 65536) {
    static bool attr = [kern] {
      return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    }();
    (void)attr;
  }
  hipLaunchKernelGGL(kern, dim3(tiles, 1, zdim), dim3(NTH), lds, s, p);
}

int g_wide = 1;   // sg_bnres_tune(0, v): the 256 x 128 weight-gradient tiles (A/B)
int g_dwide = 0;  // sg_bnres_tune(1, v): the 256 x 128 data-gradient tiles (A/B)

unsigned extent(int64_t elems) {
  if (elems * 2 >= (int64_t)1 << 31) throw std::runtime_error("bnres: operand exceeds 2 GiB (32-bit buffer offsets)");
  return (unsigned)(elems * 2);
}

}  // namespace bnres
}  // namespace sg

using namespace sg;
using namespace sg::bnres;

extern "C" {

void sg_bnres_tune(int key, int v) {
  if (key == 0) g_wide = v;
  if (key == 1) g_dwide = v;
}

// out [K4 + C][C] fp32 (zeroed by the caller) += [g | y]^T y over P pixels:
// rows 0..K4-1 = G = g^T y, rows K4.. = Gram(y).  g [P][K4], y [P][C] bf16.
// (K4 = 0: out [C][C] += Gram(y) = y^T y alone -- the forward's BN statistics
// of a 1x1 conv of y, bnres_gram_stats)
void sg_bnres_wgrad(const void* g, const void* y, void* out, int P, int K4, int C, hipStream_t s) {
  if ((K4 & 127) != 0 || (C & 63) != 0) throw std::runtime_error("bnres_wgrad: K4 % 128 and C % 64 required");
  GemmArgs p{};
  for (int i = 0; i < 16; ++i) {
    p.g.phs[i].dns = FastDiv(1);
    p.g.phs[i].dWp = FastDiv(1);
    p.g.phs[i].dHpWp = FastDiv(1);
  }
  p.M = K4 + C; p.N = C; p.K = P;
  p.a = (const bf16*)g; p.lda = K4; p.a_bytes = extent((int64_t)P * K4);
  p.a2 = (const bf16*)y; p.lda2 = C; p.a2_bytes = extent((int64_t)P * C); p.a2_split = K4;
  p.b = (const bf16*)y; p.ldb = C; p.b_bytes = p.a2_bytes;
  p.c = out; p.ldc = C; p.alpha = 1.f;
  const int nkt = (P + BK - 1) / BK;
  // 256 x 128 8-wave tiles (64 x 64 wave tiles, three-stage ring, one
  // workgroup per CU) when the G / Gram split is 256-row aligned: the split
  // count minimising ceil(tiles * sp / CUs) * (K-tiles per split + 6) (the
  // quantisation model of the conv weight gradient, igemm.hip wgrad_splits_q)
  if (C >= 128 && (K4 & 255) == 0 && g_wide) {
    const int tiles = ((p.M + 255) / 256) * ((C + 127) / 128);
    const int slots = sg_cu_count();
    int sp = 1;
    long best = -1;
    for (int s2 = 1; s2 <= 256 && nkt / s2 >= 16; ++s2) {
      const long cost = (long)((tiles * s2 + slots - 1) / slots) * ((nkt + s2 - 1) / s2 + 6);
      if (best < 0 || cost < best) {
        best = cost;
        sp = s2;
      }
    }
    p.k_per_split = ((nkt + sp - 1) / sp) * BK;
    go<256, 128, LM_KOUTER2, LM_KOUTER, OUT_F32_ATOMIC, 512, 4, 2, 3>(p, tiles, sp, s);
    return;
  }
  // 128 x 128 8-wave tiles when C fills them, else 64 x 64; split-K to ~512 workgroups
  if (C >= 128) {
    const int tiles = ((p.M + 127) / 128) * ((C + 127) / 128);
    int sp = 1;
    while (tiles * sp < 512 && sp * 2 * 4 <= nkt) sp *= 2;
    p.k_per_split = ((nkt + sp - 1) / sp) * BK;
    go<128, 128, LM_KOUTER2, LM_KOUTER, OUT_F32_ATOMIC, 512, 2, 4, 2>(p, tiles, sp, s);
  } else {
    // C == 64: 128 x 64 tiles -- the y operand (B) is re-read once per M-tile,
    // so taller tiles read it fewer times (3 vs 5 passes at K4 = 256)
    const int tiles = (p.M + 127) / 128;
    int sp = 1;
    while (tiles * sp < 768 && sp * 2 * 8 <= nkt) sp *= 2;
    p.k_per_split = ((nkt + sp - 1) / sp) * BK;
    go<128, 64, LM_KOUTER2, LM_KOUTER, OUT_F32_ATOMIC, 256, 2, 2, 2>(p, tiles, sp, s);
  }
}

// dx [P][C] bf16 = [g | y] bd^T + bias (bd [C][K4 + C] bf16, bias [C] fp32).
// stats != nullptr (with mask: the producer BN's 1-bit ReLU map [P][C/8]):
// the epilogue also sums the masked output into 32 atomic slot rows
// stats[32][2][C] (zeroed by the caller) -- stats_mode 3, the producer BN's
// identity-sum backward.
void sg_bnres_dgrad(const void* g, const void* y, const void* bd, const void* bias, void* dx, int P, int K4, int C,
                    void* stats, const void* mask, hipStream_t s) {
  if ((K4 & 63) != 0 || (C & 63) != 0) throw std::runtime_error("bnres_dgrad: K4 % 64 and C % 64 required");
  GemmArgs p{};
  for (int i = 0; i < 16; ++i) {
    p.g.phs[i].dns = FastDiv(1);
    p.g.phs[i].dWp = FastDiv(1);
    p.g.phs[i].dHpWp = FastDiv(1);
  }
  p.M = P; p.N = C; p.K = K4 + C;
  p.a = (const bf16*)g; p.lda = K4; p.a_bytes = extent((int64_t)P * K4);
  p.a2 = (const bf16*)y; p.lda2 = C; p.a2_bytes = extent((int64_t)P * C); p.a2_split = K4;
  p.b = (const bf16*)bd; p.ldb = K4 + C; p.b_bytes = extent((int64_t)C * (K4 + C));
  p.c = dx; p.ldc = C; p.alpha = 1.f; p.beta = 0.f; p.bias = (const float*)bias;
  p.k_per_split = ((p.K + BK - 1) / BK) * BK;
  p.lds_epilogue = 1;
  p.early_issue = 1;
  if (stats) {
    p.stats = (float*)stats;
    p.stats_mode = 3;
    p.bnb_mask = (const uint8_t*)mask;
  }
  // tiles as igemm's launcher picks them for these shapes: 8-wave 128 x 128
  // (two workgroups per CU) once there are enough tiles, else 4-wave 128 x 64
  const long t128 = (long)((P + 127) / 128) * ((C + 127) / 128);
  if (C >= 128 && t128 >= 512 && g_dwide) {  // (A/B: sg_bnres_tune(1, 1))
    go<256, 128, LM_KMAJOR2, LM_KMAJOR, OUT_BF16, 512, 4, 2, 3>(p, (int)(((P + 255) / 256) * ((C + 127) / 128)), 1, s);
  } else if (C >= 128 && t128 >= 512) {
    go<128, 128, LM_KMAJOR2, LM_KMAJOR, OUT_BF16, 512, 2, 4, 2>(p, (int)t128, 1, s);
  } else {
    const int tiles = ((P + 127) / 128) * ((C + 63) / 64);
    go<128, 64, LM_KMAJOR2, LM_KMAJOR, OUT_BF16, 256, 2, 2, 2>(p, tiles, 1, s);
  }
}

// coefficients: see coef_k.  gws = the 32 slot rows [32][2][K4] of sum g~.
void sg_bnres_coef(const void* G, const void* w, const void* gws, const void* mean, const void* invstd,
                   const void* gamma, int P, int K4, int C, void* coef, void* wf, void* wu, void* dgamma, void* dbeta,
                   hipStream_t s) {
  hipLaunchKernelGGL(coef_k, dim3((K4 + 3) / 4), dim3(256), 0, s, (const float*)G, (const bf16*)w,
                     (const float*)gws, (const float*)mean, (const float*)invstd, (const float*)gamma, 1.f / (float)P,
                     K4, C, (float*)coef, (float*)wf, (float*)wu, (float*)dgamma, (float*)dbeta);
}

// combination: see combine_k (cs: cs_rows slot rows of column sums).  bias and wdot (C floats + the int gate flag
// at wdot + C) zeroed by the caller.
void sg_bnres_combine(const void* G, const void* T, const void* M, const void* cs, int cs_rows, const void* coef,
                      const void* w, int K4, int C, void* dw, void* bd, void* bias, void* wdot, const void* gamma2,
                      const void* beta2, float tau, hipStream_t s) {
  if ((K4 & 63) != 0 || (C & 63) != 0) throw std::runtime_error("bnres_combine: K4 % 64 and C % 64 required");
  hipLaunchKernelGGL(combine_k, dim3(C / 64, K4 / 16 + C / 64), dim3(256), 0, s, (const float*)G, (const float*)T,
                     (const float*)M, (const float*)cs, (const float*)coef, (const bf16*)w, K4, C, (float*)dw,
                     (bf16*)bd, (float*)bias, (float*)wdot, (const float*)gamma2, (const float*)beta2, tau, cs_rows);
}

// g = dy * bit(mask), sum g -> ws[32][2][C] (first half; zeroed by the caller)
void sg_bnres_masksum(const void* dy, const void* mask, void* g, void* ws, int64_t R, int C, hipStream_t s) {
  if ((C & 7) != 0) throw std::runtime_error("bnres_masksum: C % 8 required");
  const int chunks = C / 8, CT = chunks < 64 ? chunks : 64;
  const int cb = (chunks + CT - 1) / CT;
  int bands = (int)((R + 255) / 256);
  if (bands > 1024 / cb) bands = 1024 / cb;
  if (bands < 1) bands = 1;
  const int rpb = (int)((R + bands - 1) / bands);
  hipLaunchKernelGGL(masksum_k, dim3(bands, cb), dim3(256), 0, s, (const bf16*)dy, (const uint8_t*)mask, (bf16*)g,
                     (float*)ws, R, C, rpb);
}

// x [N][H][W][C] bf16 -> y [N][Ho][Wo][C] = x[:, ::st, ::st, :] (place: the
// reverse, zeros at the other pixels of dx [N][H][W][C]); C % 8 == 0
void sg_strided_pick(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int st, int place,
                     hipStream_t s) {
  if ((C & 7) != 0) throw std::runtime_error("strided_pick: C % 8 required");
  const int64_t total = (int64_t)N * (place ? H * W : Ho * Wo) * (C / 8);
  if (total >= ((int64_t)1 << 31) || (int64_t)N * H * W * (C / 8) >= ((int64_t)1 << 31))
    throw std::runtime_error("strided_pick: tensor too large for 32-bit indexing");
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (place)
    hipLaunchKernelGGL(place_k, dim3(blocks), dim3(256), 0, s, (const uint4*)x, (uint4*)y, (unsigned)total,
                       (unsigned)(C / 8), (unsigned)W, (unsigned)H, (unsigned)Wo, (unsigned)Ho, (unsigned)st);
  else
    hipLaunchKernelGGL(pick_k, dim3(blocks), dim3(256), 0, s, (const uint4*)x, (uint4*)y, (unsigned)total,
                       (unsigned)(C / 8), (unsigned)Wo, (unsigned)Ho, (unsigned)W, (unsigned)H, (unsigned)st);
}

void sg_bnres_fold(const void* w3, const void* wd, const void* s3, const void* f3, const void* sd, const void* fd, int N,
                   int K1, int K2, void* wf, void* shift, void* ones, hipStream_t s) {
  hipLaunchKernelGGL(fold_k, dim3(N), dim3(256), 0, s, (const bf16*)w3, (const bf16*)wd, (const float*)s3,
                     (const float*)f3, (const float*)sd, (const float*)fd, N, K1, K2, (bf16*)wf, (float*)shift,
                     (float*)ones);
}

void sg_bnres_gram_stats(const void* w, const void* gram, const void* cs, int cs_rows, int K4, int C, void* ws,
                         hipStream_t s) {
  hipLaunchKernelGGL(gram_stats_k, dim3(K4), dim3(256), 0, s, (const bf16*)w, (const float*)gram, (const float*)cs,
                     cs_rows, K4, C, (float*)ws);
}

}  // extern "C"

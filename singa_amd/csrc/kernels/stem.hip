// ImageNet stem forward: 7x7 / stride-2 / pad-3 convolution over the
// "paired-tap" input (models/resnet.py PairedStemConv: each 16-byte vector
// holds two horizontally adjacent pixels x 3 channels + 2 zeros, the conv is
// a 7 x 4 conv with horizontal dilation 2 over pair vectors; reduction 224 =
// 7 rows x 4 pair-taps x 8), 64 filters, bf16 NHWC output plus the fused
// BatchNorm statistics of the output (the 32 atomic slot rows of igemm's
// epilogue, sums of the bf16-rounded values).
//
// The reference computes the first conv as per-image im2col + sgemm
// (src/worker/layer.cc:75-81).  Through the generic implicit-GEMM kernel
// (igemm.hip) every output pixel gathers 28 scattered 16-byte vectors per
// tile and a 128-pixel tile covers ~1.1 output rows, so input rows are
// fetched again for every tile (~1.4 ms of the b1024 ResNet-50 step).
//
// Here a persistent workgroup walks output ROW PAIRS taken from a dynamic
// queue (common.h: a workgroup that starts late takes fewer):
// the filters (64 x 224, 29 KB) are loaded into LDS once, and per row pair
// the 9 input rows it needs are staged in LDS with coalesced row loads (zero
// rows / zero margins = the padding), the next pair's rows already in flight
// in registers while this pair's MFMAs run.  Wave (wm, wn) computes output
// row wm of the pair (Wo / 16 pixel blocks) x 32 filters; every A fragment
// (one pair-tap's 8 values of one pixel) is one ds_read_b128 from the patch.
// The BatchNorm partial sums stay in registers across the whole range and
// are reduced once per workgroup.
#include "common.h"

namespace sg {
namespace stem {

constexpr int K = 64;         // filters
constexpr int KR = 224;       // reduction: 7 x 4 x 8
constexpr int WROW = 232;     // LDS filter row in bf16 (224 + 8: 16 B against bank conflicts)
constexpr int PR = 9;         // input rows behind two output rows
constexpr int NT = 256;
constexpr int PF = 9;         // register-staged 16-byte vectors per thread (next pair's patch): PR*PW <= PF*NT

struct Args {
  const bf16* x;   // [N][H][W][8] paired input
  const bf16* w;   // [64][224]
  bf16* y;         // [N][Ho][Wo][64]
  float* stats;    // [32][2][64] slot rows (zeroed by the caller) or null
  int N, H, W, Ho, Wo;
  int pairs;       // N * Ho / 2
  int* wq;         // dynamic row-pair queue slot (common.h) or null: static blockIdx partition
  int lds_main;    // bytes of the patch + filter images (the ticket slot follows)
};

template <int TM>  // Wo / 16 pixel blocks per output row
__global__ void __launch_bounds__(NT, 2) stem_fwd_k(const Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int PW = a.W + 4;  // patch row: 2 zero vectors of margin each side
  char* patch = smem;
  char* wl = smem + PR * PW * 16;
  const int t = threadIdx.x;
  const int ln = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;  // output row of the pair, filter half
  const int g4 = ln >> 4;

  // this workgroup's row pairs: P0 = bx, P1 = bx + G, P2 = bx + 2G, then
  // (with a queue) P_i = 3G + ticket, tickets taken two pairs ahead;
  // (without) P_i = bx + i G
  const int G = (int)gridDim.x;
  int pp = (int)blockIdx.x, pn = pp + G;
  const int hp = a.Ho >> 1;  // row pairs per image

  for (int e = t; e < K * (KR / 8); e += NT) {
    const int k = e / (KR / 8), c = e - k * (KR / 8);
    *(uint4*)(wl + k * WROW * 2 + c * 16) = ((const uint4*)a.w)[e];
  }

  // global -> registers: the PR input rows of row pair pp (zero outside the image)
  uint4 v[PF];
  auto load = [&](int64_t pp) {
    const int n = (int)(pp / hp);
    const int ih0 = (int)(pp - (int64_t)n * hp) * 4 - 3;  // 2 * (2 * pair) - pad
    const uint4* xin = (const uint4*)a.x + (int64_t)n * a.H * a.W;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int e = t + u * NT;
      const int pr = e / PW, pc = e - pr * PW;
      const int ih = ih0 + pr, iw = pc - 2;
      uint4 z = make_uint4(0, 0, 0, 0);
      if (e < PR * PW && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) z = xin[(int64_t)ih * a.W + iw];
      v[u] = z;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int e = t + u * NT;
      if (e < PR * PW) *(uint4*)(patch + e * 16) = v[u];
    }
  };

  float s_sum[2][4], s_sq[2][4];  // BN partial sums of this lane's 8 filters
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_sum[j][r] = s_sq[j][r] = 0.f;

  int* sQ = (int*)(smem + a.lds_main);  // ticket broadcast
  int ticket = 0;
  bool first = true;
  if (pp < a.pairs) load(pp);
  while (pp < a.pairs) {
    __syncthreads();  // every wave done reading the previous patch (and the filters are in)
    store();
    if (t == 0) {
      // P_{i+2}: static for i = 0, else the ticket taken in the previous iteration
      *sQ = first ? pp + 2 * G : (a.wq ? 3 * G + ticket : pn + G);
      if (a.wq) ticket = wq_take(a.wq, 0);  // P_{i+3}
    }
    first = false;
    __syncthreads();
    const int pnn = __builtin_amdgcn_readfirstlane(*sQ);
    if (pn < a.pairs) load(pn);  // in flight during this pair's MFMAs
    f32x4 acc[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 7; ++kk) {
      // k = 32 kk + 8 g4 + c: filter row kk, pair-tap g4 (dilation 2: 2 vectors apart)
      bf16x8 fa[TM], fb[2];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *(const bf16x8*)(patch + ((2 * wm + kk) * PW + 2 * (i * 16 + (ln & 15)) + 2 * g4) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[j] = *(const bf16x8*)(wl + (wn * 32 + j * 16 + (ln & 15)) * WROW * 2 + (kk * 4 + g4) * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    // acc[i][j][r] = y[pixel i*16 + (ln & 15)][filter wn*32 + j*16 + 4 g4 + r]
    const int n = (int)(pp / hp);
    const int oy = (int)(pp - (int64_t)n * hp) * 2 + wm;
    bf16* yrow = a.y + ((int64_t)n * a.Ho + oy) * a.Wo * K;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ox = i * 16 + (ln & 15);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = (bf16)acc[i][j][r];
          const float f = (float)o[r];
          s_sum[j][r] += f;
          s_sq[j][r] += f * f;
        }
        *(bf16x4*)(yrow + (int64_t)ox * K + wn * 32 + j * 16 + 4 * g4) = o;
      }
    }
    pp = pn;
    pn = pnn;
  }
  if (a.wq && t == 0) wq_done(a.wq, 1);
  if (!a.stats) return;
  // reduce the 16 lanes of equal g4 (same filters, different pixels) and the
  // two waves of equal wn (the two output rows) through LDS, then one atomic
  // per (filter, sum) into slot row blockIdx.x % 32
  __syncthreads();
  float* red = (float*)smem;  // [4 waves][64 lanes][16]
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[(wid * 64 + ln) * 16 + j * 4 + r] = s_sum[j][r];
      red[(wid * 64 + ln) * 16 + 8 + j * 4 + r] = s_sq[j][r];
    }
  __syncthreads();
  if (t < 2 * K) {  // one thread per (filter, which sum)
    const int f = t & (K - 1), q = t >> 6;
    const int wnf = f >> 5, j = (f >> 4) & 1, gg = (f >> 2) & 3, r = f & 3;
    float acc = 0.f;
    for (int w2 = 0; w2 < 2; ++w2) {
      const int wv = w2 * 2 + wnf;
      for (int i = 0; i < 16; ++i) acc += red[(wv * 64 + gg * 16 + i) * 16 + q * 8 + j * 4 + r];
    }
    atomicAdd(a.stats + (blockIdx.x & 31) * 2 * K + q * K + f, acc);
  }
}

}  // namespace stem
}  // namespace sg

extern "C" {
int sg_ws_prezeroed();  // batchnorm.hip: one-shot 'workspace pre-zeroed' flag (per-step arena)

// Returns 1 when the stem kernel took the shape (C = 8 paired input, 64
// filters, Wo = 112 or 64 output pixels per row, even Ho), 0 otherwise (the
// caller falls back to the generic convolution).  stats: the 32 x 2 x 64 slot
// rows, zeroed by the caller, or null.
int sg_stem_fwd(const void* x, const void* w, void* y, void* stats, int N, int H, int W, int Ho, int Wo,
                hipStream_t s) {
  using namespace sg::stem;
  if ((Ho & 1) != 0 || N <= 0 || (Wo != 112 && Wo != 64) || 2 * Wo + 1 > W || PR * (W + 4) > PF * NT ||
      (int64_t)N * Ho / 2 >= (1LL << 31))
    return 0;
  const int lds_main = PR * (W + 4) * 16 + K * WROW * 2;
  Args a{(const sg::bf16*)x, (const sg::bf16*)w, (sg::bf16*)y, (float*)stats, N, H, W, Ho, Wo, N * Ho / 2,
         sg_workq_slot(), lds_main};
  if (stats && !sg_ws_prezeroed())  // (consumes the one-shot flag, as igemm's conv launches do)
    sg_zero_async(stats, sizeof(float) * 32 * 2 * K, s);
  const int lds = (lds_main > 4 * 64 * 16 * 4 ? lds_main : 4 * 64 * 16 * 4) + 16;
  const int cap = 2 * sg_cu_count();  // two workgroups per CU
  const int grid = a.pairs < cap ? a.pairs : cap;
  auto go = [&](auto kern) {
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, s, a);
  };
  if (Wo == 112) go(stem_fwd_k<7>);
  else go(stem_fwd_k<4>);
  return 1;
}

}  // extern "C"

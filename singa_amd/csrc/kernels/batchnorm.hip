// BatchNorm2d (NHWC / [R][C] rows) and per-channel column reductions.
//
// Design for MI355X (HBM-bound ops, every byte counts):
//  * Reductions are two-stage: each workgroup reduces a band of rows for its
//    channel slice in registers + LDS and emits ONE partial per channel.
//    Default (fast): the partial is atomically added into one of 32 slot
//    rows ws[band % 32][2][C] (32 adders per address; ws zeroed per call) and
//    the finalize sums 32 rows.  Deterministic mode (sg_set_deterministic):
//    every band stores its partial into its own row ws[band][2][C] with plain
//    stores and the finalize sums the rows in a fixed order -- bitwise
//    reproducible, at the cost of a longer finalize.  (History: v1 ended every
//    workgroup with atomics on the same addresses, 20x below HBM bandwidth;
//    v2 summed up to 1024 partials with one thread per channel, 150 us per
//    BN layer.)  Atomic-order noise is amplified by 50 BN layers into visibly
//    different training runs, hence the mode.
//  * The conv epilogue can produce the same [tiles][2][C] partials for the
//    BN that consumes its output (igemm.hip, GemmArgs::stats).
//  * Thread mapping is 2-D: a thread owns a fixed 8-channel (16-byte) slice
//    and walks rows, so per-channel coefficients are loaded once into
//    registers and no per-element channel index math (64-bit modulo) is done.
//  * The backward finalize turns (sum dy, sum dy*xhat) into three per-channel
//    coefficients so the apply pass is dx = k*g + b*x + a, and accumulates
//    dgamma/dbeta straight into the flat fp32 gradient buffer.
//  * With fused BN+ReLU (no residual) the ReLU mask is recomputed from
//    x*scale+shift instead of re-reading the output (one HBM pass fewer).
//
// Reference: per-channel bias-gradient reduction K4 (include/mshadow/cuda/
// tensor_gpu-inl.cuh:135-168) and F2 (src/worker/layer.cc:107); BatchNorm
// itself is a north-star addition (not in the reference).
#include <stdexcept>

#include "common.h"

namespace sg {

// MASK_BITS: the ReLU mask of a fused BN(+residual)+ReLU output, one bit per
// element (8 channels per byte, row-major [R][C/8]) written by the forward
// apply: the backward reads 1/16 of the bytes it would read from the bf16
// output (which stays materialised only as the next layer's input).
enum MaskMode : int { MASK_NONE = 0, MASK_Y = 1, MASK_AFFINE = 2, MASK_BITS = 3 };
constexpr int NSLOT = 32;      // atomic partial-sum slot rows of the fast mode
constexpr int FIN_GROUPS = 4;  // band groups per finalize workgroup (256 threads = 64 channels x 4)
static int g_bn_det = 0;       // deterministic reductions (set by sg_set_deterministic)
static thread_local int g_ws_prezeroed = 0; // (per OS thread) next launch's workspace is already zeroed (per-step arena): skip its zeroing

struct Tile2D {
  int CT, RT, tx, ty, c0;
  bool cok;
};
template <int V>
__device__ __forceinline__ Tile2D tile2d(int C) {
  Tile2D t;
  const int chunks = C / V;
  t.CT = chunks < 64 ? chunks : 64;
  t.RT = blockDim.x / t.CT;
  t.tx = threadIdx.x % t.CT;
  t.ty = threadIdx.x / t.CT;
  t.c0 = (blockIdx.y * t.CT + t.tx) * V;
  t.cok = t.ty < t.RT && t.c0 < C;
  return t;
}

// Gradient of a max-pool's INPUT gathered straight from the pooled gradient
// dyp [N][Ho][Wo][C] and the 8-bit window argmax (the fused stem BN+ReLU+
// max-pool: its BN backward reads this instead of a materialised max-pool
// backward output).  Row r = (n, ih, iw) of the BN input, channels c0..c0+7.
struct PoolG {
  const bf16* dy;
  const uint8_t* arg;
  int H, W, Ho, Wo, kh, kw, sh, sw, ph, pw;
  FastDiv dW, dH;
};
__device__ __forceinline__ void pool_grad8(const PoolG& q, int64_t r, int C, int c0, float* g) {
  const unsigned rr = (unsigned)r;
  const unsigned t = q.dW.div(rr);
  const int iw = (int)(rr - t * (unsigned)q.W);
  const unsigned n = q.dH.div(t);
  const int ih = (int)(t - n * (unsigned)q.H);
  const int oh0 = max(0, (ih + q.ph - q.kh + q.sh) / q.sh), oh1 = min(q.Ho - 1, (ih + q.ph) / q.sh);
  const int ow0 = max(0, (iw + q.pw - q.kw + q.sw) / q.sw), ow1 = min(q.Wo - 1, (iw + q.pw) / q.sw);
#pragma unroll
  for (int k = 0; k < 8; ++k) g[k] = 0.f;
  for (int oh = oh0; oh <= oh1; ++oh) {
    const int a = ih + q.ph - oh * q.sh;
    if (a < 0 || a >= q.kh) continue;
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int b = iw + q.pw - ow * q.sw;
      if (b < 0 || b >= q.kw) continue;
      const int64_t o = (((int64_t)n * q.Ho + oh) * q.Wo + ow) * C + c0;
      const uint2 pk = *(const uint2*)(q.arg + o);
      const bf16x8 d = *(const bf16x8*)(q.dy + o);
      const unsigned want = (unsigned)(a * q.kw + b);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        g[k] += (((k < 4 ? pk.x : pk.y) >> (8 * (k & 3))) & 0xffu) == want ? (float)d[k] : 0.f;
    }
  }
}

// ---------------------------------------------------------------------------
// Stage 1: per-band partial column sums.
//   MODE 0: p0 = sum x, p1 = sum x^2
//   MODE 1: g = dy (masked), xh = (x-mean)*invstd: p0 = sum g, p1 = sum g*xh
// ws layout: [band][2][C] fp32
// ---------------------------------------------------------------------------
template <typename T, int MODE, int V, bool PG = false>
__global__ void __launch_bounds__(256) colpart_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                 const T* __restrict__ y, const float* __restrict__ scale,
                                                 const float* __restrict__ shift, const float* __restrict__ mean,
                                                 const float* __restrict__ invstd, float* __restrict__ ws, int64_t R,
                                                 int C, int rows_per_band, int mask_mode, int det,
                                                 const T* __restrict__ x2 = nullptr,
                                                 const float* __restrict__ mean2 = nullptr,
                                                 const float* __restrict__ invstd2 = nullptr,
                                                 float* __restrict__ ws2 = nullptr, const PoolG pg = PoolG{},
                                                 const int* __restrict__ gate = nullptr) {
  // gated launch (the identity-sum BN backward's exact fallback): nothing to
  // do unless the gate is set
  if (gate != nullptr && *gate == 0) return;
  // MODE 2 = MODE 1 plus a second BN fed the same gradient (the downsample
  // branch of a residual block): also p2 = sum g*xh2, into ws2 [band][2][C]
  // as (p0, p2) -- its own instantiation, the plain reduction is untouched
  __shared__ float red[256 * V];
  const Tile2D t = tile2d<V>(C);
  constexpr bool dual = MODE == 2;
  float a0[V], a1[V], a2[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { a0[i] = 0.f; a1[i] = 0.f; a2[i] = 0.f; }
  float mu[V], is[V], sc[V], sf[V], mu2[V], is2[V];
  if (MODE >= 1 && t.cok) {
    ldc<V>(mean + t.c0, mu);
    ldc<V>(invstd + t.c0, is);
    if constexpr (dual) {
      ldc<V>(mean2 + t.c0, mu2);
      ldc<V>(invstd2 + t.c0, is2);
    }
    if (mask_mode == MASK_AFFINE) {
      ldc<V>(scale + t.c0, sc);
      ldc<V>(shift + t.c0, sf);
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_band;
  const int64_t r1 = min(R, r0 + rows_per_band);
  if (t.cok) {
    int64_t r = r0 + t.ty;
    // two rows per iteration keeps two independent 16-B loads per stream in flight
    for (; r + t.RT < r1; r += 2 * t.RT) {
      float v0[V], v1[V];
      ldv_nt<T, V>(x + r * C + t.c0, v0);
      ldv_nt<T, V>(x + (r + t.RT) * C + t.c0, v1);
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          a0[i] += v0[i] + v1[i];
          a1[i] += v0[i] * v0[i] + v1[i] * v1[i];
        }
      } else {
        float g0[V], g1[V];
        if constexpr (PG) {
          pool_grad8(pg, r, C, t.c0, g0);
          pool_grad8(pg, r + t.RT, C, t.c0, g1);
        } else {
          ldv_nt<T, V>(dy + r * C + t.c0, g0);
          ldv_nt<T, V>(dy + (r + t.RT) * C + t.c0, g1);
        }
        if (mask_mode == MASK_Y) {
          float y0[V], y1[V];
          ldv_nt<T, V>(y + r * C + t.c0, y0);
          ldv_nt<T, V>(y + (r + t.RT) * C + t.c0, y1);
#pragma unroll
          for (int i = 0; i < V; ++i) {
            g0[i] = y0[i] > 0.f ? g0[i] : 0.f;
            g1[i] = y1[i] > 0.f ? g1[i] : 0.f;
          }
        } else if (V == 8 && mask_mode == MASK_BITS) {
          const uint8_t* mb = (const uint8_t*)y;
          const unsigned m0 = mb[(r * C + t.c0) >> 3], m1 = mb[((r + t.RT) * C + t.c0) >> 3];
#pragma unroll
          for (int i = 0; i < V; ++i) {
            g0[i] = (m0 >> i) & 1u ? g0[i] : 0.f;
            g1[i] = (m1 >> i) & 1u ? g1[i] : 0.f;
          }
        } else if (mask_mode == MASK_AFFINE) {
#pragma unroll
          for (int i = 0; i < V; ++i) {
            g0[i] = v0[i] * sc[i] + sf[i] > 0.f ? g0[i] : 0.f;
            g1[i] = v1[i] * sc[i] + sf[i] > 0.f ? g1[i] : 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < V; ++i) {
          a0[i] += g0[i] + g1[i];
          a1[i] += g0[i] * (v0[i] - mu[i]) * is[i] + g1[i] * (v1[i] - mu[i]) * is[i];
        }
        if constexpr (dual) {
          float w0[V], w1[V];
          ldv_nt<T, V>(x2 + r * C + t.c0, w0);
          ldv_nt<T, V>(x2 + (r + t.RT) * C + t.c0, w1);
#pragma unroll
          for (int i = 0; i < V; ++i) a2[i] += g0[i] * (w0[i] - mu2[i]) * is2[i] + g1[i] * (w1[i] - mu2[i]) * is2[i];
        }
      }
    }
    for (; r < r1; r += t.RT) {
      float v0[V];
      ldv_nt<T, V>(x + r * C + t.c0, v0);
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < V; ++i) { a0[i] += v0[i]; a1[i] += v0[i] * v0[i]; }
      } else {
        float g0[V];
        if constexpr (PG) pool_grad8(pg, r, C, t.c0, g0);
        else ldv_nt<T, V>(dy + r * C + t.c0, g0);
        if (mask_mode == MASK_Y) {
          float y0[V];
          ldv_nt<T, V>(y + r * C + t.c0, y0);
#pragma unroll
          for (int i = 0; i < V; ++i) g0[i] = y0[i] > 0.f ? g0[i] : 0.f;
        } else if (V == 8 && mask_mode == MASK_BITS) {
          const unsigned m0 = ((const uint8_t*)y)[(r * C + t.c0) >> 3];
#pragma unroll
          for (int i = 0; i < V; ++i) g0[i] = (m0 >> i) & 1u ? g0[i] : 0.f;
        } else if (mask_mode == MASK_AFFINE) {
#pragma unroll
          for (int i = 0; i < V; ++i) g0[i] = v0[i] * sc[i] + sf[i] > 0.f ? g0[i] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < V; ++i) { a0[i] += g0[i]; a1[i] += g0[i] * (v0[i] - mu[i]) * is[i]; }
        if constexpr (dual) {
          float w0[V];
          ldv_nt<T, V>(x2 + r * C + t.c0, w0);
#pragma unroll
          for (int i = 0; i < V; ++i) a2[i] += g0[i] * (w0[i] - mu2[i]) * is2[i];
        }
      }
    }
  }
  // reduce over ty in LDS, then one partial per channel: plain store into
  // row `band` (deterministic) or atomic add into slot band % 32.  Thread j
  // owns channel offset j of the workgroup's CT*V channels, so each
  // wave-instruction of atomics covers 256 contiguous bytes (the full-rate
  // shape for float atomics).
  const int64_t orow = (int64_t)(det ? blockIdx.x : (blockIdx.x & (NSLOT - 1))) * 2 * C;
  float* out = ws + orow;
  const int CW = t.CT * V;                          // channels of this workgroup
  const int cbase = blockIdx.y * t.CT * V;          // first channel
  for (int pass = 0; pass < (dual ? 3 : 2); ++pass) {
    const float* acc = pass == 0 ? a0 : pass == 1 ? a1 : a2;
    __syncthreads();
    if (t.ty < t.RT) {
#pragma unroll
      for (int i = 0; i < V; ++i) red[threadIdx.x * V + i] = acc[i];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < CW; j += blockDim.x) {
      if (cbase + j >= C) break;
      float sum = red[j];
      for (int k = 1; k < t.RT; ++k) sum += red[k * CW + j];
      // pass 0 (sum g) goes to both workspaces, pass 2 is the second BN's row 1
      float* dst = pass < 2 ? out + pass * C : ws2 + orow + C;
      if (det) dst[cbase + j] = sum;
      else atomicAdd(dst + cbase + j, sum);
      if (pass == 0 && dual) {
        if (det) ws2[orow + cbase + j] = sum;
        else atomicAdd(ws2 + orow + cbase + j, sum);
      }
    }
  }
}

// Deterministic ordered sum of nb partial rows ws[k][2][C] for the 64
// channels of this workgroup: thread (c, grp) sums rows grp, grp+4, ... in
// order, then the 4 group sums are added in fixed order.  Returns true for the
// thread that owns channel c (grp == 0) with the totals in *s0, *s1.
__device__ __forceinline__ bool band_sum(const float* __restrict__ ws, int nb, int C, int* cout, float* s0,
                                         float* s1) {
  __shared__ float red[2][FIN_GROUPS][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a = 0.f, b = 0.f;
  if (c < C) {
    for (int k = grp; k < nb; k += FIN_GROUPS) {
      a += ws[(int64_t)k * 2 * C + c];
      b += ws[(int64_t)k * 2 * C + C + c];
    }
  }
  red[0][grp][cl] = a;
  red[1][grp][cl] = b;
  __syncthreads();
  if (grp != 0 || c >= C) return false;
#pragma unroll
  for (int g = 1; g < FIN_GROUPS; ++g) {
    a += red[0][g][cl];
    b += red[1][g][cl];
  }
  *cout = c;
  *s0 = a;
  *s1 = b;
  return true;
}

// colsum finalize: out0[c] (+)= sum, out1[c] (+)= sumsq
__global__ void colsum_finalize_k(const float* __restrict__ ws, int nb, int C, float* __restrict__ out0,
                                  float* __restrict__ out1, int accumulate) {
  int c;
  float s0, s1;
  if (!band_sum(ws, nb, C, &c, &s0, &s1)) return;
  if (out0) out0[c] = accumulate ? out0[c] + s0 : s0;
  if (out1) out1[c] = accumulate ? out1[c] + s1 : s1;
}

// forward finalize: mean/var -> invstd, scale/shift, running stats
__global__ void bn_fwd_finalize_k(const float* __restrict__ ws, int nb, int C, const float* __restrict__ gamma,
                                  const float* __restrict__ beta, float* __restrict__ run_mean,
                                  float* __restrict__ run_var, float* __restrict__ mean, float* __restrict__ invstd,
                                  float* __restrict__ scale, float* __restrict__ shift, float count, float momentum,
                                  float eps) {
  int c;
  float s0, s1;
  if (!band_sum(ws, nb, C, &c, &s0, &s1)) return;
  float mu = s0 / count;
  float var = fmaxf(s1 / count - mu * mu, 0.f);
  float is = rsqrtf(var + eps);
  mean[c] = mu;
  invstd[c] = is;
  float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - mu * g * is;
  if (run_mean) {
    float unbiased = count > 1.f ? var * count / (count - 1.f) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
  }
}

// backward finalize: coefficients for dx = k*g + b*x + a; dgamma/dbeta
// accumulated into dg/db (the flat fp32 gradient buffer views).
__global__ void bn_bwd_finalize_k(const float* __restrict__ ws, int nb, int C, const float* __restrict__ gamma,
                                  const float* __restrict__ mean, const float* __restrict__ invstd,
                                  float* __restrict__ coef, float* __restrict__ dg, float* __restrict__ db,
                                  float count) {
  int c;
  float sdy, sdyx;
  if (!band_sum(ws, nb, C, &c, &sdy, &sdyx)) return;
  float is = invstd[c];
  float k = (gamma ? gamma[c] : 1.f) * is;
  float bcoef = -k * is * sdyx / count;
  float acoef = -k * sdy / count - bcoef * mean[c];
  coef[c] = k;
  coef[C + c] = bcoef;
  coef[2 * C + c] = acoef;
  if (dg) dg[c] += sdyx;
  if (db) db[c] += sdy;
}

// BN(+ReLU) backward of a BN whose output feeds ONE convolution and nothing
// else, without a reduction pass over (dy, x): sdy = sum of the ReLU-masked
// gradient comes from that conv's data-gradient epilogue (ws1: NSLOT slot
// rows, first half); for sum(g~ * xhat), with y = relu(gamma*xhat + beta) the
// conv input, g~ = dy*[y>0] and x_hat = (y - beta)/gamma wherever y > 0,
//   sum_p g~ xhat = (sum_p dy*y - beta*sdy) / gamma,
// and sum_p dy[p,c]*y[p,c] = sum_{k,taps} W[k,c,tap]*dW[k,c,tap] (the adjoint
// of the convolution, padding included), accumulated per input channel by the
// conv's weight-gradient epilogue into `wdot`.  The recovery divides by gamma:
// `flag` is raised when any |gamma_c| < tau (or |beta_c| > 4 |gamma_c|: the recovered sum divides by gamma after subtracting beta sum(g~), so a larger ratio amplifies the bf16 rounding of y and the wgrad error -- 4.25 % at 15x in tests/test_models_gpu.py gate_edge), and then the gated
// exact reduction (colpart_k over dy, x and the mask bits, into ws2) runs and
// the finalize uses its sums instead.  (The gate itself is evaluated by the
// conv's <W, dW> pass, wdot_colsum_k in igemm.hip, into the flag.)
__global__ void bn_bwd_finalize_wdot_k(const float* __restrict__ ws1, const float* __restrict__ ws2, int nb, int C,
                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                       const float* __restrict__ wdot, const int* __restrict__ flag,
                                       const float* __restrict__ mean, const float* __restrict__ invstd,
                                       float* __restrict__ coef, float* __restrict__ dg, float* __restrict__ db,
                                       float count) {
  int c;
  float sdy, sdyx;
  const bool exact = *flag != 0;
  if (!band_sum(exact ? ws2 : ws1, nb, C, &c, &sdy, &sdyx)) return;
  if (!exact) sdyx = (wdot[c] - beta[c] * sdy) / gamma[c];
  float is = invstd[c];
  float k = gamma[c] * is;
  float bcoef = -k * is * sdyx / count;
  float acoef = -k * sdy / count - bcoef * mean[c];
  coef[c] = k;
  coef[C + c] = bcoef;
  coef[2 * C + c] = acoef;
  if (dg) dg[c] += sdyx;
  if (db) db[c] += sdy;
}

// inference: scale/shift from running stats
__global__ void bn_infer_params_k(const float* __restrict__ gamma, const float* __restrict__ beta,
                                  const float* __restrict__ run_mean, const float* __restrict__ run_var,
                                  float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ mean,
                                  float* __restrict__ invstd, int C, float eps) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float is = rsqrtf(run_var[c] + eps);
  float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - run_mean[c] * g * is;
  if (mean) mean[c] = run_mean[c];
  if (invstd) invstd[c] = is;
}

// y = act(x*scale + shift + res).  UR rows (stride = grid row step) are
// loaded before any is stored, so each thread keeps UR (x2 with a residual)
// 16-byte loads in flight: the kernel is HBM-bound and one load per thread
// per iteration leaves the memory pipeline half idle.
template <typename T, int V, bool AFF2 = false, bool CS = false>
__device__ __forceinline__ void bn_apply_row(const float* v0, const float* rv, const float* sc, const float* sf,
                                             T* y, uint8_t* mask, int64_t o, int relu, const float* sc2 = nullptr,
                                             const float* sf2 = nullptr, float* cs = nullptr) {
  float v[V];
  if constexpr (AFF2) {
    // the residual is itself a BN input (a downsample branch): res = x2*scale2 + shift2,
    // rounded to T as the separate BN pass would have stored it (bitwise-equal results)
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = v0[k] * sc[k] + sf[k] + (float)(T)(rv[k] * sc2[k] + sf2[k]);
  } else {
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = v0[k] * sc[k] + sf[k] + (rv ? rv[k] : 0.f);
  }
  if (relu) {
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = fmaxf(v[k], 0.f);
  }
  stv_nt<T, V>(y + o, v);
  if constexpr (CS) {  // column sums of the stored output
#pragma unroll
    for (int k = 0; k < V; ++k) cs[k] += (float)(T)v[k];
  }
  if (V == 8 && mask) {  // bit k = (stored output of channel c0+k) > 0
    unsigned b = 0;
#pragma unroll
    for (int k = 0; k < V; ++k) b |= ((float)(T)v[k] > 0.f ? 1u : 0u) << k;
    mask[o >> 3] = (uint8_t)b;
  }
}

// Rows of one workgroup: rpw > 0 -- the contiguous block [bid*rpw, +rpw)
// (every workgroup streams one contiguous span; the grid is as large as the
// tensor needs), rpw == 0 -- the legacy grid-stride walk.  Measured on
// MI355X (tools/probes/bw_probe.hip, profiles/bw_probe_copy.jsonl): a
// 1.6 GB copy runs at 6.0-6.5 TB/s with contiguous per-workgroup spans and
// non-temporal accesses vs 4.5-4.7 TB/s grid-stride over 2048 workgroups.
struct RowSpan {
  int64_t r, end, step;
};
__device__ __forceinline__ RowSpan row_span(const Tile2D& t, int64_t R, int64_t rpw) {
  RowSpan s;
  if (rpw > 0) {
    const int64_t r0 = (int64_t)blockIdx.x * rpw;
    s.r = r0 + t.ty;
    s.end = r0 + rpw < R ? r0 + rpw : R;
    s.step = t.RT;
  } else {
    s.r = (int64_t)blockIdx.x * t.RT + t.ty;
    s.end = R;
    s.step = (int64_t)t.RT * gridDim.x;
  }
  return s;
}

template <typename T, int V, int UR, bool AFF2 = false, bool CS = false>
__global__ void __launch_bounds__(256) bn_apply_k(const T* __restrict__ x, const float* __restrict__ scale,
                                                  const float* __restrict__ shift, const T* __restrict__ res,
                                                  T* __restrict__ y, uint8_t* __restrict__ mask, int64_t R, int C,
                                                  int relu, int64_t rpw, const float* __restrict__ scale2,
                                                  const float* __restrict__ shift2, float* __restrict__ colsum = nullptr) {
  const Tile2D t = tile2d<V>(C);
  // CS (a separate instantiation, C % 64 == 0 host-checked: every thread
  // owns a channel chunk): also the column sums of the output, reduced over
  // the workgroup's row lanes in LDS, one atomic per channel
  float csum[V];
#pragma unroll
  for (int k = 0; k < V; ++k) csum[k] = 0.f;
  if (!CS && !t.cok) return;
  float sc[V], sf[V], sc2[V], sf2[V];
  ldc<V>(scale + t.c0, sc);
  ldc<V>(shift + t.c0, sf);
  if constexpr (AFF2) {  // a separate instantiation: the plain apply's code is untouched
    ldc<V>(scale2 + t.c0, sc2);
    ldc<V>(shift2 + t.c0, sf2);
  }
  RowSpan sp = row_span(t, R, rpw);
  const int64_t step = sp.step;
  int64_t r = sp.r;
  for (; r + (UR - 1) * step < sp.end; r += UR * step) {
    float v[UR][V], rv[UR][V];
#pragma unroll
    for (int u = 0; u < UR; ++u) ldv_nt<T, V>(x + (r + u * step) * C + t.c0, v[u]);
    if (res) {
#pragma unroll
      for (int u = 0; u < UR; ++u) ldv_nt<T, V>(res + (r + u * step) * C + t.c0, rv[u]);
    }
#pragma unroll
    for (int u = 0; u < UR; ++u)
      bn_apply_row<T, V, AFF2, CS>(v[u], res ? rv[u] : nullptr, sc, sf, y, mask, (r + u * step) * C + t.c0, relu,
                                   sc2, sf2, csum);
  }
  for (; r < sp.end; r += step) {
    float v[V], rv[V];
    const int64_t o = r * C + t.c0;
    ldv_nt<T, V>(x + o, v);
    if (res) ldv_nt<T, V>(res + o, rv);
    bn_apply_row<T, V, AFF2, CS>(v, res ? rv : nullptr, sc, sf, y, mask, o, relu, sc2, sf2, csum);
  }
  if constexpr (CS) {
    __shared__ float red[256 * V];
#pragma unroll
    for (int k = 0; k < V; ++k) red[threadIdx.x * V + k] = csum[k];
    __syncthreads();
    const int CW = t.CT * V;
    for (int j = threadIdx.x; j < CW; j += blockDim.x) {
      const int cc = blockIdx.y * CW + j;
      float a = 0.f;
      for (int q = 0; q < t.RT; ++q) a += red[(q * t.CT + j / V) * V + (j % V)];
      atomicAdd(colsum + (int64_t)(blockIdx.x & (NSLOT - 1)) * C + cc, a);  // 32 slot rows: no hot addresses
    }
  }
}

// g = mask(dy); dx = k*g + b*x + a; dres = g (residual branch).  UR rows
// are loaded before any is stored (see bn_apply_k).
template <typename T, int V, bool PG = false>
__device__ __forceinline__ void bn_bwd_load(const T* x, const T* dy, const T* y, int64_t o, int mask_mode, float* v,
                                            float* g, float* yy, unsigned& mb, const PoolG* pg = nullptr,
                                            int64_t row = 0, int C = 0, int c0 = 0) {
  ldv_nt<T, V>(x + o, v);
  if constexpr (PG) pool_grad8(*pg, row, C, c0, g);
  else ldv_nt<T, V>(dy + o, g);
  if (mask_mode == MASK_Y) ldv_nt<T, V>(y + o, yy);
  else if (V == 8 && mask_mode == MASK_BITS) mb = ((const uint8_t*)y)[o >> 3];
}

template <typename T, int V, bool DUAL = false>
__device__ __forceinline__ void bn_bwd_row(const float* v, float* g, const float* yy, unsigned mb, const float* kk,
                                           const float* bb, const float* aa, const float* sc, const float* sf,
                                           T* dx, T* dres, int64_t o, int mask_mode, const T* x2 = nullptr,
                                           const float* k2 = nullptr, const float* b2 = nullptr,
                                           const float* a2 = nullptr, T* dx2 = nullptr) {
  if (mask_mode == MASK_Y) {
#pragma unroll
    for (int k = 0; k < V; ++k) g[k] = yy[k] > 0.f ? g[k] : 0.f;
  } else if (V == 8 && mask_mode == MASK_BITS) {
#pragma unroll
    for (int k = 0; k < V; ++k) g[k] = (mb >> k) & 1u ? g[k] : 0.f;
  } else if (mask_mode == MASK_AFFINE) {
#pragma unroll
    for (int k = 0; k < V; ++k) g[k] = v[k] * sc[k] + sf[k] > 0.f ? g[k] : 0.f;
  }
  if (dres) stv_nt<T, V>(dres + o, g);
  float o8[V];
#pragma unroll
  for (int k = 0; k < V; ++k) o8[k] = kk[k] * g[k] + bb[k] * v[k] + aa[k];
  stv_nt<T, V>(dx + o, o8);
  if constexpr (DUAL) {  // the second BN (downsample branch) fed the same g
    float w[V];
    ldv_nt<T, V>(x2 + o, w);
#pragma unroll
    for (int k = 0; k < V; ++k) o8[k] = k2[k] * g[k] + b2[k] * w[k] + a2[k];
    stv_nt<T, V>(dx2 + o, o8);
  }
}

template <typename T, int V, int UR, bool DUAL = false, bool PG = false>
__global__ void __launch_bounds__(256) bn_bwd_apply_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                      const T* __restrict__ y, const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      const float* __restrict__ coef, T* __restrict__ dx,
                                                      T* __restrict__ dres, int64_t R, int C, int mask_mode,
                                                      int64_t rpw, const T* __restrict__ x2 = nullptr,
                                                      const float* __restrict__ coef2 = nullptr,
                                                      T* __restrict__ dx2 = nullptr, const PoolG pg = PoolG{}) {
  const Tile2D t = tile2d<V>(C);
  if (!t.cok) return;
  float kk[V], bb[V], aa[V], sc[V], sf[V], k2[V], b2[V], a2[V];
  ldc<V>(coef + t.c0, kk);
  ldc<V>(coef + C + t.c0, bb);
  ldc<V>(coef + 2 * C + t.c0, aa);
  if constexpr (DUAL) {
    ldc<V>(coef2 + t.c0, k2);
    ldc<V>(coef2 + C + t.c0, b2);
    ldc<V>(coef2 + 2 * C + t.c0, a2);
  }
  if (mask_mode == MASK_AFFINE) {
    ldc<V>(scale + t.c0, sc);
    ldc<V>(shift + t.c0, sf);
  }
  RowSpan sp = row_span(t, R, rpw);
  const int64_t step = sp.step;
  int64_t r = sp.r;
  for (; r + (UR - 1) * step < sp.end; r += UR * step) {
    float v[UR][V], g[UR][V], yy[UR][V];
    unsigned mb[UR] = {};
#pragma unroll
    for (int u = 0; u < UR; ++u)
      bn_bwd_load<T, V, PG>(x, dy, y, (r + u * step) * C + t.c0, mask_mode, v[u], g[u], yy[u], mb[u], &pg,
                            r + u * step, C, t.c0);
#pragma unroll
    for (int u = 0; u < UR; ++u)
      bn_bwd_row<T, V, DUAL>(v[u], g[u], yy[u], mb[u], kk, bb, aa, sc, sf, dx, dres, (r + u * step) * C + t.c0,
                             mask_mode, x2, k2, b2, a2, dx2);
  }
  for (; r < sp.end; r += step) {
    float v[V], g[V], yy[V];
    unsigned mb = 0;
    const int64_t o = r * C + t.c0;
    bn_bwd_load<T, V, PG>(x, dy, y, o, mask_mode, v, g, yy, mb, &pg, r, C, t.c0);
    bn_bwd_row<T, V, DUAL>(v, g, yy, mb, kk, bb, aa, sc, sf, dx, dres, o, mask_mode, x2, k2, b2, a2, dx2);
  }
}

// Column sums of a [R][C] tensor ACCUMULATED into out[C] with one atomic per
// column per workgroup: rl row lanes x C/8 column vectors per workgroup, a
// contiguous span of rpb rows each, LDS combine of the row lanes.
template <typename T>
__global__ void __launch_bounds__(256) colsum_acc_k(const T* __restrict__ x, float* __restrict__ out, int64_t R,
                                                    int C, int64_t rpb) {
  extern __shared__ float red[];  // [rl][C]
  const int cv = C >> 3, rl = blockDim.x / cv;
  const int lane_r = threadIdx.x / cv, c0 = (threadIdx.x - lane_r * cv) * 8;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < R ? r0 + rpb : R;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int64_t r = r0 + lane_r; r < r1; r += rl) {
    float v[8];
    ldv<T, 8>(x + r * C + c0, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += v[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[lane_r * C + c0 + e] = acc[e];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float t = 0.f;
    for (int l = 0; l < rl; ++l) t += red[l * C + c];
    atomicAdd(out + c, t);
  }
}

}  // namespace sg

using namespace sg;


// number of row bands for a [R][C] column reduction
extern "C" int sg_colreduce_bands(int64_t R, int C) {
  const int V = (C % 8 == 0) ? 8 : 1;
  const int chunks = C / V;
  const int CT = chunks < 64 ? chunks : 64;
  const int cblocks = (chunks + CT - 1) / CT;
  int64_t want = 1024 / cblocks;  // ~4 workgroups per CU in total
  if (want < 1) want = 1;
  int64_t minrows = 64;
  int64_t bands = (R + minrows - 1) / minrows;
  if (bands > want) bands = want;
  return (int)(bands < 1 ? 1 : bands);
}

// workspace floats needed by a [R][C] column reduction: bands*2*C
extern "C" int64_t sg_colreduce_ws(int64_t R, int C) {
  return (int64_t)(g_bn_det ? sg_colreduce_bands(R, C) : NSLOT) * 2 * C;
}
extern "C" void sg_bn_set_deterministic(int on) { g_bn_det = on; }
// Rows per iteration of the HBM-bound apply kernels (1, 2 or 4; 0 = the
// measured default: 1, and 2 for the backward apply on the legacy
// grid-stride walk).
// tools/bench_bn.py on MI355X (profiles/bn_apply_bandwidth_b512.jsonl): both
// run at 90-100% of a torch copy's bandwidth (4.5-6.3 TB/s) already with one
// row in flight; deeper unrolls only add VGPR pressure.
static int g_bn_ur = 0;
extern "C" void sg_bn_set_unroll(int ur) { g_bn_ur = (ur == 1 || ur == 2 || ur == 4) ? ur : 0; }
#define BN_UR_LAUNCH(K, UR0, T_, V_, ...)                                                   \
  do {                                                                                     \
    const int ur_ = g_bn_ur ? g_bn_ur : (UR0);                                              \
    if (ur_ == 4) hipLaunchKernelGGL((K<T_, V_, 4>), __VA_ARGS__);                         \
    else if (ur_ == 1) hipLaunchKernelGGL((K<T_, V_, 1>), __VA_ARGS__);                    \
    else hipLaunchKernelGGL((K<T_, V_, 2>), __VA_ARGS__);                                  \
  } while (0)
// The next launch that owns a slot-atomic workspace finds it pre-zeroed
// (one-shot flag: consumed by that launch)
extern "C" void sg_set_ws_prezeroed(int on) { g_ws_prezeroed = on; }
extern "C" int sg_ws_prezeroed() {
  const int pz = g_ws_prezeroed;
  g_ws_prezeroed = 0;
  return pz;
}
extern "C" void sg_zero(void* p, int64_t bytes, hipStream_t s) { sg_zero_async(p, (size_t)bytes, s); }
extern "C" int sg_bn_deterministic() { return g_bn_det; }

// rows the finalize sums for a reduction launched on `grid`
static inline int fin_rows(const dim3& grid) { return g_bn_det ? (int)grid.x : NSLOT; }
static inline void zero_ws(void* ws, int C, hipStream_t s) {
  const int pz = g_ws_prezeroed;  // one-shot: set by the caller for this launch only
  g_ws_prezeroed = 0;
  if (!g_bn_det && !pz) sg_zero_async(ws, sizeof(float) * NSLOT * 2 * C, s);
}

static inline dim3 fin_grid(int C) { return dim3((C + 63) / 64); }

static inline void colgrid(int64_t R, int C, dim3& grid, int& rpb, int& V) {
  V = (C % 8 == 0) ? 8 : 1;
  const int chunks = C / V;
  const int CT = chunks < 64 ? chunks : 64;
  const int cblocks = (chunks + CT - 1) / CT;
  // deterministic: the partial-row workspace is sized by sg_colreduce_bands;
  // slot atomics: one band per 16 rows per thread (a contiguous span per
  // workgroup, the grid sized to the tensor -- see bn_apply_k)
  int64_t bands = sg_colreduce_bands(R, C);
  if (!g_bn_det) {
    const int64_t rpw = (int64_t)(256 / CT) * 16;
    const int64_t nb = (R + rpw - 1) / rpw;
    if (nb > bands) bands = nb < 1048576 ? nb : 1048576;
  }
  rpb = (int)((R + bands - 1) / bands);
  grid = dim3((unsigned)bands, cblocks);
}

// Rows per thread of the contiguous-span apply (0: legacy grid-stride over
// at most 2048 workgroups).  2 measured best over ResNet-50 shapes
// (tools/bench_bn.py, profiles/bn_apply_bandwidth_spans_b512.jsonl): +15-30 %
// over the grid-stride walk, 5.6-6.8 TB/s.
static int g_bn_rpt = 2;
extern "C" void sg_bn_set_rows_per_thread(int rpt) { g_bn_rpt = rpt < 0 ? 0 : rpt; }
static inline dim3 apply_grid(int64_t R, int C, int V, int64_t& rpw) {
  const int chunks = C / V;
  const int CT = chunks < 64 ? chunks : 64;
  const int cblocks = (chunks + CT - 1) / CT;
  const int RT = 256 / CT;
  if (g_bn_rpt > 0) {
    rpw = (int64_t)RT * g_bn_rpt;
    const int64_t rb = (R + rpw - 1) / rpw;
    return dim3((unsigned)(rb < 1 ? 1 : rb), cblocks);
  }
  rpw = 0;
  int64_t rb = (R + RT - 1) / RT;
  int64_t cap = 2048 / cblocks;
  if (cap < 1) cap = 1;
  if (rb > cap) rb = cap;
  return dim3((unsigned)(rb < 1 ? 1 : rb), cblocks);
}

#define DISPATCH_FT(dtype, ...) \
  if ((dtype) == kF32) {        \
    typedef float T;            \
    __VA_ARGS__;                \
  } else {                      \
    typedef bf16 T;             \
    __VA_ARGS__;                \
  }

#define DISPATCH_V(Vv, ...)       \
  if ((Vv) == 8) {                \
    constexpr int VV = 8;         \
    __VA_ARGS__;                  \
  } else {                        \
    constexpr int VV = 1;         \
    __VA_ARGS__;                  \
  }

extern "C" {

// out0/out1 (fp32 [C]) = column sums (accumulate != 0: added to existing)
void sg_colsum(const void* x, void* ws, void* out0, void* out1, int64_t R, int C, int dtype, int accumulate,
               hipStream_t s) {
  if (accumulate && !out1 && !g_bn_det && C % 8 == 0 && C <= 2048 && R <= (int64_t)1 << 20) {
    // bias gradient accumulated into a flat-store view: one launch (no
    // workspace zeroing, no finalize pass) -- these are launch-latency bound
    const int cv = C / 8, rl = 256 / cv;
    int64_t chunks = (R + 31) / 32;
    const unsigned grid = (unsigned)(chunks < 512 ? chunks : 512);
    const int64_t rpb = (R + grid - 1) / grid;
    DISPATCH_FT(dtype, hipLaunchKernelGGL(colsum_acc_k<T>, dim3(grid), dim3(rl * cv), (size_t)rl * C * sizeof(float), s,
                                          (const T*)x, (float*)out0, R, C, rpb));
    return;
  }
  dim3 grid;
  int rpb, V;
  colgrid(R, C, grid, rpb, V);
  zero_ws(ws, C, s);
  DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((colpart_k<T, 0, VV>), grid, dim3(256), 0, s, (const T*)x,
                                                      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                                      (float*)ws, R, C, rpb, 0, g_bn_det)));
  hipLaunchKernelGGL(colsum_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws, fin_rows(grid), C,
                     (float*)out0, (float*)out1, accumulate);
}

void sg_bn_fwd_stats(const void* x, void* ws, const void* gamma, const void* beta, void* run_mean, void* run_var,
                     void* mean, void* invstd, void* scale, void* shift, int64_t R, int C, float momentum, float eps,
                     int dtype, hipStream_t s) {
  dim3 grid;
  int rpb, V;
  colgrid(R, C, grid, rpb, V);
  zero_ws(ws, C, s);
  DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((colpart_k<T, 0, VV>), grid, dim3(256), 0, s, (const T*)x,
                                                      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                                      (float*)ws, R, C, rpb, 0, g_bn_det)));
  hipLaunchKernelGGL(bn_fwd_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws, fin_rows(grid), C,
                     (const float*)gamma, (const float*)beta, (float*)run_mean, (float*)run_var, (float*)mean,
                     (float*)invstd, (float*)scale, (float*)shift, (float)R, momentum, eps);
}

// finalize only: the per-tile column sums were produced by the conv
// epilogue (igemm stats) into ws [nb][2][C]
void sg_bn_fwd_from_ws(const void* ws, int nb, const void* gamma, const void* beta, void* run_mean, void* run_var,
                       void* mean, void* invstd, void* scale, void* shift, int64_t R, int C, float momentum,
                       float eps, hipStream_t s) {
  hipLaunchKernelGGL(bn_fwd_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws, nb, C,
                     (const float*)gamma, (const float*)beta, (float*)run_mean, (float*)run_var, (float*)mean,
                     (float*)invstd, (float*)scale, (float*)shift, (float)R, momentum, eps);
}

void sg_bn_infer_params(const void* gamma, const void* beta, const void* run_mean, const void* run_var, void* scale,
                        void* shift, void* mean, void* invstd, int C, float eps, hipStream_t s) {
  hipLaunchKernelGGL(bn_infer_params_k, dim3((C + 255) / 256), dim3(256), 0, s, (const float*)gamma,
                     (const float*)beta, (const float*)run_mean, (const float*)run_var, (float*)scale,
                     (float*)shift, (float*)mean, (float*)invstd, C, eps);
}

// mask (optional, C % 8 == 0 only): 1-bit ReLU mask [R][C/8] of the output
void sg_bn_apply(const void* x, const void* scale, const void* shift, const void* res, void* y, void* mask, int64_t R,
                 int C, int relu, int dtype, hipStream_t s) {
  const int V = (C % 8 == 0) ? 8 : 1;
  int64_t rpw;
  dim3 grid = apply_grid(R, C, V, rpw);
  DISPATCH_FT(dtype, DISPATCH_V(V, BN_UR_LAUNCH(bn_apply_k, 1, T, VV, grid, dim3(256), 0, s, (const T*)x,
                                                      (const float*)scale, (const float*)shift, (const T*)res, (T*)y,
                                                      (uint8_t*)mask, R, C, relu, rpw, nullptr, nullptr)));
}

// sg_bn_apply (bf16, no residual, C % 64 == 0) that also ADDS the column sums
// of the stored output into 32 slot rows colsum[32][C] (zeroed by the caller:
// one row per workgroup & 31 -- a single row made thousands of workgroups'
// atomics collide on C addresses, 8x slower than the apply itself): the input
// column sums of a consuming fused residual tail (bnres.hip), for free in
// this HBM-bound pass instead of a separate read of its output
void sg_bn_apply_cs(const void* x, const void* scale, const void* shift, void* y, void* mask, void* colsum, int64_t R,
                    int C, int relu, hipStream_t s) {
  if ((C & 63) != 0) throw std::runtime_error("bn_apply_cs: C % 64 required");
  int64_t rpw;
  dim3 grid = apply_grid(R, C, 8, rpw);
  hipLaunchKernelGGL((bn_apply_k<bf16, 8, 2, false, true>), grid, dim3(256), 0, s, (const bf16*)x,
                     (const float*)scale, (const float*)shift, (const bf16*)nullptr, (bf16*)y, (uint8_t*)mask, R, C,
                     relu, rpw, nullptr, nullptr, (float*)colsum);
}

// y = act(x*scale + shift + x2*scale2 + shift2): a BN whose residual is the
// (not materialised) output of a second BN -- the downsample branch
void sg_bn_apply2(const void* x, const void* scale, const void* shift, const void* x2, const void* scale2,
                  const void* shift2, void* y, void* mask, int64_t R, int C, int relu, int dtype, hipStream_t s) {
  const int V = (C % 8 == 0) ? 8 : 1;
  int64_t rpw;
  dim3 grid = apply_grid(R, C, V, rpw);
  DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((bn_apply_k<T, VV, 1, true>), grid, dim3(256), 0, s,
                                                      (const T*)x, (const float*)scale, (const float*)shift,
                                                      (const T*)x2, (T*)y, (uint8_t*)mask, R, C, relu, rpw,
                                                      (const float*)scale2, (const float*)shift2)));
}

// Full BN backward: reduce + finalize (coef, dgamma/dbeta accumulation) + apply.
// mask_mode: 0 none, 1 mask from y (y>0), 2 mask from x*scale+shift>0,
// 3 mask bits (y points at the [R][C/8] bitmask; C % 8 == 0).
void sg_bn_bwd(const void* x, const void* dy, const void* y, const void* scale, const void* shift, const void* mean,
               const void* invstd, const void* gamma, void* ws, void* coef, void* dg, void* db, void* dx, void* dres,
               int64_t R, int C, int mask_mode, int dtype, hipStream_t s) {
  dim3 grid;
  int rpb, V;
  colgrid(R, C, grid, rpb, V);
  zero_ws(ws, C, s);
  DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((colpart_k<T, 1, VV>), grid, dim3(256), 0, s, (const T*)x,
                                                      (const T*)dy, (const T*)y, (const float*)scale,
                                                      (const float*)shift, (const float*)mean, (const float*)invstd,
                                                      (float*)ws, R, C, rpb, mask_mode, g_bn_det)));
  hipLaunchKernelGGL(bn_bwd_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws, fin_rows(grid), C,
                     (const float*)gamma, (const float*)mean, (const float*)invstd, (float*)coef, (float*)dg,
                     (float*)db, (float)R);
  int64_t rpw;
  dim3 ag = apply_grid(R, C, V, rpw);
  DISPATCH_FT(dtype, DISPATCH_V(V, BN_UR_LAUNCH(bn_bwd_apply_k, g_bn_rpt ? 1 : 2, T, VV, ag, dim3(256), 0, s, (const T*)x,
                                                      (const T*)dy, (const T*)y, (const float*)scale,
                                                      (const float*)shift, (const float*)coef, (T*)dx, (T*)dres, R,
                                                      C, mask_mode, rpw)));
}

// BN(+ReLU) backward of the fused stem BN+ReLU+max-pool: the gradient at
// the BN output is gathered from the pooled gradient dyp and the window
// argmax inside the reduction and apply passes -- the full-resolution
// max-pool backward output is never written (bf16, C % 8 == 0, ReLU mask
// recomputed from x).
void sg_bn_bwd_pool(const void* x, const void* dyp, const void* arg, const void* scale, const void* shift,
                    const void* mean, const void* invstd, const void* gamma, void* ws, void* coef, void* dg, void* db,
                    void* dx, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph,
                    int pw, hipStream_t s) {
  const int64_t R = (int64_t)N * H * W;
  PoolG pg{(const bf16*)dyp, (const uint8_t*)arg, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, FastDiv(W), FastDiv(H)};
  dim3 grid;
  int rpb, V;
  colgrid(R, C, grid, rpb, V);
  if (V != 8) throw std::runtime_error("sg_bn_bwd_pool: needs C % 8 == 0");
  zero_ws(ws, C, s);
  hipLaunchKernelGGL((colpart_k<bf16, 1, 8, true>), grid, dim3(256), 0, s, (const bf16*)x, nullptr, nullptr,
                     (const float*)scale, (const float*)shift, (const float*)mean, (const float*)invstd, (float*)ws,
                     R, C, rpb, (int)MASK_AFFINE, g_bn_det, nullptr, nullptr, nullptr, nullptr, pg);
  hipLaunchKernelGGL(bn_bwd_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws, fin_rows(grid), C,
                     (const float*)gamma, (const float*)mean, (const float*)invstd, (float*)coef, (float*)dg,
                     (float*)db, (float)R);
  int64_t rpw;
  dim3 ag = apply_grid(R, C, 8, rpw);
  hipLaunchKernelGGL((bn_bwd_apply_k<bf16, 8, 2, false, true>), ag, dim3(256), 0, s, (const bf16*)x, nullptr,
                     nullptr, (const float*)scale, (const float*)shift, (const float*)coef, (bf16*)dx, nullptr, R, C,
                     (int)MASK_AFFINE, rpw, nullptr, nullptr, nullptr, pg);
}

// Backward of y = relu(BN1(x) + BN2(x2)) (mask bits from the forward): one
// reduction pass for both BNs (sum g shared), two finalizes, one apply pass
// writing dx and dx2 -- the residual gradient g is never materialised.
void sg_bn_bwd2(const void* x, const void* dy, const void* mask, const void* mean, const void* invstd,
                const void* gamma, const void* x2, const void* mean2, const void* invstd2, const void* gamma2,
                void* ws, void* ws2, void* coef, void* coef2, void* dg, void* db, void* dg2, void* db2, void* dx,
                void* dx2, int64_t R, int C, int dtype, hipStream_t s) {
  dim3 grid;
  int rpb, V;
  colgrid(R, C, grid, rpb, V);
  zero_ws(ws, C, s);
  if (!g_bn_det) sg_zero_async(ws2, sizeof(float) * NSLOT * 2 * C, s);
  DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((colpart_k<T, 2, VV>), grid, dim3(256), 0, s, (const T*)x,
                                                      (const T*)dy, (const T*)mask, nullptr, nullptr,
                                                      (const float*)mean, (const float*)invstd, (float*)ws, R, C, rpb,
                                                      (int)MASK_BITS, g_bn_det, (const T*)x2, (const float*)mean2,
                                                      (const float*)invstd2, (float*)ws2)));
  hipLaunchKernelGGL(bn_bwd_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws, fin_rows(grid), C,
                     (const float*)gamma, (const float*)mean, (const float*)invstd, (float*)coef, (float*)dg,
                     (float*)db, (float)R);
  hipLaunchKernelGGL(bn_bwd_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws2, fin_rows(grid), C,
                     (const float*)gamma2, (const float*)mean2, (const float*)invstd2, (float*)coef2, (float*)dg2,
                     (float*)db2, (float)R);
  int64_t rpw;
  dim3 ag = apply_grid(R, C, V, rpw);
  DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((bn_bwd_apply_k<T, VV, 1, true>), ag, dim3(256), 0, s,
                                                      (const T*)x, (const T*)dy, (const T*)mask, nullptr, nullptr,
                                                      (const float*)coef, (T*)dx, nullptr, R, C, (int)MASK_BITS, rpw,
                                                      (const T*)x2, (const float*)coef2, (T*)dx2)));
}

// BN backward whose reduction was fused into the producing conv dgrad's
// epilogue (sums in ws [nb][2][C]): finalize + apply only.
// The identity-sum BN(+ReLU) backward (see bn_bwd_finalize_wdot_k): bf16,
// C % 8 == 0, ReLU mask as the forward's bits, non-deterministic mode.
// ws1: the dgrad epilogue's NSLOT slot rows; wdot [C]; ws2: NSLOT x 2 x C
// scratch for the gated exact reduction; flag: one int of scratch.
void sg_bn_bwd_wdot(const void* x, const void* dy, const void* mask, const void* scale, const void* shift,
                    const void* mean, const void* invstd, const void* gamma, const void* beta, const void* ws1,
                    const void* wdot, void* ws2, void* flag, void* coef, void* dg, void* db, void* dx, int64_t R,
                    int C, float tau, hipStream_t s) {
  // flag: raised (or not) by the consuming conv's wdot pass (wdot_colsum_k)
  (void)tau;
  dim3 grid;
  int rpb, V;
  colgrid(R, C, grid, rpb, V);
  // the gated reduction is normally a no-op: a grid of a few hundred
  // workgroups that read the gate and exit (the full band grid -- up to
  // 6272 workgroups -- cost ~20 us per launch doing nothing, 0.65 ms per
  // ResNet-50 step); when the gate is raised the same grid streams longer bands
  const unsigned cap = grid.y >= 512 ? 1u : 512u / grid.y;
  if (grid.x > cap) {
    grid.x = cap;
    rpb = (int)((R + cap - 1) / cap);
  }
  zero_ws(ws2, C, s);
  hipLaunchKernelGGL((colpart_k<bf16, 1, 8>), grid, dim3(256), 0, s, (const bf16*)x, (const bf16*)dy,
                     (const bf16*)mask, (const float*)scale, (const float*)shift, (const float*)mean,
                     (const float*)invstd, (float*)ws2, R, C, rpb, (int)MASK_BITS, 0, (const bf16*)nullptr,
                     (const float*)nullptr, (const float*)nullptr, (float*)nullptr, PoolG{}, (const int*)flag);
  hipLaunchKernelGGL(bn_bwd_finalize_wdot_k, fin_grid(C), dim3(256), 0, s, (const float*)ws1, (const float*)ws2,
                     NSLOT, C, (const float*)gamma, (const float*)beta, (const float*)wdot, (const int*)flag,
                     (const float*)mean, (const float*)invstd, (float*)coef, (float*)dg, (float*)db, (float)R);
  int64_t rpw;
  dim3 ag = apply_grid(R, C, 8, rpw);
  BN_UR_LAUNCH(bn_bwd_apply_k, g_bn_rpt ? 1 : 2, bf16, 8, ag, dim3(256), 0, s, (const bf16*)x, (const bf16*)dy,
               (const bf16*)mask, (const float*)scale, (const float*)shift, (const float*)coef, (bf16*)dx,
               (bf16*)nullptr, R, C, (int)MASK_BITS, rpw);
}

void sg_bn_bwd_from_ws(const void* x, const void* dy, const void* y, const void* scale, const void* shift,
                       const void* mean, const void* invstd, const void* gamma, const void* ws, int nb, void* coef,
                       void* dg, void* db, void* dx, void* dres, int64_t R, int C, int mask_mode, int dtype,
                       hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_k, fin_grid(C), dim3(256), 0, s, (const float*)ws, nb, C, (const float*)gamma,
                     (const float*)mean, (const float*)invstd, (float*)coef, (float*)dg, (float*)db, (float)R);
  const int V = (C % 8 == 0) ? 8 : 1;
  int64_t rpw;
  dim3 ag = apply_grid(R, C, V, rpw);
  DISPATCH_FT(dtype, DISPATCH_V(V, BN_UR_LAUNCH(bn_bwd_apply_k, g_bn_rpt ? 1 : 2, T, VV, ag, dim3(256), 0, s, (const T*)x,
                                                      (const T*)dy, (const T*)y, (const float*)scale,
                                                      (const float*)shift, (const float*)coef, (T*)dx, (T*)dres, R,
                                                      C, mask_mode, rpw)));
}

}  // extern "C"

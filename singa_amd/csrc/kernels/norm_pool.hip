// Pooling (max/avg, padded, NHWC), global average pooling and across-channel
// LRN.  (BatchNorm and the column reductions live in batchnorm.hip.)
//
// Reference: Pooling/UnPooling plans (include/mshadow/tensor_expr_ext.h:
// 787-850), channel pooling for LRN (:916-941, F8/F9 in src/worker/layer.cc:
// 356-377).  Layout: activations are [N][H][W][C] (channels_last).
#include <stdlib.h>

#include "common.h"

namespace sg {

// ---------------------------------------------------------------------------
// Pooling, NHWC.  Max pooling stores the argmax window offset (uint8) so the
// backward pass is an exact gather (no atomics, no tie double counting; the
// reference re-compared values, include/mshadow/tensor_base.h:265-267).
// ---------------------------------------------------------------------------
struct PoolGeom {
  int N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw;
};

// One workgroup row of blocks per output row (n, oh): thread item
// i = ow * CV + cv (V channels each); no 64-bit index division per thread.
template <typename T, int V>
__global__ void maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ arg, PoolGeom g) {
  const int CV = g.C / V;
  const int row = blockIdx.x;  // n * Ho + oh
  const int n = row / g.Ho, oh = row - n * g.Ho;
  const int items = g.Wo * CV;
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < items; i += gridDim.y * blockDim.x) {
    const int ow = i / CV, cv = i - ow * CV;
    float m[V];
    uint8_t best[V];
#pragma unroll
    for (int k = 0; k < V; ++k) { m[k] = -INFINITY; best[k] = 0; }
    for (int r = 0; r < g.kh; ++r) {
      const int ih = oh * g.sh - g.ph + r;
      if (ih < 0 || ih >= g.H) continue;
      const T* xr = x + (((int64_t)n * g.H + ih) * g.W) * g.C + cv * V;
      for (int s = 0; s < g.kw; ++s) {
        const int iw = ow * g.sw - g.pw + s;
        if (iw < 0 || iw >= g.W) continue;
        float v[V];
        ldv<T, V>(xr + (int64_t)iw * g.C, v);
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (v[k] > m[k]) { m[k] = v[k]; best[k] = (uint8_t)(r * g.kw + s); }
      }
    }
    const int64_t o = ((int64_t)row * g.Wo + ow) * g.C + cv * V;
    stv<T, V>(y + o, m);
    if (arg) {
      if constexpr (V == 8) {  // the 8 window indices of this vector: one 8-byte store
        uint2 pk;
        pk.x = best[0] | (best[1] << 8) | (best[2] << 16) | ((unsigned)best[3] << 24);
        pk.y = best[4] | (best[5] << 8) | (best[6] << 16) | ((unsigned)best[7] << 24);
        *(uint2*)(arg + o) = pk;
      } else {
#pragma unroll
        for (int k = 0; k < V; ++k) arg[o + k] = best[k];
      }
    }
  }
}

// Fused BatchNorm-apply + ReLU + max pooling (the ResNet stem): the window
// maximum of bf16(relu(x*scale + shift)) -- the same bf16 values a separate
// BN+ReLU pass would write -- with the argmax for the backward gather; the
// full-resolution BN output is never written (its ReLU mask is recomputed from
// x in the BN backward).  bf16, C % 8 == 0.
__global__ void bn_relu_maxpool_fwd_k(const bf16* __restrict__ x, const float* __restrict__ scale,
                                      const float* __restrict__ shift, bf16* __restrict__ y,
                                      uint8_t* __restrict__ arg, PoolGeom g) {
  constexpr int V = 8;
  const int CV = g.C / V;
  const int row = blockIdx.x;  // n * Ho + oh
  const int n = row / g.Ho, oh = row - n * g.Ho;
  const int items = g.Wo * CV;
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < items; i += gridDim.y * blockDim.x) {
    const int ow = i / CV, cv = i - ow * CV;
    float sc[V], sf[V];
    ldc<V>(scale + cv * V, sc);
    ldc<V>(shift + cv * V, sf);
    float m[V];
    uint8_t best[V];
#pragma unroll
    for (int k = 0; k < V; ++k) { m[k] = -INFINITY; best[k] = 0; }
    for (int r = 0; r < g.kh; ++r) {
      const int ih = oh * g.sh - g.ph + r;
      if (ih < 0 || ih >= g.H) continue;
      const bf16* xr = x + (((int64_t)n * g.H + ih) * g.W) * g.C + cv * V;
      for (int s = 0; s < g.kw; ++s) {
        const int iw = ow * g.sw - g.pw + s;
        if (iw < 0 || iw >= g.W) continue;
        float v[V];
        ldv<bf16, V>(xr + (int64_t)iw * g.C, v);
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const float b = (float)(bf16)fmaxf(v[k] * sc[k] + sf[k], 0.f);
          if (b > m[k]) { m[k] = b; best[k] = (uint8_t)(r * g.kw + s); }
        }
      }
    }
    const int64_t o = ((int64_t)row * g.Wo + ow) * g.C + cv * V;
    stv<bf16, V>(y + o, m);
    uint2 pk;
    pk.x = best[0] | (best[1] << 8) | (best[2] << 16) | ((unsigned)best[3] << 24);
    pk.y = best[4] | (best[5] << 8) | (best[6] << 16) | ((unsigned)best[7] << 24);
    *(uint2*)(arg + o) = pk;
  }
}

// bn_relu_maxpool_fwd_k over 2x2 blocks of outputs (3x3 / stride 2 / pad 1,
// Ho and Wo even): the 4 windows of outputs {2i, 2i+1} x {2j, 2j+1} span the
// 5 x 5 input pixels from (4i-1, 4j-1), each loaded and BN+ReLU-transformed
// once (25 instead of 36); taps are visited in the same row-major order, so
// the argmax tie-breaking is unchanged.  Thread = (n, i, j, 8-channel chunk).
__global__ void __launch_bounds__(256) bn_relu_maxpool_332_blk_k(const bf16* __restrict__ x,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift,
                                                               bf16* __restrict__ y, uint8_t* __restrict__ arg,
                                                               int H, int W, int C, int Ho, int Wo, uint32_t total,
                                                               FastDiv dCV, FastDiv dJ, FastDiv dI) {
  constexpr int V = 8;
  const int CV = C >> 3;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const uint32_t p = dCV.div(e);
    const int cv = (int)(e - p * (uint32_t)CV);
    const uint32_t q = dJ.div(p);
    const int j = (int)(p - q * (uint32_t)(Wo >> 1));
    const uint32_t n = dI.div(q);
    const int i = (int)(q - n * (uint32_t)(Ho >> 1));
    float sc[V], sf[V];
    ldc<V>(scale + cv * V, sc);
    ldc<V>(shift + cv * V, sf);
    float m[2][2][V];
    unsigned best[2][2][V];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int k = 0; k < V; ++k) { m[a][b][k] = -INFINITY; best[a][b][k] = 0; }
#pragma unroll
    for (int lr = 0; lr < 5; ++lr) {
      const int ih = 4 * i - 1 + lr;
      if (ih < 0 || ih >= H) continue;
      const bf16* xr = x + (((int64_t)n * H + ih) * W) * C + cv * V;
#pragma unroll
      for (int lc = 0; lc < 5; ++lc) {
        const int iw = 4 * j - 1 + lc;
        if (iw < 0 || iw >= W) continue;
        float v[V];
        ldv<bf16, V>(xr + (int64_t)iw * C, v);
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = (float)(bf16)fmaxf(v[k] * sc[k] + sf[k], 0.f);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int r = lr - 2 * a;
          if (r < 0 || r > 2) continue;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int t = lc - 2 * b;
            if (t < 0 || t > 2) continue;
#pragma unroll
            for (int k = 0; k < V; ++k)
              if (v[k] > m[a][b][k]) { m[a][b][k] = v[k]; best[a][b][k] = (unsigned)(r * 3 + t); }
          }
        }
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int64_t o = (((int64_t)n * Ho + 2 * i + a) * Wo + 2 * j + b) * C + cv * V;
        stv<bf16, V>(y + o, m[a][b]);
        uint2 pk;
        pk.x = best[a][b][0] | (best[a][b][1] << 8) | (best[a][b][2] << 16) | (best[a][b][3] << 24);
        pk.y = best[a][b][4] | (best[a][b][5] << 8) | (best[a][b][6] << 16) | (best[a][b][7] << 24);
        *(uint2*)(arg + o) = pk;
      }
  }
}

// One workgroup row of blocks per input row (n, ih): gather the gradient of
// the windows whose argmax is this pixel.
template <typename T, int V>
__global__ void maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ arg, T* __restrict__ dx,
                              PoolGeom g) {
  const int CV = g.C / V;
  const int row = blockIdx.x;  // n * H + ih
  const int n = row / g.H, ih = row - n * g.H;
  const int oh0 = max(0, (ih + g.ph - g.kh + g.sh) / g.sh), oh1 = min(g.Ho - 1, (ih + g.ph) / g.sh);
  const int items = g.W * CV;
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < items; i += gridDim.y * blockDim.x) {
    const int iw = i / CV, cv = i - iw * CV;
    const int ow0 = max(0, (iw + g.pw - g.kw + g.sw) / g.sw), ow1 = min(g.Wo - 1, (iw + g.pw) / g.sw);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int r = ih + g.ph - oh * g.sh;
      if (r < 0 || r >= g.kh) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int s = iw + g.pw - ow * g.sw;
        if (s < 0 || s >= g.kw) continue;
        const int64_t o = (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + cv * V;
        float d[V];
        ldv<T, V>(dy + o, d);
        const unsigned want = (unsigned)(r * g.kw + s);
        if constexpr (V == 8) {
          const uint2 pk = *(const uint2*)(arg + o);
#pragma unroll
          for (int k = 0; k < V; ++k) acc[k] += (((k < 4 ? pk.x : pk.y) >> (8 * (k & 3))) & 0xffu) == want ? d[k] : 0.f;
        } else {
#pragma unroll
          for (int k = 0; k < V; ++k) acc[k] += arg[o + k] == want ? d[k] : 0.f;
        }
      }
    }
    stv_nt<T, V>(dx + ((int64_t)row * g.W + iw) * g.C + cv * V, acc);
  }
}

// 3x3 / stride 2 / pad 1 max-pool backward (the ResNet stem), bf16 NHWC,
// 8 channels per thread over a flat (n, ih, iw, c/8) index: the covering
// windows in closed form -- input row ih is covered by output row (ih+1)/2
// (tap (ih+1)&1) and, for odd ih, also by (ih+1)/2-1 (tap 2) -- with
// constant-divisor index splits, no window loops, non-temporal stores.
__global__ void __launch_bounds__(256) maxpool_bwd_332_k(const bf16* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                       bf16* __restrict__ dx, int H, int W, int C, int Ho, int Wo,
                                                       uint32_t total, FastDiv dCV, FastDiv dW, FastDiv dH) {
  const int CV = C >> 3;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t p = dCV.div(i);
    const int cv = (int)(i - p * (uint32_t)CV);
    const uint32_t q = dW.div(p);
    const int iw = (int)(p - q * (uint32_t)W);
    const uint32_t n = dH.div(q);
    const int ih = (int)(q - n * (uint32_t)H);
    int ohs[2], rs[2], ows[2], ss[2];
    int nh = 0, nw = 0;
    {
      const int o = (ih + 1) >> 1, r = (ih + 1) & 1;
      if (o < Ho) { ohs[nh] = o; rs[nh] = r; ++nh; }
      if (r == 0 && o >= 1) { ohs[nh] = o - 1; rs[nh] = 2; ++nh; }
    }
    {
      const int o = (iw + 1) >> 1, t = (iw + 1) & 1;
      if (o < Wo) { ows[nw] = o; ss[nw] = t; ++nw; }
      if (t == 0 && o >= 1) { ows[nw] = o - 1; ss[nw] = 2; ++nw; }
    }
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a >= nh) break;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (b >= nw) break;
        const int64_t o = (((int64_t)n * Ho + ohs[a]) * Wo + ows[b]) * C + cv * 8;
        const uint2 pk = *(const uint2*)(arg + o);
        const bf16x8 d = *(const bf16x8*)(dy + o);
        const unsigned want = (unsigned)(rs[a] * 3 + ss[b]);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          acc[k] += (((k < 4 ? pk.x : pk.y) >> (8 * (k & 3))) & 0xffu) == want ? (float)d[k] : 0.f;
      }
    }
    stv_nt<bf16, 8>(dx + (int64_t)i * 8, acc);
  }
}

// Variant of maxpool_bwd_332_k over 2x2 blocks of input pixels: rows
// {2i-1, 2i} x columns {2j-1, 2j} are covered by exactly the windows
// {i-1, i} x {j-1, j}, so each (dy, argmax) vector is loaded once per block
// (4 loads for 4 outputs instead of 9).  Thread = (n, i, j, 8-channel chunk),
// i in [0, Ho], j in [0, Wo] (H = 2 Ho, W = 2 Wo: the host checks).
__global__ void __launch_bounds__(256) maxpool_bwd_332_blk_k(const bf16* __restrict__ dy,
                                                           const uint8_t* __restrict__ arg, bf16* __restrict__ dx,
                                                           int H, int W, int C, int Ho, int Wo, uint32_t total,
                                                           FastDiv dCV, FastDiv dJ, FastDiv dI) {
  const int CV = C >> 3;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const uint32_t p = dCV.div(e);
    const int cv = (int)(e - p * (uint32_t)CV);
    const uint32_t q = dJ.div(p);
    const int j = (int)(p - q * (uint32_t)(Wo + 1));
    const uint32_t n = dI.div(q);
    const int i = (int)(q - n * (uint32_t)(Ho + 1));
    // window (a, b) in {i-1, i} x {j-1, j}: dy / argmax vectors (zero / no match when outside)
    bf16x8 d[2][2];
    uint2 pk[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = i - 1 + a, ow = j - 1 + b;
        const bool ok = oh >= 0 && oh < Ho && ow >= 0 && ow < Wo;
        const int64_t o = (((int64_t)n * Ho + (ok ? oh : 0)) * Wo + (ok ? ow : 0)) * C + cv * 8;
        pk[a][b] = ok ? *(const uint2*)(arg + o) : make_uint2(0xffffffffu, 0xffffffffu);
        d[a][b] = *(const bf16x8*)(dy + o);
      }
    // input pixel (ih, iw) = (2i-1+u, 2j-1+v): window row i-1 covers it at tap 2 (u = 0), row i at tap u
    // (0 for the odd row, 1 for the even one); likewise for columns
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ih = 2 * i - 1 + u;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int iw = 2 * j - 1 + v;
        if (iw < 0 || iw >= W) continue;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (a == 0 && u == 1) continue;  // the even row lies only in window row i
          const int r = a == 0 ? 2 : u;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (b == 0 && v == 1) continue;
            const unsigned want = (unsigned)(r * 3 + (b == 0 ? 2 : v));
#pragma unroll
            for (int k = 0; k < 8; ++k)
              acc[k] += (((k < 4 ? pk[a][b].x : pk[a][b].y) >> (8 * (k & 3))) & 0xffu) == want ? (float)d[a][b][k]
                                                                                                 : 0.f;
          }
        }
        stv_nt<bf16, 8>(dx + (((int64_t)n * H + ih) * W + iw) * C + cv * 8, acc);
      }
    }
  }
}

template <typename T, int V>
__global__ void avgpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, PoolGeom g, int count_pad) {
  const int CV = g.C / V;
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * CV;
  SG_GRID_STRIDE(i, total) {
    const int cv = (int)(i % CV);
    const int p = (int)(i / CV);
    const int ow = p % g.Wo;
    const int t2 = p / g.Wo;
    const int oh = t2 % g.Ho;
    const int n = t2 / g.Ho;
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    int cnt = 0;
    for (int r = 0; r < g.kh; ++r) {
      const int ih = oh * g.sh - g.ph + r;
      if (ih < 0 || ih >= g.H) continue;
      for (int s = 0; s < g.kw; ++s) {
        const int iw = ow * g.sw - g.pw + s;
        if (iw < 0 || iw >= g.W) continue;
        float v[V];
        ldv<T, V>(x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + cv * V, v);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += v[k];
        ++cnt;
      }
    }
    const float d = 1.f / (count_pad ? (float)(g.kh * g.kw) : (float)max(cnt, 1));
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] *= d;
    stv<T, V>(y + (int64_t)p * g.C + cv * V, acc);
  }
}

template <typename T, int V>
__global__ void avgpool_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, PoolGeom g, int count_pad) {
  const int CV = g.C / V;
  const int64_t total = (int64_t)g.N * g.H * g.W * CV;
  SG_GRID_STRIDE(i, total) {
    const int cv = (int)(i % CV);
    const int p = (int)(i / CV);
    const int iw = p % g.W;
    const int t2 = p / g.W;
    const int ih = t2 % g.H;
    const int n = t2 / g.H;
    const int oh0 = max(0, (ih + g.ph - g.kh + g.sh) / g.sh), oh1 = min(g.Ho - 1, (ih + g.ph) / g.sh);
    const int ow0 = max(0, (iw + g.pw - g.kw + g.sw) / g.sw), ow1 = min(g.Wo - 1, (iw + g.pw) / g.sw);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int r = ih + g.ph - oh * g.sh;
      if (r < 0 || r >= g.kh) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int s = iw + g.pw - ow * g.sw;
        if (s < 0 || s >= g.kw) continue;
        float d;
        if (count_pad) d = (float)(g.kh * g.kw);
        else {
          const int h0 = max(oh * g.sh - g.ph, 0), h1 = min(oh * g.sh - g.ph + g.kh, g.H);
          const int w0 = max(ow * g.sw - g.pw, 0), w1 = min(ow * g.sw - g.pw + g.kw, g.W);
          d = (float)max((h1 - h0) * (w1 - w0), 1);
        }
        float v[V];
        ldv<T, V>(dy + (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + cv * V, v);
        const float inv = 1.f / d;
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += v[k] * inv;
      }
    }
    stv<T, V>(dx + (int64_t)p * g.C + cv * V, acc);
  }
}

// global average pool [N][HW][C] -> [N][C]; one thread per (n, V channels)
template <typename T, int V>
__global__ void gap_fwd_k(const T* __restrict__ x, T* __restrict__ y, int N, int HW, int C) {
  const int64_t total = (int64_t)N * C / V;
  SG_GRID_STRIDE(i, total) {
    int64_t n = i / (C / V);
    int c0 = (int)(i % (C / V)) * V;
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    for (int p = 0; p < HW; ++p) {
      float v[V];
      ldv<T, V>(x + ((int64_t)n * HW + p) * C + c0, v);
#pragma unroll
      for (int k = 0; k < V; ++k) acc[k] += v[k];
    }
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] *= 1.f / HW;
    stv<T, V>(y + n * C + c0, acc);
  }
}
template <typename T, int V>
__global__ void gap_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int N, int HW, int C) {
  const int64_t total = (int64_t)N * HW * C / V;
  SG_GRID_STRIDE(i, total) {
    int64_t e = i * V;
    int c0 = (int)(e % C);
    int64_t n = e / ((int64_t)HW * C);
    float v[V];
    ldv<T, V>(dy + n * C + c0, v);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] *= 1.f / HW;
    stv<T, V>(dx + e, v);
  }
}

// LRN across channels (NHWC: the window is contiguous).
// norm = k + alpha/n * sum_{|c'-c|<=n/2} x^2 ; y = x * norm^-beta
template <typename T>
__global__ void lrn_fwd_k(const T* __restrict__ x, T* __restrict__ y, float* __restrict__ norm, int64_t R, int C,
                          int size, float alpha, float beta, float knorm) {
  const int64_t total = R * C;
  const int half = size / 2;
  SG_GRID_STRIDE(i, total) {
    int c = (int)(i % C);
    int64_t base = i - c;
    float s = 0.f;
    for (int d = -half; d <= half; ++d) {
      int cc = c + d;
      if (cc >= 0 && cc < C) {
        float v = to_f32(x[base + cc]);
        s += v * v;
      }
    }
    float nm = knorm + alpha / size * s;
    norm[i] = nm;
    y[i] = from_f32<T>(to_f32(x[i]) * __powf(nm, -beta));
  }
}
// dx = dy*norm^-b - 2*b*alpha/n * x * sum_{window} (dy*x*norm^(-b-1))
template <typename T>
__global__ void lrn_bwd_k(const T* __restrict__ x, const T* __restrict__ dy, const float* __restrict__ norm,
                          T* __restrict__ dx, int64_t R, int C, int size, float alpha, float beta) {
  const int64_t total = R * C;
  const int half = size / 2;
  SG_GRID_STRIDE(i, total) {
    int c = (int)(i % C);
    int64_t base = i - c;
    float s = 0.f;
    for (int d = -half; d <= half; ++d) {
      int cc = c + d;
      if (cc >= 0 && cc < C) {
        float nm = norm[base + cc];
        s += to_f32(dy[base + cc]) * to_f32(x[base + cc]) * __powf(nm, -beta - 1.f);
      }
    }
    float xv = to_f32(x[i]);
    dx[i] = from_f32<T>(to_f32(dy[i]) * __powf(norm[i], -beta) - 2.f * beta * alpha / size * xv * s);
  }
}

// ---- LRN, pixel-staged (C % 8 == 0) ----
// The per-element kernels above redo the whole channel window per output
// element from global memory with a 64-bit modulo, and the backward raises
// every window member's norm to a power again (5 powf per element):
// AlexNet b512's two LRNs took 38 % + 11 % of its step.  Here each workgroup
// stages ppb pixels' squared inputs (and, backward, dy*x*norm^(-beta-1))
// into zero-padded LDS rows, each thread owns 8 contiguous channels of one
// pixel (16-byte loads/stores), and window sums read LDS.  The forward
// writes no fp32 norm tensor: the backward recomputes it from x (k passed).
// x^y for x > 0 on the hardware log2 / exp2 (v_log_f32, v_exp_f32): HIP's
// __powf is the accurate OCML pow (~150 VALU with its special cases), which
// made the LRN kernels VALU-bound at 8 pows per thread (PMC: ~1400 VALU per wave)
__device__ __forceinline__ float fast_pow_pos(float x, float y) {
  return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}

// Window sums: each thread reads its 8 channels plus SZ-1 neighbours ONCE
// (8 + 2*half LDS words, compile-time SZ: fully unrolled) and slides.
template <int SZ>
__device__ __forceinline__ void window8(const float* row, int c0, float out[8]) {
  constexpr int H = SZ / 2;
  float w[8 + 2 * H];
#pragma unroll
  for (int i = 0; i < 8 + 2 * H; ++i) w[i] = row[c0 - H + i];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < SZ; ++i) s += w[i];
  out[0] = s;
#pragma unroll
  for (int e = 1; e < 8; ++e) {
    s += w[e + SZ - 1] - w[e - 1];
    out[e] = s;
  }
}

template <typename T, bool BWD, int SZ, bool RELU = false>
__global__ void __launch_bounds__(256) lrn_rows_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                  T* __restrict__ out, int64_t R, int C, float alpha, float beta,
                                                  float knorm) {
  extern __shared__ float lds[];
  constexpr int half = SZ / 2;
  const int tpp = C >> 3;             // threads per pixel
  const int ppb = blockDim.x / tpp;   // pixels per workgroup (host: blockDim.x == ppb * tpp)
  const int Wd = C + 2 * half;        // padded LDS row
  float* sq = lds;
  float* tt = lds + ppb * Wd;
  const int lp = threadIdx.x / tpp, c0 = (threadIdx.x - lp * tpp) * 8;
  for (int i = threadIdx.x; i < ppb * 2 * half; i += blockDim.x) {
    const int pp = i / (2 * half), j = i - pp * 2 * half;
    const int col = j < half ? j : C + j;
    sq[pp * Wd + col] = 0.f;
    if (BWD) tt[pp * Wd + col] = 0.f;
  }
  float* srow = sq + lp * Wd + half;
  float* trow = tt + lp * Wd + half;
  const float an = alpha / SZ;
  // persistent over pixel chunks: ~4 KB of work per chunk is far too little
  // to pay a workgroup dispatch each (73K workgroups for AlexNet's conv1 LRN)
  const int64_t nchunk = (R + ppb - 1) / ppb;
  for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
    const int64_t pix = ch * ppb + lp;
    const bool ok = pix < R;
    float xv[8], gv[8];
    if (ok) {
      ldv<T, 8>(x + pix * C + c0, xv);
      if (BWD) ldv<T, 8>(dy + pix * C + c0, gv);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { xv[e] = 0.f; gv[e] = 0.f; }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) srow[c0 + e] = xv[e] * xv[e];
    __syncthreads();
    float nm[8], pb[8];
    window8<SZ>(srow, c0, nm);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      nm[e] = knorm + an * nm[e];
      pb[e] = fast_pow_pos(nm[e], -beta);
    }
    if constexpr (!BWD) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = xv[e] * pb[e];
      if (ok) stv<T, 8>(out + pix * C + c0, o);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) trow[c0 + e] = gv[e] * xv[e] * pb[e] * __builtin_amdgcn_rcpf(nm[e]);
      __syncthreads();
      const float f = 2.f * beta * an;
      float sm[8], o[8];
      window8<SZ>(trow, c0, sm);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = gv[e] * pb[e] - f * xv[e] * sm[e];
        if (RELU && !(xv[e] > 0.f)) o[e] = 0.f;  // x is a ReLU output: its backward, folded
      }
      if (ok) stv<T, 8>(out + pix * C + c0, o);
    }
    __syncthreads();  // LDS rows are rewritten by the next chunk
  }
}

}  // namespace sg

using namespace sg;

#define DISPATCH_FT(dtype, ...) \
  if ((dtype) == kF32) {        \
    typedef float T;            \
    __VA_ARGS__;                \
  } else {                      \
    typedef bf16 T;             \
    __VA_ARGS__;                \
  }

extern "C" {

#define DISPATCH_V(Vv, ...)       \
  if ((Vv) == 8) {                \
    constexpr int VV = 8;         \
    __VA_ARGS__;                  \
  } else {                        \
    constexpr int VV = 1;         \
    __VA_ARGS__;                  \
  }

void sg_pool_fwd(const void* x, void* y, void* arg, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw,
                 int sh, int sw, int ph, int pw, int is_max, int count_pad, int dtype, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw};
  const int V = (C % 8 == 0) ? 8 : 1;
  const int64_t total = (int64_t)N * Ho * Wo * (C / V);
  if (is_max) {
    const int ych = (int)(((int64_t)Wo * (C / V) + 255) / 256);
    DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((maxpool_fwd_k<T, VV>), dim3(N * Ho, ych),
                                                        dim3(256), 0, s, (const T*)x, (T*)y, (uint8_t*)arg, g)));
  } else {
    DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((avgpool_fwd_k<T, VV>), dim3(sg_grid(total, 256, 16384)),
                                                        dim3(256), 0, s, (const T*)x, (T*)y, g, count_pad)));
  }
}
void sg_pool_bwd(const void* dy, const void* arg, void* dx, int N, int H, int W, int C, int Ho, int Wo, int kh,
                 int kw, int sh, int sw, int ph, int pw, int is_max, int count_pad, int dtype, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw};
  const int V = (C % 8 == 0) ? 8 : 1;
  const int64_t total = (int64_t)N * H * W * (C / V);
  static const int blk = getenv("SG_POOL_BLK") ? atoi(getenv("SG_POOL_BLK")) : 1;
  const int64_t tblk = (int64_t)N * (Ho + 1) * (Wo + 1) * (C / 8);
  if (blk && is_max && dtype == 1 && V == 8 && kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 &&
      H == 2 * Ho && W == 2 * Wo && tblk < (int64_t)UINT32_MAX) {
    hipLaunchKernelGGL(maxpool_bwd_332_blk_k, dim3(sg_grid(tblk, 256, 16384)), dim3(256), 0, s, (const bf16*)dy,
                       (const uint8_t*)arg, (bf16*)dx, H, W, C, Ho, Wo, (uint32_t)tblk, FastDiv(C / 8),
                       FastDiv(Wo + 1), FastDiv(Ho + 1));
  } else if (is_max && dtype == 1 && V == 8 && kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 &&
      total < (int64_t)UINT32_MAX && Ho == (H + 1) / 2 && Wo == (W + 1) / 2) {
    hipLaunchKernelGGL(maxpool_bwd_332_k, dim3(sg_grid(total, 256, 16384)), dim3(256), 0, s, (const bf16*)dy,
                       (const uint8_t*)arg, (bf16*)dx, H, W, C, Ho, Wo, (uint32_t)total, FastDiv(C / 8), FastDiv(W),
                       FastDiv(H));
  } else if (is_max) {
    const int ych = (int)(((int64_t)W * (C / V) + 255) / 256);
    DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((maxpool_bwd_k<T, VV>), dim3(N * H, ych),
                                                        dim3(256), 0, s, (const T*)dy, (const uint8_t*)arg, (T*)dx,
                                                        g)));
  } else {
    DISPATCH_FT(dtype, DISPATCH_V(V, hipLaunchKernelGGL((avgpool_bwd_k<T, VV>), dim3(sg_grid(total, 256, 16384)),
                                                        dim3(256), 0, s, (const T*)dy, (T*)dx, g, count_pad)));
  }
}
void sg_bn_relu_maxpool(const void* x, const void* scale, const void* shift, void* y, void* arg, int N, int H, int W,
                        int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw};
  static const int blk = getenv("SG_POOL_BLK") ? atoi(getenv("SG_POOL_BLK")) : 1;
  const int64_t tblk = (int64_t)N * (Ho / 2) * (Wo / 2) * (C / 8);
  if (blk && kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 && (Ho & 1) == 0 && (Wo & 1) == 0 &&
      (C & 7) == 0 && Ho == (H + 1) / 2 && Wo == (W + 1) / 2 && tblk < (int64_t)UINT32_MAX) {
    hipLaunchKernelGGL(bn_relu_maxpool_332_blk_k, dim3(sg_grid(tblk, 256, 16384)), dim3(256), 0, s, (const bf16*)x,
                       (const float*)scale, (const float*)shift, (bf16*)y, (uint8_t*)arg, H, W, C, Ho, Wo,
                       (uint32_t)tblk, FastDiv(C / 8), FastDiv(Wo / 2), FastDiv(Ho / 2));
    return;
  }
  const int ych = (int)(((int64_t)Wo * (C / 8) + 255) / 256);
  hipLaunchKernelGGL(bn_relu_maxpool_fwd_k, dim3(N * Ho, ych), dim3(256), 0, s, (const bf16*)x, (const float*)scale,
                     (const float*)shift, (bf16*)y, (uint8_t*)arg, g);
}
void sg_gap_fwd(const void* x, void* y, int N, int HW, int C, int dtype, hipStream_t s) {
  if (C % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((gap_fwd_k<T, 8>), dim3(sg_grid((int64_t)N * C / 8)), dim3(256), 0, s,
                                          (const T*)x, (T*)y, N, HW, C));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((gap_fwd_k<T, 1>), dim3(sg_grid((int64_t)N * C)), dim3(256), 0, s,
                                          (const T*)x, (T*)y, N, HW, C));
  }
}
void sg_gap_bwd(const void* dy, void* dx, int N, int HW, int C, int dtype, hipStream_t s) {
  if (C % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((gap_bwd_k<T, 8>), dim3(sg_grid((int64_t)N * HW * C / 8, 256, 8192)),
                                          dim3(256), 0, s, (const T*)dy, (T*)dx, N, HW, C));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((gap_bwd_k<T, 1>), dim3(sg_grid((int64_t)N * HW * C, 256, 8192)),
                                          dim3(256), 0, s, (const T*)dy, (T*)dx, N, HW, C));
  }
}
void sg_lrn_fwd(const void* x, void* y, void* norm, int64_t R, int C, int size, float alpha, float beta, float knorm,
                int dtype, hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(lrn_fwd_k<T>, dim3(sg_grid(R * C, 256, 16384)), dim3(256), 0, s,
                                        (const T*)x, (T*)y, (float*)norm, R, C, size, alpha, beta, knorm));
}
// pixel-staged LRN (C % 8 == 0, C <= 2048): bwd = 0 -> out = y; bwd = 1 -> out = dx (norm recomputed from x);
// bwd = 2 -> dx with the ReLU mask of x (x > 0) applied
void sg_lrn_rows(const void* x, const void* dy, void* out, int64_t R, int C, int size, float alpha, float beta,
                 float knorm, int bwd, int dtype, hipStream_t s) {
  const int tpp = C / 8;
  const int ppb = 256 / tpp;
  const int half = size / 2;
  const size_t lds = (size_t)(bwd ? 2 : 1) * ppb * (C + 2 * half) * sizeof(float);
  const int64_t nchunk = (R + ppb - 1) / ppb;
  const dim3 grid((unsigned)(nchunk < 4096 ? nchunk : 4096)), block(ppb * tpp);
#define LRN_GO(SZ)                                                                                             \
  if (bwd == 2) {                                                                                              \
    DISPATCH_FT(dtype, hipLaunchKernelGGL((lrn_rows_k<T, true, SZ, true>), grid, block, lds, s, (const T*)x,    \
                                          (const T*)dy, (T*)out, R, C, alpha, beta, knorm));                    \
  } else if (bwd) {                                                                                            \
    DISPATCH_FT(dtype, hipLaunchKernelGGL((lrn_rows_k<T, true, SZ>), grid, block, lds, s, (const T*)x,          \
                                          (const T*)dy, (T*)out, R, C, alpha, beta, knorm));                    \
  } else {                                                                                                     \
    DISPATCH_FT(dtype, hipLaunchKernelGGL((lrn_rows_k<T, false, SZ>), grid, block, lds, s, (const T*)x, nullptr, \
                                          (T*)out, R, C, alpha, beta, knorm));                                  \
  }
  switch (size) {  // (host-checked: odd, 1..9)
    case 1: LRN_GO(1); break;
    case 3: LRN_GO(3); break;
    case 5: LRN_GO(5); break;
    case 7: LRN_GO(7); break;
    default: LRN_GO(9); break;
  }
#undef LRN_GO
}
void sg_lrn_bwd(const void* x, const void* dy, const void* norm, void* dx, int64_t R, int C, int size, float alpha,
                float beta, int dtype, hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(lrn_bwd_k<T>, dim3(sg_grid(R * C, 256, 16384)), dim3(256), 0, s,
                                        (const T*)x, (const T*)dy, (const float*)norm, (T*)dx, R, C, size, alpha,
                                        beta));
}

}  // extern "C"

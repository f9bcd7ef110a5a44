// Channel reductions, BatchNorm2d (train/infer/backward, NHWC with fused
// ReLU and residual add), pooling (max/avg, padded, NHWC), global average
// pooling and across-channel LRN.
//
// Reference: bias-gradient reductions K3/K4 (include/mshadow/cuda/
// tensor_gpu-inl.cuh:96-168), Pooling/UnPooling plans (include/mshadow/
// tensor_expr_ext.h:787-850), channel pooling for LRN (:916-941, F8/F9 in
// src/worker/layer.cc:356-377).  BatchNorm is a north-star addition.
//
// Layout: activations are [R = N*H*W][C] with C contiguous (channels_last),
// which makes every per-channel statistic a coalesced column reduction.
#include "common.h"

namespace sg {

// ---------------------------------------------------------------------------
// Column reduction: out0[c] += sum_r f0(x[r][c]), out1[c] += sum_r x^2 (opt).
// Block = 256 threads laid out as (CT = channels/8 per block) x (256/CT) rows.
// Each thread accumulates 8 consecutive channels with one 16-B load per row.
// ---------------------------------------------------------------------------
template <typename T, int V>
__device__ __forceinline__ void ldv(const T* p, float* v) {
  if constexpr (V == 8) {
    if constexpr (sizeof(T) == 2) {
      bf16x8 t = *(const bf16x8*)p;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (float)t[i];
    } else {
      float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = to_f32(p[i]);
  }
}
template <typename T, int V>
__device__ __forceinline__ void stv(T* p, const float* v) {
  if constexpr (V == 8) {
    if constexpr (sizeof(T) == 2) {
      bf16x8 t;
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] = (bf16)v[i];
      *(bf16x8*)p = t;
    } else {
      *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i] = from_f32<T>(v[i]);
  }
}
// mode 0: sum(x), sum(x^2)  (BN stats / bias grad)
// mode 1: BN backward: sum(dyeff), sum(dyeff*xhat) where dyeff = dy masked
//         by (y > 0) if y != null; xhat = (x-mean)*invstd.
template <typename T, int MODE, int V>
__global__ void __launch_bounds__(256) colreduce_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                   const T* __restrict__ y, const float* __restrict__ mean,
                                                   const float* __restrict__ invstd, float* __restrict__ out0,
                                                   float* __restrict__ out1, int64_t R, int C, int rows_per_block) {
  __shared__ float red0[256 * V];
  const int CT = min(C, 64 * V) / V;  // threads across channels
  const int RT = 256 / CT;             // threads across rows
  const int tx = threadIdx.x % CT, ty = threadIdx.x / CT;
  const int c0 = blockIdx.y * (CT * V) + tx * V;
  const bool active = (ty < RT) && (c0 < C);
  float a0[V], a1[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { a0[i] = 0.f; a1[i] = 0.f; }
  float mu[V], is[V];
  if (MODE == 1 && active) {
#pragma unroll
    for (int i = 0; i < V; ++i) { mu[i] = mean[c0 + i]; is[i] = invstd[c0 + i]; }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(R, r0 + rows_per_block);
  if (active) {
    for (int64_t r = r0 + ty; r < r1; r += RT) {
      float v[V];
      if (MODE == 0) {
        ldv<T, V>(x + r * C + c0, v);
#pragma unroll
        for (int i = 0; i < V; ++i) { a0[i] += v[i]; a1[i] += v[i] * v[i]; }
      } else {
        float g[V];
        ldv<T, V>(dy + r * C + c0, g);
        if (y) {
          float yy[V];
          ldv<T, V>(y + r * C + c0, yy);
#pragma unroll
          for (int i = 0; i < V; ++i) g[i] = yy[i] > 0.f ? g[i] : 0.f;
        }
        ldv<T, V>(x + r * C + c0, v);
#pragma unroll
        for (int i = 0; i < V; ++i) { a0[i] += g[i]; a1[i] += g[i] * (v[i] - mu[i]) * is[i]; }
      }
    }
  }
  // reduce across ty through LDS, two passes (a0, a1)
  float* sm = red0;
  for (int pass = 0; pass < 2; ++pass) {
    float* acc = pass == 0 ? a0 : a1;
    float* out = pass == 0 ? out0 : out1;
    if (out == nullptr) continue;
    __syncthreads();
    if (ty < RT) {
#pragma unroll
      for (int i = 0; i < V; ++i) sm[threadIdx.x * V + i] = acc[i];
    }
    __syncthreads();
    if (ty == 0 && c0 < C) {
      for (int k = 1; k < RT; ++k) {
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] += sm[(k * CT + tx) * V + i];
      }
#pragma unroll
      for (int i = 0; i < V; ++i) atomicAdd(out + c0 + i, acc[i]);
    }
  }
}

// finalize BN statistics: mean/var from sums; running stats; scale/shift.
__global__ void bn_finalize_k(const float* __restrict__ sum, const float* __restrict__ sumsq,
                              const float* __restrict__ gamma, const float* __restrict__ beta,
                              float* __restrict__ run_mean, float* __restrict__ run_var, float* __restrict__ mean,
                              float* __restrict__ invstd, float* __restrict__ scale, float* __restrict__ shift, int C,
                              float count, float momentum, float eps) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mu = sum[c] / count;
  float var = fmaxf(sumsq[c] / count - mu * mu, 0.f);
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

// inference: scale/shift from running stats
__global__ void bn_infer_params_k(const float* __restrict__ gamma, const float* __restrict__ beta,
                                  const float* __restrict__ run_mean, const float* __restrict__ run_var,
                                  float* __restrict__ scale, float* __restrict__ shift, int C, float eps) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float is = rsqrtf(run_var[c] + eps);
  float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - run_mean[c] * g * is;
}

// y = act(x*scale[c] + shift[c] + res)
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_apply_k(const T* __restrict__ x, const float* __restrict__ scale,
                                                  const float* __restrict__ shift, const T* __restrict__ res,
                                                  T* __restrict__ y, int64_t R, int C, int relu) {
  const int64_t nv = R * C / V;
  SG_GRID_STRIDE(i, nv) {
    const int c0 = (int)((i * V) % C);
    float v[V];
    ldv<T, V>(x + i * V, v);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = v[k] * scale[c0 + k] + shift[c0 + k];
    if (res) {
      float rv[V];
      ldv<T, V>(res + i * V, rv);
#pragma unroll
      for (int k = 0; k < V; ++k) v[k] += rv[k];
    }
    if (relu) {
#pragma unroll
      for (int k = 0; k < V; ++k) v[k] = fmaxf(v[k], 0.f);
    }
    stv<T, V>(y + i * V, v);
  }
}

// dx = invstd*gamma*(dyeff - sdy/count - xhat*sdyx/count); dres = dyeff (opt)
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_bwd_apply_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                      const T* __restrict__ y, const float* __restrict__ mean,
                                                      const float* __restrict__ invstd,
                                                      const float* __restrict__ gamma, const float* __restrict__ sdy,
                                                      const float* __restrict__ sdyx, T* __restrict__ dx,
                                                      T* __restrict__ dres, int64_t R, int C, float inv_count) {
  const int64_t nv = R * C / V;
  SG_GRID_STRIDE(i, nv) {
    const int c0 = (int)((i * V) % C);
    float v[V], g[V];
    ldv<T, V>(x + i * V, v);
    ldv<T, V>(dy + i * V, g);
    if (y) {
      float yy[V];
      ldv<T, V>(y + i * V, yy);
#pragma unroll
      for (int k = 0; k < V; ++k) g[k] = yy[k] > 0.f ? g[k] : 0.f;
    }
    if (dres) stv<T, V>(dres + i * V, g);
    float o[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int c = c0 + k;
      float is = invstd[c];
      float xh = (v[k] - mean[c]) * is;
      float gm = gamma ? gamma[c] : 1.f;
      o[k] = gm * is * (g[k] - sdy[c] * inv_count - xh * sdyx[c] * inv_count);
    }
    stv<T, V>(dx + i * V, o);
  }
}

// ---------------------------------------------------------------------------
// Pooling, NHWC.  Max pooling stores the argmax window offset (uint8) so the
// backward pass is an exact gather (no atomics, no tie double counting; the
// reference re-compared values, include/mshadow/tensor_base.h:265-267).
// ---------------------------------------------------------------------------
struct PoolGeom {
  int N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw;
};

template <typename T>
__global__ void maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ arg, PoolGeom g) {
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * g.C;
  SG_GRID_STRIDE(i, total) {
    int c = (int)(i % g.C);
    int64_t p = i / g.C;
    int ow = (int)(p % g.Wo);
    p /= g.Wo;
    int oh = (int)(p % g.Ho);
    int n = (int)(p / g.Ho);
    float m = -INFINITY;
    int best = 0;
    for (int r = 0; r < g.kh; ++r) {
      int ih = oh * g.sh - g.ph + r;
      if (ih < 0 || ih >= g.H) continue;
      for (int s = 0; s < g.kw; ++s) {
        int iw = ow * g.sw - g.pw + s;
        if (iw < 0 || iw >= g.W) continue;
        float v = to_f32(x[(((int64_t)n * g.H + ih) * g.W + iw) * g.C + c]);
        if (v > m) { m = v; best = r * g.kw + s; }
      }
    }
    y[i] = from_f32<T>(m);
    if (arg) arg[i] = (uint8_t)best;
  }
}

template <typename T>
__global__ void maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ arg, T* __restrict__ dx,
                              PoolGeom g) {
  const int64_t total = (int64_t)g.N * g.H * g.W * g.C;
  SG_GRID_STRIDE(i, total) {
    int c = (int)(i % g.C);
    int64_t p = i / g.C;
    int iw = (int)(p % g.W);
    p /= g.W;
    int ih = (int)(p % g.H);
    int n = (int)(p / g.H);
    // output windows that contain (ih, iw)
    int oh0 = max(0, (ih + g.ph - g.kh + g.sh) / g.sh), oh1 = min(g.Ho - 1, (ih + g.ph) / g.sh);
    int ow0 = max(0, (iw + g.pw - g.kw + g.sw) / g.sw), ow1 = min(g.Wo - 1, (iw + g.pw) / g.sw);
    float acc = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      int r = ih + g.ph - oh * g.sh;
      if (r < 0 || r >= g.kh) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        int s = iw + g.pw - ow * g.sw;
        if (s < 0 || s >= g.kw) continue;
        int64_t o = (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + c;
        if (arg[o] == r * g.kw + s) acc += to_f32(dy[o]);
      }
    }
    dx[i] = from_f32<T>(acc);
  }
}

template <typename T>
__global__ void avgpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, PoolGeom g, int count_pad) {
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * g.C;
  SG_GRID_STRIDE(i, total) {
    int c = (int)(i % g.C);
    int64_t p = i / g.C;
    int ow = (int)(p % g.Wo);
    p /= g.Wo;
    int oh = (int)(p % g.Ho);
    int n = (int)(p / g.Ho);
    float acc = 0.f;
    int cnt = 0;
    for (int r = 0; r < g.kh; ++r) {
      int ih = oh * g.sh - g.ph + r;
      if (ih < 0 || ih >= g.H) continue;
      for (int s = 0; s < g.kw; ++s) {
        int iw = ow * g.sw - g.pw + s;
        if (iw < 0 || iw >= g.W) continue;
        acc += to_f32(x[(((int64_t)n * g.H + ih) * g.W + iw) * g.C + c]);
        ++cnt;
      }
    }
    float d = count_pad ? (float)(g.kh * g.kw) : (float)max(cnt, 1);
    y[i] = from_f32<T>(acc / d);
  }
}

template <typename T>
__global__ void avgpool_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, PoolGeom g, int count_pad) {
  const int64_t total = (int64_t)g.N * g.H * g.W * g.C;
  SG_GRID_STRIDE(i, total) {
    int c = (int)(i % g.C);
    int64_t p = i / g.C;
    int iw = (int)(p % g.W);
    p /= g.W;
    int ih = (int)(p % g.H);
    int n = (int)(p / g.H);
    int oh0 = max(0, (ih + g.ph - g.kh + g.sh) / g.sh), oh1 = min(g.Ho - 1, (ih + g.ph) / g.sh);
    int ow0 = max(0, (iw + g.pw - g.kw + g.sw) / g.sw), ow1 = min(g.Wo - 1, (iw + g.pw) / g.sw);
    float acc = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      int r = ih + g.ph - oh * g.sh;
      if (r < 0 || r >= g.kh) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        int s = iw + g.pw - ow * g.sw;
        if (s < 0 || s >= g.kw) continue;
        float d;
        if (count_pad) d = (float)(g.kh * g.kw);
        else {
          int h0 = max(oh * g.sh - g.ph, 0), h1 = min(oh * g.sh - g.ph + g.kh, g.H);
          int w0 = max(ow * g.sw - g.pw, 0), w1 = min(ow * g.sw - g.pw + g.kw, g.W);
          d = (float)max((h1 - h0) * (w1 - w0), 1);
        }
        acc += to_f32(dy[(((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + c]) / d;
      }
    }
    dx[i] = from_f32<T>(acc);
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

static inline void colreduce_grid(int64_t R, int C, dim3& grid, int& rpb) {
  const int vw = (C % 8 == 0) ? 8 : 1;
  const int ctile = C < 64 * vw ? C : 64 * vw;
  const int cblocks = (C + ctile - 1) / ctile;
  // aim for ~2048 blocks total, at least 64 rows each
  int64_t rb = 2048 / cblocks;
  if (rb < 1) rb = 1;
  rpb = (int)((R + rb - 1) / rb);
  if (rpb < 64) rpb = 64;
  int64_t nb = (R + rpb - 1) / rpb;
  grid = dim3((unsigned)nb, (unsigned)cblocks);
}

extern "C" {

// out0/out1 must be zeroed by the caller (fp32 [C]); C % 8 == 0.
void sg_colsum(const void* x, void* out0, void* out1, int64_t R, int C, int dtype, hipStream_t s) {
  dim3 grid;
  int rpb;
  colreduce_grid(R, C, grid, rpb);
  if (C % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((colreduce_k<T, 0, 8>), grid, dim3(256), 0, s, (const T*)x, nullptr,
                                          nullptr, nullptr, nullptr, (float*)out0, (float*)out1, R, C, rpb));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((colreduce_k<T, 0, 1>), grid, dim3(256), 0, s, (const T*)x, nullptr,
                                          nullptr, nullptr, nullptr, (float*)out0, (float*)out1, R, C, rpb));
  }
}
void sg_bn_bwd_reduce(const void* x, const void* dy, const void* y, const void* mean, const void* invstd, void* sdy,
                      void* sdyx, int64_t R, int C, int dtype, hipStream_t s) {
  dim3 grid;
  int rpb;
  colreduce_grid(R, C, grid, rpb);
  if (C % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((colreduce_k<T, 1, 8>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy,
                                          (const T*)y, (const float*)mean, (const float*)invstd, (float*)sdy,
                                          (float*)sdyx, R, C, rpb));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((colreduce_k<T, 1, 1>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy,
                                          (const T*)y, (const float*)mean, (const float*)invstd, (float*)sdy,
                                          (float*)sdyx, R, C, rpb));
  }
}
void sg_bn_finalize(const void* sum, const void* sumsq, const void* gamma, const void* beta, void* run_mean,
                    void* run_var, void* mean, void* invstd, void* scale, void* shift, int C, float count,
                    float momentum, float eps, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_k, dim3((C + 255) / 256), dim3(256), 0, s, (const float*)sum, (const float*)sumsq,
                     (const float*)gamma, (const float*)beta, (float*)run_mean, (float*)run_var, (float*)mean,
                     (float*)invstd, (float*)scale, (float*)shift, C, count, momentum, eps);
}
void sg_bn_infer_params(const void* gamma, const void* beta, const void* run_mean, const void* run_var, void* scale,
                        void* shift, int C, float eps, hipStream_t s) {
  hipLaunchKernelGGL(bn_infer_params_k, dim3((C + 255) / 256), dim3(256), 0, s, (const float*)gamma,
                     (const float*)beta, (const float*)run_mean, (const float*)run_var, (float*)scale,
                     (float*)shift, C, eps);
}
void sg_bn_apply(const void* x, const void* scale, const void* shift, const void* res, void* y, int64_t R, int C,
                 int relu, int dtype, hipStream_t s) {
  if (C % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((bn_apply_k<T, 8>), dim3(sg_grid(R * C / 8, 256, 8192)), dim3(256), 0, s,
                                          (const T*)x, (const float*)scale, (const float*)shift, (const T*)res,
                                          (T*)y, R, C, relu));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((bn_apply_k<T, 1>), dim3(sg_grid(R * C, 256, 8192)), dim3(256), 0, s,
                                          (const T*)x, (const float*)scale, (const float*)shift, (const T*)res,
                                          (T*)y, R, C, relu));
  }
}
void sg_bn_bwd_apply(const void* x, const void* dy, const void* y, const void* mean, const void* invstd,
                     const void* gamma, const void* sdy, const void* sdyx, void* dx, void* dres, int64_t R, int C,
                     int dtype, hipStream_t s) {
  if (C % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((bn_bwd_apply_k<T, 8>), dim3(sg_grid(R * C / 8, 256, 8192)), dim3(256), 0,
                                          s, (const T*)x, (const T*)dy, (const T*)y, (const float*)mean,
                                          (const float*)invstd, (const float*)gamma, (const float*)sdy,
                                          (const float*)sdyx, (T*)dx, (T*)dres, R, C, 1.f / (float)R));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL((bn_bwd_apply_k<T, 1>), dim3(sg_grid(R * C, 256, 8192)), dim3(256), 0, s,
                                          (const T*)x, (const T*)dy, (const T*)y, (const float*)mean,
                                          (const float*)invstd, (const float*)gamma, (const float*)sdy,
                                          (const float*)sdyx, (T*)dx, (T*)dres, R, C, 1.f / (float)R));
  }
}

void sg_pool_fwd(const void* x, void* y, void* arg, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw,
                 int sh, int sw, int ph, int pw, int is_max, int count_pad, int dtype, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw};
  int64_t total = (int64_t)N * Ho * Wo * C;
  if (is_max) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL(maxpool_fwd_k<T>, dim3(sg_grid(total, 256, 16384)), dim3(256), 0, s,
                                          (const T*)x, (T*)y, (uint8_t*)arg, g));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL(avgpool_fwd_k<T>, dim3(sg_grid(total, 256, 16384)), dim3(256), 0, s,
                                          (const T*)x, (T*)y, g, count_pad));
  }
}
void sg_pool_bwd(const void* dy, const void* arg, void* dx, int N, int H, int W, int C, int Ho, int Wo, int kh,
                 int kw, int sh, int sw, int ph, int pw, int is_max, int count_pad, int dtype, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw};
  int64_t total = (int64_t)N * H * W * C;
  if (is_max) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL(maxpool_bwd_k<T>, dim3(sg_grid(total, 256, 16384)), dim3(256), 0, s,
                                          (const T*)dy, (const uint8_t*)arg, (T*)dx, g));
  } else {
    DISPATCH_FT(dtype, hipLaunchKernelGGL(avgpool_bwd_k<T>, dim3(sg_grid(total, 256, 16384)), dim3(256), 0, s,
                                          (const T*)dy, (T*)dx, g, count_pad));
  }
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
void sg_lrn_bwd(const void* x, const void* dy, const void* norm, void* dx, int64_t R, int C, int size, float alpha,
                float beta, int dtype, hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(lrn_bwd_k<T>, dim3(sg_grid(R * C, 256, 16384)), dim3(256), 0, s,
                                        (const T*)x, (const T*)dy, (const float*)norm, (T*)dx, R, C, size, alpha,
                                        beta));
}

}  // extern "C"

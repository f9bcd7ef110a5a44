// Elementwise kernels (activations, residual add, casts, dropout, axpby).
//
// Replaces the reference's generic mshadow MapPlan kernel (K1/K2,
// include/mshadow/cuda/tensor_gpu-inl.cuh:56-92) and the cxxnet_op functors
// (include/mshadow/cxxnet_op.h:14-112) with per-op wave64 kernels that move
// 16 bytes per lane per access (8 bf16 or 4 fp32) in a grid-stride loop.
#include <stdexcept>

#include "common.h"

namespace sg {

enum UnaryOp : int {
  U_RELU = 0, U_SIGMOID = 1, U_TANH = 2, U_STANH = 3, U_GELU = 4,
  U_IDENTITY = 5, U_SOFTPLUS = 6, U_SQUARE = 7, U_ABS = 8, U_EXP = 9,
  U_LEAKY = 10, U_ELU = 11, U_SELU = 12, U_GELU_TANH = 13, U_SQRT = 14,
  U_NEG = 15, U_RECIP = 16, U_LOG = 17, U_SIGN = 18,
  // ONNX / SINGA glue math (autograd erf, trig, rounding, softsign, scalar ops)
  U_ERF = 19, U_COS = 20, U_SIN = 21, U_TAN = 22, U_COSH = 23, U_SINH = 24, U_ACOS = 25, U_ASIN = 26,
  U_ATAN = 27, U_ACOSH = 28, U_ASINH = 29, U_ATANH = 30, U_CEIL = 31, U_FLOOR = 32, U_ROUND = 33,
  U_SOFTSIGN = 34, U_SCALE = 35, U_ADDS = 36, U_RSQRT = 37, U_POWS = 38
};

__device__ __forceinline__ float unary_f(int op, float x, float a) {
  switch (op) {
    case U_RELU: return x > 0.f ? x : 0.f;
    case U_SIGMOID: return 1.f / (1.f + __expf(-x));
    case U_TANH: return tanhf(x);
    case U_STANH: return 1.7159047f * tanhf(0.66666667f * x);  // LeCun scaled tanh
    case U_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118f));
    case U_GELU_TANH: {
      float u = 0.7978845608f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case U_IDENTITY: return x;
    case U_SOFTPLUS: return x > 20.f ? x : log1pf(__expf(x));
    case U_SQUARE: return x * x;
    case U_ABS: return fabsf(x);
    case U_EXP: return __expf(x);
    case U_LEAKY: return x > 0.f ? x : a * x;
    case U_ELU: return x > 0.f ? x : a * (__expf(x) - 1.f);
    case U_SELU: {
      const float l = 1.0507009873554805f, al = 1.6732632423543772f;
      return x > 0.f ? l * x : l * al * (__expf(x) - 1.f);
    }
    case U_SQRT: return sqrtf(x);
    case U_NEG: return -x;
    case U_RECIP: return 1.f / x;
    case U_LOG: return __logf(x);
    case U_SIGN: return (float)((x > 0.f) - (x < 0.f));
    case U_ERF: return erff(x);
    case U_COS: return cosf(x);
    case U_SIN: return sinf(x);
    case U_TAN: return tanf(x);
    case U_COSH: return coshf(x);
    case U_SINH: return sinhf(x);
    case U_ACOS: return acosf(x);
    case U_ASIN: return asinf(x);
    case U_ATAN: return atanf(x);
    case U_ACOSH: return acoshf(x);
    case U_ASINH: return asinhf(x);
    case U_ATANH: return atanhf(x);
    case U_CEIL: return ceilf(x);
    case U_FLOOR: return floorf(x);
    case U_ROUND: return rintf(x);  // half to even (ONNX Round)
    case U_SOFTSIGN: return x / (1.f + fabsf(x));
    case U_SCALE: return a * x;
    case U_ADDS: return x + a;
    case U_RSQRT: return rsqrtf(x);
    case U_POWS: return powf(x, a);
  }
  return x;
}

// Gradient given input x, output y, upstream dy.
__device__ __forceinline__ float unary_b(int op, float x, float y, float dy, float a) {
  switch (op) {
    case U_RELU: return x > 0.f ? dy : 0.f;
    case U_SIGMOID: return dy * y * (1.f - y);
    case U_TANH: return dy * (1.f - y * y);
    case U_STANH: return dy * (0.66666667f * 1.7159047f - 0.66666667f / 1.7159047f * y * y);
    case U_GELU: {
      const float c = 0.3989422804f;  // 1/sqrt(2*pi)
      float cdf = 0.5f * (1.f + erff(x * 0.70710678118f));
      return dy * (cdf + x * c * __expf(-0.5f * x * x));
    }
    case U_GELU_TANH: {
      float x3 = x * x * x;
      float u = 0.7978845608f * (x + 0.044715f * x3);
      float t = tanhf(u);
      float du = 0.7978845608f * (1.f + 3.f * 0.044715f * x * x);
      return dy * (0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du);
    }
    case U_IDENTITY: return dy;
    case U_SOFTPLUS: return dy / (1.f + __expf(-x));
    case U_SQUARE: return dy * 2.f * x;
    case U_ABS: return dy * (float)((x > 0.f) - (x < 0.f));
    case U_EXP: return dy * y;
    case U_LEAKY: return x > 0.f ? dy : a * dy;
    case U_ELU: return x > 0.f ? dy : dy * (y + a);
    case U_SELU: {
      const float l = 1.0507009873554805f, al = 1.6732632423543772f;
      return x > 0.f ? l * dy : dy * (y + l * al);
    }
    case U_SQRT: return dy * 0.5f / y;
    case U_NEG: return -dy;
    case U_RECIP: return -dy * y * y;
    case U_LOG: return dy / x;
    case U_SIGN: return 0.f;
    case U_ERF: return dy * 1.1283791671f * __expf(-x * x);
    case U_COS: return -dy * sinf(x);
    case U_SIN: return dy * cosf(x);
    case U_TAN: return dy * (1.f + y * y);
    case U_COSH: return dy * sinhf(x);
    case U_SINH: return dy * coshf(x);
    case U_ACOS: return -dy * rsqrtf(1.f - x * x);
    case U_ASIN: return dy * rsqrtf(1.f - x * x);
    case U_ATAN: return dy / (1.f + x * x);
    case U_ACOSH: return dy * rsqrtf(x * x - 1.f);
    case U_ASINH: return dy * rsqrtf(x * x + 1.f);
    case U_ATANH: return dy / (1.f - x * x);
    case U_CEIL: case U_FLOOR: case U_ROUND: return 0.f;
    case U_SOFTSIGN: {
      const float d = 1.f + fabsf(x);
      return dy / (d * d);
    }
    case U_SCALE: return a * dy;
    case U_ADDS: return dy;
    case U_RSQRT: return -0.5f * dy * y * y * y;
    case U_POWS: return dy * a * powf(x, a - 1.f);
  }
  return dy;
}

template <typename T> struct Vec;
template <> struct Vec<float> { static constexpr int N = 4; typedef float4 V; };
template <> struct Vec<bf16> { static constexpr int N = 8; typedef uint4 V; };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* o) {
  if constexpr (sizeof(T) == 4) {
    float4 v = *(const float4*)p;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    bf16x8 v = *(const bf16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
  }
}
template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float* o) {
  if constexpr (sizeof(T) == 4) {
    *(float4*)p = make_float4(o[0], o[1], o[2], o[3]);
  } else {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (bf16)o[i];
    *(bf16x8*)p = v;
  }
}

template <typename T>
__device__ __forceinline__ void load_vec8(const T* p, float* o) {
  if constexpr (sizeof(T) == 4) {
    load_vec<float>(p, o);
    load_vec<float>(p + 4, o + 4);
  } else {
    load_vec<bf16>(p, o);
  }
}
template <typename T>
__device__ __forceinline__ void store_vec8(T* p, const float* o) {
  if constexpr (sizeof(T) == 4) {
    store_vec<float>(p, o);
    store_vec<float>(p + 4, o + 4);
  } else {
    store_vec<bf16>(p, o);
  }
}

// OP >= 0: the op as a compile-time constant (the hot activations: the
// per-element switch folds away -- as a runtime switch over all 38 ops the
// exact-erf GELU ran at 0.6x a device copy's bandwidth); OP < 0: runtime op
template <typename T, int OP = -1>
__global__ void unary_fwd_k(int op_rt, const T* __restrict__ x, T* __restrict__ y, int64_t n, float a) {
  constexpr int V = Vec<T>::N;
  const int op = OP >= 0 ? OP : op_rt;
  const int64_t nv = n / V;
  SG_GRID_STRIDE(i, nv) {
    float v[V];
    load_vec(x + i * V, v);
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = unary_f(op, v[j], a);
    store_vec(y + i * V, v);
  }
  // tail
  int64_t t = nv * V + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) y[t] = from_f32<T>(unary_f(op, to_f32(x[t]), a));
}

template <typename T, int OP = -1>
__global__ void unary_bwd_k(int op_rt, const T* __restrict__ x, const T* __restrict__ y,
                            const T* __restrict__ dy, T* __restrict__ dx, int64_t n, float a) {
  constexpr int V = Vec<T>::N;
  const int op = OP >= 0 ? OP : op_rt;
  const int64_t nv = n / V;
  SG_GRID_STRIDE(i, nv) {
    float xv[V], yv[V], gv[V];
    if (x) load_vec(x + i * V, xv); else { for (int j = 0; j < V; ++j) xv[j] = 0.f; }
    if (y) load_vec(y + i * V, yv); else { for (int j = 0; j < V; ++j) yv[j] = 0.f; }
    load_vec(dy + i * V, gv);
#pragma unroll
    for (int j = 0; j < V; ++j) gv[j] = unary_b(op, xv[j], yv[j], gv[j], a);
    store_vec(dx + i * V, gv);
  }
  int64_t t = nv * V + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) {
    float xv = x ? to_f32(x[t]) : 0.f, yv = y ? to_f32(y[t]) : 0.f;
    dx[t] = from_f32<T>(unary_b(op, xv, yv, to_f32(dy[t]), a));
  }
}

// y = relu?(alpha*a + beta*b)   (residual add, fused ReLU)
template <typename T>
__global__ void add_act_k(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y,
                          int64_t n, float alpha, float beta, int relu) {
  constexpr int V = Vec<T>::N;
  const int64_t nv = n / V;
  SG_GRID_STRIDE(i, nv) {
    float av[V], bv[V];
    load_vec(a + i * V, av);
    load_vec(b + i * V, bv);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float r = alpha * av[j] + beta * bv[j];
      av[j] = relu ? fmaxf(r, 0.f) : r;
    }
    store_vec(y + i * V, av);
  }
  int64_t t = nv * V + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) {
    float r = alpha * to_f32(a[t]) + beta * to_f32(b[t]);
    y[t] = from_f32<T>(relu ? fmaxf(r, 0.f) : r);
  }
}

// dx = (y > 0) ? dy : 0  where y is the (post-ReLU) output; optional second
// output dres = dx (the residual branch gets the same gradient).
template <typename T>
__global__ void relu_bwd_from_y_k(const T* __restrict__ y, const T* __restrict__ dy, T* __restrict__ dx,
                                  int64_t n) {
  constexpr int V = Vec<T>::N;
  const int64_t nv = n / V;
  SG_GRID_STRIDE(i, nv) {
    float yv[V], gv[V];
    load_vec(y + i * V, yv);
    load_vec(dy + i * V, gv);
#pragma unroll
    for (int j = 0; j < V; ++j) gv[j] = yv[j] > 0.f ? gv[j] : 0.f;
    store_vec(dx + i * V, gv);
  }
  int64_t t = nv * V + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) dx[t] = to_f32(y[t]) > 0.f ? dy[t] : from_f32<T>(0.f);
}

// out = g * bit(mask): the masked gradient of a fused BN(+residual)+ReLU
// output, from its 1-bit ReLU mask (byte i holds elements 8i..8i+7, bit r =
// element 8i+r); n % 8 == 0 (host-checked), 16-byte vectors
__global__ void mask_bits_apply_k(const uint4* __restrict__ g, const uint8_t* __restrict__ mask, uint4* __restrict__ out,
                                  int64_t nv) {
  SG_GRID_STRIDE(i, nv) {
    const unsigned m = mask[i];
    const uint4 v = g[i];
    unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned lo = (m >> (2 * j)) & 1u ? 0x0000ffffu : 0u, hi = (m >> (2 * j + 1)) & 1u ? 0xffff0000u : 0u;
      w[j] &= lo | hi;
    }
    out[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <typename TI, typename TO>
__global__ void cast_k(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  const int64_t nv = n / 4;
  SG_GRID_STRIDE(i, nv) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = to_f32(x[i * 4 + j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) y[i * 4 + j] = from_f32<TO>(v[j]);
  }
  int64_t t = nv * 4 + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) y[t] = from_f32<TO>(to_f32(x[t]));
}

// Dropout: mask byte (1 = keep) and y = x * mask / pkeep.  Inverted dropout,
// identity at inference is handled on the host (fixes reference quirk:
// dropout applied at test time, src/worker/layer.cc:142-152).
template <typename T>
__global__ void dropout_fwd_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ mask,
                              int64_t n, float pkeep, uint64_t seed, uint64_t offset,
                              const int64_t* __restrict__ epoch) {
  const float scale = 1.f / pkeep;
  // graph replays: the host-side (seed, offset) are frozen in the captured
  // launch, so the Philox key also mixes a device-resident step counter that
  // the captured step advances -> a fresh mask on every replay
  if (epoch) seed += (uint64_t)(*epoch) * 0x9E3779B97F4A7C15ull;
  const int64_t nq = (n + 3) / 4;
  SG_GRID_STRIDE(i, nq) {
    uint4 r = Philox::gen(seed, offset + i, 0);
    uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t e = i * 4 + j;
      if (e < n) {
        bool keep = Philox::u01(rr[j]) <= pkeep;
        mask[e] = keep;
        y[e] = from_f32<T>(keep ? to_f32(x[e]) * scale : 0.f);
      }
    }
  }
}
template <typename T>
__global__ void dropout_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ mask, T* __restrict__ dx,
                              int64_t n, float pkeep) {
  const float scale = 1.f / pkeep;
  SG_GRID_STRIDE(i, n) { dx[i] = from_f32<T>(mask[i] ? to_f32(dy[i]) * scale : 0.f); }
}

// 8 elements per thread (n % 8 == 0): 16-byte data accesses and one 8-byte
// mask store instead of scalar bytes.  Element e still takes word e % 4 of
// Philox quad e / 4, so the masks are bit-identical to dropout_fwd_k's.
template <typename T>
__global__ void dropout_fwd8_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ mask,
                               int64_t n, float pkeep, uint64_t seed, uint64_t offset,
                               const int64_t* __restrict__ epoch) {
  const float scale = 1.f / pkeep;
  if (epoch) seed += (uint64_t)(*epoch) * 0x9E3779B97F4A7C15ull;
  const int64_t n8 = n / 8;
  SG_GRID_STRIDE(i, n8) {
    const uint4 r0 = Philox::gen(seed, offset + 2 * i, 0), r1 = Philox::gen(seed, offset + 2 * i + 1, 0);
    const uint32_t rr[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    float v[8];
    load_vec8(x + i * 8, v);
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool keep = Philox::u01(rr[j]) <= pkeep;
      m |= (uint64_t)keep << (8 * j);
      v[j] = keep ? v[j] * scale : 0.f;
    }
    store_vec8(y + i * 8, v);
    *(uint64_t*)(mask + i * 8) = m;
  }
}
template <typename T>
__global__ void dropout_bwd8_k(const T* __restrict__ dy, const uint8_t* __restrict__ mask, T* __restrict__ dx,
                               int64_t n, float pkeep) {
  const float scale = 1.f / pkeep;
  const int64_t n8 = n / 8;
  SG_GRID_STRIDE(i, n8) {
    float v[8];
    load_vec8(dy + i * 8, v);
    const uint64_t m = *(const uint64_t*)(mask + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ((m >> (8 * j)) & 0xff) ? v[j] * scale : 0.f;
    store_vec8(dx + i * 8, v);
  }
}

// uniform / gaussian fill (Param init, reference C8 Random<cpu/gpu>)
template <typename T>
__global__ void rand_fill_k(T* __restrict__ y, int64_t n, int dist, float a, float b, uint64_t seed,
                            uint64_t offset) {
  const int64_t nq = (n + 3) / 4;
  SG_GRID_STRIDE(i, nq) {
    uint4 r = Philox::gen(seed, offset + i, 1);
    float u[4] = {Philox::u01(r.x), Philox::u01(r.y), Philox::u01(r.z), Philox::u01(r.w)};
    float o[4];
    if (dist == 0) {  // uniform [a, b)
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = a + (b - a) * (1.f - u[j]);
    } else {  // gaussian mean a, std b (Box-Muller)
      float r0 = sqrtf(-2.f * __logf(u[0])), r1 = sqrtf(-2.f * __logf(u[2]));
      float t0 = 6.283185307f * u[1], t1 = 6.283185307f * u[3];
      o[0] = a + b * r0 * __cosf(t0);
      o[1] = a + b * r0 * __sinf(t0);
      o[2] = a + b * r1 * __cosf(t1);
      o[3] = a + b * r1 * __sinf(t1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t e = i * 4 + j;
      if (e < n) y[e] = from_f32<T>(o[j]);
    }
  }
}

// NCHW fp32 image batch -> NHWC bf16 with channel padding (stem input prep).
template <typename TI>
__global__ void nchw_to_nhwc_pad_k(const TI* __restrict__ x, bf16* __restrict__ y, int N, int C, int H,
                                   int W, int Cp) {
  const int64_t total = (int64_t)N * H * W;
  SG_GRID_STRIDE(p, total) {
    int64_t n = p / (H * W);
    int64_t hw = p - n * H * W;
    bf16x8 v;
    for (int c0 = 0; c0 < Cp; c0 += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int c = c0 + j;
        v[j] = (bf16)(c < C ? to_f32(x[(n * C + c) * H * W + hw]) : 0.f);
      }
      *(bf16x8*)(y + p * Cp + c0) = v;
    }
  }
}

// Stem input in "paired-tap" layout for a stride-2 conv over C <= 3
// channels: y[n][h][w'][0..7] = {x(h, w'-1, 0..2), x(h, w', 0..2), 0, 0} for
// w' in [0, W] (zero outside the image).  One 16-byte vector then carries two
// horizontally adjacent taps, so the 7x7/2 stem is a 7x4 conv with horizontal
// dilation 2 over 8 channels: 224 reduction elements per output instead of
// 392 with the channel-padded layout (ResNetStem, models/resnet.py).
// (32-bit indices with constant-divisor splits: the int64 divisions of a
// v1 made this pass VALU-bound at ~3 TB/s)
__global__ void nchw_to_pairs_k(const float* __restrict__ x, bf16* __restrict__ y, int N, int C, int H, int W,
                                uint32_t total, FastDiv dW1, FastDiv dH) {
  const int W1 = W + 1;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < total; p += gridDim.x * blockDim.x) {
    const uint32_t nh = dW1.div(p);
    const int w = (int)(p - nh * (uint32_t)W1);
    const uint32_t n = dH.div(nh);
    const int h = (int)(nh - n * (uint32_t)H);
    const float* xb = x + ((int64_t)n * C * H + h) * (int64_t)W;  // channel c at xb + c*H*W
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      v[j] = (bf16)((j < C && w >= 1) ? xb[(int64_t)j * H * W + w - 1] : 0.f);
      v[3 + j] = (bf16)((j < C && w < W) ? xb[(int64_t)j * H * W + w] : 0.f);
    }
    v[6] = (bf16)0.f;
    v[7] = (bf16)0.f;
    *(bf16x8*)(y + (int64_t)p * 8) = v;
  }
}

// Vector form for W % 4 == 0 and C == 3 (every ImageNet stem): a thread
// owns four consecutive output columns w' = 4q..4q+3, reads one 16-byte
// float4 per channel plus the column to its left, and writes 64 contiguous
// bytes.  The scalar form above re-reads every input twice with 4-byte loads;
// measured on the b1024 stem both run at ~3.2 TB/s (451 vs 454 us,
// profiles/r5/r50_b1024_kernel_stats_r6d.txt), so the pass is bound by the
// memory system, not by its instruction count.
__global__ void nchw_to_pairs4_k(const float* __restrict__ x, bf16* __restrict__ y, int H, int W, uint32_t total,
                                 FastDiv dQ, FastDiv dH) {
  const int Q = (W >> 2) + 1;  // W+1 output columns in ceil((W+1)/4) groups
  const uint32_t HW = (uint32_t)H * (uint32_t)W;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < total; p += gridDim.x * blockDim.x) {
    const uint32_t nh = dQ.div(p);
    const int q = (int)(p - nh * (uint32_t)Q);
    const uint32_t n = dH.div(nh);
    const uint32_t h = nh - n * (uint32_t)H;
    const float* xb = x + (int64_t)n * 3 * HW + (int64_t)h * W;
    const int w0 = q << 2;
    float c[3][5];  // c[j][i] = x(h, w0 - 1 + i, j)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float* xr = xb + (int64_t)j * HW;
      c[j][0] = w0 >= 1 ? xr[w0 - 1] : 0.f;
      if (w0 < W) {
        const float4 f = *(const float4*)(xr + w0);
        c[j][1] = f.x, c[j][2] = f.y, c[j][3] = f.z, c[j][4] = f.w;
      } else {
        c[j][1] = c[j][2] = c[j][3] = c[j][4] = 0.f;
      }
    }
    bf16* yp = y + ((int64_t)nh * (W + 1) + w0) * 8;
    const int nout = min(4, W + 1 - w0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < nout) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          v[j] = (bf16)c[j][i];
          v[3 + j] = (bf16)c[j][i + 1];
        }
        v[6] = (bf16)0.f;
        v[7] = (bf16)0.f;
        *(bf16x8*)(yp + i * 8) = v;
      }
    }
  }
}

// zero the fp32 element ranges [off, off + len) listed as int64 pairs in a
// device table (a lazily-zeroed gradient buffer: everything but the slices
// whose producers overwrite them), one launch for all ranges
__global__ void zero_ranges_k(float* __restrict__ base, const int64_t* __restrict__ r) {
  const int64_t off = r[2 * blockIdx.y], len = r[2 * blockIdx.y + 1];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < len; e += (int64_t)gridDim.x * blockDim.x)
    base[off + e] = 0.f;
}

}  // namespace sg

using namespace sg;

#define DISPATCH_FT(dtype, ...)                 \
  if ((dtype) == kF32) {                        \
    typedef float T;                            \
    __VA_ARGS__;                                \
  } else {                                      \
    typedef bf16 T;                             \
    __VA_ARGS__;                                \
  }

extern "C" {

// the hot activations get their own instantiation (compile-time op)
#define UNARY_HOT(F, ...)                                             \
  switch (op) {                                                      \
    case U_RELU: F(U_RELU, __VA_ARGS__); break;                      \
    case U_GELU: F(U_GELU, __VA_ARGS__); break;                      \
    case U_GELU_TANH: F(U_GELU_TANH, __VA_ARGS__); break;            \
    case U_TANH: F(U_TANH, __VA_ARGS__); break;                      \
    case U_SIGMOID: F(U_SIGMOID, __VA_ARGS__); break;                \
    default: F(-1, __VA_ARGS__);                                     \
  }
#define UFWD(OPC, T_)                                                                                         \
  hipLaunchKernelGGL((unary_fwd_k<T_, OPC>), dim3(sg_grid(n / Vec<T_>::N + 1)), dim3(256), 0, s, op, (const T_*)x, \
                     (T_*)y, n, a)
#define UBWD(OPC, T_)                                                                                          \
  hipLaunchKernelGGL((unary_bwd_k<T_, OPC>), dim3(sg_grid(n / Vec<T_>::N + 1)), dim3(256), 0, s, op, (const T_*)x, \
                     (const T_*)y, (const T_*)dy, (T_*)dx, n, a)

void sg_unary_fwd(int op, const void* x, void* y, int64_t n, int dtype, float a, hipStream_t s) {
  DISPATCH_FT(dtype, UNARY_HOT(UFWD, T));
}
void sg_unary_bwd(int op, const void* x, const void* y, const void* dy, void* dx, int64_t n, int dtype, float a,
                  hipStream_t s) {
  DISPATCH_FT(dtype, UNARY_HOT(UBWD, T));
}
#undef UFWD
#undef UBWD
#undef UNARY_HOT
void sg_add_act(const void* a, const void* b, void* y, int64_t n, int dtype, float alpha, float beta, int relu,
                hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(add_act_k<T>, dim3(sg_grid(n / Vec<T>::N + 1)), dim3(256), 0, s,
                                        (const T*)a, (const T*)b, (T*)y, n, alpha, beta, relu));
}
void sg_zero_ranges(void* base, const void* ranges, int nr, hipStream_t s) {
  if (nr <= 0) return;
  hipLaunchKernelGGL(sg::zero_ranges_k, dim3(512, nr), dim3(256), 0, s, (float*)base, (const int64_t*)ranges);
}
void sg_mask_bits_apply(const void* g, const void* mask, void* out, int64_t n, hipStream_t s) {
  const int64_t nv = n / 8;
  hipLaunchKernelGGL(mask_bits_apply_k, dim3(sg_grid(nv)), dim3(256), 0, s, (const uint4*)g, (const uint8_t*)mask,
                     (uint4*)out, nv);
}
void sg_relu_bwd_from_y(const void* y, const void* dy, void* dx, int64_t n, int dtype, hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(relu_bwd_from_y_k<T>, dim3(sg_grid(n / Vec<T>::N + 1)), dim3(256), 0, s,
                                        (const T*)y, (const T*)dy, (T*)dx, n));
}
void sg_cast(const void* x, int dtx, void* y, int dty, int64_t n, hipStream_t s) {
  dim3 g(sg_grid(n / 4 + 1)), b(256);
  if (dtx == kF32 && dty == kBF16) hipLaunchKernelGGL((cast_k<float, bf16>), g, b, 0, s, (const float*)x, (bf16*)y, n);
  else if (dtx == kBF16 && dty == kF32) hipLaunchKernelGGL((cast_k<bf16, float>), g, b, 0, s, (const bf16*)x, (float*)y, n);
  else if (dtx == kF32 && dty == kF32) hipLaunchKernelGGL((cast_k<float, float>), g, b, 0, s, (const float*)x, (float*)y, n);
  else hipLaunchKernelGGL((cast_k<bf16, bf16>), g, b, 0, s, (const bf16*)x, (bf16*)y, n);
}
void sg_dropout_fwd(const void* x, void* y, void* mask, int64_t n, int dtype, float pkeep, uint64_t seed,
                    uint64_t offset, const void* epoch, hipStream_t s) {
  if (n % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL(dropout_fwd8_k<T>, dim3(sg_grid(n / 8)), dim3(256), 0, s, (const T*)x,
                                          (T*)y, (uint8_t*)mask, n, pkeep, seed, offset, (const int64_t*)epoch));
    return;
  }
  DISPATCH_FT(dtype, hipLaunchKernelGGL(dropout_fwd_k<T>, dim3(sg_grid(n / 4 + 1)), dim3(256), 0, s, (const T*)x,
                                        (T*)y, (uint8_t*)mask, n, pkeep, seed, offset, (const int64_t*)epoch));
}
void sg_dropout_bwd(const void* dy, const void* mask, void* dx, int64_t n, int dtype, float pkeep, hipStream_t s) {
  if (n % 8 == 0) {
    DISPATCH_FT(dtype, hipLaunchKernelGGL(dropout_bwd8_k<T>, dim3(sg_grid(n / 8)), dim3(256), 0, s, (const T*)dy,
                                          (const uint8_t*)mask, (T*)dx, n, pkeep));
    return;
  }
  DISPATCH_FT(dtype, hipLaunchKernelGGL(dropout_bwd_k<T>, dim3(sg_grid(n)), dim3(256), 0, s, (const T*)dy,
                                        (const uint8_t*)mask, (T*)dx, n, pkeep));
}
void sg_rand_fill(void* y, int64_t n, int dtype, int dist, float a, float b, uint64_t seed, uint64_t offset,
                  hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(rand_fill_k<T>, dim3(sg_grid(n / 4 + 1)), dim3(256), 0, s, (T*)y, n, dist,
                                        a, b, seed, offset));
}
void sg_nchw_to_pairs(const void* x, void* y, int N, int C, int H, int W, hipStream_t s) {
  const int64_t total = (int64_t)N * H * (W + 1);
  if (total >= (int64_t)UINT32_MAX) throw std::runtime_error("nchw_to_pairs: more than 2^32 pixel pairs");
  if (C == 3 && W % 4 == 0 && ((uintptr_t)x & 15) == 0) {
    const int64_t t4 = (int64_t)N * H * (W / 4 + 1);
    hipLaunchKernelGGL(nchw_to_pairs4_k, dim3(sg_grid(t4)), dim3(256), 0, s, (const float*)x, (bf16*)y, H, W,
                       (uint32_t)t4, FastDiv(W / 4 + 1), FastDiv(H));
    return;
  }
  hipLaunchKernelGGL(nchw_to_pairs_k, dim3(sg_grid(total)), dim3(256), 0, s, (const float*)x, (bf16*)y, N, C, H, W,
                     (uint32_t)total, FastDiv(W + 1), FastDiv(H));
}

void sg_nchw_to_nhwc_pad(const void* x, void* y, int N, int C, int H, int W, int Cp, hipStream_t s) {
  hipLaunchKernelGGL(nchw_to_nhwc_pad_k<float>, dim3(sg_grid((int64_t)N * H * W)), dim3(256), 0, s, (const float*)x,
                     (bf16*)y, N, C, H, W, Cp);
}
// bf16 NCHW input (a model that casts its fp32 images first, e.g. AlexNet)
void sg_nchw_to_nhwc_pad_bf16(const void* x, void* y, int N, int C, int H, int W, int Cp, hipStream_t s) {
  hipLaunchKernelGGL(nchw_to_nhwc_pad_k<bf16>, dim3(sg_grid((int64_t)N * H * W)), dim3(256), 0, s, (const bf16*)x,
                     (bf16*)y, N, C, H, W, Cp);
}

}  // extern "C"

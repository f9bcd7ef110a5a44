// Row softmax, fused softmax + cross-entropy (forward + backward + top-k), and
// LayerNorm forward/backward.
//
// The reference computes Softmax on the device (K5,
// include/mshadow/cuda/tensor_gpu-inl.cuh:172-228) but the NLL loss, top-k
// precision and gradient on the host (SoftmaxLossLayer, src/worker/layer.cc:
// 718-764) and caps labels at 10 classes (:728).  Here one workgroup per row
// does everything in a single pass over the logits staged in LDS, for any
// class count.
#include "common.h"

namespace sg {

// one 256-thread block per row; row staged through LDS (C <= 16384 floats)
template <typename T>
__global__ void softmax_fwd_k(const T* __restrict__ x, float* __restrict__ y_f32, T* __restrict__ y_t, int C) {
  extern __shared__ float srow[];
  __shared__ float sh[8];
  const int64_t r = blockIdx.x;
  const T* xr = x + r * C;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float v = to_f32(xr[c]);
    srow[c] = v;
    m = fmaxf(m, v);
  }
  m = block_max(m, sh);
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float e = __expf(srow[c] - m);
    srow[c] = e;
    s += e;
  }
  s = block_sum(s, sh);
  const float inv = 1.f / s;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float p = srow[c] * inv;
    if (y_f32) y_f32[r * C + c] = p;
    if (y_t) y_t[r * C + c] = from_f32<T>(p);
  }
}

// dx = y * (dy - sum(dy * y))
template <typename T>
__global__ void softmax_bwd_k(const T* __restrict__ y, const T* __restrict__ dy, T* __restrict__ dx, int C) {
  __shared__ float sh[8];
  const int64_t r = blockIdx.x;
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) s += to_f32(y[r * C + c]) * to_f32(dy[r * C + c]);
  s = block_sum(s, sh);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float yv = to_f32(y[r * C + c]);
    dx[r * C + c] = from_f32<T>(yv * (to_f32(dy[r * C + c]) - s));
  }
}

// Fused softmax cross-entropy.  labels: int32 class ids, or (soft_target)
// a [B][C] probability matrix.  Outputs: loss[r] (fp32), correct[r] (1 if
// the label is within the top-k), dx = (p - t) * grad_scale (may be null).
template <typename T>
__global__ void softmax_xent_k(const T* __restrict__ x, const int* __restrict__ labels,
                               const float* __restrict__ soft_t, float* __restrict__ loss,
                               float* __restrict__ correct, T* __restrict__ dx, int C, int topk,
                               float grad_scale) {
  extern __shared__ float srow[];
  __shared__ float sh[8];
  const int64_t r = blockIdx.x;
  const T* xr = x + r * C;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float v = to_f32(xr[c]);
    srow[c] = v;
    m = fmaxf(m, v);
  }
  m = block_max(m, sh);
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) s += __expf(srow[c] - m);
  s = block_sum(s, sh);
  const float lse = m + __logf(s);
  float l;
  if (soft_t == nullptr) {
    const int lab = labels[r];
    const float xl = (lab >= 0 && lab < C) ? srow[lab] : 0.f;
    // rank of the label: #classes with a strictly larger logit
    int cnt = 0;
    for (int c = threadIdx.x; c < C; c += blockDim.x) cnt += srow[c] > xl;
    float fc = block_sum((float)cnt, sh);
    l = lse - xl;
    if (threadIdx.x == 0) {
      loss[r] = l;
      if (correct) correct[r] = (fc < (float)topk) ? 1.f : 0.f;
    }
    if (dx) {
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float p = __expf(srow[c] - lse);
        dx[r * C + c] = from_f32<T>((p - (c == lab ? 1.f : 0.f)) * grad_scale);
      }
    }
  } else {
    const float* tr = soft_t + r * C;
    float acc = 0.f, tsum = 0.f;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      acc += tr[c] * (lse - srow[c]);
      tsum += tr[c];
    }
    acc = block_sum(acc, sh);
    tsum = block_sum(tsum, sh);
    if (threadIdx.x == 0) {
      loss[r] = acc;
      if (correct) correct[r] = 0.f;
    }
    if (dx) {
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float p = __expf(srow[c] - lse);
        dx[r * C + c] = from_f32<T>((p * tsum - tr[c]) * grad_scale);
      }
    }
  }
}

// LayerNorm over the last dim D (BERT).  mean/rstd saved in fp32.
template <typename T>
__global__ void layernorm_fwd_k(const T* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
                                T* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd, int D,
                                float eps) {
  __shared__ float sh[8];
  const int64_t r = blockIdx.x;
  const T* xr = x + r * D;
  float s = 0.f;
  for (int c = threadIdx.x; c < D; c += blockDim.x) s += to_f32(xr[c]);
  const float mu = block_sum(s, sh) / D;
  float v = 0.f;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float d = to_f32(xr[c]) - mu;
    v += d * d;
  }
  const float rs = rsqrtf(block_sum(v, sh) / D + eps);
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float o = (to_f32(xr[c]) - mu) * rs;
    if (g) o = o * g[c];
    if (b) o += b[c];
    y[r * D + c] = from_f32<T>(o);
  }
  if (threadIdx.x == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)); dg/db via atomics.
template <typename T>
__global__ void layernorm_bwd_k(const T* __restrict__ x, const T* __restrict__ dy, const float* __restrict__ g,
                                const float* __restrict__ mean, const float* __restrict__ rstd, T* __restrict__ dx,
                                float* __restrict__ dg, float* __restrict__ db, int D) {
  __shared__ float sh[8];
  const int64_t r = blockIdx.x;
  const float mu = mean[r], rs = rstd[r];
  float a = 0.f, bsum = 0.f;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float xh = (to_f32(x[r * D + c]) - mu) * rs;
    float gy = to_f32(dy[r * D + c]) * (g ? g[c] : 1.f);
    a += gy;
    bsum += gy * xh;
  }
  a = block_sum(a, sh) / D;
  bsum = block_sum(bsum, sh) / D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float xh = (to_f32(x[r * D + c]) - mu) * rs;
    float dyv = to_f32(dy[r * D + c]);
    float gy = dyv * (g ? g[c] : 1.f);
    dx[r * D + c] = from_f32<T>(rs * (gy - a - xh * bsum));
    if (dg) atomicAdd(dg + c, dyv * xh);
    if (db) atomicAdd(db + c, dyv);
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

void sg_softmax_fwd(const void* x, void* y, int64_t R, int C, int dtype, int out_f32, hipStream_t s) {
  size_t sm = (size_t)C * sizeof(float);
  DISPATCH_FT(dtype, hipLaunchKernelGGL(softmax_fwd_k<T>, dim3(R), dim3(256), sm, s, (const T*)x,
                                        out_f32 ? (float*)y : nullptr, out_f32 ? nullptr : (T*)y, C));
}
void sg_softmax_bwd(const void* y, const void* dy, void* dx, int64_t R, int C, int dtype, hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(softmax_bwd_k<T>, dim3(R), dim3(256), 0, s, (const T*)y, (const T*)dy,
                                        (T*)dx, C));
}
void sg_softmax_xent(const void* x, const void* labels, const void* soft_t, void* loss, void* correct, void* dx,
                     int64_t R, int C, int dtype, int topk, float grad_scale, hipStream_t s) {
  size_t sm = (size_t)C * sizeof(float);
  DISPATCH_FT(dtype, hipLaunchKernelGGL(softmax_xent_k<T>, dim3(R), dim3(256), sm, s, (const T*)x,
                                        (const int*)labels, (const float*)soft_t, (float*)loss, (float*)correct,
                                        (T*)dx, C, topk, grad_scale));
}
void sg_layernorm_fwd(const void* x, const void* g, const void* b, void* y, void* mean, void* rstd, int64_t R, int D,
                      int dtype, float eps, hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(layernorm_fwd_k<T>, dim3(R), dim3(256), 0, s, (const T*)x,
                                        (const float*)g, (const float*)b, (T*)y, (float*)mean, (float*)rstd, D, eps));
}
void sg_layernorm_bwd(const void* x, const void* dy, const void* g, const void* mean, const void* rstd, void* dx,
                      void* dg, void* db, int64_t R, int D, int dtype, hipStream_t s) {
  DISPATCH_FT(dtype, hipLaunchKernelGGL(layernorm_bwd_k<T>, dim3(R), dim3(256), 0, s, (const T*)x, (const T*)dy,
                                        (const float*)g, (const float*)mean, (const float*)rstd, (T*)dx, (float*)dg,
                                        (float*)db, D));
}

}  // extern "C"

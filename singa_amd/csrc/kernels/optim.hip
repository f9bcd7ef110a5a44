// Fused multi-tensor optimisers over ONE flat fp32 parameter buffer, plus the
// EASGD elastic-averaging and RandomSync sparse-exchange kernels.
//
// Reference: Updater::Update variants (src/utils/updater.cc:62-182, F13) and
// the ParamManager's single contiguous param buffer (src/utils/param_manager.
// cc:40-69), EASGD (src/utils/param.cc:244-284, F14) and RandomSync
// (src/utils/param.cc:130-241).
//
// All parameters of a model live in one flat fp32 buffer (w), with matching
// flat gradient (g) and state buffers (s1, s2).  A host-built chunk table
// (start, len, segment id) lets a single launch cover every tensor while still
// applying per-parameter lr/wd multipliers (ParamProto.learning_rate_
// multiplier / weight_decay_multiplier).  lr and the step counter are read
// from device memory (hp[0] = lr, hp[1] = step) so a captured HIP graph can be
// replayed with a changing schedule.  Optionally the kernel also writes a
// bf16 copy of the updated weights (mixed-precision compute copy).
//
// Reference quirks fixed here: grad_scale applies
// to the whole gradient for every updater, and Nesterov's momentum is set.
#include "common.h"

namespace sg {

enum OptKind : int { O_SGD = 0, O_NESTEROV_REF = 1, O_ADAGRAD = 2, O_RMSPROP = 3, O_ADADELTA = 4, O_ADAM = 5,
                     O_SGD_REF = 6 };

struct OptArgs {
  float momentum, dampening, wd, grad_scale;
  float beta1, beta2, eps, rho;
  int nesterov, adamw;
};

// One element of every update rule: w, optimizer state h1 / h2 (in / out).
template <int KIND>
__device__ __forceinline__ void opt_elem(float& wv, float gv, float& h1, float& h2, float lr, float wd, float bc1,
                                         float bc2, const OptArgs& a) {
  if (KIND == O_SGD) {
    gv += wd * wv;
    if (a.momentum != 0.f) {
      float b = h1;
      b = a.momentum * b + (1.f - a.dampening) * gv;
      h1 = b;
      gv = a.nesterov ? gv + a.momentum * b : b;
    }
    wv -= lr * gv;
  } else if (KIND == O_SGD_REF) {  // reference: h = m*h + lr*g; w -= h
    gv += wd * wv;
    if (a.momentum > 0.f) {
      float h = a.momentum * h1 + lr * gv;
      h1 = h;
      wv -= h;
    } else {
      wv -= lr * gv;
    }
  } else if (KIND == O_NESTEROV_REF) {  // h0=h; h=m*h+lr*g; w -= (1+m)h - m h0
    gv += wd * wv;
    float h0 = h1;
    float h = a.momentum * h0 + lr * gv;
    h1 = h;
    wv -= (1.f + a.momentum) * h - a.momentum * h0;
  } else if (KIND == O_ADAGRAD) {
    gv += wd * wv;
    float h = h1 + gv * gv;
    h1 = h;
    wv -= lr * gv / sqrtf(h + a.eps);
  } else if (KIND == O_RMSPROP) {
    gv += wd * wv;
    float h = a.rho * h1 + (1.f - a.rho) * gv * gv;
    h1 = h;
    wv -= lr * gv / sqrtf(h + a.eps);
  } else if (KIND == O_ADADELTA) {
    gv += wd * wv;
    float h = a.rho * h1 + (1.f - a.rho) * gv * gv;
    float u = h2;
    float d = gv * sqrtf(u + a.eps) / sqrtf(h + a.eps);
    h1 = h;
    h2 = a.rho * u + (1.f - a.rho) * d * d;
    wv -= lr * d;
  } else if (KIND == O_ADAM) {
    if (!a.adamw) gv += wd * wv;
    float m = a.beta1 * h1 + (1.f - a.beta1) * gv;
    float v = a.beta2 * h2 + (1.f - a.beta2) * gv * gv;
    h1 = m;
    h2 = v;
    float upd = (m / bc1) / (sqrtf(v / bc2) + a.eps);
    if (a.adamw) upd += wd * wv;
    wv -= lr * upd;
  }
}

template <int KIND>
__global__ void __launch_bounds__(256) opt_k(float* __restrict__ w, const float* __restrict__ g,
                                             float* __restrict__ s1, float* __restrict__ s2, bf16* __restrict__ wlow,
                                             const int64_t* __restrict__ cstart, const int* __restrict__ clen,
                                             const int* __restrict__ cseg, const float* __restrict__ seg_lr,
                                             const float* __restrict__ seg_wd, const float* __restrict__ hp,
                                             OptArgs a) {
  const int chunk = blockIdx.x;
  const int64_t st = cstart[chunk];
  const int len = clen[chunk];
  const int seg = cseg[chunk];
  const float lr = hp[0] * seg_lr[seg];
  const float wd = a.wd * seg_wd[seg];
  const float t = hp[1];
  float bc1 = 1.f, bc2 = 1.f;
  if (KIND == O_ADAM) {
    bc1 = 1.f - __powf(a.beta1, t);
    bc2 = 1.f - __powf(a.beta2, t);
  }
  // 16-byte vectors over the chunk (chunk starts are 4-element aligned: the
  // flat store aligns every parameter), scalar tail
  const int n4 = (st & 3) == 0 ? len >> 2 : 0;
  for (int q = threadIdx.x; q < n4; q += blockDim.x) {
    const int64_t e = st + 4 * (int64_t)q;
    float4 wv = *(const float4*)(w + e), gv = *(const float4*)(g + e);
    float4 h1 = s1 ? *(const float4*)(s1 + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 h2 = s2 ? *(const float4*)(s2 + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    opt_elem<KIND>(wv.x, gv.x * a.grad_scale, h1.x, h2.x, lr, wd, bc1, bc2, a);
    opt_elem<KIND>(wv.y, gv.y * a.grad_scale, h1.y, h2.y, lr, wd, bc1, bc2, a);
    opt_elem<KIND>(wv.z, gv.z * a.grad_scale, h1.z, h2.z, lr, wd, bc1, bc2, a);
    opt_elem<KIND>(wv.w, gv.w * a.grad_scale, h1.w, h2.w, lr, wd, bc1, bc2, a);
    *(float4*)(w + e) = wv;
    if (s1) *(float4*)(s1 + e) = h1;
    if (s2) *(float4*)(s2 + e) = h2;
    if (wlow) {
      bf16x4 lo;
      lo[0] = (bf16)wv.x; lo[1] = (bf16)wv.y; lo[2] = (bf16)wv.z; lo[3] = (bf16)wv.w;
      *(bf16x4*)(wlow + e) = lo;
    }
  }
  for (int i = 4 * n4 + threadIdx.x; i < len; i += blockDim.x) {
    const int64_t e = st + i;
    float wv = w[e], h1 = s1 ? s1[e] : 0.f, h2 = s2 ? s2[e] : 0.f;
    opt_elem<KIND>(wv, g[e] * a.grad_scale, h1, h2, lr, wd, bc1, bc2, a);
    w[e] = wv;
    if (s1) s1[e] = h1;
    if (s2) s2[e] = h2;
    if (wlow) wlow[e] = (bf16)wv;
  }
}

// squared L2 norm of a flat buffer into out[0] (atomic); for grad clipping
__global__ void sqnorm_k(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
  __shared__ float sh[8];
  float s = 0.f;
  SG_GRID_STRIDE(i, n) { s += x[i] * x[i]; }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

// EASGD worker side: d = alpha*(w - c); w -= d.  d is then summed across
// ranks (all-reduce) and added to the centre: c += sum_i d_i.
__global__ void easgd_diff_k(float* __restrict__ w, const float* __restrict__ c, float* __restrict__ d, int64_t n,
                             float alpha) {
  SG_GRID_STRIDE(i, n) {
    float dv = alpha * (w[i] - c[i]);
    d[i] = dv;
    w[i] -= dv;
  }
}

__global__ void axpy_k(float* __restrict__ y, const float* __restrict__ x, int64_t n, float a) {
  SG_GRID_STRIDE(i, n) { y[i] += a * x[i]; }
}

// RandomSync: sample m indices of an n-element buffer as the arithmetic
// progression idx(k) = (b + k*a) mod n with gcd(a, n) = 1 (a permutation:
// no duplicates), so every rank derives the same set from (a, b) with no
// index traffic.  gather: out[k] = w[idx] - snap[idx].
__global__ void rsync_gather_k(const float* __restrict__ w, const float* __restrict__ snap, float* __restrict__ out,
                               int64_t m, int64_t n, int64_t a, int64_t b) {
  SG_GRID_STRIDE(k, m) {
    int64_t idx = (int64_t)(((uint64_t)b + ((uint64_t)k * (uint64_t)a) % (uint64_t)n) % (uint64_t)n);
    out[k] = w[idx] - snap[idx];
  }
}
// scatter: w[idx] = snap[idx] + delta_sum[k]; snap[idx] = w[idx]
__global__ void rsync_scatter_k(float* __restrict__ w, float* __restrict__ snap, const float* __restrict__ dsum,
                                int64_t m, int64_t n, int64_t a, int64_t b) {
  SG_GRID_STRIDE(k, m) {
    int64_t idx = (int64_t)(((uint64_t)b + ((uint64_t)k * (uint64_t)a) % (uint64_t)n) % (uint64_t)n);
    float nv = snap[idx] + dsum[k];
    w[idx] = nv;
    snap[idx] = nv;
  }
}

}  // namespace sg

using namespace sg;

extern "C" {

void sg_opt_update(int kind, void* w, const void* g, void* s1, void* s2, void* wlow, const void* cstart,
                   const void* clen, const void* cseg, const void* seg_lr, const void* seg_wd, const void* hp,
                   int nchunks, float momentum, float dampening, float wd, float grad_scale, float beta1, float beta2,
                   float eps, float rho, int nesterov, int adamw, hipStream_t s) {
  OptArgs a{momentum, dampening, wd, grad_scale, beta1, beta2, eps, rho, nesterov, adamw};
#define L(K)                                                                                                        \
  hipLaunchKernelGGL(opt_k<K>, dim3(nchunks), dim3(256), 0, s, (float*)w, (const float*)g, (float*)s1, (float*)s2, \
                     (bf16*)wlow, (const int64_t*)cstart, (const int*)clen, (const int*)cseg, (const float*)seg_lr,  \
                     (const float*)seg_wd, (const float*)hp, a)
  switch (kind) {
    case O_SGD: L(O_SGD); break;
    case O_NESTEROV_REF: L(O_NESTEROV_REF); break;
    case O_ADAGRAD: L(O_ADAGRAD); break;
    case O_RMSPROP: L(O_RMSPROP); break;
    case O_ADADELTA: L(O_ADADELTA); break;
    case O_ADAM: L(O_ADAM); break;
    case O_SGD_REF: L(O_SGD_REF); break;
  }
#undef L
}
void sg_sqnorm(const void* x, int64_t n, void* out, hipStream_t s) {
  hipLaunchKernelGGL(sqnorm_k, dim3(sg_grid(n, 256, 1024)), dim3(256), 0, s, (const float*)x, n, (float*)out);
}
void sg_easgd_diff(void* w, const void* c, void* d, int64_t n, float alpha, hipStream_t s) {
  hipLaunchKernelGGL(easgd_diff_k, dim3(sg_grid(n)), dim3(256), 0, s, (float*)w, (const float*)c, (float*)d, n, alpha);
}
void sg_axpy(void* y, const void* x, int64_t n, float a, hipStream_t s) {
  hipLaunchKernelGGL(axpy_k, dim3(sg_grid(n)), dim3(256), 0, s, (float*)y, (const float*)x, n, a);
}
void sg_rsync_gather(const void* w, const void* snap, void* out, int64_t m, int64_t n, int64_t a, int64_t b,
                     hipStream_t s) {
  hipLaunchKernelGGL(rsync_gather_k, dim3(sg_grid(m)), dim3(256), 0, s, (const float*)w, (const float*)snap,
                     (float*)out, m, n, a, b);
}
void sg_rsync_scatter(void* w, void* snap, const void* dsum, int64_t m, int64_t n, int64_t a, int64_t b,
                      hipStream_t s) {
  hipLaunchKernelGGL(rsync_scatter_k, dim3(sg_grid(m)), dim3(256), 0, s, (float*)w, (float*)snap,
                     (const float*)dsum, m, n, a, b);
}

}  // extern "C"

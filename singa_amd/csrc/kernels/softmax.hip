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
#include <stdlib.h>

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


// ---- short rows (C <= 64*NJ): one WAVE per row, the row in registers ----
// Attention probabilities (C = sequence length, ~50K rows of 128) ran one
// 256-thread block per row through LDS: 3/4 of every block idle and two block
// barriers per row.  Here lane l owns columns l, l+64, ... (coalesced), the
// reductions are wave shuffles, and the output dtype is independent of the
// input (fp32 scores -> bf16 probabilities in the same pass).
template <typename TI, typename TO, int NJ>
__global__ void __launch_bounds__(256) softmax_rows_k(const TI* __restrict__ x, TO* __restrict__ y, int64_t R, int C) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const TI* xr = x + r * C;
  float v[NJ];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < C ? to_f32(xr[c]) : -INFINITY;
    m = fmaxf(m, v[j]);
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    v[j] = lane + 64 * j < C ? __expf(v[j] - m) : 0.f;
    s += v[j];
  }
  const float inv = 1.f / wave_sum(s);
  TO* yr = y + r * C;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    if (c < C) yr[c] = from_f32<TO>(v[j] * inv);
  }
}

template <typename T, int NJ>
__global__ void __launch_bounds__(256) softmax_bwd_rows_k(const T* __restrict__ y, const T* __restrict__ dy,
                                                          T* __restrict__ dx, int64_t R, int C) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  float yv[NJ], gv[NJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    yv[j] = c < C ? to_f32(y[r * C + c]) : 0.f;
    gv[j] = c < C ? to_f32(dy[r * C + c]) : 0.f;
    s += yv[j] * gv[j];
  }
  s = wave_sum(s);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    if (c < C) dx[r * C + c] = from_f32<T>(yv[j] * (gv[j] - s));
  }
}

// ---- LayerNorm backward, rows batched per workgroup ----
// The per-row kernel above adds every row's dgamma/dbeta contribution with a
// global atomic per element: 2*D atomics per row, all rows hammering the same
// D addresses (BERT: 4096 rows x 1536 atomics, 128 us per call, 21 % of the
// step).  Here each wave owns a row at a time, lane l owns the 4-column
// groups 4*(l + 64*j), dgamma/dbeta partials stay in registers across the
// workgroup's rows, the 4 waves combine through LDS, and each workgroup
// issues ONE atomic per column.
template <typename T> struct V4;
template <> struct V4<float> {
  __device__ static void ld(const float* p, float v[4]) {
    const float4 t = *(const float4*)p;
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  __device__ static void st(float* p, const float v[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
};
template <> struct V4<bf16> {
  __device__ static void ld(const bf16* p, float v[4]) {
    const bf16x4 t = *(const bf16x4*)p;
    v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
  }
  __device__ static void st(bf16* p, const float v[4]) {
    bf16x4 t;
    t[0] = (bf16)v[0]; t[1] = (bf16)v[1]; t[2] = (bf16)v[2]; t[3] = (bf16)v[3];
    *(bf16x4*)p = t;
  }
};

// LayerNorm forward, one WAVE per row (D % 4 == 0, D <= 2048): lane l owns
// the 4-column groups 4*(l + 64*j), the row stays in registers, mean and
// variance are wave shuffles (the block-per-row kernel above pays two block
// barriers per row for 768 columns)
template <typename T, int NJ>
__global__ void __launch_bounds__(256) layernorm_fwd_rows_k(const T* __restrict__ x, const float* __restrict__ g,
                                                            const float* __restrict__ b, T* __restrict__ y,
                                                            float* __restrict__ mean, float* __restrict__ rstd,
                                                            int64_t R, int D, float eps) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  float v[NJ][4], gv[NJ][4], bv[NJ][4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
      V4<T>::ld(x + r * D + c, v[j]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = 0.f;
    }
  }
  // gamma / beta as 16-byte loads issued with the row's (their latency hides
  // behind the reductions instead of following them)
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    const float4 g4 = (g && c < D) ? *(const float4*)(g + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 b4 = (b && c < D) ? *(const float4*)(b + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    gv[j][0] = g4.x; gv[j][1] = g4.y; gv[j][2] = g4.z; gv[j][3] = g4.w;
    bv[j][0] = b4.x; bv[j][1] = b4.y; bv[j][2] = b4.z; bv[j][3] = b4.w;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += v[j][e];
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mu;
        q += d * d;
      }
    }
  }
  const float rs = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mu) * rs * gv[j][e] + bv[j][e];
      V4<T>::st(y + r * D + c, o);
    }
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

template <typename T, int NJ>
__global__ void __launch_bounds__(256) layernorm_bwd_rows_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                            const float* __restrict__ g, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, T* __restrict__ dx,
                                                            float* __restrict__ dg, float* __restrict__ db, int64_t R,
                                                            int D, int rpb) {
  extern __shared__ float red[];  // [4 waves][2][D]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float gw[NJ][4], adg[NJ][4], adb[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gw[j][e] = (g && c < D) ? g[c + e] : 1.f;
      adg[j][e] = 0.f;
      adb[j][e] = 0.f;
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < R ? r0 + rpb : R;
  const float invD = 1.f / D;
  for (int64_t r = r0 + wave; r < r1; r += 4) {
    const float mu = mean[r], rs = rstd[r];
    float xh[NJ][4], dv[NJ][4];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c < D) {
        V4<T>::ld(x + r * D + c, xh[j]);
        V4<T>::ld(dy + r * D + c, dv[j]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) { xh[j][e] = mu; dv[j][e] = 0.f; }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[j][e] = (xh[j][e] - mu) * rs;
        const float gy = dv[j][e] * gw[j][e];
        a += gy;
        b += gy * xh[j][e];
      }
    }
    a = wave_sum(a) * invD;
    b = wave_sum(b) * invD;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c < D) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = rs * (dv[j][e] * gw[j][e] - a - xh[j][e] * b);
          adg[j][e] += dv[j][e] * xh[j][e];
          adb[j][e] += dv[j][e];
        }
        V4<T>::st(dx + r * D + c, o);
      }
    }
  }
  if (!dg && !db) return;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[(wave * 2) * D + c + e] = adg[j][e];
        red[(wave * 2 + 1) * D + c + e] = adb[j][e];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      s0 += red[(w * 2) * D + c];
      s1 += red[(w * 2 + 1) * D + c];
    }
    if (dg) atomicAdd(dg + c, s0);
    if (db) atomicAdd(db + c, s1);
  }
}

// LayerNorm backward v2: RPW rows per wave, software-pipelined (the next
// row's x / dy loads are issued before this row's reductions), and the
// dgamma / dbeta partial sums of each workgroup go to its own workspace row
// with plain stores; ln_fold_k folds the rows into dg / db (8 rows per
// thread, one atomic per (row chunk, column)).  v1's single-level atomics
// serialise every workgroup on the same 2D addresses, which is why it had to
// run with few, long workgroups (latency-bound: 15 us isolated, 23 us in the
// BERT step for a 6 MB row block).
// DROP: the LayerNorm of a residual sum s = x + dropout(a) (DropAddLayerNorm):
// also writes a's gradient da = dx * keep / pkeep (keep: the forward's byte
// mask, nullptr = keep all) and sums its columns -- the bias gradient of the
// Linear that produced a -- as a third partial row.
template <typename T, int NJ, int RPW, bool DROP = false>
__global__ void __launch_bounds__(256) layernorm_bwd2_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const float* __restrict__ g, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, T* __restrict__ dx,
                                                        float* __restrict__ ws, int64_t R, int D,
                                                        const uint8_t* __restrict__ dmask = nullptr,
                                                        float pkeep = 1.f, T* __restrict__ da = nullptr) {
  constexpr int P = DROP ? 3 : 2;  // partial rows: dgamma, dbeta (, column sums of da)
  extern __shared__ float red[];  // [4 waves][P][D]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float gw[NJ][4], adg[NJ][4], adb[NJ][4], acs[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    const float4 g4 = (g && c < D) ? *(const float4*)(g + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    gw[j][0] = g4.x; gw[j][1] = g4.y; gw[j][2] = g4.z; gw[j][3] = g4.w;
#pragma unroll
    for (int e = 0; e < 4; ++e) { adg[j][e] = 0.f; adb[j][e] = 0.f; acs[j][e] = 0.f; }
  }
  const int64_t rb = ((int64_t)blockIdx.x * 4 + wave) * RPW;
  const float invD = 1.f / D, dscale = 1.f / pkeep;
  float xn[NJ][4], dn[NJ][4];
  uint32_t mn[NJ];
  // unconditional loads (columns past D re-read column 0, then zeroed): a
  // load inside the divergent c < D branch gets an s_waitcnt vmcnt(0) at the
  // branch join, which would also drain the next row's prefetch
  const uint8_t* mp = dmask ? dmask : (const uint8_t*)x;  // (a valid address when there is no mask)
  auto load = [&](int64_t r) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = 4 * (lane + 64 * j);
      const int cc = c < D ? c : 0;
      V4<T>::ld(x + r * D + cc, xn[j]);
      V4<T>::ld(dy + r * D + cc, dn[j]);
      mn[j] = 0x01010101u;
      if constexpr (DROP) {
        const uint32_t mw = *(const uint32_t*)(mp + r * D + cc);
        mn[j] = dmask ? mw : 0x01010101u;
      }
      if (c >= D) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { xn[j][e] = 0.f; dn[j][e] = 0.f; }
      }
    }
  };
  if (rb < R) load(rb);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int64_t r = rb + i;
    if (r >= R) break;
    float xh[NJ][4], dv[NJ][4];
    uint32_t mk[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      mk[j] = mn[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) { xh[j][e] = xn[j][e]; dv[j][e] = dn[j][e]; }
    }
    if (i + 1 < RPW && r + 1 < R) load(r + 1);  // the next row in flight during this one
    const float mu = mean[r], rs = rstd[r];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[j][e] = (xh[j][e] - mu) * rs;
        const float gy = dv[j][e] * gw[j][e];
        a += gy;
        b += gy * xh[j][e];
      }
    a = wave_sum(a) * invD;
    b = wave_sum(b) * invD;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c < D) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = rs * (dv[j][e] * gw[j][e] - a - xh[j][e] * b);
          adg[j][e] += dv[j][e] * xh[j][e];
          adb[j][e] += dv[j][e];
        }
        V4<T>::st(dx + r * D + c, o);
        if constexpr (DROP) {
          float q[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            // the unfused dropout backward's arithmetic on the stored dx
            q[e] = ((mk[j] >> (8 * e)) & 0xffu) ? (float)(T)o[e] * dscale : 0.f;
            acs[j][e] += (float)(T)q[e];
          }
          V4<T>::st(da + r * D + c, q);
        }
      }
    }
  }
  if (!ws) return;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[(wave * P) * D + c + e] = adg[j][e];
        red[(wave * P + 1) * D + c + e] = adb[j][e];
        if (DROP) red[(wave * P + 2) * D + c + e] = acs[j][e];
      }
    }
  }
  __syncthreads();
  float* wr = ws + (int64_t)blockIdx.x * P * D;
  for (int c = threadIdx.x; c < P * D; c += 256) {
    const int h = c / D, cc = c - h * D;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += red[(w * P + h) * D + cc];
    wr[c] = s;
  }
}

// fold the per-workgroup partial rows [nb][P][D] into out0 / out1 / out2 (+=)
__global__ void __launch_bounds__(256) ln_fold_k(const float* __restrict__ ws, int nb, int D, int P,
                                                 float* __restrict__ o0, float* __restrict__ o1,
                                                 float* __restrict__ o2) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= P * D) return;
  const int r0 = blockIdx.y * 8, r1 = r0 + 8 < nb ? r0 + 8 : nb;
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += ws[(int64_t)r * P * D + c];
  const int h = c / D;
  float* o = h == 0 ? o0 : h == 1 ? o1 : o2;
  if (o) atomicAdd(o + (c - h * D), s);
}

// y = LayerNorm(s), s = x + dropout(a) in one pass (one wave per row): the
// dropout mask is the separate dropout kernel's Philox stream element for
// element (dropout_fwd8_k: counter offset + 2 (e / 8) + ((e / 4) & 1)), and
// every intermediate is rounded to T where the unfused chain stores it, so the
// result is bitwise the dropout -> add -> LayerNorm chain's.  Writes s (the
// backward's input), the byte mask, y and the row statistics.  pkeep >= 1:
// no dropout (mask untouched).
template <typename T, int NJ>
__global__ void __launch_bounds__(256) drop_add_ln_fwd_k(const T* __restrict__ x, const T* __restrict__ a,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         T* __restrict__ s_out, uint8_t* __restrict__ dmask,
                                                         T* __restrict__ y, float* __restrict__ mean,
                                                         float* __restrict__ rstd, int64_t R, int D, float eps,
                                                         float pkeep, uint64_t seed, uint64_t offset,
                                                         const int64_t* __restrict__ epoch) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  if (epoch) seed += (uint64_t)(*epoch) * 0x9E3779B97F4A7C15ull;
  const bool drop = pkeep < 1.f;
  const float scale = 1.f / pkeep;
  float v[NJ][4], av[NJ][4];
  // unconditional loads (columns past D re-read column 0, then zeroed): no
  // vmcnt(0) at a divergent branch join between them
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    const int cc = c < D ? c : 0;
    V4<T>::ld(x + r * D + cc, v[j]);
    V4<T>::ld(a + r * D + cc, av[j]);
    if (c >= D) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[j][e] = 0.f; av[j][e] = 0.f; }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
      const int64_t e0 = r * D + c;
      uint32_t mb = 0;
      if (drop) {
        const uint4 rr = Philox::gen(seed, offset + 2 * (uint64_t)(e0 >> 3) + (uint64_t)((e0 >> 2) & 1), 0);
        const uint32_t w4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool keep = Philox::u01(w4[e]) <= pkeep;
          mb |= (uint32_t)keep << (8 * e);
          av[j][e] = (float)(T)(keep ? av[j][e] * scale : 0.f);
        }
        *(uint32_t*)(dmask + e0) = mb;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = (float)(T)(v[j][e] + av[j][e]);
      V4<T>::st(s_out + e0, v[j]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) s += v[j][e];
  }
  float gv[NJ][4], bv[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    const float4 g4 = (g && c < D) ? *(const float4*)(g + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 b4 = (b && c < D) ? *(const float4*)(b + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    gv[j][0] = g4.x; gv[j][1] = g4.y; gv[j][2] = g4.z; gv[j][3] = g4.w;
    bv[j][0] = b4.x; bv[j][1] = b4.y; bv[j][2] = b4.z; bv[j][3] = b4.w;
  }
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mu;
        q += d * d;
      }
    }
  }
  const float rs = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < D) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mu) * rs * gv[j][e] + bv[j][e];
      V4<T>::st(y + r * D + c, o);
    }
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
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
// short rows (C <= 1024): one wave per row; in_dt / out_dt: kF32 or kBF16
void sg_softmax_rows(const void* x, void* y, int64_t R, int C, int in_dt, int out_dt, hipStream_t s) {
  const int nj = (C + 63) / 64;
  const dim3 grid((unsigned)((R + 3) / 4));
#define SMR(TI, TO, NJ) hipLaunchKernelGGL((softmax_rows_k<TI, TO, NJ>), grid, dim3(256), 0, s, (const TI*)x, (TO*)y, R, C)
#define SMR_NJ(TI, TO)                                                 \
  if (nj <= 1) { SMR(TI, TO, 1); } else if (nj <= 2) { SMR(TI, TO, 2); } \
  else if (nj <= 4) { SMR(TI, TO, 4); } else if (nj <= 8) { SMR(TI, TO, 8); } else { SMR(TI, TO, 16); }
  if (in_dt == kF32 && out_dt == kF32) { SMR_NJ(float, float); }
  else if (in_dt == kF32) { SMR_NJ(float, bf16); }
  else if (out_dt == kF32) { SMR_NJ(bf16, float); }
  else { SMR_NJ(bf16, bf16); }
#undef SMR_NJ
#undef SMR
}
void sg_softmax_bwd(const void* y, const void* dy, void* dx, int64_t R, int C, int dtype, hipStream_t s) {
  if (C <= 1024) {
    const int nj = (C + 63) / 64;
    const dim3 grid((unsigned)((R + 3) / 4));
#define SMB(NJ) DISPATCH_FT(dtype, hipLaunchKernelGGL((softmax_bwd_rows_k<T, NJ>), grid, dim3(256), 0, s, (const T*)y, \
                                                      (const T*)dy, (T*)dx, R, C))
    if (nj <= 1) { SMB(1); } else if (nj <= 2) { SMB(2); } else if (nj <= 4) { SMB(4); }
    else if (nj <= 8) { SMB(8); } else { SMB(16); }
#undef SMB
    return;
  }
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
  if (D % 4 == 0 && D <= 2048) {
    const int nj = (D + 255) / 256;
    const dim3 grid((unsigned)((R + 3) / 4));
#define LNF(NJ)                                                                                                     \
  DISPATCH_FT(dtype, hipLaunchKernelGGL((layernorm_fwd_rows_k<T, NJ>), grid, dim3(256), 0, s, (const T*)x,          \
                                        (const float*)g, (const float*)b, (T*)y, (float*)mean, (float*)rstd, R, D, eps))
    if (nj <= 1) { LNF(1); } else if (nj <= 2) { LNF(2); } else if (nj <= 3) { LNF(3); } else if (nj <= 4) { LNF(4); }
    else { LNF(8); }
#undef LNF
    return;
  }
  DISPATCH_FT(dtype, hipLaunchKernelGGL(layernorm_fwd_k<T>, dim3(R), dim3(256), 0, s, (const T*)x,
                                        (const float*)g, (const float*)b, (T*)y, (float*)mean, (float*)rstd, D, eps));
}
// rows per wave of the v2 backward (SG_LNB_RPW: 1, 2, 4 or 8; read once) and
// its workspace (floats) for R x D.  BERT-base (4096 x 768 rows, one box,
// alternating: profiles/r6/ab_lnb_rows_per_wave.txt): 2 rows 4 477-4 484 seq/s,
// 1 row 4 461-4 466, 4 rows 4 442-4 448, 8 rows 4 333 -- two rows per wave
// (512 workgroups) keep more rows in flight per CU than four (256)
static int lnb_rpw() {
  static const int v = [] {
    const char* e = getenv("SG_LNB_RPW");
    const int r = e ? atoi(e) : 2;
    return (r == 1 || r == 2 || r == 4 || r == 8) ? r : 2;
  }();
  return v;
}
int64_t sg_layernorm_bwd_ws(int64_t R, int D) {
  const int rpw = lnb_rpw();
  const int64_t nb = (R + 4 * rpw - 1) / (4 * rpw);
  return (D % 4 == 0 && D <= 2048) ? nb * 2 * D : 0;
}
#define LNB_RPW_DISPATCH(X)          \
  switch (lnb_rpw()) {               \
    case 1: { X(1); break; }         \
    case 8: { X(8); break; }         \
    case 4: { X(4); break; }         \
    default: { X(2); break; }        \
  }

// ws (sg_layernorm_bwd_ws floats, any contents) selects the v2 kernel
void sg_layernorm_bwd_v2(const void* x, const void* dy, const void* g, const void* mean, const void* rstd, void* dx,
                         void* dg, void* db, void* ws, int64_t R, int D, int dtype, hipStream_t s) {
  const int64_t nb = (R + 4 * lnb_rpw() - 1) / (4 * lnb_rpw());
  const size_t lds = (size_t)8 * D * sizeof(float);
  const int nj = (D + 255) / 256;
  float* w = (dg || db) ? (float*)ws : nullptr;
#define LNB2R(NJ, RPW)                                                                                          \
  DISPATCH_FT(dtype, hipLaunchKernelGGL((layernorm_bwd2_k<T, NJ, RPW>), dim3((unsigned)nb), dim3(256), lds, s, \
                                        (const T*)x, (const T*)dy, (const float*)g, (const float*)mean,         \
                                        (const float*)rstd, (T*)dx, w, R, D, nullptr, 1.f, nullptr))
#define LNB2_1(RPW) LNB2R(1, RPW)
#define LNB2_2(RPW) LNB2R(2, RPW)
#define LNB2_3(RPW) LNB2R(3, RPW)
#define LNB2_4(RPW) LNB2R(4, RPW)
#define LNB2_8(RPW) LNB2R(8, RPW)
  if (nj <= 1) { LNB_RPW_DISPATCH(LNB2_1) } else if (nj <= 2) { LNB_RPW_DISPATCH(LNB2_2) }
  else if (nj <= 3) { LNB_RPW_DISPATCH(LNB2_3) } else if (nj <= 4) { LNB_RPW_DISPATCH(LNB2_4) }
  else { LNB_RPW_DISPATCH(LNB2_8) }
#undef LNB2_1
#undef LNB2_2
#undef LNB2_3
#undef LNB2_4
#undef LNB2_8
#undef LNB2R
  if (w)
    hipLaunchKernelGGL(ln_fold_k, dim3((unsigned)((2 * D + 255) / 256), (unsigned)((nb + 7) / 8)), dim3(256), 0, s,
                       (const float*)w, (int)nb, D, 2, (float*)dg, (float*)db, (float*)nullptr);
}

// DropAddLayerNorm: forward (drop_add_ln_fwd_k; D % 8 == 0, D <= 2048) and
// backward (layernorm_bwd2_k<DROP>: dx = ds, da, and dgamma / dbeta / colsum(da)
// folded into dg / db / cs (+=; ws: sg_layernorm_bwd_ws * 3 / 2 floats))
void sg_drop_add_ln_fwd(const void* x, const void* a, const void* g, const void* b, void* s_out, void* mask, void* y,
                        void* mean, void* rstd, int64_t R, int D, int dtype, float eps, float pkeep, uint64_t seed,
                        uint64_t offset, const void* epoch, hipStream_t s) {
  const int nj = (D + 255) / 256;
  const dim3 grid((unsigned)((R + 3) / 4));
#define DALF(NJ)                                                                                                  \
  DISPATCH_FT(dtype, hipLaunchKernelGGL((drop_add_ln_fwd_k<T, NJ>), grid, dim3(256), 0, s, (const T*)x,         \
                                        (const T*)a, (const float*)g, (const float*)b, (T*)s_out, (uint8_t*)mask, \
                                        (T*)y, (float*)mean, (float*)rstd, R, D, eps, pkeep, seed, offset,        \
                                        (const int64_t*)epoch))
  if (nj <= 1) { DALF(1); } else if (nj <= 2) { DALF(2); } else if (nj <= 3) { DALF(3); } else if (nj <= 4) { DALF(4); }
  else { DALF(8); }
#undef DALF
}

void sg_drop_add_ln_bwd(const void* x, const void* dy, const void* g, const void* mean, const void* rstd,
                        const void* mask, float pkeep, void* dx, void* da, void* dg, void* db, void* cs, void* ws,
                        int64_t R, int D, int dtype, hipStream_t s) {
  const int64_t nb = (R + 4 * lnb_rpw() - 1) / (4 * lnb_rpw());
  const size_t lds = (size_t)12 * D * sizeof(float);
  const int nj = (D + 255) / 256;
#define LNBDR(NJ, RPW)                                                                                          \
  DISPATCH_FT(dtype, hipLaunchKernelGGL((layernorm_bwd2_k<T, NJ, RPW, true>), dim3((unsigned)nb), dim3(256), lds, \
                                        s, (const T*)x, (const T*)dy, (const float*)g, (const float*)mean,       \
                                        (const float*)rstd, (T*)dx, (float*)ws, R, D, (const uint8_t*)mask, pkeep, \
                                        (T*)da))
#define LNBD_1(RPW) LNBDR(1, RPW)
#define LNBD_2(RPW) LNBDR(2, RPW)
#define LNBD_3(RPW) LNBDR(3, RPW)
#define LNBD_4(RPW) LNBDR(4, RPW)
#define LNBD_8(RPW) LNBDR(8, RPW)
  if (nj <= 1) { LNB_RPW_DISPATCH(LNBD_1) } else if (nj <= 2) { LNB_RPW_DISPATCH(LNBD_2) }
  else if (nj <= 3) { LNB_RPW_DISPATCH(LNBD_3) } else if (nj <= 4) { LNB_RPW_DISPATCH(LNBD_4) }
  else { LNB_RPW_DISPATCH(LNBD_8) }
#undef LNBD_1
#undef LNBD_2
#undef LNBD_3
#undef LNBD_4
#undef LNBD_8
#undef LNBDR
  hipLaunchKernelGGL(ln_fold_k, dim3((unsigned)((3 * D + 255) / 256), (unsigned)((nb + 7) / 8)), dim3(256), 0, s,
                     (const float*)ws, (int)nb, D, 3, (float*)dg, (float*)db, (float*)cs);
}

void sg_layernorm_bwd(const void* x, const void* dy, const void* g, const void* mean, const void* rstd, void* dx,
                      void* dg, void* db, int64_t R, int D, int dtype, hipStream_t s) {
  if (D % 4 == 0 && D <= 2048) {
    // ~128 workgroups, whole waves' worth of rows each (R = 4096 -> 32 rows
    // per workgroup): measured 15.2 us vs 23.8 us with 512 and 33.9 us with
    // 1024 (tools/lnb_ab.py, profiles/lnb_ab.jsonl) -- every workgroup adds
    // into the same D addresses, so fewer, longer workgroups contend less.
    // SINGA_AMD_LNB_WG overrides for A/B
    static const int64_t wg = [] {
      const char* e = getenv("SINGA_AMD_LNB_WG");
      const int64_t v = e ? atoll(e) : 128;
      return v > 0 ? v : 128;
    }();
    int64_t rpb = (R + wg - 1) / wg;
    rpb = rpb < 4 ? 4 : (rpb + 3) / 4 * 4;
    const int64_t nb = (R + rpb - 1) / rpb;
    const size_t lds = (size_t)8 * D * sizeof(float);
    const int nj = (D + 255) / 256;
#define LNB(NJ)                                                                                                  \
  DISPATCH_FT(dtype, hipLaunchKernelGGL((layernorm_bwd_rows_k<T, NJ>), dim3(nb), dim3(256), lds, s, (const T*)x, \
                                        (const T*)dy, (const float*)g, (const float*)mean, (const float*)rstd,    \
                                        (T*)dx, (float*)dg, (float*)db, R, D, (int)rpb))
    if (nj <= 1) { LNB(1); } else if (nj <= 2) { LNB(2); } else if (nj <= 4) { LNB(4); } else { LNB(8); }
#undef LNB
    return;
  }
  DISPATCH_FT(dtype, hipLaunchKernelGGL(layernorm_bwd_k<T>, dim3(R), dim3(256), 0, s, (const T*)x, (const T*)dy,
                                        (const float*)g, (const float*)mean, (const float*)rstd, (T*)dx, (float*)dg,
                                        (float*)db, D));
}

}  // extern "C"

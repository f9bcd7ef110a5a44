// "Glue" kernels: layout / indexing / broadcast / reduction ops that move or
// combine tensors without being matrix products.
//
// The reference expresses these as mshadow expression plans evaluated by
// the generic MapPlan kernel (reshape, swapaxis, pad, crop, mirror,
// broadcast, repmat, sum_rows, sumall_except_dim:
// include/mshadow/tensor_expr_ext.h:354-577,706-912, K1-K4 in
// include/mshadow/cuda/tensor_gpu-inl.cuh) and as the connection layers'
// slice / concat copies (src/worker/base_layer.cc:85-173).  Here each is a
// wave64 kernel over an N-d index space whose per-operand strides come from
// the host (dimensions already coalesced there, so most launches see 1-3
// dims); indices are split with 32-bit multiplicative division when the
// space fits, never with 64-bit integer division per element.
//   copy_nd       strided copy + dtype conversion (transpose / permute, channels-last
//                 conversion, concat / split / slice, expand / tile / repeat, casts)
//   binary_nd     broadcasting arithmetic / comparison / logic
//   where_nd      broadcasting select
//   reduce        sum / mean / max / min / sum-of-squares over the middle dim of [outer][red][inner]
//   index_select  row gather (embedding forward, Gather)
//   index_add     atomic row scatter-add (embedding backward)
//   gather_el / scatter_el   ONNX GatherElements / ScatterElements along one axis
//   pad_nd / pad_bwd         constant / reflect / edge padding and its gradient
//   fill, clamp_affine       constant fill; y = clamp(a x + b, lo, hi) (clip, hardsigmoid)
#include <stdexcept>
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace sg {

constexpr int MAXD = 8, MAXOP = 4;

struct Nd {
  int nd;
  int small;  // every size and the total < 2^31: 32-bit index math with FastDiv
  int64_t size[MAXD];
  FastDiv dv[MAXD];
  int64_t st[MAXOP][MAXD];  // element strides of operands 0..3 (0: output)
};

template <int NOP>
__device__ __forceinline__ void nd_off(const Nd& d, int64_t i, int64_t* off) {
#pragma unroll
  for (int o = 0; o < NOP; ++o) off[o] = 0;
  if (d.small) {
    uint32_t u = (uint32_t)i;
    for (int k = d.nd - 1; k >= 0; --k) {
      const uint32_t q = d.dv[k].div(u);
      const int64_t r = (int64_t)(u - q * (uint32_t)d.size[k]);
#pragma unroll
      for (int o = 0; o < NOP; ++o) off[o] += r * d.st[o][k];
      u = q;
    }
  } else {
    for (int k = d.nd - 1; k >= 0; --k) {
      const int64_t q = i / d.size[k];
      const int64_t r = i - q * d.size[k];
#pragma unroll
      for (int o = 0; o < NOP; ++o) off[o] += r * d.st[o][k];
      i = q;
    }
  }
}

template <typename T> __device__ __forceinline__ float ld_f(const T* p) { return (float)p[0]; }
template <typename T> __device__ __forceinline__ T cvt_to(float v) { return (T)v; }
template <> __device__ __forceinline__ bf16 cvt_to<bf16>(float v) { return (bf16)v; }

// conversions between storage types (integers kept exact through int64)
template <typename To, typename Ti> __device__ __forceinline__ To conv(Ti v) {
  if constexpr (std::is_same<To, Ti>::value) return v;
  else if constexpr (std::is_same<To, bf16>::value) return (bf16)(float)v;
  else if constexpr (std::is_same<Ti, bf16>::value) return (To)(float)v;
  else return (To)v;
}

template <typename Ti, typename To>
__global__ void copy_nd_k(const Ti* __restrict__ src, To* __restrict__ dst, const Nd d, int64_t n) {
  SG_GRID_STRIDE(i, n) {
    int64_t off[2];
    nd_off<2>(d, i, off);
    dst[off[0]] = conv<To>(src[off[1]]);
  }
}

enum BinOp : int {
  B_ADD = 0, B_SUB = 1, B_MUL = 2, B_DIV = 3, B_POW = 4, B_MAX = 5, B_MIN = 6,
  B_LT = 7, B_LE = 8, B_GT = 9, B_GE = 10, B_EQ = 11, B_NE = 12, B_AND = 13, B_OR = 14, B_XOR = 15
};

__device__ __forceinline__ float bin_f(int op, float a, float b) {
  switch (op) {
    case B_ADD: return a + b;
    case B_SUB: return a - b;
    case B_MUL: return a * b;
    case B_DIV: return a / b;
    case B_POW: return powf(a, b);
    case B_MAX: return fmaxf(a, b);
    case B_MIN: return fminf(a, b);
    case B_LT: return a < b ? 1.f : 0.f;
    case B_LE: return a <= b ? 1.f : 0.f;
    case B_GT: return a > b ? 1.f : 0.f;
    case B_GE: return a >= b ? 1.f : 0.f;
    case B_EQ: return a == b ? 1.f : 0.f;
    case B_NE: return a != b ? 1.f : 0.f;
    case B_AND: return (a != 0.f && b != 0.f) ? 1.f : 0.f;
    case B_OR: return (a != 0.f || b != 0.f) ? 1.f : 0.f;
    case B_XOR: return ((a != 0.f) != (b != 0.f)) ? 1.f : 0.f;
  }
  return 0.f;
}

// out = alpha * (a OP b): alpha folds the scalar factors of an operator's backward
template <typename T>
__global__ void binary_nd_k(int op, const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ out,
                            const Nd d, int64_t n, float alpha) {
  SG_GRID_STRIDE(i, n) {
    int64_t off[3];
    nd_off<3>(d, i, off);
    out[off[0]] = cvt_to<T>(alpha * bin_f(op, ld_f(a + off[1]), ld_f(b + off[2])));
  }
}

template <typename T>
__global__ void where_nd_k(const uint8_t* __restrict__ c, const T* __restrict__ a, const T* __restrict__ b,
                           T* __restrict__ out, const Nd d, int64_t n) {
  SG_GRID_STRIDE(i, n) {
    int64_t off[4];
    nd_off<4>(d, i, off);
    out[off[0]] = c[off[3]] ? a[off[1]] : b[off[2]];
  }
}

enum RedOp : int { R_SUM = 0, R_MEAN = 1, R_MAX = 2, R_MIN = 3, R_SUMSQ = 4 };

__device__ __forceinline__ float red_init(int op) {
  return op == R_MAX ? -INFINITY : op == R_MIN ? INFINITY : 0.f;
}
__device__ __forceinline__ float red_acc(int op, float acc, float v) {
  switch (op) {
    case R_MAX: return fmaxf(acc, v);
    case R_MIN: return fminf(acc, v);
    case R_SUMSQ: return acc + v * v;
    default: return acc + v;
  }
}
__device__ __forceinline__ float red_comb(int op, float a, float b) {
  return op == R_MAX ? fmaxf(a, b) : op == R_MIN ? fminf(a, b) : a + b;
}

// inner == 1: one 256-thread block per row (grid-stride over rows).
// parts > 1 (sum-type ops, fp32 out pre-zeroed): each row split over `parts`
// blocks that add their partial sums atomically.
template <typename T, typename OT>
__global__ void __launch_bounds__(256) reduce_rows_k(const T* __restrict__ x, OT* __restrict__ y, int64_t rows,
                                                     int64_t red, int op, float scale, int parts) {
  __shared__ float sh[8];
  const int64_t per = (red + parts - 1) / parts;
  for (int64_t bid = blockIdx.x; bid < rows * parts; bid += gridDim.x) {
    const int64_t r = bid / parts, part = bid - r * parts;
    const int64_t lo = part * per, hi = min(red, lo + per);
    const T* xr = x + r * red;
    float acc = red_init(op);
    for (int64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) acc = red_acc(op, acc, (float)xr[j]);
    // block combine
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc = red_comb(op, acc, __shfl_xor(acc, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = sh[0];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) t = red_comb(op, t, sh[w]);
      if (parts > 1) atomicAdd((float*)y + r, t * scale);
      else y[r] = cvt_to<OT>(op == R_MAX || op == R_MIN ? t : t * scale);
    }
  }
}

// inner > 1: one thread per (outer, inner) output walking the reduced dim
template <typename T, typename OT>
__global__ void reduce_cols_k(const T* __restrict__ x, OT* __restrict__ y, int64_t outer, int64_t red, int64_t inner,
                              int op, float scale) {
  SG_GRID_STRIDE(e, outer * inner) {
    const int64_t o = e / inner, k = e - o * inner;
    const T* p = x + o * red * inner + k;
    float acc = red_init(op);
    for (int64_t j = 0; j < red; ++j) acc = red_acc(op, acc, (float)p[j * inner]);
    y[e] = cvt_to<OT>(op == R_MAX || op == R_MIN ? acc : acc * scale);
  }
}

// dst[o][j][k] = src[o][idx[j]][k]  (units of V: 16-byte vectors when the rows allow)
template <typename V, typename I>
__global__ void index_select_k(const V* __restrict__ src, const I* __restrict__ idx, V* __restrict__ dst,
                               int64_t outer, int64_t nsrc, int64_t inner, int64_t nidx) {
  SG_GRID_STRIDE(e, outer * nidx * inner) {
    const int64_t k = e % inner, oj = e / inner;
    const int64_t j = oj % nidx, o = oj / nidx;
    int64_t r = (int64_t)idx[j];
    r = r < 0 ? r + nsrc : r;
    r = r < 0 ? 0 : (r >= nsrc ? nsrc - 1 : r);  // clamp out-of-range ids (no fault)
    dst[e] = src[(o * nsrc + r) * inner + k];
  }
}

// dst[o][idx[j]][k] += alpha * src[o][j][k]   (fp32 dst, atomics)
template <typename T, typename I>
__global__ void index_add_k(float* __restrict__ dst, const I* __restrict__ idx, const T* __restrict__ src,
                            int64_t outer, int64_t ndst, int64_t inner, int64_t nidx, float alpha) {
  SG_GRID_STRIDE(e, outer * nidx * inner) {
    const int64_t k = e % inner, oj = e / inner;
    const int64_t j = oj % nidx, o = oj / nidx;
    int64_t r = (int64_t)idx[j];
    r = r < 0 ? r + ndst : r;
    if (r >= 0 && r < ndst) atomicAdd(dst + (o * ndst + r) * inner + k, alpha * (float)src[e]);
  }
}

// GatherElements: out[o][j][k] = src[o][idx[o][j][k]][k]; ScatterElements
// (mode 0 assign, 1 add into fp32): dst[o][idx[o][j][k]][k] = upd[o][j][k]
template <typename T, typename I>
__global__ void gather_el_k(const T* __restrict__ src, const I* __restrict__ idx, T* __restrict__ out, int64_t outer,
                            int64_t nsrc, int64_t nidx, int64_t inner) {
  SG_GRID_STRIDE(e, outer * nidx * inner) {
    const int64_t k = e % inner, o = e / (inner * nidx);
    int64_t r = (int64_t)idx[e];
    r = r < 0 ? r + nsrc : r;
    r = r < 0 ? 0 : (r >= nsrc ? nsrc - 1 : r);
    out[e] = src[(o * nsrc + r) * inner + k];
  }
}
template <typename T, typename I>
__global__ void scatter_el_k(T* __restrict__ dst, const I* __restrict__ idx, const T* __restrict__ upd, int64_t outer,
                             int64_t ndst, int64_t nidx, int64_t inner, int add) {
  SG_GRID_STRIDE(e, outer * nidx * inner) {
    const int64_t k = e % inner, o = e / (inner * nidx);
    int64_t r = (int64_t)idx[e];
    r = r < 0 ? r + ndst : r;
    if (r < 0 || r >= ndst) continue;
    T* p = dst + (o * ndst + r) * inner + k;
    if (add) {
      if constexpr (sizeof(T) == 4) atomicAdd((float*)p, (float)upd[e]);
    } else {
      *p = upd[e];
    }
  }
}

struct PadGeom {
  int nd, mode;  // 0 constant, 1 reflect, 2 edge
  int64_t osz[MAXD], isz[MAXD], before[MAXD], ist[MAXD];
};

__device__ __forceinline__ bool pad_map(int mode, int64_t o, int64_t before, int64_t n, int64_t& i) {
  i = o - before;
  if (i >= 0 && i < n) return true;
  if (mode == 0) return false;
  if (mode == 2) {
    i = i < 0 ? 0 : n - 1;
    return true;
  }
  // reflect (no edge repeat), period 2(n-1)
  if (n == 1) {
    i = 0;
    return true;
  }
  const int64_t p = 2 * (n - 1);
  int64_t m = i % p;
  m = m < 0 ? m + p : m;
  i = m < n ? m : p - m;
  return true;
}

template <typename T>
__global__ void pad_nd_k(const T* __restrict__ x, T* __restrict__ y, const PadGeom g, int64_t n, float value) {
  SG_GRID_STRIDE(e, n) {
    int64_t rem = e, off = 0;
    bool inside = true;
    for (int k = g.nd - 1; k >= 0; --k) {
      const int64_t q = rem / g.osz[k];
      const int64_t o = rem - q * g.osz[k];
      rem = q;
      int64_t i;
      inside = inside && pad_map(g.mode, o, g.before[k], g.isz[k], i);
      off += (inside ? i : 0) * g.ist[k];
    }
    y[e] = inside ? x[off] : cvt_to<T>(value);
  }
}
// gradient of pad_nd: dx (fp32, zeroed, dense) += dy at the mapped input element
template <typename T>
__global__ void pad_bwd_k(const T* __restrict__ dy, float* __restrict__ dx, const PadGeom g, int64_t n) {
  SG_GRID_STRIDE(e, n) {
    int64_t rem = e, off = 0;
    bool inside = true;
    for (int k = g.nd - 1; k >= 0; --k) {
      const int64_t q = rem / g.osz[k];
      const int64_t o = rem - q * g.osz[k];
      rem = q;
      int64_t i;
      inside = inside && pad_map(g.mode, o, g.before[k], g.isz[k], i);
      off += (inside ? i : 0) * g.ist[k];
    }
    if (inside) atomicAdd(dx + off, (float)dy[e]);
  }
}

// ---- k-th largest |x| by radix select on the float bits (exact, on device,
// no host synchronisation: the sparse-gradient threshold of DistOpt's top-K
// exchange, replacing a full sort / kthvalue of the gradient every step).
// Three histogram passes over bits [31:21], [20:10], [9:0] of |x| (the sign
// cleared, non-negative floats order as unsigned ints); after each pass one
// thread walks the bins from the top and fixes those bits of the answer.
struct KthState {
  uint32_t prefix;  // bits of the answer fixed so far
  uint32_t k;       // rank still to find inside the current prefix (1 = largest)
};
__global__ void kth_init_k(KthState* st, uint32_t* hist, uint32_t k) {
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) hist[i] = 0;
  if (threadIdx.x == 0) {
    st->prefix = 0;
    st->k = k;
  }
}
__global__ void __launch_bounds__(256) kth_hist_k(const float* __restrict__ x, int64_t n, const KthState* st,
                                                  int pass, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[2048];
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int shift = pass == 0 ? 21 : pass == 1 ? 10 : 0;
  const uint32_t bmask = pass == 2 ? 0x3FFu : 0x7FFu;
  const uint32_t pmask = pass == 0 ? 0u : pass == 1 ? 0xFFE00000u : 0xFFFFFC00u;
  const uint32_t pre = st->prefix & pmask;
  SG_GRID_STRIDE(i, n) {
    const uint32_t b = __float_as_uint(x[i]) & 0x7FFFFFFFu;
    if ((b & pmask) == pre) atomicAdd(&h[(b >> shift) & bmask], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}
__global__ void kth_select_k(KthState* st, uint32_t* hist, int pass, float* out) {
  if (threadIdx.x == 0) {
    const int shift = pass == 0 ? 21 : pass == 1 ? 10 : 0;
    const int nb = pass == 2 ? 1024 : 2048;
    uint32_t k = st->k, cum = 0;
    int sel = 0;
    for (int b = nb - 1; b >= 0; --b) {
      if (cum + hist[b] >= k) {
        sel = b;
        break;
      }
      cum += hist[b];
    }
    st->prefix |= (uint32_t)sel << shift;
    st->k = k - cum;
    if (pass == 2) *out = __uint_as_float(st->prefix);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) hist[i] = 0;  // ready for the next pass
}

__global__ void iadd_i64_k(int64_t* __restrict__ p, int64_t n, int64_t v) {
  SG_GRID_STRIDE(i, n) { p[i] += v; }
}

template <typename T>
__global__ void fill_k(T* __restrict__ p, int64_t n, T v) {
  SG_GRID_STRIDE(i, n) { p[i] = v; }
}

// y = clamp(a*x + b, lo, hi); backward dx = dy * a inside (lo, hi)
template <typename T>
__global__ void clamp_affine_k(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ out, int64_t n,
                               float a, float b, float lo, float hi) {
  SG_GRID_STRIDE(i, n) {
    const float z = a * (float)x[i] + b;
    if (dy) out[i] = cvt_to<T>((z > lo && z < hi) ? a * (float)dy[i] : 0.f);
    else out[i] = cvt_to<T>(fminf(fmaxf(z, lo), hi));
  }
}

}  // namespace sg

using namespace sg;

namespace {

// host: build an Nd from sizes + per-operand strides (already coalesced)
Nd make_nd(int nd, const int64_t* size, const int64_t* const* st, int nop) {
  if (nd > MAXD || nd < 0) throw std::runtime_error("glue: too many dimensions");
  Nd d{};
  d.nd = nd;
  int64_t total = 1;
  bool small = true;
  for (int k = 0; k < nd; ++k) {
    d.size[k] = size[k];
    total *= size[k];
    small = small && size[k] > 0 && size[k] < ((int64_t)1 << 31);
    d.dv[k] = FastDiv((uint32_t)(size[k] > 0 ? (size[k] < ((int64_t)1 << 31) ? size[k] : 1) : 1));
    for (int o = 0; o < nop; ++o) d.st[o][k] = st[o][k];
  }
  d.small = small && total < ((int64_t)1 << 31);
  return d;
}

int64_t numel(int nd, const int64_t* size) {
  int64_t n = 1;
  for (int k = 0; k < nd; ++k) n *= size[k];
  return n;
}

template <typename Ti>
void copy_to(int dto, const Ti* src, void* dst, const Nd& d, int64_t n, hipStream_t s) {
  dim3 g(sg_grid(n, 256, 8192)), b(256);
  switch (dto) {
    case kF32: hipLaunchKernelGGL((copy_nd_k<Ti, float>), g, b, 0, s, src, (float*)dst, d, n); break;
    case kBF16: hipLaunchKernelGGL((copy_nd_k<Ti, bf16>), g, b, 0, s, src, (bf16*)dst, d, n); break;
    case kI32: hipLaunchKernelGGL((copy_nd_k<Ti, int32_t>), g, b, 0, s, src, (int32_t*)dst, d, n); break;
    case kI64: hipLaunchKernelGGL((copy_nd_k<Ti, int64_t>), g, b, 0, s, src, (int64_t*)dst, d, n); break;
    case kU8: hipLaunchKernelGGL((copy_nd_k<Ti, uint8_t>), g, b, 0, s, src, (uint8_t*)dst, d, n); break;
    case kF16: hipLaunchKernelGGL((copy_nd_k<Ti, uint16_t>), g, b, 0, s, src, (uint16_t*)dst, d, n); break;
    default: throw std::runtime_error("copy_nd: unsupported output dtype");
  }
}

}  // namespace

extern "C" {

// dst (dtype dto, strides dst_st) = src (dtype dti, strides src_st) over `size`
void sg_copy_nd(const void* src, int dti, void* dst, int dto, int nd, const int64_t* size, const int64_t* dst_st,
                const int64_t* src_st, hipStream_t s) {
  const int64_t* st[2] = {dst_st, src_st};
  const Nd d = make_nd(nd, size, st, 2);
  const int64_t n = numel(nd, size);
  if (n <= 0) return;
  if (dti == kF16 || dto == kF16) {  // raw 16-bit moves only (no f16 arithmetic here)
    if (dti != dto) throw std::runtime_error("copy_nd: fp16 conversion unsupported");
    hipLaunchKernelGGL((copy_nd_k<uint16_t, uint16_t>), dim3(sg_grid(n, 256, 8192)), dim3(256), 0, s,
                       (const uint16_t*)src, (uint16_t*)dst, d, n);
    return;
  }
  switch (dti) {
    case kF32: copy_to(dto, (const float*)src, dst, d, n, s); break;
    case kBF16: copy_to(dto, (const bf16*)src, dst, d, n, s); break;
    case kI32: copy_to(dto, (const int32_t*)src, dst, d, n, s); break;
    case kI64: copy_to(dto, (const int64_t*)src, dst, d, n, s); break;
    case kU8: copy_to(dto, (const uint8_t*)src, dst, d, n, s); break;
    default: throw std::runtime_error("copy_nd: unsupported input dtype");
  }
}

void sg_binary_nd(int op, const void* a, const void* b, void* out, int dt, int nd, const int64_t* size,
                  const int64_t* out_st, const int64_t* a_st, const int64_t* b_st, float alpha, hipStream_t s) {
  const int64_t* st[3] = {out_st, a_st, b_st};
  const Nd d = make_nd(nd, size, st, 3);
  const int64_t n = numel(nd, size);
  if (n <= 0) return;
  dim3 g(sg_grid(n, 256, 8192)), bl(256);
  if (dt == kF32) hipLaunchKernelGGL(binary_nd_k<float>, g, bl, 0, s, op, (const float*)a, (const float*)b,
                                     (float*)out, d, n, alpha);
  else if (dt == kBF16) hipLaunchKernelGGL(binary_nd_k<bf16>, g, bl, 0, s, op, (const bf16*)a, (const bf16*)b,
                                           (bf16*)out, d, n, alpha);
  else throw std::runtime_error("binary_nd: fp32 / bf16 only");
}

void sg_where_nd(const void* c, const void* a, const void* b, void* out, int dt, int nd, const int64_t* size,
                 const int64_t* out_st, const int64_t* a_st, const int64_t* b_st, const int64_t* c_st,
                 hipStream_t s) {
  const int64_t* st[4] = {out_st, a_st, b_st, c_st};
  const Nd d = make_nd(nd, size, st, 4);
  const int64_t n = numel(nd, size);
  if (n <= 0) return;
  dim3 g(sg_grid(n, 256, 8192)), bl(256);
  if (dt == kF32) hipLaunchKernelGGL(where_nd_k<float>, g, bl, 0, s, (const uint8_t*)c, (const float*)a,
                                     (const float*)b, (float*)out, d, n);
  else if (dt == kBF16) hipLaunchKernelGGL(where_nd_k<bf16>, g, bl, 0, s, (const uint8_t*)c, (const bf16*)a,
                                           (const bf16*)b, (bf16*)out, d, n);
  else if (dt == kI64) hipLaunchKernelGGL(where_nd_k<int64_t>, g, bl, 0, s, (const uint8_t*)c, (const int64_t*)a,
                                          (const int64_t*)b, (int64_t*)out, d, n);
  else throw std::runtime_error("where_nd: fp32 / bf16 / int64 only");
}

// y[outer][inner] = op over j of x[outer][j][inner] (x dense); out dtype dto.
// Sum-type ops over one long row run split across blocks with fp32 atomics
// (the output is zeroed here).
void sg_reduce(const void* x, int dti, void* y, int dto, int64_t outer, int64_t red, int64_t inner, int op,
               hipStream_t s) {
  if (outer * inner <= 0) return;
  const float scale = op == R_MEAN ? 1.f / (float)(red > 0 ? red : 1) : 1.f;
  if (inner == 1) {
    int parts = 1;
    if (outer < 64 && red >= 65536 && (op == R_SUM || op == R_MEAN || op == R_SUMSQ) && dto == kF32) {
      parts = (int)std::min<int64_t>(1024 / outer + 1, red / 16384);
      sg_zero_async(y, outer * sizeof(float), s);
    }
    dim3 g((unsigned)std::min<int64_t>(outer * parts, 65535)), b(256);
#define RR(TI, TO) hipLaunchKernelGGL((reduce_rows_k<TI, TO>), g, b, 0, s, (const TI*)x, (TO*)y, outer, red, op, scale, parts)
    if (dti == kF32 && dto == kF32) RR(float, float);
    else if (dti == kBF16 && dto == kF32) RR(bf16, float);
    else if (dti == kBF16 && dto == kBF16) RR(bf16, bf16);
    else if (dti == kF32 && dto == kBF16) RR(float, bf16);
    else throw std::runtime_error("reduce: fp32 / bf16 only");
#undef RR
    return;
  }
  dim3 g(sg_grid(outer * inner, 256, 8192)), b(256);
#define RC(TI, TO) hipLaunchKernelGGL((reduce_cols_k<TI, TO>), g, b, 0, s, (const TI*)x, (TO*)y, outer, red, inner, op, scale)
  if (dti == kF32 && dto == kF32) RC(float, float);
  else if (dti == kBF16 && dto == kF32) RC(bf16, float);
  else if (dti == kBF16 && dto == kBF16) RC(bf16, bf16);
  else if (dti == kF32 && dto == kBF16) RC(float, bf16);
  else throw std::runtime_error("reduce: fp32 / bf16 only");
#undef RC
}

void sg_index_select(const void* src, const void* idx, int idx64, void* dst, int64_t outer, int64_t nsrc, int64_t inner,
                     int64_t nidx, int esize, hipStream_t s) {
  const int64_t rb = inner * esize;
  const bool v16 = rb % 16 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0;
  const bool v4 = !v16 && rb % 4 == 0 && (uintptr_t)src % 4 == 0 && (uintptr_t)dst % 4 == 0;
  const int64_t u = v16 ? 16 : v4 ? 4 : esize;
  const int64_t in_u = rb / u;
  dim3 g(sg_grid(outer * nidx * in_u, 256, 8192)), b(256);
#define IS(V, I) hipLaunchKernelGGL((index_select_k<V, I>), g, b, 0, s, (const V*)src, (const I*)idx, (V*)dst, outer, nsrc, in_u, nidx)
#define IS2(V) { if (idx64) IS(V, int64_t); else IS(V, int32_t); }
  if (u == 16) IS2(uint4)
  else if (u == 4) IS2(uint32_t)
  else if (u == 2) IS2(uint16_t)
  else if (u == 8) IS2(uint64_t)
  else IS2(uint8_t)
#undef IS2
#undef IS
}

void sg_index_add(void* dst, const void* idx, int idx64, const void* src, int dts, int64_t outer, int64_t ndst,
                  int64_t inner, int64_t nidx, float alpha, hipStream_t s) {
  dim3 g(sg_grid(outer * nidx * inner, 256, 8192)), b(256);
#define IA(T, I) hipLaunchKernelGGL((index_add_k<T, I>), g, b, 0, s, (float*)dst, (const I*)idx, (const T*)src, outer, ndst, inner, nidx, alpha)
  if (dts == kF32) { if (idx64) IA(float, int64_t); else IA(float, int32_t); }
  else if (dts == kBF16) { if (idx64) IA(bf16, int64_t); else IA(bf16, int32_t); }
  else throw std::runtime_error("index_add: fp32 / bf16 source only");
#undef IA
}

void sg_gather_el(const void* src, const void* idx, int idx64, void* out, int dt, int64_t outer, int64_t nsrc,
                  int64_t nidx, int64_t inner, hipStream_t s) {
  dim3 g(sg_grid(outer * nidx * inner, 256, 8192)), b(256);
#define GE(T) { if (idx64) hipLaunchKernelGGL((gather_el_k<T, int64_t>), g, b, 0, s, (const T*)src, (const int64_t*)idx, (T*)out, outer, nsrc, nidx, inner); \
                else hipLaunchKernelGGL((gather_el_k<T, int32_t>), g, b, 0, s, (const T*)src, (const int32_t*)idx, (T*)out, outer, nsrc, nidx, inner); }
  if (dt == kF32) GE(float) else if (dt == kBF16) GE(bf16) else if (dt == kI64) GE(int64_t) else GE(int32_t)
#undef GE
}

void sg_scatter_el(void* dst, const void* idx, int idx64, const void* upd, int dt, int64_t outer, int64_t ndst,
                   int64_t nidx, int64_t inner, int add, hipStream_t s) {
  if (add && dt != kF32) throw std::runtime_error("scatter_el: accumulation needs fp32");
  dim3 g(sg_grid(outer * nidx * inner, 256, 8192)), b(256);
#define SE(T) { if (idx64) hipLaunchKernelGGL((scatter_el_k<T, int64_t>), g, b, 0, s, (T*)dst, (const int64_t*)idx, (const T*)upd, outer, ndst, nidx, inner, add); \
                else hipLaunchKernelGGL((scatter_el_k<T, int32_t>), g, b, 0, s, (T*)dst, (const int32_t*)idx, (const T*)upd, outer, ndst, nidx, inner, add); }
  if (dt == kF32) SE(float) else if (dt == kBF16) SE(bf16) else if (dt == kI64) SE(int64_t) else SE(int32_t)
#undef SE
}

// y (dense, out sizes) = pad(x (sizes isz, strides ist)); mode 0 constant / 1 reflect / 2 edge
void sg_pad_nd(const void* x, void* y, int dt, int nd, const int64_t* osz, const int64_t* isz, const int64_t* ist,
               const int64_t* before, int mode, float value, hipStream_t s) {
  if (nd > MAXD) throw std::runtime_error("pad: too many dimensions");
  PadGeom g{};
  g.nd = nd;
  g.mode = mode;
  for (int k = 0; k < nd; ++k) { g.osz[k] = osz[k]; g.isz[k] = isz[k]; g.ist[k] = ist[k]; g.before[k] = before[k]; }
  const int64_t n = numel(nd, osz);
  if (n <= 0) return;
  dim3 gr(sg_grid(n, 256, 8192)), b(256);
  if (dt == kF32) hipLaunchKernelGGL(pad_nd_k<float>, gr, b, 0, s, (const float*)x, (float*)y, g, n, value);
  else if (dt == kBF16) hipLaunchKernelGGL(pad_nd_k<bf16>, gr, b, 0, s, (const bf16*)x, (bf16*)y, g, n, value);
  else throw std::runtime_error("pad: fp32 / bf16 only");
}

// dx (fp32, zeroed by the caller, dense with strides ist) += gradient of pad_nd from dy (dense, out sizes)
void sg_pad_bwd(const void* dy, void* dx, int dt, int nd, const int64_t* osz, const int64_t* isz, const int64_t* ist,
                const int64_t* before, int mode, hipStream_t s) {
  PadGeom g{};
  g.nd = nd;
  g.mode = mode;
  for (int k = 0; k < nd; ++k) { g.osz[k] = osz[k]; g.isz[k] = isz[k]; g.ist[k] = ist[k]; g.before[k] = before[k]; }
  const int64_t n = numel(nd, osz);
  if (n <= 0) return;
  dim3 gr(sg_grid(n, 256, 8192)), b(256);
  if (dt == kF32) hipLaunchKernelGGL(pad_bwd_k<float>, gr, b, 0, s, (const float*)dy, (float*)dx, g, n);
  else if (dt == kBF16) hipLaunchKernelGGL(pad_bwd_k<bf16>, gr, b, 0, s, (const bf16*)dy, (float*)dx, g, n);
  else throw std::runtime_error("pad_bwd: fp32 / bf16 only");
}

void sg_fill(void* p, int64_t n, int dt, double v, hipStream_t s) {
  if (n <= 0) return;
  dim3 g(sg_grid(n, 256, 8192)), b(256);
  switch (dt) {
    case kF32: hipLaunchKernelGGL(fill_k<float>, g, b, 0, s, (float*)p, n, (float)v); break;
    case kBF16: hipLaunchKernelGGL(fill_k<bf16>, g, b, 0, s, (bf16*)p, n, (bf16)(float)v); break;
    case kI32: hipLaunchKernelGGL(fill_k<int32_t>, g, b, 0, s, (int32_t*)p, n, (int32_t)v); break;
    case kI64: hipLaunchKernelGGL(fill_k<int64_t>, g, b, 0, s, (int64_t*)p, n, (int64_t)v); break;
    case kU8: hipLaunchKernelGGL(fill_k<uint8_t>, g, b, 0, s, (uint8_t*)p, n, (uint8_t)v); break;
    default: throw std::runtime_error("fill: unsupported dtype");
  }
}

// out[0] = the k-th largest |x[i]| (1 <= k <= n); ws: >= 2048 + 2 uint32 of scratch
void sg_kth_largest_abs(const void* x, int64_t n, int64_t k, void* out, void* ws, hipStream_t s) {
  if (n <= 0) return;
  if (k < 1) k = 1;
  if (k > n) k = n;
  uint32_t* hist = (uint32_t*)ws;
  KthState* st = (KthState*)(hist + 2048);
  hipLaunchKernelGGL(kth_init_k, dim3(1), dim3(256), 0, s, st, hist, (uint32_t)k);
  for (int pass = 0; pass < 3; ++pass) {
    hipLaunchKernelGGL(kth_hist_k, dim3(sg_grid(n, 256, 2048)), dim3(256), 0, s, (const float*)x, n, st, pass, hist);
    hipLaunchKernelGGL(kth_select_k, dim3(1), dim3(256), 0, s, st, hist, pass, (float*)out);
  }
}

// p[i] += v on int64 counters (the device RNG epoch a captured step advances)
void sg_iadd_i64(void* p, int64_t n, int64_t v, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(iadd_i64_k, dim3(sg_grid(n, 64, 64)), dim3(64), 0, s, (int64_t*)p, n, v);
}

void sg_clamp_affine(const void* x, const void* dy, void* out, int64_t n, int dt, float a, float b, float lo, float hi,
                     hipStream_t s) {
  if (n <= 0) return;
  dim3 g(sg_grid(n, 256, 8192)), bl(256);
  if (dt == kF32) hipLaunchKernelGGL(clamp_affine_k<float>, g, bl, 0, s, (const float*)x, (const float*)dy,
                                     (float*)out, n, a, b, lo, hi);
  else hipLaunchKernelGGL(clamp_affine_k<bf16>, g, bl, 0, s, (const bf16*)x, (const bf16*)dy, (bf16*)out, n, a, b,
                          lo, hi);
}

}  // extern "C"

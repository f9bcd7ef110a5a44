// Shared device helpers for the singa_amd gfx950 (CDNA4) kernel library.
//
// Everything here is written for wave64 / MI355X only: lane masks are 64-bit,
// reductions use 64-wide shuffles (the reference's 32-wide warp-synchronous
// reduction idiom, include/mshadow/cuda/cuda_reduce.cuh:40-112, is deliberately
// NOT reproduced), and bf16 is handled through clang's native __bf16 type so
// that hipcc emits v_cvt_pk_bf16_f32 for conversions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sg {

constexpr int kWave = 64;

typedef __bf16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

// dtype codes shared with the python side (singa_amd/ops/native.py)
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kI32 = 3, kI64 = 4, kU8 = 5 };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// Wave-wide all-reduce (every lane active): DPP within each 16-lane row
// (quad_perm xor 1, xor 2, row_half_mirror, row_mirror), then the four row
// results by readlane -- VALU-only, ~10x shorter than the six ds_bpermute
// round trips of a shfl_xor butterfly (which dominated the wave-per-row
// LayerNorm / softmax kernels).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  v += dpp_f<0x141>(v);  // row_half_mirror: the other quad of each 8
  v += dpp_f<0x140>(v);  // row_mirror: the other half of each 16
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// Block-wide sum; `sh` must hold >= blockDim.x/64 floats. Result broadcast.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, sh[i]);
  return t;
}

// Philox4x32-10 counter-based RNG (reproducible per (seed, offset)).
struct Philox {
  __device__ static inline uint4 round(uint4 c, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
  }
  __device__ static inline uint4 gen(uint64_t seed, uint64_t counter, uint32_t sub) {
    uint4 c = make_uint4((uint32_t)counter, (uint32_t)(counter >> 32), sub, 0u);
    uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c = round(c, k);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    return c;
  }
  __device__ static inline float u01(uint32_t x) {  // (0,1]
    return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
  }
};

// Fast unsigned division by a runtime constant (Granlund-Montgomery style),
// used by implicit-GEMM loaders to split flat pixel indices without v_div.
struct FastDiv {
  uint32_t d, m, s;
  __host__ __device__ FastDiv() : d(1), m(0), s(0) {}
  __host__ FastDiv(uint32_t div) : d(div) {
    s = 0;
    while ((1u << s) < div) ++s;
    uint64_t one = 1;
    m = (uint32_t)(((one << 32) * ((one << s) - div)) / div + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (uint32_t)(((uint64_t)__umulhi(n, m) + n) >> s);
  }
};

// V-wide (8 x 16-bit or 8 x fp32, or scalar) vector loads/stores to fp32 regs
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
// Non-temporal variants for the HBM-streaming passes (BatchNorm apply):
// tensors far larger than the caches, read or written exactly once
template <typename T, int V>
__device__ __forceinline__ void ldv_nt(const T* p, float* v) {
  if constexpr (V == 8 && sizeof(T) == 2) {
    bf16x8 t = __builtin_nontemporal_load((const bf16x8*)p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)t[i];
  } else if constexpr (V == 8) {
    typedef float nt4 __attribute__((ext_vector_type(4)));
    nt4 a = __builtin_nontemporal_load((const nt4*)p), b = __builtin_nontemporal_load((const nt4*)(p + 4));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[4 + i] = b[i];
    }
  } else {
    ldv<T, V>(p, v);
  }
}
template <typename T, int V>
__device__ __forceinline__ void stv_nt(T* p, const float* v) {
  if constexpr (V == 8 && sizeof(T) == 2) {
    bf16x8 t;
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = (bf16)v[i];
    __builtin_nontemporal_store(t, (bf16x8*)p);
  } else if constexpr (V == 8) {
    typedef float nt4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(nt4{v[0], v[1], v[2], v[3]}, (nt4*)p);
    __builtin_nontemporal_store(nt4{v[4], v[5], v[6], v[7]}, (nt4*)(p + 4));
  } else {
    stv<T, V>(p, v);
  }
}

template <int V>
__device__ __forceinline__ void ldc(const float* p, float* v) {
  if constexpr (V == 8) {
    float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = p[i];
  }
}

}  // namespace sg

#define SG_GRID_STRIDE(i, n) \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

static inline int sg_grid(int64_t n, int block = 256, int cap = 4096) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

// Zero a small device workspace with a kernel (16-byte stores).  Used instead
// of hipMemsetAsync for the atomic-accumulation slots, so the zeroing is an
// ordinary kernel node when the launch is captured into a hipGraph.
// SG_ZERO_MEMSET=1 switches back to hipMemsetAsync (diagnostics).
__global__ static void sg_zero_k(float4* __restrict__ p, int64_t n4) {
  SG_GRID_STRIDE(i, n4) { p[i] = make_float4(0.f, 0.f, 0.f, 0.f); }
}
static inline void sg_zero_async(void* p, size_t bytes, hipStream_t s) {
  static const int use_memset = [] {
    const char* e = getenv("SG_ZERO_MEMSET");
    return e && e[0] == '1';
  }();
  if (use_memset || (bytes & 15) || ((uintptr_t)p & 15)) {
    hipMemsetAsync(p, 0, bytes, s);
    return;
  }
  const int64_t n4 = (int64_t)(bytes / 16);
  hipLaunchKernelGGL(sg_zero_k, dim3(sg_grid(n4, 256, 1024)), dim3(256), 0, s, (float4*)p, n4);
}

// ------------------------------------------------------------------------------
// Dynamic work queue of the persistent kernels (sk_gemm_k, conv3x3_k,
// stem_fwd_k).  A persistent grid sized to the CU count with work split
// STATICALLY by blockIdx straggles as soon as some CUs are busy with other
// work (RCCL's channel kernels during the overlapped gradient all-reduce): a
// workgroup that starts late still owns its whole share.  Instead every
// workgroup takes its next unit from a device counter, so late starters take
// less.  A queue slot holds QMAX counters (one per independent unit sequence,
// e.g. per column slice and XCD), each on its own 64-byte line, and a
// done-counter; the last workgroup to finish resets the slot, so the next
// launch (or the next replay of a captured graph) starts from zero with no
// host work.  Eager launches take slots from a per-device ring
// (sg_workq_slot), so kernels running concurrently on different streams never
// share one; a thread that is capturing a HIP graph takes fresh slots from the
// capture's own arena (workq.hip), so a graph's frozen slots are never handed
// to other work while the graph can still be replayed.
// ------------------------------------------------------------------------------
constexpr int QSTRIDE = 16;                  // ints between counters (64 B)
constexpr int QMAX = 128;                    // counters per slot
constexpr int QSLOT = (QMAX + 1) * QSTRIDE;  // ints per slot (the done-counter last)

namespace sg {
// ticket of queue q (one lane calls it; agent-scope vector atomic)
__device__ __forceinline__ int wq_take(int* slot, int q) {
  return __hip_atomic_fetch_add(slot + q * QSTRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane per workgroup, after its last ticket: the last workgroup of the
// grid resets the slot's first nq counters and the done-counter
__device__ __forceinline__ void wq_done(int* slot, int nq) {
  const int total = (int)(gridDim.x * gridDim.y * gridDim.z);
  int* done = slot + QMAX * QSTRIDE;
  // every ticket this lane took has been PERFORMED before the done-count:
  // a kernel that takes tickets ahead can exit with one whose result it never
  // reads (stem_fwd_k), and the compiler does not wait for an unused return;
  // landing after the last workgroup's reset, it would leave the counter at
  // 1 for the next launch on this slot -- a skipped work unit
  __builtin_amdgcn_s_waitcnt(0);
  if (__hip_atomic_fetch_add(done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == total - 1) {
    for (int i = 0; i < nq; ++i)
      __hip_atomic_exchange(slot + i * QSTRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_exchange(done, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}
}  // namespace sg

extern "C" {
// a zeroed queue slot of the current device (nullptr: dynamic queues are
// switched off -- SG_WORKQ=0 / sg_workq_set(0) -- and the kernels fall back
// to the static blockIdx partition)
int* sg_workq_slot();
// compute units of the current device (cached)
int sg_cu_count();
}

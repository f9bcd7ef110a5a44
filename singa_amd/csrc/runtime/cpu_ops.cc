// CppCPU compute backend (see cpu_ops.h).  Reference: mshadow's CPU
// evaluation loops and its BLAS binding (include/mshadow/tensor_cpu-inl.hpp:52-165,
// include/mshadow/dot_engine-inl.hpp), the layer math of src/worker/layer.cc:18-764
// (convolution via unpack_patch2col + dot, pooling, LRN, softmax loss), and
// the Random<cpu> of include/mshadow/random.h.  Designed for a many-core host:
// a persistent worker pool, a packed AVX2/FMA GEMM micro-kernel, per-image
// parallel im2col convolution with fixed-order (deterministic) weight-gradient
// reduction, and row-parallel loss / normalisation kernels.
#include "cpu_ops.h"

#include <math.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace sgrt {
namespace cpu {

// ---------------------------------------------------------------- pool
namespace {

thread_local bool t_in_task = false;

class Pool {
 public:
  explicit Pool(int n) : nworkers_(std::max(0, n - 1)) {
    for (int i = 0; i < nworkers_; ++i) th_.emplace_back([this] { Worker(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_.store(true, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return nworkers_ + 1; }

  // Back-to-back parallel regions (a training step issues dozens) must not
  // pay a futex wake / sleep per worker each: workers spin on the job
  // generation for a short while after finishing a job and only then sleep
  // on the condition variable; the caller spins on the active count likewise.
  void Run(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& f) {
    if (n <= 0) return;
    grain = std::max<int64_t>(1, grain);
    if (nworkers_ == 0 || n <= grain || t_in_task || !busy_.try_lock()) {
      f(0, n);
      return;
    }
    int64_t nchunks = std::min<int64_t>((n + grain - 1) / grain, (int64_t)size() * 4);
    int64_t chunk = (n + nchunks - 1) / nchunks;
    job_ = &f;
    n_ = n;
    chunk_ = chunk;
    next_.store(0, std::memory_order_relaxed);
    active_.store(nworkers_, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(m_);  // a sleeper checks gen_ under m_: no lost wake-up
      gen_.fetch_add(1, std::memory_order_release);
    }
    if (sleepers_.load(std::memory_order_acquire) > 0) cv_.notify_all();
    t_in_task = true;
    Work(f, n, chunk);
    t_in_task = false;
    if (!SpinUntil([this] { return active_.load(std::memory_order_acquire) == 0; })) {
      std::unique_lock<std::mutex> g(m_);
      done_.wait(g, [this] { return active_.load(std::memory_order_acquire) == 0; });
    }
    job_ = nullptr;
    busy_.unlock();
  }

 private:
  template <typename P>
  bool SpinUntil(P&& pred) const {
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0;; ++it) {
      if (pred()) return true;
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
      if ((it & 63) == 63 && std::chrono::steady_clock::now() - t0 > spin_) return false;
    }
  }
  void Work(const std::function<void(int64_t, int64_t)>& f, int64_t n, int64_t chunk) {
    for (;;) {
      int64_t b = next_.fetch_add(chunk, std::memory_order_relaxed);
      if (b >= n) break;
      f(b, std::min(n, b + chunk));
    }
  }
  void Worker() {
    uint64_t seen = 0;
    for (;;) {
      if (!SpinUntil([&] { return stop_.load(std::memory_order_acquire) ||
                                  gen_.load(std::memory_order_acquire) != seen; })) {
        std::unique_lock<std::mutex> g(m_);
        sleepers_.fetch_add(1, std::memory_order_acq_rel);
        cv_.wait(g, [&] { return stop_.load(std::memory_order_acquire) ||
                                 gen_.load(std::memory_order_acquire) != seen; });
        sleepers_.fetch_sub(1, std::memory_order_acq_rel);
      }
      if (stop_.load(std::memory_order_acquire)) return;
      seen = gen_.load(std::memory_order_acquire);
      t_in_task = true;
      Work(*job_, n_, chunk_);
      t_in_task = false;
      if (active_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> g(m_);
        done_.notify_one();
      }
    }
  }

  static std::chrono::microseconds SpinBudget() {
    const char* v = getenv("SINGA_AMD_CPU_SPIN_US");
    return std::chrono::microseconds(v ? std::max(0, atoi(v)) : 200);
  }

  int nworkers_;
  std::vector<std::thread> th_;
  std::mutex m_, busy_;
  std::condition_variable cv_, done_;
  const std::function<void(int64_t, int64_t)>* job_ = nullptr;
  int64_t n_ = 0, chunk_ = 1;
  std::atomic<int64_t> next_{0};
  std::atomic<int> active_{0}, sleepers_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
  std::chrono::microseconds spin_ = SpinBudget();
};

int DefaultThreads() {
  for (const char* k : {"SINGA_AMD_CPU_THREADS", "OMP_NUM_THREADS"}) {
    const char* v = getenv(k);
    if (v && atoi(v) > 0) return atoi(v);
  }
  unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(h, 64u));
}

std::mutex g_pool_mu;
Pool* g_pool = nullptr;
pid_t g_pool_pid = 0;

Pool& GetPool() {
  std::lock_guard<std::mutex> g(g_pool_mu);
  // a forked child inherits the object but not the worker threads: the old
  // pool is abandoned (never joined) and a fresh one started
  if (!g_pool || g_pool_pid != getpid()) {
    g_pool = new Pool(DefaultThreads());
    g_pool_pid = getpid();
  }
  return *g_pool;
}

}  // namespace

void ParallelFor(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& f) {
  GetPool().Run(n, grain, f);
}
int NumThreads() { return GetPool().size(); }

// ---------------------------------------------------------------- GEMM
namespace {

constexpr int MR = 6, NR = 16, KC = 512;

void MicroScalar(const float* a, const float* b, int64_t kc, float* c) {
  float acc[MR][NR] = {};
  for (int64_t k = 0; k < kc; ++k, a += MR, b += NR)
    for (int r = 0; r < MR; ++r)
      for (int j = 0; j < NR; ++j) acc[r][j] += a[r] * b[j];
  memcpy(c, acc, sizeof(acc));
}

#if defined(__x86_64__)
__attribute__((target("avx2,fma"))) void MicroAvx2(const float* a, const float* b, int64_t kc, float* c) {
  __m256 c00 = _mm256_setzero_ps(), c01 = c00, c10 = c00, c11 = c00, c20 = c00, c21 = c00, c30 = c00, c31 = c00,
         c40 = c00, c41 = c00, c50 = c00, c51 = c00;
  for (int64_t k = 0; k < kc; ++k, a += MR, b += NR) {
    const __m256 b0 = _mm256_loadu_ps(b), b1 = _mm256_loadu_ps(b + 8);
    __m256 ar = _mm256_broadcast_ss(a + 0);
    c00 = _mm256_fmadd_ps(ar, b0, c00);
    c01 = _mm256_fmadd_ps(ar, b1, c01);
    ar = _mm256_broadcast_ss(a + 1);
    c10 = _mm256_fmadd_ps(ar, b0, c10);
    c11 = _mm256_fmadd_ps(ar, b1, c11);
    ar = _mm256_broadcast_ss(a + 2);
    c20 = _mm256_fmadd_ps(ar, b0, c20);
    c21 = _mm256_fmadd_ps(ar, b1, c21);
    ar = _mm256_broadcast_ss(a + 3);
    c30 = _mm256_fmadd_ps(ar, b0, c30);
    c31 = _mm256_fmadd_ps(ar, b1, c31);
    ar = _mm256_broadcast_ss(a + 4);
    c40 = _mm256_fmadd_ps(ar, b0, c40);
    c41 = _mm256_fmadd_ps(ar, b1, c41);
    ar = _mm256_broadcast_ss(a + 5);
    c50 = _mm256_fmadd_ps(ar, b0, c50);
    c51 = _mm256_fmadd_ps(ar, b1, c51);
  }
  _mm256_storeu_ps(c + 0, c00);
  _mm256_storeu_ps(c + 8, c01);
  _mm256_storeu_ps(c + 16, c10);
  _mm256_storeu_ps(c + 24, c11);
  _mm256_storeu_ps(c + 32, c20);
  _mm256_storeu_ps(c + 40, c21);
  _mm256_storeu_ps(c + 48, c30);
  _mm256_storeu_ps(c + 56, c31);
  _mm256_storeu_ps(c + 64, c40);
  _mm256_storeu_ps(c + 72, c41);
  _mm256_storeu_ps(c + 80, c50);
  _mm256_storeu_ps(c + 88, c51);
}
#endif

typedef void (*MicroFn)(const float*, const float*, int64_t, float*);

MicroFn PickMicro() {
#if defined(__x86_64__)
  if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return MicroAvx2;
#endif
  return MicroScalar;
}

const MicroFn g_micro = PickMicro();

}  // namespace

void Gemm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A, int64_t lda, const float* B,
          int64_t ldb, float beta, float* C, int64_t ldc, const float* bias, bool relu) {
  if (M <= 0 || N <= 0) return;
  const int64_t mb = (M + MR - 1) / MR, nb = (N + NR - 1) / NR;
  if (K <= 0) {  // C = beta C + bias
    ParallelFor(M, std::max<int64_t>(1, 16384 / N), [&](int64_t m0, int64_t m1) {
      for (int64_t m = m0; m < m1; ++m)
        for (int64_t n = 0; n < N; ++n) {
          float v = beta != 0.f ? beta * C[m * ldc + n] : 0.f;
          if (bias) v += bias[n];
          C[m * ldc + n] = relu && v < 0.f ? 0.f : v;
        }
    });
    return;
  }
  const int64_t kc_max = std::min<int64_t>(K, KC);
  std::vector<float> ap((size_t)mb * MR * kc_max), bp((size_t)nb * NR * kc_max);
  // tiles: groups of row blocks x groups of column panels
  const int64_t RG = 8, CG = 4;
  const int64_t tr = (mb + RG - 1) / RG, tc = (nb + CG - 1) / CG;
  const double flops_per_kc = 2.0 * (double)M * (double)N;
  for (int64_t k0 = 0; k0 < K; k0 += KC) {
    const int64_t kc = std::min<int64_t>(KC, K - k0);
    const bool first = k0 == 0, last = k0 + kc >= K;
    const int64_t pgrain = flops_per_kc * kc < 2e6 ? 1 << 30 : 1;
    // pack op(A)[m][k0:k0+kc] -> ap[blk][k][MR]
    ParallelFor(mb, pgrain == 1 ? 4 : pgrain, [&](int64_t b0, int64_t b1) {
      for (int64_t blk = b0; blk < b1; ++blk) {
        float* dst = ap.data() + (size_t)blk * MR * kc;
        for (int r = 0; r < MR; ++r) {
          const int64_t m = blk * MR + r;
          if (m >= M) {
            for (int64_t k = 0; k < kc; ++k) dst[k * MR + r] = 0.f;
          } else if (ta) {
            const float* src = A + (k0)*lda + m;
            for (int64_t k = 0; k < kc; ++k) dst[k * MR + r] = src[k * lda];
          } else {
            const float* src = A + m * lda + k0;
            for (int64_t k = 0; k < kc; ++k) dst[k * MR + r] = src[k];
          }
        }
      }
    });
    // pack op(B)[k0:k0+kc][n] -> bp[panel][k][NR]
    ParallelFor(nb, pgrain == 1 ? 2 : pgrain, [&](int64_t p0, int64_t p1) {
      for (int64_t p = p0; p < p1; ++p) {
        float* dst = bp.data() + (size_t)p * NR * kc;
        const int64_t n0 = p * NR, nn = std::min<int64_t>(NR, N - n0);
        if (!tb) {
          for (int64_t k = 0; k < kc; ++k) {
            const float* src = B + (k0 + k) * ldb + n0;
            int64_t j = 0;
            for (; j < nn; ++j) dst[k * NR + j] = src[j];
            for (; j < NR; ++j) dst[k * NR + j] = 0.f;
          }
        } else {
          for (int64_t j = 0; j < NR; ++j) {
            if (j < nn) {
              const float* src = B + (n0 + j) * ldb + k0;
              for (int64_t k = 0; k < kc; ++k) dst[k * NR + j] = src[k];
            } else {
              for (int64_t k = 0; k < kc; ++k) dst[k * NR + j] = 0.f;
            }
          }
        }
      }
    });
    const int64_t tgrain = flops_per_kc * kc < 2e6 ? tr * tc : 1;
    ParallelFor(tr * tc, tgrain, [&](int64_t t0, int64_t t1) {
      alignas(32) float acc[MR * NR];
      for (int64_t t = t0; t < t1; ++t) {
        const int64_t gr = t / tc, gc = t % tc;
        for (int64_t p = gc * CG; p < std::min(nb, (gc + 1) * CG); ++p) {
          const float* bpp = bp.data() + (size_t)p * NR * kc;
          const int64_t n0 = p * NR, nn = std::min<int64_t>(NR, N - n0);
          for (int64_t blk = gr * RG; blk < std::min(mb, (gr + 1) * RG); ++blk) {
            g_micro(ap.data() + (size_t)blk * MR * kc, bpp, kc, acc);
            const int64_t m0 = blk * MR, mm = std::min<int64_t>(MR, M - m0);
            for (int64_t r = 0; r < mm; ++r) {
              float* c = C + (m0 + r) * ldc + n0;
              const float* a = acc + r * NR;
              for (int64_t j = 0; j < nn; ++j) {
                float v = alpha * a[j];
                if (first) {
                  if (beta != 0.f) v += beta * c[j];
                } else {
                  v += c[j];
                }
                if (last) {
                  if (bias) v += bias[n0 + j];
                  if (relu && v < 0.f) v = 0.f;
                }
                c[j] = v;
              }
            }
          }
        }
      }
    });
  }
}

// ---------------------------------------------------------------- unary
namespace {

inline float UnF(int op, float x, float a) {
  switch (op) {
    case 0: return x > 0.f ? x : 0.f;
    case 1: return 1.f / (1.f + expf(-x));
    case 2: return tanhf(x);
    case 3: return 1.7159047f * tanhf(0.66666667f * x);
    case 4: return 0.5f * x * (1.f + erff(x * 0.70710678118f));
    case 5: return x;
    case 6: return x > 20.f ? x : log1pf(expf(x));
    case 7: return x * x;
    case 8: return fabsf(x);
    case 9: return expf(x);
    case 10: return x > 0.f ? x : a * x;
    case 11: return x > 0.f ? x : a * (expf(x) - 1.f);
    case 12: {
      const float l = 1.0507009873554805f, al = 1.6732632423543772f;
      return x > 0.f ? l * x : l * al * (expf(x) - 1.f);
    }
    case 13: {
      const float u = 0.7978845608f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case 14: return sqrtf(x);
    case 15: return -x;
    case 16: return 1.f / x;
    case 17: return logf(x);
    case 18: return (float)((x > 0.f) - (x < 0.f));
    case 19: return erff(x);
    case 20: return cosf(x);
    case 21: return sinf(x);
    case 22: return tanf(x);
    case 23: return coshf(x);
    case 24: return sinhf(x);
    case 25: return acosf(x);
    case 26: return asinf(x);
    case 27: return atanf(x);
    case 28: return acoshf(x);
    case 29: return asinhf(x);
    case 30: return atanhf(x);
    case 31: return ceilf(x);
    case 32: return floorf(x);
    case 33: return rintf(x);
    case 34: return x / (1.f + fabsf(x));
    case 35: return a * x;
    case 36: return x + a;
    case 37: return 1.f / sqrtf(x);
    case 38: return powf(x, a);
  }
  return x;
}

inline float UnB(int op, float x, float y, float dy, float a) {
  switch (op) {
    case 0: return x > 0.f ? dy : 0.f;
    case 1: return dy * y * (1.f - y);
    case 2: return dy * (1.f - y * y);
    case 3: return dy * (0.66666667f * 1.7159047f - 0.66666667f / 1.7159047f * y * y);
    case 4: {
      const float cdf = 0.5f * (1.f + erff(x * 0.70710678118f));
      return dy * (cdf + x * 0.3989422804f * expf(-0.5f * x * x));
    }
    case 5: return dy;
    case 6: return dy / (1.f + expf(-x));
    case 7: return dy * 2.f * x;
    case 8: return dy * (float)((x > 0.f) - (x < 0.f));
    case 9: return dy * y;
    case 10: return x > 0.f ? dy : a * dy;
    case 11: return x > 0.f ? dy : dy * (y + a);
    case 12: {
      const float l = 1.0507009873554805f, al = 1.6732632423543772f;
      return x > 0.f ? l * dy : dy * (y + l * al);
    }
    case 13: {
      const float u = 0.7978845608f * (x + 0.044715f * x * x * x), t = tanhf(u);
      const float du = 0.7978845608f * (1.f + 3.f * 0.044715f * x * x);
      return dy * (0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du);
    }
    case 14: return dy * 0.5f / y;
    case 15: return -dy;
    case 16: return -dy * y * y;
    case 17: return dy / x;
    case 18: return 0.f;
    case 19: return dy * 1.1283791671f * expf(-x * x);
    case 20: return -dy * sinf(x);
    case 21: return dy * cosf(x);
    case 22: return dy * (1.f + y * y);
    case 23: return dy * sinhf(x);
    case 24: return dy * coshf(x);
    case 25: return -dy / sqrtf(1.f - x * x);
    case 26: return dy / sqrtf(1.f - x * x);
    case 27: return dy / (1.f + x * x);
    case 28: return dy / sqrtf(x * x - 1.f);
    case 29: return dy / sqrtf(x * x + 1.f);
    case 30: return dy / (1.f - x * x);
    case 31: case 32: case 33: return 0.f;
    case 34: {
      const float d = 1.f + fabsf(x);
      return dy / (d * d);
    }
    case 35: return a * dy;
    case 36: return dy;
    case 37: return -0.5f * dy * y * y * y;
    case 38: return dy * a * powf(x, a - 1.f);
  }
  return dy;
}

constexpr int64_t kEw = 1 << 15;  // elementwise grain

}  // namespace

void UnaryFwd(int op, const float* x, float* y, int64_t n, float a) {
  ParallelFor(n, kEw, [&](int64_t b, int64_t e) {
    if (op == 0) {
      for (int64_t i = b; i < e; ++i) y[i] = x[i] > 0.f ? x[i] : 0.f;
    } else {
      for (int64_t i = b; i < e; ++i) y[i] = UnF(op, x[i], a);
    }
  });
}

void UnaryBwd(int op, const float* x, const float* y, const float* dy, float* dx, int64_t n, float a) {
  ParallelFor(n, kEw, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) dx[i] = UnB(op, x ? x[i] : 0.f, y ? y[i] : 0.f, dy[i], a);
  });
}

// ---------------------------------------------------------------- N-d copy / binary
namespace {

inline float Bf16ToF(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
inline uint16_t FToBf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                          // round to nearest even
  return (uint16_t)(u >> 16);
}
inline double Load(const void* p, int dt, int64_t i) {
  switch (dt) {
    case 0: return ((const float*)p)[i];
    case 1: return Bf16ToF(((const uint16_t*)p)[i]);
    case 3: return ((const int32_t*)p)[i];
    case 4: return (double)((const int64_t*)p)[i];
    case 5: return ((const uint8_t*)p)[i];
    case 6: return ((const double*)p)[i];
  }
  return 0.0;
}
inline void Store(void* p, int dt, int64_t i, double v) {
  switch (dt) {
    case 0: ((float*)p)[i] = (float)v; break;
    case 1: ((uint16_t*)p)[i] = FToBf16((float)v); break;
    case 3: ((int32_t*)p)[i] = (int32_t)v; break;
    case 4: ((int64_t*)p)[i] = (int64_t)v; break;
    case 5: ((uint8_t*)p)[i] = (uint8_t)v; break;
    case 6: ((double*)p)[i] = v; break;
  }
}
int Esize(int dt) {
  static const int s[] = {4, 2, 2, 4, 8, 1, 8};
  return dt >= 0 && dt <= 6 ? s[dt] : 1;
}

// iterate the outer (nd-1) dims of a row range: fn(inner_count, offsets...)
template <int NOP, typename F>
void NdRows(int nd, const int64_t* size, const int64_t* const* st, int64_t r0, int64_t r1, F&& fn) {
  // rows = prod(size[0..nd-2]); inner dim = size[nd-1]
  int64_t idx[8] = {0};
  int64_t rem = r0;
  for (int d = nd - 2; d >= 0; --d) {
    idx[d] = rem % size[d];
    rem /= size[d];
  }
  int64_t off[NOP];
  for (int o = 0; o < NOP; ++o) {
    off[o] = 0;
    for (int d = 0; d < nd - 1; ++d) off[o] += idx[d] * st[o][d];
  }
  for (int64_t r = r0; r < r1; ++r) {
    fn(off);
    for (int d = nd - 2; d >= 0; --d) {
      for (int o = 0; o < NOP; ++o) off[o] += st[o][d];
      if (++idx[d] < size[d]) break;
      for (int o = 0; o < NOP; ++o) off[o] -= st[o][d] * size[d];
      idx[d] = 0;
    }
  }
}

}  // namespace

void CopyNd(const void* src, int dti, void* dst, int dto, int nd, const int64_t* size, const int64_t* dst_st,
            const int64_t* src_st) {
  if (nd <= 0) {
    Store(dst, dto, 0, Load(src, dti, 0));
    return;
  }
  int64_t rows = 1;
  for (int d = 0; d < nd - 1; ++d) rows *= size[d];
  const int64_t inner = size[nd - 1], so = dst_st[nd - 1], si = src_st[nd - 1];
  const int64_t* st[2] = {dst_st, src_st};
  const int es = Esize(dti);
  ParallelFor(rows, std::max<int64_t>(1, kEw / std::max<int64_t>(inner, 1)), [&](int64_t r0, int64_t r1) {
    NdRows<2>(nd, size, st, r0, r1, [&](const int64_t* off) {
      if (dti == dto && so == 1 && si == 1) {
        memcpy((char*)dst + off[0] * es, (const char*)src + off[1] * es, inner * es);
      } else if (dti == 0 && dto == 0) {
        float* d = (float*)dst + off[0];
        const float* s = (const float*)src + off[1];
        for (int64_t i = 0; i < inner; ++i) d[i * so] = s[i * si];
      } else {
        for (int64_t i = 0; i < inner; ++i) Store(dst, dto, off[0] + i * so, Load(src, dti, off[1] + i * si));
      }
    });
  });
}

namespace {
inline float BinOp(int op, float a, float b) {
  switch (op) {
    case 0: return a + b;
    case 1: return a - b;
    case 2: return a * b;
    case 3: return a / b;
    case 4: return powf(a, b);
    case 5: return a > b ? a : b;
    case 6: return a < b ? a : b;
    case 7: return (float)(a < b);
    case 8: return (float)(a <= b);
    case 9: return (float)(a > b);
    case 10: return (float)(a >= b);
    case 11: return (float)(a == b);
    case 12: return (float)(a != b);
    case 13: return (float)(a != 0.f && b != 0.f);
    case 14: return (float)(a != 0.f || b != 0.f);
    case 15: return (float)((a != 0.f) != (b != 0.f));
  }
  return a;
}
// alpha * (a OP b), as the GPU kernel (alpha folds an operator's backward scale)
inline float BinF(int op, float a, float b, float alpha) { return alpha == 1.f ? BinOp(op, a, b) : alpha * BinOp(op, a, b); }
}  // namespace

void BinaryNd(int op, const float* a, const float* b, float* out, int nd, const int64_t* size, const int64_t* os,
              const int64_t* as, const int64_t* bs, float alpha) {
  if (nd <= 0) {
    out[0] = BinF(op, a[0], b[0], alpha);
    return;
  }
  int64_t rows = 1;
  for (int d = 0; d < nd - 1; ++d) rows *= size[d];
  const int64_t inner = size[nd - 1], so = os[nd - 1], sa = as[nd - 1], sb = bs[nd - 1];
  const int64_t* st[3] = {os, as, bs};
  ParallelFor(rows, std::max<int64_t>(1, kEw / std::max<int64_t>(inner, 1)), [&](int64_t r0, int64_t r1) {
    NdRows<3>(nd, size, st, r0, r1, [&](const int64_t* off) {
      float* o = out + off[0];
      const float* x = a + off[1];
      const float* y = b + off[2];
      if (so == 1 && sa == 1 && sb == 1 && alpha == 1.f) {
        switch (op) {
          case 0: for (int64_t i = 0; i < inner; ++i) o[i] = x[i] + y[i]; return;
          case 1: for (int64_t i = 0; i < inner; ++i) o[i] = x[i] - y[i]; return;
          case 2: for (int64_t i = 0; i < inner; ++i) o[i] = x[i] * y[i]; return;
          default: break;
        }
      }
      for (int64_t i = 0; i < inner; ++i) o[i * so] = BinF(op, x[i * sa], y[i * sb], alpha);
    });
  });
}

void Fill(void* p, int64_t n, int dt, double v) {
  ParallelFor(n, kEw * 4, [&](int64_t b, int64_t e) {
    if (dt == 0) {
      float f = (float)v, *q = (float*)p;
      for (int64_t i = b; i < e; ++i) q[i] = f;
    } else {
      for (int64_t i = b; i < e; ++i) Store(p, dt, i, v);
    }
  });
}

void WhereNd(const uint8_t* c, const float* a, const float* b, float* out, int nd, const int64_t* size,
             const int64_t* os, const int64_t* as, const int64_t* bs, const int64_t* cs) {
  if (nd <= 0) {
    out[0] = c[0] ? a[0] : b[0];
    return;
  }
  int64_t rows = 1;
  for (int d = 0; d < nd - 1; ++d) rows *= size[d];
  const int64_t inner = size[nd - 1];
  const int64_t* st[4] = {os, as, bs, cs};
  ParallelFor(rows, std::max<int64_t>(1, kEw / std::max<int64_t>(inner, 1)), [&](int64_t r0, int64_t r1) {
    NdRows<4>(nd, size, st, r0, r1, [&](const int64_t* off) {
      for (int64_t i = 0; i < inner; ++i)
        out[off[0] + i * os[nd - 1]] =
            c[off[3] + i * cs[nd - 1]] ? a[off[1] + i * as[nd - 1]] : b[off[2] + i * bs[nd - 1]];
    });
  });
}

void ClampAffine(const float* x, const float* dy, float* y, int64_t n, float a, float b, float lo, float hi) {
  ParallelFor(n, kEw, [&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const float z = a * x[i] + b;
      y[i] = dy ? ((z > lo && z < hi) ? dy[i] * a : 0.f) : std::min(std::max(z, lo), hi);
    }
  });
}

// ---- kMnistImage augmentation (the intent of the reference's commented-out
// parser code, src/worker/layer.cc:406-438: elastic distortion, scaling,
// rotation / shear, resize).  Coordinates follow the normalised-grid
// convention with pixel centres at (2i+1)/n - 1 (align_corners = false).

// out[b] = img[b] sampled bilinearly (zero outside) at theta[b] . (xn, yn, 1)
// + disp[b][y][x] (normalised units; disp may be null)
void AffineElasticSample(const float* img, const float* theta, const float* disp, float* out, int B, int H, int W) {
  ParallelFor((int64_t)B * H, std::max<int64_t>(1, kEw / std::max(W, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const int b = (int)(r / H), y = (int)(r % H);
      const float* t = theta + 6 * b;
      const float* im = img + (int64_t)b * H * W;
      const float yn = (2.f * y + 1.f) / H - 1.f;
      for (int x = 0; x < W; ++x) {
        const float xn = (2.f * x + 1.f) / W - 1.f;
        float gx = t[0] * xn + t[1] * yn + t[2], gy = t[3] * xn + t[4] * yn + t[5];
        if (disp) {
          const float* d = disp + (((int64_t)b * H + y) * W + x) * 2;
          gx += d[0];
          gy += d[1];
        }
        const float px = ((gx + 1.f) * W - 1.f) * 0.5f, py = ((gy + 1.f) * H - 1.f) * 0.5f;
        const float fx = std::floor(px), fy = std::floor(py);
        const int x0 = (int)fx, y0 = (int)fy;
        const float ax = px - fx, ay = py - fy;
        auto at = [&](int yy, int xx) -> float {
          return (yy >= 0 && yy < H && xx >= 0 && xx < W) ? im[(int64_t)yy * W + xx] : 0.f;
        };
        out[r * W + x] = (1.f - ay) * ((1.f - ax) * at(y0, x0) + ax * at(y0, x0 + 1)) +
                         ay * ((1.f - ax) * at(y0 + 1, x0) + ax * at(y0 + 1, x0 + 1));
      }
    }
  });
}

// separable 'same' Gaussian blur of N planes [N][H][W] (zero padding)
void GaussBlur2D(const float* in, float* out, int N, int H, int W, const float* g, int k) {
  const int hk = k / 2;
  std::vector<float> tmp((size_t)N * H * W);
  ParallelFor((int64_t)N * H, std::max<int64_t>(1, kEw / std::max(W * k, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const float* src = in + r * W;
      float* dst = tmp.data() + r * W;
      for (int x = 0; x < W; ++x) {
        float a = 0.f;
        for (int j = 0; j < k; ++j) {
          const int xx = x + j - hk;
          if (xx >= 0 && xx < W) a += g[j] * src[xx];
        }
        dst[x] = a;
      }
    }
  });
  ParallelFor((int64_t)N * H, std::max<int64_t>(1, kEw / std::max(W * k, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t n = r / H;
      const int y = (int)(r % H);
      for (int x = 0; x < W; ++x) {
        float a = 0.f;
        for (int j = 0; j < k; ++j) {
          const int yy = y + j - hk;
          if (yy >= 0 && yy < H) a += g[j] * tmp[((size_t)n * H + yy) * W + x];
        }
        out[r * W + x] = a;
      }
    }
  });
}

// bilinear resize [B][H][W] -> [B][h][w] (half-pixel centres, edge clamp)
void ResizeBilinear(const float* in, float* out, int B, int H, int W, int h, int w) {
  const float sy = (float)H / h, sx = (float)W / w;
  ParallelFor((int64_t)B * h, std::max<int64_t>(1, kEw / std::max(w, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const int b = (int)(r / h), y = (int)(r % h);
      float fy = std::max((y + 0.5f) * sy - 0.5f, 0.f);
      const int y0 = std::min((int)fy, H - 1), y1 = std::min(y0 + 1, H - 1);
      const float ay = fy - y0;
      const float* im = in + (int64_t)b * H * W;
      for (int x = 0; x < w; ++x) {
        float fx = std::max((x + 0.5f) * sx - 0.5f, 0.f);
        const int x0 = std::min((int)fx, W - 1), x1 = std::min(x0 + 1, W - 1);
        const float ax = fx - x0;
        out[r * w + x] = (1.f - ay) * ((1.f - ax) * im[(int64_t)y0 * W + x0] + ax * im[(int64_t)y0 * W + x1]) +
                         ay * ((1.f - ax) * im[(int64_t)y1 * W + x0] + ax * im[(int64_t)y1 * W + x1]);
      }
    }
  });
}

// EASGD elastic difference (reference ElasticParam, src/utils/param.cc:244-284):
// d = alpha (w - c); w -= d.  With c_add (the centre update after the
// exchange) : c += s instead (s = the summed differences).
void EasgdDiff(float* w, const float* c, float* d, int64_t n, float alpha) {
  ParallelFor(n, kEw, [&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const float v = alpha * (w[i] - c[i]);
      d[i] = v;
      w[i] -= v;
    }
  });
}

// RandomSync (src/utils/param.cc:130-241) over the index progression
// idx_j = (b + j a) mod n, j < m: gather w - snapshot, and scatter
// snapshot + summed delta back into both w and the snapshot.
void RsyncGather(const float* w, const float* snap, float* buf, int64_t m, int64_t n, int64_t a, int64_t b) {
  ParallelFor(m, kEw, [&](int64_t j0, int64_t j1) {
    for (int64_t j = j0; j < j1; ++j) {
      const int64_t i = (int64_t)(((__int128)b + (__int128)j * a) % n);
      buf[j] = w[i] - snap[i];
    }
  });
}
void RsyncScatter(float* w, float* snap, const float* buf, int64_t m, int64_t n, int64_t a, int64_t b) {
  ParallelFor(m, kEw, [&](int64_t j0, int64_t j1) {
    for (int64_t j = j0; j < j1; ++j) {
      const int64_t i = (int64_t)(((__int128)b + (__int128)j * a) % n);
      const float v = snap[i] + buf[j];
      w[i] = v;
      snap[i] = v;
    }
  });
}

void Reduce(const float* x, float* y, int64_t outer, int64_t red, int64_t inner, int op) {
  auto init = [op]() -> double { return op == 2 ? -INFINITY : op == 3 ? INFINITY : 0.0; };
  if (inner == 1) {
    ParallelFor(outer, std::max<int64_t>(1, kEw / std::max<int64_t>(red, 1)), [&](int64_t o0, int64_t o1) {
      for (int64_t o = o0; o < o1; ++o) {
        const float* r = x + o * red;
        double acc = init();
        for (int64_t j = 0; j < red; ++j) {
          const double v = r[j];
          acc = op == 2 ? std::max(acc, v) : op == 3 ? std::min(acc, v) : op == 4 ? acc + v * v : acc + v;
        }
        y[o] = (float)(op == 1 ? acc / (double)red : acc);
      }
    });
    return;
  }
  ParallelFor(outer * inner, std::max<int64_t>(1, kEw / std::max<int64_t>(red, 1)), [&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t o = i / inner, c = i % inner;
      const float* r = x + o * red * inner + c;
      double acc = init();
      for (int64_t j = 0; j < red; ++j) {
        const double v = r[j * inner];
        acc = op == 2 ? std::max(acc, v) : op == 3 ? std::min(acc, v) : op == 4 ? acc + v * v : acc + v;
      }
      y[i] = (float)(op == 1 ? acc / (double)red : acc);
    }
  });
}

// ---------------------------------------------------------------- softmax / loss
void SoftmaxRows(const float* x, float* y, int64_t rows, int64_t C) {
  ParallelFor(rows, std::max<int64_t>(1, 4096 / std::max<int64_t>(C, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const float* a = x + r * C;
      float* o = y + r * C;
      float m = -INFINITY;
      for (int64_t j = 0; j < C; ++j) m = std::max(m, a[j]);
      double s = 0.0;
      for (int64_t j = 0; j < C; ++j) {
        o[j] = expf(a[j] - m);
        s += o[j];
      }
      const float inv = (float)(1.0 / s);
      for (int64_t j = 0; j < C; ++j) o[j] *= inv;
    }
  });
}

void SoftmaxRowsBwd(const float* y, const float* dy, float* dx, int64_t rows, int64_t C) {
  ParallelFor(rows, std::max<int64_t>(1, 4096 / std::max<int64_t>(C, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const float *p = y + r * C, *g = dy + r * C;
      double s = 0.0;
      for (int64_t j = 0; j < C; ++j) s += (double)g[j] * p[j];
      const float fs = (float)s;
      for (int64_t j = 0; j < C; ++j) dx[r * C + j] = p[j] * (g[j] - fs);
    }
  });
}

void SoftmaxXent(const float* x, const void* lab, int lab64, const float* t, float* loss, float* correct, float* dx,
                 int64_t B, int64_t C, int topk, float gs) {
  ParallelFor(B, std::max<int64_t>(1, 4096 / std::max<int64_t>(C, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const float* a = x + r * C;
      float m = -INFINITY;
      for (int64_t j = 0; j < C; ++j) m = std::max(m, a[j]);
      double s = 0.0;
      for (int64_t j = 0; j < C; ++j) s += exp((double)a[j] - m);
      const double lse = m + log(s);
      if (t) {  // soft targets
        const float* tt = t + r * C;
        double l = 0.0, tsum = 0.0;
        for (int64_t j = 0; j < C; ++j) {
          l += tt[j] * (lse - a[j]);
          tsum += tt[j];
        }
        loss[r] = (float)l;
        correct[r] = 0.f;
        if (dx)
          for (int64_t j = 0; j < C; ++j)
            dx[r * C + j] = (float)((exp((double)a[j] - lse) * tsum - tt[j]) * gs);
      } else {
        int64_t y = lab64 ? ((const int64_t*)lab)[r] : ((const int32_t*)lab)[r];
        y = std::min<int64_t>(std::max<int64_t>(y, 0), C - 1);
        const float xl = a[y];
        loss[r] = (float)(lse - xl);
        int64_t rank = 0;
        for (int64_t j = 0; j < C; ++j) rank += a[j] > xl;
        correct[r] = rank < topk ? 1.f : 0.f;
        if (dx) {
          for (int64_t j = 0; j < C; ++j) dx[r * C + j] = (float)(exp((double)a[j] - lse) * gs);
          dx[r * C + y] -= gs;
        }
      }
    }
  });
}

// ---------------------------------------------------------------- convolution
namespace {

struct ConvGeom {
  int C, H, W, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, g, Cg, Kg;
  int64_t crs() const { return (int64_t)Cg * R * S; }
  int64_t hw() const { return (int64_t)Ho * Wo; }
};

// col[(c, r, s)][(oh, ow)] of group gi of one image
void Im2col(const ConvGeom& q, const float* x, int gi, float* col) {
  for (int c = 0; c < q.Cg; ++c) {
    const float* xc = x + (int64_t)(gi * q.Cg + c) * q.H * q.W;
    for (int r = 0; r < q.R; ++r)
      for (int s = 0; s < q.S; ++s) {
        float* dst = col + (((int64_t)c * q.R + r) * q.S + s) * q.hw();
        for (int oh = 0; oh < q.Ho; ++oh) {
          const int ih = oh * q.sh - q.ph + r * q.dh;
          float* d = dst + (int64_t)oh * q.Wo;
          if (ih < 0 || ih >= q.H) {
            memset(d, 0, sizeof(float) * q.Wo);
            continue;
          }
          const float* xr = xc + (int64_t)ih * q.W;
          const int off = s * q.dw - q.pw;
          if (q.sw == 1) {
            // valid ow range: 0 <= ow + off < W
            const int lo = std::max(0, -off), hi = std::min(q.Wo, q.W - off);
            for (int ow = 0; ow < std::min(lo, q.Wo); ++ow) d[ow] = 0.f;
            if (hi > lo) memcpy(d + lo, xr + lo + off, sizeof(float) * (hi - lo));
            for (int ow = std::max(hi, lo); ow < q.Wo; ++ow) d[ow] = 0.f;
          } else {
            for (int ow = 0; ow < q.Wo; ++ow) {
              const int iw = ow * q.sw + off;
              d[ow] = (iw >= 0 && iw < q.W) ? xr[iw] : 0.f;
            }
          }
        }
      }
  }
}

void Col2im(const ConvGeom& q, const float* col, int gi, float* dx) {
  for (int c = 0; c < q.Cg; ++c) {
    float* xc = dx + (int64_t)(gi * q.Cg + c) * q.H * q.W;
    for (int r = 0; r < q.R; ++r)
      for (int s = 0; s < q.S; ++s) {
        const float* src = col + (((int64_t)c * q.R + r) * q.S + s) * q.hw();
        for (int oh = 0; oh < q.Ho; ++oh) {
          const int ih = oh * q.sh - q.ph + r * q.dh;
          if (ih < 0 || ih >= q.H) continue;
          float* xr = xc + (int64_t)ih * q.W;
          const float* sr = src + (int64_t)oh * q.Wo;
          const int off = s * q.dw - q.pw;
          for (int ow = 0; ow < q.Wo; ++ow) {
            const int iw = ow * q.sw + off;
            if (iw >= 0 && iw < q.W) xr[iw] += sr[ow];
          }
        }
      }
  }
}

bool Is1x1(const ConvGeom& q) {
  return q.R == 1 && q.S == 1 && q.sh == 1 && q.sw == 1 && q.ph == 0 && q.pw == 0 && q.Ho == q.H && q.Wo == q.W;
}

// image ranges for P fixed slots (deterministic partial sums)
inline void SlotRange(int N, int P, int64_t s, int* n0, int* n1) {
  *n0 = (int)((int64_t)N * s / P);
  *n1 = (int)((int64_t)N * (s + 1) / P);
}

}  // namespace

void ConvFwd(const float* x, const float* w, const float* bias, float* y, int N, int C, int H, int W, int K, int R,
             int S, int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups) {
  const ConvGeom q{C, H, W, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups, C / groups, K / groups};
  const bool one = Is1x1(q);
  auto image = [&](int n, std::vector<float>& col) {
    const float* xn = x + (int64_t)n * C * H * W;
    float* yn = y + (int64_t)n * K * q.hw();
    for (int gi = 0; gi < groups; ++gi) {
      const float* b = xn + (int64_t)gi * q.Cg * H * W;
      if (!one) {
        Im2col(q, xn, gi, col.data());
        b = col.data();
      }
      // y[Kg][HW] = w_g[Kg][CgRS] @ col[CgRS][HW]
      Gemm(false, false, q.Kg, q.hw(), q.crs(), 1.f, w + (int64_t)gi * q.Kg * q.crs(), q.crs(), b, q.hw(), 0.f,
           yn + (int64_t)gi * q.Kg * q.hw(), q.hw(), nullptr, false);
      if (bias)
        for (int k = 0; k < q.Kg; ++k) {
          float* yk = yn + ((int64_t)gi * q.Kg + k) * q.hw();
          const float bv = bias[gi * q.Kg + k];
          for (int64_t i = 0; i < q.hw(); ++i) yk[i] += bv;
        }
    }
  };
  const int P = NumThreads();
  if (N >= P || N >= 4) {
    ParallelFor(N, 1, [&](int64_t n0, int64_t n1) {
      std::vector<float> col(one ? 0 : q.crs() * q.hw());
      for (int64_t n = n0; n < n1; ++n) image((int)n, col);
    });
  } else {
    std::vector<float> col(one ? 0 : q.crs() * q.hw());
    for (int n = 0; n < N; ++n) image(n, col);
  }
}

void ConvBwd(const float* x, const float* w, const float* dy, float* dx, float* dwt, float* db, int N, int C, int H,
             int W, int K, int R, int S, int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups) {
  const ConvGeom q{C, H, W, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups, C / groups, K / groups};
  const bool one = Is1x1(q);
  const int64_t wsz = (int64_t)K * q.crs();
  const int P = std::max(1, std::min(NumThreads(), N));
  std::vector<float> part(dwt ? (size_t)P * wsz : 0, 0.f);
  // slot s: images [n0, n1) -> partial dW_s (+ dx of its own images)
  ParallelFor(P, 1, [&](int64_t s0, int64_t s1) {
    std::vector<float> col(q.crs() * q.hw()), dcol(dx ? q.crs() * q.hw() : 0);
    for (int64_t s = s0; s < s1; ++s) {
      int n0, n1;
      SlotRange(N, P, s, &n0, &n1);
      float* pw_ = dwt ? part.data() + (size_t)s * wsz : nullptr;
      for (int n = n0; n < n1; ++n) {
        const float* xn = x + (int64_t)n * C * H * W;
        const float* dyn = dy + (int64_t)n * K * q.hw();
        float* dxn = dx ? dx + (int64_t)n * C * H * W : nullptr;
        if (dxn && !one) memset(dxn, 0, sizeof(float) * C * H * W);
        for (int gi = 0; gi < groups; ++gi) {
          const float* dyg = dyn + (int64_t)gi * q.Kg * q.hw();
          if (pw_) {
            const float* b = xn + (int64_t)gi * q.Cg * H * W;
            if (!one) {
              Im2col(q, xn, gi, col.data());
              b = col.data();
            }
            // dW_g[Kg][CgRS] += dy_g[Kg][HW] @ col^T   (col stored [CgRS][HW] = [N][K])
            Gemm(false, true, q.Kg, q.crs(), q.hw(), 1.f, dyg, q.hw(), b, q.hw(), 1.f,
                 pw_ + (int64_t)gi * q.Kg * q.crs(), q.crs(), nullptr, false);
          }
          if (dxn) {
            // dcol[CgRS][HW] = w_g^T @ dy_g   (w_g stored [Kg][CgRS] = [K][M])
            float* target = one ? dxn + (int64_t)gi * q.Cg * H * W : dcol.data();
            Gemm(true, false, q.crs(), q.hw(), q.Kg, 1.f, w + (int64_t)gi * q.Kg * q.crs(), q.crs(), dyg, q.hw(), 0.f,
                 target, q.hw(), nullptr, false);
            if (!one) Col2im(q, dcol.data(), gi, dxn);
          }
        }
      }
    }
  });
  if (dwt) {
    ParallelFor(wsz, 4096, [&](int64_t i0, int64_t i1) {
      for (int64_t i = i0; i < i1; ++i) {
        float acc = dwt[i];
        for (int s = 0; s < P; ++s) acc += part[(size_t)s * wsz + i];
        dwt[i] = acc;
      }
    });
  }
  if (db) {
    ParallelFor(K, 1, [&](int64_t k0, int64_t k1) {
      for (int64_t k = k0; k < k1; ++k) {
        double acc = 0.0;
        for (int n = 0; n < N; ++n) {
          const float* d = dy + ((int64_t)n * K + k) * q.hw();
          for (int64_t i = 0; i < q.hw(); ++i) acc += d[i];
        }
        db[k] += (float)acc;
      }
    });
  }
}

// ---------------------------------------------------------------- pooling
void PoolFwd(const float* x, float* y, int32_t* arg, int N, int C, int H, int W, int Ho, int Wo, int kh, int kw,
             int sh, int sw, int ph, int pw, int is_max, int count_include_pad) {
  ParallelFor((int64_t)N * C, 4, [&](int64_t p0, int64_t p1) {
    for (int64_t p = p0; p < p1; ++p) {
      const float* xp = x + p * H * W;
      float* yp = y + p * Ho * Wo;
      int32_t* ap = arg ? arg + p * Ho * Wo : nullptr;
      for (int oh = 0; oh < Ho; ++oh)
        for (int ow = 0; ow < Wo; ++ow) {
          int hs = oh * sh - ph, ws = ow * sw - pw;
          int he = std::min(hs + kh, H + ph), we = std::min(ws + kw, W + pw);
          const int pool = (he - hs) * (we - ws);
          hs = std::max(hs, 0);
          ws = std::max(ws, 0);
          he = std::min(he, H);
          we = std::min(we, W);
          if (is_max) {
            float m = -INFINITY;
            int mi = hs * W + ws;
            for (int ih = hs; ih < he; ++ih)
              for (int iw = ws; iw < we; ++iw) {
                const float v = xp[ih * W + iw];
                if (v > m || isnan(v)) {
                  m = v;
                  mi = ih * W + iw;
                }
              }
            yp[oh * Wo + ow] = m;
            if (ap) ap[oh * Wo + ow] = mi;
          } else {
            double s = 0.0;
            for (int ih = hs; ih < he; ++ih)
              for (int iw = ws; iw < we; ++iw) s += xp[ih * W + iw];
            const int div = count_include_pad ? pool : (he - hs) * (we - ws);
            yp[oh * Wo + ow] = div > 0 ? (float)(s / div) : 0.f;
          }
        }
    }
  });
}

void PoolBwd(const float* dy, const int32_t* arg, float* dx, int N, int C, int H, int W, int Ho, int Wo, int kh,
             int kw, int sh, int sw, int ph, int pw, int is_max, int count_include_pad) {
  ParallelFor((int64_t)N * C, 4, [&](int64_t p0, int64_t p1) {
    for (int64_t p = p0; p < p1; ++p) {
      float* dxp = dx + p * H * W;
      const float* dyp = dy + p * Ho * Wo;
      memset(dxp, 0, sizeof(float) * H * W);
      if (is_max) {
        const int32_t* ap = arg + p * Ho * Wo;
        for (int64_t i = 0; i < (int64_t)Ho * Wo; ++i) dxp[ap[i]] += dyp[i];
        continue;
      }
      for (int oh = 0; oh < Ho; ++oh)
        for (int ow = 0; ow < Wo; ++ow) {
          int hs = oh * sh - ph, ws = ow * sw - pw;
          int he = std::min(hs + kh, H + ph), we = std::min(ws + kw, W + pw);
          const int pool = (he - hs) * (we - ws);
          hs = std::max(hs, 0);
          ws = std::max(ws, 0);
          he = std::min(he, H);
          we = std::min(we, W);
          const int div = count_include_pad ? pool : (he - hs) * (we - ws);
          if (div <= 0) continue;
          const float g = dyp[oh * Wo + ow] / (float)div;
          for (int ih = hs; ih < he; ++ih)
            for (int iw = ws; iw < we; ++iw) dxp[ih * W + iw] += g;
        }
    }
  });
}

// ---------------------------------------------------------------- LRN
void LrnFwd(const float* x, float* y, int N, int C, int HW, int size, float alpha, float beta, float k) {
  const int half = size / 2;
  const float a = alpha / size;
  ParallelFor((int64_t)N * HW, 256, [&](int64_t i0, int64_t i1) {
    std::vector<float> sq(C);
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t n = i / HW, p = i % HW;
      const float* xp = x + n * C * HW + p;
      float* yp = y + n * C * HW + p;
      for (int c = 0; c < C; ++c) sq[c] = xp[(int64_t)c * HW] * xp[(int64_t)c * HW];
      for (int c = 0; c < C; ++c) {
        float s = 0.f;
        for (int j = std::max(0, c - half); j <= std::min(C - 1, c + half); ++j) s += sq[j];
        yp[(int64_t)c * HW] = xp[(int64_t)c * HW] * powf(k + a * s, -beta);
      }
    }
  });
}

void LrnBwd(const float* x, const float* dy, float* dx, int N, int C, int HW, int size, float alpha, float beta,
            float k) {
  const int half = size / 2;
  const float a = alpha / size;
  ParallelFor((int64_t)N * HW, 256, [&](int64_t i0, int64_t i1) {
    std::vector<float> sq(C), nrm(C), t(C);
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t n = i / HW, p = i % HW;
      const float* xp = x + n * C * HW + p;
      const float* gp = dy + n * C * HW + p;
      float* dp = dx + n * C * HW + p;
      for (int c = 0; c < C; ++c) sq[c] = xp[(int64_t)c * HW] * xp[(int64_t)c * HW];
      for (int c = 0; c < C; ++c) {
        float s = 0.f;
        for (int j = std::max(0, c - half); j <= std::min(C - 1, c + half); ++j) s += sq[j];
        nrm[c] = k + a * s;
        t[c] = gp[(int64_t)c * HW] * xp[(int64_t)c * HW] * powf(nrm[c], -beta - 1.f);
      }
      for (int c = 0; c < C; ++c) {
        float s = 0.f;
        for (int j = std::max(0, c - half); j <= std::min(C - 1, c + half); ++j) s += t[j];
        dp[(int64_t)c * HW] = gp[(int64_t)c * HW] * powf(nrm[c], -beta) - 2.f * beta * a * xp[(int64_t)c * HW] * s;
      }
    }
  });
}

// ---------------------------------------------------------------- RNG (Philox4x32-10, as common.h)
namespace {
struct U4 {
  uint32_t x, y, z, w;
};
inline U4 Philox(uint64_t seed, uint64_t counter, uint32_t sub) {
  U4 c{(uint32_t)counter, (uint32_t)(counter >> 32), sub, 0u};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
inline float U01(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }
}  // namespace

void DropoutFwd(const float* x, float* y, uint8_t* mask, int64_t n, float pkeep, uint64_t seed, uint64_t offset) {
  const float scale = 1.f / pkeep;
  ParallelFor((n + 3) / 4, 4096, [&](int64_t q0, int64_t q1) {
    for (int64_t q = q0; q < q1; ++q) {
      const U4 r = Philox(seed, offset + q, 0);
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
      for (int j = 0; j < 4; ++j) {
        const int64_t e = q * 4 + j;
        if (e >= n) break;
        const bool keep = U01(rr[j]) <= pkeep;
        mask[e] = keep;
        y[e] = keep ? x[e] * scale : 0.f;
      }
    }
  });
}

void DropoutBwd(const float* dy, const uint8_t* mask, float* dx, int64_t n, float pkeep) {
  const float scale = 1.f / pkeep;
  ParallelFor(n, kEw, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) dx[i] = mask[i] ? dy[i] * scale : 0.f;
  });
}

void RandFill(float* y, int64_t n, int dist, float a, float b, uint64_t seed, uint64_t offset) {
  ParallelFor((n + 3) / 4, 4096, [&](int64_t q0, int64_t q1) {
    for (int64_t q = q0; q < q1; ++q) {
      const U4 r = Philox(seed, offset + q, 1);
      const float u[4] = {U01(r.x), U01(r.y), U01(r.z), U01(r.w)};
      float o[4];
      if (dist == 0) {
        for (int j = 0; j < 4; ++j) o[j] = a + (b - a) * (1.f - u[j]);
      } else {
        const float r0 = sqrtf(-2.f * logf(u[0])), r1 = sqrtf(-2.f * logf(u[2]));
        const float t0 = 6.283185307f * u[1], t1 = 6.283185307f * u[3];
        o[0] = a + b * r0 * cosf(t0);
        o[1] = a + b * r0 * sinf(t0);
        o[2] = a + b * r1 * cosf(t1);
        o[3] = a + b * r1 * sinf(t1);
      }
      for (int j = 0; j < 4; ++j)
        if (q * 4 + j < n) y[q * 4 + j] = o[j];
    }
  });
}

// ---------------------------------------------------------------- normalisation
void BatchNormFwd(const float* x, const float* gamma, const float* beta, float* rm, float* rv, float* y, float* mean,
                  float* invstd, int N, int C, int64_t HW, int training, float momentum, float eps, int relu,
                  const float* residual) {
  const int64_t cnt = (int64_t)N * HW;
  ParallelFor(C, 1, [&](int64_t c0, int64_t c1) {
    for (int64_t c = c0; c < c1; ++c) {
      float mu, var;
      if (training) {
        double s = 0.0, s2 = 0.0;
        for (int n = 0; n < N; ++n) {
          const float* p = x + ((int64_t)n * C + c) * HW;
          for (int64_t i = 0; i < HW; ++i) s += p[i];
        }
        const double m = s / cnt;
        for (int n = 0; n < N; ++n) {
          const float* p = x + ((int64_t)n * C + c) * HW;
          for (int64_t i = 0; i < HW; ++i) s2 += (p[i] - m) * (p[i] - m);
        }
        mu = (float)m;
        var = (float)(s2 / cnt);
        rm[c] = (1.f - momentum) * rm[c] + momentum * mu;
        rv[c] = (1.f - momentum) * rv[c] + momentum * var * (float)cnt / (float)std::max<int64_t>(cnt - 1, 1);
      } else {
        mu = rm[c];
        var = rv[c];
      }
      const float is = 1.f / sqrtf(var + eps);
      mean[c] = mu;
      invstd[c] = is;
      const float sc = gamma[c] * is, sf = beta[c] - mu * sc;
      for (int n = 0; n < N; ++n) {
        const int64_t o = ((int64_t)n * C + c) * HW;
        for (int64_t i = 0; i < HW; ++i) {
          float v = x[o + i] * sc + sf;
          if (residual) v += residual[o + i];
          y[o + i] = relu && v < 0.f ? 0.f : v;
        }
      }
    }
  });
}

void BatchNormBwd(const float* x, const float* dy, const float* gamma, const float* mean, const float* invstd,
                  const float* y_for_mask, int relu_x, const float* scale, const float* shift, float* dx, float* dg,
                  float* db, float* dres, int N, int C, int64_t HW) {
  const int64_t cnt = (int64_t)N * HW;
  ParallelFor(C, 1, [&](int64_t c0, int64_t c1) {
    for (int64_t c = c0; c < c1; ++c) {
      const float mu = mean[c], is = invstd[c];
      const float sc = relu_x ? scale[c] : 0.f, sf = relu_x ? shift[c] : 0.f;
      auto grad = [&](int64_t o) -> float {
        if (y_for_mask) return y_for_mask[o] > 0.f ? dy[o] : 0.f;
        if (relu_x) return x[o] * sc + sf > 0.f ? dy[o] : 0.f;
        return dy[o];
      };
      double sdy = 0.0, sdyx = 0.0;
      for (int n = 0; n < N; ++n) {
        const int64_t o = ((int64_t)n * C + c) * HW;
        for (int64_t i = 0; i < HW; ++i) {
          const float g = grad(o + i);
          sdy += g;
          sdyx += g * (x[o + i] - mu) * is;
        }
      }
      const float a = (float)(sdy / cnt), b = (float)(sdyx / cnt), k = gamma[c] * is;
      for (int n = 0; n < N; ++n) {
        const int64_t o = ((int64_t)n * C + c) * HW;
        for (int64_t i = 0; i < HW; ++i) {
          const float g = grad(o + i);
          dx[o + i] = k * (g - a - (x[o + i] - mu) * is * b);
          if (dres) dres[o + i] = g;
        }
      }
      dg[c] += (float)sdyx;
      db[c] += (float)sdy;
    }
  });
}

void LayerNormFwd(const float* x, const float* g, const float* b, float* y, float* mean, float* rstd, int64_t R,
                  int64_t D, float eps) {
  ParallelFor(R, std::max<int64_t>(1, 4096 / std::max<int64_t>(D, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const float* p = x + r * D;
      double s = 0.0, s2 = 0.0;
      for (int64_t j = 0; j < D; ++j) s += p[j];
      const double m = s / D;
      for (int64_t j = 0; j < D; ++j) s2 += (p[j] - m) * (p[j] - m);
      const float rs = (float)(1.0 / sqrt(s2 / D + eps));
      mean[r] = (float)m;
      rstd[r] = rs;
      for (int64_t j = 0; j < D; ++j) {
        float v = (p[j] - (float)m) * rs;
        if (g) v *= g[j];
        if (b) v += b[j];
        y[r * D + j] = v;
      }
    }
  });
}

void LayerNormBwd(const float* x, const float* dy, const float* g, const float* mean, const float* rstd, float* dx,
                  float* dg, float* db, int64_t R, int64_t D) {
  ParallelFor(R, std::max<int64_t>(1, 4096 / std::max<int64_t>(D, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const float *p = x + r * D, *gy = dy + r * D;
      const float m = mean[r], rs = rstd[r];
      double sa = 0.0, sb = 0.0;
      for (int64_t j = 0; j < D; ++j) {
        const float gg = g ? gy[j] * g[j] : gy[j];
        sa += gg;
        sb += gg * (p[j] - m) * rs;
      }
      const float a = (float)(sa / D), bb = (float)(sb / D);
      for (int64_t j = 0; j < D; ++j) {
        const float gg = g ? gy[j] * g[j] : gy[j];
        dx[r * D + j] = rs * (gg - a - (p[j] - m) * rs * bb);
      }
    }
  });
  if (dg || db) {  // column sums in a fixed order
    ParallelFor(D, 64, [&](int64_t j0, int64_t j1) {
      for (int64_t j = j0; j < j1; ++j) {
        double sg = 0.0, sbv = 0.0;
        for (int64_t r = 0; r < R; ++r) {
          const float gyv = dy[r * D + j];
          sg += gyv * (x[r * D + j] - mean[r]) * rstd[r];
          sbv += gyv;
        }
        if (dg) dg[j] += (float)sg;
        if (db) db[j] += (float)sbv;
      }
    });
  }
}

// ---------------------------------------------------------------- indexing
void IndexSelect(const void* src, const void* idx, int idx64, void* dst, int64_t outer, int64_t nsrc, int64_t inner,
                 int64_t nidx, int esize) {
  ParallelFor(outer * nidx, std::max<int64_t>(1, kEw / std::max<int64_t>(inner, 1)), [&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t o = i / nidx, j = i % nidx;
      int64_t s = idx64 ? ((const int64_t*)idx)[j] : ((const int32_t*)idx)[j];
      s = std::min<int64_t>(std::max<int64_t>(s, 0), nsrc - 1);
      memcpy((char*)dst + (i * inner) * esize, (const char*)src + ((o * nsrc + s) * inner) * esize, inner * esize);
    }
  });
}

void IndexAdd(float* dst, const void* idx, int idx64, const float* src, int64_t outer, int64_t ndst, int64_t inner,
              int64_t nidx, float alpha) {
  // parallel over (outer, inner column blocks): every destination element is
  // owned by one task, indices are visited in order (deterministic)
  const int64_t cb = 256, ncb = (inner + cb - 1) / cb;
  ParallelFor(outer * ncb, 1, [&](int64_t t0, int64_t t1) {
    for (int64_t t = t0; t < t1; ++t) {
      const int64_t o = t / ncb, c0 = (t % ncb) * cb, c1 = std::min(inner, c0 + cb);
      for (int64_t j = 0; j < nidx; ++j) {
        int64_t d = idx64 ? ((const int64_t*)idx)[j] : ((const int32_t*)idx)[j];
        if (d < 0 || d >= ndst) continue;
        float* out = dst + (o * ndst + d) * inner;
        const float* in = src + (o * nidx + j) * inner;
        for (int64_t c = c0; c < c1; ++c) out[c] += alpha * in[c];
      }
    }
  });
}

}  // namespace cpu
}  // namespace sgrt

// Host side of the persistent kernels' dynamic work queues (common.h) and a
// CU-occupancy probe for the interference rehearsal.
//
// Queue slots live in one small device array per GPU, allocated and zeroed
// once (outside any capture: the allocation runs with the thread's capture
// mode relaxed and zeroes through a private non-blocking stream), handed out
// round-robin.  A slot is reset on the device by the last workgroup of the
// kernel that used it, so a slot is reusable as soon as that kernel ends; the
// ring only has to be larger than the number of persistent kernels that can
// run at the same time.
//
// A captured HIP graph freezes the slot each of its persistent kernels was
// given, while later launches keep advancing the ring -- so two graphs (or a
// graph and eager launches) replayed at the same time could share a slot.
// Captures therefore take their slots from a private ARENA instead: while a
// thread captures (sg_workq_arena_begin .. sg_workq_arena_end) every slot it
// is handed is a fresh one of that arena, never handed out again, and the
// arena is freed with its graph (sg_workq_arena_free).  Several threads
// capturing into one graph (the loopback world's ranks) each use their own.
#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "common.h"

namespace {
constexpr int kRing = 256;
constexpr int kMaxDev = 16;
int* g_ring[kMaxDev] = {};
std::atomic<unsigned> g_next[kMaxDev];
std::mutex g_mu;
int g_cus[kMaxDev] = {};
int g_on = -1;

constexpr int kArenaChunk = 64;  // slots per arena allocation

// a device allocation of `slots` zeroed queue slots, made outside any capture
// (this thread's capture mode relaxed; zeroed through a private stream)
int* alloc_zeroed_slots(int slots) {
  hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&m);
  int* p = nullptr;
  const size_t bytes = sizeof(int) * QSLOT * (size_t)slots;
  if (hipMalloc(&p, bytes) == hipSuccess) {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) {
      (void)hipMemsetAsync(p, 0, bytes, s);
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    } else {
      (void)hipFree(p);
      p = nullptr;
    }
  }
  (void)hipThreadExchangeStreamCaptureMode(&m);
  return p;
}

struct Arena {
  std::vector<int*> chunks;
  int used = kArenaChunk;  // slots taken from the last chunk
  int* take() {
    if (used == kArenaChunk) {
      int* c = alloc_zeroed_slots(kArenaChunk);
      if (!c) return nullptr;
      chunks.push_back(c);
      used = 0;
    }
    return chunks.back() + (size_t)(used++) * QSLOT;
  }
  ~Arena() {
    for (int* c : chunks) (void)hipFree(c);
  }
};
thread_local Arena* t_arena = nullptr;

int cur_dev() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d < 0 || d >= kMaxDev ? 0 : d;
}

int* ring_of(int d) {
  if (g_ring[d]) return g_ring[d];
  std::lock_guard<std::mutex> g(g_mu);
  if (g_ring[d]) return g_ring[d];
  g_ring[d] = alloc_zeroed_slots(kRing);
  return g_ring[d];
}

// spin until the device's constant 100 MHz clock passes `until`
__global__ void cu_hog_k(uint64_t ticks, int* started) {
  extern __shared__ char lds[];  // requested at (nearly) a CU's whole LDS: one workgroup per CU
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) {
    lds[0] = 1;
    atomicAdd(started, 1);
  }
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}
}  // namespace

extern "C" {

void sg_workq_set(int on) { g_on = on ? 1 : 0; }

int sg_workq_enabled() {
  if (g_on < 0) {
    const char* e = getenv("SG_WORKQ");
    g_on = (e && e[0] == '0') ? 0 : 1;
  }
  return g_on;
}

int* sg_workq_slot() {
  if (!sg_workq_enabled()) return nullptr;
  if (t_arena) return t_arena->take();  // a capture: a slot of its own
  const int d = cur_dev();
  int* r = ring_of(d);
  if (!r) return nullptr;
  const unsigned i = g_next[d].fetch_add(1, std::memory_order_relaxed) % kRing;
  return r + (size_t)i * QSLOT;
}

// Route this thread's slots to a new arena (call before a capture begins,
// on the capture's device); returns its handle.
void* sg_workq_arena_begin() {
  Arena* a = new Arena();
  t_arena = a;
  return a;
}
// Stop routing (the capture ended or was abandoned); the arena lives on with
// the graph that addresses it.
void sg_workq_arena_end() { t_arena = nullptr; }
// Free an arena once no graph that addresses it can run any more.
void sg_workq_arena_free(void* h) {
  Arena* a = (Arena*)h;
  if (t_arena == a) t_arena = nullptr;
  delete a;
}
int sg_workq_arena_slots(void* h) {
  const Arena* a = (const Arena*)h;
  return a->chunks.empty() ? 0 : (int)(a->chunks.size() - 1) * kArenaChunk + a->used;
}

int sg_cu_count() {
  const int d = cur_dev();
  if (g_cus[d] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0) n = 256;
    g_cus[d] = n;
  }
  return g_cus[d];
}

// Interference rehearsal: occupy `ncu` compute units for `us` microseconds
// with one sleeping workgroup each (each requests `lds_bytes` of LDS, by
// default 160 KB, so no other workgroup that needs more than the rest can
// share its CU), on stream s -- a stand-in for RCCL's channel kernels
// holding CUs while the gradient all-reduce overlaps the backward.
// `started` (device int, optional) counts the workgroups that got a CU.
void sg_cu_hog(int ncu, double us, int lds_bytes, int* started, hipStream_t s) {
  if (ncu <= 0) return;
  const int lds = lds_bytes > 0 ? lds_bytes : 160 * 1024;
  static bool attr = hipFuncSetAttribute((const void*)cu_hog_k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024) == hipSuccess;
  (void)attr;
  static int* dummy = nullptr;
  if (!started) {
    if (!dummy) (void)hipMalloc(&dummy, sizeof(int));
    started = dummy;
  }
  const uint64_t ticks = (uint64_t)(us * 100.0);  // 100 MHz constant clock
  hipLaunchKernelGGL(cu_hog_k, dim3(ncu), dim3(64), lds, s, ticks, started);
}

}  // extern "C"

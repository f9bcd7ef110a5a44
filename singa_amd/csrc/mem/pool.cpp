// Native memory pools: the framework's own device (HBM) and host allocators.
//
// Reference counterparts: mshadow's AllocSpace / FreeSpace
// (include/mshadow/tensor.h:206-385, tensor_gpu-inl.hpp) and the Blob /
// SyncedMemory pair (src/utils/blob.cc:83-298) that owned every parameter
// and activation buffer of the reference.  Here:
//
//   * DevicePool: a caching allocator over hipMalloc for one GPU.  Blocks are
//     rounded to size classes (512 B granularity up to 1 MiB, 2 MiB above),
//     kept on per-size free lists and reused without touching the driver;
//     a block freed while a stream may still be using it is parked with an
//     event recorded on that stream and becomes reusable once the event has
//     completed (no host synchronisation on the free path).
//   * HostPool: 64-byte-aligned pageable blocks (CppCPU tensors) or pinned
//     hipHostMalloc blocks (staging buffers for host <-> device copies).
//   * Blocks are handed to PyTorch as DLPack tensors: storage owned by the
//     pool, returned to it by the capsule's deleter when the last tensor
//     referencing it dies.  PyTorch then only provides views / metadata.
//
// Exposed to Python (module _C) by register_mem(); singa_amd/memory.py wraps it.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <tuple>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

// ------------------------------------------------------------- DLPack ABI
// (the stable v0.x structs, declared here so no header is needed)
struct DLDevice {
  int32_t device_type;
  int32_t device_id;
};
struct DLDataType {
  uint8_t code, bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor* self);
};
constexpr int32_t kDLCPU = 1;

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

size_t round_size(size_t n) {
  if (n == 0) n = 1;
  if (n <= (1u << 20)) return (n + 511) & ~(size_t)511;
  return (n + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
}

struct Stats {
  uint64_t allocs = 0, frees = 0, hits = 0, driver_allocs = 0;
  uint64_t in_use = 0, reserved = 0, peak_in_use = 0;
};

// A device block: its size class, the stream it was allocated on (the stream
// whose order makes reuse safe), the pool that owns it (0 = the default
// pool, > 0 = a private pool of one HIP graph) and the other streams that
// used it (record_stream): a free with foreign uses waits for events.
struct BlockInfo {
  size_t size;
  uintptr_t stream;
  int pool;
  std::vector<uintptr_t> uses;
  bool in_capture = false;  // a default-pool block handed out while its stream was being captured
};
struct Pending {
  void* ptr;
  BlockInfo info;
  std::vector<hipEvent_t> evs;
};

thread_local int t_pool = 0;  // private pool of the capture this thread is running (0: default pool)

// hipMalloc / hipFree / event queries are "potentially unsafe" while a
// stream is captured in the default (global) mode and would invalidate the
// capture; the pool's own driver calls are not part of any captured work, so
// they run with this thread's capture mode relaxed (as PyTorch's allocator
// does around cudaMalloc)
struct RelaxedCapture {
  hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
  RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
  ~RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
};

class DevicePool {
 public:
  explicit DevicePool(int dev) : dev_(dev) {}

  // Stream-ordered caching: a block freed by its allocation stream is reused
  // at once by the next allocation on that SAME stream (later work on the
  // stream is ordered after every use of the old tensor) -- no event, no
  // host sync on the hot path.  Allocations while a HIP graph is captured
  // come from that graph's private pool and stay with it.
  void* alloc(size_t n, uintptr_t stream) {
    const size_t sz = round_size(n);
    const int pool = t_pool;
    std::lock_guard<std::mutex> g(mu_);
    ++st_.allocs;
    if (!pending_.empty()) reap_locked();
    void* p = nullptr;
    auto it = free_.find(std::make_tuple(pool, stream, sz));
    if (it != free_.end() && !it->second.empty()) {
      p = it->second.back();
      it->second.pop_back();
      ++st_.hits;
    } else {
      p = driver_alloc_locked(sz);
    }
    live_[p] = BlockInfo{sz, stream, pool, {}, pool == 0 && capturing(stream)};
    st_.in_use += sz;
    if (st_.in_use > st_.peak_in_use) st_.peak_in_use = st_.in_use;
    return p;
  }

  void free(void* p) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.find(p);
    if (it == live_.end()) throw std::runtime_error("DevicePool::free: pointer not from this pool");
    BlockInfo b = std::move(it->second);
    live_.erase(it);
    ++st_.frees;
    st_.in_use -= b.size;
    if (b.pool > 0 && dead_.count(b.pool)) b.pool = 0;  // its graph is gone: back to the default pool
    const bool capt = capturing(b.stream);
    if ((capt || b.in_capture) && b.pool == 0) {
      // a default-pool block used by a capture outside any private pool (freed
      // during the capture, or handed out inside it): the graph may address it
      // on every replay, so it is never handed out again (nor returned to the
      // driver).  Model captures use private pools instead (memory.graph_pool)
      parked_.push_back(std::make_pair(p, b.size));
      return;
    }
    if (b.uses.empty()) {
      free_[std::make_tuple(b.pool, b.stream, b.size)].push_back(p);
      return;
    }
    if (capt || anyc(b.uses)) {  // cross-stream use inside a capture: keep it out of circulation with its pool
      held_[b.pool].push_back(std::make_pair(p, b.size));
      return;
    }
    Pending pd{p, b, {}};
    RelaxedCapture rc;
    for (uintptr_t s : b.uses) {
      hipEvent_t ev;
      hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
      hip_check(hipEventRecord(ev, (hipStream_t)s), "hipEventRecord");
      pd.evs.push_back(ev);
    }
    pending_.push_back(std::move(pd));
  }

  // the block containing ptr (a view may point inside it) is also used on stream s
  void record_stream(void* ptr, uintptr_t s) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.upper_bound(ptr);
    if (it == live_.begin()) return;
    --it;
    if ((char*)ptr >= (char*)it->first + it->second.size) return;  // not a pool block
    if (s == it->second.stream) return;
    for (uintptr_t u : it->second.uses)
      if (u == s) return;
    it->second.uses.push_back(s);
  }
  bool owns(void* ptr) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.upper_bound(ptr);
    if (it == live_.begin()) return false;
    --it;
    return (char*)ptr < (char*)it->first + it->second.size;
  }

  int new_pool() {
    std::lock_guard<std::mutex> g(mu_);
    return ++last_pool_;
  }
  // the graph of private pool id is destroyed: its cached blocks go back to
  // the driver, its live blocks (tensors that outlived the graph) rejoin the
  // default pool when they are freed
  void release_pool(int id) {
    if (id <= 0) return;
    std::lock_guard<std::mutex> g(mu_);
    dead_.insert(id);
    for (auto it = free_.begin(); it != free_.end();) {
      if (std::get<0>(it->first) == id) {
        for (void* q : it->second) driver_free_locked(q, std::get<2>(it->first));
        it = free_.erase(it);
      } else {
        ++it;
      }
    }
    auto h = held_.find(id);
    if (h != held_.end()) {
      for (auto& b : h->second) driver_free_locked(b.first, b.second);
      held_.erase(h);
    }
  }

  void release() {
    std::lock_guard<std::mutex> g(mu_);
    release_locked();
  }

  py::dict stats() {
    std::lock_guard<std::mutex> g(mu_);
    reap_locked();
    py::dict d;
    d["allocs"] = st_.allocs;
    d["frees"] = st_.frees;
    d["cache_hits"] = st_.hits;
    d["driver_allocs"] = st_.driver_allocs;
    d["in_use_bytes"] = st_.in_use;
    d["reserved_bytes"] = st_.reserved;
    d["peak_in_use_bytes"] = st_.peak_in_use;
    d["pending_frees"] = (uint64_t)pending_.size();
    d["parked_blocks"] = (uint64_t)parked_.size();
    d["live_blocks"] = (uint64_t)live_.size();
    return d;
  }
  void reset_peak() {
    std::lock_guard<std::mutex> g(mu_);
    st_.peak_in_use = st_.in_use;
  }
  int device() const { return dev_; }

 private:
  static bool capturing(uintptr_t s) {
    if (!s) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing((hipStream_t)s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
  }
  static bool anyc(const std::vector<uintptr_t>& v) {
    for (uintptr_t s : v)
      if (capturing(s)) return true;
    return false;
  }
  void* driver_alloc_locked(size_t sz) {
    RelaxedCapture rc;
    int cur = 0;
    hip_check(hipGetDevice(&cur), "hipGetDevice");
    if (cur != dev_) hip_check(hipSetDevice(dev_), "hipSetDevice");
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, sz);
    if (e != hipSuccess) {  // out of memory: drop the default pool's cache once and retry
      (void)hipGetLastError();
      release_locked();
      e = hipMalloc(&p, sz);
    }
    if (cur != dev_) hipSetDevice(cur);
    hip_check(e, "hipMalloc");
    ++st_.driver_allocs;
    st_.reserved += sz;
    return p;
  }
  void driver_free_locked(void* p, size_t sz) {
    RelaxedCapture rc;
    hipFree(p);
    st_.reserved -= sz;
  }
  void reap_locked() {
    if (pending_.empty()) return;
    RelaxedCapture rc;
    for (size_t i = 0; i < pending_.size();) {
      bool done = true;
      for (hipEvent_t ev : pending_[i].evs)
        if (hipEventQuery(ev) != hipSuccess) {
          done = false;
          break;
        }
      if (done) {
        for (hipEvent_t ev : pending_[i].evs) hipEventDestroy(ev);
        const BlockInfo& b = pending_[i].info;
        const int pool = (b.pool > 0 && dead_.count(b.pool)) ? 0 : b.pool;
        free_[std::make_tuple(pool, b.stream, b.size)].push_back(pending_[i].ptr);
        pending_[i] = std::move(pending_.back());
        pending_.pop_back();
      } else {
        ++i;
      }
    }
  }
  void release_locked() {  // the default pool's cached blocks (never parked / private ones)
    reap_locked();
    for (auto it = free_.begin(); it != free_.end();) {
      if (std::get<0>(it->first) == 0) {
        for (void* q : it->second) driver_free_locked(q, std::get<2>(it->first));
        it = free_.erase(it);
      } else {
        ++it;
      }
    }
  }

  int dev_;
  std::mutex mu_;
  std::map<std::tuple<int, uintptr_t, size_t>, std::vector<void*>> free_;
  std::map<void*, BlockInfo> live_;
  std::vector<Pending> pending_;
  std::vector<std::pair<void*, size_t>> parked_;
  std::map<int, std::vector<std::pair<void*, size_t>>> held_;
  std::set<int> dead_;
  int last_pool_ = 0;
  Stats st_;
};

class HostPool {
 public:
  explicit HostPool(bool pinned) : pinned_(pinned) {}
  void* alloc(size_t n) {
    const size_t sz = round_size(n);
    std::lock_guard<std::mutex> g(mu_);
    ++st_.allocs;
    void* p = nullptr;
    auto it = free_.find(sz);
    if (it != free_.end() && !it->second.empty()) {
      p = it->second.back();
      it->second.pop_back();
      ++st_.hits;
    } else {
      if (pinned_) {
        hip_check(hipHostMalloc(&p, sz, hipHostMallocDefault), "hipHostMalloc");
      } else if (posix_memalign(&p, 64, sz) != 0) {
        throw std::bad_alloc();
      }
      ++st_.driver_allocs;
      st_.reserved += sz;
    }
    sizes_[p] = sz;
    st_.in_use += sz;
    if (st_.in_use > st_.peak_in_use) st_.peak_in_use = st_.in_use;
    return p;
  }
  void free(void* p) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = sizes_.find(p);
    if (it == sizes_.end()) throw std::runtime_error("HostPool::free: pointer not from this pool");
    ++st_.frees;
    st_.in_use -= it->second;
    free_[it->second].push_back(p);
    sizes_.erase(it);
  }
  void release() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : free_)
      for (void* p : kv.second) {
        if (pinned_) hipHostFree(p);
        else ::free(p);
        st_.reserved -= kv.first;
      }
    free_.clear();
  }
  py::dict stats() {
    std::lock_guard<std::mutex> g(mu_);
    py::dict d;
    d["allocs"] = st_.allocs;
    d["frees"] = st_.frees;
    d["cache_hits"] = st_.hits;
    d["driver_allocs"] = st_.driver_allocs;
    d["in_use_bytes"] = st_.in_use;
    d["reserved_bytes"] = st_.reserved;
    d["peak_in_use_bytes"] = st_.peak_in_use;
    return d;
  }

 private:
  bool pinned_;
  std::mutex mu_;
  std::map<size_t, std::vector<void*>> free_;
  std::map<void*, size_t> sizes_;
  Stats st_;
};

// pools live for the whole process (freed blocks of tensors that outlive
// interpreter teardown must still find their pool)
std::mutex g_mu;
std::map<int, DevicePool*> g_dev;
HostPool* g_host[2] = {nullptr, nullptr};

DevicePool& dev_pool(int d) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_dev.find(d);
  if (it == g_dev.end()) it = g_dev.emplace(d, new DevicePool(d)).first;
  return *it->second;
}
HostPool& host_pool(bool pinned) {
  std::lock_guard<std::mutex> g(g_mu);
  HostPool*& h = g_host[pinned ? 1 : 0];
  if (!h) h = new HostPool(pinned);
  return *h;
}

struct Ctx {
  std::vector<int64_t> shape, strides;
  void* ptr;
  int kind;  // 0 device, 1 host pageable, 2 host pinned, 3 view (owned by `keep`)
  int dev;
  uintptr_t stream;
  std::shared_ptr<void> keep;
};

void dl_deleter(DLManagedTensor* self) {
  Ctx* c = (Ctx*)self->manager_ctx;
  try {
    if (c->kind == 0) dev_pool(c->dev).free(c->ptr);
    else if (c->kind == 1 || c->kind == 2) host_pool(c->kind == 2).free(c->ptr);
  } catch (...) {
  }
  delete c;
  delete self;
}

void capsule_dtor(PyObject* cap) {
  // an unconsumed capsule (never handed to a framework) still owns the block
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* m = (DLManagedTensor*)PyCapsule_GetPointer(cap, "dltensor");
    if (m && m->deleter) m->deleter(m);
  }
}

// dtype: (code, bits) -- code 0 int, 1 uint, 2 float, 4 bfloat
py::object make_capsule(std::vector<int64_t> shape, int code, int bits, int kind, int dev, int32_t dl_device_type,
                        uintptr_t stream, std::vector<int64_t> strides) {
  int64_t n = 1;
  for (int64_t s : shape) {
    if (s < 0) throw std::invalid_argument("negative dimension");
    n *= s;
  }
  if (!strides.empty() && strides.size() != shape.size()) throw std::invalid_argument("strides rank != shape rank");
  const size_t bytes = (size_t)n * (bits / 8);
  void* p = kind == 0 ? dev_pool(dev).alloc(bytes, stream) : host_pool(kind == 2).alloc(bytes);
  auto* c = new Ctx{shape, std::vector<int64_t>(shape.size()), p, kind, dev, stream, nullptr};
  if (!strides.empty()) {
    c->strides = strides;  // a dense permutation of the shape (e.g. NHWC memory of an NCHW view)
  } else {
    int64_t st = 1;
    for (int i = (int)shape.size() - 1; i >= 0; --i) {
      c->strides[i] = st;
      st *= shape[i];
    }
  }
  auto* m = new DLManagedTensor{};
  m->dl_tensor.data = p;
  m->dl_tensor.device = DLDevice{kind == 0 ? dl_device_type : kDLCPU, kind == 0 ? dev : 0};
  m->dl_tensor.ndim = (int32_t)shape.size();
  m->dl_tensor.dtype = DLDataType{(uint8_t)code, (uint8_t)bits, 1};
  m->dl_tensor.shape = c->shape.data();
  m->dl_tensor.strides = c->strides.data();
  m->dl_tensor.byte_offset = 0;
  m->manager_ctx = c;
  m->deleter = dl_deleter;
  return py::reinterpret_steal<py::object>(PyCapsule_New(m, "dltensor", capsule_dtor));
}

// --------------------------------------------------------------- SyncedBlob
// The reference's SyncedMemory (src/utils/blob.cc:83-143): one logical buffer
// with a host and a device copy allocated lazily from the pools and a head
// state saying which copy is current.  Reading a side syncs it from the other
// if needed (stream-ordered copies; the host read waits for its copy);
// taking a side for writing makes it the only valid one.  The device side
// may instead be an EXTERNAL region (e.g. a parameter's slice of the flat
// parameter store), which the blob mirrors but never frees.
class SyncedBlob : public std::enable_shared_from_this<SyncedBlob> {
 public:
  enum Head { UNINIT = 0, AT_CPU = 1, AT_GPU = 2, SYNCED = 3 };
  SyncedBlob(size_t bytes, int dev, uintptr_t ext, bool pinned)
      : bytes_(bytes), dev_(dev), d_((void*)ext), ext_(ext != 0), pinned_(pinned) {
    if (ext_) head_ = AT_GPU;  // the external region holds the data
  }
  ~SyncedBlob() {
    if (h_) host_pool(pinned_).free(h_);
    if (d_ && !ext_) dev_pool(dev_).free(d_);
  }
  uintptr_t cpu_ptr(uintptr_t stream) {
    to_cpu(stream);
    return (uintptr_t)h_;
  }
  uintptr_t gpu_ptr(uintptr_t stream) {
    to_gpu(stream);
    return (uintptr_t)d_;
  }
  uintptr_t mutable_cpu_ptr(uintptr_t stream) {
    to_cpu(stream);
    head_ = AT_CPU;
    return (uintptr_t)h_;
  }
  uintptr_t mutable_gpu_ptr(uintptr_t stream) {
    to_gpu(stream);
    head_ = AT_GPU;
    return (uintptr_t)d_;
  }
  int head() const { return head_; }
  size_t bytes() const { return bytes_; }

 private:
  void alloc_h() {
    if (!h_) h_ = host_pool(pinned_).alloc(bytes_);
  }
  void alloc_d() {
    if (!d_) d_ = dev_pool(dev_).alloc(bytes_, 0);
  }
  void to_cpu(uintptr_t stream) {
    if (head_ == UNINIT) {
      alloc_h();
      memset(h_, 0, bytes_);
      head_ = AT_CPU;
    } else if (head_ == AT_GPU) {
      alloc_h();
      hip_check(hipMemcpyAsync(h_, d_, bytes_, hipMemcpyDeviceToHost, (hipStream_t)stream), "hipMemcpyAsync D2H");
      hip_check(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
      head_ = SYNCED;
    }
  }
  void to_gpu(uintptr_t stream) {
    if (head_ == UNINIT) {
      alloc_d();
      hip_check(hipMemsetAsync(d_, 0, bytes_, (hipStream_t)stream), "hipMemsetAsync");
      head_ = AT_GPU;
    } else if (head_ == AT_CPU) {
      alloc_d();
      hip_check(hipMemcpyAsync(d_, h_, bytes_, hipMemcpyHostToDevice, (hipStream_t)stream), "hipMemcpyAsync H2D");
      head_ = SYNCED;
    }
  }
  size_t bytes_;
  int dev_;
  void* h_ = nullptr;
  void* d_ = nullptr;
  bool ext_, pinned_;
  int head_ = UNINIT;
};

// DLPack view of a blob side (the capsule keeps the blob alive)
py::object blob_view(std::shared_ptr<SyncedBlob> b, uintptr_t ptr, bool on_device, int dev, int32_t dl_type,
                     std::vector<int64_t> shape, int code, int bits) {
  auto* c = new Ctx{shape, std::vector<int64_t>(shape.size()), (void*)ptr, 3, dev, 0, b};
  int64_t st = 1;
  for (int i = (int)shape.size() - 1; i >= 0; --i) {
    c->strides[i] = st;
    st *= shape[i];
  }
  if ((size_t)st * (bits / 8) > b->bytes()) {
    delete c;
    throw std::invalid_argument("blob view larger than the blob");
  }
  auto* m = new DLManagedTensor{};
  m->dl_tensor.data = (void*)ptr;
  m->dl_tensor.device = DLDevice{on_device ? dl_type : kDLCPU, on_device ? dev : 0};
  m->dl_tensor.ndim = (int32_t)shape.size();
  m->dl_tensor.dtype = DLDataType{(uint8_t)code, (uint8_t)bits, 1};
  m->dl_tensor.shape = c->shape.data();
  m->dl_tensor.strides = c->strides.data();
  m->manager_ctx = c;
  m->deleter = dl_deleter;
  return py::reinterpret_steal<py::object>(PyCapsule_New(m, "dltensor", capsule_dtor));
}

// ------------------------------------------------------------ native Tensor
// The framework's tensor handle: the mshadow Tensor / Shape and Blob of the
// reference (include/mshadow/tensor.h:206-385 -- dptr, shape, stride;
// include/utils/blob.h:94-163 -- count, shape, data) over this file's pools.
// A Storage is one allocation (a pool block, or a foreign DLPack buffer the
// handle keeps alive); a Tensor is (storage, byte offset, shape, strides in
// elements, dtype, device).  Views (reshape, permute, slice, select, expand,
// squeeze / unsqueeze, as_strided) are metadata over the same storage; DLPack
// export hands the bytes to PyTorch / NumPy without a copy and keeps the
// storage alive for as long as the importer holds them.
struct Storage {
  void* ptr = nullptr;
  size_t bytes = 0;
  int kind = 0;  // 0 device pool, 1 host pageable pool, 2 host pinned pool, 3 foreign (DLPack import)
  int dev = 0;
  DLManagedTensor* foreign = nullptr;
  ~Storage() {
    try {
      if (kind == 0 && ptr) dev_pool(dev).free(ptr);
      else if ((kind == 1 || kind == 2) && ptr) host_pool(kind == 2).free(ptr);
      else if (kind == 3 && foreign && foreign->deleter) foreign->deleter(foreign);
    } catch (...) {
    }
  }
};

struct NTensor {
  std::shared_ptr<Storage> st;
  int64_t offset = 0;  // bytes from st->ptr
  std::vector<int64_t> shape, strides;
  int code = 2, bits = 32;
  int32_t dl_type = kDLCPU;
  int dev = 0;

  int64_t numel() const {
    int64_t n = 1;
    for (int64_t v : shape) n *= v;
    return n;
  }
  int itemsize() const { return bits / 8; }
  uintptr_t data_ptr() const { return (uintptr_t)st->ptr + offset; }
  static std::vector<int64_t> dense_strides(const std::vector<int64_t>& shape) {
    std::vector<int64_t> r(shape.size());
    int64_t st = 1;
    for (int i = (int)shape.size() - 1; i >= 0; --i) {
      r[i] = st;
      st *= shape[i];
    }
    return r;
  }
  bool is_contiguous() const {
    int64_t exp = 1;
    for (int i = (int)shape.size() - 1; i >= 0; --i) {
      if (shape[i] != 1 && strides[i] != exp) return false;
      exp *= shape[i];
    }
    return true;
  }
  bool is_channels_last() const {  // 4-D NCHW logical shape over dense NHWC memory
    if (shape.size() != 4) return false;
    const int64_t C = shape[1], H = shape[2], W = shape[3];
    return (C == 1 || strides[1] == 1) && (W == 1 || strides[3] == C) && (H == 1 || strides[2] == W * C) &&
           (shape[0] == 1 || strides[0] == H * W * C);
  }
  int norm_dim(int d, int rank) const {
    if (d < 0) d += rank;
    if (d < 0 || d >= rank) throw std::out_of_range("dimension out of range");
    return d;
  }
  NTensor view_of(std::vector<int64_t> shp, std::vector<int64_t> str, int64_t off) const {
    NTensor t = *this;
    t.shape = std::move(shp);
    t.strides = std::move(str);
    t.offset = off;
    return t;
  }
  // reshape: a view when the strides allow it (dense row-major layout), else an error
  NTensor reshape(std::vector<int64_t> shp) const {
    int64_t known = 1, infer = -1;
    for (size_t i = 0; i < shp.size(); ++i) {
      if (shp[i] == -1) {
        if (infer >= 0) throw std::invalid_argument("reshape: more than one -1");
        infer = (int64_t)i;
      } else {
        if (shp[i] < 0) throw std::invalid_argument("reshape: negative dimension");
        known *= shp[i];
      }
    }
    const int64_t n = numel();
    if (infer >= 0) {
      if (known == 0 || n % known) throw std::invalid_argument("reshape: cannot infer the -1 dimension");
      shp[infer] = n / known;
    } else if (known != n) {
      throw std::invalid_argument("reshape: element count changes");
    }
    if (!is_contiguous()) throw std::invalid_argument("reshape of a non-contiguous tensor: copy it first");
    return view_of(shp, dense_strides(shp), offset);
  }
  NTensor permute(std::vector<int> dims) const {
    const int r = (int)shape.size();
    if ((int)dims.size() != r) throw std::invalid_argument("permute: rank mismatch");
    std::vector<int64_t> shp(r), str(r);
    std::vector<bool> seen(r, false);
    for (int i = 0; i < r; ++i) {
      const int d = norm_dim(dims[i], r);
      if (seen[d]) throw std::invalid_argument("permute: repeated dimension");
      seen[d] = true;
      shp[i] = shape[d];
      str[i] = strides[d];
    }
    return view_of(shp, str, offset);
  }
  NTensor transpose(int a, int b) const {
    std::vector<int> dims(shape.size());
    for (size_t i = 0; i < dims.size(); ++i) dims[i] = (int)i;
    std::swap(dims[norm_dim(a, (int)shape.size())], dims[norm_dim(b, (int)shape.size())]);
    return permute(dims);
  }
  NTensor slice(int d, int64_t start, int64_t stop, int64_t step) const {
    d = norm_dim(d, (int)shape.size());
    if (step <= 0) throw std::invalid_argument("slice: step must be positive");
    const int64_t n = shape[d];
    if (start < 0) start += n;
    if (stop < 0) stop += n;
    start = std::min(std::max<int64_t>(start, 0), n);
    stop = std::min(std::max<int64_t>(stop, start), n);
    std::vector<int64_t> shp = shape, str = strides;
    shp[d] = (stop - start + step - 1) / step;
    str[d] = strides[d] * step;
    return view_of(shp, str, offset + start * strides[d] * itemsize());
  }
  NTensor select(int d, int64_t i) const {
    d = norm_dim(d, (int)shape.size());
    if (i < 0) i += shape[d];
    if (i < 0 || i >= shape[d]) throw std::out_of_range("select: index out of range");
    std::vector<int64_t> shp = shape, str = strides;
    shp.erase(shp.begin() + d);
    str.erase(str.begin() + d);
    return view_of(shp, str, offset + i * strides[d] * itemsize());
  }
  NTensor unsqueeze(int d) const {
    const int r = (int)shape.size() + 1;
    if (d < 0) d += r;
    if (d < 0 || d >= r) throw std::out_of_range("unsqueeze: dimension out of range");
    std::vector<int64_t> shp = shape, str = strides;
    const int64_t s = d < (int)shape.size() ? strides[d] * shape[d] : 1;
    shp.insert(shp.begin() + d, 1);
    str.insert(str.begin() + d, s);
    return view_of(shp, str, offset);
  }
  NTensor squeeze(int d) const {
    d = norm_dim(d, (int)shape.size());
    if (shape[d] != 1) return *this;
    std::vector<int64_t> shp = shape, str = strides;
    shp.erase(shp.begin() + d);
    str.erase(str.begin() + d);
    return view_of(shp, str, offset);
  }
  NTensor expand(std::vector<int64_t> shp) const {  // broadcast size-1 (or new leading) dims with stride 0
    if (shp.size() < shape.size()) throw std::invalid_argument("expand: fewer dimensions");
    const size_t lead = shp.size() - shape.size();
    std::vector<int64_t> str(shp.size(), 0);
    for (size_t i = 0; i < shp.size(); ++i) {
      if (i < lead) {
        if (shp[i] < 0) throw std::invalid_argument("expand: -1 for a new dimension");
        continue;
      }
      const int64_t cur = shape[i - lead];
      if (shp[i] == -1) shp[i] = cur;
      if (cur == shp[i]) str[i] = strides[i - lead];
      else if (cur != 1) throw std::invalid_argument("expand: only size-1 dimensions broadcast");
    }
    return view_of(shp, str, offset);
  }
  NTensor as_strided(std::vector<int64_t> shp, std::vector<int64_t> str, int64_t elem_offset) const {
    if (shp.size() != str.size()) throw std::invalid_argument("as_strided: rank mismatch");
    int64_t hi = elem_offset;  // the largest element reached must lie inside the storage
    for (size_t i = 0; i < shp.size(); ++i) {
      if (shp[i] < 0 || str[i] < 0) throw std::invalid_argument("as_strided: negative size / stride");
      if (shp[i] > 0) hi += (shp[i] - 1) * str[i];
    }
    if (elem_offset < 0 || (size_t)(hi + 1) * itemsize() > st->bytes)
      throw std::out_of_range("as_strided: view outside the storage");
    return view_of(shp, str, elem_offset * itemsize());
  }
  py::object to_dlpack() const {
    auto* c = new Ctx{shape, strides, (void*)data_ptr(), 3, dev, 0, st};
    auto* m = new DLManagedTensor{};
    m->dl_tensor.data = (void*)data_ptr();
    m->dl_tensor.device = DLDevice{dl_type, dl_type == kDLCPU ? 0 : dev};
    m->dl_tensor.ndim = (int32_t)shape.size();
    m->dl_tensor.dtype = DLDataType{(uint8_t)code, (uint8_t)bits, 1};
    m->dl_tensor.shape = c->shape.data();
    m->dl_tensor.strides = c->strides.data();
    m->dl_tensor.byte_offset = 0;
    m->manager_ctx = c;
    m->deleter = dl_deleter;
    return py::reinterpret_steal<py::object>(PyCapsule_New(m, "dltensor", capsule_dtor));
  }
};

NTensor ntensor_empty(std::vector<int64_t> shape, int code, int bits, int kind, int dev, int32_t dl_device_type,
                      uintptr_t stream, bool channels_last) {
  if (bits % 8 || bits <= 0) throw std::invalid_argument("dtype bits must be a positive multiple of 8");
  NTensor t;
  t.shape = shape;
  for (int64_t v : shape)
    if (v < 0) throw std::invalid_argument("negative dimension");
  const size_t bytes = (size_t)t.numel() * (bits / 8);
  auto st = std::make_shared<Storage>();
  st->kind = kind;
  st->dev = dev;
  st->bytes = bytes;
  st->ptr = kind == 0 ? dev_pool(dev).alloc(bytes, stream) : host_pool(kind == 2).alloc(bytes);
  t.st = st;
  t.code = code;
  t.bits = bits;
  t.dev = kind == 0 ? dev : 0;
  t.dl_type = kind == 0 ? dl_device_type : kDLCPU;
  if (channels_last && shape.size() == 4) {
    const int64_t C = shape[1], H = shape[2], W = shape[3];
    t.strides = {H * W * C, 1, W * C, C};
  } else {
    t.strides = NTensor::dense_strides(shape);
  }
  return t;
}

// import a DLPack capsule (any producer): the handle owns the managed tensor
// and calls its deleter when the last view of the storage dies
NTensor ntensor_from_dlpack(py::capsule cap) {
  PyObject* o = cap.ptr();
  if (!PyCapsule_IsValid(o, "dltensor")) throw std::invalid_argument("not an unconsumed DLPack capsule");
  auto* m = (DLManagedTensor*)PyCapsule_GetPointer(o, "dltensor");
  PyCapsule_SetName(o, "used_dltensor");  // consumed: the capsule destructor no longer frees it
  const DLTensor& d = m->dl_tensor;
  NTensor t;
  t.shape.assign(d.shape, d.shape + d.ndim);
  t.strides = d.strides ? std::vector<int64_t>(d.strides, d.strides + d.ndim) : NTensor::dense_strides(t.shape);
  t.code = d.dtype.code;
  t.bits = d.dtype.bits * (d.dtype.lanes ? d.dtype.lanes : 1);
  t.dl_type = d.device.device_type;
  t.dev = d.device.device_id;
  auto st = std::make_shared<Storage>();
  st->kind = 3;
  st->foreign = m;
  st->ptr = (char*)d.data + d.byte_offset;
  int64_t hi = 0;
  for (int i = 0; i < d.ndim; ++i)
    if (t.shape[i] > 0) hi += (t.shape[i] - 1) * t.strides[i];
  st->bytes = t.numel() ? (size_t)(hi + 1) * t.itemsize() : 0;
  st->dev = t.dev;
  t.st = st;
  return t;
}

}  // namespace

void register_mem(py::module& m) {
  py::module_ mm = m.def_submodule("mem", "native device / host memory pools (DLPack-exported blocks)");
  mm.def("empty", &make_capsule, py::arg("shape"), py::arg("code"), py::arg("bits"), py::arg("kind"),
         py::arg("device") = 0, py::arg("dl_device_type") = 10, py::arg("stream") = 0,
         py::arg("strides") = std::vector<int64_t>(),
         "allocate a dense block from a pool (stream-ordered on `stream`) and return a DLPack capsule owning it");
  mm.def("device_stats", [](int d) { return dev_pool(d).stats(); });
  mm.def("reset_peak", [](int d) { dev_pool(d).reset_peak(); });
  mm.def("record_stream", [](int d, uintptr_t ptr, uintptr_t s) { dev_pool(d).record_stream((void*)ptr, s); });
  mm.def("owns", [](int d, uintptr_t ptr) { return dev_pool(d).owns((void*)ptr); });
  mm.def("new_pool", [](int d) { return dev_pool(d).new_pool(); });
  mm.def("release_pool", [](int d, int id) { dev_pool(d).release_pool(id); });
  mm.def("set_pool", [](int id) {
    const int prev = t_pool;
    t_pool = id;
    return prev;
  }, "this thread's allocations go to private pool `id` (0: default); returns the previous id");
  mm.def("host_stats", [](bool pinned) { return host_pool(pinned).stats(); }, py::arg("pinned") = false);
  mm.def("empty_cache", [](int d) { dev_pool(d).release(); });
  mm.def("empty_host_cache", [](bool pinned) { host_pool(pinned).release(); }, py::arg("pinned") = false);
  py::class_<SyncedBlob, std::shared_ptr<SyncedBlob>>(mm, "SyncedBlob")
      .def(py::init<size_t, int, uintptr_t, bool>(), py::arg("bytes"), py::arg("device") = 0, py::arg("ext") = 0,
           py::arg("pinned") = true)
      .def("cpu_ptr", &SyncedBlob::cpu_ptr, py::arg("stream") = 0, py::call_guard<py::gil_scoped_release>())
      .def("gpu_ptr", &SyncedBlob::gpu_ptr, py::arg("stream") = 0)
      .def("mutable_cpu_ptr", &SyncedBlob::mutable_cpu_ptr, py::arg("stream") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("mutable_gpu_ptr", &SyncedBlob::mutable_gpu_ptr, py::arg("stream") = 0)
      .def_property_readonly("head", &SyncedBlob::head)
      .def_property_readonly("bytes", &SyncedBlob::bytes);
  mm.def("blob_view", &blob_view, py::arg("blob"), py::arg("ptr"), py::arg("on_device"), py::arg("device"),
         py::arg("dl_device_type"), py::arg("shape"), py::arg("code"), py::arg("bits"));
  py::class_<NTensor>(mm, "Tensor", "framework-owned tensor handle: pool storage + offset, shape, strides, dtype, device")
      .def_static("empty", &ntensor_empty, py::arg("shape"), py::arg("code"), py::arg("bits"), py::arg("kind"),
                  py::arg("device") = 0, py::arg("dl_device_type") = 10, py::arg("stream") = 0,
                  py::arg("channels_last") = false)
      .def_static("from_dlpack", &ntensor_from_dlpack, py::arg("capsule"))
      .def_property_readonly("shape", [](const NTensor& t) { return py::tuple(py::cast(t.shape)); })
      .def_property_readonly("strides", [](const NTensor& t) { return py::tuple(py::cast(t.strides)); })
      .def_property_readonly("ndim", [](const NTensor& t) { return (int)t.shape.size(); })
      .def_property_readonly("dtype", [](const NTensor& t) { return py::make_tuple(t.code, t.bits); })
      .def_property_readonly("device", [](const NTensor& t) { return py::make_tuple(t.dl_type, t.dev); })
      .def_property_readonly("offset", [](const NTensor& t) { return t.offset; })
      .def_property_readonly("itemsize", &NTensor::itemsize)
      .def_property_readonly("storage_bytes", [](const NTensor& t) { return t.st->bytes; })
      .def_property_readonly("storage_kind", [](const NTensor& t) { return t.st->kind; })
      .def_property_readonly("storage_refs", [](const NTensor& t) { return (long)t.st.use_count(); })
      .def("numel", &NTensor::numel)
      .def("nbytes", [](const NTensor& t) { return t.numel() * t.itemsize(); })
      .def("data_ptr", &NTensor::data_ptr)
      .def("is_contiguous", &NTensor::is_contiguous)
      .def("is_channels_last", &NTensor::is_channels_last)
      .def("same_storage", [](const NTensor& a, const NTensor& b) { return a.st == b.st; })
      .def("reshape", &NTensor::reshape)
      .def("permute", &NTensor::permute)
      .def("transpose", &NTensor::transpose)
      .def("slice", &NTensor::slice, py::arg("dim"), py::arg("start"), py::arg("stop"), py::arg("step") = 1)
      .def("select", &NTensor::select)
      .def("unsqueeze", &NTensor::unsqueeze)
      .def("squeeze", &NTensor::squeeze)
      .def("expand", &NTensor::expand)
      .def("as_strided", &NTensor::as_strided, py::arg("shape"), py::arg("strides"), py::arg("offset") = 0)
      .def("to_dlpack", &NTensor::to_dlpack)
      .def("__dlpack__", [](const NTensor& t, py::object) { return t.to_dlpack(); }, py::arg("stream") = py::none())
      .def("__dlpack_device__", [](const NTensor& t) { return py::make_tuple(t.dl_type, t.dl_type == kDLCPU ? 0 : t.dev); });
  mm.def("dl_device_type", [](py::capsule cap) {
    auto* t = (DLManagedTensor*)PyCapsule_GetPointer(cap.ptr(), PyCapsule_GetName(cap.ptr()));
    if (!t) throw std::runtime_error("not a DLPack capsule");
    return t->dl_tensor.device.device_type;
  });
}

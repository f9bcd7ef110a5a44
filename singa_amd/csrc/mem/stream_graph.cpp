// Framework-owned HIP streams, events and graphs.
//
// Reference counterparts: the reference has no device streams at all (its
// CUDA path was compiled out, include/mshadow/tensor_gpu-inl.hpp:26-93 only
// initialised a device); its only overlap machinery was the ZeroMQ actor
// threads.  Here the runtime owns:
//   * Stream -- hipStreamCreateWithPriority (non-blocking); the communicator's
//     comm stream is one of these (high priority);
//   * Event  -- hipEventCreateWithFlags (timing optional): record / wait /
//     query / synchronize / elapsed_ms -- the fork / join of bucketed
//     all-reduces and the exposed-communication timers;
//   * Graph  -- a training step captured with hipStreamBeginCapture on a
//     framework stream (thread-local capture mode), instantiated once and
//     replayed with hipGraphLaunch: the executor of Model(use_graph=True).
// Handles are plain integers to Python (uintptr_t hipStream_t / hipEvent_t),
// so the kernels' launchers take them like any other stream.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void hchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

class Stream {
 public:
  Stream(int device, int priority) : dev_(device) {
    int cur = 0;
    hchk(hipGetDevice(&cur), "hipGetDevice");
    if (cur != device) hchk(hipSetDevice(device), "hipSetDevice");
    hipError_t e = hipStreamCreateWithPriority(&s_, hipStreamNonBlocking, priority);
    if (cur != device) hipSetDevice(cur);
    hchk(e, "hipStreamCreateWithPriority");
  }
  // never destroyed: a handle may live on in another runtime's bookkeeping
  // (PyTorch's allocator keeps the streams a tensor was record_stream'ed on
  // and records events there when the tensor dies, possibly long after this
  // object); streams are few and created once per role
  ~Stream() = default;
  uintptr_t handle() const { return (uintptr_t)s_; }
  int device() const { return dev_; }
  void synchronize() {
    py::gil_scoped_release nogil;
    hchk(hipStreamSynchronize(s_), "hipStreamSynchronize");
  }
  bool query() { return hipStreamQuery(s_) == hipSuccess; }

 private:
  hipStream_t s_ = nullptr;
  int dev_;
};

class Event {
 public:
  explicit Event(bool timing) {
    hchk(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming), "hipEventCreate");
  }
  ~Event() {
    if (e_) hipEventDestroy(e_);
  }
  uintptr_t handle() const { return (uintptr_t)e_; }
  void record(uintptr_t s) { hchk(hipEventRecord(e_, (hipStream_t)s), "hipEventRecord"); }
  // stream s waits (on the device) until the work this event captured is done
  void wait(uintptr_t s) { hchk(hipStreamWaitEvent((hipStream_t)s, e_, 0), "hipStreamWaitEvent"); }
  bool query() { return hipEventQuery(e_) == hipSuccess; }
  void synchronize() {
    py::gil_scoped_release nogil;
    hchk(hipEventSynchronize(e_), "hipEventSynchronize");
  }
  float elapsed_ms(const Event& end) {
    float ms = 0.f;
    hchk(hipEventElapsedTime(&ms, e_, end.e_), "hipEventElapsedTime");
    return ms;
  }

 private:
  hipEvent_t e_ = nullptr;
};

class Graph {
 public:
  Graph() = default;
  ~Graph() { reset(); }
  // capture everything enqueued on stream s (and on streams forked from it
  // through events) by THIS thread until end()
  // mode: 1 thread-local (the default), 2 relaxed (a capture that several
  // threads enqueue into -- the loopback world's rank threads), 0 global
  void begin(uintptr_t s, int mode) {
    if (capturing_) throw std::runtime_error("Graph.begin: already capturing");
    reset();
    const hipStreamCaptureMode m = mode == 0   ? hipStreamCaptureModeGlobal
                                   : mode == 2 ? hipStreamCaptureModeRelaxed
                                               : hipStreamCaptureModeThreadLocal;
    hchk(hipStreamBeginCapture((hipStream_t)s, m), "hipStreamBeginCapture");
    s_ = (hipStream_t)s;
    capturing_ = true;
  }
  void end() {
    if (!capturing_) throw std::runtime_error("Graph.end: not capturing");
    capturing_ = false;
    hipGraph_t g = nullptr;
    static const bool dbg = [] {
      const char* e = getenv("SG_LOOP_DEBUG");
      return e && e[0] == '1';
    }();
    if (dbg) fprintf(stderr, "[graph] end capture\n");
    hchk(hipStreamEndCapture(s_, &g), "hipStreamEndCapture");
    g_ = g;
    if (dbg) {
      size_t n = 0;
      (void)hipGraphGetNodes(g_, nullptr, &n);
      fprintf(stderr, "[graph] captured %zu nodes; instantiate\n", n);
    }
    hchk(hipGraphInstantiate(&exec_, g_, nullptr, nullptr, 0), "hipGraphInstantiate");
    if (dbg) fprintf(stderr, "[graph] instantiated\n");
    size_t n = 0;
    hchk(hipGraphGetNodes(g_, nullptr, &n), "hipGraphGetNodes");
    nodes_ = n;
  }
  // abandon a capture that failed midway (the stream leaves capture mode)
  void abort() {
    if (!capturing_) return;
    capturing_ = false;
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(s_, &g);
    if (g) hipGraphDestroy(g);
    (void)hipGetLastError();
  }
  void replay(uintptr_t s) {
    if (!exec_) throw std::runtime_error("Graph.replay: nothing captured");
    hchk(hipGraphLaunch(exec_, (hipStream_t)s), "hipGraphLaunch");
  }
  size_t nodes() const { return nodes_; }
  bool ready() const { return exec_ != nullptr; }
  void reset() {
    if (exec_) hipGraphExecDestroy(exec_);
    if (g_) hipGraphDestroy(g_);
    exec_ = nullptr;
    g_ = nullptr;
    nodes_ = 0;
  }

 private:
  hipStream_t s_ = nullptr;
  hipGraph_t g_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  size_t nodes_ = 0;
  bool capturing_ = false;
};

// Framework-owned current stream, per thread and device: set by
// singa_amd.stream.Stream's context manager, read by every kernel launcher
// (ops/native.py stream()).  -1 = not set: the launchers then follow the
// caller's PyTorch current stream (tests that drive work on torch streams).
constexpr int kMaxDev = 16;
thread_local intptr_t t_cur[kMaxDev] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};

}  // namespace

void register_stream_graph(py::module& m) {
  py::module_ sm = m.def_submodule("rt", "framework-owned HIP streams, events and graphs");
  py::class_<Stream>(sm, "Stream")
      .def(py::init<int, int>(), py::arg("device") = 0, py::arg("priority") = 0)
      .def_property_readonly("handle", &Stream::handle)
      .def_property_readonly("device", &Stream::device)
      .def("synchronize", &Stream::synchronize)
      .def("query", &Stream::query);
  py::class_<Event>(sm, "Event")
      .def(py::init<bool>(), py::arg("timing") = false)
      .def_property_readonly("handle", &Event::handle)
      .def("record", &Event::record)
      .def("wait", &Event::wait)
      .def("query", &Event::query)
      .def("synchronize", &Event::synchronize)
      .def("elapsed_ms", &Event::elapsed_ms);
  py::class_<Graph>(sm, "Graph")
      .def(py::init<>())
      .def("begin", &Graph::begin, py::arg("stream"), py::arg("mode") = 1)
      .def("end", &Graph::end)
      .def("abort", &Graph::abort)
      .def("replay", &Graph::replay)
      .def("reset", &Graph::reset)
      .def_property_readonly("nodes", &Graph::nodes)
      .def_property_readonly("ready", &Graph::ready);
  sm.def("stream_priority_range", []() {
    int lo = 0, hi = 0;
    hchk(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    return py::make_tuple(lo, hi);
  });
  // current stream / device of this thread (framework state, no PyTorch query)
  sm.def("set_current", [](int device, intptr_t handle) {
    if (device < 0 || device >= kMaxDev) throw std::runtime_error("rt.set_current: device out of range");
    const intptr_t old = t_cur[device];
    t_cur[device] = handle;
    return old;
  });
  // (the device is hipGetDevice's every time, ~50 ns: PyTorch's set_device
  // and the runtime's own calls change it, so it is never cached)
  sm.def("current", [](int device) -> intptr_t {
    if (device < 0 && hipGetDevice(&device) != hipSuccess) return -1;
    return device < kMaxDev ? t_cur[device] : -1;
  });
  sm.def("get_device", []() {
    int d = 0;
    hchk(hipGetDevice(&d), "hipGetDevice");
    return d;
  });
  sm.def("set_device", [](int device) { hchk(hipSetDevice(device), "hipSetDevice"); });
  sm.def("device_synchronize", [](int device) {
    int cur = 0;
    hchk(hipGetDevice(&cur), "hipGetDevice");
    if (device >= 0 && device != cur) hchk(hipSetDevice(device), "hipSetDevice");
    hipError_t e;
    {
      py::gil_scoped_release nogil;
      e = hipDeviceSynchronize();
    }
    if (device >= 0 && device != cur) (void)hipSetDevice(cur);
    hchk(e, "hipDeviceSynchronize");
  });
  // host <-> device copies ordered on stream s; the call returns when the
  // copy is complete (the host side may be pageable memory owned by the caller)
  sm.def("memcpy_d2h", [](uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t s) {
    py::gil_scoped_release nogil;
    hchk(hipMemcpyAsync((void*)dst, (const void*)src, bytes, hipMemcpyDeviceToHost, (hipStream_t)s), "hipMemcpyAsync D2H");
    hchk(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize");
  });
  sm.def("memcpy_h2d", [](uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t s) {
    py::gil_scoped_release nogil;
    hchk(hipMemcpyAsync((void*)dst, (const void*)src, bytes, hipMemcpyHostToDevice, (hipStream_t)s), "hipMemcpyAsync H2D");
    hchk(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize");
  });
  sm.def("is_capturing", [](uintptr_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hchk(hipStreamIsCapturing((hipStream_t)s, &cs), "hipStreamIsCapturing");
    return cs != hipStreamCaptureStatusNone;
  });
}

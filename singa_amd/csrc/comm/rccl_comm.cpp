// Native RCCL communicator (one process per GPU, collectives over xGMI).
//
// Replaces the reference's transport -- the ZeroMQ Router with its PING/PONG
// rendezvous (src/utils/router.cc:16-123) and the ParamManager's per-param
// Put / Get / Sync messages (src/utils/param_manager.cc:103-234) -- with
// direct RCCL calls: the unique id travels through the rendezvous store
// (Python side), every collective is enqueued on the HIP stream the caller
// passes (a dedicated comm stream for overlap, or the compute stream inside
// a captured HIP graph), and nothing here goes through torch.distributed.
//
// Exposed to Python (module _C) as RcclComm + rccl_unique_id(); the
// Python wrapper (singa_amd/parallel/rccl.py) owns streams / events.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

// dtype codes shared with singa_amd/ops/native.py (F32, BF16, F16, I32, I64, U8)
ncclDataType_t dtype_of(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
    case 6: return ncclFloat64;
  }
  throw std::runtime_error("RCCL: unsupported dtype code " + std::to_string(dt));
}

ncclRedOp_t op_of(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
  }
  throw std::runtime_error("RCCL: unsupported reduction op " + std::to_string(op));
}

typedef uintptr_t P;
#define VP(x) ((void*)(x))
#define CVP(x) ((const void*)(x))
#define ST(x) ((hipStream_t)(x))

class RcclComm {
 public:
  RcclComm(py::bytes uid, int nranks, int rank, int device) : nranks_(nranks), rank_(rank) {
    std::string s = uid;
    if (s.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RCCL: unique id must be 128 bytes");
    ncclUniqueId id;
    memcpy(&id, s.data(), sizeof(id));
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("RCCL: hipSetDevice failed");
    py::gil_scoped_release nogil;  // blocks until every rank joined
    check(ncclCommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
  }
  explicit RcclComm(ncclComm_t c, int nranks, int rank) : comm_(c), nranks_(nranks), rank_(rank) {}
  ~RcclComm() {
    if (comm_) ncclCommDestroy(comm_);
  }

  int nranks() const { return nranks_; }
  int rank() const { return rank_; }

  void all_reduce(P send, P recv, size_t count, int dt, int op, P s) {
    check(ncclAllReduce(CVP(send), VP(recv), count, dtype_of(dt), op_of(op), comm_, ST(s)), "AllReduce");
  }
  void reduce_scatter(P send, P recv, size_t recvcount, int dt, int op, P s) {
    check(ncclReduceScatter(CVP(send), VP(recv), recvcount, dtype_of(dt), op_of(op), comm_, ST(s)), "ReduceScatter");
  }
  void all_gather(P send, P recv, size_t sendcount, int dt, P s) {
    check(ncclAllGather(CVP(send), VP(recv), sendcount, dtype_of(dt), comm_, ST(s)), "AllGather");
  }
  void broadcast(P send, P recv, size_t count, int dt, int root, P s) {
    check(ncclBroadcast(CVP(send), VP(recv), count, dtype_of(dt), root, comm_, ST(s)), "Broadcast");
  }
  void reduce(P send, P recv, size_t count, int dt, int op, int root, P s) {
    check(ncclReduce(CVP(send), VP(recv), count, dtype_of(dt), op_of(op), root, comm_, ST(s)), "Reduce");
  }
  void all_to_all(P send, P recv, size_t count, int dt, P s) {
    check(ncclAllToAll(CVP(send), VP(recv), count, dtype_of(dt), comm_, ST(s)), "AllToAll");
  }
  void send(P buf, size_t count, int dt, int peer, P s) {
    check(ncclSend(CVP(buf), count, dtype_of(dt), peer, comm_, ST(s)), "Send");
  }
  void recv(P buf, size_t count, int dt, int peer, P s) {
    check(ncclRecv(VP(buf), count, dtype_of(dt), peer, comm_, ST(s)), "Recv");
  }
  // color < 0: this rank joins no sub-communicator (returns None)
  RcclComm* split(int color, int key) {
    ncclComm_t nc = nullptr;
    {
      py::gil_scoped_release nogil;
      check(ncclCommSplit(comm_, color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &nc, nullptr), "CommSplit");
    }
    if (!nc) return nullptr;
    int n = 0, r = 0;
    check(ncclCommCount(nc, &n), "CommCount");
    check(ncclCommUserRank(nc, &r), "CommUserRank");
    return new RcclComm(nc, n, r);
  }
  std::string async_error() {
    ncclResult_t e = ncclSuccess;
    check(ncclCommGetAsyncError(comm_, &e), "CommGetAsyncError");
    return e == ncclSuccess ? std::string() : std::string(ncclGetErrorString(e));
  }
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  void destroy() {
    if (comm_) {
      py::gil_scoped_release nogil;
      ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
  }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
};

}  // namespace

void register_rccl(py::module& m) {
  m.def("rccl_unique_id", []() {
    ncclUniqueId id;
    check(ncclGetUniqueId(&id), "GetUniqueId");
    return py::bytes(id.internal, sizeof(id.internal));
  });
  m.def("rccl_version", []() {
    int v = 0;
    check(ncclGetVersion(&v), "GetVersion");
    return v;
  });
  m.def("rccl_group_start", []() { check(ncclGroupStart(), "GroupStart"); });
  m.def("rccl_group_end", []() { check(ncclGroupEnd(), "GroupEnd"); });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<py::bytes, int, int, int>(), py::arg("uid"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"))
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("rank", &RcclComm::rank)
      .def("all_reduce", &RcclComm::all_reduce)
      .def("reduce_scatter", &RcclComm::reduce_scatter)
      .def("all_gather", &RcclComm::all_gather)
      .def("broadcast", &RcclComm::broadcast)
      .def("reduce", &RcclComm::reduce)
      .def("all_to_all", &RcclComm::all_to_all)
      .def("send", &RcclComm::send)
      .def("recv", &RcclComm::recv)
      .def_static("group_start", []() { check(ncclGroupStart(), "GroupStart"); })
      .def_static("group_end", []() { check(ncclGroupEnd(), "GroupEnd"); })
      .def("split", &RcclComm::split, py::return_value_policy::take_ownership)
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort)
      .def("destroy", &RcclComm::destroy);
}

// Loopback communicator: N ranks as N threads of ONE process, behind the
// exact call surface of the native RCCL binding (RcclComm: pointer, count,
// dtype code, op code, stream).  It lets the real Python wrapper
// (singa_amd/parallel/rccl.py RcclCommunicator), DistOpt's buckets (fp32 and
// bf16 staging), the sharded EASGD centre and the pipeline bridges run at
// world sizes 2..8 on ONE GPU -- or on host memory in CPU CI -- before an
// 8-GPU node is available.  The reference exercised its exchange only as
// real multi-process traffic (src/utils/param_manager.cc:103-234,
// src/server/server.cc:45-214); this is the in-process rehearsal of the
// RCCL replacement.
//
// Semantics (chosen to be at least as strict as RCCL's):
//   * collectives: every rank of a group calls the same sequence; each call
//     is synchronous -- the caller's stream is drained before its send buffer
//     is read (device mode), peers' inputs are read between two group
//     barriers, and each rank writes only its own receive buffer after the
//     second barrier (so in-place calls are safe);
//   * point-to-point: an ungrouped send is a RENDEZVOUS -- it returns only
//     after the matching receive consumed it (RCCL's large-message
//     behaviour), so two ranks that both send before they receive deadlock
//     here as they would on RCCL (reported as a timeout, not a hang);
//     inside group_start()/group_end() the sends are deposited first, then
//     the receives complete, then the sends are awaited -- the grouped
//     pairing that makes crossing 1F1B exchanges safe;
//   * abort() (any rank) fails every waiter of the world immediately.
// Device mode (device >= 0) moves data with stream-ordered copies on the
// caller's stream followed by a stream synchronize; host mode (device < 0)
// reads and writes host pointers directly.  Reductions run on the host in
// rank order (deterministic), fp32 accumulation for 16/32-bit floats.
//
// Captured mode: when the caller's stream is being captured -- every rank
// thread capturing its training step into ONE HIP graph (parallel/loop.py
// WorldGraph) -- nothing can run or be waited for, so an all-reduce becomes a
// graph node instead.  The world's ranks all enqueue onto the capture's one
// origin stream (a rank thread's compute AND comm stream, while it captures),
// so stream order is the dependency: once every rank has reached the
// collective (a barrier: all their earlier work is enqueued) group rank 0
// enqueues one device reduction over every rank's buffers
// (kernels/loopred.hip), and a second barrier keeps any rank's later work
// behind it.  (Cross-stream waits between the ranks' side streams were the
// first design; this HIP runtime's hipStreamEndCapture crashes on a capture in
// which two non-origin streams wait on each other's events --
// tools/capture_threads_probe.py xrank1 -- while the real N > 1 pattern, one
// comm stream forked from and joined to the capture stream once per bucket,
// captures and replays correctly: tests/test_captured_world_gpu.py.)  Every
// HIP call of this path is made with the Python GIL held, which serialises it
// with the other rank threads' launches into the shared capture.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

namespace py = pybind11;

extern "C" int sg_loop_allreduce(const void* const* sends, void* const* recvs, int n, int64_t count, int dt, int op,
                                 hipStream_t s);

namespace {

typedef uintptr_t P;

size_t dt_size(int dt) {
  switch (dt) {
    case 0: case 3: return 4;
    case 1: case 2: return 2;
    case 4: case 6: return 8;
    case 5: return 1;
  }
  throw std::runtime_error("LoopComm: unsupported dtype code " + std::to_string(dt));
}

float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint16_t f_to_bf16(float f) {  // round to nearest even (NaN kept quiet)
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct Group;

struct World {
  explicit World(int n, double timeout_s) : n(n), timeout_s(timeout_s) {}
  int n;
  double timeout_s;
  std::mutex mu;
  std::condition_variable cv;
  std::string aborted;  // non-empty: every waiter fails with this reason
  // p2p mailboxes keyed (global src, global dst)
  struct Msg {
    std::vector<char> data;
    bool consumed = false;
  };
  std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> boxes;
  std::map<std::tuple<const void*, long, int>, std::shared_ptr<Group>> splits;  // (parent, split seq, color)

  template <class Pred>
  void wait(std::unique_lock<std::mutex>& lk, Pred pred, const char* what) {
    const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    while (!pred()) {
      if (!aborted.empty()) throw std::runtime_error(std::string("LoopComm ") + what + ": aborted (" + aborted + ")");
      if (cv.wait_until(lk, end) == std::cv_status::timeout && !pred())
        throw std::runtime_error(std::string("LoopComm ") + what + ": timed out after " +
                                 std::to_string(timeout_s) + " s (deadlock or a missing peer)");
    }
    if (!aborted.empty()) throw std::runtime_error(std::string("LoopComm ") + what + ": aborted (" + aborted + ")");
  }
};

struct Slot {
  P send = 0, recv = 0;
  size_t count = 0;
  int dt = 0, op = 0, root = 0, kind = 0;
  long color = 0, key = 0;
};

// the ranks of one communicator (the world or a split of it)
struct Group {
  Group(std::vector<int> g) : members(std::move(g)), slots(members.size()) {}
  std::vector<int> members;  // global ranks, group order
  std::vector<Slot> slots;

  int arrived = 0;
  long gen = 0;
  long splits = 0;
  // generation barrier over the group (caller holds the world lock)
  void barrier(World& w, std::unique_lock<std::mutex>& lk, const char* what) {
    const long g = gen;
    if (++arrived == (int)members.size()) {
      arrived = 0;
      ++gen;
      w.cv.notify_all();
      return;
    }
    w.wait(lk, [&] { return gen != g; }, what);
  }
};

thread_local int t_group_depth = 0;
struct PendingP2P {
  bool is_send;
  class LoopComm* c;
  P buf;
  size_t count;
  int dt, peer;
  P stream;
};
thread_local std::vector<PendingP2P> t_pending;

class LoopComm {
 public:
  LoopComm(std::shared_ptr<World> w, std::shared_ptr<Group> g, int rank, int device)
      : w_(std::move(w)), g_(std::move(g)), rank_(rank), dev_(device) {}

  int nranks() const { return (int)g_->members.size(); }
  int rank() const { return rank_; }
  int device() const { return dev_; }

  // ------------------------------------------------------------- data moves
  void sync(P s) {
    if (dev_ >= 0 && hipStreamSynchronize((hipStream_t)s) != hipSuccess)
      throw std::runtime_error("LoopComm: hipStreamSynchronize failed");
  }
  void read(void* dst, P src, size_t bytes, P s) {
    if (!bytes) return;
    if (dev_ < 0) {
      memcpy(dst, (const void*)src, bytes);
      return;
    }
    if (hipMemcpyAsync(dst, (const void*)src, bytes, hipMemcpyDeviceToHost, (hipStream_t)s) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)s) != hipSuccess)
      throw std::runtime_error("LoopComm: device -> host copy failed");
  }
  void write(P dst, const void* src, size_t bytes, P s) {
    if (!bytes) return;
    if (dev_ < 0) {
      memcpy((void*)dst, src, bytes);
      return;
    }
    if (hipMemcpyAsync((void*)dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)s) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)s) != hipSuccess)
      throw std::runtime_error("LoopComm: host -> device copy failed");
  }

  static void reduce_into(std::vector<char>& acc, const std::vector<char>& x, size_t n, int dt, int op, bool first) {
    if (first) {
      acc = x;
      return;
    }
    auto f = [op](double a, double b) {
      switch (op) {
        case 0: case 4: return a + b;
        case 1: return a * b;
        case 2: return a > b ? a : b;
        case 3: return a < b ? a : b;
      }
      throw std::runtime_error("LoopComm: unsupported reduction op");
    };
    auto ff = [op](float a, float b) {
      switch (op) {
        case 0: case 4: return a + b;
        case 1: return a * b;
        case 2: return a > b ? a : b;
        case 3: return a < b ? a : b;
      }
      throw std::runtime_error("LoopComm: unsupported reduction op");
    };
    switch (dt) {
      case 0: {
        float* a = (float*)acc.data();
        const float* b = (const float*)x.data();
        for (size_t i = 0; i < n; ++i) a[i] = ff(a[i], b[i]);
        break;
      }
      case 1: {
        uint16_t* a = (uint16_t*)acc.data();
        const uint16_t* b = (const uint16_t*)x.data();
        for (size_t i = 0; i < n; ++i) a[i] = f_to_bf16(ff(bf16_to_f(a[i]), bf16_to_f(b[i])));
        break;
      }
      case 2: {
        _Float16* a = (_Float16*)acc.data();
        const _Float16* b = (const _Float16*)x.data();
        for (size_t i = 0; i < n; ++i) a[i] = (_Float16)ff((float)a[i], (float)b[i]);
        break;
      }
      case 3: {
        int32_t* a = (int32_t*)acc.data();
        const int32_t* b = (const int32_t*)x.data();
        for (size_t i = 0; i < n; ++i) a[i] = (int32_t)f(a[i], b[i]);
        break;
      }
      case 4: {
        int64_t* a = (int64_t*)acc.data();
        const int64_t* b = (const int64_t*)x.data();
        for (size_t i = 0; i < n; ++i) a[i] = op == 2 ? std::max(a[i], b[i]) : op == 3 ? std::min(a[i], b[i])
                                              : op == 1 ? a[i] * b[i] : a[i] + b[i];
        break;
      }
      case 5: {
        uint8_t* a = (uint8_t*)acc.data();
        const uint8_t* b = (const uint8_t*)x.data();
        for (size_t i = 0; i < n; ++i) a[i] = (uint8_t)f(a[i], b[i]);
        break;
      }
      case 6: {
        double* a = (double*)acc.data();
        const double* b = (const double*)x.data();
        for (size_t i = 0; i < n; ++i) a[i] = f(a[i], b[i]);
        break;
      }
    }
  }
  static void finish_avg(std::vector<char>& acc, size_t n, int dt, int op, int nr) {
    if (op != 4) return;
    switch (dt) {
      case 0: for (size_t i = 0; i < n; ++i) ((float*)acc.data())[i] /= (float)nr; break;
      case 1:
        for (size_t i = 0; i < n; ++i) {
          uint16_t* a = (uint16_t*)acc.data();
          a[i] = f_to_bf16(bf16_to_f(a[i]) / (float)nr);
        }
        break;
      case 2: for (size_t i = 0; i < n; ++i) ((_Float16*)acc.data())[i] /= (_Float16)nr; break;
      case 6: for (size_t i = 0; i < n; ++i) ((double*)acc.data())[i] /= (double)nr; break;
      default: throw std::runtime_error("LoopComm: avg needs a floating dtype");
    }
  }

  // One collective: post my slot, barrier, compute my output from the
  // peers' buffers, barrier (every read done), write my output.
  template <class Compute>
  void collective(Slot me, P s, const char* what, Compute compute) {
    py::gil_scoped_release nogil;
    sync(s);  // my inputs are complete
    std::vector<char> out;
    bool have = false;
    {
      std::unique_lock<std::mutex> lk(w_->mu);
      g_->slots[rank_] = me;
      g_->barrier(*w_, lk, what);
      std::vector<Slot> peers = g_->slots;
      lk.unlock();
      have = compute(peers, out);
      lk.lock();
      g_->barrier(*w_, lk, what);
    }
    if (have) write(me.recv, out.data(), out.size(), s);
  }

  bool capturing(P s) const {
    if (dev_ < 0) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing((hipStream_t)s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
  }
  void hchk(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("LoopComm (captured) ") + what + ": " + hipGetErrorString(e));
  }
  // group barrier with the GIL released (the peers need it to reach theirs)
  std::vector<Slot> gbarrier(const Slot* mine, const char* what) {
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(w_->mu);
    if (mine) g_->slots[rank_] = *mine;
    g_->barrier(*w_, lk, what);
    return g_->slots;
  }
  static bool dbg() {
    static int on = [] {
      const char* e = getenv("SG_LOOP_DEBUG");
      return e && e[0] == '1' ? 1 : 0;
    }();
    return on;
  }
  // the captured all-reduce (see the header): called with the GIL held
  void captured_all_reduce(P send, P recv, size_t count, int dt, int op, P s) {
    if (dbg()) fprintf(stderr, "[loop r%d] captured all_reduce count=%zu dt=%d stream=%p\n", rank_, count, dt, (void*)s);
    if (nranks() > 16) throw std::runtime_error("LoopComm (captured): at most 16 ranks");
    Slot me{send, recv, count, dt, op};
    me.kind = 1;
    me.root = 0;
    me.key = (long)s;
    std::vector<Slot> ps = gbarrier(&me, "all_reduce (captured)");  // every rank's earlier work is enqueued
    for (const Slot& p : ps)
      if (p.count != count || p.dt != dt || p.op != op || p.key != (long)s)
        throw std::runtime_error("LoopComm all_reduce (captured): ranks disagree on count / dtype / op / stream "
                                 "(every rank must capture onto the world's one stream)");
    if (rank_ == 0) {
      std::vector<const void*> sends(ps.size());
      std::vector<void*> recvs(ps.size());
      for (size_t j = 0; j < ps.size(); ++j) {
        sends[j] = (const void*)ps[j].send;
        recvs[j] = (void*)ps[j].recv;
      }
      if (sg_loop_allreduce(sends.data(), recvs.data(), (int)ps.size(), (int64_t)count, dt, op, (hipStream_t)s) != 0)
        throw std::runtime_error("LoopComm all_reduce (captured): unsupported dtype / op or launch failure");
    }
    gbarrier(nullptr, "all_reduce (captured)");  // the reduction is enqueued before any rank's later work
    if (dbg()) fprintf(stderr, "[loop r%d] captured all_reduce done\n", rank_);
  }
  void no_capture(P s, const char* what) {
    if (capturing(s))
      throw std::runtime_error(std::string("LoopComm ") + what + ": not supported inside a captured graph "
                                                                 "(only all_reduce is)");
  }

  void all_reduce(P send, P recv, size_t count, int dt, int op, P s) {
    if (capturing(s)) {
      if (op == 1 || (dt != 0 && dt != 1 && dt != 6))
        throw std::runtime_error("LoopComm all_reduce (captured): sum / avg / max / min of f32, bf16, f64 only");
      captured_all_reduce(send, recv, count, dt, op, s);
      return;
    }
    const size_t b = count * dt_size(dt);
    collective(Slot{send, recv, count, dt, op}, s, "all_reduce", [&](std::vector<Slot>& ps, std::vector<char>& out) {
      std::vector<char> x(b);
      for (size_t j = 0; j < ps.size(); ++j) {
        read(x.data(), ps[j].send, b, s);
        reduce_into(out, x, count, dt, op, j == 0);
      }
      finish_avg(out, count, dt, op, (int)ps.size());
      return true;
    });
  }
  void reduce_scatter(P send, P recv, size_t recvcount, int dt, int op, P s) {
    no_capture(s, "reduce_scatter");
    const size_t e = dt_size(dt), b = recvcount * e;
    collective(Slot{send, recv, recvcount, dt, op}, s, "reduce_scatter",
               [&](std::vector<Slot>& ps, std::vector<char>& out) {
                 std::vector<char> x(b);
                 for (size_t j = 0; j < ps.size(); ++j) {
                   read(x.data(), ps[j].send + (P)rank_ * b, b, s);
                   reduce_into(out, x, recvcount, dt, op, j == 0);
                 }
                 finish_avg(out, recvcount, dt, op, (int)ps.size());
                 return true;
               });
  }
  void all_gather(P send, P recv, size_t sendcount, int dt, P s) {
    no_capture(s, "all_gather");
    const size_t b = sendcount * dt_size(dt);
    collective(Slot{send, recv, sendcount, dt}, s, "all_gather", [&](std::vector<Slot>& ps, std::vector<char>& out) {
      out.resize(b * ps.size());
      for (size_t j = 0; j < ps.size(); ++j) read(out.data() + j * b, ps[j].send, b, s);
      return true;
    });
  }
  void broadcast(P send, P recv, size_t count, int dt, int root, P s) {
    no_capture(s, "broadcast");
    const size_t b = count * dt_size(dt);
    collective(Slot{send, recv, count, dt, 0, root}, s, "broadcast",
               [&](std::vector<Slot>& ps, std::vector<char>& out) {
                 if (root < 0 || root >= (int)ps.size()) throw std::runtime_error("LoopComm broadcast: bad root");
                 if (rank_ == root && send == recv) return false;
                 out.resize(b);
                 read(out.data(), ps[root].send, b, s);
                 return true;
               });
  }
  void reduce(P send, P recv, size_t count, int dt, int op, int root, P s) {
    no_capture(s, "reduce");
    const size_t b = count * dt_size(dt);
    collective(Slot{send, recv, count, dt, op, root}, s, "reduce", [&](std::vector<Slot>& ps, std::vector<char>& out) {
      if (rank_ != root) return false;
      std::vector<char> x(b);
      for (size_t j = 0; j < ps.size(); ++j) {
        read(x.data(), ps[j].send, b, s);
        reduce_into(out, x, count, dt, op, j == 0);
      }
      finish_avg(out, count, dt, op, (int)ps.size());
      return true;
    });
  }
  void all_to_all(P send, P recv, size_t count, int dt, P s) {
    no_capture(s, "all_to_all");
    const size_t b = count * dt_size(dt);
    collective(Slot{send, recv, count, dt}, s, "all_to_all", [&](std::vector<Slot>& ps, std::vector<char>& out) {
      out.resize(b * ps.size());
      for (size_t j = 0; j < ps.size(); ++j) read(out.data() + j * b, ps[j].send + (P)rank_ * b, b, s);
      return true;
    });
  }

  // ------------------------------------------------------------- p2p
  void send(P buf, size_t count, int dt, int peer, P s) {
    no_capture(s, "send");
    if (t_group_depth > 0) {
      t_pending.push_back(PendingP2P{true, this, buf, count, dt, peer, s});
      return;
    }
    py::gil_scoped_release nogil;
    auto m = deposit(buf, count, dt, peer, s);
    await_consumed(m);
  }
  void recv(P buf, size_t count, int dt, int peer, P s) {
    no_capture(s, "recv");
    if (t_group_depth > 0) {
      t_pending.push_back(PendingP2P{false, this, buf, count, dt, peer, s});
      return;
    }
    py::gil_scoped_release nogil;
    take(buf, count, dt, peer, s);
  }
  std::shared_ptr<World::Msg> deposit(P buf, size_t count, int dt, int peer, P s) {
    check_peer(peer);
    sync(s);
    auto m = std::make_shared<World::Msg>();
    m->data.resize(count * dt_size(dt));
    read(m->data.data(), buf, m->data.size(), s);
    std::lock_guard<std::mutex> lk(w_->mu);
    w_->boxes[{g_->members[rank_], g_->members[peer]}].push_back(m);
    w_->cv.notify_all();
    return m;
  }
  void await_consumed(const std::shared_ptr<World::Msg>& m) {
    std::unique_lock<std::mutex> lk(w_->mu);
    w_->wait(lk, [&] { return m->consumed; }, "send (unmatched: both peers sending first deadlocks on RCCL too)");
  }
  void take(P buf, size_t count, int dt, int peer, P s) {
    check_peer(peer);
    std::shared_ptr<World::Msg> m;
    {
      std::unique_lock<std::mutex> lk(w_->mu);
      auto& q = w_->boxes[{g_->members[peer], g_->members[rank_]}];
      w_->wait(lk, [&] { return !q.empty(); }, "recv");
      m = q.front();
      q.pop_front();
    }
    const size_t b = count * dt_size(dt);
    if (m->data.size() != b) {
      std::lock_guard<std::mutex> lk(w_->mu);
      m->consumed = true;
      w_->cv.notify_all();
      throw std::runtime_error("LoopComm recv: message of " + std::to_string(m->data.size()) + " bytes, receive of " +
                               std::to_string(b) + " bytes (mismatched send / recv pairing)");
    }
    sync(s);
    write(buf, m->data.data(), b, s);
    std::lock_guard<std::mutex> lk(w_->mu);
    m->consumed = true;
    w_->cv.notify_all();
  }
  void check_peer(int peer) {
    if (peer < 0 || peer >= nranks()) throw std::runtime_error("LoopComm: peer out of range");
  }

  static void group_start() { ++t_group_depth; }
  static void group_end() {
    if (t_group_depth <= 0) throw std::runtime_error("LoopComm: group_end without group_start");
    if (--t_group_depth > 0) return;
    std::vector<PendingP2P> ops;
    ops.swap(t_pending);
    py::gil_scoped_release nogil;
    std::vector<std::shared_ptr<World::Msg>> sent;
    for (auto& o : ops)
      if (o.is_send) sent.push_back(o.c->deposit(o.buf, o.count, o.dt, o.peer, o.stream));
    for (auto& o : ops)
      if (!o.is_send) o.c->take(o.buf, o.count, o.dt, o.peer, o.stream);
    for (size_t i = 0, k = 0; i < ops.size(); ++i)
      if (ops[i].is_send) ops[i].c->await_consumed(sent[k++]);
  }

  // ------------------------------------------------------------- structure
  LoopComm* split(int color, int key) {
    std::shared_ptr<Group> ng;
    int nr = -1;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(w_->mu);
      Slot me;
      me.color = color;
      me.key = key;
      g_->slots[rank_] = me;
      const long seq = g_->splits;
      g_->barrier(*w_, lk, "split");
      if (color >= 0) {
        std::vector<std::pair<long, int>> mem;  // (key, group rank)
        for (int j = 0; j < nranks(); ++j)
          if (g_->slots[j].color == color) mem.push_back({g_->slots[j].key, j});
        std::sort(mem.begin(), mem.end());
        std::vector<int> glob;
        for (size_t i = 0; i < mem.size(); ++i) {
          glob.push_back(g_->members[mem[i].second]);
          if (mem[i].second == rank_) nr = (int)i;
        }
        auto& slot = w_->splits[std::make_tuple((const void*)g_.get(), seq, color)];
        if (!slot) slot = std::make_shared<Group>(glob);
        ng = slot;
      }
      g_->barrier(*w_, lk, "split");
      if (rank_ == 0) ++g_->splits;
      g_->barrier(*w_, lk, "split");
    }
    if (!ng) return nullptr;
    return new LoopComm(w_, ng, nr, dev_);
  }
  std::string async_error() {
    std::lock_guard<std::mutex> lk(w_->mu);
    return w_->aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(w_->mu);
    if (w_->aborted.empty()) w_->aborted = "rank " + std::to_string(g_->members[rank_]) + " aborted";
    w_->cv.notify_all();
  }
  void destroy() {}

 private:
  std::shared_ptr<World> w_;
  std::shared_ptr<Group> g_;
  int rank_, dev_;
};

// the shared state handed to each rank's thread
struct LoopWorld {
  LoopWorld(int n, double timeout_s) : w(std::make_shared<World>(n, timeout_s)) {
    std::vector<int> all(n);
    for (int i = 0; i < n; ++i) all[i] = i;
    g = std::make_shared<Group>(all);
  }
  std::shared_ptr<World> w;
  std::shared_ptr<Group> g;
};

}  // namespace

void register_loop(py::module& m) {
  py::class_<LoopWorld, std::shared_ptr<LoopWorld>>(m, "LoopWorld")
      .def(py::init<int, double>(), py::arg("nranks"), py::arg("timeout_s") = 60.0)
      .def_property_readonly("nranks", [](const LoopWorld& w) { return w.w->n; });
  py::class_<LoopComm>(m, "LoopComm")
      .def(py::init([](std::shared_ptr<LoopWorld> w, int rank, int device) {
             if (rank < 0 || rank >= w->w->n) throw std::invalid_argument("LoopComm: rank out of range");
             return new LoopComm(w->w, w->g, rank, device);
           }),
           py::arg("world"), py::arg("rank"), py::arg("device") = -1)
      .def_property_readonly("nranks", &LoopComm::nranks)
      .def_property_readonly("rank", &LoopComm::rank)
      .def_property_readonly("device", &LoopComm::device)
      .def_property_readonly("loopback", [](const LoopComm&) { return true; })
      .def("all_reduce", &LoopComm::all_reduce)
      .def("reduce_scatter", &LoopComm::reduce_scatter)
      .def("all_gather", &LoopComm::all_gather)
      .def("broadcast", &LoopComm::broadcast)
      .def("reduce", &LoopComm::reduce)
      .def("all_to_all", &LoopComm::all_to_all)
      .def("send", &LoopComm::send)
      .def("recv", &LoopComm::recv)
      .def_static("group_start", &LoopComm::group_start)
      .def_static("group_end", &LoopComm::group_end)
      .def("split", &LoopComm::split, py::return_value_policy::take_ownership)
      .def("async_error", &LoopComm::async_error)
      .def("abort", &LoopComm::abort)
      .def("destroy", &LoopComm::destroy);
}

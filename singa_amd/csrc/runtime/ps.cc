// Native parameter server + client (reference C25 Server::Run,
// src/server/server.cc:45-214; C26 pm prototype PMServer / PMClient,
// src/server/pm_server.cc, src/worker/pm_client.cc; C12 sync variants
// ElasticParam / RandomSyncParam, src/utils/param.cc:130-284; C15 Router
// handshake, src/utils/router.cc:16-86).
//
// On an MI355X node the training path replaces the PS with RCCL collectives
// (parallel/distopt.py, parallel/easgd.py).  This is the host-side PS for the
// reference's asynchronous deployments (worker groups on different hosts or
// GPUs exchanging with key-sharded servers every sync_frequency steps) and for
// the pm benchmark: plain TCP instead of ZeroMQ, one handler thread per
// connection (the reference's zactor pool; concurrent messages on one key are
// serialised by a per-key lock, server.cc:130-156), deferred Gets that block
// until the key has been Put (server.cc:158-173), and kStop counting
// (server.cc:145-147, 203-211).
//
// Wire format (little-endian): a fixed 48-byte header, then `n` fp32 values.
//   magic u32 | type u16 | flags u16 | id i32 | step i32 | f0 f32 | pad u32 |
//   a i64 | b i64 | n u64
// Every request gets exactly one reply (same header layout, type echoed) on
// the same connection, so a client may pipeline requests and collect the
// replies in order (PMClient Update + Collect, pm_client.cc:221-287).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

namespace sgrt {

namespace {

constexpr uint32_t kMagic = 0x31414753u;  // "SGA1"

// (a signal landing in a blocking call returns EINTR: retry, do not fail)
bool send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n > 0) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n > 0) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
void tune_socket(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

}  // namespace

// ---------------------------------------------------------------------------
// server
// ---------------------------------------------------------------------------
// The value is a shared buffer: a reply shares it instead of copying (a
// connection's writer thread may still be sending an older version while a
// new request replaces it); an in-place update copies-on-write while any
// queued reply still refers to it.  "Still refers" is the `inflight` count,
// incremented under the entry mutex when a reply is queued and released by
// the writer (release) after the send; mut() reads it with acquire, so the
// send's reads happen-before any later in-place write.  (shared_ptr's
// use_count() is a relaxed load and orders nothing -- ThreadSanitizer
// flagged the update racing the send under the multi-client stress test.)
struct Buf : std::vector<float> {
  std::atomic<int> inflight{0};
  Buf() = default;
  explicit Buf(size_t n) : std::vector<float>(n) {}
  Buf(const Buf& o) : std::vector<float>(o) {}
};
using FBuf = std::shared_ptr<Buf>;
struct PSEntry {
  std::mutex mu;
  FBuf w;
  std::vector<float> s1, s2;
  int64_t nupdates = 0;
  std::vector<float>& mut() {  // the value, unshared, for an in-place update (entry mutex held)
    if (w->inflight.load(std::memory_order_acquire) > 0) w = std::make_shared<Buf>(*w);
    return *w;
  }
  FBuf reply() {  // the value as a queued reply (entry mutex held)
    w->inflight.fetch_add(1, std::memory_order_relaxed);
    return w;
  }
};

struct PServer::Impl {
  int port = 0, listen_fd = -1;
  int nworkers = 1;
  UpdateArgs upd;
  std::string lr_method = "kFixed";
  double lr_base = 0.01, lr_final = 0.0, lr_gamma = 1.0, lr_pow = 0.0;
  int lr_freq = 1;
  std::mutex mu;  // guards `params` (the map), ready cv, stop counting
  std::condition_variable cv;
  std::map<int, std::unique_ptr<PSEntry>> params;
  int nstop = 0;
  std::atomic<bool> closing{false};
  std::thread acceptor;
  std::vector<std::thread> handlers;
  std::vector<int> conn_fds;
  std::atomic<int64_t> nmsg{0};

  PSEntry* find(int id, bool wait) {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      auto it = params.find(id);
      if (it != params.end()) return it->second.get();
      if (!wait || closing) return nullptr;
      // deferred kGet (server.cc:79-95).  A system_clock deadline: libstdc++
      // maps a steady_clock wait_for onto pthread_cond_clockwait, which the
      // GCC 11 ThreadSanitizer does not intercept (it then reports the
      // re-lock inside the wait as a double lock)
      cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(100));
    }
  }

  // One connection: this thread reads and processes requests in order and
  // queues the replies; a writer thread sends them.  Reading never waits for
  // the peer to drain replies, so a client may pipeline any volume of
  // requests before collecting (the pm pattern) without a TCP deadlock.
  void handle(int fd) {
    std::mutex qmu;
    std::condition_variable qcv;
    std::deque<std::pair<PSHeader, FBuf>> q;
    bool done = false;
    std::thread writer([&] {
      for (;;) {
        std::pair<PSHeader, FBuf> item;
        {
          std::unique_lock<std::mutex> lk(qmu);
          qcv.wait(lk, [&] { return done || !q.empty(); });
          if (q.empty()) return;
          item = std::move(q.front());
          q.pop_front();
        }
        const PSHeader& r = item.first;
        const bool ok = send_all(fd, &r, sizeof(r)) && (!r.n || send_all(fd, item.second->data(), r.n * sizeof(float)));
        if (item.second) item.second->inflight.fetch_sub(1, std::memory_order_release);
        if (!ok) {
          ::shutdown(fd, SHUT_RDWR);  // the reader sees the error and ends the connection
          return;
        }
      }
    });
    FBuf in = std::make_shared<Buf>();
    for (;;) {
      PSHeader h;
      if (!recv_all(fd, &h, sizeof(h)) || h.magic != kMagic) break;
      if (in.use_count() > 1 || !in) in = std::make_shared<Buf>();
      in->resize(h.n);
      if (h.n && !recv_all(fd, in->data(), h.n * sizeof(float))) break;
      nmsg++;
      PSHeader r = h;
      r.n = 0;
      FBuf out;
      switch (h.type) {
        case kPSPing:
          break;
        case kPSPut: {  // create or overwrite (HandlePutMsg, param.cc:24-39)
          {
            std::lock_guard<std::mutex> lk(mu);
            auto& slot = params[h.id];
            if (!slot) slot.reset(new PSEntry());
            std::lock_guard<std::mutex> lk2(slot->mu);
            slot->s1.assign(in->size(), 0.f);
            slot->s2.assign(in->size(), 0.f);
            slot->w = std::move(in);
            in = std::make_shared<Buf>();
          }
          cv.notify_all();
          break;
        }
        case kPSGet: {
          PSEntry* e = find(h.id, true);
          if (!e) { r.flags = 1; break; }
          std::lock_guard<std::mutex> lk(e->mu);
          out = e->reply();  // shared, no copy
          break;
        }
        case kPSUpdate: {  // gradient -> server-side updater -> new value
          PSEntry* e = find(h.id, true);
          if (!e) { r.flags = 1; break; }
          std::lock_guard<std::mutex> lk(e->mu);
          if (e->w->size() != in->size()) { r.flags = 1; break; }
          UpdateArgs a = upd;
          const int64_t step = h.step >= 0 ? h.step : e->nupdates;
          a.lr = (float)LearningRate(lr_method, lr_base, lr_final, lr_freq, lr_gamma, lr_pow, step);
          a.t = (float)(step + 1);
          if (h.f0 > 0.f) a.grad_scale = h.f0;
          OptUpdate(a, e->mut().data(), in->data(), e->s1.data(), e->s2.data(), (int64_t)in->size());
          e->nupdates++;
          out = e->reply();
          break;
        }
        case kPSReplace: {  // pm HandleUpdateMsg: replace, reply the value (param.cc:57-61)
          PSEntry* e = find(h.id, true);
          if (!e) { r.flags = 1; break; }
          std::lock_guard<std::mutex> lk(e->mu);
          // the optimiser state (s1 / s2) is sized by the Put: a value of
          // another size would let a later Update write past their end
          if (e->w->size() != in->size()) { r.flags = 1; break; }
          e->w = std::move(in);  // the received buffer becomes the value and the reply: no copy
          in = std::make_shared<Buf>();
          e->nupdates++;
          out = e->reply();
          break;
        }
        case kPSElastic: {  // d = alpha (w_worker - c); c += d; reply d (param.cc:244-258)
          PSEntry* e = find(h.id, true);
          if (!e) { r.flags = 1; break; }
          std::lock_guard<std::mutex> lk(e->mu);
          if (e->w->size() != in->size()) { r.flags = 1; break; }
          out = std::make_shared<Buf>(in->size());
          out->inflight.store(1, std::memory_order_relaxed);  // a fresh reply buffer: counted like a shared one
          const float alpha = h.f0;
          float* c = e->mut().data();
          const float* wv = in->data();
          float* dv = out->data();
          for (size_t i = 0; i < in->size(); ++i) {
            const float d = alpha * (wv[i] - c[i]);
            c[i] += d;
            dv[i] = d;
          }
          e->nupdates++;
          break;
        }
        case kPSRandom: {  // c[idx] += delta; reply the old c[idx] (param.cc:141-171)
          PSEntry* e = find(h.id, true);
          if (!e) { r.flags = 1; break; }
          std::lock_guard<std::mutex> lk(e->mu);
          const int64_t n = (int64_t)e->w->size();
          // untrusted progression: an empty value (modulo by zero) or a / b
          // outside [0, n) (negative indices) is rejected
          if (n == 0 || h.a < 0 || h.a >= n || h.b < 0 || h.b >= n) { r.flags = 1; break; }
          out = std::make_shared<Buf>(in->size());
          out->inflight.store(1, std::memory_order_relaxed);  // a fresh reply buffer: counted like a shared one
          std::vector<float>& c = e->mut();
          // the sample is the progression idx_i = (a + i*b) mod n shared by
          // every rank (parallel/easgd.py RandomSync): no index traffic
          for (size_t i = 0; i < in->size(); ++i) {
            const int64_t idx = (int64_t)((h.a + (int64_t)i * h.b) % n);
            (*out)[i] = c[idx];
            c[idx] += (*in)[i];
          }
          e->nupdates++;
          break;
        }
        case kPSStop: {
          std::lock_guard<std::mutex> lk(mu);
          nstop++;
          cv.notify_all();
          break;
        }
        default:
          r.flags = 2;
      }
      r.n = out ? out->size() : 0;
      {
        std::lock_guard<std::mutex> lk(qmu);
        q.emplace_back(r, std::move(out));
      }
      qcv.notify_one();
    }
    {
      std::lock_guard<std::mutex> lk(qmu);
      done = true;
    }
    qcv.notify_one();
    writer.join();
    for (auto& it : q)  // replies never sent (the connection failed): release their buffers
      if (it.second) it.second->inflight.fetch_sub(1, std::memory_order_release);
    q.clear();
    {
      // forget the fd BEFORE closing it: Close() must never shut down a
      // number the kernel has already handed to another socket
      std::lock_guard<std::mutex> lk(mu);
      for (auto& c : conn_fds)
        if (c == fd) c = -1;
    }
    ::close(fd);
  }
};

PServer::PServer(int port, int nworkers) : d_(new Impl()) {
  d_->nworkers = nworkers;
  d_->listen_fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (d_->listen_fd < 0) throw std::runtime_error("PServer: socket() failed");
  int one = 1;
  setsockopt(d_->listen_fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  addr.sin_port = htons((uint16_t)port);
  if (::bind(d_->listen_fd, (sockaddr*)&addr, sizeof(addr)) != 0 || ::listen(d_->listen_fd, 64) != 0) {
    ::close(d_->listen_fd);
    throw std::runtime_error("PServer: cannot bind/listen on port " + std::to_string(port));
  }
  socklen_t len = sizeof(addr);
  getsockname(d_->listen_fd, (sockaddr*)&addr, &len);
  d_->port = ntohs(addr.sin_port);
  Impl* d = d_.get();
  d_->acceptor = std::thread([d] {
    while (!d->closing) {
      const int fd = ::accept(d->listen_fd, nullptr, nullptr);
      if (fd < 0) {
        if (d->closing) break;
        continue;
      }
      tune_socket(fd);
      std::lock_guard<std::mutex> lk(d->mu);
      d->conn_fds.push_back(fd);
      d->handlers.emplace_back([d, fd] { d->handle(fd); });
    }
  });
}

PServer::~PServer() { Close(); }

int PServer::port() const { return d_->port; }
int64_t PServer::messages() const { return d_->nmsg.load(); }

void PServer::SetUpdater(const UpdateArgs& a, const std::string& method, double base, double final_lr, int freq,
                         double gamma, double pw) {
  std::lock_guard<std::mutex> lk(d_->mu);
  d_->upd = a;
  d_->lr_method = method;
  d_->lr_base = base;
  d_->lr_final = final_lr;
  d_->lr_freq = freq;
  d_->lr_gamma = gamma;
  d_->lr_pow = pw;
}

bool PServer::WaitStop(double timeout_s) {
  std::unique_lock<std::mutex> lk(d_->mu);
  const auto until = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (d_->nstop < d_->nworkers) {
    if (timeout_s >= 0 && std::chrono::steady_clock::now() >= until) return false;
    d_->cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(100));
  }
  return true;
}

std::vector<float> PServer::Value(int id) {
  PSEntry* e = d_->find(id, false);
  if (!e) return {};
  std::lock_guard<std::mutex> lk(e->mu);
  return *e->w;
}

void PServer::Close() {
  if (!d_ || d_->closing.exchange(true)) return;
  ::shutdown(d_->listen_fd, SHUT_RDWR);
  ::close(d_->listen_fd);
  if (d_->acceptor.joinable()) d_->acceptor.join();
  std::vector<std::thread> hs;
  {
    std::lock_guard<std::mutex> lk(d_->mu);
    for (int fd : d_->conn_fds)
      if (fd >= 0) ::shutdown(fd, SHUT_RDWR);  // unblock handlers stuck in recv / send
    hs.swap(d_->handlers);
  }
  d_->cv.notify_all();
  for (auto& t : hs)
    if (t.joinable()) t.join();
}

// ---------------------------------------------------------------------------
// client
// ---------------------------------------------------------------------------
PSClient::PSClient(const std::vector<std::string>& endpoints, int retries, double retry_s) {
  for (const auto& ep : endpoints) {
    const auto colon = ep.rfind(':');
    if (colon == std::string::npos) throw std::invalid_argument("PSClient: endpoint must be host:port: " + ep);
    const std::string host = ep.substr(0, colon), port = ep.substr(colon + 1);
    int fd = -1;
    // Router::Connect: retry until the server is up (router.cc:16-44)
    for (int attempt = 0; attempt <= retries && fd < 0; ++attempt) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) == 0 && res) {
        fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
        if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
          ::close(fd);
          fd = -1;
        }
        freeaddrinfo(res);
      }
      if (fd < 0) std::this_thread::sleep_for(std::chrono::duration<double>(retry_s));
    }
    if (fd < 0) throw std::runtime_error("PSClient: cannot connect to " + ep);
    tune_socket(fd);
    fds_.push_back(fd);
    pending_.emplace_back();
    // PING/PONG handshake
    PSHeader h{};
    h.magic = kMagic;
    h.type = kPSPing;
    Send(h, nullptr, fds_.size() - 1);
    PSHeader r;
    if (!Recv(fds_.size() - 1, &r, nullptr, 0) || r.type != kPSPing)
      throw std::runtime_error("PSClient: handshake with " + ep + " failed");
  }
}

PSClient::~PSClient() {
  for (int fd : fds_) ::close(fd);
}

int PSClient::server_of(int id) const { return id % (int)fds_.size(); }  // key sharding (param_manager.cc:112)

void PSClient::Send(const PSHeader& h, const float* data, size_t server) {
  if (!send_all(fds_[server], &h, sizeof(h)) || (h.n && !send_all(fds_[server], data, h.n * sizeof(float))))
    throw std::runtime_error(std::string("PSClient: send failed: ") + std::strerror(errno));
}

bool PSClient::Recv(size_t server, PSHeader* r, float* out, uint64_t cap) {
  if (!recv_all(fds_[server], r, sizeof(*r)) || r->magic != kMagic) return false;
  if (r->n) {
    if (out && r->n <= cap) return recv_all(fds_[server], out, r->n * sizeof(float));
    std::vector<float> sink(r->n);  // caller did not want the payload
    return recv_all(fds_[server], sink.data(), r->n * sizeof(float));
  }
  return true;
}

static PSHeader make_header(int type, int id, uint64_t n) {
  PSHeader h{};
  h.magic = kMagic;
  h.type = (uint16_t)type;
  h.id = id;
  h.step = -1;
  h.n = n;
  return h;
}

uint64_t PSClient::Request(const PSHeader& h, const float* data, float* out, uint64_t cap) {
  const int s = server_of(h.id);
  Send(h, data, s);
  PSHeader r;
  if (!Recv(s, &r, out, cap)) throw std::runtime_error("PSClient: receive failed");
  if (r.flags) throw std::runtime_error("PSClient: server rejected request type " + std::to_string(h.type) +
                                        " for key " + std::to_string(h.id));
  if (out && r.n > cap)  // the payload was drained (stream stays in sync) but not delivered
    throw std::runtime_error("PSClient: reply of " + std::to_string(r.n) + " floats exceeds the " +
                             std::to_string(cap) + "-float buffer for key " + std::to_string(h.id));
  return r.n;
}

void PSClient::Put(int id, const float* w, uint64_t n) { Request(make_header(kPSPut, id, n), w, nullptr, 0); }

uint64_t PSClient::Get(int id, float* out, uint64_t cap) { return Request(make_header(kPSGet, id, 0), nullptr, out, cap); }

void PSClient::Update(int id, const float* grad, float* w_out, uint64_t n, int step, float grad_scale) {
  PSHeader h = make_header(kPSUpdate, id, n);
  h.step = step;
  h.f0 = grad_scale;
  Request(h, grad, w_out, n);
}

void PSClient::Elastic(int id, float* w, uint64_t n, float alpha) {
  PSHeader h = make_header(kPSElastic, id, n);
  h.f0 = alpha;
  std::vector<float> d(n);
  Request(h, w, d.data(), n);
  for (uint64_t i = 0; i < n; ++i) w[i] -= d[i];  // worker side of ElasticParam (param.cc:269-284)
}

void PSClient::RandomSync(int id, const float* delta, float* old_out, uint64_t m, int64_t a, int64_t b) {
  PSHeader h = make_header(kPSRandom, id, m);
  h.a = a;
  h.b = b;
  Request(h, delta, old_out, m);
}

void PSClient::PushReplace(int id, const float* w, uint64_t n) {
  const int s = server_of(id);
  Send(make_header(kPSReplace, id, n), w, s);
  pending_[s].push_back(id);
}

void PSClient::PushUpdate(int id, const float* grad, uint64_t n, int step, float grad_scale) {
  PSHeader h = make_header(kPSUpdate, id, n);
  h.step = step;
  h.f0 = grad_scale;
  const int s = server_of(id);
  Send(h, grad, s);
  pending_[s].push_back(id);
}

int PSClient::Collect(const std::vector<float*>& outs, const std::vector<uint64_t>& caps,
                      const std::vector<int>& ids) {
  // replies arrive in issue order per server; route each to its key's buffer
  std::map<int, size_t> where;
  for (size_t i = 0; i < ids.size(); ++i) where[ids[i]] = i;
  int got = 0;
  std::string err;  // every pending reply is drained first, then a rejection / overflow is reported
  for (size_t s = 0; s < fds_.size(); ++s) {
    for (int id : pending_[s]) {
      auto it = where.find(id);
      PSHeader r;
      const bool ok = it != where.end() ? Recv(s, &r, outs[it->second], caps[it->second]) : Recv(s, &r, nullptr, 0);
      if (!ok) throw std::runtime_error("PSClient: collect failed");
      if (err.empty() && r.flags) err = "PSClient: server rejected a pushed request for key " + std::to_string(id);
      if (err.empty() && it != where.end() && r.n > caps[it->second])
        err = "PSClient: reply for key " + std::to_string(id) + " exceeds its buffer";
      got++;
    }
    pending_[s].clear();
  }
  if (!err.empty()) throw std::runtime_error(err);
  return got;
}

void PSClient::Stop() {
  for (size_t s = 0; s < fds_.size(); ++s) {
    Send(make_header(kPSStop, 0, 0), nullptr, s);
    PSHeader r;
    Recv(s, &r, nullptr, 0);
  }
}

}  // namespace sgrt

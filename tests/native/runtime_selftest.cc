// Native self-test of the host runtime (_core sources), built WITHOUT Python
// under ThreadSanitizer and AddressSanitizer+UBSan by
// tests/test_sanitizers_cpu.py (the reference had no sanitizer
// build; its parser double buffer, include/worker/base_layer.h:510-537, and
// the unlocked paramid2version_ map were never checked).
//
// Exercises every concurrent path of the runtime: several Prefetcher threads
// (producer thread + consumer) over one shard folder, early destruction of a
// Prefetcher while its producer is mid-batch, crash-tolerant append, split,
// the graph sort / JSON export, the threaded C++ updaters, the mmap LMDB
// B+tree walker (argv[2]: a database written by tests/lmdb_writer.py), and the
// parameter server under load: several client threads doing Put / Get /
// Update / pipelined PushUpdate + Collect / Elastic / RandomSync on SHARED
// keys, Gets deferred until another thread's Put, and kStop counting
// (the reference's concurrency hot-spot, src/server/server.cc:45-214).
// The CppCPU compute backend (cpu_ops.cc) runs GEMMs and convolutions from
// several caller threads at once: one owns the worker pool, the others run
// inline, and every result must equal the single-threaded reference.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../singa_amd/csrc/runtime/cpu_ops.h"
#include "../../singa_amd/csrc/runtime/runtime.h"

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(2);                                                  \
    }                                                                \
  } while (0)

using namespace sgrt;

static void write_shard(const std::string& dir, int n, int dim) {
  Shard s(dir, Shard::kCreate);
  for (int i = 0; i < n; ++i) {
    ImageRecord r;
    r.shape = {dim};
    r.label = i % 10;
    r.pixel.resize(dim);
    for (int j = 0; j < dim; ++j) r.pixel[j] = (char)((i + j) & 0xff);
    CHECK(s.Insert("k" + std::to_string(i), EncodeRecord(r)));
  }
  CHECK(!s.Insert("k0", "dup"));  // key de-duplication per writer session
  s.Flush();
}

int main(int argc, char** argv) {
  std::string root = argc > 1 ? argv[1] : "/tmp/sg_selftest";
  const int n = 257, dim = 64, batch = 16;
  write_shard(root + "/a", n, dim);
  {
    Shard r(root + "/a", Shard::kRead);
    CHECK(r.Count() == n);
  }
  {  // append mode keeps the records and accepts new keys
    Shard a(root + "/a", Shard::kAppend);
    ImageRecord rec;
    rec.shape = {dim};
    rec.pixel.assign(dim, 1);
    CHECK(a.Insert("extra", EncodeRecord(rec)));
    a.Flush();
  }
  {
    Shard r(root + "/a", Shard::kRead);
    CHECK(r.Count() == n + 1);
  }
  // concurrent prefetchers, each with its own producer thread
  std::vector<std::thread> ts;
  std::vector<long> sums(4, 0);
  for (int t = 0; t < 4; ++t) {
    ts.emplace_back([&, t] {
      Prefetcher p(root + "/a", batch, dim, 1.0f / 255, 0.f, true);
      std::vector<float> img((size_t)batch * dim);
      std::vector<int32_t> lab(batch);
      for (int it = 0; it < 60; ++it) {
        int got = p.Next(img.data(), lab.data());
        CHECK(got == batch);
        for (int i = 0; i < got; ++i) sums[t] += lab[i];
      }
    });
  }
  for (auto& t : ts) t.join();
  for (int t = 1; t < 4; ++t) CHECK(sums[t] == sums[0]);  // same deterministic stream
  // destroy a prefetcher while its producer is filling the next batch
  for (int k = 0; k < 20; ++k) {
    Prefetcher p(root + "/a", batch, dim, 1.0f, 0.f, true);
    std::vector<float> img((size_t)batch * dim);
    std::vector<int32_t> lab(batch);
    p.Next(img.data(), lab.data());
  }
  // non-looping prefetcher drains the shard, then returns short batches
  {
    Prefetcher p(root + "/a", batch, dim, 1.0f, 0.f, false);
    std::vector<float> img((size_t)batch * dim);
    std::vector<int32_t> lab(batch);
    long total = 0;
    for (int it = 0; it < 40; ++it) total += p.Next(img.data(), lab.data());
    CHECK(total == n + 1);
  }
  auto parts = SplitShardN(3, root + "/a", root + "/part");
  long tot = 0;
  for (auto c : parts) tot += c;
  CHECK(tot == n + 1);
  Graph g;
  g.AddEdge("data", "fc1");
  g.AddEdge("fc1", "loss");
  g.AddEdge("data", "loss");
  auto order = g.Sort();
  CHECK(order.size() == 3 && order.front() == "data" && order.back() == "loss");
  CHECK(g.ToJson({0, 1, 0}).find("\"links\"") != std::string::npos);
  // ---- threaded updaters: the pool split must equal one serial pass
  {
    const int64_t nn = 1 << 20;
    std::vector<float> w(nn), w2, gr(nn), s1(nn, 0.f), s2(nn, 0.f), t1(nn, 0.f), t2(nn, 0.f);
    for (int64_t i = 0; i < nn; ++i) {
      w[i] = std::sin(0.001f * i);
      gr[i] = std::cos(0.003f * i);
    }
    w2 = w;
    UpdateArgs a;
    a.kind = kAdam;
    a.lr = 0.01f;
    OptUpdate(a, w.data(), gr.data(), s1.data(), s2.data(), nn);
    for (int64_t o = 0; o < nn; o += 4096)  // chunked calls: element-wise identical
      OptUpdate(a, w2.data() + o, gr.data() + o, t1.data() + o, t2.data() + o, 4096);
    for (int64_t i = 0; i < nn; i += 997) CHECK(w[i] == w2[i]);
  }
  // ---- LMDB reader: walk, count, decode, from two threads at once
  if (argc > 2) {
    std::vector<std::thread> lt;
    std::vector<int64_t> cnt(2, 0);
    for (int t = 0; t < 2; ++t)
      lt.emplace_back([&, t] {
        LmdbReader rd(argv[2]);
        std::string k, v;
        while (rd.Next(&k, &v)) {
          ImageRecord rec;
          bool enc = false;
          CHECK(DecodeDatum(v, &rec, &enc));
          cnt[t]++;
        }
        CHECK(cnt[t] == rd.Count());
      });
    for (auto& t : lt) t.join();
    CHECK(cnt[0] == cnt[1] && cnt[0] > 0);
  }
  // ---- parameter server under concurrent clients
  {
    const int nthreads = 4, nkeys = 6, len = 4096, iters = 40;
    PServer srv(0, nthreads);
    UpdateArgs ua;
    ua.kind = kSGDRef;
    ua.momentum = 0.9f;
    srv.SetUpdater(ua, "kFixed", 0.01, 0.0, 1, 0.5, 0.75);
    const std::string ep = "127.0.0.1:" + std::to_string(srv.port());
    std::atomic<int> puts_done{0};
    std::vector<std::thread> cl;
    for (int t = 0; t < nthreads; ++t) {
      cl.emplace_back([&, t] {
        PSClient c({ep});
        std::vector<float> buf(len), out(len);
        if (t == 0) {
          // the Gets of the other threads on these keys may arrive first:
          // the server defers them until this Put
          std::this_thread::sleep_for(std::chrono::milliseconds(50));
          for (int k = 0; k < nkeys; ++k) {
            for (int i = 0; i < len; ++i) buf[i] = 0.001f * (k + 1) * i;
            c.Put(k, buf.data(), len);
          }
          puts_done = 1;
        } else {
          CHECK(c.Get(t % nkeys, out.data(), len) == (uint64_t)len);  // deferred Get
          CHECK(std::fabs(out[7] - 0.001f * (t % nkeys + 1) * 7) < 1e-6f);
        }
        while (!puts_done) std::this_thread::yield();
        std::vector<float> g(len, 1e-3f * (t + 1)), old(64);
        for (int it = 0; it < iters; ++it) {
          const int k = (it + t) % nkeys;  // shared keys, overlapping across threads
          switch (it % 4) {
            case 0: c.Update(k, g.data(), out.data(), len, it, 1.f); break;
            case 1: {  // pipelined pushes to every key, one Collect
              std::vector<int> ids;
              std::vector<std::vector<float>> outs(nkeys, std::vector<float>(len));
              std::vector<float*> ptrs;
              std::vector<uint64_t> caps;
              for (int j = 0; j < nkeys; ++j) {
                c.PushUpdate(j, g.data(), len, it, 1.f);
                ids.push_back(j);
                ptrs.push_back(outs[j].data());
                caps.push_back(len);
              }
              CHECK(c.Collect(ptrs, caps, ids) == nkeys);
              break;
            }
            case 2: {
              CHECK(c.Get(k, buf.data(), len) == (uint64_t)len);
              c.Elastic(k, buf.data(), len, 0.25f);
              break;
            }
            default: {
              std::vector<float> delta(64, 1e-4f);
              c.RandomSync(k, delta.data(), old.data(), 64, (it * 7 + t) % len, 17);
            }
          }
        }
        c.Stop();
      });
    }
    for (auto& t : cl) t.join();
    CHECK(srv.WaitStop(30.0));
    for (int k = 0; k < nkeys; ++k) {
      auto v = srv.Value(k);
      CHECK((int)v.size() == len);
      for (float x : v) CHECK(std::isfinite(x));
    }
    srv.Close();
  }
  {  // CppCPU kernels: concurrent callers of the persistent pool
    namespace C = sgrt::cpu;
    const int M = 37, N = 45, K = 70;
    std::vector<float> A(M * K), B(K * N), ref(M * N, 0.f);
    for (int i = 0; i < M * K; ++i) A[i] = std::sin(0.37f * i);
    for (int i = 0; i < K * N; ++i) B[i] = std::cos(0.11f * i);
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N; ++n) {
        double acc = 0;
        for (int k = 0; k < K; ++k) acc += (double)A[m * K + k] * B[k * N + n];
        ref[m * N + n] = (float)acc;
      }
    // conv: 3 images, 4 -> 6 channels, 3x3, stride 1, pad 1, 2 groups
    const int Nn = 3, Ci = 4, H = 7, W = 6, Ko = 6, R = 3;
    std::vector<float> x(Nn * Ci * H * W), w(Ko * (Ci / 2) * R * R), dy(Nn * Ko * H * W);
    for (size_t i = 0; i < x.size(); ++i) x[i] = std::sin(0.05f * i);
    for (size_t i = 0; i < w.size(); ++i) w[i] = std::cos(0.3f * i);
    for (size_t i = 0; i < dy.size(); ++i) dy[i] = std::sin(0.7f * i);
    std::vector<float> dw0(w.size(), 0.f), dx0(x.size());
    C::ConvBwd(x.data(), w.data(), dy.data(), dx0.data(), dw0.data(), nullptr, Nn, Ci, H, W, Ko, R, R, H, W, 1, 1, 1,
               1, 1, 1, 2);
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int t = 0; t < 4; ++t)
      th.emplace_back([&, t] {
        for (int it = 0; it < 3; ++it) {
          std::vector<float> Cm(M * N, 0.f);
          if (t % 2)
            C::Gemm(false, false, M, N, K, 1.f, A.data(), K, B.data(), N, 0.f, Cm.data(), N, nullptr, false);
          else  // same product from the transposed storage of B
          {
            std::vector<float> Bt(N * K);
            for (int k = 0; k < K; ++k)
              for (int n = 0; n < N; ++n) Bt[n * K + k] = B[k * N + n];
            C::Gemm(false, true, M, N, K, 1.f, A.data(), K, Bt.data(), K, 0.f, Cm.data(), N, nullptr, false);
          }
          for (int i = 0; i < M * N; ++i)
            if (std::fabs(Cm[i] - ref[i]) > 1e-4f * (1.f + std::fabs(ref[i]))) bad++;
          std::vector<float> dw(w.size(), 0.f), dx(x.size());
          C::ConvBwd(x.data(), w.data(), dy.data(), dx.data(), dw.data(), nullptr, Nn, Ci, H, W, Ko, R, R, H, W, 1, 1,
                     1, 1, 1, 1, 2);
          for (size_t i = 0; i < dw.size(); ++i) bad += dw[i] != dw0[i];  // fixed-order reduction: bitwise
          for (size_t i = 0; i < dx.size(); ++i) bad += dx[i] != dx0[i];
        }
      });
    for (auto& t : th) t.join();
    CHECK(bad.load() == 0);
  }
  std::printf("runtime selftest ok\n");
  return 0;
}

// Native self-test of the host runtime (_core sources), built WITHOUT Python
// under ThreadSanitizer and AddressSanitizer+UBSan by
// tests/test_sanitizers_cpu.py (the reference had no sanitizer
// build; its parser double buffer, include/worker/base_layer.h:510-537, and
// the unlocked paramid2version_ map were never checked).
//
// Exercises every concurrent path of the runtime: several Prefetcher threads
// (producer thread + consumer) over one shard folder, early destruction of a
// Prefetcher while its producer is mid-batch, crash-tolerant append, split,
// and the graph sort / JSON export.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

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
  std::printf("runtime selftest ok\n");
  return 0;
}

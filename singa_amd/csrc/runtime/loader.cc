// Data loader (reference C28, tools/data_loader/data_loader.cc:1-150 and
// data_source.cc:20-77): MNIST idx files -> Shard of SingleLabelImageRecord,
// and shard splitting (Split: first `num` records vs the rest; SplitN: n
// near-equal shards, shard 0 takes the remainder).  Shards are opened in
// kAppend mode so an interrupted run can be restarted (the Shard truncates to
// the last complete tuple and re-keys, src/utils/shard.cc:175-206).
//
// Differences from the reference: every MNIST record gets a key (its index,
// zero-padded); the reference left the key empty so de-duplication dropped
// every record after the first in one session.
#include <sys/stat.h>

#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "runtime.h"

namespace sgrt {

static uint32_t read_be32(std::ifstream& f) {
  unsigned char b[4];
  f.read(reinterpret_cast<char*>(b), 4);
  if (!f) throw std::runtime_error("truncated idx header");
  return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | uint32_t(b[3]);
}

static void make_dir(const std::string& p) { ::mkdir(p.c_str(), 0775); }

int64_t LoadMnist(const std::string& imagefile, const std::string& labelfile, const std::string& folder,
                  int64_t limit) {
  std::ifstream img(imagefile, std::ios::binary), lab(labelfile, std::ios::binary);
  if (!img.is_open()) throw std::runtime_error("unable to open " + imagefile);
  if (!lab.is_open()) throw std::runtime_error("unable to open " + labelfile);
  if (read_be32(img) != 2051) throw std::runtime_error("incorrect image file magic (want 2051)");
  if (read_be32(lab) != 2049) throw std::runtime_error("incorrect label file magic (want 2049)");
  uint32_t n = read_be32(img), nl = read_be32(lab);
  if (n != nl) throw std::runtime_error("image / label count mismatch");
  uint32_t h = read_be32(img), w = read_be32(img);
  make_dir(folder);
  Shard shard(folder, Shard::kAppend);
  int64_t before = shard.Count();
  std::string pix(size_t(h) * w, '\0');
  char key[32];
  int64_t inserted = 0;
  int64_t total = limit > 0 && limit < int64_t(n) ? limit : int64_t(n);
  for (int64_t i = 0; i < total; ++i) {
    img.read(&pix[0], pix.size());
    char label;
    lab.read(&label, 1);
    if (!img || !lab) throw std::runtime_error("truncated idx payload");
    ImageRecord r;
    r.shape = {int32_t(h), int32_t(w)};
    r.label = static_cast<unsigned char>(label);
    r.pixel = pix;
    std::snprintf(key, sizeof(key), "%08lld", static_cast<long long>(i));
    if (shard.Insert(key, EncodeRecord(r))) ++inserted;
  }
  shard.Flush();
  (void)before;
  return inserted;
}

static int64_t copy_n(Shard& from, Shard& to, int64_t n) {
  std::string k, v;
  int64_t c = 0;
  for (; c < n && from.Next(&k, &v); ++c) to.Insert(k, v);
  to.Flush();
  return c;
}

std::vector<int64_t> SplitShard(int64_t num, const std::string& input, const std::string& prefix) {
  Shard origin(input, Shard::kRead);
  int64_t total = origin.Count();
  if (num >= total) throw std::runtime_error("the sub shard should be smaller than the original shard");
  make_dir(prefix + "-0");
  make_dir(prefix + "-1");
  Shard s0(prefix + "-0", Shard::kAppend);
  int64_t a = copy_n(origin, s0, num);
  Shard s1(prefix + "-1", Shard::kAppend);
  int64_t b = copy_n(origin, s1, total - num);
  return {a, b};
}

std::vector<int64_t> SplitShardN(int nshards, const std::string& input, const std::string& prefix) {
  Shard origin(input, Shard::kRead);
  int64_t total = origin.Count();
  if (nshards <= 0 || nshards >= total) throw std::runtime_error("too many sub-shards");
  std::vector<int64_t> counts;
  for (int i = 0; i < nshards; ++i) {
    std::string path = prefix + "-" + std::to_string(i);
    make_dir(path);
    Shard si(path, Shard::kAppend);
    int64_t num = total / nshards + (i == 0 ? total % nshards : 0);
    counts.push_back(copy_n(origin, si, num));
  }
  return counts;
}

}  // namespace sgrt

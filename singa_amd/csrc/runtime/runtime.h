// Host-side C++17 runtime of singa_amd (module _core).
//
//  * Shard      -- bit-compatible re-implementation of the reference's
//                  append-only record file (C20, src/utils/shard.cc:7-206):
//                  [size_t keylen][key][size_t vallen][val] tuples, 100 MB
//                  write buffer, key de-duplication per writer, crash-tolerant
//                  append mode (truncate to the last complete tuple).
//  * Record     -- protobuf wire-format encoder/decoder for singa.Record /
//                  SingleLabelImageRecord (src/proto/model.proto:279-305)
//                  without linking libprotobuf.
//  * Prefetcher -- background std::thread that reads + decodes the next batch
//                  of records into a float image buffer and int labels while
//                  the device computes (the ParserLayer double buffer,
//                  include/worker/base_layer.h:469-560, done natively).
//  * Graph      -- DFS topological sort and node-link JSON export of the layer
//                  DAG (C19, src/utils/graph.cc:8-101).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <fstream>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace sgrt {

class Shard {
 public:
  enum Mode { kRead = 0, kCreate = 1, kAppend = 2 };
  Shard(const std::string& folder, int mode, int64_t capacity = 104857600);
  ~Shard();
  // returns false at end of file or on a truncated tuple
  bool Next(std::string* key, std::string* val);
  // returns false if the key already exists in this writer session or val is empty
  bool Insert(const std::string& key, const std::string& val);
  void Flush();
  void SeekToFirst();
  int64_t Count();
  const std::string& path() const { return path_; }

 private:
  int64_t PrepareForAppend(const std::string& path);
  std::string path_;
  int mode_;
  std::fstream file_;
  std::vector<char> buf_;
  int64_t capacity_, bufsize_ = 0, offset_ = 0;
  std::unordered_set<std::string> keys_;
};

struct ImageRecord {
  std::vector<int32_t> shape;
  int32_t label = 0;
  std::string pixel;
  std::vector<float> data;
};
std::string EncodeRecord(const ImageRecord& r);
bool DecodeRecord(const std::string& bytes, ImageRecord* r);

// Decode one record into a float buffer of `dim` values: pixel bytes are read
// as UNSIGNED (fixes reference quirk: RGBImageLayer casts through signed char,
// src/worker/layer.cc:599); `data` floats are used if present.
// Loader (C28): MNIST idx -> shard; Split / SplitN of a shard folder.
int64_t LoadMnist(const std::string& imagefile, const std::string& labelfile, const std::string& folder,
                  int64_t limit = 0);
std::vector<int64_t> SplitShard(int64_t num, const std::string& input, const std::string& prefix);
std::vector<int64_t> SplitShardN(int nshards, const std::string& input, const std::string& prefix);

bool DecodeRecordToFloat(const std::string& bytes, float* out, int64_t dim, float scale, float bias, int32_t* label);

class Prefetcher {
 public:
  Prefetcher(const std::string& folder, int batch, int64_t dim, float scale, float bias, bool loop);
  ~Prefetcher();
  // Blocks until the next batch is ready; copies it out; starts the next one.
  // Returns the number of valid samples (< batch only at end when !loop).
  int Next(float* images, int32_t* labels);

 private:
  void Fill();
  Shard shard_;
  int batch_;
  int64_t dim_;
  float scale_, bias_;
  bool loop_;
  std::vector<float> img_;
  std::vector<int32_t> lab_;
  int ready_n_ = 0;
  bool ready_ = false, stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
};

struct Graph {
  std::vector<std::string> names;
  std::vector<std::vector<int>> dst;  // adjacency (src -> dst)
  std::unordered_map<std::string, int> index;
  int AddNode(const std::string& name);
  void AddEdge(const std::string& src, const std::string& dst);
  // topological order (DFS, sources first); throws on cycles
  std::vector<std::string> Sort() const;
  std::string ToJson(const std::vector<int>& color) const;
};

}  // namespace sgrt

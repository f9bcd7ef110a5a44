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
#include <memory>
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

// ---- LMDB (lmdb_reader.cc): read-only cursor over data.mdb, Caffe Datum ---
class LmdbReader {
 public:
  explicit LmdbReader(const std::string& path);  // an LMDB directory or its data.mdb
  ~LmdbReader();
  int64_t Count() const;
  void SeekToFirst();
  bool Next(std::string* key, std::string* val);  // false at the end (in key order)

 private:
  struct Impl;
  std::unique_ptr<Impl> d_;
};
// Caffe Datum bytes -> ImageRecord (shape [c, h, w]); *encoded = Datum.encoded
bool DecodeDatum(const std::string& bytes, ImageRecord* r, bool* encoded);

// ---- updaters (updater.cc) ------------------------------------------------
enum UpdKind : int { kSGD = 0, kNesterovRef = 1, kAdaGrad = 2, kRMSProp = 3, kAdaDelta = 4, kAdam = 5, kSGDRef = 6 };
struct UpdateArgs {
  int kind = kSGD;
  float lr = 0.01f, wd = 0.f, grad_scale = 1.f, t = 1.f;
  float momentum = 0.f, dampening = 0.f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, rho = 0.9f;
  bool nesterov = false, adamw = false;
};
int UpdaterKind(const std::string& name);
// w -= update(g) over n fp32 elements; s1/s2 = optimiser slots (history /
// update / Adam moments); optional per-element lr / wd multipliers and mask
void OptUpdate(const UpdateArgs& a, float* w, const float* g, float* s1, float* s2, int64_t n,
               const float* lr_vec = nullptr, const float* wd_vec = nullptr, const uint8_t* mask = nullptr);
double LearningRate(const std::string& method, double base, double final_lr, int freq, double gamma, double pw,
                    int64_t step);

// ---- parameter server (ps.cc) ---------------------------------------------
enum PSType : uint16_t { kPSPing = 0, kPSPut = 1, kPSGet = 2, kPSUpdate = 3, kPSReplace = 4, kPSElastic = 5,
                         kPSRandom = 6, kPSStop = 7 };
struct PSHeader {
  uint32_t magic;
  uint16_t type, flags;
  int32_t id, step;
  float f0;
  uint32_t pad;
  int64_t a, b;
  uint64_t n;
};
static_assert(sizeof(PSHeader) == 48, "PS wire header");

class PServer {
 public:
  // port 0 = any free port (see port()); nworkers = kStop messages to expect
  PServer(int port, int nworkers);
  ~PServer();
  int port() const;
  int64_t messages() const;
  void SetUpdater(const UpdateArgs& a, const std::string& method, double base, double final_lr, int freq,
                  double gamma, double pw);
  bool WaitStop(double timeout_s);  // true once every worker sent kStop
  std::vector<float> Value(int id);
  void Close();

 private:
  struct Impl;
  std::unique_ptr<Impl> d_;
};

class PSClient {
 public:
  PSClient(const std::vector<std::string>& endpoints, int retries = 10, double retry_s = 1.0);
  ~PSClient();
  int nservers() const { return (int)fds_.size(); }
  int server_of(int id) const;
  void Put(int id, const float* w, uint64_t n);
  uint64_t Get(int id, float* out, uint64_t cap);
  void Update(int id, const float* grad, float* w_out, uint64_t n, int step = -1, float grad_scale = 0.f);
  void Elastic(int id, float* w, uint64_t n, float alpha);
  void RandomSync(int id, const float* delta, float* old_out, uint64_t m, int64_t a, int64_t b);
  void PushReplace(int id, const float* w, uint64_t n);
  void PushUpdate(int id, const float* grad, uint64_t n, int step = -1, float grad_scale = 0.f);
  int Collect(const std::vector<float*>& outs, const std::vector<uint64_t>& caps, const std::vector<int>& ids);
  void Stop();

 private:
  void Send(const PSHeader& h, const float* data, size_t server);
  bool Recv(size_t server, PSHeader* r, float* out, uint64_t cap);
  uint64_t Request(const PSHeader& h, const float* data, float* out, uint64_t cap);
  std::vector<int> fds_;
  std::vector<std::vector<int>> pending_;
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

// Shard record file, Record wire codec and the batch Prefetcher.
// See runtime.h for the reference components these re-implement.
#include <sys/stat.h>
#include <sys/types.h>

#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "runtime.h"

namespace sgrt {

static void mkdirs(const std::string& dir) {
  std::string cur;
  for (size_t i = 0; i < dir.size(); ++i) {
    cur.push_back(dir[i]);
    if (dir[i] == '/' || i + 1 == dir.size()) ::mkdir(cur.c_str(), 0755);
  }
}

Shard::Shard(const std::string& folder, int mode, int64_t capacity)
    : path_(folder + "/shard.dat"), mode_(mode), capacity_(capacity) {
  if (mode == kRead) {
    file_.open(path_, std::ios::in | std::ios::binary);
    if (!file_.is_open()) throw std::runtime_error("cannot open shard for read: " + path_);
    buf_.resize(capacity_);
  } else if (mode == kCreate) {
    mkdirs(folder);
    file_.open(path_, std::ios::out | std::ios::binary | std::ios::trunc);
    if (!file_.is_open()) throw std::runtime_error("cannot create shard: " + path_);
    buf_.resize(capacity_);
  } else if (mode == kAppend) {
    mkdirs(folder);
    int64_t last = PrepareForAppend(path_);
    file_.open(path_, std::ios::in | std::ios::out | std::ios::binary);
    if (!file_.is_open()) {
      file_.clear();
      file_.open(path_, std::ios::out | std::ios::binary | std::ios::trunc);
    }
    file_.seekp(last);
    buf_.resize(capacity_);
  } else {
    throw std::runtime_error("bad shard mode");
  }
}

Shard::~Shard() {
  if (mode_ != kRead) Flush();
  file_.close();
}

// Scan the existing file, remember every complete key, truncate a partial
// tail (a crashed write).  Returns the byte offset to append at.
int64_t Shard::PrepareForAppend(const std::string& path) {
  std::ifstream in(path, std::ios::in | std::ios::binary);
  if (!in.is_open()) return 0;
  int64_t last = 0;
  while (true) {
    size_t klen = 0, vlen = 0;
    if (!in.read((char*)&klen, sizeof(size_t))) break;
    std::string key(klen, '\0');
    if (!in.read(&key[0], klen)) break;
    if (!in.read((char*)&vlen, sizeof(size_t))) break;
    in.seekg(vlen, std::ios::cur);
    if (!in.good()) break;
    int64_t pos = in.tellg();
    in.seekg(0, std::ios::end);
    int64_t end = in.tellg();
    if (pos > end) break;
    in.seekg(pos);
    keys_.insert(key);
    last = pos;
  }
  in.close();
  // truncate anything after `last`
  if (::truncate(path.c_str(), last) != 0) { /* new file */ }
  return last;
}

bool Shard::Insert(const std::string& key, const std::string& val) {
  if (keys_.count(key) || val.empty()) return false;
  const int64_t need = 2 * (int64_t)sizeof(size_t) + key.size() + val.size();
  if (bufsize_ + need > capacity_) Flush();
  if (need > capacity_) {  // oversized tuple: write straight through
    size_t kl = key.size(), vl = val.size();
    file_.write((const char*)&kl, sizeof(size_t));
    file_.write(key.data(), kl);
    file_.write((const char*)&vl, sizeof(size_t));
    file_.write(val.data(), vl);
  } else {
    size_t kl = key.size(), vl = val.size();
    char* p = buf_.data() + bufsize_;
    memcpy(p, &kl, sizeof(size_t)); p += sizeof(size_t);
    memcpy(p, key.data(), kl); p += kl;
    memcpy(p, &vl, sizeof(size_t)); p += sizeof(size_t);
    memcpy(p, val.data(), vl);
    bufsize_ += need;
  }
  keys_.insert(key);
  return true;
}

void Shard::Flush() {
  if (mode_ == kRead) return;
  if (bufsize_ > 0) file_.write(buf_.data(), bufsize_);
  file_.flush();
  bufsize_ = 0;
}

bool Shard::Next(std::string* key, std::string* val) {
  size_t klen = 0, vlen = 0;
  if (!file_.read((char*)&klen, sizeof(size_t))) return false;
  key->resize(klen);
  if (klen && !file_.read(&(*key)[0], klen)) return false;
  if (!file_.read((char*)&vlen, sizeof(size_t))) return false;
  val->resize(vlen);
  if (vlen && !file_.read(&(*val)[0], vlen)) return false;
  return true;
}

void Shard::SeekToFirst() {
  file_.clear();
  file_.seekg(0);
}

int64_t Shard::Count() {
  if (mode_ != kRead) Flush();
  std::ifstream in(path_, std::ios::in | std::ios::binary);
  int64_t n = 0;
  while (true) {
    size_t klen = 0, vlen = 0;
    if (!in.read((char*)&klen, sizeof(size_t))) break;
    in.seekg(klen, std::ios::cur);
    if (!in.read((char*)&vlen, sizeof(size_t))) break;
    in.seekg(vlen, std::ios::cur);
    if (!in.good()) break;
    ++n;
  }
  return n;
}

// ---------------- protobuf wire format -------------------------------------
static void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
static bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t* v) {
  uint64_t r = 0;
  int sh = 0;
  while (p < end && sh < 64) {
    uint8_t b = *p++;
    r |= (uint64_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
    sh += 7;
  }
  return false;
}

static std::string encode_image(const ImageRecord& r) {
  std::string s;
  for (int32_t d : r.shape) {  // repeated int32 shape = 1 (unpacked, proto2 default)
    put_varint(s, (1 << 3) | 0);
    put_varint(s, (uint64_t)(int64_t)d);
  }
  put_varint(s, (2 << 3) | 0);
  put_varint(s, (uint64_t)(int64_t)r.label);
  if (!r.pixel.empty()) {
    put_varint(s, (3 << 3) | 2);
    put_varint(s, r.pixel.size());
    s += r.pixel;
  }
  for (float f : r.data) {  // repeated float data = 4 (unpacked)
    put_varint(s, (4 << 3) | 5);
    s.append((const char*)&f, 4);
  }
  return s;
}

std::string EncodeRecord(const ImageRecord& r) {
  std::string s;
  put_varint(s, (1 << 3) | 0);  // type = kSingleLabelImage
  put_varint(s, 0);
  std::string img = encode_image(r);
  put_varint(s, (2 << 3) | 2);
  put_varint(s, img.size());
  s += img;
  return s;
}

static bool skip_field(const uint8_t*& p, const uint8_t* end, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return get_varint(p, end, &v);
    case 1: p += 8; return p <= end;
    case 2: if (!get_varint(p, end, &v)) return false; p += v; return p <= end;
    case 5: p += 4; return p <= end;
  }
  return false;
}

static bool decode_image(const uint8_t* p, const uint8_t* end, ImageRecord* r) {
  while (p < end) {
    uint64_t tag;
    if (!get_varint(p, end, &tag)) return false;
    int field = (int)(tag >> 3), wt = (int)(tag & 7);
    uint64_t v;
    if (field == 1 && wt == 0) {
      if (!get_varint(p, end, &v)) return false;
      r->shape.push_back((int32_t)v);
    } else if (field == 1 && wt == 2) {  // packed shape
      if (!get_varint(p, end, &v)) return false;
      const uint8_t* e = p + v;
      while (p < e) {
        uint64_t x;
        if (!get_varint(p, e, &x)) return false;
        r->shape.push_back((int32_t)x);
      }
    } else if (field == 2 && wt == 0) {
      if (!get_varint(p, end, &v)) return false;
      r->label = (int32_t)v;
    } else if (field == 3 && wt == 2) {
      if (!get_varint(p, end, &v)) return false;
      if (p + v > end) return false;
      r->pixel.assign((const char*)p, v);
      p += v;
    } else if (field == 4 && wt == 5) {
      float f;
      if (p + 4 > end) return false;
      memcpy(&f, p, 4);
      p += 4;
      r->data.push_back(f);
    } else if (field == 4 && wt == 2) {  // packed floats
      if (!get_varint(p, end, &v)) return false;
      if (p + v > end) return false;
      size_t nf = v / 4;
      size_t o = r->data.size();
      r->data.resize(o + nf);
      memcpy(r->data.data() + o, p, nf * 4);
      p += v;
    } else if (!skip_field(p, end, wt)) {
      return false;
    }
  }
  return true;
}

bool DecodeRecord(const std::string& bytes, ImageRecord* r) {
  const uint8_t* p = (const uint8_t*)bytes.data();
  const uint8_t* end = p + bytes.size();
  while (p < end) {
    uint64_t tag;
    if (!get_varint(p, end, &tag)) return false;
    int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if (field == 2 && wt == 2) {
      uint64_t len;
      if (!get_varint(p, end, &len) || p + len > end) return false;
      if (!decode_image(p, p + len, r)) return false;
      p += len;
    } else if (!skip_field(p, end, wt)) {
      return false;
    }
  }
  return true;
}

bool DecodeRecordToFloat(const std::string& bytes, float* out, int64_t dim, float scale, float bias, int32_t* label) {
  ImageRecord r;
  if (!DecodeRecord(bytes, &r)) return false;
  *label = r.label;
  if (!r.data.empty()) {
    int64_t n = std::min<int64_t>(dim, (int64_t)r.data.size());
    for (int64_t i = 0; i < n; ++i) out[i] = r.data[i] * scale + bias;
    for (int64_t i = n; i < dim; ++i) out[i] = 0.f;
  } else {
    const uint8_t* px = (const uint8_t*)r.pixel.data();
    int64_t n = std::min<int64_t>(dim, (int64_t)r.pixel.size());
    for (int64_t i = 0; i < n; ++i) out[i] = (float)px[i] * scale + bias;
    for (int64_t i = n; i < dim; ++i) out[i] = 0.f;
  }
  return true;
}

// ---------------- Prefetcher -------------------------------------------------
Prefetcher::Prefetcher(const std::string& folder, int batch, int64_t dim, float scale, float bias, bool loop)
    : shard_(folder, Shard::kRead), batch_(batch), dim_(dim), scale_(scale), bias_(bias), loop_(loop),
      img_((size_t)batch * dim), lab_(batch) {
  th_ = std::thread([this] { Fill(); });
}

Prefetcher::~Prefetcher() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void Prefetcher::Fill() {
  std::string key, val;
  while (true) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return stop_ || !ready_; });
    if (stop_) return;
    lk.unlock();
    int n = 0;
    while (n < batch_) {
      if (!shard_.Next(&key, &val)) {
        if (!loop_) break;
        shard_.SeekToFirst();  // wrap around (fixes reference quirk #25)
        if (!shard_.Next(&key, &val)) break;
      }
      if (DecodeRecordToFloat(val, img_.data() + (int64_t)n * dim_, dim_, scale_, bias_, &lab_[n])) ++n;
    }
    lk.lock();
    ready_n_ = n;
    ready_ = true;
    cv_.notify_all();
  }
}

int Prefetcher::Next(float* images, int32_t* labels) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [this] { return ready_; });
  int n = ready_n_;
  memcpy(images, img_.data(), sizeof(float) * (size_t)n * dim_);
  memcpy(labels, lab_.data(), sizeof(int32_t) * n);
  ready_ = false;
  cv_.notify_all();
  return n;
}

}  // namespace sgrt

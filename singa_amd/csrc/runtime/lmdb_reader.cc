// Native read-only LMDB cursor + Caffe Datum decoder for the kLMDBData layer
// (reference LMDBDataLayer, src/worker/layer.cc:237-328, which links liblmdb
// and walks an MDB_cursor with MDB_FIRST / MDB_NEXT, wrapping at the end;
// Datum -> Record conversion at :278-295).  Neither liblmdb nor the Python
// lmdb module exists in this environment, so the on-disk format (LMDB data
// version 1, 64-bit build) is read directly from an mmap of data.mdb:
//
//   page header (16 B): pgno u64 | pad u16 | flags u16 | lower u16 | upper u16
//                       (overflow pages: lower/upper = page count u32)
//   meta pages 0 and 1: header + MDB_meta {magic 0xBEEFC0DE u32, version u32,
//       address u64, mapsize u64, dbs[2] x MDB_db(48 B), last_pg u64,
//       txnid u64}; the page size lives in dbs[FREE].md_pad; the valid meta
//       is the one with the larger txnid; MAIN db = dbs[1], md_root = root.
//   branch / leaf pages: u16 node offsets after the header, count =
//       (lower - 16) / 2; node = lo u16 | hi u16 | flags u16 | ksize u16 |
//       key | data.  Branch child pgno = lo | hi<<16 | flags<<32; leaf data
//       size = lo | hi<<16; F_BIGDATA (1): data is the u64 pgno of an
//       overflow page whose payload follows its header.
//
// Iteration is an in-order walk of the B+tree (keys come out sorted, as with
// MDB_NEXT).  Sub-databases / dupsort trees (F_SUBDATA / F_DUPDATA) are not
// used by Caffe-style datasets and are rejected.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "runtime.h"

namespace sgrt {

namespace {
constexpr uint32_t kMdbMagic = 0xBEEFC0DEu;
constexpr int kPageHdr = 16;
constexpr uint16_t P_BRANCH = 0x01, P_LEAF = 0x02, P_OVERFLOW = 0x04, P_LEAF2 = 0x20;
constexpr uint16_t F_BIGDATA = 0x01, F_SUBDATA = 0x02, F_DUPDATA = 0x04;

template <typename T>
T rd(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}
}  // namespace

struct LmdbReader::Impl {
  int fd = -1;
  const uint8_t* base = nullptr;
  size_t size = 0;
  uint32_t psize = 4096;
  uint64_t root = ~0ull, entries = 0;
  // cursor: stack of (page, index)
  std::vector<std::pair<uint64_t, int>> stack;
  bool at_end = true;

  const uint8_t* page(uint64_t pg) const {
    if ((pg + 1) * (uint64_t)psize > size) throw std::runtime_error("lmdb: page number out of range");
    return base + pg * psize;
  }
  int nkeys(const uint8_t* p) const { return (rd<uint16_t>(p + 12) - kPageHdr) >> 1; }
  const uint8_t* node(const uint8_t* p, int i) const {
    const uint16_t off = rd<uint16_t>(p + kPageHdr + 2 * i);
    if (off + 8 > psize) throw std::runtime_error("lmdb: node offset out of range");
    return p + off;
  }
  // descend from pg to its leftmost leaf, pushing (page, 0) entries
  void descend(uint64_t pg) {
    for (int depth = 0; depth < 64; ++depth) {
      const uint8_t* p = page(pg);
      const uint16_t flags = rd<uint16_t>(p + 10);
      stack.emplace_back(pg, 0);
      if (flags & P_LEAF2) throw std::runtime_error("lmdb: LEAF2 (dupfixed) pages are not supported");
      if (flags & P_LEAF) return;
      if (!(flags & P_BRANCH)) throw std::runtime_error("lmdb: unexpected page type");
      if (nkeys(p) == 0) throw std::runtime_error("lmdb: empty branch page");
      const uint8_t* n = node(p, 0);
      pg = (uint64_t)rd<uint16_t>(n) | ((uint64_t)rd<uint16_t>(n + 2) << 16) | ((uint64_t)rd<uint16_t>(n + 4) << 32);
    }
    throw std::runtime_error("lmdb: tree too deep");
  }
  // advance to the next leaf entry (stack top points at a leaf); false at end
  bool settle() {
    while (!stack.empty()) {
      auto& top = stack.back();
      const uint8_t* p = page(top.first);
      if (top.second < nkeys(p)) {
        if (rd<uint16_t>(p + 10) & P_LEAF) return true;
        const uint8_t* n = node(p, top.second);
        const uint64_t child =
            (uint64_t)rd<uint16_t>(n) | ((uint64_t)rd<uint16_t>(n + 2) << 16) | ((uint64_t)rd<uint16_t>(n + 4) << 32);
        descend(child);
        continue;
      }
      stack.pop_back();
      if (!stack.empty()) stack.back().second++;
    }
    return false;
  }
};

LmdbReader::LmdbReader(const std::string& path) : d_(new Impl()) {
  std::string file = path;
  struct stat st;
  if (stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) file = path + "/data.mdb";
  d_->fd = ::open(file.c_str(), O_RDONLY);
  if (d_->fd < 0) throw std::runtime_error("lmdb: cannot open " + file);
  if (fstat(d_->fd, &st) != 0 || st.st_size < 2 * kPageHdr + 136) throw std::runtime_error("lmdb: file too small");
  d_->size = (size_t)st.st_size;
  void* m = ::mmap(nullptr, d_->size, PROT_READ, MAP_SHARED, d_->fd, 0);
  if (m == MAP_FAILED) throw std::runtime_error("lmdb: mmap failed");
  d_->base = (const uint8_t*)m;
  // meta 0 gives the page size; the newer of the two metas wins
  auto meta = [&](size_t off, uint64_t* txn, uint64_t* root, uint64_t* entries, uint32_t* psize) {
    if (off + kPageHdr + 136 > d_->size) return false;
    const uint8_t* mm = d_->base + off + kPageHdr;
    if (rd<uint32_t>(mm) != kMdbMagic) return false;
    if (rd<uint32_t>(mm + 4) != 1) throw std::runtime_error("lmdb: unsupported data version");
    const uint8_t* dbs = mm + 24;  // magic, version, address, mapsize
    *psize = rd<uint32_t>(dbs);    // dbs[FREE].md_pad = page size
    const uint8_t* main = dbs + 48;
    if (rd<uint16_t>(main + 4) & 0x04) throw std::runtime_error("lmdb: dupsort databases are not supported");
    *entries = rd<uint64_t>(main + 32);
    *root = rd<uint64_t>(main + 40);
    *txn = rd<uint64_t>(dbs + 96 + 8);
    return true;
  };
  uint64_t t0 = 0, r0 = 0, e0 = 0, t1 = 0, r1 = 0, e1 = 0;
  uint32_t ps0 = 0, ps1 = 0;
  if (!meta(0, &t0, &r0, &e0, &ps0)) throw std::runtime_error("lmdb: bad meta page (not an LMDB file?)");
  const bool m1 = ps0 >= 512 && meta(ps0, &t1, &r1, &e1, &ps1);
  d_->psize = ps0;
  if (m1 && t1 > t0) {
    d_->root = r1;
    d_->entries = e1;
  } else {
    d_->root = r0;
    d_->entries = e0;
  }
  SeekToFirst();
}

LmdbReader::~LmdbReader() {
  if (d_->base) ::munmap((void*)d_->base, d_->size);
  if (d_->fd >= 0) ::close(d_->fd);
}

int64_t LmdbReader::Count() const { return (int64_t)d_->entries; }

void LmdbReader::SeekToFirst() {
  d_->stack.clear();
  d_->at_end = true;
  if (d_->root == ~0ull || d_->entries == 0) return;  // P_INVALID root: empty database
  d_->descend(d_->root);
  d_->at_end = !d_->settle();
}

bool LmdbReader::Next(std::string* key, std::string* val) {
  if (d_->at_end) return false;
  auto& top = d_->stack.back();
  const uint8_t* p = d_->page(top.first);
  const uint8_t* n = d_->node(p, top.second);
  const uint16_t flags = rd<uint16_t>(n + 4), ksize = rd<uint16_t>(n + 6);
  if (flags & (F_SUBDATA | F_DUPDATA)) throw std::runtime_error("lmdb: sub-databases / dup data not supported");
  const uint64_t dsize = (uint64_t)rd<uint16_t>(n) | ((uint64_t)rd<uint16_t>(n + 2) << 16);
  key->assign((const char*)n + 8, ksize);
  const uint8_t* data = n + 8 + ksize;
  if (flags & F_BIGDATA) {
    const uint64_t opg = rd<uint64_t>(data);
    const uint8_t* op = d_->page(opg);
    if (!(rd<uint16_t>(op + 10) & P_OVERFLOW)) throw std::runtime_error("lmdb: bad overflow page");
    if ((opg * d_->psize) + kPageHdr + dsize > d_->size) throw std::runtime_error("lmdb: overflow data out of range");
    val->assign((const char*)op + kPageHdr, dsize);
  } else {
    if ((size_t)(data - p) + dsize > d_->psize) throw std::runtime_error("lmdb: node data out of range");
    val->assign((const char*)data, dsize);
  }
  top.second++;
  d_->at_end = !d_->settle();
  return true;
}

// Caffe Datum (src/proto/model.proto:288-299): channels=1 height=2 width=3
// data=4 (bytes) label=5 float_data=6 (repeated float, packed or not)
// encoded=7 -> an ImageRecord with shape [channels, height, width].
bool DecodeDatum(const std::string& bytes, ImageRecord* r, bool* encoded) {
  const uint8_t* p = (const uint8_t*)bytes.data();
  const uint8_t* e = p + bytes.size();
  auto varint = [&](uint64_t* v) {
    *v = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
      const uint8_t b = *p++;
      *v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return true;
    }
    return false;
  };
  int64_t ch = 0, h = 0, w = 0;
  *encoded = false;
  r->pixel.clear();
  r->data.clear();
  r->label = 0;
  while (p < e) {
    uint64_t tag;
    if (!varint(&tag)) return false;
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    uint64_t v = 0;
    if (wt == 0) {
      if (!varint(&v)) return false;
      if (field == 1) ch = (int64_t)v;
      else if (field == 2) h = (int64_t)v;
      else if (field == 3) w = (int64_t)v;
      else if (field == 5) r->label = (int32_t)v;
      else if (field == 7) *encoded = v != 0;
    } else if (wt == 2) {
      if (!varint(&v) || (uint64_t)(e - p) < v) return false;
      if (field == 4) r->pixel.assign((const char*)p, v);
      else if (field == 6) {
        for (uint64_t i = 0; i + 4 <= v; i += 4) r->data.push_back(rd<float>(p + i));
      }
      p += v;
    } else if (wt == 5) {
      if (e - p < 4) return false;
      if (field == 6) r->data.push_back(rd<float>(p));
      p += 4;
    } else if (wt == 1) {
      if (e - p < 8) return false;
      p += 8;
    } else {
      return false;
    }
  }
  r->shape = {(int32_t)ch, (int32_t)h, (int32_t)w};
  return true;
}

}  // namespace sgrt

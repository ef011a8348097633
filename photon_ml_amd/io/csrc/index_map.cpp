// photon_ml_amd off-heap feature index map: an mmap'd open-addressing hash table (name <-> index).
//
// Replaces PalDB (photon-api/.../index/PalDBIndexMap.scala:43-278, PalDBIndexMapBuilder.scala) used by the
// reference for feature spaces too large for an in-heap map (> 200k features). The file is built once (offline,
// FeatureIndexingDriver) and then memory-mapped read-only by every process: lookups touch only the pages they
// need, nothing is deserialised, and many ranks on one host share the page cache.
//
// File layout (little endian):
//   char magic[8] = "PMLIDX01"; uint64 n; uint64 nbuckets (power of two); uint64 blob_bytes
//   uint32 bucket[nbuckets]          (entry id + 1, 0 = empty), linear probing on FNV-1a 64
//   uint64 offset[n + 1]             (byte offsets of key i in the blob; key id == position)
//   char blob[blob_bytes]
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <atomic>
#include <functional>
#include <string_view>

// Build id (photon_ml_amd/ops/build.py: content hash of the sources + compile command, -DPML_BUILD_ID=...): the
// loaders compare it with the tree's sources and refuse a stale library.
#ifndef PML_BUILD_ID
#define PML_BUILD_ID "unstamped-build!"
#endif
__attribute__((used)) static const char pml_build_stamp[] = "PML_BUILD_ID=" PML_BUILD_ID;

static inline uint64_t fnv1a(const char* s, size_t n) {
  uint64_t h = 1469598103934665603ULL;
  for (size_t i = 0; i < n; ++i) { h ^= (unsigned char)s[i]; h *= 1099511628211ULL; }
  return h;
}

struct IndexMapFile {
  void* base = nullptr;
  size_t size = 0;
  uint64_t n = 0, nb = 0, blob_bytes = 0;
  const uint32_t* buckets = nullptr;
  const uint64_t* offsets = nullptr;
  const char* blob = nullptr;
};

extern "C" {

const char* pml_build_id() { return pml_build_stamp + 13; }

// keys: concatenated bytes; offs: int64[n + 1]. Returns 0 on success, -1 on I/O error, -2 on duplicate key.
int pml_im_build(const char* keys, const int64_t* offs, int64_t n, const char* path) {
  uint64_t nb = 16;
  while (nb < (uint64_t)n * 2) nb <<= 1;
  std::vector<uint32_t> buckets(nb, 0);
  for (int64_t i = 0; i < n; ++i) {
    const char* k = keys + offs[i];
    size_t len = (size_t)(offs[i + 1] - offs[i]);
    uint64_t b = fnv1a(k, len) & (nb - 1);
    while (buckets[b] != 0) {
      int64_t j = (int64_t)buckets[b] - 1;
      size_t lj = (size_t)(offs[j + 1] - offs[j]);
      if (lj == len && memcmp(keys + offs[j], k, len) == 0) return -2;
      b = (b + 1) & (nb - 1);
    }
    buckets[b] = (uint32_t)(i + 1);
  }
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  uint64_t hdr[3] = {(uint64_t)n, nb, (uint64_t)(n > 0 ? offs[n] : 0)};
  fwrite("PMLIDX01", 1, 8, f);
  fwrite(hdr, 8, 3, f);
  fwrite(buckets.data(), 4, nb, f);
  std::vector<uint64_t> o(n + 1);
  for (int64_t i = 0; i <= n; ++i) o[i] = (uint64_t)(n > 0 ? offs[i] : 0);
  fwrite(o.data(), 8, (size_t)n + 1, f);
  if (n > 0) fwrite(keys, 1, (size_t)offs[n], f);
  return fclose(f) == 0 ? 0 : -1;
}

void* pml_im_open(const char* path) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); return nullptr; }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  if (st.st_size < 32 || memcmp(p, "PMLIDX01", 8) != 0) { munmap(p, (size_t)st.st_size); return nullptr; }
  IndexMapFile* h = new IndexMapFile();
  h->base = p; h->size = (size_t)st.st_size;
  const uint64_t* hdr = (const uint64_t*)((const char*)p + 8);
  h->n = hdr[0]; h->nb = hdr[1]; h->blob_bytes = hdr[2];
  h->buckets = (const uint32_t*)((const char*)p + 32);
  h->offsets = (const uint64_t*)((const char*)h->buckets + 4 * h->nb);
  h->blob = (const char*)(h->offsets + h->n + 1);
  return h;
}

void pml_im_close(void* hp) {
  IndexMapFile* h = (IndexMapFile*)hp;
  if (!h) return;
  munmap(h->base, h->size);
  delete h;
}

int64_t pml_im_size(void* hp) { return hp ? (int64_t)((IndexMapFile*)hp)->n : -1; }

int64_t pml_im_lookup(void* hp, const char* k, int64_t len) {
  IndexMapFile* h = (IndexMapFile*)hp;
  if (!h || h->n == 0) return -1;
  uint64_t b = fnv1a(k, (size_t)len) & (h->nb - 1);
  while (true) {
    uint32_t e = h->buckets[b];
    if (e == 0) return -1;
    uint64_t j = e - 1;
    uint64_t lj = h->offsets[j + 1] - h->offsets[j];
    if ((int64_t)lj == len && memcmp(h->blob + h->offsets[j], k, (size_t)len) == 0) return (int64_t)j;
    b = (b + 1) & (h->nb - 1);
  }
}

// batch lookup: keys concatenated with offsets[n + 1]; out[n] = index or -1
void pml_im_lookup_many(void* hp, const char* keys, const int64_t* offs, int64_t n, int64_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = pml_im_lookup(hp, keys + offs[i], offs[i + 1] - offs[i]);
}

// copies key `id` into buf (if cap allows); returns its length or -1
int64_t pml_im_name(void* hp, int64_t id, char* buf, int64_t cap) {
  IndexMapFile* h = (IndexMapFile*)hp;
  if (!h || id < 0 || (uint64_t)id >= h->n) return -1;
  uint64_t a = h->offsets[id], b = h->offsets[id + 1];
  int64_t len = (int64_t)(b - a);
  if (buf && cap >= len) memcpy(buf, h->blob + a, (size_t)len);
  return len;
}
}

// ===============================================================================================================
// PalDB V1 stores (the reference's off-heap index format), natively: mmap'd reader with PalDB's own slot probing,
// and a writer that produces the bytes of the Python reference writer (io/paldb.py write_store) and of the
// reference's shipped stores.
//
// Reference: photon-api/.../index/PalDBIndexMap.scala:43-278 (one store per partition, both directions per store,
// global index = local index + sum of the preceding partitions' sizes, partition = nonNegativeMod(key.hashCode, n))
// and photon-client/.../index/FeatureIndexingDriver.scala:262-291 (stores built per partition). On-disk layout:
// see io/paldb.py. Keys cross the C ABI as UTF-8 strings separated by NUL bytes (one Python encode for a batch).
// ===============================================================================================================
#include <algorithm>
#include <cmath>
#include <string>
#include <thread>

namespace pdb {

static thread_local std::string g_err;

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// MurmurHash3 x86 32-bit, seed 42 (PalDB HashUtils)
static uint32_t murmur3_32(const uint8_t* d, size_t n, uint32_t seed = 42) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h = seed;
  size_t nb = n / 4;
  for (size_t i = 0; i < nb; ++i) {
    uint32_t k = (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) |
                 ((uint32_t)d[4 * i + 3] << 24);
    k *= c1; k = rotl32(k, 15); k *= c2;
    h ^= k; h = rotl32(h, 13); h = h * 5 + 0xe6546b64u;
  }
  const uint8_t* t = d + 4 * nb;
  uint32_t k = 0;
  switch (n & 3) {
    case 3: k ^= (uint32_t)t[2] << 16; [[fallthrough]];
    case 2: k ^= (uint32_t)t[1] << 8; [[fallthrough]];
    case 1: k ^= t[0]; k *= c1; k = rotl32(k, 15); k *= c2; h ^= k;
  }
  h ^= (uint32_t)n;
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}

static inline void pack_varint(std::string& out, uint64_t v) {   // LongPacker.packLong
  while (v >= 0x80) { out.push_back((char)((v & 0x7f) | 0x80)); v >>= 7; }
  out.push_back((char)v);
}
static inline int varint_len(uint64_t v) { int n = 1; while (v >= 0x80) { v >>= 7; ++n; } return n; }

// LongPacker.unpackLong; returns false past `end`
static inline bool unpack_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (p >= end) return false;
    uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}

// UTF-8 -> UTF-16 code units (supplementary code points as surrogate pairs, like Java strings)
static bool utf16_units(const char* s, size_t n, std::vector<uint16_t>& u) {
  u.clear();
  const uint8_t* p = (const uint8_t*)s;
  const uint8_t* e = p + n;
  while (p < e) {
    uint32_t c = *p++;
    int extra = 0;
    if (c < 0x80) {
    } else if ((c & 0xe0) == 0xc0) { c &= 0x1f; extra = 1; }
    else if ((c & 0xf0) == 0xe0) { c &= 0x0f; extra = 2; }
    else if ((c & 0xf8) == 0xf0) { c &= 0x07; extra = 3; }
    else return false;
    for (int i = 0; i < extra; ++i) {
      if (p >= e || (*p & 0xc0) != 0x80) return false;
      c = (c << 6) | (*p++ & 0x3f);
    }
    if (c >= 0x10000) {
      c -= 0x10000;
      u.push_back((uint16_t)(0xd800 + (c >> 10)));
      u.push_back((uint16_t)(0xdc00 + (c & 0x3ff)));
    } else {
      u.push_back((uint16_t)c);
    }
  }
  return true;
}

static void utf8_append(std::string& out, uint32_t c) {
  if (c < 0x80) out.push_back((char)c);
  else if (c < 0x800) { out.push_back((char)(0xc0 | (c >> 6))); out.push_back((char)(0x80 | (c & 0x3f))); }
  else if (c < 0x10000) {
    out.push_back((char)(0xe0 | (c >> 12))); out.push_back((char)(0x80 | ((c >> 6) & 0x3f)));
    out.push_back((char)(0x80 | (c & 0x3f)));
  } else {
    out.push_back((char)(0xf0 | (c >> 18))); out.push_back((char)(0x80 | ((c >> 12) & 0x3f)));
    out.push_back((char)(0x80 | ((c >> 6) & 0x3f))); out.push_back((char)(0x80 | (c & 0x3f)));
  }
}

static inline int32_t java_hash(const std::vector<uint16_t>& u) {
  uint32_t h = 0;
  for (uint16_t x : u) h = 31u * h + x;
  return (int32_t)h;
}

// PalDB StorageSerialization of an int / a string (the only types an index store holds)
static void ser_int(std::string& out, int64_t v) {
  if (v >= -1 && v <= 8) { out.push_back((char)(v + 5)); return; }
  if (v >= 0 && v < 255) { out.push_back((char)14); out.push_back((char)v); return; }
  if (v < 0) { out.push_back((char)15); pack_varint(out, (uint64_t)(-v)); }
  else { out.push_back((char)16); pack_varint(out, (uint64_t)v); }
}
static void ser_str(std::string& out, const std::vector<uint16_t>& u) {
  out.push_back((char)103);
  pack_varint(out, u.size());
  for (uint16_t x : u) pack_varint(out, x);
}

struct Block { int32_t klen, count, slots, slot_size, idx_off; int64_t data_off; };

struct Store {
  const uint8_t* base = nullptr;
  size_t size = 0;
  int32_t key_count = 0, max_len = 0;
  int64_t index_start = 0, data_start = 0;
  std::vector<Block> blocks;
  std::vector<int32_t> by_len;        // key length -> block (or -1)

  ~Store() { if (base) munmap((void*)base, size); }

  bool open(const char* path) {
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) { g_err = std::string("cannot open ") + path; return false; }
    struct stat st;
    if (fstat(fd, &st) != 0) { ::close(fd); g_err = "fstat failed"; return false; }
    size = (size_t)st.st_size;
    void* p = size ? mmap(nullptr, size, PROT_READ, MAP_SHARED, fd, 0) : MAP_FAILED;
    ::close(fd);
    if (p == MAP_FAILED) { size = 0; g_err = std::string("cannot map ") + path; return false; }
    base = (const uint8_t*)p;
    return parse(path);
  }

  bool need(size_t pos, size_t n, const char* path) {
    if (pos + n > size) { g_err = std::string(path) + ": truncated PalDB header"; return false; }
    return true;
  }
  int32_t be32(size_t pos) const {
    return (int32_t)(((uint32_t)base[pos] << 24) | ((uint32_t)base[pos + 1] << 16) | ((uint32_t)base[pos + 2] << 8) |
                     (uint32_t)base[pos + 3]);
  }
  int64_t be64(size_t pos) const { return ((int64_t)(uint32_t)be32(pos) << 32) | (uint32_t)be32(pos + 4); }

  bool parse(const char* path) {
    if (!need(0, 2, path)) return false;
    size_t n = ((size_t)base[0] << 8) | base[1];
    if (!need(2, n, path) || n != 8 || memcmp(base + 2, "PALDB_V1", 8) != 0) {
      g_err = std::string(path) + ": not a PalDB V1 store";
      return false;
    }
    size_t pos = 2 + n + 8;                 // + timestamp
    if (!need(pos, 12, path)) return false;
    key_count = be32(pos); int32_t n_len = be32(pos + 4); max_len = be32(pos + 8);
    pos += 12;
    if (n_len < 0 || max_len < 0 || max_len > (1 << 20)) { g_err = std::string(path) + ": bad header"; return false; }
    by_len.assign((size_t)max_len + 1, -1);
    for (int32_t i = 0; i < n_len; ++i) {
      if (!need(pos, 28, path)) return false;
      Block b{be32(pos), be32(pos + 4), be32(pos + 8), be32(pos + 12), be32(pos + 16), be64(pos + 20)};
      pos += 28;
      if (b.klen <= 0 || b.klen > max_len || b.slots <= 0 || b.slot_size <= b.klen) {
        g_err = std::string(path) + ": bad key-length block";
        return false;
      }
      by_len[(size_t)b.klen] = (int32_t)blocks.size();
      blocks.push_back(b);
    }
    if (!need(pos, 16, path)) return false;
    if (be32(pos) != 0) { g_err = std::string(path) + ": custom PalDB serializers are not supported"; return false; }
    index_start = be32(pos + 4);
    data_start = be64(pos + 8);
    for (const Block& b : blocks) {
      if ((uint64_t)index_start + (uint64_t)b.idx_off + (uint64_t)b.slots * (uint64_t)b.slot_size > size ||
          (uint64_t)data_start + (uint64_t)b.data_off > size) {
        g_err = std::string(path) + ": index / data section outside the file";
        return false;
      }
    }
    return true;
  }

  // value bytes of serialized key `k` (PalDB's probe: hash slot, linear probing, offset 0 = absent)
  const uint8_t* find(const std::string& k, const uint8_t** vend) const {
    if (k.size() >= by_len.size() || by_len[k.size()] < 0) return nullptr;
    const Block& b = blocks[(size_t)by_len[k.size()]];
    uint64_t s = (uint64_t)(murmur3_32((const uint8_t*)k.data(), k.size()) & 0x7fffffffu) % (uint64_t)b.slots;
    const uint8_t* ix = base + index_start + b.idx_off;
    const uint8_t* end = base + size;
    for (int32_t probe = 0; probe < b.slots; ++probe) {
      const uint8_t* slot = ix + s * (uint64_t)b.slot_size;
      const uint8_t* q = slot + b.klen;
      uint64_t off;
      if (!unpack_varint(q, slot + b.slot_size, off) || off == 0) return nullptr;
      if (memcmp(slot, k.data(), (size_t)b.klen) == 0) {
        const uint8_t* v = base + data_start + b.data_off + off;
        uint64_t vlen;
        if (v >= end || !unpack_varint(v, end, vlen) || v + vlen > end) return nullptr;
        *vend = v + vlen;
        return v;
      }
      s = (s + 1 == (uint64_t)b.slots) ? 0 : s + 1;
    }
    return nullptr;
  }
};

static bool de_int(const uint8_t* v, const uint8_t* e, int64_t& out) {
  if (v >= e) return false;
  uint8_t c = *v++;
  if (c >= 4 && c <= 13) { out = (int64_t)c - 5; return v == e; }
  if (c == 14) { if (v >= e) return false; out = *v++; return v == e; }
  if (c == 15 || c == 16) {
    uint64_t x;
    if (!unpack_varint(v, e, x)) return false;
    out = c == 15 ? -(int64_t)x : (int64_t)x;
    return v == e;
  }
  return false;
}

static bool de_str(const uint8_t* v, const uint8_t* e, std::string& out) {
  if (v >= e || *v++ != 103) return false;
  uint64_t n;
  if (!unpack_varint(v, e, n)) return false;
  out.clear();
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t u;
    if (!unpack_varint(v, e, u) || u > 0xffff) return false;
    if (u >= 0xd800 && u < 0xdc00 && i + 1 < n) {        // surrogate pair -> one code point
      const uint8_t* v2 = v;
      uint64_t lo;
      if (unpack_varint(v2, e, lo) && lo >= 0xdc00 && lo < 0xe000) {
        v = v2; ++i;
        utf8_append(out, 0x10000 + (((uint32_t)u - 0xd800) << 10) + ((uint32_t)lo - 0xdc00));
        continue;
      }
    }
    utf8_append(out, (uint32_t)u);
  }
  return v == e;
}

struct Map {
  std::vector<Store*> parts;
  std::vector<int64_t> offsets;          // [P + 1] global index of each partition's local index 0
  ~Map() { for (Store* s : parts) delete s; }
};

// NUL-separated keys -> [n + 1] byte offsets (key i = blob[offs[i], offs[i + 1] - 1)); false if the count differs
static bool split_nul(const char* blob, int64_t len, int64_t n, std::vector<int64_t>& offs) {
  offs.assign((size_t)n + 1, 0);
  if (n == 0) { offs[0] = len + 1; return len == 0; }
  int64_t i = 0, pos = 0;
  while (i < n) {
    const void* z = memchr(blob + pos, 0, (size_t)(len - pos));
    int64_t end = z ? (int64_t)((const char*)z - blob) : len;
    offs[(size_t)i] = pos;
    ++i;
    pos = end + 1;
    if (!z) break;
  }
  offs[(size_t)n] = len + 1;
  return i == n && pos == len + 1;
}

static void run_parallel(int64_t n, int64_t min_per_thread, const std::function<void(int64_t, int64_t)>& fn) {
  int64_t nt = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  nt = std::max<int64_t>(1, std::min(nt, n / std::max<int64_t>(min_per_thread, 1)));
  if (nt <= 1) { fn(0, n); return; }
  std::vector<std::thread> th;
  for (int64_t t = 0; t < nt; ++t) th.emplace_back(fn, n * t / nt, n * (t + 1) / nt);
  for (auto& x : th) x.join();
}

// sorts idx by key bytes (= code point order for UTF-8): chunks sorted in parallel, then merged pairwise
template <class Less>
static void parallel_sort(std::vector<int64_t>& idx, Less less) {
  const int64_t n = (int64_t)idx.size();
  int64_t T = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  while (T > 1 && n / T < (1 << 16)) T >>= 1;
  if (T <= 1) { std::sort(idx.begin(), idx.end(), less); return; }
  std::vector<int64_t> bounds;
  for (int64_t t = 0; t <= T; ++t) bounds.push_back(n * t / T);
  {
    std::vector<std::thread> th;
    for (int64_t t = 0; t < T; ++t)
      th.emplace_back([&, t] { std::sort(idx.begin() + bounds[(size_t)t], idx.begin() + bounds[(size_t)t + 1], less); });
    for (auto& x : th) x.join();
  }
  std::vector<int64_t> tmp((size_t)n);
  std::vector<int64_t>* src = &idx;
  std::vector<int64_t>* dst = &tmp;
  while (bounds.size() > 2) {
    std::vector<int64_t> nb;
    std::vector<std::thread> th;
    for (size_t i = 0; i + 1 < bounds.size(); i += 2) {
      int64_t lo = bounds[i], mid = bounds[i + 1], hi = i + 2 < bounds.size() ? bounds[i + 2] : mid;
      nb.push_back(lo);
      th.emplace_back([=] {
        std::merge(src->begin() + lo, src->begin() + mid, src->begin() + mid, src->begin() + hi, dst->begin() + lo, less);
      });
    }
    nb.push_back(n);
    for (auto& x : th) x.join();
    bounds.swap(nb);
    std::swap(src, dst);
  }
  if (src != &idx) idx.swap(tmp);
}

// one store holding key i -> i and i -> key i for the keys in `idx` order (io/paldb.py write_store byte layout).
// Entries 0..n-1 are (name -> index), n..2n-1 (index -> name), PalDB's insertion order. All serialized bytes live in
// one buffer; the only sequential step is the slot assignment (linear probing in insertion order over a byte map).
static int write_store(const char* path, const char* blob, const std::vector<int64_t>& offs,
                       const std::vector<int64_t>& idx, int64_t timestamp) {
  const int64_t n = (int64_t)idx.size();
  const int64_t m = 2 * n;
  // serialized name of entry i < n: kbuf[kofs[i], kofs[i + 1]); ints are serialized on the fly
  std::vector<int64_t> klen((size_t)n + 1, 0);
  std::atomic<bool> bad{false};
  auto key_of = [&](int64_t i) {
    int64_t j = idx[(size_t)i];
    return std::string_view(blob + offs[(size_t)j], (size_t)(offs[(size_t)j + 1] - 1 - offs[(size_t)j]));
  };
  run_parallel(n, 1 << 14, [&](int64_t a, int64_t b) {
    std::vector<uint16_t> u;
    std::string k;
    for (int64_t i = a; i < b; ++i) {
      auto kv = key_of(i);
      if (!utf16_units(kv.data(), kv.size(), u)) bad = true;
      k.clear();
      ser_str(k, u);
      klen[(size_t)i + 1] = (int64_t)k.size();
    }
  });
  if (bad) { g_err = "invalid UTF-8 key"; return -3; }
  for (int64_t i = 0; i < n; ++i) klen[(size_t)i + 1] += klen[(size_t)i];
  std::string kbuf((size_t)klen[(size_t)n], '\0');
  run_parallel(n, 1 << 14, [&](int64_t a, int64_t b) {
    std::vector<uint16_t> u;
    std::string k;
    for (int64_t i = a; i < b; ++i) {
      auto kv = key_of(i);
      utf16_units(kv.data(), kv.size(), u);
      k.clear();
      ser_str(k, u);
      memcpy(&kbuf[(size_t)klen[(size_t)i]], k.data(), k.size());
    }
  });
  auto int_ser = [](int64_t v, char* out) {      // serialized int into out (<= 11 bytes); returns its length
    std::string t;
    ser_int(t, v);
    memcpy(out, t.data(), t.size());
    return (int)t.size();
  };
  auto int_len = [](int64_t v) -> int {
    if (v >= -1 && v <= 8) return 1;
    if (v >= 0 && v < 255) return 2;
    return 1 + varint_len((uint64_t)(v < 0 ? -v : v));
  };
  auto key_len = [&](int64_t e) -> int64_t { return e < n ? klen[(size_t)e + 1] - klen[(size_t)e] : int_len(e - n); };
  auto val_len = [&](int64_t e) -> int64_t { return e < n ? int_len(e) : klen[(size_t)(e - n) + 1] - klen[(size_t)(e - n)]; };
  // entries grouped by serialized key length, insertion order inside a group (counting sort)
  int64_t max_len = 0;
  for (int64_t e = 0; e < m; ++e) max_len = std::max(max_len, key_len(e));
  std::vector<int64_t> start((size_t)max_len + 2, 0);
  for (int64_t e = 0; e < m; ++e) ++start[(size_t)key_len(e) + 1];
  for (int64_t L = 0; L <= max_len; ++L) start[(size_t)L + 1] += start[(size_t)L];
  std::vector<int64_t> order((size_t)m);
  {
    std::vector<int64_t> pos(start.begin(), start.end() - 1);
    for (int64_t e = 0; e < m; ++e) order[(size_t)pos[(size_t)key_len(e)]++] = e;
  }
  std::vector<Block> meta;
  std::vector<std::string> index_parts, data_parts;
  int64_t index_off = 0, data_off = 0;
  std::vector<uint64_t> doff((size_t)m);
  for (int64_t L = 1; L <= max_len; ++L) {
    const int64_t a = start[(size_t)L], b = start[(size_t)L + 1];
    if (a == b) continue;
    const int32_t count = (int32_t)(b - a);
    const int32_t slots = (int32_t)std::floor((double)count / 0.75 + 0.5);     // Java Math.round(count / 0.75)
    // data stream: one reserved byte (offset 0 = empty slot), then varint length + value per entry
    uint64_t pos = 1;
    int maxv = 1;
    for (int64_t r = a; r < b; ++r) {
      doff[(size_t)r] = pos;
      maxv = std::max(maxv, varint_len(pos));
      uint64_t vl = (uint64_t)val_len(order[(size_t)r]);
      pos += (uint64_t)varint_len(vl) + vl;
    }
    std::string data((size_t)pos, '\0');
    const int32_t slot_size = (int32_t)L + maxv;
    std::vector<uint32_t> home((size_t)count);
    auto key_ptr = [&](int64_t e, char* tmp) -> const char* {
      if (e < n) return kbuf.data() + klen[(size_t)e];
      int_ser(e - n, tmp);
      return tmp;
    };
    run_parallel(count, 1 << 14, [&](int64_t x, int64_t y) {
      char tmp[16];
      std::string vl;
      for (int64_t r = a + x; r < a + y; ++r) {
        int64_t e = order[(size_t)r];
        const char* k = key_ptr(e, tmp);
        home[(size_t)(r - a)] =
            (uint32_t)((uint64_t)(murmur3_32((const uint8_t*)k, (size_t)L) & 0x7fffffffu) % (uint64_t)slots);
        // value bytes
        char* d = &data[(size_t)doff[(size_t)r]];
        int64_t len = val_len(e);
        vl.clear();
        pack_varint(vl, (uint64_t)len);
        memcpy(d, vl.data(), vl.size());
        d += vl.size();
        if (e < n) int_ser(e, d);
        else memcpy(d, kbuf.data() + klen[(size_t)(e - n)], (size_t)len);
      }
    });
    // slot of every entry: linear probing in insertion order (sequential; a byte map of the slots)
    std::vector<uint8_t> used((size_t)slots, 0);
    std::vector<uint32_t> slot((size_t)count);
    for (int32_t r = 0; r < count; ++r) {
      uint32_t q = home[(size_t)r];
      while (used[q]) q = (q + 1 == (uint32_t)slots) ? 0 : q + 1;
      used[q] = 1;
      slot[(size_t)r] = q;
    }
    std::string index((size_t)slots * (size_t)slot_size, '\0');
    run_parallel(count, 1 << 14, [&](int64_t x, int64_t y) {
      char tmp[16];
      std::string vo;
      for (int64_t r = a + x; r < a + y; ++r) {
        char* dst = &index[(size_t)slot[(size_t)(r - a)] * (size_t)slot_size];
        memcpy(dst, key_ptr(order[(size_t)r], tmp), (size_t)L);
        vo.clear();
        pack_varint(vo, doff[(size_t)r]);
        memcpy(dst + L, vo.data(), vo.size());
      }
    });
    meta.push_back(Block{(int32_t)L, count, slots, slot_size, (int32_t)index_off, data_off});
    index_off += (int64_t)index.size();
    data_off += (int64_t)data.size();
    index_parts.push_back(std::move(index));
    data_parts.push_back(std::move(data));
  }
  std::string head;
  auto be32 = [&](int32_t v) { for (int s = 24; s >= 0; s -= 8) head.push_back((char)((uint32_t)v >> s)); };
  auto be64 = [&](int64_t v) { for (int s = 56; s >= 0; s -= 8) head.push_back((char)((uint64_t)v >> s)); };
  head.push_back(0); head.push_back(8); head += "PALDB_V1";            // writeUTF
  be64(timestamp);
  int32_t total = 0, ml = 0;
  for (const Block& b : meta) { total += b.count; ml = std::max(ml, b.klen); }
  be32(total); be32((int32_t)meta.size()); be32(ml);
  for (const Block& b : meta) { be32(b.klen); be32(b.count); be32(b.slots); be32(b.slot_size); be32(b.idx_off); be64(b.data_off); }
  be32(0);                                                             // no custom serializers
  int32_t index_start = (int32_t)head.size() + 12;
  be32(index_start);
  be64((int64_t)index_start + index_off);
  std::string tmp = std::string(path) + ".tmp." + std::to_string((long)getpid());
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) { g_err = std::string("cannot write ") + tmp; return -1; }
  bool ok = fwrite(head.data(), 1, head.size(), f) == head.size();
  for (const auto& s : index_parts) ok = ok && fwrite(s.data(), 1, s.size(), f) == s.size();
  for (const auto& s : data_parts) ok = ok && fwrite(s.data(), 1, s.size(), f) == s.size();
  ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), path) != 0) { unlink(tmp.c_str()); g_err = std::string("cannot write ") + path; return -1; }
  return 0;
}

}  // namespace pdb

extern "C" {

const char* pml_pdb_last_error() { return pdb::g_err.c_str(); }

// Java String.hashCode partition (Spark HashPartitioner: nonNegativeMod) of n NUL-separated UTF-8 keys
int pml_pdb_partitions(const char* blob, int64_t len, int64_t n, int32_t n_parts, int32_t* out) {
  std::vector<int64_t> offs;
  if (!pdb::split_nul(blob, len, n, offs)) { pdb::g_err = "key count mismatch"; return -1; }
  std::atomic<bool> bad{false};
  pdb::run_parallel(n, 1 << 14, [&](int64_t a, int64_t b) {
    std::vector<uint16_t> u;
    for (int64_t i = a; i < b; ++i) {
      if (!pdb::utf16_units(blob + offs[(size_t)i], (size_t)(offs[(size_t)i + 1] - 1 - offs[(size_t)i]), u)) bad = true;
      int32_t m = pdb::java_hash(u) % n_parts;
      out[i] = m < 0 ? m + n_parts : m;
    }
  });
  if (bad) { pdb::g_err = "invalid UTF-8 key"; return -3; }
  return 0;
}

// One store of n keys (NUL-separated, in local-index order): key i -> i and i -> key i. 0 on success.
int pml_pdb_write_store(const char* path, const char* blob, int64_t len, int64_t n, int64_t timestamp) {
  std::vector<int64_t> offs;
  if (!pdb::split_nul(blob, len, n, offs)) { pdb::g_err = "key count mismatch"; return -1; }
  std::vector<int64_t> idx((size_t)n);
  for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = i;
  return pdb::write_store(path, blob, offs, idx, timestamp);
}

// FeatureIndexingDriver with PalDB output: n keys (NUL-separated, duplicates allowed) hash-partitioned over
// n_parts stores (paths NUL-separated), local indices in sorted (code point) order of the distinct keys per
// partition. sizes_out[p] = distinct keys of partition p. 0 on success.
int pml_pdb_build(const char* blob, int64_t len, int64_t n, int32_t n_parts, const char* paths, int64_t paths_len,
                  int64_t timestamp, int64_t* sizes_out) {
  std::vector<int64_t> offs, poffs;
  if (!pdb::split_nul(blob, len, n, offs)) { pdb::g_err = "key count mismatch"; return -1; }
  if (!pdb::split_nul(paths, paths_len, n_parts, poffs)) { pdb::g_err = "path count mismatch"; return -1; }
  std::vector<int32_t> part((size_t)n);
  int rc = pml_pdb_partitions(blob, len, n, n_parts, part.data());
  if (rc) return rc;
  std::vector<std::vector<int64_t>> members((size_t)n_parts);
  for (int64_t i = 0; i < n; ++i) members[(size_t)part[(size_t)i]].push_back(i);
  auto key = [&](int64_t i) {
    return std::string_view(blob + offs[(size_t)i], (size_t)(offs[(size_t)i + 1] - 1 - offs[(size_t)i]));
  };
  std::atomic<int> err{0};
  auto build_part = [&](int64_t p) {
    auto& m = members[(size_t)p];
    auto less = [&](int64_t a, int64_t b) { return key(a) < key(b); };                      // bytes = code points
    if (n_parts == 1) pdb::parallel_sort(m, less);
    else std::sort(m.begin(), m.end(), less);
    m.erase(std::unique(m.begin(), m.end(), [&](int64_t a, int64_t b) { return key(a) == key(b); }), m.end());
    sizes_out[p] = (int64_t)m.size();
    int r = pdb::write_store(paths + poffs[(size_t)p], blob, offs, m, timestamp);
    if (r) err = r;
  };
  if (n_parts == 1) build_part(0);
  else pdb::run_parallel(n_parts, 1, [&](int64_t a, int64_t b) { for (int64_t p = a; p < b; ++p) build_part(p); });
  return err.load();
}

// Open the n_parts stores (paths NUL-separated) of one namespace as one map; nullptr on error (pml_pdb_last_error)
void* pml_pdb_open(const char* paths, int64_t paths_len, int32_t n_parts) {
  std::vector<int64_t> poffs;
  if (!pdb::split_nul(paths, paths_len, n_parts, poffs)) { pdb::g_err = "path count mismatch"; return nullptr; }
  pdb::Map* m = new pdb::Map();
  m->offsets.push_back(0);
  for (int32_t p = 0; p < n_parts; ++p) {
    pdb::Store* s = new pdb::Store();
    m->parts.push_back(s);
    if (!s->open(paths + poffs[(size_t)p])) { delete m; return nullptr; }
    if (s->key_count % 2) { pdb::g_err = "odd key count: not a two-way index store"; delete m; return nullptr; }
    m->offsets.push_back(m->offsets.back() + s->key_count / 2);        // PalDBIndexMap: size / 2 per store
  }
  return m;
}

void pml_pdb_close(void* h) { delete (pdb::Map*)h; }

int64_t pml_pdb_size(void* h) { return ((pdb::Map*)h)->offsets.back(); }

int64_t pml_pdb_part_offset(void* h, int32_t p) { return ((pdb::Map*)h)->offsets[(size_t)p]; }

// global indices of n NUL-separated UTF-8 keys (-1 = absent)
int pml_pdb_get_indices(void* hp, const char* blob, int64_t len, int64_t n, int64_t* out) {
  pdb::Map* m = (pdb::Map*)hp;
  std::vector<int64_t> offs;
  if (!pdb::split_nul(blob, len, n, offs)) { pdb::g_err = "key count mismatch"; return -1; }
  const int32_t P = (int32_t)m->parts.size();
  std::atomic<bool> bad{false};
  pdb::run_parallel(n, 1 << 13, [&](int64_t a, int64_t b) {
    std::vector<uint16_t> u;
    std::string k;
    for (int64_t i = a; i < b; ++i) {
      out[i] = -1;
      const char* ks = blob + offs[(size_t)i];
      const size_t kl = (size_t)(offs[(size_t)i + 1] - 1 - offs[(size_t)i]);
      int32_t h;
      k.clear();
      bool ascii = true;
      for (size_t c = 0; c < kl; ++c) ascii &= (unsigned char)ks[c] < 0x80;
      if (ascii) {
        // ASCII key: one UTF-16 unit per byte, each unit its own one-byte varint
        uint32_t hh = 0;
        for (size_t c = 0; c < kl; ++c) hh = 31u * hh + (unsigned char)ks[c];
        h = (int32_t)hh;
        k.push_back((char)103);
        pdb::pack_varint(k, kl);
        k.append(ks, kl);
      } else {
        if (!pdb::utf16_units(ks, kl, u)) { bad = true; continue; }
        h = pdb::java_hash(u);
        pdb::ser_str(k, u);
      }
      int32_t p = h % P;
      if (p < 0) p += P;
      const uint8_t* ve;
      const uint8_t* v = m->parts[(size_t)p]->find(k, &ve);
      int64_t local;
      if (v && pdb::de_int(v, ve, local)) out[i] = m->offsets[(size_t)p] + local;
    }
  });
  if (bad) { pdb::g_err = "invalid UTF-8 key"; return -3; }
  return 0;
}

// Feature names of n global indices, NUL-separated, in a malloc'd buffer *out (free with pml_pdb_free; an absent
// index gives an empty name and found[i] = 0). Returns the buffer's length (without a trailing NUL).
int64_t pml_pdb_get_names(void* hp, const int64_t* idx, int64_t n, char** out, uint8_t* found) {
  pdb::Map* m = (pdb::Map*)hp;
  const int64_t dim = m->offsets.back();
  int64_t T = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  T = std::max<int64_t>(1, std::min<int64_t>(T, n / 8192));
  std::vector<std::string> part((size_t)T);
  auto work = [&](int64_t t) {
    int64_t a = n * t / T, b = n * (t + 1) / T;
    std::string k, name;
    std::string& o = part[(size_t)t];
    for (int64_t i = a; i < b; ++i) {
      int64_t g = idx[i];
      found[i] = 0;
      if (g >= 0 && g < dim) {
        size_t p = (size_t)(std::upper_bound(m->offsets.begin(), m->offsets.end(), g) - m->offsets.begin() - 1);
        k.clear();
        pdb::ser_int(k, g - m->offsets[p]);
        const uint8_t* ve;
        const uint8_t* v = m->parts[p]->find(k, &ve);
        if (v && pdb::de_str(v, ve, name)) { o += name; found[i] = 1; }
      }
      o.push_back('\0');
    }
  };
  if (T == 1) work(0);
  else {
    std::vector<std::thread> th;
    for (int64_t t = 0; t < T; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  int64_t total = 0;
  for (const auto& s : part) total += (int64_t)s.size();
  char* buf = (char*)malloc((size_t)std::max<int64_t>(total, 1));
  char* q = buf;
  for (const auto& s : part) { memcpy(q, s.data(), s.size()); q += s.size(); }
  *out = buf;
  return total > 0 ? total - 1 : 0;         // drop the last separator
}

void pml_pdb_free(char* p) { free(p); }

}  // extern "C"

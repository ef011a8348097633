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
#include <vector>

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

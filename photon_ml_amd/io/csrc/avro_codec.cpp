// photon_ml_amd native Avro Object Container File codec (C++17, pybind11).
//
// Replaces the JVM Avro 1.7.7 stack the reference uses (photon-client/.../data/avro/{AvroUtils,AvroDataReader,
// ModelProcessingUtils,ScoreProcessingUtils}.scala). Supports the full Avro binary encoding (null, boolean, int,
// long, float, double, bytes, string, record, enum, array, map, union, fixed, named-type references with
// namespaces), OCF containers with the "null", "deflate" (zlib raw) and "snappy" (own implementation + CRC32C
// trailer) codecs, generic decode to Python objects, generic encode from Python objects, and a columnar fast path
// for training data: records are decoded straight into numpy arrays (labels, weights, offsets, uids, id tags) and
// one CSR triplet per feature bag with interned "name\u0001term" keys — no per-record Python objects.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <map>
#include <memory>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

// Build id (photon_ml_amd/ops/build.py: content hash of the sources + compile command, -DPML_BUILD_ID=...): the
// loaders compare it with the tree's sources and refuse a stale library.
#ifndef PML_BUILD_ID
#define PML_BUILD_ID "unstamped-build!"
#endif
__attribute__((used)) static const char pml_build_stamp[] = "PML_BUILD_ID=" PML_BUILD_ID;

namespace py = pybind11;

// ============================================================================================================
// Minimal JSON (schemas / metadata only)
// ============================================================================================================
struct JVal {
  enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  double num = 0;
  std::string s;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;
  const JVal* get(const std::string& k) const {
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct JParser {
  const std::string& s;
  size_t i = 0;
  explicit JParser(const std::string& str) : s(str) {}
  void ws() {
    while (i < s.size() && isspace((unsigned char)s[i])) ++i;
  }
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("JSON parse error: ") + m); }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c == '\\') {
        char e = s[i++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            unsigned cp = std::stoul(s.substr(i, 4), nullptr, 16);
            i += 4;
            if (cp < 0x80) out += (char)cp;
            else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
            else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
            break;
          }
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    ++i;
    return out;
  }
  JVal val() {
    ws();
    JVal v;
    if (i >= s.size()) fail("eof");
    char c = s[i];
    if (c == '{') {
      v.t = JVal::OBJ; ++i; ws();
      if (s[i] == '}') { ++i; return v; }
      while (true) {
        ws(); std::string k = str(); ws();
        if (s[i] != ':') fail("expected :");
        ++i;
        v.obj.emplace_back(k, val()); ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == '}') { ++i; break; }
        fail("expected , or }");
      }
    } else if (c == '[') {
      v.t = JVal::ARR; ++i; ws();
      if (s[i] == ']') { ++i; return v; }
      while (true) {
        v.arr.push_back(val()); ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == ']') { ++i; break; }
        fail("expected , or ]");
      }
    } else if (c == '"') {
      v.t = JVal::STR; v.s = str();
    } else if (s.compare(i, 4, "true") == 0) { v.t = JVal::BOOL; v.b = true; i += 4; }
    else if (s.compare(i, 5, "false") == 0) { v.t = JVal::BOOL; i += 5; }
    else if (s.compare(i, 4, "null") == 0) { v.t = JVal::NUL; i += 4; }
    else {
      size_t j = i;
      while (j < s.size() && (isdigit((unsigned char)s[j]) || s[j] == '-' || s[j] == '+' || s[j] == '.' ||
                              s[j] == 'e' || s[j] == 'E')) ++j;
      v.t = JVal::NUM; v.num = std::stod(s.substr(i, j - i)); i = j;
    }
    return v;
  }
};

// ============================================================================================================
// Schema
// ============================================================================================================
enum class AT { NUL, BOOL, INT, LONG, FLOAT, DOUBLE, BYTES, STRING, RECORD, ENUM, ARRAY, MAP, UNION, FIXED };

struct Node {
  AT t = AT::NUL;
  std::string name;  // full name for named types
  std::vector<std::pair<std::string, Node*>> fields;
  Node* items = nullptr;  // array items / map values
  std::vector<Node*> branches;
  std::vector<std::string> symbols;
  int fixed_size = 0;
};

struct Schema {
  std::vector<std::unique_ptr<Node>> pool;
  std::map<std::string, Node*> named;
  Node* root = nullptr;
  std::string json;

  Node* mk() { pool.emplace_back(new Node()); return pool.back().get(); }

  static std::string full(const std::string& n, const std::string& ns) {
    if (n.find('.') != std::string::npos || ns.empty()) return n;
    return ns + "." + n;
  }

  Node* lookup(const std::string& n, const std::string& ns) {
    auto it = named.find(full(n, ns));
    if (it != named.end()) return it->second;
    it = named.find(n);
    if (it != named.end()) return it->second;
    // match by short name
    for (auto& kv : named) {
      auto p = kv.first.rfind('.');
      if ((p == std::string::npos ? kv.first : kv.first.substr(p + 1)) == n) return kv.second;
    }
    return nullptr;
  }

  Node* parse(const JVal& v, const std::string& ns) {
    if (v.t == JVal::STR) {
      const std::string& s = v.s;
      Node* n;
      if (s == "null") { n = mk(); n->t = AT::NUL; return n; }
      if (s == "boolean") { n = mk(); n->t = AT::BOOL; return n; }
      if (s == "int") { n = mk(); n->t = AT::INT; return n; }
      if (s == "long") { n = mk(); n->t = AT::LONG; return n; }
      if (s == "float") { n = mk(); n->t = AT::FLOAT; return n; }
      if (s == "double") { n = mk(); n->t = AT::DOUBLE; return n; }
      if (s == "bytes") { n = mk(); n->t = AT::BYTES; return n; }
      if (s == "string") { n = mk(); n->t = AT::STRING; return n; }
      Node* r = lookup(s, ns);
      if (!r) throw std::runtime_error("unknown Avro type reference: " + s);
      return r;
    }
    if (v.t == JVal::ARR) {
      Node* n = mk(); n->t = AT::UNION;
      for (auto& b : v.arr) n->branches.push_back(parse(b, ns));
      return n;
    }
    if (v.t != JVal::OBJ) throw std::runtime_error("bad schema node");
    const JVal* tp = v.get("type");
    if (!tp) throw std::runtime_error("schema object without type");
    if (tp->t != JVal::STR) return parse(*tp, ns);
    const std::string& t = tp->s;
    if (t == "record" || t == "error" || t == "enum" || t == "fixed") {
      const JVal* nm = v.get("name");
      const JVal* nsv = v.get("namespace");
      std::string nns = nsv && nsv->t == JVal::STR ? nsv->s : ns;
      std::string fname = full(nm ? nm->s : "anon", nns);
      auto dot = fname.rfind('.');
      std::string child_ns = dot == std::string::npos ? "" : fname.substr(0, dot);
      Node* n = mk();
      n->name = fname;
      named[fname] = n;
      if (t == "enum") {
        n->t = AT::ENUM;
        for (auto& sym : v.get("symbols")->arr) n->symbols.push_back(sym.s);
      } else if (t == "fixed") {
        n->t = AT::FIXED; n->fixed_size = (int)v.get("size")->num;
      } else {
        n->t = AT::RECORD;
        for (auto& f : v.get("fields")->arr) n->fields.emplace_back(f.get("name")->s, parse(*f.get("type"), child_ns));
      }
      return n;
    }
    if (t == "array") { Node* n = mk(); n->t = AT::ARRAY; n->items = parse(*v.get("items"), ns); return n; }
    if (t == "map") { Node* n = mk(); n->t = AT::MAP; n->items = parse(*v.get("values"), ns); return n; }
    JVal s; s.t = JVal::STR; s.s = t;
    return parse(s, ns);
  }

  explicit Schema(const std::string& j) : json(j) {
    JParser p(j);
    JVal v = p.val();
    root = parse(v, "");
  }
};

// ============================================================================================================
// Binary reader / writer
// ============================================================================================================
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const uint8_t* b, size_t n) : p(b), end(b + n) {}
  [[noreturn]] void fail() { throw std::runtime_error("Avro decode: unexpected end of data"); }
  int64_t varlong() {
    uint64_t v = 0; int shift = 0;
    while (true) {
      if (p >= end) fail();
      uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
      if (shift > 63) throw std::runtime_error("varint too long");
    }
    return (int64_t)((v >> 1) ^ (~(v & 1) + 1));
  }
  double dbl() { if (end - p < 8) fail(); double d; memcpy(&d, p, 8); p += 8; return d; }
  float flt() { if (end - p < 4) fail(); float f; memcpy(&f, p, 4); p += 4; return f; }
  std::string str() {
    int64_t n = varlong();
    if (n < 0 || end - p < n) fail();
    std::string s((const char*)p, (size_t)n); p += n; return s;
  }
  void skip(int64_t n) { if (n < 0 || end - p < n) fail(); p += n; }
};

struct Writer {
  std::string buf;
  void varlong(int64_t v) {
    uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
    while (z & ~0x7FULL) { buf.push_back((char)((z & 0x7F) | 0x80)); z >>= 7; }
    buf.push_back((char)z);
  }
  void dbl(double d) { char b[8]; memcpy(b, &d, 8); buf.append(b, 8); }
  void flt(float f) { char b[4]; memcpy(b, &f, 4); buf.append(b, 4); }
  void str(const std::string& s) { varlong((int64_t)s.size()); buf.append(s); }
};

// generic skip
static void skip_value(Reader& r, const Node* n) {
  switch (n->t) {
    case AT::NUL: return;
    case AT::BOOL: r.skip(1); return;
    case AT::INT: case AT::LONG: case AT::ENUM: r.varlong(); return;
    case AT::FLOAT: r.skip(4); return;
    case AT::DOUBLE: r.skip(8); return;
    case AT::BYTES: case AT::STRING: r.skip(r.varlong()); return;
    case AT::FIXED: r.skip(n->fixed_size); return;
    case AT::RECORD: for (auto& f : n->fields) skip_value(r, f.second); return;
    case AT::UNION: { int64_t k = r.varlong(); skip_value(r, n->branches.at((size_t)k)); return; }
    case AT::ARRAY: case AT::MAP: {
      while (true) {
        int64_t c = r.varlong();
        if (c == 0) break;
        if (c < 0) { int64_t sz = r.varlong(); r.skip(sz); continue; }
        for (int64_t i = 0; i < c; ++i) {
          if (n->t == AT::MAP) r.skip(r.varlong());
          skip_value(r, n->items);
        }
      }
      return;
    }
  }
}

static py::object decode_generic(Reader& r, const Node* n) {
  switch (n->t) {
    case AT::NUL: return py::none();
    case AT::BOOL: { if (r.p >= r.end) r.fail(); bool b = *r.p++ != 0; return py::bool_(b); }
    case AT::INT: case AT::LONG: return py::int_(r.varlong());
    case AT::FLOAT: return py::float_(r.flt());
    case AT::DOUBLE: return py::float_(r.dbl());
    case AT::STRING: return py::str(r.str());
    case AT::BYTES: { std::string s = r.str(); return py::bytes(s); }
    case AT::FIXED: { std::string s((const char*)r.p, (size_t)n->fixed_size); r.skip(n->fixed_size); return py::bytes(s); }
    case AT::ENUM: return py::str(n->symbols.at((size_t)r.varlong()));
    case AT::UNION: { int64_t k = r.varlong(); return decode_generic(r, n->branches.at((size_t)k)); }
    case AT::RECORD: {
      py::dict d;
      for (auto& f : n->fields) d[py::str(f.first)] = decode_generic(r, f.second);
      return d;
    }
    case AT::ARRAY: {
      py::list l;
      while (true) {
        int64_t c = r.varlong();
        if (c == 0) break;
        if (c < 0) { c = -c; r.varlong(); }
        for (int64_t i = 0; i < c; ++i) l.append(decode_generic(r, n->items));
      }
      return l;
    }
    case AT::MAP: {
      py::dict d;
      while (true) {
        int64_t c = r.varlong();
        if (c == 0) break;
        if (c < 0) { c = -c; r.varlong(); }
        for (int64_t i = 0; i < c; ++i) { std::string k = r.str(); d[py::str(k)] = decode_generic(r, n->items); }
      }
      return d;
    }
  }
  return py::none();
}

// union branch choice for a Python value
static int pick_branch(const Node* n, const py::handle& v) {
  auto& br = n->branches;
  for (size_t i = 0; i < br.size(); ++i) {
    AT t = br[i]->t;
    if (v.is_none()) { if (t == AT::NUL) return (int)i; continue; }
    if (py::isinstance<py::bool_>(v)) { if (t == AT::BOOL) return (int)i; continue; }
    if (py::isinstance<py::int_>(v)) { if (t == AT::LONG || t == AT::INT) return (int)i; continue; }
    if (py::isinstance<py::float_>(v)) { if (t == AT::DOUBLE || t == AT::FLOAT) return (int)i; continue; }
    if (py::isinstance<py::str>(v)) { if (t == AT::STRING || t == AT::ENUM) return (int)i; continue; }
    if (py::isinstance<py::bytes>(v)) { if (t == AT::BYTES || t == AT::FIXED) return (int)i; continue; }
    if (py::isinstance<py::dict>(v)) { if (t == AT::RECORD || t == AT::MAP) return (int)i; continue; }
    if (py::isinstance<py::list>(v) || py::isinstance<py::tuple>(v)) { if (t == AT::ARRAY) return (int)i; continue; }
  }
  // numeric promotion: int value into a double branch
  if (py::isinstance<py::int_>(v))
    for (size_t i = 0; i < br.size(); ++i)
      if (br[i]->t == AT::DOUBLE || br[i]->t == AT::FLOAT) return (int)i;
  throw std::runtime_error("no union branch matches value");
}

static void encode_generic(Writer& w, const Node* n, const py::handle& v) {
  switch (n->t) {
    case AT::NUL: return;
    case AT::BOOL: w.buf.push_back(v.cast<bool>() ? 1 : 0); return;
    case AT::INT: case AT::LONG: w.varlong(v.cast<int64_t>()); return;
    case AT::FLOAT: w.flt(v.cast<float>()); return;
    case AT::DOUBLE: w.dbl(v.cast<double>()); return;
    case AT::STRING: w.str(py::str(v).cast<std::string>()); return;
    case AT::BYTES: w.str(v.cast<std::string>()); return;
    case AT::FIXED: w.buf.append(v.cast<std::string>()); return;
    case AT::ENUM: {
      std::string s = v.cast<std::string>();
      for (size_t i = 0; i < n->symbols.size(); ++i)
        if (n->symbols[i] == s) { w.varlong((int64_t)i); return; }
      throw std::runtime_error("bad enum symbol " + s);
    }
    case AT::UNION: { int k = pick_branch(n, v); w.varlong(k); encode_generic(w, n->branches[(size_t)k], v); return; }
    case AT::RECORD: {
      py::dict d = py::reinterpret_borrow<py::dict>(v);
      for (auto& f : n->fields) {
        py::str key(f.first);
        if (d.contains(key)) encode_generic(w, f.second, d[key]);
        else encode_generic(w, f.second, py::none());
      }
      return;
    }
    case AT::ARRAY: {
      py::sequence seq = py::reinterpret_borrow<py::sequence>(v);
      if (py::len(seq) > 0) {
        w.varlong((int64_t)py::len(seq));
        for (auto item : seq) encode_generic(w, n->items, item);
      }
      w.varlong(0);
      return;
    }
    case AT::MAP: {
      py::dict d = py::reinterpret_borrow<py::dict>(v);
      if (py::len(d) > 0) {
        w.varlong((int64_t)py::len(d));
        for (auto kv : d) { w.str(py::str(kv.first).cast<std::string>()); encode_generic(w, n->items, kv.second); }
      }
      w.varlong(0);
      return;
    }
  }
}

// ============================================================================================================
// Codecs
// ============================================================================================================
static uint32_t crc32c_table[256];
static void init_crc32c() {
  static bool done = false;
  if (done) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
    crc32c_table[i] = c;
  }
  done = true;
}
// Avro's snappy codec appends the big-endian CRC32 (ISO-HDLC, the zlib crc32) of the uncompressed data
static uint32_t crc32_iso(const std::string& s) {
  return (uint32_t)crc32(0L, (const Bytef*)s.data(), (uInt)s.size());
}

static std::string snappy_decompress(const uint8_t* p, size_t n) {
  const uint8_t* end = p + n;
  uint64_t len = 0; int shift = 0;
  while (true) {
    if (p >= end) throw std::runtime_error("snappy: truncated header");
    uint8_t b = *p++;
    len |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) break;
    shift += 7;
  }
  std::string out;
  out.reserve(len);
  while (p < end) {
    uint8_t tag = *p++;
    int type = tag & 3;
    if (type == 0) {
      uint32_t l = tag >> 2;
      if (l >= 60) {
        int nb = (int)l - 59; l = 0;
        for (int i = 0; i < nb; ++i) l |= (uint32_t)p[i] << (8 * i);
        p += nb;
      }
      l += 1;
      if ((size_t)(end - p) < l) throw std::runtime_error("snappy: bad literal");
      out.append((const char*)p, l); p += l;
    } else {
      uint32_t l, off;
      if (type == 1) { l = ((tag >> 2) & 7) + 4; off = ((uint32_t)(tag >> 5) << 8) | *p++; }
      else if (type == 2) { l = (tag >> 2) + 1; off = p[0] | (p[1] << 8); p += 2; }
      else { l = (tag >> 2) + 1; off = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); p += 4; }
      if (off == 0 || off > out.size()) throw std::runtime_error("snappy: bad copy offset");
      size_t start = out.size() - off;
      for (uint32_t i = 0; i < l; ++i) out.push_back(out[start + i]);
    }
  }
  if (out.size() != len) throw std::runtime_error("snappy: length mismatch");
  return out;
}

// Snappy compressor (the format's greedy LZ77 scheme): the input is cut into 64 KiB fragments; in each, a
// 4-byte hash table of earlier positions proposes match candidates, a verified match of >= 4 bytes is emitted as
// copy elements (1-byte offset form for 4..11 bytes within 2 KiB, else 2-byte offsets, at most 64 bytes each),
// everything else as literal runs. Unmatched stretches are skipped over progressively faster (one extra byte
// per 32 misses), as in the reference implementation, so incompressible data costs little.
static void snappy_emit_literal(std::string& out, const char* p, size_t l) {
  while (l > 0) {
    const size_t c = std::min<size_t>(l, 65536);
    const uint32_t lm1 = (uint32_t)(c - 1);
    if (lm1 < 60) out.push_back((char)(lm1 << 2));
    else if (lm1 < 256) { out.push_back((char)(60 << 2)); out.push_back((char)lm1); }
    else { out.push_back((char)(61 << 2)); out.push_back((char)(lm1 & 0xFF)); out.push_back((char)(lm1 >> 8)); }
    out.append(p, c);
    p += c;
    l -= c;
  }
}

static void snappy_emit_copy(std::string& out, size_t off, size_t len) {
  while (len > 0) {
    // leave at least 4 bytes for the last element (copies are 4+ bytes in the 1-byte-offset form)
    size_t c = std::min<size_t>(len, 64);
    if (len > 64 && len - 64 < 4) c = len - 4;
    if (c >= 4 && c <= 11 && off < 2048) {
      out.push_back((char)(((c - 4) << 2) | 1 | ((off >> 8) << 5)));
      out.push_back((char)(off & 0xFF));
    } else {
      out.push_back((char)(((c - 1) << 2) | 2));
      out.push_back((char)(off & 0xFF));
      out.push_back((char)((off >> 8) & 0xFF));
    }
    len -= c;
  }
}

static inline uint32_t snappy_load32(const char* p) { uint32_t v; memcpy(&v, p, 4); return v; }

static std::string snappy_compress(const std::string& in) {
  std::string out;
  out.reserve(in.size() / 2 + 16);
  uint64_t n = in.size();
  while (true) { uint8_t b = n & 0x7F; n >>= 7; if (n) { out.push_back((char)(b | 0x80)); } else { out.push_back((char)b); break; } }
  const char* base = in.data();
  const int HBITS = 14;
  std::vector<int32_t> table(1u << HBITS);
  for (size_t frag = 0; frag < in.size(); frag += 65536) {
    const size_t flen = std::min<size_t>(in.size() - frag, 65536);
    const char* fp = base + frag;
    std::fill(table.begin(), table.end(), -1);
    size_t lit = 0, i = 0;
    uint32_t skip = 32;
    while (i + 4 <= flen) {
      const uint32_t cur = snappy_load32(fp + i);
      const uint32_t h = (cur * 0x1E35A7BDu) >> (32 - HBITS);
      const int32_t cand = table[h];
      table[h] = (int32_t)i;
      if (cand >= 0 && snappy_load32(fp + cand) == cur) {
        size_t len = 4;
        while (i + len < flen && fp[cand + len] == fp[i + len]) ++len;
        snappy_emit_literal(out, fp + lit, i - lit);
        snappy_emit_copy(out, i - (size_t)cand, len);
        i += len;
        lit = i;
        skip = 32;
        continue;
      }
      i += skip++ >> 5;
    }
    snappy_emit_literal(out, fp + lit, flen - lit);
  }
  return out;
}

static std::string inflate_raw(const uint8_t* p, size_t n) {
  z_stream zs; memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -15) != Z_OK) throw std::runtime_error("inflateInit2 failed");
  zs.next_in = (Bytef*)p; zs.avail_in = (uInt)n;
  std::string out;
  char buf[1 << 16];
  int ret;
  do {
    zs.next_out = (Bytef*)buf; zs.avail_out = sizeof(buf);
    ret = inflate(&zs, Z_NO_FLUSH);
    if (ret != Z_OK && ret != Z_STREAM_END) { inflateEnd(&zs); throw std::runtime_error("inflate failed"); }
    out.append(buf, sizeof(buf) - zs.avail_out);
  } while (ret != Z_STREAM_END);
  inflateEnd(&zs);
  return out;
}

static std::string deflate_raw(const std::string& in, int level) {
  z_stream zs; memset(&zs, 0, sizeof(zs));
  if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) throw std::runtime_error("deflateInit2");
  zs.next_in = (Bytef*)in.data(); zs.avail_in = (uInt)in.size();
  std::string out;
  char buf[1 << 16];
  int ret;
  do {
    zs.next_out = (Bytef*)buf; zs.avail_out = sizeof(buf);
    ret = deflate(&zs, Z_FINISH);
    out.append(buf, sizeof(buf) - zs.avail_out);
  } while (ret != Z_STREAM_END);
  deflateEnd(&zs);
  return out;
}

// ============================================================================================================
// OCF container
// ============================================================================================================
struct OCF {
  std::string data;  // whole file
  std::string schema_json, codec;
  std::unique_ptr<Schema> schema;
  std::vector<std::pair<int64_t, std::string>> blocks;  // (count, decompressed bytes)

  explicit OCF(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("cannot open " + path);
    const std::streamsize fsz = f.tellg();
    f.seekg(0);
    data.resize((size_t)std::max<std::streamsize>(fsz, 0));
    if (fsz > 0 && !f.read(&data[0], fsz)) throw std::runtime_error("cannot read " + path);
    if (data.size() < 4 || data.compare(0, 4, std::string("Obj\x01", 4)) != 0)
      throw std::runtime_error("not an Avro object container file: " + path);
    Reader r((const uint8_t*)data.data() + 4, data.size() - 4);
    // metadata map
    while (true) {
      int64_t c = r.varlong();
      if (c == 0) break;
      if (c < 0) { c = -c; r.varlong(); }
      for (int64_t i = 0; i < c; ++i) {
        std::string k = r.str(), v = r.str();
        if (k == "avro.schema") schema_json = v;
        else if (k == "avro.codec") codec = v;
      }
    }
    if (codec.empty()) codec = "null";
    std::string sync((const char*)r.p, 16); r.skip(16);
    schema.reset(new Schema(schema_json));
    while (r.p < r.end) {
      int64_t cnt = r.varlong();
      int64_t sz = r.varlong();
      if (sz < 0 || r.end - r.p < sz) throw std::runtime_error("truncated block");
      const uint8_t* b = r.p; r.skip(sz);
      std::string blk;
      if (codec == "null") blk.assign((const char*)b, (size_t)sz);
      else if (codec == "deflate") blk = inflate_raw(b, (size_t)sz);
      else if (codec == "snappy") {
        if (sz < 4) throw std::runtime_error("snappy block too small");
        blk = snappy_decompress(b, (size_t)sz - 4);
        uint32_t want = ((uint32_t)b[sz - 4] << 24) | ((uint32_t)b[sz - 3] << 16) | ((uint32_t)b[sz - 2] << 8) | b[sz - 1];
        if (crc32_iso(blk) != want) throw std::runtime_error("snappy block CRC mismatch");
      } else throw std::runtime_error("unsupported Avro codec: " + codec);
      blocks.emplace_back(cnt, std::move(blk));
      if (r.end - r.p < 16) throw std::runtime_error("missing sync marker");
      if (memcmp(r.p, sync.data(), 16) != 0) throw std::runtime_error("sync marker mismatch");
      r.skip(16);
    }
  }
};

static py::tuple read_ocf(const std::string& path) {
  OCF o(path);
  py::list recs;
  for (auto& b : o.blocks) {
    Reader r((const uint8_t*)b.second.data(), b.second.size());
    for (int64_t i = 0; i < b.first; ++i) recs.append(decode_generic(r, o.schema->root));
  }
  return py::make_tuple(o.schema_json, recs, o.codec);
}

static std::string read_schema(const std::string& path) {
  OCF o(path);
  return o.schema_json;
}

static void write_ocf(const std::string& path, const std::string& schema_json, py::list records,
                      const std::string& codec, int block_records) {
  Schema sch(schema_json);
  std::string out("Obj\x01", 4);
  Writer hdr;
  hdr.varlong(2);
  hdr.str("avro.schema"); hdr.str(schema_json);
  hdr.str("avro.codec"); hdr.str(codec);
  hdr.varlong(0);
  out += hdr.buf;
  std::string sync(16, '\0');
  std::mt19937_64 rng(0x5eed1234abcdULL ^ (uint64_t)records.size());
  for (int i = 0; i < 16; ++i) sync[i] = (char)(rng() & 0xFF);
  out += sync;
  size_t n = py::len(records);
  size_t i = 0;
  while (i < n) {
    size_t m = std::min<size_t>(n - i, (size_t)std::max(block_records, 1));
    Writer body;
    for (size_t k = 0; k < m; ++k) encode_generic(body, sch.root, records[i + k]);
    std::string payload;
    if (codec == "null") payload = body.buf;
    else if (codec == "deflate") payload = deflate_raw(body.buf, 6);
    else if (codec == "snappy") {
      payload = snappy_compress(body.buf);
      uint32_t c = crc32_iso(body.buf);
      payload.push_back((char)(c >> 24)); payload.push_back((char)(c >> 16));
      payload.push_back((char)(c >> 8)); payload.push_back((char)c);
    } else throw std::runtime_error("unsupported codec " + codec);
    Writer bh; bh.varlong((int64_t)m); bh.varlong((int64_t)payload.size());
    out += bh.buf; out += payload; out += sync;
    i += m;
  }
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path);
  f.write(out.data(), (std::streamsize)out.size());
}

// ============================================================================================================
// Columnar training-data fast path
// ============================================================================================================
static bool is_numeric(AT t) { return t == AT::INT || t == AT::LONG || t == AT::FLOAT || t == AT::DOUBLE || t == AT::BOOL; }

static double read_number(Reader& r, const Node* n, bool& ok) {
  switch (n->t) {
    case AT::INT: case AT::LONG: ok = true; return (double)r.varlong();
    case AT::FLOAT: ok = true; return r.flt();
    case AT::DOUBLE: ok = true; return r.dbl();
    case AT::BOOL: { ok = true; bool b = *r.p++ != 0; return b ? 1.0 : 0.0; }
    case AT::STRING: { std::string s = r.str(); try { ok = true; return std::stod(s); } catch (...) { ok = false; return NAN; } }
    case AT::NUL: ok = false; return NAN;
    case AT::UNION: { int64_t k = r.varlong(); return read_number(r, n->branches.at((size_t)k), ok); }
    default: skip_value(r, n); ok = false; return NAN;
  }
}

static bool read_string_like(Reader& r, const Node* n, std::string& out) {
  switch (n->t) {
    case AT::STRING: case AT::BYTES: {
      const int64_t len = r.varlong();
      if (len < 0 || r.end - r.p < len) r.fail();
      out.assign((const char*)r.p, (size_t)len);
      r.p += len;
      return true;
    }
    case AT::INT: case AT::LONG: out = std::to_string(r.varlong()); return true;
    case AT::DOUBLE: { std::ostringstream o; o << r.dbl(); out = o.str(); return true; }
    case AT::FLOAT: { std::ostringstream o; o << r.flt(); out = o.str(); return true; }
    case AT::BOOL: { bool b = *r.p++ != 0; out = b ? "true" : "false"; return true; }
    case AT::ENUM: out = n->symbols.at((size_t)r.varlong()); return true;
    case AT::NUL: return false;
    case AT::UNION: { int64_t k = r.varlong(); return read_string_like(r, n->branches.at((size_t)k), out); }
    default: skip_value(r, n); return false;
  }
}

static const Node* strip_null_union(const Node* n) {
  if (n->t != AT::UNION) return n;
  const Node* keep = nullptr;
  for (auto* b : n->branches)
    if (b->t != AT::NUL) { if (keep) return n; keep = b; }
  return keep ? keep : n;
}

// Is this node a feature bag (array of records with name + value fields)?
static bool is_bag(const Node* n) {
  n = strip_null_union(n);
  if (n->t != AT::ARRAY) return false;
  const Node* it = strip_null_union(n->items);
  if (it->t != AT::RECORD) return false;
  bool has_name = false, has_value = false;
  for (auto& f : it->fields) { if (f.first == "name") has_name = true; if (f.first == "value") has_value = true; }
  return has_name && has_value;
}

// Feature-key interner: ids in first-appearance order; an open-addressing table of 16-byte slots {id + 1, key
// length, 16 hash bits, the key's first 8 bytes}. A probe is one cache line, and keys of <= 8 bytes (and most
// misses) are decided inside the slot without touching the key arena -- at millions of distinct keys per file
// the arena access was the second cache miss of every lookup.
struct Interner {
  struct Slot { uint32_t id; uint16_t len; uint16_t h; uint64_t pfx; };
  std::vector<std::string> keys;
  std::vector<Slot> slots;
  size_t mask = 0;
  static uint64_t hash(const char* p, size_t n) {
    // 8 bytes per multiply (the byte-wise FNV-1a loop was ~40 cycles of a ~300-cycle lookup), then a final mix
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      memcpy(&w, p + i, 8);
      h = (h ^ w) * 0xFF51AFD7ED558CCDull;
      h ^= h >> 32;
    }
    if (i < n) {
      uint64_t w = 0;
      memcpy(&w, p + i, n - i);
      h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
    }
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
    return h;
  }
  void reserve(size_t n_keys) {                       // slots for n_keys without rehashing on the way
    size_t cap = 1024;
    while (cap < 2 * (n_keys + 1)) cap *= 2;
    keys.reserve(n_keys);
    if (slots.empty()) {
      slots.assign(cap, Slot{0, 0, 0, 0});
      mask = cap - 1;
      return;
    }
    while (slots.size() < cap) grow();
  }
  static uint64_t prefix(const char* p, size_t n) {
    uint64_t v = 0;
    memcpy(&v, p, n < 8 ? n : 8);
    return v;
  }
  void grow() {
    const size_t cap = std::max<size_t>(1024, slots.size() * 2);
    std::vector<Slot> ns(cap, Slot{0, 0, 0, 0});
    const size_t m = cap - 1;
    for (const Slot& sl : slots) {
      if (!sl.id) continue;
      const std::string& k = keys[sl.id - 1];
      size_t j = hash(k.data(), k.size()) & m;
      while (ns[j].id) j = (j + 1) & m;
      ns[j] = sl;
    }
    slots.swap(ns);
    mask = m;
  }
  int32_t get(const std::string& k) {
    if ((keys.size() + 1) * 2 > slots.size()) grow();
    const uint64_t h64 = hash(k.data(), k.size());
    const uint16_t h = (uint16_t)(h64 >> 48);
    const uint16_t len = (uint16_t)std::min<size_t>(k.size(), 0xFFFF);
    const uint64_t pf = prefix(k.data(), k.size());
    size_t j = h64 & mask;
    while (slots[j].id) {
      const Slot& sl = slots[j];
      if (sl.h == h && sl.len == len && sl.pfx == pf && (k.size() <= 8 || keys[sl.id - 1] == k))
        return (int32_t)(sl.id - 1);
      j = (j + 1) & mask;
    }
    const int32_t id = (int32_t)keys.size();
    keys.push_back(k);
    slots[j] = Slot{(uint32_t)id + 1, len, h, pf};
    return id;
  }
};

struct BagOut {
  std::vector<int64_t> rowptr{0};
  std::vector<int32_t> keys;
  std::vector<double> vals;
};

// Decode TrainingExample-like files into columns. Files are decoded in parallel (one worker per file, up to the
// hardware threads; PML_AVRO_THREADS overrides), each into its own columns and its own feature-key interner;
// the merge walks the files in order, so feature ids (first-appearance order), rows and every column are exactly
// what a sequential decode produces. Per-record work avoids allocations: field roles and the bag item layout
// are resolved once per file schema, feature keys are assembled in one reused buffer.
struct FileCols {
  std::vector<double> label, weight, offset;
  std::vector<std::string> uid;
  std::vector<uint8_t> has_uid;
  std::vector<std::vector<int32_t>> tags;         // per requested id tag: code of each record's value
  std::vector<Interner> tag_intern;               // per requested id tag: its distinct values (missing = "")
  std::map<std::string, BagOut> bags;
  Interner intern;
  std::string label_used;
  int64_t n = 0;
  void swap_into(FileCols& other) {   // other <- this (an empty FileCols): releases other's memory
    std::swap(label, other.label); std::swap(weight, other.weight); std::swap(offset, other.offset);
    std::swap(uid, other.uid); std::swap(has_uid, other.has_uid); std::swap(tags, other.tags);
    std::swap(tag_intern, other.tag_intern);
    std::swap(bags, other.bags); std::swap(intern, other.intern); std::swap(label_used, other.label_used);
    std::swap(n, other.n);
  }
};

struct ColumnarOpts {
  std::vector<std::string> label_fields;
  std::string weight_field, offset_field, uid_field, metadata_field, delimiter;
  std::vector<std::string> bags_wanted, id_tags;
  // distinct feature keys of the largest file decoded so far in this call: later files size their interner for it
  // up front instead of doubling through ~10 rehashes (files of one dataset have similar vocabularies)
  std::atomic<size_t>* intern_hint = nullptr;
};

static void decode_columnar_file(const std::string& path, const ColumnarOpts& op, FileCols& fc) {
  OCF o(path);
  if (op.intern_hint) fc.intern.reserve(op.intern_hint->load());
  const Node* root = o.schema->root;
  if (root->t != AT::RECORD) throw std::runtime_error("top-level Avro schema must be a record: " + path);
  const size_t nf = root->fields.size();
  std::map<std::string, int> tag_index;
  for (size_t t = 0; t < op.id_tags.size(); ++t) tag_index.emplace(op.id_tags[t], (int)t);
  fc.tags.assign(op.id_tags.size(), {});
  fc.tag_intern.assign(op.id_tags.size(), Interner());
  // field roles: 0 skip, 1 label, 2 weight, 3 offset, 4 uid, 5 meta, 6 bag, 7 tag
  std::vector<int> role(nf, 0), tag_of(nf, -1);
  std::vector<BagOut*> bag_of(nf, nullptr);
  int label_idx = -1;
  for (auto& lf : op.label_fields) {
    for (size_t i = 0; i < nf; ++i)
      if (root->fields[i].first == lf) { label_idx = (int)i; break; }
    if (label_idx >= 0) { fc.label_used = lf; break; }
  }
  for (size_t i = 0; i < nf; ++i) {
    const std::string& fn = root->fields[i].first;
    const Node* fnode = root->fields[i].second;
    if ((int)i == label_idx) role[i] = 1;
    else if (fn == op.weight_field) role[i] = 2;
    else if (fn == op.offset_field) role[i] = 3;
    else if (fn == op.uid_field) role[i] = 4;
    else if (fn == op.metadata_field) role[i] = 5;
    else if (tag_index.count(fn)) { role[i] = 7; tag_of[i] = tag_index[fn]; }
    else if (is_bag(fnode)) {
      bool want = op.bags_wanted.empty();
      for (auto& b : op.bags_wanted) if (b == fn) want = true;
      if (want) { role[i] = 6; bag_of[i] = &fc.bags[fn]; }
    }
  }
  // bag item layout per (item record node): 0 skip, 1 name, 2 term, 3 value
  std::map<const Node*, std::vector<int>> item_roles;
  auto roles_of = [&](const Node* it) -> const std::vector<int>& {
    auto f = item_roles.find(it);
    if (f != item_roles.end()) return f->second;
    std::vector<int> v(it->fields.size(), 0);
    for (size_t j = 0; j < it->fields.size(); ++j) {
      const std::string& nm = it->fields[j].first;
      v[j] = nm == "name" ? 1 : nm == "term" ? 2 : nm == "value" ? 3 : 0;
    }
    return item_roles.emplace(it, std::move(v)).first->second;
  };
  std::vector<std::string> rec_tags(op.id_tags.size());
  std::vector<uint8_t> rec_has(op.id_tags.size());
  std::string key, name, term, u, sval;
  const Node* last_item = nullptr;
  const std::vector<int>* last_roles = nullptr;
  for (auto& blk : o.blocks) {
    Reader r((const uint8_t*)blk.second.data(), blk.second.size());
    for (int64_t rec = 0; rec < blk.first; ++rec) {
      double lab = NAN, wt = NAN, off = NAN;
      bool hu = false;
      u.clear();
      std::fill(rec_has.begin(), rec_has.end(), 0);
      for (size_t i = 0; i < nf; ++i) {
        const Node* fnode = root->fields[i].second;
        bool ok;
        switch (role[i]) {
          case 1: lab = read_number(r, fnode, ok); break;
          case 2: wt = read_number(r, fnode, ok); break;
          case 3: off = read_number(r, fnode, ok); break;
          case 4: hu = read_string_like(r, fnode, u); break;
          case 7: {
            const int t = tag_of[i];
            if (read_string_like(r, fnode, sval)) { rec_tags[t] = sval; rec_has[t] = 1; }
            break;
          }
          case 5: {
            const Node* m = fnode;
            if (m->t == AT::UNION) { int64_t k = r.varlong(); m = m->branches.at((size_t)k); }
            if (m->t != AT::MAP) { skip_value(r, m); break; }
            while (true) {
              int64_t c = r.varlong();
              if (c == 0) break;
              if (c < 0) { c = -c; r.varlong(); }
              for (int64_t k = 0; k < c; ++k) {
                std::string mk = r.str();
                bool has = read_string_like(r, m->items, sval);
                auto ti = tag_index.find(mk);
                if (has && ti != tag_index.end() && !rec_has[ti->second]) {
                  rec_tags[ti->second] = sval;
                  rec_has[ti->second] = 1;
                }
              }
            }
            break;
          }
          case 6: {
            BagOut& bo = *bag_of[i];
            const Node* arr = fnode;
            if (arr->t == AT::UNION) { int64_t k = r.varlong(); arr = arr->branches.at((size_t)k); }
            if (arr->t != AT::ARRAY) { skip_value(r, arr); break; }
            const Node* item = arr->items;
            while (true) {
              int64_t c = r.varlong();
              if (c == 0) break;
              if (c < 0) { c = -c; r.varlong(); }
              for (int64_t k = 0; k < c; ++k) {
                const Node* it = item;
                if (it->t == AT::UNION) { int64_t b = r.varlong(); it = it->branches.at((size_t)b); }
                if (it != last_item) { last_roles = &roles_of(it); last_item = it; }
                const std::vector<int>& fr = *last_roles;
                name.clear();
                term.clear();
                double val = NAN;
                for (size_t j = 0; j < it->fields.size(); ++j) {
                  const Node* fnd = it->fields[j].second;
                  switch (fr[j]) {
                    case 1: read_string_like(r, fnd, name); break;
                    case 2: if (!read_string_like(r, fnd, term)) term.clear(); break;
                    case 3: { bool okv; val = read_number(r, fnd, okv); break; }
                    default: skip_value(r, fnd);
                  }
                }
                key.assign(name);
                key.append(op.delimiter);
                key.append(term);
                bo.keys.push_back(fc.intern.get(key));
                bo.vals.push_back(val);
              }
            }
            break;
          }
          default: skip_value(r, fnode);
        }
      }
      fc.label.push_back(lab); fc.weight.push_back(wt); fc.offset.push_back(off);
      fc.uid.push_back(hu ? u : std::string()); fc.has_uid.push_back(hu ? 1 : 0);
      for (size_t t = 0; t < rec_tags.size(); ++t)
        fc.tags[t].push_back(fc.tag_intern[t].get(rec_has[t] ? rec_tags[t] : std::string()));
      for (auto& b : fc.bags) b.second.rowptr.push_back((int64_t)b.second.keys.size());
      ++fc.n;
    }
  }
  if (op.intern_hint) {
    size_t cur = op.intern_hint->load();
    while (fc.intern.keys.size() > cur && !op.intern_hint->compare_exchange_weak(cur, fc.intern.keys.size())) {}
  }
}

static py::dict read_columnar(const std::vector<std::string>& paths, const std::vector<std::string>& label_fields,
                              const std::string& weight_field, const std::string& offset_field,
                              const std::string& uid_field, const std::string& metadata_field,
                              const std::vector<std::string>& bags_wanted, const std::vector<std::string>& id_tags,
                              const std::string& delimiter, bool tag_strings) {
  std::atomic<size_t> intern_hint{0};
  ColumnarOpts op{label_fields, weight_field, offset_field, uid_field, metadata_field, delimiter, bags_wanted,
                  id_tags, &intern_hint};
  const size_t nfile = paths.size();
  // Files are decoded by a worker pool. This thread walks them IN FILE ORDER as each is done and takes the only
  // order-dependent decisions -- global ids of the feature keys and id-tag values (first appearance), every file's
  // row and entry offsets; the columns themselves are then copied by all threads, each file straight into its slice
  // of the output arrays (the serial append of round 5 was most of a 10M-record read on 16 threads). A file's
  // decoded columns are freed once copied.
  std::vector<FileCols> files(nfile);
  std::vector<std::string> errors(nfile);
  std::vector<uint8_t> done(nfile, 0);
  Interner intern;
  int64_t n = 0;
  std::string label_used;
  std::vector<Interner> tag_intern(id_tags.size());
  std::map<std::string, int64_t> bag_total;                  // bag -> entries so far (std::map: sorted output)
  struct FilePlan {
    int64_t row0 = 0;
    std::vector<int32_t> remap;                               // file key id -> global key id
    std::vector<std::vector<int32_t>> tag_remap;              // per tag: file code -> global code
    std::map<std::string, int64_t> nnz0;                      // bag -> first entry of this file's slice
  };
  std::vector<FilePlan> plan(nfile);
  auto plan_one = [&](size_t f) {
    FileCols& fc = files[f];
    FilePlan& pl = plan[f];
    if (label_used.empty()) label_used = fc.label_used;
    pl.row0 = n;
    pl.remap.resize(fc.intern.keys.size());
    for (size_t k = 0; k < pl.remap.size(); ++k) pl.remap[k] = intern.get(fc.intern.keys[k]);
    fc.intern = Interner();                                  // the file's key strings are no longer needed
    pl.tag_remap.resize(id_tags.size());
    for (size_t t = 0; t < id_tags.size(); ++t) {
      auto& tr = pl.tag_remap[t];
      tr.resize(fc.tag_intern[t].keys.size());
      for (size_t k = 0; k < tr.size(); ++k) tr[k] = tag_intern[t].get(fc.tag_intern[t].keys[k]);
    }
    for (auto& b : fc.bags) bag_total.emplace(b.first, 0);
    for (auto& b : bag_total) {
      pl.nnz0[b.first] = b.second;
      auto src = fc.bags.find(b.first);
      if (src != fc.bags.end()) b.second += (int64_t)src->second.keys.size();
    }
    n += fc.n;
  };
  unsigned nt = std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = std::getenv("PML_AVRO_THREADS")) nt = (unsigned)std::max(1, atoi(e));
  {
    py::gil_scoped_release nogil;
    const unsigned nd = (unsigned)std::min<size_t>(nt, std::max<size_t>(nfile, 1));
    const size_t ahead = 2 * (size_t)nd;      // files decoded beyond the planning position, at most
    std::mutex mu;
    std::condition_variable cv;
    size_t next = 0, planned = 0;
    auto work = [&]() {
      while (true) {
        size_t f;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return next >= nfile || next < planned + ahead; });
          if (next >= nfile) return;
          f = next++;
        }
        try { decode_columnar_file(paths[f], op, files[f]); }
        catch (const std::exception& ex) { errors[f] = ex.what(); }
        {
          std::lock_guard<std::mutex> lk(mu);
          done[f] = 1;
        }
        cv.notify_all();
      }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nd; ++t) pool.emplace_back(work);
    bool failed = false;
    for (size_t f = 0; f < nfile; ++f) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done[f] != 0; });
      }
      if (!errors[f].empty()) failed = true;
      if (!failed) plan_one(f);
      else FileCols().swap_into(files[f]);
      {
        std::lock_guard<std::mutex> lk(mu);
        planned = f + 1;
      }
      cv.notify_all();
    }
    for (auto& t : pool) t.join();
  }
  for (size_t f = 0; f < nfile; ++f)
    if (!errors[f].empty()) throw std::runtime_error(errors[f]);
  // output arrays (allocated with the GIL), filled by file in parallel without it
  py::array_t<double> a_label(n), a_weight(n), a_offset(n);
  py::array_t<uint8_t> a_has_uid(n);
  std::vector<py::array_t<int32_t>> a_tags;
  for (size_t t = 0; t < id_tags.size(); ++t) a_tags.emplace_back(n);
  struct BagArrays { py::array_t<int64_t> rowptr; py::array_t<int32_t> keys; py::array_t<double> vals; };
  std::map<std::string, BagArrays> a_bags;
  for (auto& b : bag_total)
    a_bags.emplace(b.first, BagArrays{py::array_t<int64_t>(n + 1), py::array_t<int32_t>(b.second),
                                      py::array_t<double>(b.second)});
  bool any_uid = false;
  for (auto& fc : files)
    for (uint8_t h : fc.has_uid) if (h) { any_uid = true; break; }
  py::list uid_list(any_uid ? n : 0);
  if (any_uid) {                                              // Python strings: with the GIL, in order
    py::ssize_t i = 0;
    for (auto& fc : files)
      for (auto& u : fc.uid) uid_list[i++] = py::str(u);
  }
  {
    double* pl_ = a_label.mutable_data();
    double* pw = a_weight.mutable_data();
    double* po = a_offset.mutable_data();
    uint8_t* ph = a_has_uid.mutable_data();
    std::vector<int32_t*> ptag;
    for (auto& a : a_tags) ptag.push_back(a.mutable_data());
    struct BagPtrs { int64_t* rp; int32_t* k; double* v; };
    std::map<std::string, BagPtrs> pb;
    for (auto& b : a_bags) pb[b.first] = BagPtrs{b.second.rowptr.mutable_data(), b.second.keys.mutable_data(),
                                                 b.second.vals.mutable_data()};
    for (auto& b : pb) b.second.rp[0] = 0;
    py::gil_scoped_release nogil;
    std::atomic<size_t> nextf{0};
    auto fill = [&]() {
      for (size_t f; (f = nextf.fetch_add(1)) < nfile;) {
        FileCols& fc = files[f];
        const FilePlan& pl = plan[f];
        const int64_t r0 = pl.row0, m = fc.n;
        if (m) {
          memcpy(pl_ + r0, fc.label.data(), sizeof(double) * m);
          memcpy(pw + r0, fc.weight.data(), sizeof(double) * m);
          memcpy(po + r0, fc.offset.data(), sizeof(double) * m);
          memcpy(ph + r0, fc.has_uid.data(), m);
        }
        for (size_t t = 0; t < ptag.size(); ++t)
          for (int64_t i = 0; i < m; ++i) ptag[t][r0 + i] = pl.tag_remap[t][(size_t)fc.tags[t][(size_t)i]];
        for (auto& b : pb) {
          const int64_t base = pl.nnz0.at(b.first);
          auto src = fc.bags.find(b.first);
          if (src == fc.bags.end()) {
            for (int64_t r = 1; r <= m; ++r) b.second.rp[r0 + r] = base;
            continue;
          }
          const BagOut& bo = src->second;
          const size_t nk = bo.keys.size();
          for (size_t q = 0; q < nk; ++q) b.second.k[base + (int64_t)q] = pl.remap[(size_t)bo.keys[q]];
          if (nk) memcpy(b.second.v + base, bo.vals.data(), sizeof(double) * nk);
          for (int64_t r = 1; r <= m; ++r) b.second.rp[r0 + r] = base + bo.rowptr[(size_t)r];
        }
        FileCols().swap_into(fc);
      }
    };
    std::vector<std::thread> pool;
    const unsigned nf = (unsigned)std::max<size_t>(1, std::min<size_t>(nt, nfile));
    for (unsigned t = 1; t < nf; ++t) pool.emplace_back(fill);
    fill();
    for (auto& t : pool) t.join();
  }
  py::dict out;
  out["n"] = n;
  out["label_field"] = label_used;
  out["label"] = a_label;
  out["weight"] = a_weight;
  out["offset"] = a_offset;
  out["uid"] = uid_list;
  out["has_uid"] = a_has_uid;
  py::dict tg, tc;
  for (size_t t = 0; t < id_tags.size(); ++t) {
    // codes into the tag's table of distinct values (first-appearance order); per-record strings on request only
    tc[py::str(id_tags[t])] = py::make_tuple(a_tags[t], py::cast(tag_intern[t].keys));
    if (tag_strings) {
      const int32_t* codes = a_tags[t].data();
      py::list l((py::ssize_t)n);
      std::vector<py::str> tab;
      tab.reserve(tag_intern[t].keys.size());
      for (auto& k : tag_intern[t].keys) tab.emplace_back(k);
      for (int64_t i = 0; i < n; ++i) l[(py::ssize_t)i] = tab[(size_t)codes[i]];
      tg[py::str(id_tags[t])] = l;
    }
  }
  out["id_tags"] = tg;
  out["id_tag_codes"] = tc;
  py::dict bg;
  for (auto& b : a_bags) bg[py::str(b.first)] = py::make_tuple(b.second.rowptr, b.second.keys, b.second.vals);
  out["bags"] = bg;
  out["vocab"] = py::cast(intern.keys);
  return out;
}

// ============================================================================================================
// Shard assembly: the bags' (row pointer, interned key, value) triplets of the decoded records -> one shard CSR
// (keys mapped through the shard's index map, unmapped keys dropped, the intercept appended, every row sorted by
// column, duplicate features detected). Row ranges in parallel; the output is what _bags_to_csr produces
// (photon-client/.../data/avro/AvroDataReader.scala:317-353: merged bags, intercept, duplicate rejection).
// ============================================================================================================
static py::tuple assemble_shard(int64_t n, py::list parts, py::array_t<int64_t, py::array::c_style> vocab_to_col,
                                int64_t dim, int64_t intercept_col, bool check_duplicates, int threads) {
  struct Part { const int64_t* rp; const int32_t* k; const double* v; };
  std::vector<Part> ps;
  std::vector<py::object> keep;
  for (auto h : parts) {
    py::tuple t = py::reinterpret_borrow<py::tuple>(h);
    auto rp = t[0].cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
    auto k = t[1].cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
    auto v = t[2].cast<py::array_t<double, py::array::c_style | py::array::forcecast>>();
    if (rp.size() != n + 1) throw std::runtime_error("assemble_shard: row pointer length != n + 1");
    if (k.size() != v.size() || (int64_t)k.size() != rp.data()[n]) throw std::runtime_error("assemble_shard: sizes");
    ps.push_back({rp.data(), k.data(), v.data()});
    keep.push_back(rp); keep.push_back(k); keep.push_back(v);
  }
  const int64_t* vc = vocab_to_col.data();
  const int64_t nv = (int64_t)vocab_to_col.size();
  unsigned nt = threads > 0 ? (unsigned)threads : std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = std::getenv("PML_AVRO_THREADS")) nt = (unsigned)std::max(1, atoi(e));
  nt = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nt, n / 4096 + 1));
  std::vector<int64_t> indptr((size_t)n + 1, 0);
  std::vector<int64_t> dup_row(nt, -1), dup_col(nt, -1);
  auto col_of = [&](int32_t key) -> int64_t { return key >= 0 && key < nv ? vc[key] : -1; };
  {
    py::gil_scoped_release nogil;
    auto range = [&](unsigned t, int64_t& a, int64_t& b) { a = n * t / nt; b = n * (t + 1) / nt; };
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t)
      pool.emplace_back([&, t] {
        int64_t a, b; range(t, a, b);
        for (int64_t r = a; r < b; ++r) {
          int64_t c = intercept_col >= 0 ? 1 : 0;
          for (auto& p : ps)
            for (int64_t q = p.rp[r]; q < p.rp[r + 1]; ++q) c += col_of(p.k[q]) >= 0;
          indptr[(size_t)r + 1] = c;
        }
      });
    for (auto& th : pool) th.join();
  }
  for (int64_t r = 0; r < n; ++r) indptr[(size_t)r + 1] += indptr[(size_t)r];
  const int64_t nnz = indptr[(size_t)n];
  const bool wide = std::max(dim, nnz) >= ((int64_t)1 << 31);
  py::array_t<double> data(nnz);
  py::array idx = wide ? (py::array)py::array_t<int64_t>(nnz) : (py::array)py::array_t<int32_t>(nnz);
  double* dp = data.mutable_data();
  int32_t* i32 = wide ? nullptr : (int32_t*)idx.mutable_data();
  int64_t* i64 = wide ? (int64_t*)idx.mutable_data() : nullptr;
  std::vector<int64_t> out_ptr;
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t)
      pool.emplace_back([&, t] {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        std::vector<std::pair<int64_t, double>> row;
        for (int64_t r = a; r < b; ++r) {
          row.clear();
          for (auto& p : ps)
            for (int64_t q = p.rp[r]; q < p.rp[r + 1]; ++q) {
              const int64_t c = col_of(p.k[q]);
              if (c >= 0) row.emplace_back(c, p.v[q]);
            }
          if (intercept_col >= 0) row.emplace_back(intercept_col, 1.0);
          std::stable_sort(row.begin(), row.end(),
                           [](const std::pair<int64_t, double>& x, const std::pair<int64_t, double>& y) {
                             return x.first < y.first;
                           });
          int64_t o = indptr[(size_t)r];
          for (size_t j = 0; j < row.size(); ++j) {
            if (j > 0 && row[j].first == row[j - 1].first && dup_row[t] < 0) {
              dup_row[t] = r;
              dup_col[t] = row[j].first;
            }
            dp[o] = row[j].second;
            if (i32) i32[o] = (int32_t)row[j].first; else i64[o] = row[j].first;
            ++o;
          }
        }
      });
    for (auto& th : pool) th.join();
  }
  int64_t first_dup = -1, first_col = -1;
  for (unsigned t = 0; t < nt; ++t)
    if (dup_row[t] >= 0) { first_dup = dup_row[t]; first_col = dup_col[t]; break; }
  py::array_t<int64_t> ip((py::ssize_t)indptr.size(), indptr.data());
  return py::make_tuple(ip, idx, data, first_dup, first_col);
}

// Synthetic TrainingExample OCF (photon-avro-schemas TrainingExample: uid, label, features[{name, term, value}],
// weight, offset, metadataMap{userId}) written natively for ingest benchmarks: ``nnz_per_record`` distinct
// features per record from a Zipf-like vocabulary of ``vocab`` names, ``n_entities`` user ids.
static int64_t gen_training_examples(const std::string& path, int64_t n_records, int nnz_per_record, int64_t vocab,
                                     int64_t n_entities, uint64_t seed, const std::string& codec, int block_records) {
  py::gil_scoped_release nogil;
  static const char* schema =
      "{\"type\":\"record\",\"name\":\"TrainingExampleAvro\",\"namespace\":\"com.linkedin.photon.avro.generated\","
      "\"fields\":[{\"name\":\"uid\",\"type\":[\"null\",\"string\"],\"default\":null},"
      "{\"name\":\"label\",\"type\":\"double\"},"
      "{\"name\":\"features\",\"type\":{\"type\":\"array\",\"items\":{\"type\":\"record\",\"name\":"
      "\"FeatureAvro\",\"fields\":[{\"name\":\"name\",\"type\":\"string\"},{\"name\":\"term\",\"type\":"
      "\"string\"},{\"name\":\"value\",\"type\":\"double\"}]}}},"
      "{\"name\":\"weight\",\"type\":[\"null\",\"double\"],\"default\":null},"
      "{\"name\":\"offset\",\"type\":[\"null\",\"double\"],\"default\":null},"
      "{\"name\":\"metadataMap\",\"type\":[\"null\",{\"type\":\"map\",\"values\":\"string\"}],"
      "\"default\":null}]}";
  std::string out("Obj\x01", 4);
  Writer hdr;
  hdr.varlong(2);
  hdr.str("avro.schema"); hdr.str(schema);
  hdr.str("avro.codec"); hdr.str(codec);
  hdr.varlong(0);
  out += hdr.buf;
  std::mt19937_64 rng(seed);
  std::string sync(16, '\0');
  for (int i = 0; i < 16; ++i) sync[i] = (char)(rng() & 0xFF);
  out += sync;
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::normal_distribution<double> N01(0.0, 1.0);
  std::vector<int64_t> feats;
  int64_t written = 0;
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path);
  f.write(out.data(), (std::streamsize)out.size());
  for (int64_t i = 0; i < n_records;) {
    const int64_t m = std::min<int64_t>(n_records - i, std::max(block_records, 1));
    Writer body;
    for (int64_t k = 0; k < m; ++k, ++i) {
      body.varlong(1); body.str("u" + std::to_string(seed) + "_" + std::to_string(i));
      body.dbl(U(rng) < 0.3 ? 1.0 : 0.0);
      feats.clear();
      while ((int)feats.size() < nnz_per_record) {   // distinct Zipf-like feature ids (u^3 skew)
        const double u = U(rng);
        const int64_t id = std::min<int64_t>(vocab - 1, (int64_t)(u * u * u * (double)vocab));
        if (std::find(feats.begin(), feats.end(), id) == feats.end()) feats.push_back(id);
      }
      body.varlong((int64_t)feats.size());
      for (int64_t id : feats) { body.str("f" + std::to_string(id)); body.str(""); body.dbl(N01(rng)); }
      body.varlong(0);
      body.varlong(0);                 // weight: null
      body.varlong(0);                 // offset: null
      body.varlong(1);                 // metadataMap: map
      body.varlong(1); body.str("userId"); body.str("e" + std::to_string((int64_t)(U(rng) * (double)n_entities)));
      body.varlong(0);
      written += (int64_t)feats.size();
    }
    std::string payload;
    if (codec == "null") payload = body.buf;
    else if (codec == "deflate") payload = deflate_raw(body.buf, 1);
    else if (codec == "snappy") {
      payload = snappy_compress(body.buf);
      uint32_t c = crc32_iso(body.buf);
      payload.push_back((char)(c >> 24)); payload.push_back((char)(c >> 16));
      payload.push_back((char)(c >> 8)); payload.push_back((char)c);
    } else throw std::runtime_error("unsupported codec " + codec);
    Writer bh; bh.varlong(m); bh.varlong((int64_t)payload.size());
    f.write(bh.buf.data(), (std::streamsize)bh.buf.size());
    f.write(payload.data(), (std::streamsize)payload.size());
    f.write(sync.data(), 16);
  }
  return written;
}

// BayesianLinearModelAvro records straight from flat model arrays (GAME model save; reference
// ModelProcessingUtils.saveGameModelToHDFS / AvroUtils): model k = coefficients [ptr[k], ptr[k+1]) with feature
// codes ``code`` (indices into the NUL-separated ``names`` blob of "name<delim>term" keys), values ``means`` and
// optional ``variances``. Per model: coefficients with |mean| > threshold, ordered by decreasing |mean| (stable), as
// name/term/value triples. Blocks of ``block_records`` models are encoded and compressed on all cores, written in
// order; the bytes equal write_ocf of the same records (same header, sync marker and codec settings).
static int64_t write_linear_models(const std::string& path, const std::string& schema_json, py::list model_ids,
                                   py::array_t<int64_t, py::array::c_style | py::array::forcecast> ptr,
                                   py::array_t<int64_t, py::array::c_style | py::array::forcecast> code,
                                   py::array_t<double, py::array::c_style | py::array::forcecast> means,
                                   py::object variances, const std::string& names, const std::string& model_class,
                                   py::object loss_function, double threshold, const std::string& codec,
                                   int block_records, const std::string& delimiter) {
  const int64_t M = (int64_t)py::len(model_ids);
  if (ptr.size() != M + 1) throw std::runtime_error("ptr must hold n_models + 1 offsets");
  std::vector<std::string> ids((size_t)M);
  for (int64_t k = 0; k < M; ++k) ids[(size_t)k] = py::str(model_ids[(size_t)k]).cast<std::string>();
  const int64_t* P = ptr.data();
  const int64_t* C = code.data();
  const double* V = means.data();
  py::array_t<double, py::array::c_style | py::array::forcecast> var_arr;
  const double* VAR = nullptr;
  if (!variances.is_none()) {
    var_arr = variances.cast<py::array_t<double, py::array::c_style | py::array::forcecast>>();
    if (var_arr.size() != means.size()) throw std::runtime_error("variances / means length mismatch");
    VAR = var_arr.data();
  }
  if (code.size() != means.size() || (M && P[M] > (int64_t)means.size())) throw std::runtime_error("bad offsets");
  const bool has_loss = !loss_function.is_none();
  const std::string loss = has_loss ? loss_function.cast<std::string>() : std::string();
  // name / term of every code
  std::vector<std::pair<std::string, std::string>> nt;
  {
    size_t a = 0;
    while (a <= names.size()) {
      size_t z = names.find('\0', a);
      if (z == std::string::npos) z = names.size();
      std::string key = names.substr(a, z - a);
      size_t d = delimiter.empty() ? std::string::npos : key.find(delimiter);
      if (d == std::string::npos) nt.emplace_back(key, std::string());
      else nt.emplace_back(key.substr(0, d), key.substr(d + delimiter.size()));
      a = z + 1;
      if (z == names.size()) break;
    }
  }
  for (int64_t t = 0; t < (M ? P[M] : 0); ++t)
    if (C[t] < 0 || C[t] >= (int64_t)nt.size()) throw std::runtime_error("feature code outside the names table");
  const int64_t B = std::max(block_records, 1);
  const int64_t nblocks = (M + B - 1) / B;
  std::vector<std::string> payloads((size_t)nblocks);
  {
    py::gil_scoped_release nogil;
    std::atomic<int64_t> next{0};
    auto work = [&]() {
      std::vector<int64_t> kept;
      for (int64_t blk; (blk = next.fetch_add(1)) < nblocks;) {
        Writer body;
        for (int64_t k = blk * B; k < std::min(M, (blk + 1) * B); ++k) {
          kept.clear();
          for (int64_t t = P[k]; t < P[k + 1]; ++t)
            if (std::fabs(V[t]) > threshold) kept.push_back(t);
          std::stable_sort(kept.begin(), kept.end(),
                           [&](int64_t a, int64_t b) { return std::fabs(V[a]) > std::fabs(V[b]); });
          body.str(ids[(size_t)k]);
          body.str(model_class);
          if (!kept.empty()) {
            body.varlong((int64_t)kept.size());
            for (int64_t t : kept) { body.str(nt[(size_t)C[t]].first); body.str(nt[(size_t)C[t]].second); body.dbl(V[t]); }
          }
          body.varlong(0);
          if (VAR) {
            body.varlong(1);
            if (!kept.empty()) {
              body.varlong((int64_t)kept.size());
              for (int64_t t : kept) { body.str(nt[(size_t)C[t]].first); body.str(nt[(size_t)C[t]].second); body.dbl(VAR[t]); }
            }
            body.varlong(0);
          } else {
            body.varlong(0);
          }
          if (has_loss) { body.varlong(1); body.str(loss); } else body.varlong(0);
        }
        std::string payload;
        if (codec == "null") payload = body.buf;
        else if (codec == "deflate") payload = deflate_raw(body.buf, 6);
        else if (codec == "snappy") {
          payload = snappy_compress(body.buf);
          uint32_t c = crc32_iso(body.buf);
          payload.push_back((char)(c >> 24)); payload.push_back((char)(c >> 16));
          payload.push_back((char)(c >> 8)); payload.push_back((char)c);
        }
        payloads[(size_t)blk] = std::move(payload);
      }
    };
    if (codec != "null" && codec != "deflate" && codec != "snappy") throw std::runtime_error("unsupported codec " + codec);
    const int nt_ = (int)std::max<int64_t>(1, std::min<int64_t>(nblocks, std::max(1u, std::thread::hardware_concurrency())));
    std::vector<std::thread> th;
    for (int i = 1; i < nt_; ++i) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
  }
  std::string out("Obj\x01", 4);
  Writer hdr;
  hdr.varlong(2);
  hdr.str("avro.schema"); hdr.str(schema_json);
  hdr.str("avro.codec"); hdr.str(codec);
  hdr.varlong(0);
  out += hdr.buf;
  std::string sync(16, '\0');
  std::mt19937_64 rng(0x5eed1234abcdULL ^ (uint64_t)M);
  for (int i = 0; i < 16; ++i) sync[i] = (char)(rng() & 0xFF);
  out += sync;
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path);
  f.write(out.data(), (std::streamsize)out.size());
  for (int64_t blk = 0; blk < nblocks; ++blk) {
    const int64_t m = std::min(M, (blk + 1) * B) - blk * B;
    Writer bh; bh.varlong(m); bh.varlong((int64_t)payloads[(size_t)blk].size());
    f.write(bh.buf.data(), (std::streamsize)bh.buf.size());
    f.write(payloads[(size_t)blk].data(), (std::streamsize)payloads[(size_t)blk].size());
    f.write(sync.data(), 16);
  }
  if (!f) throw std::runtime_error("write failed: " + path);
  return M;
}

PYBIND11_MODULE(libpml_avro, m) {
  m.def("build_id", []() { return std::string(pml_build_stamp + 13); });
  m.doc() = "photon_ml_amd native Avro OCF codec";
  m.def("read_ocf", &read_ocf, "Decode an OCF file -> (schema_json, [records], codec)");
  m.def("read_schema", &read_schema);
  m.def("write_ocf", &write_ocf, py::arg("path"), py::arg("schema_json"), py::arg("records"),
        py::arg("codec") = "deflate", py::arg("block_records") = 4096);
  m.def("write_linear_models", &write_linear_models, py::arg("path"), py::arg("schema_json"), py::arg("model_ids"),
        py::arg("ptr"), py::arg("code"), py::arg("means"), py::arg("variances"), py::arg("names"),
        py::arg("model_class"), py::arg("loss_function"), py::arg("threshold"), py::arg("codec") = "deflate",
        py::arg("block_records") = 4096, py::arg("delimiter") = std::string("\x01"));
  m.def("read_columnar", &read_columnar, py::arg("paths"), py::arg("label_fields"), py::arg("weight_field"),
        py::arg("offset_field"), py::arg("uid_field"), py::arg("metadata_field"), py::arg("bags"),
        py::arg("id_tags"), py::arg("delimiter") = std::string("\x01"), py::arg("tag_strings") = true);
  m.def("assemble_shard", &assemble_shard, py::arg("n"), py::arg("parts"), py::arg("vocab_to_col"), py::arg("dim"),
        py::arg("intercept_col"), py::arg("check_duplicates"), py::arg("threads") = 0);
  m.def("gen_training_examples", &gen_training_examples, py::arg("path"), py::arg("n_records"),
        py::arg("nnz_per_record"), py::arg("vocab"), py::arg("n_entities"), py::arg("seed"),
        py::arg("codec") = std::string("deflate"), py::arg("block_records") = 4096);
  m.def("snappy_compress", [](const std::string& s) { return py::bytes(snappy_compress(s)); });
  m.def("snappy_roundtrip", [](const std::string& s) {
    std::string c = snappy_compress(s);
    return snappy_decompress((const uint8_t*)c.data(), c.size()) == s;
  });
  init_crc32c();
}

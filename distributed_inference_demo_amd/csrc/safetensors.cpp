// safetensors reader: 8-byte little-endian header length, a JSON header
// {name: {"dtype", "shape", "data_offsets": [begin, end]}, "__metadata__": {...}}, then the data
// block the offsets index.  Sharded checkpoints: an index JSON {"weight_map": {name: file}} beside
// the shards.  Everything from the file is bounds-checked: a checkpoint is untrusted input.
#include "safetensors.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <memory>
#include <set>

namespace st {
namespace {

// Minimal JSON value tree: enough for safetensors headers and HF index files.
struct Value {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  double num = 0;
  bool is_int = false;
  int64_t ival = 0;
  std::string str;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;
  const Value* get(const char* k) const {
    for (const auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), end_(p + n) {}
  bool parse(Value* v) {
    if (!value(v, 0)) return false;
    ws();
    return p_ == end_;
  }

 private:
  const char* p_;
  const char* end_;
  void ws() {
    while (p_ < end_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) p_++;
  }
  bool lit(const char* s) {
    const size_t n = strlen(s);
    if ((size_t)(end_ - p_) < n || memcmp(p_, s, n)) return false;
    p_ += n;
    return true;
  }
  static void utf8(uint32_t c, std::string* out) {
    if (c < 0x80) {
      out->push_back((char)c);
    } else if (c < 0x800) {
      out->push_back((char)(0xC0 | (c >> 6)));
      out->push_back((char)(0x80 | (c & 0x3F)));
    } else if (c < 0x10000) {
      out->push_back((char)(0xE0 | (c >> 12)));
      out->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      out->push_back((char)(0x80 | (c & 0x3F)));
    } else {
      out->push_back((char)(0xF0 | (c >> 18)));
      out->push_back((char)(0x80 | ((c >> 12) & 0x3F)));
      out->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      out->push_back((char)(0x80 | (c & 0x3F)));
    }
  }
  bool hex4(uint32_t* c) {
    if (end_ - p_ < 4) return false;
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
      const char h = *p_++;
      v <<= 4;
      if (h >= '0' && h <= '9') v |= h - '0';
      else if (h >= 'a' && h <= 'f') v |= h - 'a' + 10;
      else if (h >= 'A' && h <= 'F') v |= h - 'A' + 10;
      else return false;
    }
    *c = v;
    return true;
  }
  bool string(std::string* out) {
    if (p_ >= end_ || *p_ != '"') return false;
    p_++;
    while (p_ < end_ && *p_ != '"') {
      if (*p_ != '\\') {
        out->push_back(*p_++);
        continue;
      }
      if (++p_ >= end_) return false;
      const char e = *p_++;
      switch (e) {
        case '"': case '\\': case '/': out->push_back(e); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t c;
          if (!hex4(&c)) return false;
          if (c >= 0xD800 && c < 0xDC00) {  // surrogate pair
            uint32_t lo;
            if (!lit("\\u") || !hex4(&lo) || lo < 0xDC00 || lo >= 0xE000) return false;
            c = 0x10000 + ((c - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(c, out);
          break;
        }
        default: return false;
      }
    }
    if (p_ >= end_) return false;
    p_++;
    return true;
  }
  bool number(Value* v) {
    const char* s = p_;
    bool integral = true;
    if (p_ < end_ && *p_ == '-') p_++;
    if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) return false;
    while (p_ < end_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '+' ||
                         *p_ == '-')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') integral = false;
      p_++;
    }
    const std::string t(s, p_);
    v->kind = Value::NUM;
    v->num = strtod(t.c_str(), nullptr);
    if (integral && t.size() <= 18) {  // exact for every offset a file can hold
      v->is_int = true;
      v->ival = strtoll(t.c_str(), nullptr, 10);
    }
    return true;
  }
  bool value(Value* v, int depth) {
    if (depth > 64) return false;
    ws();
    if (p_ >= end_) return false;
    switch (*p_) {
      case '{': {
        p_++;
        v->kind = Value::OBJ;
        ws();
        if (p_ < end_ && *p_ == '}') { p_++; return true; }
        for (;;) {
          ws();
          std::string k;
          if (!string(&k)) return false;
          ws();
          if (p_ >= end_ || *p_++ != ':') return false;
          v->obj.emplace_back(std::move(k), Value());
          if (!value(&v->obj.back().second, depth + 1)) return false;
          ws();
          if (p_ >= end_) return false;
          if (*p_ == ',') { p_++; continue; }
          if (*p_ == '}') { p_++; return true; }
          return false;
        }
      }
      case '[': {
        p_++;
        v->kind = Value::ARR;
        ws();
        if (p_ < end_ && *p_ == ']') { p_++; return true; }
        for (;;) {
          v->arr.emplace_back();
          if (!value(&v->arr.back(), depth + 1)) return false;
          ws();
          if (p_ >= end_) return false;
          if (*p_ == ',') { p_++; continue; }
          if (*p_ == ']') { p_++; return true; }
          return false;
        }
      }
      case '"': v->kind = Value::STR; return string(&v->str);
      case 't': v->kind = Value::BOOL; return lit("true");
      case 'f': v->kind = Value::BOOL; return lit("false");
      case 'n': v->kind = Value::NUL; return lit("null");
      default: return number(v);
    }
  }
};

Dtype dtype_of(const std::string& s, uint64_t* esz) {
  if (s == "F32") { *esz = 4; return F32; }
  if (s == "F16") { *esz = 2; return F16; }
  if (s == "BF16") { *esz = 2; return BF16; }
  static const struct { const char* n; uint64_t e; } other[] = {
      {"F64", 8}, {"I64", 8}, {"U64", 8}, {"I32", 4}, {"U32", 4}, {"I16", 2}, {"U16", 2},
      {"I8", 1},  {"U8", 1},  {"BOOL", 1}, {"F8_E4M3", 1}, {"F8_E5M2", 1}};
  for (const auto& o : other)
    if (s == o.n) { *esz = o.e; return OTHER; }
  *esz = 0;
  return OTHER;
}

bool read_text(const std::string& path, std::string* out, std::string* err) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) { *err = "cannot open " + path; return false; }
  struct stat sb;
  if (fstat(fd, &sb) || sb.st_size > (64 << 20)) { ::close(fd); *err = "bad index file " + path; return false; }
  out->resize((size_t)sb.st_size);
  size_t got = 0;
  while (got < out->size()) {
    const ssize_t r = ::read(fd, &(*out)[got], out->size() - got);
    if (r <= 0) { ::close(fd); *err = "read failed: " + path; return false; }
    got += (size_t)r;
  }
  ::close(fd);
  return true;
}

}  // namespace

Checkpoint::~Checkpoint() {
  for (auto& m : maps_) munmap(m.base, m.len);
}

bool Checkpoint::map_file(const std::string& path, std::string* err) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) { *err = "cannot open " + path; return false; }
  struct stat sb;
  if (fstat(fd, &sb) || sb.st_size < 8) { ::close(fd); *err = "not a safetensors file (too short): " + path; return false; }
  const size_t len = (size_t)sb.st_size;
  void* base = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (base == MAP_FAILED) { *err = "mmap failed: " + path; return false; }
  maps_.push_back({base, len});
  const uint8_t* b = (const uint8_t*)base;
  uint64_t hlen = 0;
  for (int i = 0; i < 8; i++) hlen |= (uint64_t)b[i] << (8 * i);
  if (hlen > len - 8) { *err = "header length past the end of " + path; return false; }
  // the upstream safetensors format caps the JSON header at 100 MB; a larger one is not a checkpoint
  // (and would only make the recursive parser build a huge tree from untrusted input)
  if (hlen > (100ull << 20)) { *err = "safetensors header of " + std::to_string(hlen) + " B exceeds the 100 MB cap in " + path; return false; }
  Value root;
  if (!Parser((const char*)b + 8, (size_t)hlen).parse(&root) || root.kind != Value::OBJ) {
    *err = "malformed safetensors header: " + path;
    return false;
  }
  const uint8_t* data = b + 8 + hlen;
  const uint64_t dlen = len - 8 - hlen;
  for (const auto& kv : root.obj) {
    if (kv.first == "__metadata__") continue;
    const Value& t = kv.second;
    const Value* dt = t.get("dtype");
    const Value* sh = t.get("shape");
    const Value* off = t.get("data_offsets");
    if (t.kind != Value::OBJ || !dt || dt->kind != Value::STR || !sh || sh->kind != Value::ARR || !off ||
        off->kind != Value::ARR || off->arr.size() != 2) {
      *err = "bad tensor entry '" + kv.first + "' in " + path;
      return false;
    }
    Tensor ten;
    uint64_t esz = 0;
    ten.dtype = dtype_of(dt->str, &esz);
    ten.dtype_name = dt->str;
    if (!esz) { *err = "unknown dtype " + dt->str + " of '" + kv.first + "'"; return false; }
    uint64_t numel = 1;
    for (const auto& d : sh->arr) {
      if (!d.is_int || d.ival < 0) { *err = "bad shape of '" + kv.first + "'"; return false; }
      if (d.ival && numel > UINT64_MAX / (uint64_t)d.ival) { *err = "shape overflow of '" + kv.first + "'"; return false; }
      numel *= (uint64_t)d.ival;
      ten.shape.push_back(d.ival);
    }
    const Value &o0 = off->arr[0], &o1 = off->arr[1];
    if (!o0.is_int || !o1.is_int || o0.ival < 0 || o1.ival < o0.ival || (uint64_t)o1.ival > dlen) {
      *err = "data_offsets of '" + kv.first + "' outside the data block of " + path;
      return false;
    }
    ten.bytes = (uint64_t)(o1.ival - o0.ival);
    if (numel > UINT64_MAX / esz || ten.bytes != numel * esz) {
      *err = "data_offsets of '" + kv.first + "' disagree with its shape and dtype";
      return false;
    }
    ten.data = data + o0.ival;
    if (!tensors_.emplace(kv.first, std::move(ten)).second) {
      *err = "duplicate tensor '" + kv.first + "'";
      return false;
    }
  }
  return true;
}

bool Checkpoint::open(const std::string& path, std::string* err) {
  const bool index = path.size() >= 5 && path.compare(path.size() - 5, 5, ".json") == 0;
  if (!index) return map_file(path, err);
  std::string text;
  if (!read_text(path, &text, err)) return false;
  Value root;
  const Value* wm = nullptr;
  if (!Parser(text.data(), text.size()).parse(&root) || root.kind != Value::OBJ || !(wm = root.get("weight_map")) ||
      wm->kind != Value::OBJ) {
    *err = "malformed checkpoint index " + path;
    return false;
  }
  const size_t slash = path.find_last_of('/');
  const std::string dir = slash == std::string::npos ? "" : path.substr(0, slash + 1);
  std::set<std::string> shards;
  for (const auto& kv : wm->obj) {
    if (kv.second.kind != Value::STR || kv.second.str.empty() || kv.second.str.find('/') != std::string::npos) {
      *err = "bad shard name for '" + kv.first + "' in " + path;  // shards live beside the index
      return false;
    }
    shards.insert(kv.second.str);
  }
  for (const auto& f : shards)
    if (!map_file(dir + f, err)) return false;
  for (const auto& kv : wm->obj)
    if (!tensors_.count(kv.first)) {
      *err = "index names '" + kv.first + "' but shard " + kv.second.str + " does not hold it";
      return false;
    }
  return true;
}

const Tensor* Checkpoint::find(const std::string& name) const {
  auto it = tensors_.find(name);
  if (it == tensors_.end()) it = tensors_.find("transformer." + name);
  return it == tensors_.end() ? nullptr : &it->second;
}

}  // namespace st

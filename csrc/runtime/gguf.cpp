#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

#include "qtypes.h"

namespace mp {

namespace {
struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  void need(size_t n) {
    if ((size_t)(end - p) < n) throw std::runtime_error("gguf: truncated file");
  }
  template <class T> T rd() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint64_t n = rd<uint64_t>();
    if (n > (1ull << 32)) throw std::runtime_error("gguf: string too long");
    need(n);
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
};

double read_num(Cursor& c, uint32_t t, int64_t* iv) {
  switch (t) {
    case GV_U8: { auto v = c.rd<uint8_t>(); *iv = v; return v; }
    case GV_I8: { auto v = c.rd<int8_t>(); *iv = v; return v; }
    case GV_U16: { auto v = c.rd<uint16_t>(); *iv = v; return v; }
    case GV_I16: { auto v = c.rd<int16_t>(); *iv = v; return v; }
    case GV_U32: { auto v = c.rd<uint32_t>(); *iv = v; return v; }
    case GV_I32: { auto v = c.rd<int32_t>(); *iv = v; return v; }
    case GV_F32: { auto v = c.rd<float>(); *iv = (int64_t)v; return v; }
    case GV_BOOL: { auto v = c.rd<uint8_t>(); *iv = v != 0; return v != 0; }
    case GV_U64: { auto v = c.rd<uint64_t>(); *iv = (int64_t)v; return (double)v; }
    case GV_I64: { auto v = c.rd<int64_t>(); *iv = v; return (double)v; }
    case GV_F64: { auto v = c.rd<double>(); *iv = (int64_t)v; return v; }
  }
  throw std::runtime_error("gguf: bad value type " + std::to_string(t));
}
}  // namespace

GgufFile::GgufFile(const std::string& path) : path_(path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("gguf: cannot open " + path);
  struct stat st;
  if (fstat(fd_, &st) != 0) throw std::runtime_error("gguf: stat failed");
  size_ = (size_t)st.st_size;
  if (size_ < 24) throw std::runtime_error("gguf: file too small");
  void* m = mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0);
  if (m == MAP_FAILED) throw std::runtime_error("gguf: mmap failed");
  map_ = static_cast<uint8_t*>(m);
  Cursor c{map_, map_ + size_};
  if (c.rd<uint32_t>() != 0x46554747u) throw std::runtime_error("gguf: bad magic");
  version_ = c.rd<uint32_t>();
  if (version_ < 2 || version_ > 3) throw std::runtime_error("gguf: unsupported version");
  const uint64_t n_t = c.rd<uint64_t>();
  const uint64_t n_kv = c.rd<uint64_t>();
  if (n_t > (1u << 24) || n_kv > (1u << 24)) throw std::runtime_error("gguf: absurd counts");
  for (uint64_t i = 0; i < n_kv; ++i) {
    std::string key = c.str();
    GgufValue v;
    v.type = c.rd<uint32_t>();
    if (v.type == GV_STRING) {
      v.s = c.str();
    } else if (v.type == GV_ARRAY) {
      v.elem_type = c.rd<uint32_t>();
      uint64_t n = c.rd<uint64_t>();
      if (n > (1ull << 28)) throw std::runtime_error("gguf: array too long");
      if (v.elem_type == GV_STRING) {
        v.strs.reserve(n);
        for (uint64_t j = 0; j < n; ++j) v.strs.push_back(c.str());
      } else if (v.elem_type == GV_ARRAY) {
        throw std::runtime_error("gguf: nested arrays unsupported");
      } else {
        v.nums.reserve(n);
        int64_t iv;
        for (uint64_t j = 0; j < n; ++j) v.nums.push_back(read_num(c, v.elem_type, &iv));
      }
    } else {
      v.f = read_num(c, v.type, &v.i);
    }
    kv_[key] = std::move(v);
  }
  const int64_t align = get_int("general.alignment", 32);
  if (align <= 0 || (align & (align - 1))) throw std::runtime_error("gguf: bad alignment");
  tensors_.reserve(n_t);
  for (uint64_t i = 0; i < n_t; ++i) {
    GgufTensor t;
    t.name = c.str();
    uint32_t nd = c.rd<uint32_t>();
    if (nd == 0 || nd > 4) throw std::runtime_error("gguf: bad n_dims");
    for (uint32_t d = 0; d < nd; ++d) t.ne.push_back((int64_t)c.rd<uint64_t>());
    t.type = (int)c.rd<uint32_t>();
    t.offset = c.rd<uint64_t>();
    tensors_.push_back(std::move(t));
  }
  size_t data_start = (size_t)(c.p - map_);
  data_start = (data_start + align - 1) / align * align;
  for (size_t i = 0; i < tensors_.size(); ++i) {
    auto& t = tensors_[i];
    const int be = block_elems(t.type);
    if (be > 0) {
      if (t.ne[0] % be) throw std::runtime_error("gguf: tensor row not a block multiple: " + t.name);
      t.nbytes = (size_t)(t.nelem() / be) * block_bytes(t.type);
    }
    t.offset += data_start;
    if (t.offset + t.nbytes > size_) throw std::runtime_error("gguf: tensor out of bounds: " + t.name);
    t.data = map_ + t.offset;
    index_[t.name] = i;
  }
}

GgufFile::~GgufFile() {
  if (map_) munmap(map_, size_);
  if (fd_ >= 0) ::close(fd_);
}

const GgufValue* GgufFile::get(const std::string& k) const {
  auto it = kv_.find(k);
  return it == kv_.end() ? nullptr : &it->second;
}
int64_t GgufFile::get_int(const std::string& k, int64_t d) const {
  auto* v = get(k);
  if (!v || v->type == GV_STRING || v->type == GV_ARRAY) return d;
  return v->type == GV_F32 || v->type == GV_F64 ? (int64_t)v->f : v->i;
}
double GgufFile::get_float(const std::string& k, double d) const {
  auto* v = get(k);
  if (!v || v->type == GV_STRING || v->type == GV_ARRAY) return d;
  return v->f;
}
std::string GgufFile::get_str(const std::string& k, const std::string& d) const {
  auto* v = get(k);
  return (v && v->type == GV_STRING) ? v->s : d;
}
bool GgufFile::get_bool(const std::string& k, bool d) const {
  auto* v = get(k);
  if (!v || v->type == GV_STRING || v->type == GV_ARRAY) return d;
  return v->i != 0;
}
const GgufTensor* GgufFile::tensor(const std::string& name) const {
  auto it = index_.find(name);
  return it == index_.end() ? nullptr : &tensors_[it->second];
}

}  // namespace mp

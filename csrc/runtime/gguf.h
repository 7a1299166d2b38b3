// GGUF v2/v3 reader: mmap, zero-copy tensor views, typed KV access.
// Replaces llama.cpp's gguf.cpp + llama-model-loader (E3, upstream; not in mount).
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <map>
#include <string>
#include <vector>

namespace mp {

enum GgufVType : uint32_t {
  GV_U8 = 0, GV_I8, GV_U16, GV_I16, GV_U32, GV_I32, GV_F32, GV_BOOL, GV_STRING, GV_ARRAY, GV_U64, GV_I64, GV_F64
};

struct GgufValue {
  uint32_t type = 0;
  uint32_t elem_type = 0;           // for arrays
  int64_t i = 0;                    // integer / bool scalars
  double f = 0;                     // float scalars
  std::string s;                    // string scalar
  std::vector<std::string> strs;    // string arrays
  std::vector<double> nums;         // numeric arrays
};

struct GgufTensor {
  std::string name;
  std::vector<int64_t> ne;          // ggml order (ne[0] contiguous)
  int type = 0;
  uint64_t offset = 0;              // absolute file offset
  size_t nbytes = 0;
  const uint8_t* data = nullptr;    // mmap pointer
  int64_t nelem() const { int64_t n = 1; for (auto v : ne) n *= v; return n; }
};

class GgufFile {
 public:
  explicit GgufFile(const std::string& path);
  ~GgufFile();
  GgufFile(const GgufFile&) = delete;
  GgufFile& operator=(const GgufFile&) = delete;

  const std::string& path() const { return path_; }
  uint32_t version() const { return version_; }
  size_t file_size() const { return size_; }
  bool has(const std::string& k) const { return kv_.count(k) != 0; }
  const GgufValue* get(const std::string& k) const;
  int64_t get_int(const std::string& k, int64_t dflt) const;
  double get_float(const std::string& k, double dflt) const;
  std::string get_str(const std::string& k, const std::string& dflt) const;
  bool get_bool(const std::string& k, bool dflt) const;
  const std::map<std::string, GgufValue>& kv() const { return kv_; }
  const std::vector<GgufTensor>& tensors() const { return tensors_; }
  const GgufTensor* tensor(const std::string& name) const;

 private:
  std::string path_;
  int fd_ = -1;
  uint8_t* map_ = nullptr;
  size_t size_ = 0;
  uint32_t version_ = 0;
  std::map<std::string, GgufValue> kv_;
  std::vector<GgufTensor> tensors_;
  std::map<std::string, size_t> index_;
};

}  // namespace mp

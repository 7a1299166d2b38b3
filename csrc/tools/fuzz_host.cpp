// Host-side robustness driver for sanitizer builds: feeds untrusted inputs to the
// parsers the servers expose -- GGUF files (header, metadata, tensor table, model config, tokenizer
// construction + a round trip through every tensor's bytes) and JSON request bodies -- and reports
// how each input was handled.  Built with -fsanitize=address,undefined (make sanitize); the test
// suite (tests/test_sanitize.py) drives it with corrupted GGUF files and random JSON and fails on
// any sanitizer report.  A clean rejection (exception) is the expected outcome for bad input.
//
//   fuzz_host gguf FILE...    exit 0; prints "ok" / "rejected: <reason>" per file
//   fuzz_host json FILE...
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>

#include "gguf.h"
#include "json.h"
#include "model.h"
#include "qtypes.h"
#include "tokenizer.h"

using namespace mp;

static std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static void check_gguf(const char* path) {
  GgufFile f(path);
  size_t touched = 0;
  for (const auto& kv : f.kv()) touched += kv.first.size();
  for (const GgufTensor& t : f.tensors()) {
    // every tensor's extent must lie inside the mapping: read its first and last byte
    if (t.nbytes) touched += t.data[0] + t.data[t.nbytes - 1];
  }
  ModelConfig c = ModelConfig::from_gguf(f);
  touched += (size_t)c.n_layer;
  Tokenizer tok = Tokenizer::from_gguf(f);
  const std::vector<int32_t> ids = tok.encode("Hello world, héllo 🚀 1234", true);
  touched += tok.decode(ids).size();
  std::printf("ok %zu\n", touched & 0xFF);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: fuzz_host gguf|json FILE...\n");
    return 2;
  }
  const std::string mode = argv[1];
  for (int i = 2; i < argc; ++i) {
    try {
      if (mode == "gguf") {
        check_gguf(argv[i]);
      } else if (mode == "json") {
        const Json j = Json::parse(slurp(argv[i]));
        std::printf("ok %s\n", j.is_obj() ? "object" : "value");
      } else {
        std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
      }
    } catch (const std::exception& e) {
      std::printf("rejected: %.120s\n", e.what());
    }
  }
  return 0;
}

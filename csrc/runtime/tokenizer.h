// Tokenizers read from GGUF metadata (E11 of SURVEY.md §2.2; llama.cpp's llama-vocab.cpp is
// upstream, not in mount):
//   - "gpt2"  byte-level BPE (Llama-3: pre-tokenizer regex "llama-bpe", merges by rank)
//   - "llama" SentencePiece-style (TinyLlama / Mixtral / stories15M: U+2581 word boundary,
//             score-driven bigram merging, <0xXX> byte fallback)
// No PCRE/ICU: the Llama-3 pre-tokenizer is a hand-written matcher over code points with compact
// Unicode category tables (letters, numbers, whitespace).
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace mp {

class GgufFile;

class Tokenizer {
 public:
  enum Kind { BPE = 0, SPM = 1 };
  static Tokenizer from_gguf(const GgufFile& f);

  std::vector<int32_t> encode(const std::string& text, bool add_bos, bool parse_special = true) const;
  std::string piece(int32_t id) const;                 // bytes of one token (control -> "")
  std::string decode(const std::vector<int32_t>& ids) const;
  bool is_eog(int32_t id) const { return id == eos_ || id == eot_; }

  int n_vocab() const { return (int)tokens_.size(); }
  int bos() const { return bos_; }
  bool add_bos_default() const { return add_bos_default_; }
  int eos() const { return eos_; }
  int eot() const { return eot_; }
  Kind kind() const { return kind_; }

  // exposed for tests
  // max_digits: \p{N}{1,3} for llama-bpe, single digits (\p{N}) for the qwen2 pre-tokenizer
  static std::vector<std::string> llama3_pretokenize(const std::string& text, int max_digits = 3);

 private:
  int max_digits_ = 3;
  void encode_bpe_segment(const std::string& s, std::vector<int32_t>& out) const;
  void encode_spm_segment(const std::string& s, std::vector<int32_t>& out) const;

  Kind kind_ = SPM;
  std::vector<std::string> tokens_;
  std::vector<float> scores_;
  std::vector<int> types_;
  std::unordered_map<std::string, int32_t> tok2id_;
  std::unordered_map<std::string, int> merge_rank_;   // "a b" -> rank
  std::vector<std::pair<std::string, int32_t>> specials_;  // sorted longest first
  int32_t bos_ = -1, eos_ = -1, eot_ = -1, unk_ = 0;
  bool add_space_prefix_ = true;
  bool add_bos_default_ = true;
  int32_t byte_tok_[256];
};

// UTF-8 helpers
std::vector<uint32_t> utf8_decode(const std::string& s);
std::string utf8_encode(uint32_t cp);
bool uc_is_letter(uint32_t cp);
bool uc_is_number(uint32_t cp);
bool uc_is_space(uint32_t cp);

}  // namespace mp

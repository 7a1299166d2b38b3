#include "tokenizer.h"
#include "unicode_tables.h"

#include <algorithm>
#include <climits>
#include <queue>
#include <stdexcept>

#include "gguf.h"

namespace mp {

// ------------------------------------------------------------------ UTF-8
std::vector<uint32_t> utf8_decode(const std::string& s) {
  std::vector<uint32_t> o;
  o.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
    else { o.push_back(0xFFFD); ++i; continue; }
    if (i + n > s.size()) { o.push_back(0xFFFD); ++i; continue; }
    bool ok = true;
    for (int k = 1; k < n; ++k) {
      const unsigned char cc = (unsigned char)s[i + k];
      if ((cc >> 6) != 2) { ok = false; break; }
      cp = (cp << 6) | (cc & 0x3F);
    }
    if (!ok) { o.push_back(0xFFFD); ++i; continue; }
    o.push_back(cp);
    i += n;
  }
  return o;
}

std::string utf8_encode(uint32_t cp) {
  std::string o;
  if (cp < 0x80) o += (char)cp;
  else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) {
    o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
  } else {
    o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
    o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
  }
  return o;
}

// ------------------------------------------------------------------ Unicode categories (compact)
namespace {
using uc::Range;
using uc::kLetters;
using uc::kNumbers;
using uc::kSpaces;
template <size_t N>
bool in_ranges(const Range (&r)[N], uint32_t cp) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (cp < r[mid].a) hi = mid;
    else if (cp > r[mid].b) lo = mid + 1;
    else return true;
  }
  return false;
}
}  // namespace

bool uc_is_letter(uint32_t cp) { return cp >= 0x41 && in_ranges(kLetters, cp); }
bool uc_is_number(uint32_t cp) { return cp >= 0x30 && in_ranges(kNumbers, cp); }
bool uc_is_space(uint32_t cp) { return cp >= 0x09 && in_ranges(kSpaces, cp); }

// ------------------------------------------------------------------ Llama-3 pre-tokenizer
// (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+
std::vector<std::string> Tokenizer::llama3_pretokenize(const std::string& text, int max_digits) {
  const std::vector<uint32_t> cp = utf8_decode(text);
  const size_t n = cp.size();
  auto L = [&](size_t i) { return i < n && uc_is_letter(cp[i]); };
  auto N = [&](size_t i) { return i < n && uc_is_number(cp[i]); };
  auto S = [&](size_t i) { return i < n && uc_is_space(cp[i]); };
  auto NL = [&](size_t i) { return i < n && (cp[i] == '\r' || cp[i] == '\n'); };
  auto other = [&](size_t i) { return i < n && !uc_is_space(cp[i]) && !uc_is_letter(cp[i]) && !uc_is_number(cp[i]); };
  auto lower = [&](size_t i) -> uint32_t { return i < n && cp[i] >= 'A' && cp[i] <= 'Z' ? cp[i] + 32 : (i < n ? cp[i] : 0); };
  std::vector<std::string> out;
  size_t i = 0;
  while (i < n) {
    size_t e = 0;
    // 1. contractions
    if (cp[i] == '\'') {
      const uint32_t a = lower(i + 1), b = lower(i + 2);
      if (a == 's' || a == 't' || a == 'm' || a == 'd') e = i + 2;
      else if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) e = i + 3;
    }
    // 2. [^\r\n\p{L}\p{N}]?\p{L}+
    if (!e) {
      size_t j = i;
      if (!L(j) && !N(j) && !NL(j) && L(j + 1)) j = j + 1;
      if (L(j)) {
        while (L(j)) ++j;
        e = j;
      }
    }
    // 3. \p{N}{1,3}
    if (!e && N(i)) {
      size_t j = i;
      while (j < i + (size_t)max_digits && N(j)) ++j;
      e = j;
    }
    // 4.  ?[^\s\p{L}\p{N}]+[\r\n]*
    if (!e) {
      size_t j = i;
      if (cp[j] == ' ' && other(j + 1)) ++j;
      if (other(j)) {
        while (other(j)) ++j;
        while (NL(j)) ++j;
        e = j;
      }
    }
    if (!e && S(i)) {
      size_t run = i;
      while (S(run)) ++run;
      // 5. \s*[\r\n]+
      size_t last_nl = SIZE_MAX;
      for (size_t k = i; k < run; ++k) if (NL(k)) last_nl = k;
      if (last_nl != SIZE_MAX) e = last_nl + 1;
      // 6. \s+(?!\S)
      else if (run == n) e = run;
      else if (run - i >= 2) e = run - 1;
      // 7. \s+
      else e = run;
    }
    if (!e) e = i + 1;   // unreachable for well-formed input; keep progress
    std::string piece;
    for (size_t k = i; k < e; ++k) piece += utf8_encode(cp[k]);
    out.push_back(piece);
    i = e;
  }
  return out;
}

// ------------------------------------------------------------------ byte-level map (GPT-2)
namespace {
struct ByteMap {
  uint32_t b2u[256];
  std::unordered_map<uint32_t, uint8_t> u2b;
  ByteMap() {
    int n = 0;
    for (int b = 0; b < 256; ++b) {
      const bool keep = (b >= 33 && b <= 126) || (b >= 161 && b <= 172) || (b >= 174 && b <= 255);
      b2u[b] = keep ? (uint32_t)b : (uint32_t)(256 + n++);
      u2b[b2u[b]] = (uint8_t)b;
    }
  }
};
const ByteMap& bytemap() {
  static ByteMap m;
  return m;
}
}  // namespace

// ------------------------------------------------------------------ construction
Tokenizer Tokenizer::from_gguf(const GgufFile& f) {
  Tokenizer t;
  const std::string model = f.get_str("tokenizer.ggml.model", "llama");
  if (model == "gpt2") t.kind_ = BPE;
  else if (model == "llama") t.kind_ = SPM;
  else throw std::runtime_error("unsupported tokenizer model: " + model);
  const GgufValue* toks = f.get("tokenizer.ggml.tokens");
  if (!toks || toks->strs.empty()) throw std::runtime_error("GGUF has no tokenizer.ggml.tokens");
  t.tokens_ = toks->strs;
  const size_t V = t.tokens_.size();
  t.scores_.assign(V, 0.f);
  if (const GgufValue* sc = f.get("tokenizer.ggml.scores"))
    for (size_t i = 0; i < V && i < sc->nums.size(); ++i) t.scores_[i] = (float)sc->nums[i];
  t.types_.assign(V, 1);
  if (const GgufValue* ty = f.get("tokenizer.ggml.token_type"))
    for (size_t i = 0; i < V && i < ty->nums.size(); ++i) t.types_[i] = (int)ty->nums[i];
  for (size_t i = 0; i < V; ++i) t.tok2id_.emplace(t.tokens_[i], (int32_t)i);
  if (t.kind_ == BPE) {
    const GgufValue* m = f.get("tokenizer.ggml.merges");
    if (!m) throw std::runtime_error("BPE tokenizer without merges");
    for (size_t r = 0; r < m->strs.size(); ++r) t.merge_rank_.emplace(m->strs[r], (int)r);
  }
  t.bos_ = (int32_t)f.get_int("tokenizer.ggml.bos_token_id", t.kind_ == SPM ? 1 : -1);
  t.eos_ = (int32_t)f.get_int("tokenizer.ggml.eos_token_id", t.kind_ == SPM ? 2 : -1);
  t.eot_ = (int32_t)f.get_int("tokenizer.ggml.eot_token_id", -1);
  t.unk_ = (int32_t)f.get_int("tokenizer.ggml.unknown_token_id", 0);
  t.add_space_prefix_ = f.get_bool("tokenizer.ggml.add_space_prefix", t.kind_ == SPM);
  const std::string pre = f.get_str("tokenizer.ggml.pre", "llama-bpe");
  t.max_digits_ = pre == "qwen2" ? 1 : 3;   // qwen2 splits numbers into single digits
  t.add_bos_default_ = f.get_bool("tokenizer.ggml.add_bos_token", pre != "qwen2");
  for (size_t i = 0; i < V; ++i)
    if ((t.types_[i] == 3 || t.types_[i] == 4) && !t.tokens_[i].empty()) t.specials_.push_back({t.tokens_[i], (int32_t)i});
  std::sort(t.specials_.begin(), t.specials_.end(),
            [](const auto& a, const auto& b) { return a.first.size() > b.first.size(); });
  for (int b = 0; b < 256; ++b) {
    char buf[8];
    snprintf(buf, sizeof(buf), "<0x%02X>", b);
    auto it = t.tok2id_.find(buf);
    t.byte_tok_[b] = it == t.tok2id_.end() ? -1 : it->second;
  }
  return t;
}

// ------------------------------------------------------------------ encode
void Tokenizer::encode_bpe_segment(const std::string& s, std::vector<int32_t>& out) const {
  const ByteMap& bm = bytemap();
  for (const std::string& word : llama3_pretokenize(s, max_digits_)) {
    std::vector<std::string> sym;
    for (unsigned char c : word) sym.push_back(utf8_encode(bm.b2u[c]));
    while (sym.size() > 1) {
      int best = INT_MAX;
      size_t bi = 0;
      for (size_t i = 0; i + 1 < sym.size(); ++i) {
        auto it = merge_rank_.find(sym[i] + " " + sym[i + 1]);
        if (it != merge_rank_.end() && it->second < best) { best = it->second; bi = i; }
      }
      if (best == INT_MAX) break;
      const std::string a = sym[bi], b = sym[bi + 1];
      std::vector<std::string> nx;
      nx.reserve(sym.size());
      for (size_t i = 0; i < sym.size();) {
        if (i + 1 < sym.size() && sym[i] == a && sym[i + 1] == b) { nx.push_back(a + b); i += 2; }
        else { nx.push_back(sym[i]); ++i; }
      }
      sym.swap(nx);
    }
    for (const std::string& x : sym) {
      auto it = tok2id_.find(x);
      if (it != tok2id_.end()) { out.push_back(it->second); continue; }
      // unknown symbol: fall back to single byte-level characters
      for (uint32_t u : utf8_decode(x)) {
        auto jt = tok2id_.find(utf8_encode(u));
        out.push_back(jt == tok2id_.end() ? unk_ : jt->second);
      }
    }
  }
}

void Tokenizer::encode_spm_segment(const std::string& raw, std::vector<int32_t>& out) const {
  // whitespace escaping: ' ' -> U+2581
  std::string text;
  for (char c : raw) {
    if (c == ' ') text += "\xE2\x96\x81";
    else text += c;
  }
  struct Sym { int prev, next; size_t off, len; };
  std::vector<Sym> sy;
  {
    size_t i = 0;
    while (i < text.size()) {
      const unsigned char c = (unsigned char)text[i];
      size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
      n = std::min(n, text.size() - i);
      sy.push_back({(int)sy.size() - 1, (int)sy.size() + 1, i, n});
      i += n;
    }
    if (!sy.empty()) sy.back().next = -1;
  }
  struct Big { int l, r; float score; size_t size; };
  auto cmp = [](const Big& a, const Big& b) { return a.score < b.score || (a.score == b.score && a.l > b.l); };
  std::priority_queue<Big, std::vector<Big>, decltype(cmp)> q(cmp);
  auto try_add = [&](int l, int r) {
    if (l < 0 || r < 0) return;
    const std::string s = text.substr(sy[l].off, sy[l].len + sy[r].len);
    auto it = tok2id_.find(s);
    if (it == tok2id_.end()) return;
    q.push({l, r, scores_[it->second], s.size()});
  };
  for (size_t i = 1; i < sy.size(); ++i) try_add((int)i - 1, (int)i);
  while (!q.empty()) {
    Big b = q.top();
    q.pop();
    Sym& L = sy[b.l];
    Sym& R = sy[b.r];
    if (L.len == 0 || R.len == 0 || L.len + R.len != b.size || L.next != b.r) continue;
    L.len += R.len;
    R.len = 0;
    L.next = R.next;
    if (R.next >= 0) sy[R.next].prev = b.l;
    try_add(L.prev, b.l);
    try_add(b.l, L.next);
  }
  for (int i = sy.empty() ? -1 : 0; i >= 0; i = sy[i].next) {
    const std::string s = text.substr(sy[i].off, sy[i].len);
    auto it = tok2id_.find(s);
    if (it != tok2id_.end()) { out.push_back(it->second); continue; }
    for (unsigned char c : s) out.push_back(byte_tok_[c] >= 0 ? byte_tok_[c] : unk_);
  }
}

std::vector<int32_t> Tokenizer::encode(const std::string& text, bool add_bos, bool parse_special) const {
  std::vector<int32_t> out;
  if (add_bos && bos_ >= 0) out.push_back(bos_);
  // split out special tokens
  std::vector<std::pair<std::string, int32_t>> segs;   // id >= 0: special
  size_t i = 0, start = 0;
  if (parse_special && !specials_.empty()) {
    while (i < text.size()) {
      bool hit = false;
      if (text[i] == '<' || text[i] == '[') {
        for (auto& sp : specials_) {
          if (text.compare(i, sp.first.size(), sp.first) == 0) {
            if (i > start) segs.push_back({text.substr(start, i - start), -1});
            segs.push_back({sp.first, sp.second});
            i += sp.first.size();
            start = i;
            hit = true;
            break;
          }
        }
      }
      if (!hit) ++i;
    }
  }
  if (start < text.size()) segs.push_back({text.substr(start), -1});
  bool first_text = true;
  for (auto& s : segs) {
    if (s.second >= 0) { out.push_back(s.second); continue; }
    if (kind_ == BPE) encode_bpe_segment(s.first, out);
    else {
      std::string t = s.first;
      if (first_text && add_space_prefix_) t = " " + t;
      encode_spm_segment(t, out);
    }
    first_text = false;
  }
  return out;
}

// ------------------------------------------------------------------ decode
std::string Tokenizer::piece(int32_t id) const {
  if (id < 0 || id >= (int32_t)tokens_.size()) return "";
  const int ty = types_[id];
  if (ty == 3 || ty == 5) return "";   // control / unused
  const std::string& t = tokens_[id];
  if (kind_ == BPE) {
    if (ty == 4) return t;
    const ByteMap& bm = bytemap();
    std::string o;
    for (uint32_t u : utf8_decode(t)) {
      auto it = bm.u2b.find(u);
      if (it != bm.u2b.end()) o += (char)it->second;
      else o += utf8_encode(u);
    }
    return o;
  }
  if (ty == 6 && t.size() == 6 && t.compare(0, 3, "<0x") == 0) return std::string(1, (char)std::stoi(t.substr(3, 2), nullptr, 16));
  std::string o;
  for (size_t i = 0; i < t.size();) {
    if (t.compare(i, 3, "\xE2\x96\x81") == 0) { o += ' '; i += 3; }
    else o += t[i++];
  }
  return o;
}

std::string Tokenizer::decode(const std::vector<int32_t>& ids) const {
  std::string o;
  bool first = true;
  for (int32_t id : ids) {
    std::string p = piece(id);
    if (first && kind_ == SPM && add_space_prefix_ && !p.empty() && p[0] == ' ') p.erase(0, 1);
    if (!p.empty()) first = false;
    o += p;
  }
  return o;
}

}  // namespace mp

#include "tokenizer.h"

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
struct Range { uint32_t a, b; };
// \p{L}: letters of the major scripts (Latin, Greek, Cyrillic, Armenian, Hebrew, Arabic, Indic,
// Thai, Georgian, Hangul, Kana, CJK, fullwidth Latin, ...).
const Range kLetters[] = {
    {0x41, 0x5A}, {0x61, 0x7A}, {0xAA, 0xAA}, {0xB5, 0xB5}, {0xBA, 0xBA}, {0xC0, 0xD6}, {0xD8, 0xF6},
    {0xF8, 0x2C1}, {0x2C6, 0x2D1}, {0x2E0, 0x2E4}, {0x2EC, 0x2EC}, {0x2EE, 0x2EE}, {0x370, 0x374}, {0x376, 0x377},
    {0x37A, 0x37D}, {0x37F, 0x37F}, {0x386, 0x386}, {0x388, 0x3FF}, {0x400, 0x481}, {0x48A, 0x52F},
    {0x531, 0x556}, {0x559, 0x559}, {0x560, 0x588}, {0x5D0, 0x5EA}, {0x5EF, 0x5F2}, {0x620, 0x64A},
    {0x66E, 0x66F}, {0x671, 0x6D3}, {0x6D5, 0x6D5}, {0x6E5, 0x6E6}, {0x6EE, 0x6EF}, {0x6FA, 0x6FC},
    {0x6FF, 0x6FF}, {0x710, 0x710}, {0x712, 0x72F}, {0x74D, 0x7A5}, {0x904, 0x939}, {0x93D, 0x93D},
    {0x950, 0x950}, {0x958, 0x961}, {0x971, 0x980}, {0x985, 0x9B9}, {0xA05, 0xA39}, {0xA85, 0xAB9},
    {0xB05, 0xB39}, {0xB83, 0xBB9}, {0xC05, 0xC39}, {0xC85, 0xCB9}, {0xD05, 0xD3A}, {0xD85, 0xDC6},
    {0xE01, 0xE30}, {0xE32, 0xE33}, {0xE40, 0xE46}, {0xE81, 0xEB0}, {0xF00, 0xF00}, {0xF40, 0xF6C},
    {0x1000, 0x102A}, {0x10A0, 0x10FF}, {0x1100, 0x1248}, {0x1250, 0x135A}, {0x13A0, 0x13F5},
    {0x1401, 0x166C}, {0x1780, 0x17B3}, {0x1820, 0x1878}, {0x1E00, 0x1F15}, {0x1F18, 0x1FFC},
    {0x2071, 0x2071}, {0x207F, 0x207F}, {0x2090, 0x209C}, {0x2102, 0x2102}, {0x2107, 0x2107},
    {0x210A, 0x2113}, {0x2115, 0x2115}, {0x2119, 0x211D}, {0x2124, 0x2124}, {0x2126, 0x2126},
    {0x2128, 0x2128}, {0x212A, 0x212D}, {0x212F, 0x2139}, {0x2C00, 0x2CE4}, {0x2D00, 0x2D25},
    {0x3005, 0x3006}, {0x3031, 0x3035}, {0x303B, 0x303C}, {0x3041, 0x3096}, {0x309D, 0x309F},
    {0x30A1, 0x30FA}, {0x30FC, 0x30FF}, {0x3105, 0x312F}, {0x3131, 0x318E}, {0x31A0, 0x31BF},
    {0x31F0, 0x31FF}, {0x3400, 0x4DBF}, {0x4E00, 0x9FFF}, {0xA000, 0xA48C}, {0xA4D0, 0xA4FD},
    {0xA500, 0xA60C}, {0xA640, 0xA66E}, {0xA680, 0xA69D}, {0xA722, 0xA788}, {0xA78B, 0xA7CA},
    {0xAC00, 0xD7A3}, {0xF900, 0xFA6D}, {0xFB00, 0xFB06}, {0xFB1D, 0xFB4F}, {0xFB50, 0xFDFB},
    {0xFE70, 0xFEFC}, {0xFF21, 0xFF3A}, {0xFF41, 0xFF5A}, {0xFF66, 0xFFDC}, {0x10000, 0x1FFFF},
    {0x20000, 0x3134F},
};
// \p{N}: Nd + Nl + No of common scripts
const Range kNumbers[] = {
    {0x30, 0x39}, {0xB2, 0xB3}, {0xB9, 0xB9}, {0xBC, 0xBE}, {0x660, 0x669}, {0x6F0, 0x6F9}, {0x7C0, 0x7C9},
    {0x966, 0x96F}, {0x9E6, 0x9EF}, {0xA66, 0xA6F}, {0xAE6, 0xAEF}, {0xB66, 0xB6F}, {0xBE6, 0xBF2},
    {0xC66, 0xC6F}, {0xCE6, 0xCEF}, {0xD66, 0xD78}, {0xE50, 0xE59}, {0xED0, 0xED9}, {0xF20, 0xF33},
    {0x1040, 0x1049}, {0x1369, 0x137C}, {0x17E0, 0x17E9}, {0x1810, 0x1819}, {0x2070, 0x2070},
    {0x2074, 0x2079}, {0x2080, 0x2089}, {0x2150, 0x2182}, {0x2185, 0x2189}, {0x2460, 0x249B},
    {0x24EA, 0x24FF}, {0x2776, 0x2793}, {0x2CFD, 0x2CFD}, {0x3007, 0x3007}, {0x3021, 0x3029},
    {0x3038, 0x303A}, {0x3192, 0x3195}, {0x3220, 0x3229}, {0x3248, 0x324F}, {0x3251, 0x325F},
    {0x3280, 0x3289}, {0x32B1, 0x32BF}, {0xA620, 0xA629}, {0xFF10, 0xFF19},
};
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
bool uc_is_space(uint32_t cp) {
  return cp == 0x20 || (cp >= 0x09 && cp <= 0x0D) || cp == 0x85 || cp == 0xA0 || cp == 0x1680 ||
         (cp >= 0x2000 && cp <= 0x200A) || cp == 0x2028 || cp == 0x2029 || cp == 0x202F || cp == 0x205F ||
         cp == 0x3000;
}

// ------------------------------------------------------------------ Llama-3 pre-tokenizer
// (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+
std::vector<std::string> Tokenizer::llama3_pretokenize(const std::string& text) {
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
      while (j < i + 3 && N(j)) ++j;
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
  t.add_bos_default_ = f.get_bool("tokenizer.ggml.add_bos_token", true);
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
  for (const std::string& word : llama3_pretokenize(s)) {
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

#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace mp {

static const Json kNull;

const Json& Json::operator[](const std::string& k) const {
  if (t_ != OBJ) return kNull;
  auto it = o_.find(k);
  return it == o_.end() ? kNull : it->second;
}

// length of the valid UTF-8 sequence starting at s[i] (0 if invalid: stray continuation byte,
// overlong form, surrogate, > U+10FFFF or truncated)
static size_t utf8_len(const std::string& s, size_t i) {
  const unsigned char c = (unsigned char)s[i];
  size_t n;
  uint32_t cp;
  if (c < 0x80) return 1;
  if ((c & 0xE0) == 0xC0) { n = 2; cp = c & 0x1F; }
  else if ((c & 0xF0) == 0xE0) { n = 3; cp = c & 0x0F; }
  else if ((c & 0xF8) == 0xF0) { n = 4; cp = c & 0x07; }
  else return 0;
  if (i + n > s.size()) return 0;
  for (size_t k = 1; k < n; ++k) {
    const unsigned char d = (unsigned char)s[i + k];
    if ((d & 0xC0) != 0x80) return 0;
    cp = (cp << 6) | (d & 0x3F);
  }
  if ((n == 2 && cp < 0x80) || (n == 3 && cp < 0x800) || (n == 4 && cp < 0x10000) || cp > 0x10FFFF ||
      (cp >= 0xD800 && cp <= 0xDFFF))
    return 0;
  return n;
}

// JSON string body; bytes that are not valid UTF-8 (a token piece cut inside a character, a
// binary prompt) become U+FFFD, like the reference's lossy decoding (main.rs:68,88)
std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    if (c >= 0x80) {
      const size_t n = utf8_len(s, i);
      if (n == 0) { o += "\xEF\xBF\xBD"; ++i; }
      else { o.append(s, i, n); i += n; }
      continue;
    }
    ++i;
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof(buf), "\\u%04x", c);
          o += buf;
        } else {
          o += (char)c;
        }
    }
  }
  return o;
}

std::string Json::dump() const {
  switch (t_) {
    case NUL: return "null";
    case BOOL: return b_ ? "true" : "false";
    case NUM: {
      if (std::isfinite(n_) && n_ == std::floor(n_) && std::fabs(n_) < 1e15) {
        char buf[32];
        snprintf(buf, sizeof(buf), "%lld", (long long)n_);
        return buf;
      }
      char buf[64];
      snprintf(buf, sizeof(buf), "%.17g", n_);
      return buf;
    }
    case STR: return "\"" + json_escape(s_) + "\"";
    case ARR: {
      std::string o = "[";
      for (size_t i = 0; i < a_.size(); ++i) { if (i) o += ","; o += a_[i].dump(); }
      return o + "]";
    }
    case OBJ: {
      std::string o = "{";
      bool first = true;
      for (auto& kv : o_) {
        if (!first) o += ",";
        first = false;
        o += "\"" + json_escape(kv.first) + "\":" + kv.second.dump();
      }
      return o + "}";
    }
  }
  return "null";
}

namespace {
struct Parser {
  const char* p;
  const char* e;
  int depth = 0;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e - p) >= n && !memcmp(p, s, n)) { p += n; return true; }
    return false;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  }
  uint32_t hex4() {
    if (e - p < 4) fail("bad \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (p >= e || *p != '"') fail("expected string");
    ++p;
    std::string o;
    while (true) {
      if (p >= e) fail("unterminated string");
      char c = *p++;
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control char in string");
      if (c != '\\') { o += c; continue; }
      if (p >= e) fail("bad escape");
      char x = *p++;
      switch (x) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo = hex4();
            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else { put_utf8(o, 0xFFFD); cp = lo; }
          }
          put_utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return o;
  }
  Json val() {
    if (++depth > 256) fail("nesting too deep");
    ws();
    if (p >= e) fail("unexpected end");
    Json r;
    char c = *p;
    if (c == '{') {
      ++p;
      r = Json::object();
      ws();
      if (p < e && *p == '}') { ++p; --depth; return r; }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (p >= e || *p != ':') fail("expected ':'");
        ++p;
        r[k] = val();
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; break; }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      ++p;
      r = Json::array();
      ws();
      if (p < e && *p == ']') { ++p; --depth; return r; }
      while (true) {
        r.push(val());
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; break; }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      r = Json(str());
    } else if (lit("true")) {
      r = Json(true);
    } else if (lit("false")) {
      r = Json(false);
    } else if (lit("null")) {
      r = Json();
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      char* end = nullptr;
      std::string tmp(p, std::min<size_t>(e - p, 64));
      double d = strtod(tmp.c_str(), &end);
      if (end == tmp.c_str()) fail("bad number");
      p += end - tmp.c_str();
      r = Json(d);
    } else {
      fail("unexpected character");
    }
    --depth;
    return r;
  }
};
}  // namespace

Json Json::parse(const std::string& s) {
  Parser ps{s.data(), s.data() + s.size()};
  Json v = ps.val();
  ps.ws();
  if (ps.p != ps.e) throw std::runtime_error("json: trailing characters");
  return v;
}

}  // namespace mp

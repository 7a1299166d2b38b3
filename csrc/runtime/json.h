// Minimal JSON value / parser / writer (no dependencies).  Used for engine configs passed over
// the C API and for the orchestrator's HTTP bodies (`{"prompt": ...}`, SSE `{"msg_type","content"}`).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace mp {

class Json {
 public:
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ };
  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : t_(BOOL), b_(b) {}
  Json(double d) : t_(NUM), n_(d) {}
  Json(int i) : t_(NUM), n_(i) {}
  Json(int64_t i) : t_(NUM), n_((double)i) {}
  Json(const char* s) : t_(STR), s_(s) {}
  Json(std::string s) : t_(STR), s_(std::move(s)) {}
  static Json array() { Json j; j.t_ = ARR; return j; }
  static Json object() { Json j; j.t_ = OBJ; return j; }

  Type type() const { return t_; }
  bool is_null() const { return t_ == NUL; }
  bool is_obj() const { return t_ == OBJ; }
  bool is_str() const { return t_ == STR; }
  bool is_num() const { return t_ == NUM; }
  bool is_arr() const { return t_ == ARR; }
  bool is_bool() const { return t_ == BOOL; }

  double num() const { if (t_ != NUM) throw std::runtime_error("json: not a number"); return n_; }
  bool boolean() const { if (t_ != BOOL) throw std::runtime_error("json: not a bool"); return b_; }
  const std::string& str() const { if (t_ != STR) throw std::runtime_error("json: not a string"); return s_; }
  const std::vector<Json>& arr() const { return a_; }
  std::vector<Json>& arr() { return a_; }
  const std::map<std::string, Json>& obj() const { return o_; }

  bool has(const std::string& k) const { return t_ == OBJ && o_.count(k); }
  const Json& operator[](const std::string& k) const;
  Json& operator[](const std::string& k) { t_ = OBJ; return o_[k]; }
  void push(Json v) { t_ = ARR; a_.push_back(std::move(v)); }
  void erase(const std::string& k) { o_.erase(k); }

  double get_num(const std::string& k, double d) const { return has(k) && o_.at(k).is_num() ? o_.at(k).n_ : d; }
  int get_int(const std::string& k, int d) const { return (int)get_num(k, d); }
  bool get_bool(const std::string& k, bool d) const { return has(k) && o_.at(k).is_bool() ? o_.at(k).b_ : d; }
  std::string get_str(const std::string& k, const std::string& d) const {
    return has(k) && o_.at(k).is_str() ? o_.at(k).s_ : d;
  }

  std::string dump() const;
  static Json parse(const std::string& s);   // throws std::runtime_error on malformed input

 private:
  Type t_ = NUL;
  bool b_ = false;
  double n_ = 0;
  std::string s_;
  std::vector<Json> a_;
  std::map<std::string, Json> o_;
};

std::string json_escape(const std::string& s);

}  // namespace mp

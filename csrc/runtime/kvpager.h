// Paged KV cache bookkeeping (the reference's llama.cpp gives every sequence a fixed
// `-c 2048` KV, /root/reference/orchestrator/src/main.rs:45-46).
//
// Every stage owns one pool of fixed 64-token pages per layer (same page ids in every layer), sized
// from HBM; a sequence slot maps its positions to pages through a block table row
// [slot][max_ctx / 64].  Pages are granted when a sequence is admitted / prefilled and whenever a
// decode call would carry it into a new page, and go back to the free list on release(), so the
// pool only has to hold the tokens that are actually live (sum over slots), not n_slots x max_ctx.
// Unmapped entries point at a dedicated TRASH page (id = n_pages): idle rows of a micro-batch still
// compute and append K/V; their writes land there and are never read back as live data.
//
// The allocator is deterministic (LIFO free list seeded 0, 1, 2, ...), so every rank of a
// multi-process pipeline that replays the same engine calls derives the same tables without any
// exchange.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace mp {

class KvPager {
 public:
  static constexpr int kPage = 64;

  void init(int n_slots, int max_pages, int n_pages) {
    if (n_slots < 1 || max_pages < 1 || n_pages < 1) throw std::runtime_error("KvPager: bad geometry");
    n_slots_ = n_slots;
    max_pages_ = max_pages;
    n_pages_ = n_pages;
    table_.assign((size_t)n_slots * max_pages, n_pages);   // everything -> TRASH
    owned_.assign(n_slots, 0);
    free_.clear();
    for (int p = n_pages - 1; p >= 0; --p) free_.push_back(p);   // pop_back() yields 0, 1, 2, ...
    dirty_ = true;
  }

  // make `slot` cover positions [0, n_tokens); all-or-nothing: false (nothing granted) when the
  // pool cannot supply the missing pages
  bool ensure(int slot, int n_tokens) {
    check(slot);
    const int need = (n_tokens + kPage - 1) / kPage;
    if (need > max_pages_) throw std::runtime_error("KvPager: " + std::to_string(n_tokens) + " tokens exceed max_ctx");
    const int miss = need - owned_[slot];
    if (miss <= 0) return true;
    if (miss > (int)free_.size()) return false;
    for (int k = owned_[slot]; k < need; ++k) {
      table_[(size_t)slot * max_pages_ + k] = free_.back();
      free_.pop_back();
    }
    owned_[slot] = need;
    dirty_ = true;
    return true;
  }

  void release(int slot) {
    check(slot);
    for (int k = owned_[slot] - 1; k >= 0; --k) {
      int32_t& e = table_[(size_t)slot * max_pages_ + k];
      free_.push_back(e);
      e = n_pages_;
    }
    if (owned_[slot]) dirty_ = true;
    owned_[slot] = 0;
  }

  int owned(int slot) const { check(slot); return owned_[slot]; }
  int free_pages() const { return (int)free_.size(); }
  int n_pages() const { return n_pages_; }
  int max_pages() const { return max_pages_; }
  int trash() const { return n_pages_; }
  const std::vector<int32_t>& table() const { return table_; }
  bool dirty() const { return dirty_; }
  void clean() { dirty_ = false; }

 private:
  void check(int slot) const {
    if (slot < 0 || slot >= n_slots_) throw std::runtime_error("KvPager: bad slot " + std::to_string(slot));
  }
  int n_slots_ = 0, max_pages_ = 0, n_pages_ = 0;
  std::vector<int32_t> table_, free_;
  std::vector<int> owned_;
  bool dirty_ = false;
};

}  // namespace mp

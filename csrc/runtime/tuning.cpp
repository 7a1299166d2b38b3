#include "tuning.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace mp {

namespace {

struct KnobDef {
  const char* name;   // MIPIPE_<name>
  int dflt, lo, hi;   // valid range [lo, hi]
  bool (*valid)(int); // extra check (nullptr: range only)
};

bool ns_ok(int v) { return v == 2 || v == 3 || v == 4; }
bool nw_ok(int v) { return v == 4 || v == 8; }
bool g_ok(int v) { return v == 0 || v == 1 || v == 2 || v == 4 || v == 8; }
bool bm_ok(int v) { return v == 0 || v == 96 || v == 128 || v == 256; }
bool nw4_ok(int v) { return v == 0 || v == 4 || v == 7 || v == 8; }

const KnobDef kDefs[KNOB_COUNT] = {
    {"ATTN_PF_MAXWG", 512, 0, 1 << 30, nullptr},   // r7v: mb256 np 61.3 vs PF 65.3 us/layer
    {"ATTN_WG_TARGET", 256, 1, 1 << 20, nullptr},
    {"ATTN_NW8_MAXWG", 0, 0, 1 << 20, nullptr},   // r8n: 8 waves 10.97 vs 10.03 us (8B mb1): off
    {"GEMM2_SPLIT_WG", 256, 1, 1 << 20, nullptr},
    {"GEMVS_NS", 2, 2, 4, ns_ok},
    {"GEMVS_S", 64, 1, 1 << 20, nullptr},
    {"GEMVS2", 1, 0, 1, nullptr},
    {"GEMVS_MINWG", 256, 1, 1 << 20, nullptr},
    {"GEMVS_G", 0, 0, 8, g_ok},
    {"GEMVS_SPLIT", 0, 0, 1 << 16, nullptr},
    {"GEMVS_RPF", 1, 0, 1, nullptr},
    {"GEMVS_DOT", 1, 0, 1, nullptr},
    {"MOE_V", 2, 1, 2, nullptr},
    {"GEMV_NW", 8, 4, 8, nw_ok},
    {"GEMV2_TW", 0, 0, 2, nullptr},
    {"ATTN_WAVE", 2, 0, 2, nullptr},
    {"ATTN_WAVE_MIN", 512, 1, 1 << 30, nullptr},   // r10ac: mb64 at 8 kv heads (512 items) +2.5-3 %, mb32 (256) -2.3 %
    {"ATTN_PRE", 1, 0, 1, nullptr},
    {"GEMM4_NW", 0, 0, 8, nw4_ok},
    {"GEMM4_SPREAD", 0, 0, 2, nullptr},
    {"GEMM4_WNT", 0, 0, 2, nullptr},
    {"GEMM4_MOE64", 2, 0, 3, nullptr},   // 1: 64-row expert tiles (r8i: slower); 2: 96-row tiles at <= 80 rows per expert (r12i: Mixtral mb256 10262 -> 13662), down split 4 over K; 3: the same unsplit
    {"GEMM3_BM", 0, 0, 256, bm_ok},
    {"GEMM3_BN", 0, 0, 256, bm_ok},
    {"GEMM3_SPLIT", 0, 0, 1 << 10, nullptr},
    {"GEMM4_TW4", 1, 0, 6, nullptr},   // r10u: 70B mb256 5756 -> 5792 (gate/up only); all tiles: 5570 (r10t)
    {"GEMV_SPLIT_WAVES", 2048, 64, 1 << 20, nullptr},
    {"GEMV_SPLIT_MINSB", 4, 1, 64, nullptr},
#ifdef MIPIPE_TIMING_PROBES
#include "timing_probes.inc"
#endif
};

std::atomic<int> g_vals[KNOB_COUNT];
std::once_flag g_once;

bool ok(const KnobDef& d, int v) { return v >= d.lo && v <= d.hi && (!d.valid || d.valid(v)); }

// the knob's start value: its MIPIPE_* environment variable when valid, else the default
int initial_value(int i) {
  const KnobDef& d = kDefs[i];
  int v = d.dflt;
  const std::string env = std::string("MIPIPE_") + d.name;
  if (const char* e = std::getenv(env.c_str())) {
    char* end = nullptr;
    const long x = std::strtol(e, &end, 10);
    if (end != e && *end == 0 && ok(d, (int)x)) v = (int)x;
    else std::fprintf(stderr, "mipipe: ignoring %s=%s (invalid value; using %d)\n", env.c_str(), e, d.dflt);
  }
  return v;
}

void init() {
  for (int i = 0; i < KNOB_COUNT; ++i) g_vals[i].store(initial_value(i), std::memory_order_relaxed);
}

int find(const char* name) {
  for (int i = 0; i < KNOB_COUNT; ++i)
    if (std::strcmp(kDefs[i].name, name) == 0) return i;
  throw std::invalid_argument(std::string("set_knob: unknown knob ") + name);
}

}  // namespace

int knob(Knob k) {
  std::call_once(g_once, init);
  return g_vals[k].load(std::memory_order_relaxed);
}

void set_knob(const char* name, int value) {
  std::call_once(g_once, init);
  const int i = find(name);
  if (!ok(kDefs[i], value)) throw std::invalid_argument(std::string("set_knob: value out of range for ") + name);
  g_vals[i].store(value, std::memory_order_relaxed);
}

void reset_knob(const char* name) {
  std::call_once(g_once, init);
  const int i = find(name);
  g_vals[i].store(initial_value(i), std::memory_order_relaxed);
}

}  // namespace mp

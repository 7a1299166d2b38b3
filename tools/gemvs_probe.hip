// Timing probes of the single-stream GEMV (gemvs.hip) on the Llama-3-8B decode shapes, outside the
// library (one-off tool): this file compiles gemvs.hip and the knob registry with the timing-probe
// knobs enabled (MIPIPE_TIMING_PROBES; the shipped libmipipe.so has none), and times chains of 40
// graph-captured launches over cold weight copies, like tools/stream_probe.hip, with parts of the
// kernel skipped (knob GEMVS_PROBE: 1 no dequant / MFMA, 2 no x prologue, 4 plain epilogue store).
// Results of the probe variants are wrong by construction; only their times are used.
//   hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics -Icsrc/runtime tools/gemvs_probe.hip -o /tmp/gp && /tmp/gp
#define MIPIPE_TIMING_PROBES 1
#include "../csrc/kernels/gemvs.hip"
#include "../csrc/runtime/tuning.cpp"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Shape { const char* name; int N, K, epi, pt; bool norm; };

int main() {
  using namespace mp;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const Shape shapes[] = {
      {"o      Q4_K", 4096, 4096, EPI_ATOMIC, P_Q4_K, false},
      {"qkv    Q4_K", 6144, 4096, EPI_STORE, P_Q4_K, true},
      {"gateup Q4_K", 28672, 4096, EPI_SWIGLU, P_Q4_K, true},
      {"down   Q4_K", 4096, 14336, EPI_ATOMIC, P_Q4_K, false},
      {"down   Q6_K", 4096, 14336, EPI_ATOMIC, P_Q6_K, false},
  };
  const size_t pool = 2ull << 30;
  uint8_t* wbuf;
  CK(hipMalloc(&wbuf, pool));
  // random weight bytes (timing only), small enough scales not to matter
  {
    std::vector<uint32_t> h(1 << 22);
    uint64_t x = 88172645463325252ull;
    for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x & 0x3BFF3BFFu; }
    for (size_t off = 0; off < pool; off += h.size() * 4)
      CK(hipMemcpy(wbuf + off, h.data(), std::min(pool - off, h.size() * 4), hipMemcpyHostToDevice));
  }
  float *xf, *gamma, *y;
  f16 *xh, *hbuf;
  CK(hipMalloc(&xf, 16384 * 4));
  CK(hipMalloc(&gamma, 16384 * 4));
  CK(hipMalloc(&y, 65536 * 4));
  CK(hipMalloc(&xh, 16384 * 2));
  CK(hipMalloc(&hbuf, 32768 * 2));
  {
    std::vector<float> ones(16384, 1.f);
    CK(hipMemcpy(xf, ones.data(), 16384 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(gamma, ones.data(), 16384 * 4, hipMemcpyHostToDevice));
    CK(hipMemset(xh, 0, 16384 * 2));
  }
  const int probes[] = {0, 1, 2, 3, 4, 7};
  for (const Shape& s : shapes) {
    const int ntiles = s.N / 16, nsb = s.K / 256;
    const size_t bytes = (size_t)ntiles * nsb * chunk_bytes(s.pt);
    const int copies = (int)std::min<size_t>(40, pool / bytes);
    printf("%s  %6.1f MB:", s.name, bytes / 1e6);
    for (int pb : probes) {
      set_knob("GEMVS_PROBE", pb);
      hipGraph_t g;
      hipGraphExec_t ex;
      const int n = 40;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      for (int i = 0; i < n; ++i) {
        GemvParams p{};
        p.W = wbuf + (size_t)(i % copies) * bytes;
        p.M = 1; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = s.epi == EPI_SWIGLU ? s.N / 2 : s.N;
        p.Y = y; p.ldy = 65536; p.H = hbuf; p.ldh = 32768;
        if (s.norm) { p.Xf = xf; p.ldxf = s.K; p.gamma = gamma; p.eps = 1e-5f; p.d_norm = s.K; }
        else { p.X = xh; p.ldx = s.K; }
        launch_gemvs(s.pt, s.epi, p, false, st);
      }
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(a, st));
        CK(hipGraphLaunch(ex, st));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < best) best = ms;
      }
      CK(hipGraphExecDestroy(ex));
      CK(hipGraphDestroy(g));
      printf("  p%d %6.2f", pb, best * 1e3f / n);
      fflush(stdout);
    }
    printf("  us\n");
  }
  return 0;
}

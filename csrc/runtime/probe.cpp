// Device speed probe (probe.h): a few milliseconds of measurement per device at engine start.
#include "probe.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "kernels_api.h"
#include "log.h"
#include "qtypes.h"

#define PR_OK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("probe: ") + hipGetErrorString(e_)); \
  } while (0)

namespace mp {

void launch_init_packed(uint8_t* W, size_t nbytes, int pt, float scale, uint64_t seed, hipStream_t st);
void launch_stream_read(const void* buf, size_t bytes, float* out, hipStream_t st);

DeviceProfile probe_device(int device) {
  int prev = 0;
  PR_OK(hipGetDevice(&prev));
  PR_OK(hipSetDevice(device));
  DeviceProfile dp;
  hipStream_t st;
  PR_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  PR_OK(hipEventCreate(&e0));
  PR_OK(hipEventCreate(&e1));
  auto timed = [&](int reps, const auto& body) {
    body(0);   // warm (first touch, code load)
    PR_OK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) body(i + 1);
    PR_OK(hipEventRecord(e1, st));
    PR_OK(hipEventSynchronize(e1));
    float ms = 0;
    PR_OK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  // 1. HBM streaming read: 1 GiB (>> the 256 MiB Infinity Cache)
  {
    const size_t bytes = (size_t)1 << 30;
    void* buf = nullptr;
    float* out = nullptr;
    PR_OK(hipMalloc(&buf, bytes));
    PR_OK(hipMalloc((void**)&out, 4096 * sizeof(float)));
    PR_OK(hipMemsetAsync(buf, 0, bytes, st));
    const float ms = timed(4, [&](int) { launch_stream_read(buf, bytes, out, st); });
    dp.hbm_read_gbps = bytes / (ms * 1e-3) / 1e9;
    PR_OK(hipFree(buf));
    PR_OK(hipFree(out));
  }
  // 2. decode GEMV: Q4_K 57344 x 8192 (the 70B gate/up, 264 MB), M = 1, copies cycled so the
  //    weights come from HBM as in a real decode step
  {
    const int N = 57344, K = 8192, copies = 4;
    const PackedDims d = packed_dims(P_Q4_K, N, K);
    std::vector<uint8_t*> W(copies, nullptr);
    for (auto& w : W) {
      PR_OK(hipMalloc((void**)&w, d.bytes));
      launch_init_packed(w, d.bytes, P_Q4_K, 1.0f / 90.5f, 7, st);
    }
    f16* x = nullptr;
    f16* h = nullptr;
    PR_OK(hipMalloc((void**)&x, (size_t)d.nsb * 256 * 2));
    PR_OK(hipMalloc((void**)&h, (size_t)N / 2 * 2));
    PR_OK(hipMemsetAsync(x, 0, (size_t)d.nsb * 256 * 2, st));
    GemvParams p{};
    p.X = x; p.ldx = (int)(d.nsb * 256); p.M = 1; p.H = h; p.ldh = N / 2;
    p.ntiles = (int)d.ntiles; p.nsb = (int)d.nsb; p.n_valid = N / 2;
    const float ms = timed(8, [&](int i) {
      p.W = W[i % copies];
      launch_gemv(P_Q4_K, EPI_SWIGLU, p, 1, st);
    });
    dp.gemv_gbps = d.bytes / (ms * 1e-3) / 1e9;
    for (auto w : W) PR_OK(hipFree(w));
    PR_OK(hipFree(x));
    PR_OK(hipFree(h));
  }
  PR_OK(hipEventDestroy(e0));
  PR_OK(hipEventDestroy(e1));
  PR_OK(hipStreamDestroy(st));
  PR_OK(hipSetDevice(prev));
  MP_LOGI("device probe: GPU %d HBM read %.0f GB/s, Q4_K decode GEMV %.0f GB/s", device, dp.hbm_read_gbps,
          dp.gemv_gbps);
  return dp;
}

DeviceProfile probe_host() {
  const size_t bytes = (size_t)256 << 20;
  std::vector<uint8_t> a(bytes, 1), b(bytes, 0);
  std::memcpy(b.data(), a.data(), bytes);   // fault in
  const auto t0 = std::chrono::steady_clock::now();
  const int reps = 3;
  for (int i = 0; i < reps; ++i) std::memcpy(b.data(), a.data(), bytes);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  DeviceProfile dp;
  dp.hbm_read_gbps = reps * (double)bytes / std::max(s, 1e-9) / 1e9;
  MP_LOGI("device probe: host memcpy %.1f GB/s", dp.hbm_read_gbps);
  return dp;
}

}  // namespace mp

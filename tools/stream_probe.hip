// Calibration probe for the single-stream decode GEMVs (one-off tool, not part of the library):
// what does a dependent chain of kernels that each stream B bytes of cold weights cost on this chip,
// by grid size, loads in flight per lane and cache policy?  Every launch reads its own copy of the
// bytes (copies cycled over > 1 GB, so the 256 MiB Infinity Cache cannot serve them); 40 launches
// are captured in one hipGraph and replayed, so the per-launch time includes the kernel boundary,
// exactly like a captured decode step.
//   hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o /tmp/sp && /tmp/sp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void empty_kernel(unsigned* sink) {
  if (threadIdx.x == 1023) sink[0] = 1;
}

// each wave streams a contiguous slice [w * per, (w + 1) * per) of 1 KiB wave-instructions, D of them
// in flight (a register ring), NT: non-temporal loads
template <int D, bool NT>
__global__ __launch_bounds__(512) void stream_kernel(const u32x4* __restrict__ buf, size_t n16, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const size_t ninst = n16 / 64;
  const size_t per = (ninst + nw - 1) / nw;
  const size_t i0 = w * per, i1 = i0 + per < ninst ? i0 + per : ninst;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 ring[D];
#pragma unroll
  for (int s = 0; s < D; ++s) {
    const size_t i = i0 + s;
    const u32x4* p = buf + i * 64 + lane;
    if (i < i1) ring[s] = NT ? __builtin_nontemporal_load(p) : *p;
    else ring[s] = u32x4{0, 0, 0, 0};
  }
  for (size_t i = i0; i < i1; i += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      acc ^= ring[s];
      const size_t j = i + D + s;
      const u32x4* p = buf + j * 64 + lane;
      if (j < i1) ring[s] = NT ? __builtin_nontemporal_load(p) : *p;
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[1] = 1;
}

template <int D, bool NT>
float time_stream(const char* base, size_t bytes, int copies, int grid, int threads, unsigned* sink, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ex;
  const int n = 40;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
  for (int i = 0; i < n; ++i)
    hipLaunchKernelGGL((stream_kernel<D, NT>), dim3(grid), dim3(threads), 0, st,
                       reinterpret_cast<const u32x4*>(base + (size_t)(i % copies) * bytes), bytes / 16, sink);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
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
  return best * 1e3f / n;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  unsigned* sink;
  CK(hipMalloc(&sink, 64));
  // boundary: a graph of 40 empty 256-workgroup kernels
  {
    hipGraph_t g;
    hipGraphExec_t ex;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < 40; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(512), 0, st, sink);
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
    printf("empty kernel in a graph: %.2f us per launch\n", best * 1e3f / 40);
  }
  const size_t total = 3ull << 30;
  char* buf;
  CK(hipMalloc(&buf, total));
  CK(hipMemset(buf, 1, total));
  CK(hipDeviceSynchronize());
  // the 8B decode shapes' Q4_K bytes: o 9.4 MB, qkv 15.2 MB, down 33 MB (Q6_K 48 MB), gate/up 66 MB
  const size_t sizes[] = {9437184, 15204352, 33030144, 48168960, 66060288};
  const char* names[] = {"o", "qkv", "down", "down6", "gateup"};
  for (int si = 0; si < 5; ++si) {
    const size_t bytes = sizes[si];
    const int copies = (int)std::min<size_t>(40, total / bytes);
    for (int threads : {256, 512}) {
      for (int grid : {256, 512, 1024, 2048}) {
        float t2 = time_stream<2, true>(buf, bytes, copies, grid, threads, sink, st);
        float t4 = time_stream<4, true>(buf, bytes, copies, grid, threads, sink, st);
        float t8 = time_stream<8, true>(buf, bytes, copies, grid, threads, sink, st);
        float t4p = time_stream<4, false>(buf, bytes, copies, grid, threads, sink, st);
        printf("%-7s %6.1f MB  grid %4d x %3d thr: D2 nt %6.2f us  D4 nt %6.2f  D8 nt %6.2f  D4 plain %6.2f   (best %.2f TB/s)\n",
               names[si], bytes / 1e6, grid, threads, t2, t4, t8, t4p,
               bytes / 1e6 / std::min(std::min(t2, t4), std::min(t8, t4p)));
        fflush(stdout);
      }
    }
  }
  return 0;
}

// HBM read bandwidth of the wave-instruction footprints the decode attention uses (one-off
// measurement tool, not part of the library):
//   pattern 0: contiguous   -- 64 lanes x 16 B = one 1 KiB run per instruction
//   pattern 1: half lines   -- 16 rows x 64 B (rows 256 B apart, the other 64 B of each 128-B line
//                              read by the next instruction): the K fragment loads of attention.hip
//   pattern 2: full lines   -- 8 rows x 128 B (rows 256 B apart): the same bytes, whole lines
// Every wave streams its own 64 KiB region (like one (token, kv head) item's K pages), 2 KiB per
// step (2 instructions in flight per step, 4 steps unrolled); 2048 waves (256 CUs x 8) cover 128 MiB
// per pass; the buffer is 4 GiB so each pass reads cold data.  All three read the same bytes.
//   hipcc --offload-arch=gfx950 -O3 tools/load_pattern_bench.hip -o /tmp/lpb && /tmp/lpb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int PAT>
__global__ __launch_bounds__(256) void read_kernel(const char* __restrict__ buf, size_t region, size_t pass_off,
                                                   unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const char* base = buf + pass_off + wave * region;
  u32x4 acc = {0, 0, 0, 0};
  // one 8 KiB step = 32 rows x 256 B (32 keys of one kv head's K page), 8 instructions of 1 KiB
  for (size_t off = 0; off < region; off += 8192) {
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      size_t o;
      if (PAT == 0) o = off + i * 1024 + lane * 16;
      else if (PAT == 1) o = off + (16 * (i >> 2) + (lane & 15)) * 256 + 64 * (i & 3) + 16 * (lane >> 4);
      else o = off + (8 * (i >> 1) + (lane >> 3)) * 256 + 128 * (i & 1) + 16 * (lane & 7);
      v[i] = *reinterpret_cast<const u32x4*>(base + o);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= v[i];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

int main() {
  const size_t total = 4ull << 30, region = 64 << 10;
  const int waves = 2048, blocks = waves / 4;
  const size_t pass = (size_t)waves * region;
  char* buf;
  unsigned* sink;
  if (hipMalloc(&buf, total) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(buf, 1, total);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[3] = {"contiguous 1 KiB", "16 rows x 64 B", "8 rows x 128 B"};
  for (int pat = 0; pat < 3; ++pat) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      for (size_t p = 0; p + pass <= total; p += pass) {
        if (pat == 0) hipLaunchKernelGGL(read_kernel<0>, dim3(blocks), dim3(256), 0, 0, buf, region, p, sink);
        else if (pat == 1) hipLaunchKernelGGL(read_kernel<1>, dim3(blocks), dim3(256), 0, 0, buf, region, p, sink);
        else hipLaunchKernelGGL(read_kernel<2>, dim3(blocks), dim3(256), 0, 0, buf, region, p, sink);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("pattern %d (%s): %.1f GB/s\n", pat, names[pat], (double)(total / pass * pass) / (best * 1e-3) / 1e9);
  }
  hipFree(buf);
  hipFree(sink);
  return 0;
}

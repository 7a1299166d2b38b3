// Kernel-launch tuning knobs: one registry instead of per-call-site `static getenv` lambdas.
//
// Every knob starts from its default, is overridden once from its MIPIPE_* environment variable
// (read on first use, invalid values rejected with a warning), and can be changed at any time with
// set_knob() (C API mp_set_knob), so an in-process A/B run measures the value it names instead of
// whatever the first launch froze.  Reads are a relaxed atomic load: cheap on launch paths.
#pragma once

namespace mp {

enum Knob : int {
  KNOB_ATTN_PF_MAXWG = 0,   // decode attention: next-chunk prefetch variant while M * Hkv <= this
  KNOB_ATTN_WG_TARGET,      // decode attention: workgroup target of the automatic KV split
  KNOB_ATTN_NW8_MAXWG,      // decode attention: 8-wave workgroups while M * Hkv <= this (one split; 0 off)
  KNOB_GEMM2_SPLIT_WG,      // gemm3 / gemm4: workgroup target of the split-K (name kept from the retired gemm2)
  KNOB_GEMVS_NS,            // gemvs: weight super-blocks in flight per wave (2, 3 or 4)
  KNOB_GEMVS_S,             // gemvs: super-blocks per wave target of the work split
  KNOB_GEMVS2,              // gemvs: q+k | v of mixed-type layers in one launch (0 / 1)
  KNOB_GEMVS_MINWG,         // gemvs: fewest workgroups before halving the tiles per workgroup
  KNOB_GEMVS_G,             // gemvs: force tiles per workgroup (0 auto, 1, 2, 4, 8)
  KNOB_GEMVS_SPLIT,         // gemvs: force the k-split over the grid (0 auto)
  KNOB_GEMVS_RPF,           // gemvs: single-owner ATOMIC epilogue from a residual loaded at kernel start (0 / 1)
  KNOB_GEMVS_DOT,           // gemvs: one row on the v_dot2 form (Q4_K / Q5_K / Q6_K / Q8_0; 0 = MFMA form)
  KNOB_MOE_V,               // MoE GEMV version (1 | 2)
  KNOB_GEMV_NW,             // decode GEMV: waves per workgroup (4 | 8)
  KNOB_GEMV2_TW,            // decode GEMV: tiles per wave at M > 32 (0 auto, 1, 2)
  KNOB_ATTN_WAVE,           // decode attention: the wave-per-item kernel (0 off, 1 on, 2 auto)
  KNOB_ATTN_WAVE_MIN,       // auto: (token, kv head, split) items at or above which it is taken
  KNOB_ATTN_PRE,            // single stream: RoPE + KV append in the qkv GEMV's epilogue (0 / 1)
  KNOB_GEMM4_NW,            // gemm4: compute waves per workgroup of unsplit launches (0 auto, 7, 8; 4 = 128-row
                            // tiles of 4 waves, two workgroups per CU, split-K included)
  KNOB_GEMM4_SPREAD,        // gemm4: LDS-DMA issue after the stage barrier (0 burst, 1 spread over MFMA steps, 2 spread + waves 4-7 two steps later)
  KNOB_GEMM4_WNT,           // gemm4: non-temporal LDS-DMA of the weights (0 auto: one row block per column group, 1 on, 2 off)
  KNOB_GEMM4_MOE64,         // gemm4 MoE mode: 1 = 64-row tiles at <= 64 mean rows per expert, 2 (default) = 96-row
                            // tiles at <= 80 (two workgroups per CU), 0 = 128-row tiles
  KNOB_GEMM3_BM,            // gemm3 / gemm4: force rows per workgroup (0 auto, 128, 256; 96 gemm4 only); A/B runs only
  KNOB_GEMM3_BN,            // gemm3: force columns per workgroup (0 auto, 128, 256)
  KNOB_GEMM3_SPLIT,         // gemm3: force the split-K factor (0 auto)
  KNOB_GEMM4_TW4,           // gemm4 dense: 4 waves x 64 columns (two MFMAs per A fragment) instead of 8 x 32
                            // (0 off, 1 the 256-row tiles only, 2 also the 128-row tiles, 3 = 1 + the 128-row MoE tiles;
                            // 8 / 7 waves x 64 columns on 128-row tiles: 4 every shape, 5 gate/up only, 6 split-K only)
  KNOB_GEMV_SPLIT_WAVES,    // decode GEMV (M > 32): tile-wave target of the automatic split-K
  KNOB_GEMV_SPLIT_MINSB,    // decode GEMV: fewest super-blocks per split
#ifdef MIPIPE_TIMING_PROBES
  // timing probes that skip work (wrong results): only in a `make PROBES=1` build, never in the
  // default library, so no environment variable can corrupt a serving or bench run
  KNOB_GEMM3_PROBE,         // gemm3 timing probes (Q4_K SwiGLU 256x256 only; 0 = the real kernel)
  KNOB_ATTN_PROBE,          // decode attention timing probes (1: no V append, 2: no K append; 0 = real)
  KNOB_GEMM4_PROBE,         // gemm4 timing probes (Q4_K, dense): bit 0 no dequant, 1 no MFMA, 2 no LDS-DMA
  KNOB_GEMVS_PROBE,         // gemvs timing probes: bit 0 no dequant / MFMA, 1 no x prologue, 2 plain epilogue store
#endif
  KNOB_COUNT
};

int knob(Knob k);
// name is the knob's environment variable without the MIPIPE_ prefix (e.g. "GEMVS_NS");
// throws std::invalid_argument for an unknown name or a value outside the knob's range
void set_knob(const char* name, int value);
// back to the value the process started with (its environment variable, else the default)
void reset_knob(const char* name);

}  // namespace mp

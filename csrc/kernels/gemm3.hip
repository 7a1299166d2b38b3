// Dequant GEMM v3 (M > 64: wide decode micro-batches and prompt chunks).
//
// Y[M][N] (+)= X[M][K] W[N][K]^T with W in the T16 packed quant layout (csrc/runtime/qtypes.h).
//
// Workgroup tile BM x BN (BM = 128 | 256 rows, BN = 128 | 256 columns), 8 waves, K in stages of
// 64.  Every wave OWNS TW = BN / 128 weight tiles (16 columns each) for all BM rows: it dequantizes
// each weight element of its tiles exactly once per workgroup, straight into MFMA B fragments in
// registers (no f16 weight image in LDS, no ds_write, no duplicated dequant), and runs
// v_mfma_f32_16x16x32_f16 against the A (x) fragments that all 8 waves share from LDS.
//
//   stage s:  X rows [BM][64]      --global_load_lds-->  A[s % NB]  (f16, swizzled, shared)
//             each wave's raw quant --global_load_lds-->  R[s % NB][wave]  (its TW tiles' bytes)
//
// Everything reaches LDS by LDS-DMA (global_load_lds), so the load pipeline is NB = 3 stages deep
// with a COUNTED s_waitcnt vmcnt(loads of one stage) before each raw s_barrier: stage s+2 stays in
// flight while stage s computes (the round-1/2 GEMMs and the first v3 drained every load at every
// barrier: profiles/r6c_gemm3_probes.txt -- at one stage in flight the x/weight staging alone took
// 134 us of a 240-280 us 70B gate/up).  Per lane, a B fragment needs one dword of 4-bit quants (8
// weights) plus its row's scales: the raw image is laid out so that read is conflict-free.
//
// Measured history: v3 with an LDS-shared f16 image (dequant by all threads, ds_write, B read back):
// 882 TF on 70B gate/up M=256 (profiles/r6a_gemm3_first_light.txt), dequant not overlapped with the
// MFMAs and staging latency-bound (r6b / r6c).
//
// A image: rows of 128 B = 8 chunks of 16 B (8 consecutive k); chunk c of row r at c ^ ((r >> 1) &
// 7): every ds_read_b128 of an A fragment is bank-conflict free; global_load_lds writes
// lane-linear, so the swizzle is applied to the per-lane SOURCE address (cdna_hip_programming.md
// rule 21).  Workgroups are mapped XCD-aware (blocks b = x mod 8 share an XCD and get consecutive
// logical ids: the row blocks of one column group).  EPI_ATOMIC splits the stage range over
// blockIdx.y.
#include "kcommon.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"
#include "../runtime/tuning.h"
#include "gemm_lds.h"

#include <algorithm>
#include <utility>

namespace mpk {
using namespace mp;

// PROBE & 2: some raw bits as a "fragment" (no dequant VALU)
template <class RawT>
__device__ __forceinline__ u32x4 raw_as_u32x4(const RawT& r, int u) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&r);
  return u32x4{w[0], w[1], w[2], w[3 + u]};
}



// PROBE (timing probes only, never in the engine): bit 0 skips the MFMAs (operands kept live),
// bit 1 the dequant (B fragments read raw), bit 2 all global->LDS staging
template <int PT, int EPI, int BM, int TW, int PROBE = 0>
__global__ __launch_bounds__(512) void gemm3_kernel(const GemvParams p, const int n_mb, const int st_per_split,
                                                    const int n_stages) {
  using Q = W3<PT>;
  using G = G3Geom<PT, BM, TW>;
  constexpr int NB = G::NB, FM = BM / 16, BN = 128 * TW;
  constexpr bool BF = PT == P_BF16;
  __shared__ __attribute__((aligned(16))) char smem[NB * G::STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware logical id (bijective for any grid size)
  const int nwg = gridDim.x, bx = blockIdx.x;
  const int xcd = bx & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bx >> 3);
  const int cg = lid / n_mb, mb = lid - cg * n_mb;
  const int m0 = mb * BM;
  const int s_begin = blockIdx.y * st_per_split;
  const int s_end = min(s_begin + st_per_split, n_stages);
  if (s_begin >= s_end) return;   // uniform over the workgroup
  const int M = p.M;

  W3Src src;
  src.W = p.W; src.t0 = cg * (BN / 16) + wave * TW; src.ntiles = p.ntiles; src.nsb = p.nsb;
  auto stage_a = [&](int b) { return smem + b * G::STAGE; };
  auto stage_r = [&](int b) { return smem + b * G::STAGE + G::A_BYTES + wave * G::R_WAVE; };

  // every wave issues exactly G::A_INSTR (x) + Q::NI(TW) (its raw weight bytes) LDS-DMA
  // instructions per stage (the counted vmcnt waits below rely on it; glds_n keeps lane 0 active)
  constexpr int SPB = g3_spb<PT>(), XB = PT == P_I8 ? 1 : 2;   // stages per super-block, bytes per x element
  auto issue_a = [&](int s, int b) {
    if constexpr (PROBE & 4) return;
#pragma unroll
    for (int i = 0; i < G::A_INSTR; ++i) {   // A piece pc = 8 rows; lane -> row 8 pc + (l >> 3), chunk l & 7
      const int pc = wave * G::A_INSTR + i;
      const int row = 8 * pc + (lane >> 3);
      const int ch = (lane & 7) ^ g3_swz(row);
      const int gr = min(m0 + row, M - 1);
      glds<16>(reinterpret_cast<const char*>(p.X) + (size_t)gr * p.ldx * XB + s * 128 + 16 * ch, stage_a(b) + pc * 1024);
    }
  };
  auto issue_b = [&](int s, int b) {
    if constexpr (PROBE & 4) return;
    src.sb = s / SPB; src.q = s % SPB;
    Q::template issue<TW>(stage_r(b), src, EmitDirect{src.nt, lane});
  };
  constexpr int NIB = (PROBE & 4) ? 0 : Q::NI(TW);

  f32x4 acc[FM][TW];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int u = 0; u < TW; ++u) acc[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const Consts kc = make_consts();
  const int g = lane >> 4, rl = lane & 15;

  // One continuous LDS-read / MFMA stream over all stages.  Iteration s runs the NA = 2 FM
  // fragment steps j of stage s; A fragments are read AD steps ahead, across the stage boundary:
  // the reads of stage s+1's first fragments (and its raw bytes) start at step JB, right behind the
  // iteration's single barrier, so a stage starts with its operands already in registers and its
  // k-half-0 B fragments already dequantized (no per-stage pipe bubble).
  //   barrier of iteration s (after step JB's MFMAs): every wave has landed stage s+1 and has
  //   finished iteration s-1 (so buffer (s-1) % 3 is free) -> issue stage s+2's x rows into it and
  //   stage s+3's weight bytes into the raw slot of stage s (read, and waited for, in iteration
  //   s-1), then read stage s+1.  The weights come from HBM: issued three stages ahead they get two
  //   stages of latency (loads retire in order, so the wait for x(s+1) leaves only w(s+2) behind).
  static_assert(NB == 3, "gemm3: the cross-stage stream needs 3 stage buffers");
  constexpr int NA = 2 * FM, AD = G3_AD(BM, TW), NR = Q::NR(TW), JB = NA - AD - 1;
  static_assert(JB > FM / 2 && NA - AD > JB, "gemm3: barrier step");
  typename Q::template Raw<TW> raw;   // this stage's raw bytes
  typename Q::Prep pr[TW];
  half8_t bf[2][TW];
  u32x4 af[NA];
  auto abase = [&](int b, int kk) { return lds_addr(stage_a(b) + g3_off(rl, 4 * kk + g)); };
  // row 16 i + rl has the swizzle of rl: fragment (kk, i) = base(kk) + 2048 i (immediate offset)
  auto read_a = [&](auto jc, u32x4& dst, uint32_t base) {
    constexpr int j = decltype(jc)::value;
    ds_b128o<(j % FM) * 2048>(dst, base);
  };
  auto dequant0 = [&](const typename Q::template Raw<TW>& w, typename Q::Prep* p, int q) {
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      p[u] = Q::template prep<TW>(w, u, q, lane);
      if constexpr (PROBE & 2) bf[0][u] = __builtin_bit_cast(half8_t, raw_as_u32x4(w, u));
      else bf[0][u] = Q::template frag<TW>(w, p[u], u, 0, lane, kc);
    }
  };

  // prologue: stages 0, 1 (and 2's weights) in flight; stage 0's raw, first AD fragments, k-half-0 B fragments
  issue_a(s_begin, 0);
  issue_b(s_begin, 0);
  issue_a(min(s_begin + 1, s_end - 1), 1);
  issue_b(min(s_begin + 1, s_end - 1), 1);
  issue_b(min(s_begin + 2, s_end - 1), 2);
  wait_vmcnt<(PROBE & 4) ? 0 : G::A_INSTR + 2 * NIB>();
  __builtin_amdgcn_s_barrier();
  Q::template load<TW>(stage_r(0), lane, raw);
  {
    const uint32_t a0 = abase(0, 0);
    static_for<AD>([&](auto jc) { read_a(jc, af[decltype(jc)::value], a0); });
  }
  wait_lgkm<AD>();   // raw in (the oldest reads)
  dequant0(raw, pr, s_begin & 3);

  // one stage; the loop runs it twice per trip with the (current, next) register sets swapped, so
  // the next stage's fragments never need a register copy (their reads are still in flight at the
  // end of the stage: a v_mov would read them early)
  using RawT = typename Q::template Raw<TW>;
  using PrepT = typename Q::Prep;
  // LAST (the split's final stage, compile-time) issues nothing for a next stage: no LDS-DMA, no
  // barrier, no raw_n / af_n reads -- no LDS read is ever left unconsumed (a dead read's VGPRs are
  // recycled by the compiler while its data is in flight: tools/isa_lint.py "clobber")
  auto stage = [&](auto lastc, const int s, const int b, u32x4 (&af)[NA], u32x4 (&af_n)[NA], RawT& raw, RawT& raw_n,
                   PrepT (&pr)[TW], PrepT (&pr_n)[TW]) {
    constexpr bool LAST = decltype(lastc)::value;
    const int b1 = b == 2 ? 0 : b + 1, b2 = b1 == 2 ? 0 : b1 + 1;   // buffers of stages s+1, s+2 (= s-1)
    const uint32_t a0 = abase(b, 0), a1 = abase(b, 1);
    const uint32_t n0 = abase(b1, 0);
    static_for<NA>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      constexpr int kk = j / FM, i = j % FM;
      // reads issued after fragment j: the rest of this stage's look-ahead, plus (from step JB on)
      // the next stage's raw bytes and its first fragments (exact issue counts: completion is in
      // order, so lgkmcnt(n) retires everything but the n youngest); capped at the counter's 15
      constexpr int later = (NA - 1 - j < AD - 1 ? NA - 1 - j : AD - 1) + (!LAST && j > JB ? NR + (j - JB - 1) : 0);
      wait_lgkm<(later < 15 ? later : 15)>();
      if constexpr (PROBE & 1) {
        asm volatile("" ::"v"(af[j]));
      } else {
#pragma unroll
        for (int u = 0; u < TW; ++u) {
          if constexpr (PT == P_I8)
            acc[i][u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_mfma_i32_16x16x64_i8(
                __builtin_bit_cast(i32x4, af[j]), __builtin_bit_cast(i32x4, bf[kk][u]), __builtin_bit_cast(i32x4, acc[i][u]), 0, 0, 0));
          else acc[i][u] = mma<BF>(x_op<BF>(__builtin_bit_cast(half8_t, af[j])), bf[kk][u], acc[i][u]);
        }
      }
      if constexpr (j + AD < NA) read_a(std::integral_constant<int, j + AD>{}, af[j + AD], (j + AD) / FM ? a1 : a0);
      if constexpr (j == FM / 2) {   // k-half 1's B fragments, behind the first MFMAs
#pragma unroll
        for (int u = 0; u < TW; ++u) {
          if constexpr (PROBE & 2) bf[1][u] = __builtin_bit_cast(half8_t, raw_as_u32x4(raw, u) + 1u);
          else bf[1][u] = Q::template frag<TW>(raw, pr[u], u, 1, lane, kc);
        }
      }
      if constexpr (!LAST && j == JB) {
        wait_vmcnt<NIB>();   // x(s+1) and w(s+1) in: only w(s+2) (issued after x(s+1)) may be in flight
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue_a(min(s + 2, s_end - 1), b2);
        issue_b(min(s + 3, s_end - 1), b);
        Q::template load<TW>(stage_r(b1), lane, raw_n);
      }
      if constexpr (!LAST && j > JB) {   // stage s+1's fragment j - JB - 1 (all k-half 0: AD <= FM)
        read_a(std::integral_constant<int, j - JB - 1>{}, af_n[j - JB - 1], n0);
      }
      if constexpr (!LAST && j == NA - 2) {   // stage s+1's raw bytes are older than its last fragment read
        wait_lgkm<(j - JB < 15 ? j - JB : 15)>();
        dequant0(raw_n, pr_n, (s + 1) & 3);   // (bf[0] of stage s is consumed: last use at j = FM - 1)
      }
    });
    if constexpr (PROBE & 1) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int u = 0; u < TW; ++u) asm volatile("" ::"v"(bf[kk][u]));
    }
  };
  using F_ = std::false_type;
  using T_ = std::true_type;
  u32x4 afB[NA];
  RawT rawB;
  PrepT prB[TW];
  int s = s_begin, b = 0;
  // pairs of stages, then an odd last stage as LAST (its next-stage reads would be dead).  After
  // an even count the loop's final next-stage reads are dead too, but live up to the loop exit (the
  // back edge uses them), and the exit goes straight to the lgkmcnt(0) below
  for (; s + 1 < s_end; s += 2) {
    stage(F_{}, s, b, af, afB, raw, rawB, pr, prB);
    b = b == 2 ? 0 : b + 1;
    stage(F_{}, s + 1, b, afB, af, rawB, raw, prB, pr);
    b = b == 2 ? 0 : b + 1;
  }
  if (s < s_end) stage(T_{}, s, b, af, afB, raw, rawB, pr, prB);
  wait_vmcnt<0>();   // the clamped tail loads: drained before the workgroup's LDS is released
  wait_lgkm<0>();

  // epilogue: lane holds C[row 16 i + 4 g + v][col 16 u + r] of the wave's tiles
  const int row0 = m0 + 4 * g;
  const int col0 = cg * BN + wave * 16 * TW;
  if constexpr (PT == P_I8) {   // exact int32 sums -> f32: times the x row scale and the weight row scale
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      const float ws = p.wscale[min(col0 + 16 * u + rl, p.ntiles * 16 - 1)];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        // whole-vector bit cast: clang's __builtin_bit_cast of one ext_vector element read element 0
        const i32x4 iv = __builtin_bit_cast(i32x4, acc[i][u]);
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[i][u][v] = (float)iv[v] * (p.xscale[min(row0 + 16 * i + v, M - 1)] * ws);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < TW; ++u) {
    const int n = col0 + 16 * u + rl;
    if constexpr (EPI == EPI_SWIGLU) {
      const int o = (n >> 4) * 8 + rl;   // tile rows 0-7 gate, 8-15 up of the same 8 outputs
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float other = __shfl_xor(acc[i][u][v], 8);
          const int m = row0 + 16 * i + v;
          if (rl < 8 && m < M && o < p.n_valid) p.H[(size_t)m * p.ldh + o] = sat_f16(silu(acc[i][u][v]) * other);
        }
    } else {
      if (n < p.n_valid) {
        const float bias = (p.bias && blockIdx.y == 0) ? p.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int m = row0 + 16 * i + v;
            if (m < M) {
              float* dst = p.Y + (size_t)blockIdx.y * p.split_stride + (size_t)m * p.ldy + n;
              if constexpr (EPI == EPI_ATOMIC) unsafeAtomicAdd(dst, acc[i][u][v] + bias);
              else *dst = acc[i][u][v] + bias;
            }
          }
      }
    }
  }
}

}  // namespace mpk

namespace mp {

// A/B overrides come from the knob registry (tuning.h: atomic, validated); the split target is
// gemm2's GEMM2_SPLIT_WG, so the two GEMMs fill the grid by the same rule

template <int PT, int EPI, int BM, int TW, int PROBE>
static void gemm3_launch(const GemvParams& p, dim3 grid, int n_mb, int per, int n_stages, hipStream_t st) {
  hipLaunchKernelGGL((mpk::gemm3_kernel<PT, EPI, BM, TW, PROBE>), grid, dim3(512), 0, st, p, n_mb, per, n_stages);
}

template <int PT, int EPI, int BM, int TW>
static void gemm3_go(GemvParams p, bool allow_split, hipStream_t st) {
  if constexpr (mpk::G3Geom<PT, BM, TW>::NB < 3) {   // 16-bit 256 x 256: 3 stages do not fit in LDS
    return gemm3_go<PT, EPI, BM, 1>(p, allow_split, st);
  } else {
  constexpr int NT = 8 * TW;   // T16 tiles per workgroup
  const int n_cg = (p.ntiles + NT - 1) / NT;
  const int n_mb = (p.M + BM - 1) / BM;
  const int n_stages = p.nsb * mpk::g3_spb<PT>();
  const int wgs = n_cg * n_mb;
  int nsplit = 1;
  const int split_wg = knob(KNOB_GEMM2_SPLIT_WG);
  if (EPI == EPI_ATOMIC && allow_split) {
    if (knob(KNOB_GEMM3_SPLIT) > 0) nsplit = knob(KNOB_GEMM3_SPLIT);
    // >= 1024 k per split (16 f16 stages of 64 k, 8 int8 stages of 128 k): the 8B o / qkv at M = 256
    // in int8 otherwise ran 64 workgroups (2 splits of K 4096 at 16 int8 stages each)
    else if (wgs < split_wg) nsplit = std::max(1, std::min(split_wg / wgs, n_stages / (PT == P_I8 ? 8 : 16)));
  }
  nsplit = std::max(1, std::min(nsplit, n_stages));
  const int per = (n_stages + nsplit - 1) / nsplit;
  nsplit = (n_stages + per - 1) / per;
  const dim3 grid(wgs, nsplit);
#ifdef MIPIPE_TIMING_PROBES
  if constexpr (PT == P_Q4_K && EPI == EPI_SWIGLU && BM == 256 && TW == 2) {
    switch (knob(KNOB_GEMM3_PROBE)) {   // timing probes (tools/gemv_bench.py --knob GEMM3_PROBE=k)
      case 1: return gemm3_launch<PT, EPI, BM, TW, 1>(p, grid, n_mb, per, n_stages, st);
      case 2: return gemm3_launch<PT, EPI, BM, TW, 2>(p, grid, n_mb, per, n_stages, st);
      case 3: return gemm3_launch<PT, EPI, BM, TW, 3>(p, grid, n_mb, per, n_stages, st);
      case 4: return gemm3_launch<PT, EPI, BM, TW, 4>(p, grid, n_mb, per, n_stages, st);
      case 6: return gemm3_launch<PT, EPI, BM, TW, 6>(p, grid, n_mb, per, n_stages, st);
      default: break;
    }
  }
#endif
  gemm3_launch<PT, EPI, BM, TW, 0>(p, grid, n_mb, per, n_stages, st);
  }
}

template <int PT, int EPI>
static void gemm3_shape(GemvParams p, bool allow_split, hipStream_t st) {
  // BM: 128 rows when one 128-row block holds M; BN: 256 columns (2 tiles per wave) unless that
  // leaves fewer than half the CUs with a workgroup and the epilogue cannot split K
  const int bm = knob(KNOB_GEMM3_BM) == 128 || knob(KNOB_GEMM3_BM) == 256 ? knob(KNOB_GEMM3_BM) : (p.M <= 128 ? 128 : 256);   // (96: gemm4 only)
  const int wg256 = (p.ntiles + 15) / 16 * ((p.M + bm - 1) / bm);
  const bool splits = EPI == EPI_ATOMIC && allow_split;
  // split-K (ATOMIC) shapes: 128 columns (r6e, M = 256: 70B qkv 104 -> 77 us, o 101 -> 74, down
  // 186 -> 161, 8B down 91 -> 65); SwiGLU / store keep 256 unless that leaves half the CUs idle
  const int bn = knob(KNOB_GEMM3_BN) ? knob(KNOB_GEMM3_BN) : (splits || wg256 < 128 ? 128 : 256);
  if (bm == 128) {
    if (bn == 128) gemm3_go<PT, EPI, 128, 1>(p, allow_split, st);
    else gemm3_go<PT, EPI, 128, 2>(p, allow_split, st);
  } else {
    if (bn == 128) gemm3_go<PT, EPI, 256, 1>(p, allow_split, st);
    else gemm3_go<PT, EPI, 256, 2>(p, allow_split, st);
  }
}

template <int PT>
static void gemm3_pt(int epi, const GemvParams& p, bool allow_split, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return gemm3_shape<PT, EPI_STORE>(p, allow_split, st);
    case EPI_ATOMIC: return gemm3_shape<PT, EPI_ATOMIC>(p, allow_split, st);
    case EPI_SWIGLU: return gemm3_shape<PT, EPI_SWIGLU>(p, allow_split, st);
  }
}

void launch_gemm3(int ptype, int epi, GemvParams p, hipStream_t st, bool allow_split) {
  switch (ptype) {
    case P_Q4_K: gemm3_pt<P_Q4_K>(epi, p, allow_split, st); break;
    case P_Q5_K: gemm3_pt<P_Q5_K>(epi, p, allow_split, st); break;
    case P_Q6_K: gemm3_pt<P_Q6_K>(epi, p, allow_split, st); break;
    case P_Q8_0: gemm3_pt<P_Q8_0>(epi, p, allow_split, st); break;
    case P_Q4_0: gemm3_pt<P_Q4_0>(epi, p, allow_split, st); break;
    case P_F16: gemm3_pt<P_F16>(epi, p, allow_split, st); break;
    case P_BF16: gemm3_pt<P_BF16>(epi, p, allow_split, st); break;
    case P_I8: gemm3_pt<P_I8>(epi, p, allow_split, st); break;
  }
}

}  // namespace mp

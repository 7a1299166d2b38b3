// Host-visible launch API of the mipipe HIP kernels (implemented in csrc/kernels/*.hip).
// Every launcher is asynchronous on the given stream and graph-capturable (no allocation,
// no synchronisation inside).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 f16;

namespace mp {

enum Epilogue : int { EPI_STORE = 0, EPI_ATOMIC = 1, EPI_SWIGLU = 2 };

// Decode q|k|v epilogue of the small-M GEMV (gemvs, single stream): instead of storing raw q|k|v
// for the attention to rotate and append, the GEMV applies RoPE to q (stored rotated, f32, into Y)
// and to k, and appends k and v to the paged KV cache itself.  Its loads of pos, the block-table
// entry and the cos/sin pair are issued at kernel start, under the weight stream, so the decode
// attention that follows starts with only the block table and its K/V pages to wait for.
struct QkvAppend {
  const int32_t* pos = nullptr;    // [M]; nullptr: plain STORE epilogue
  int slot0 = 0;                   // row m's slot is slot0 + m
  const int32_t* block_table = nullptr; int max_pages = 0;
  const float2* rope_cs = nullptr; // [max_pos][hd / 2] (cos, sin)
  f16* k_cache = nullptr; f16* v_cache = nullptr;   // K [page][Hkv][64][Dp], V^T [page][Hkv][Dp][64]
  int Hq = 0, Hkv = 0, hd = 0, Dp = 0, kv_fp8 = 0;
  int col0 = 0;                    // q|k|v column of this GEMV's output column 0
};

struct GemvParams {
  const uint8_t* W;      // T16-packed weights
  const f16* X;          // activations [M][ldx] (K_pad columns, zero tail)
  int ldx;
  int M;                 // rows of X (<= 64 for gemv)
  float* Y;              // EPI_STORE / EPI_ATOMIC destination [M][ldy]
  int ldy;
  f16* H;                // EPI_SWIGLU destination [M][ldh]
  int ldh;
  int ntiles, nsb, sb_per_split;
  int n_valid;           // valid output columns
  // optional fusions (gemv2.hip):
  // deferred RMSNorm (M <= 4): X unused; the GEMV runs on f16(Xf * gamma) and accumulates
  // sum(Xf^2) per row while staging.  STORE / SWIGLU (split-free): outputs scaled by
  // rsqrt(mean(Xf^2) + eps).  ATOMIC: outputs left unscaled, the per-split partial sums of squares
  // are atomically added to ssq[m] for the consumer to apply (the fused decode attention).
  const float* Xf = nullptr;
  int ldxf = 0;
  const float* gamma = nullptr;
  float eps = 0.f;
  int d_norm = 0;                // row length of the norm (d_model; multiple of 8)
  float* ssq = nullptr;          // ATOMIC + Xf: [M] sum of squares accumulator (zeroed by the caller)
  int64_t split_stride = 0;      // STORE: split s writes Y + s * split_stride (deterministic split-K partials)
  const float* bias = nullptr;   // [n] added once (split 0) to STORE / ATOMIC outputs
  float* zero = nullptr;         // side job after the GEMV: zero_n floats cleared
  int64_t zero_n = 0;
  int m_blocks = 1;              // (unused: the retired 128-row gemm2 form)
  // P_I8 (launch_gemm3): X holds int8 rows (ldx in bytes), y = xscale[m] * wscale[n] * sum(xq * wq)
  const float* xscale = nullptr;
  const float* wscale = nullptr;
  int rpf = 0;                   // gemvs ATOMIC, one split: residual loaded at kernel start (knob GEMVS_RPF)
  QkvAppend qa;                  // gemvs STORE + fused norm: RoPE + KV append epilogue (qa.pos set)
  int probe = 0;                 // timing probes only (knob GEMVS_PROBE, `make PROBES=1`)
};

void launch_gemv(int ptype, int epi, GemvParams p, int nsplit, hipStream_t st);
// Small-M GEMV (gemvs.hip, M <= 4): whole k-range of x staged in LDS once per workgroup (fused
// RMSNorm when p.Xf is set), split-K inside the workgroup; STORE / SWIGLU write complete outputs,
// EPI_ATOMIC adds into Y by read-modify-write (nsplit 1, deterministic) or atomics (nsplit > 1)
struct GemvsPlan { int G = 1, nsplit = 1, sb_per_split = 0; size_t lds = 0; };
GemvsPlan plan_gemvs(int ntiles, int nsb, int M, int epi, bool norm, bool deterministic);
// q+k and v of a mixed-type layer in one launch (gemvs.hip): STORE, fused RMSNorm, same K
bool gemvs2_supported(int pt, int pt2);
void launch_gemvs2(int pt, int pt2, GemvParams p, GemvParams p2, hipStream_t st);
void launch_gemvs(int ptype, int epi, GemvParams p, bool deterministic, hipStream_t st, int force_G = 0,
                  int force_split = 0);
void set_gemv_tpw(int tiles_per_wave);    // M > 32 tiles per wave: 0 = auto, 1, 2 (tuning knob)
int gemv_tiles_per_wave(int M, int epi);
// split-K factor giving ~target waves for an ATOMIC-epilogue GEMV (>= 4 super-blocks per split)
// Cold-weight sweep on MI355X (tools/gemv_bench.py, 70B shapes): ~4096 tile-waves per launch
// (e.g. Wo M=16: 4 tiles/wave x 8 splits = 14 us vs 20 us at 1 tile x 2 splits).
// split-K factor of a decode GEMV launch (ATOMIC only): tile-waves over the whole grid against a
// target (knob GEMV_SPLIT_WAVES for M > 32, 4096 below), at least GEMV_SPLIT_MINSB super-blocks per
// split; implemented in gemv.hip
int gemv_auto_split(int ntiles, int nsb, int M, int epi);
void launch_unpack(int ptype, const uint8_t* W, int ntiles, int nsb, f16* out, int ldo, hipStream_t st);

// Prefill GEMM (M > 16): Y[M][N] (+)= X[M][K] W^T, MFMA tiles with in-LDS dequant.
void launch_gemm(int ptype, int epi, GemvParams p, hipStream_t st);
// (The 128-row "gemm2" form of the decode GEMV, the quantized prompt GEMM of rounds 1-4, is retired:
// gemm4 took every quantized shape in round 5; the last commit with it is d54fe81.)
// Prompt / wide-decode GEMM v3 (gemm3.hip): BM x BN = {128, 256} x {128, 256} workgroup tiles, each
// weight element dequantized once per workgroup into an f16 LDS image shared by its 8 waves,
// X and the raw quants staged by global_load_lds, 16x16x32 f16 MFMA; EPI_ATOMIC splits K over
// blockIdx.y (allow_split).  A/B overrides: knobs GEMM3_BM / GEMM3_BN / GEMM3_SPLIT (tuning.h).
void launch_gemm3(int ptype, int epi, GemvParams p, hipStream_t st, bool allow_split = true);
// Prompt / wide-decode GEMM v4 (gemm4.hip): gemm3's LDS-DMA stream on v_mfma_f32_32x32x16 (BM 128 |
// 256 rows x 256 columns, each wave owning 32 columns).  Q4_K, Q6_K, F16, BF16; false = type not
// supported (nothing launched).  _splitk: split-K partial stores like launch_gemm2_splitk.
bool gemm4_supported(int ptype);
int gemm4_splits(int ptype, int ntiles, int nsb, int M);   // K splits of a splittable launch
bool launch_gemm4(int ptype, int epi, GemvParams p, hipStream_t st, bool allow_split = true);
bool launch_gemm4_splitk(int ptype, GemvParams p, float* scratch, size_t scratch_n, hipStream_t st,
                         bool reduce = true, int* nsplit_out = nullptr);

// Y[m][n] += sum_{s < nsplit} part[s][m][n], s ascending: the fixed-order split-K reduction of the
// deterministic mode (part rows of ldp floats, splits split_stride floats apart)
void launch_splitk_reduce(const float* part, int nsplit, int64_t split_stride, int ldp, int M, int n, float* Y, int ldy,
                          hipStream_t st);

// x f32 [M][ldx] -> out f16 [M][ldo] = rmsnorm(x) * w ; also zero `zero_n` floats at `zero`
// `zero` is filled with 0, or with `bias` repeated every `bias_n` floats when bias != nullptr (the
// split-K accumulator of the next GEMV starts at the projection bias: Qwen2 q/k/v biases)
void launch_rmsnorm(const float* x, int ldx, const float* w, int d, float eps, f16* out, int ldo,
                    int M, float* zero, int64_t zero_n, hipStream_t st, const float* bias = nullptr, int bias_n = 0);
// launch_rmsnorm that first adds nsplit split-K partials (part + s * ss + row * ldp) into x and
// writes x back (gemm_splitk_store: the deferred reduction of the o / down GEMMs into the residual)
// part may be null (nothing to absorb); q8 (optional): the normalised f16 row also quantized to int8
// per row (q8 + row * ldq8, scale q8s[row]) for the int8_gemm consumer
void launch_rmsnorm_acc(float* x, int ldx, const float* w, int d, float eps, f16* out, int ldo, int M,
                        float* zero, int64_t zero_n, const float* part, int nsplit, int64_t ss, int ldp, hipStream_t st,
                        const float* bias = nullptr, int bias_n = 0, int8_t* q8 = nullptr, int ldq8 = 0,
                        float* q8s = nullptr);

// embedding gather + dequant of raw GGUF rows -> x f32 [M][ldx]
void launch_embed(int ggml_type, const uint8_t* table, int64_t row_bytes, int d, const int32_t* tokens,
                  int M, float* x, int ldx, hipStream_t st);

struct RopeKvParams {
  const float* qkv;      // [M][ldqkv]: q (Hq*hd) | k (Hkv*hd) | v (Hkv*hd)
  int ldqkv;
  int M, Hq, Hkv, hd, Dp;  // Dp: padded head dim (64 or 128)
  const int32_t* pos;    // [M]
  const int32_t* slot;   // [M] sequence slot of each token
  const int32_t* block_table;  // [n_slots][max_pages]
  int max_pages;
  const float2* rope_cs; // [max_pos][hd/2] (cos, sin)
  float q_scale;         // 1/sqrt(hd)
  f16* q_out;            // [M][Hq][Dp]
  f16* k_cache;          // pages: [n_pages][Hkv][64][Dp]
  f16* v_cache;          // pages: [n_pages][Hkv][Dp][64] (transposed)
  int kv_fp8 = 0;        // caches hold e4m3 bytes (same element layout, 1 byte each)
};
void launch_rope_kv(const RopeKvParams& p, hipStream_t st);
// int8 rows for the P_I8 GEMM prototype: Q[m][k] = round(X[m][k] / xs[m]), xs[m] = max_k |X[m][k]| / 127
void launch_quant_rows_i8(const f16* X, int ldx, int M, int K, int8_t* Q, int ldq, float* xs, hipStream_t st);
// per-row int8 re-quantization of a dense f16 weight [n_pad][nsb * 256] (launch_unpack output) into
// P_I8 chunks (4096 B per 16 rows x 256 k) + per-row scales ws[n_pad]
void launch_requant_i8(const f16* W, int ldw, int n, int n_pad, int nsb, uint8_t* out, float* ws, hipStream_t st);

struct AttnParams {
  const f16* q;          // [M][Hq][Dp]
  const int32_t* kvlen;  // [M]: keys visible to token row (pos + 1)
  const int32_t* slot;   // [M]
  const int32_t* block_table;
  int max_pages;
  const f16* k_cache;
  const f16* v_cache;
  int M, Hq, Hkv, hd, Dp;
  int tq;                // tokens per row group (same slot, consecutive); 1 for decode
  int split_len;         // positions per split (multiple of 128)
  int n_split;
  int max_kv;            // upper bound of kvlen (grid sizing)
  float* o_part;         // [n_split][M*Hq][Dp] partial (unnormalised) outputs
  float* ml_part;        // [n_split][M*Hq][2] (running max, running sum)
  f16* out;              // [M][ldo] with head h at columns h*hd..
  int ldo;
};
void launch_attention(const AttnParams& p, hipStream_t st);

// prefill flash attention (attn_prefill.hip): 128 MFMA rows (tokens x GQA heads) per workgroup,
// K/V pages staged once per workgroup in LDS, causal page skipping.  One launch per chunk: the
// tiles are (m0 | n << 16) runs of n <= 128 / G consecutive rows of ONE sequence (consecutive
// positions), q [M][Hq][Dp] with q_scale applied, out [M][ldo] (head h at columns h * hd).
constexpr int kPrefillAttnMaxTiles = 256;
struct PrefillAttnParams {
  const f16* q;
  const int32_t* pos; const int32_t* slot;
  const int32_t* block_table; int max_pages;
  const f16* k_cache; const f16* v_cache;
  int Hq, Hkv, hd, Dp;
  f16* out; int ldo;
  int M = 0;                     // rows of the chunk (partial-buffer layout)
  int n_split = 1, split_pages = 1;   // KV splits (grid.z), pages per split
  float* o_part = nullptr; float* ml_part = nullptr;   // [n_split][M*Hq][Dp], [n_split][M*Hq][2]
  int kv_fp8 = 0;                // caches hold e4m3 bytes (kv_dtype "fp8")
  int n_tiles;
  uint32_t tiles[kPrefillAttnMaxTiles];
};
void launch_attn_prefill(const PrefillAttnParams& p, hipStream_t st);
// KV split count for a chunk (sets *split_pages); max_pages_needed = last row's position / 64 + 1
int prefill_attn_splits(int n_tiles, int Hkv, int max_pages_needed, int max_split, int* split_pages);
int prefill_attn_rows_per_tile(int G);   // tokens per tile: 128 / G

// fused decode step of attention: RoPE(q, k) + KV append + split-K flash-decoding + last-arriver
// merge (replaces rope_kv + attention + combine for tq = 1)
struct DecodeAttnParams {
  const float* qkv; int ldqkv;     // [M][ldqkv] f32 projections q | k | v
  const int32_t* pos;              // [M]
  const int32_t* slot;             // [M]
  int slot0 = -1;                  // >= 0: slot of row t is slot0 + t (decode micro-batches); slot unused
  const int32_t* block_table; int max_pages;
  const float2* rope_cs;           // [max_pos][hd/2]
  float q_scale;
  f16* k_cache; f16* v_cache;
  int M, Hq, Hkv, hd, Dp;
  int split_len, n_split;
  float* o_part; float* ml_part;   // [n_split][M*Hq][Dp], [n_split][M*Hq][2]
  int32_t* counters;               // [M*Hkv] zero-initialised, self-resetting
  f16* out; int ldo;
  // deferred RMSNorm of the qkv GEMV (nullptr: qkv already final): q|k|v = rsqrt(ssq[t] / d + eps)
  // * qkv + bias (bias optional, [q|k|v])
  const float* ssq = nullptr; float eps = 0.f; int d_model = 0; const float* bias = nullptr;
  int kv_fp8 = 0;                  // caches hold e4m3 bytes (kv_dtype "fp8")
  int pre = 0;                     // q already rotated, new K / V already appended (gemvs QkvAppend)
  int probe = 0;                   // timing probes only (knob ATTN_PROBE): bit 0 skips the global V append,
                                   // bit 1 the K append (results wrong; never in production runs)
};
void launch_attn_decode(const DecodeAttnParams& p, hipStream_t st);
// the launch would take the one-split workgroup kernel that accepts pre-appended inputs (p.pre)
bool attn_decode_pre_ok(const DecodeAttnParams& p);
// Fused decode attention + output projection (single stream, M <= 4, one KV split): workgroup
// (r, kvh) runs the attention of kv head kvh's query heads, then adds their split-K slice of W_o
// (output tiles [r * 8, r * 8 + 8), k in the heads' dims) into Y with atomics.
struct AttnOParams {
  const uint8_t* W; int ptype; int ntiles, nsb;   // W_o, T16-packed
  float* Y; int ldy; int n_valid;                 // residual [M][ldy]
};
// shapes the fused kernel takes (else: launch_attn_decode + the o-projection GEMV)
bool attn_o_supported(const DecodeAttnParams& p, const AttnOParams& o);
void launch_attn_o(const DecodeAttnParams& p, const AttnOParams& o, hipStream_t st);

// greedy sampling: tokens[m] = argmax logits[m][:n] (lowest index on ties).  With scratch: a
// two-level grid of (chunk, row) workgroups and a last-arriver reduce; without: one workgroup/row.
constexpr int kArgmaxChunks = 64;
struct ArgmaxScratch {
  float* part;          // [rows][kArgmaxChunks][2]
  int32_t* counters;    // [rows], zero-initialised, self-resetting
  int rows;
};
void launch_argmax(const float* logits, int ld, int n, int M, int32_t* tokens, hipStream_t st,
                   const ArgmaxScratch* scratch = nullptr);
// temperature / top-k / top-p / min-p sampling with a counter-based RNG
struct SampleParams {
  const float* logits; int ld; int n; int M;
  float temp; int top_k; float top_p; float min_p;
  uint64_t seed; const int32_t* step;  // step counter (device) for RNG stream
  int32_t* tokens;
};
void launch_sample(const SampleParams& p, hipStream_t st);
// repetition penalties (llama.cpp penalties sampler semantics) over each row's ring of the last
// `last_n` accepted tokens (-1 = empty): every distinct token t of the window with count c gets
// l = l > 0 ? l / repeat : l * repeat, then l -= c * freq + presence.  In place, before sampling.
struct PenaltyParams {
  float* logits; int ld; int n; int M;
  const int32_t* hist; int last_n;     // [M][last_n]
  float repeat, freq, presence;
};
void launch_penalize(const PenaltyParams& p, hipStream_t st);
// append tokens[m] to row m's ring: hist[m][cnt[m] % last_n] = tokens[m]; ++cnt[m]
void launch_hist_push(int32_t* hist, int32_t* cnt, int last_n, const int32_t* tokens, int M, hipStream_t st);

// pos[i] += 1, kvlen[i] = pos[i] + 1 for i < M (graph-resident decode step advance)
void launch_advance(int32_t* pos, int32_t* kvlen, int M, int32_t* step, hipStream_t st);

// standalone SwiGLU: h[m][j] = silu(g[m][j]) * u[m][j]   (g,u f32; h f16)
void launch_swiglu(const float* gu, int ld, int F, int M, f16* h, int ldh, hipStream_t st);
// stage-boundary activation wire format: f32 residual <-> f16 / bf16 (n elements, contiguous)
enum ActDtype : int { ACT_F32 = 0, ACT_F16 = 1, ACT_BF16 = 2 };
void launch_act_pack(const float* x, void* y, int64_t n, int dtype, hipStream_t st);
void launch_act_unpack(const void* y, float* x, int64_t n, int dtype, hipStream_t st);
// f32 -> f16 row conversion (used when an activation feeds a GEMM directly)
void launch_f32_to_f16(const float* x, int ldx, int n, int M, f16* y, int ldy, hipStream_t st);

// MoE
struct MoeRouteParams {
  const float* logits;   // [M][ld] router logits
  int ld;
  int M, E, k;           // E <= 64, k <= 8
  int32_t* counts;       // [E]
  int32_t* lists;        // [E][list_cap] token-slot ids (token*k + j)
  int list_cap;
  float* weights;        // [M*k] renormalised top-k softmax weights
};
void launch_moe_route(const MoeRouteParams& p, hipStream_t st);
// router logits [M][ld] (f32, stored) from x [M][ldx] f16 and the dense f16 router R [E][K], E <= 64
void launch_router_logits(const f16* X, int ldx, const f16* R, int K, int E, int M, float* out, int ld, hipStream_t st);
struct MoeGemvParams {
  const uint8_t* W;      // [E] packed matrices, each `estride` bytes
  size_t estride;
  int ntiles, nsb;
  const f16* X; int ldx; int x_per_slot;  // x row = x_per_slot ? slot : slot / k
  int k;
  const int32_t* counts; const int32_t* lists; int list_cap;
  int E;
  f16* H; int ldh;       // SWIGLU out per slot [M*k][ldh]
  float* Y; int ldy;     // down out: atomic add weight*y into Y[token]
  const float* weights;
  int n_valid;
  int sb_per_split;      // set by the launcher
  int M = 0;             // tokens of the call (bound on rows per expert); 1..64 -> workgroup-shared x kernel
  float* Yslot = nullptr;  // deterministic mode: down out stored per slot [M*k][ldy] (weight applied,
                           // no split-K); launch_moe_combine then adds the k slots in order
};
// Y[t][n] += sum_{j < k} Yslot[t*k + j][n], j ascending (deterministic MoE combine)
void launch_moe_combine(const float* Yslot, int ld_slot, int k, int M, int n, float* Y, int ldy, hipStream_t st);
void launch_moe_route(const MoeRouteParams& p, hipStream_t st);
void launch_moe_gemv(int ptype, int epi, MoeGemvParams p, int nsplit, hipStream_t st);
// Grouped MoE dequant GEMM (gemm4.hip, any M): every routed expert's rows as one 32x32x16 MFMA GEMM
// (rows gathered by the A staging, epilogues scattered by slot).  SWIGLU (gate/up) or ATOMIC (down,
// weighted; Yslot rows in the deterministic mode).  false = type not supported (nothing launched).
bool launch_moe_gemm4(int ptype, int epi, const MoeGemvParams& p, hipStream_t st);

}  // namespace mp

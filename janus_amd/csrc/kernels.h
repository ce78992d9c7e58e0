// Launcher declarations shared by the host-side orchestration (whisper.cpp, vocoder.cpp).
#pragma once
#include "common.h"

namespace janus {

// ------------------------------------------------------------------ GEMM
enum GemmEpi { EPI_F16 = 0, EPI_GELU_F16 = 1, EPI_RESID_F32 = 2, EPI_F32 = 3, EPI_QKV = 4 };
// Largest M the skinny (decoder-step) GEMM takes: a decode batch of 64 windows x 5 sampled
// hypotheses (faster-whisper's best_of) is 320 rows.
constexpr int kSkinnyMaxRows = 512;

struct GemmArgs {
  const _Float16* A; int64_t lda;  // [M][K]
  const _Float16* W; int64_t ldw;  // [N][K]
  const float* bias;               // [N] or null
  void* C; int64_t ldc;            // fp16 or fp32 by epilogue
  const float* R; int64_t ldr;     // fp32 residual (EPI_RESID_F32), may alias C
  int M, N, K;
  // EPI_QKV (M <= 64 only): columns [0,d) -> C, [d,2d) -> kc, [2d,3d) -> vc at row pos
  _Float16* kc = nullptr; _Float16* vc = nullptr; int pos = 0, n_ctx = 0, qkv_d = 0;
  const int32_t* roff = nullptr;  // EPI_QKV: row r's cache row is pos + roff[r] (staggered rows)
  // EPI_RESID_F32 (M <= 64 only): also write the LayerNorm pieces of the new rows,
  // ln_part[row][col / 16] (see SkinnyLnArgs)
  float2* ln_part = nullptr;
  // grouped (block-diagonal) product, M <= 64 only: output columns [g*a_group_cols,
  // (g+1)*a_group_cols) read A columns [g*K, (g+1)*K) — per-head projections
  int a_group_cols = 0;
  // M <= 64 only: outputs up to this many columns also split their rows over blocks
  // (0 = JANUS_SKINNY_MSPLIT_N or 2048, tuned on a whole GPU; 1024 on a half-GPU CU mask)
  int msplit_n = 0;
  // a decoder step (rows = decode batch): M <= kSkinnyMaxRows runs on the skinny kernel
  // (rows split over blocks) instead of the 128 x 128 / 256 x 256 tile kernels
  bool decode_rows = false;
  // EPI_RESID_F32 (M <= 64 only): the LayerNorm of the NEW residual rows, fused: the
  // output rows are stored write-through (sc1), every block adds to its row block's
  // counter ln_cnt[blockIdx.y] once its stores have drained, and the last block of each
  // row block to arrive normalises that block's rows (sc1 loads, one row per wave) into
  // ln_out [M][N] fp16 with (ln_g, ln_b, ln_eps) and re-arms its counter (ln_cnt: at
  // least ceil(M / 16) ints, zero on entry).
  const float* ln_g = nullptr; const float* ln_b = nullptr; float ln_eps = 1e-5f;
  _Float16* ln_out = nullptr; int* ln_cnt = nullptr;
  // M <= 64 only: A = LayerNorm(lnin_x) (fp32 [M][K], row stride lnin_ldx) computed in
  // every block's prologue into an fp16 LDS tile — the pre-LN block needs no separate
  // LayerNorm launch (A / lda are then unused).
  const float* lnin_x = nullptr; int64_t lnin_ldx = 0;
  const float* lnin_g = nullptr; const float* lnin_b = nullptr; float lnin_eps = 1e-5f;
};
void gemm_launch(int epi, const GemmArgs& p, hipStream_t s);
// the general large-M kernel (128 x 128 tiles, any N / K % 8), for shapes gemm_big rejects
void gemm_nt128_launch(int epi, const GemmArgs& p, hipStream_t s);
// the encoder-size kernel (gemm_big.hip): 256 x 256 tiles, N % 256 == 0, K % 64 == 0
bool gemm_big_supported(int epi, const GemmArgs& p);
void gemm_big_launch(int epi, const GemmArgs& p, hipStream_t s);
// x[M][N] += A W^T + bias (fp32, in place), then out[M][N] = LayerNorm(x) fp16 (gamma g,
// beta b, eps) — one launch for the decoder's attention output projection + the next
// LayerNorm (resid_ln_kernel in gemm.hip; bit-identical to the two launches it replaces).
struct ResidLnArgs {
  const _Float16* A; int64_t lda;  // [M][K]
  const _Float16* W; int64_t ldw;  // [N][K]
  const float* bias;               // [N] or null
  float* x; int64_t ldx;           // [M][N] residual stream, ldx == N
  const float* g; const float* b; float eps;
  _Float16* out;                   // [M][N]
  int M, N, K;
};
bool resid_ln_supported(int N, int K);
void resid_ln_launch(const ResidLnArgs& p, hipStream_t s);

// M <= 64 GEMM with the LayerNorm of its fp32 A operand fused (decoder pre-LN blocks).
// EPI_QKV: columns [0, d) -> C, [d, 2d) -> kc[row][pos], [2d, 3d) -> vc[row][pos].
// LayerNorm fused into the consumer through row-statistic PIECES: the kernel that
// produces a residual-stream row writes, per 16-column group g, part[row][g] =
// (sum, M2 about the group mean); the consumer combines the K/16 pieces of a row
// (Chan's parallel variance) and normalises its A fragments on load. No separate
// LayerNorm launch, no atomics, deterministic.
struct SkinnyLnArgs {
  const float* x; int64_t ldx;
  const float2* part;               // [M][K/16] pieces of x's rows
  const float* gamma; const float* beta; float eps;
  const _Float16* W; int64_t ldw;
  const float* bias;
  void* C; int64_t ldc;
  int M, N, K;
  _Float16* kc; _Float16* vc; int pos, n_ctx, qkv_d;
};
void gemm_skinny_ln_launch(int epi, const SkinnyLnArgs& p, hipStream_t s);

// ------------------------------------------------------------- LayerNorm
// out[r][:] = fp16( (x[r]-mean)/sqrt(var+eps) * g + b ), x fp32 [rows][d]
// out[w][k][lane] = mfma.h xshfl<2^k>(in[w][lane]) (kernel test entry)
void wave_xor_launch(const float* in, float* out, int n_waves, hipStream_t s);
void layernorm_launch(const float* x, const float* g, const float* b, _Float16* out, int rows,
                      int d, float eps, hipStream_t s);
// fp32 out variant (final encoder LN keeps fp32 for the cross-attention K/V GEMMs' input)
void layernorm_f32_launch(const float* x, const float* g, const float* b, float* out, int rows,
                          int d, float eps, hipStream_t s);

// ------------------------------------------------------------ attention
// Encoder self-attention over T positions, head_dim 64. qkv fp16 [B*T][3*d]
// (q | k | v, head h at columns h*64), out fp16 [B*T][d].
void attention_launch(const _Float16* qkv, _Float16* out, int B, int T, int H, float scale,
                      hipStream_t s);
// One query per (b, h) against Tkv cached keys (decoder self/cross attention).
// q[b*q_bs + h*64 + d]; k/v[b*kv_bs + t*kv_rs + h*64 + d]; out[b*o_bs + h*64 + d].
// tkv: device int32 per batch row (NULL => Tkv for all).
void decode_attention_launch(const _Float16* q, int64_t q_bs, const _Float16* k, const _Float16* v,
                             int64_t kv_bs, int64_t kv_rs, int Tkv, const int32_t* tkv,
                             _Float16* out, int64_t o_bs, int B, int H, float scale,
                             hipStream_t s);

// Split-key (flash-decoding) variant for d <= 512: all heads of a row per block.
// part_o: f32 [B][splits][d], part_ml: f32 [B][splits][H][2] workspaces.
// Decoder cross-attention over the encoder output with absorbed K/V projections
// (xattn.hip). xattn_absorb builds Wqk [H*D][D] fp16 and bqk [H*D] f32 (scores in the
// exp2 domain) from the fp32 q/k projections; xattn_launch takes qk [B][H*D] fp16 and
// enc [B][Te][D] fp16 and writes c [B][H*D] fp16 (softmax-weighted encoder rows per
// head) via per-split partials part_c [B][nsplit][H][D] f32 and part_ml [B][nsplit][H][2].
bool xattn_supported(int D, int H);
int xattn_split_count(int Te, int requested);
void xattn_absorb(const float* wq, const float* bq, const float* wk, int D, int H,
                  _Float16* wqk, float* bqk, hipStream_t s);
// pairs (nullable, device int4 [npairs] = {b0, b1, e, -}): decoder rows b0 and b1 (b1 < 0:
// none) attend to encoder row e of enc, read once for both (H <= 8, D <= 512); without it
// row b reads enc row b.
void xattn_launch(const _Float16* qk, const _Float16* enc, int B, int Te, int D, int H,
                  int nsplit, float* part_c, float* part_ml, _Float16* out, hipStream_t s,
                  bool combine = true, const int4* pairs = nullptr, int npairs = 0, bool rev = false);
// Groups of <= 6 decoder rows sharing an encoder row, one block per (split, group):
// groups [device] int [ngroups][8] = {e, row_0 .. row_5 (-1: none), -}; partials as
// xattn_launch(combine = false) writes them (merged by xattn_combine_vproj_launch).
void xattn_group_launch(const _Float16* qk, const _Float16* enc, int Te, int D, int H, int nsplit,
                        float* part_c, float* part_ml, hipStream_t s, const int* groups, int ngroups,
                        int rows_per_group);
// The split merge of xattn_launch(..., combine = false) fused with the per-head value
// projection: out[b][64h + j] = merge_s(part)[b][h] . wv[64h + j]^T + bv[64h + j]
// (wv [H*64][D] fp16, out row stride ldo); bit-identical to the merge kernel followed by the
// block-diagonal skinny GEMM.
bool xattn_cvp_supported(int D, int H);
void xattn_combine_vproj_launch(const float* part_c, const float* part_ml, int nsplit, int B, int H,
                                int D, const _Float16* wv, const float* bv, _Float16* out, int64_t ldo,
                                hipStream_t s);

int decode_split_count(int Tkv);
void decode_attention_split_launch(const _Float16* q, int64_t q_bs, const _Float16* k,
                                   const _Float16* v, int64_t kv_bs, int64_t kv_rs, int Tkv,
                                   _Float16* out, int64_t o_bs, int B, int H, float scale,
                                   float* part_o, float* part_ml, hipStream_t s,
                                   const int32_t* roff = nullptr, int max_roff = 0);

// ----------------------------------------------------------------- conv
enum Act { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_TANH = 3 };

// Implicit-GEMM 1-D convolution on MFMA, time-major [B][T][C] fp16 activations.
// For output row r (0 <= r < n_rows) of phase ph, tap j reads input row
//   r*in_stride + j*dil + in_off            (zero outside [0, T_in))
// and writes output time  r*out_stride + out_off + ph  (skipped outside [0, T_out)).
// Weights are pre-packed by conv_pack_weights (blocked [ph][chunk][group][Cout][KB]).
struct ConvArgs {
  const _Float16* in; int64_t in_bs; int T_in; int Cin;
  const _Float16* w; const float* bias;
  _Float16* out; int64_t out_bs; int T_out; int Cout;
  const _Float16* res; int64_t res_bs;  // added after post_act (fp16, [B][T_out][Cout]); may be null
  int taps, dil, in_stride, in_off, out_stride, out_off, n_rows, phases;
  int pre_act, post_act;
  float out_scale; int accumulate;      // out = (accumulate ? out : 0) + out_scale * y
  int B;
  int post_acc_silu = 0;                // out = silu(out) after the accumulation
  int remap = -1;                       // tile order: 0 dispatch, 1 XCD runs of row blocks,
                                        // 2 XCD runs over the whole grid; -1 = default
};
// The same products on hipBLASLt (blaslt.cpp), a comparison point only (the product path
// runs gemm_big): true when the library ran the GEMM (plain and residual epilogues; GELU
// as bias + an exact-GELU pass), false when it has no workspace-free plan for the shape.
bool gemm_lt_launch(int epi, const GemmArgs& g, hipStream_t s);
// x = gelu_erf(x) in place on fp16 [M][N] (row stride ld, N % 8 == 0)
void gelu_inplace_f16_launch(_Float16* x, int64_t ld, int M, int N, hipStream_t s);

struct ConvPack { int ck, kb, chunks, groups; int64_t phase_elems; };
ConvPack conv_pack_geometry(int Cin, int Cout, int taps);
// Pack fp32 PyTorch weights into the blocked fp16 layout (device pointers).
//   transposed=0: w is Conv1d [Cout][Cin][taps], phases=1
//   transposed=1: w is ConvTranspose1d [Cin][Cout][2u] (stride u): phases=u, 2 taps/phase
void conv_pack_weights(const float* w, _Float16* packed, int Cin, int Cout, int taps,
                       int transposed, int u, hipStream_t s);
void conv_launch(const ConvArgs& a, hipStream_t s);

// Fused ResBlock1 unit (resunit.hip): out = (acc ? out : 0) + scale *
//   (x + c2(silu(c1(silu(x)) + b1)) + b2), C in {16, 32}, weights packed [C][KP].
struct ResUnitArgs {
  const _Float16* x; _Float16* out;
  const _Float16* w1; const float* b1;
  const _Float16* w2; const float* b2;
  int B, T, C, k, d;
  float scale; int accumulate;
  // out = silu(out) after the accumulation: the last unit of a ParallelBlock stores the
  // SiLU its consumer (the next upsampler, or conv_post) would apply on every read
  int post_silu = 0;
};
int resunit_kp(int C, int k);
bool resunit_supported(int C, int k);
void resunit_pack(const float* w, _Float16* out, int C, int k, hipStream_t s);
void resunit_launch(const ResUnitArgs& a, hipStream_t s);

// ------------------------------------------------------------------ VAD
// Silero-vad v5 16 kHz weights (vad.hip), fp32 device pointers by published name.
struct VadWeights {
  const float* basis;                // stft.forward_basis_buffer [258][256]
  const float* w0; const float* b0;  // encoder.0 [128][129][3]
  const float* w1; const float* b1;  // encoder.1 [64][128][3]
  const float* w2; const float* b2;  // encoder.2 [64][64][3]
  const float* w3; const float* b3;  // encoder.3 [128][64][3]
  const float* wih; const float* whh; const float* bih; const float* bhh;  // LSTMCell(128, 128)
  const float* wo; const float* bo;  // decoder.2 Conv1d(128, 1, 1)
};
// pcm [device] [n_streams][n_chunks][chunk_len] (each chunk decimated by `decim` to 512
// samples); ctx_state [n_streams][64], hc_state [n_streams][2][128] in/out; prob
// [n_streams][n_chunks].
void silero_vad_launch(const float* pcm, int n_streams, int n_chunks, int chunk_len, int decim,
                       const VadWeights& W, float* ctx_state, float* hc_state, float* prob,
                       hipStream_t s);

// ------------------------------------------------------------------ mel
void mel_launch(const float* pcm, const int64_t* offsets, int B, const float* basis,
                const float* filters, float* logmel, uint32_t* maxkey, int n_frames_out,
                int decim, hipStream_t s);
void mel_normalize_launch(const float* logmel, const uint32_t* maxkey, _Float16* out,
                          const int64_t* offsets, int decim, int B, int frames, int n_mels,
                          int out_ld, hipStream_t s);

}  // namespace janus

// Decoder-loop kernels (decoder.hip).
#pragma once
#include "common.h"

namespace janus {

struct DecodeRules {
  int eot;
  int suppress_blank, blank;     // SuppressBlank at the first sampled token
  int ts_begin;                  // first timestamp token id; -1 disables timestamp rules
  int no_timestamps;             // <|notimestamps|> (always suppressed in timestamp mode)
  int max_initial_ts;            // max_initial_timestamp index (-1: none)
  int target;                    // token whose raw softmax probability is tracked (no-speech), -1: none
  float inv_temp;                // 0: greedy (argmax); > 0: sample at temperature 1 / inv_temp
                                 // (Gumbel-max over the rule-filtered logits, noise from
                                 // sample_noise(seed of the row, position, token))
};

// Per-row rule state carried across steps (computed by the selector for the next step).
struct RowRules {
  int sample_begin;       // no token sampled yet
  int suppress_all_ts;    // last two sampled were timestamps
  int suppress_text;      // last was a timestamp, penultimate was not: text (< eot) banned
  int ts_floor;           // timestamps < ts_floor banned (-1: none)
  int last_stamp;         // last sampled timestamp token (-1: none)
  int pad[3];
};

// Per (row, 16-column block) partial statistics of the rule-filtered logits.
struct LogitPart {
  float m_all, s_all;     // max / sum exp(v - m_all) over allowed tokens
  float m_text;           // max over allowed text tokens (< ts_begin)
  float m_ts, s_ts;       // max / sum exp over allowed timestamp tokens
  float b_all_v; int b_all_i;  // argmax over allowed (first index on ties); sampling: of the
                               // perturbed key logit * inv_temp + gumbel
  float b_ts_v; int b_ts_i;    // the same over allowed timestamps
  float t_v;              // raw logit of DecodeRules::target (-inf if not in this block)
  float m_raw, s_raw;     // max / sum exp over ALL tokens (unfiltered softmax)
  float b_all_r, b_ts_r;  // the logits of b_all_i / b_ts_i (= b_*_v when greedy)
};

// Sampling noise (decode at temperature > 0): a counter-based hash of (row seed, position,
// token), so a row's draws do not depend on its batch neighbours or the tile schedule and
// the CPU oracle can regenerate them (oracle/whisper.py sample_noise).
__host__ __device__ inline uint32_t noise_mix(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__host__ __device__ inline uint32_t noise_base(uint32_t seed, int pos) {
  return noise_mix(seed ^ noise_mix((uint32_t)pos * 0x9e3779b9u + 0x7f4a7c15u));
}
// uniform u = an odd multiple of 2^-24 in (0, 1), exact in f32; Gumbel(0, 1) = -log(-log u)
__device__ inline float sample_gumbel(uint32_t base, int token) {
  const uint32_t h = noise_mix(base ^ ((uint32_t)token * 0x27d4eb2fu));
  const float u = (float)((h >> 8) | 1u) * 0x1p-24f;
  return -logf(-logf(u));
}

void cast_f16_f32_launch(const _Float16* in, float* out, int64_t n, hipStream_t s);
void cast_f32_f16_launch(const float* in, _Float16* out, int64_t n, hipStream_t s);
// x[b] = tok_emb[token] + pos_emb[pos]; part (nullable): LayerNorm pieces of x
// (SkinnyLnArgs), d % 16 == 0
// x[b] = tok_emb[token] + pos_emb[pos]; optionally the first layer's LayerNorm of the
// row into ln_out [B][d] fp16 (d <= 512, eps 1e-5).
// roff (nullable, device int32 [B]): per-row position offsets — row b is at pos + roff[b]
// (staggered decode: janus_decode_rows.pos_offset)
void embed_launch(const _Float16* tok_emb, const float* pos_emb, const int32_t* tokens,
                  int ld_tokens, int pos, int d, float* x, float2* part, int B, hipStream_t s,
                  const float* ln_g = nullptr, const float* ln_b = nullptr,
                  _Float16* ln_out = nullptr, const int32_t* roff = nullptr);
void kv_store_launch(const _Float16* qkv, int d, int pos, int n_ctx, _Float16* kc, _Float16* vc,
                     int B, hipStream_t s);
void init_tokens_launch(int32_t* tokens, int ld, const int32_t* prompt, int plen, int32_t* done,
                        float* sum_lp, int32_t* n_tok, int B, hipStream_t s);
// per-row prompts: tokens [B][ld] arrive pre-filled (prompt, then -1); only the counters reset
void init_counters_launch(int32_t* done, float* sum_lp, int32_t* n_tok, float* nsp, int B,
                          hipStream_t s);
void select_launch(const float* logits, int V, const DecodeRules& R, const uint8_t* smask,
                   int32_t* tokens, int ld, int pos, int sample_begin_pos, int32_t* done,
                   float* sum_lp, int32_t* n_tok, int B, hipStream_t s);
void rules_init_launch(RowRules* rules, int B, hipStream_t s);
// logits = A[B][K] . W[V][K]^T computed block-wise with the filtered statistics reduced
// in the epilogue (no logits in HBM); nblk = logits_partial_blocks(V) merged partials per row
// (one per block of the launch).
int logits_partial_blocks(int V, int K, int max_blocks = 256);
// lnx: A = LayerNorm(lnx) (fp32 [B][K], eps 1e-5) computed in-block instead of read
void logits_partial_launch(const _Float16* A, int lda, const _Float16* W, int K, int V, int B,
                           const DecodeRules& R, const uint8_t* smask, const RowRules* rules,
                           LogitPart* parts, hipStream_t s,
                           const float* lnx = nullptr, int ldx = 0, const float* ln_g = nullptr,
                           const float* ln_b = nullptr, int max_blocks = 256,
                           const uint32_t* seeds = nullptr, int pos = 0,
                           const float* row_inv_temp = nullptr);
// R.inv_temp > 0: seeds [B] (device) per-row noise seeds, pos = the position whose logits
// these are (the sampled token goes to pos + 1); row_inv_temp [B] (device, nullable): row
// b samples at 1 / row_inv_temp[b] instead of R.inv_temp (several temperatures in one call)
// plen [B] (device, nullable = all rows sample from pos + 1 >= 1): rows with pos + 1 <
// plen[b] are still inside their own prompt and keep the forced token. At a row's first
// sampled step (pos + 1 == plen[b]) nsp[b] (nullable) gets the raw softmax probability of
// DecodeRules::target (Whisper's no_speech_prob).
void select_partials_launch(const LogitPart* parts, int nblk, const DecodeRules& R,
                            RowRules* rules, int32_t* tokens, int ld, int pos, int32_t* done,
                            float* sum_lp, int32_t* n_tok, int B, hipStream_t s,
                            const int32_t* plen = nullptr, float* nsp = nullptr,
                            const int32_t* roff = nullptr);
// select_partials_launch at pos followed by embed_launch at pos + 1, in one launch
void select_embed_launch(const LogitPart* parts, int nblk, const DecodeRules& R, RowRules* rules,
                         int32_t* tokens, int ld, int pos, int32_t* done, float* sum_lp,
                         int32_t* n_tok, int B, hipStream_t s, const int32_t* plen, float* nsp,
                         const _Float16* tok_emb, const float* pos_emb, int d, float* x,
                         float2* part, const float* ln_g, const float* ln_b, _Float16* ln_out,
                         const int32_t* roff = nullptr);
void build_mask_launch(const int32_t* list, int n, uint8_t* mask, int V, hipStream_t s);
// out [B][V] = sample_gumbel(noise_base(seeds[b], pos), t)
void sample_gumbel_launch(const uint32_t* seeds, int B, int pos, int V, float* out, hipStream_t s);

}  // namespace janus

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
};

void cast_f16_f32_launch(const _Float16* in, float* out, int64_t n, hipStream_t s);
void cast_f32_f16_launch(const float* in, _Float16* out, int64_t n, hipStream_t s);
void embed_launch(const _Float16* tok_emb, const float* pos_emb, const int32_t* tokens,
                  int ld_tokens, int pos, int d, float* x, int B, hipStream_t s);
void kv_store_launch(const _Float16* qkv, int d, int pos, int n_ctx, _Float16* kc, _Float16* vc,
                     int B, hipStream_t s);
void init_tokens_launch(int32_t* tokens, int ld, const int32_t* prompt, int plen, int32_t* done,
                        float* sum_lp, int32_t* n_tok, int B, hipStream_t s);
void select_launch(const float* logits, int V, const DecodeRules& R, const uint8_t* smask,
                   int32_t* tokens, int ld, int pos, int sample_begin_pos, int32_t* done,
                   float* sum_lp, int32_t* n_tok, int B, hipStream_t s);
void build_mask_launch(const int32_t* list, int n, uint8_t* mask, int V, hipStream_t s);

}  // namespace janus

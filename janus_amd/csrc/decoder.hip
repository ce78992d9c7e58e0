// Small kernels of the greedy Whisper decoder loop (batched over utterances, one
// token per step) and of the encoder/decoder glue.
//
// The token selector restates the logit filters faster-whisper's greedy path applies
// (transcribe(beam_size=1, language='en'), transcriber.py:53-57; CTranslate2
// Whisper generate with the OpenAI decoding rules: SuppressBlank, SuppressTokens,
// ApplyTimestampRules incl. max_initial_timestamp, then argmax) and accumulates the
// chosen token's log-probability (avg_logprob).
#include <cfloat>
#include "mfma.h"
#include "kernels.h"
#include "decoder.h"

namespace janus {

__global__ void cast_f16_f32_kernel(const _Float16* __restrict__ in, float* __restrict__ out,
                                    int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (float)in[i];
}

void cast_f16_f32_launch(const _Float16* in, float* out, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  cast_f16_f32_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(in, out, n);
  JANUS_LAUNCH_CHECK();
}

__global__ void cast_f32_f16_kernel(const float* __restrict__ in, _Float16* __restrict__ out,
                                    int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (_Float16)in[i];
}

void cast_f32_f16_launch(const float* in, _Float16* out, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  cast_f32_f16_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(in, out, n);
  JANUS_LAUNCH_CHECK();
}

// x[b][:] = tok_emb[tokens[b][pos]] + pos_emb[pos]   (fp32 residual stream)
__global__ void embed_kernel(const _Float16* __restrict__ tok_emb, const float* __restrict__ pos_emb,
                             const int32_t* __restrict__ tokens, int ld_tokens, int pos, int d,
                             float* __restrict__ x) {
  const int b = blockIdx.x;
  const int tok = tokens[(int64_t)b * ld_tokens + pos];
  for (int i = threadIdx.x; i < d; i += blockDim.x)
    x[(int64_t)b * d + i] = (float)tok_emb[(int64_t)tok * d + i] + pos_emb[(int64_t)pos * d + i];
}

void embed_launch(const _Float16* tok_emb, const float* pos_emb, const int32_t* tokens,
                  int ld_tokens, int pos, int d, float* x, int B, hipStream_t s) {
  embed_kernel<<<B, 256, 0, s>>>(tok_emb, pos_emb, tokens, ld_tokens, pos, d, x);
  JANUS_LAUNCH_CHECK();
}

// qkv[b][d:3d] -> kcache[b][pos][:], vcache[b][pos][:]
__global__ void kv_store_kernel(const _Float16* __restrict__ qkv, int d, int pos, int n_ctx,
                                _Float16* __restrict__ kc, _Float16* __restrict__ vc) {
  const int b = blockIdx.x;
  const _Float16* src = qkv + (int64_t)b * 3 * d;
  _Float16* kd = kc + ((int64_t)b * n_ctx + pos) * d;
  _Float16* vd = vc + ((int64_t)b * n_ctx + pos) * d;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    kd[i] = src[d + i];
    vd[i] = src[2 * d + i];
  }
}

void kv_store_launch(const _Float16* qkv, int d, int pos, int n_ctx, _Float16* kc, _Float16* vc,
                     int B, hipStream_t s) {
  kv_store_kernel<<<B, 256, 0, s>>>(qkv, d, pos, n_ctx, kc, vc);
  JANUS_LAUNCH_CHECK();
}

__global__ void init_tokens_kernel(int32_t* tokens, int ld, const int32_t* prompt, int plen,
                                   int32_t* done, float* sum_lp, int32_t* n_tok) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < ld; i += blockDim.x)
    tokens[(int64_t)b * ld + i] = i < plen ? prompt[i] : -1;
  if (threadIdx.x == 0) { done[b] = 0; sum_lp[b] = 0.f; n_tok[b] = 0; }
}

void init_tokens_launch(int32_t* tokens, int ld, const int32_t* prompt, int plen, int32_t* done,
                        float* sum_lp, int32_t* n_tok, int B, hipStream_t s) {
  init_tokens_kernel<<<B, 256, 0, s>>>(tokens, ld, prompt, plen, done, sum_lp, n_tok);
  JANUS_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ select
struct RowRules {
  int sample_begin;       // no token sampled yet
  int suppress_all_ts;    // last two sampled were timestamps
  int suppress_text;      // last was a timestamp, penultimate was not: text (< eot) banned
  int ts_floor;           // timestamps < ts_floor banned (-1: none)
};

__device__ __forceinline__ bool allowed(int t, const uint8_t* smask, const DecodeRules& R,
                                        const RowRules& rr, bool ban_all_text) {
  if (smask[t]) return false;
  if (rr.sample_begin && R.suppress_blank && (t == R.blank || t == R.eot)) return false;
  if (R.ts_begin >= 0) {
    if (t == R.no_timestamps) return false;
    const bool is_ts = t >= R.ts_begin;
    if (rr.suppress_all_ts && is_ts) return false;
    if (rr.suppress_text && t < R.eot) return false;
    if (is_ts && t < rr.ts_floor) return false;
    if (rr.sample_begin) {
      if (!is_ts) return false;
      if (R.max_initial_ts >= 0 && t > R.ts_begin + R.max_initial_ts) return false;
    }
    if (ban_all_text && !is_ts) return false;
  }
  return true;
}

template <class Op>
__device__ __forceinline__ float block_reduce(float v, float* red, Op op) {
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = op(r, red[k]);
  return r;
}

__global__ __launch_bounds__(256) void select_kernel(const float* __restrict__ logits, int V,
                                                     DecodeRules R, const uint8_t* __restrict__ smask,
                                                     int32_t* __restrict__ tokens, int ld, int pos,
                                                     int sample_begin_pos, int32_t* __restrict__ done,
                                                     float* __restrict__ sum_lp,
                                                     int32_t* __restrict__ n_tok) {
  __shared__ float red[8];
  __shared__ RowRules rr;
  __shared__ unsigned long long best;
  const int b = blockIdx.x, tid = threadIdx.x;
  int32_t* row_tok = tokens + (int64_t)b * ld;
  if (done[b]) {
    if (tid == 0) row_tok[pos + 1] = R.eot;
    return;
  }
  __shared__ int last_ts_pos;
  const int nsamp = pos + 1 - sample_begin_pos;  // tokens sampled so far
  if (tid == 0) { last_ts_pos = -1; best = 0ull; }
  __syncthreads();
  if (R.ts_begin >= 0) {
    int lp = -1;
    for (int i = sample_begin_pos + tid; i <= pos; i += blockDim.x)
      if (row_tok[i] >= R.ts_begin) lp = i;
    if (lp >= 0) atomicMax(&last_ts_pos, lp);
  }
  __syncthreads();
  if (tid == 0) {
    rr.sample_begin = nsamp == 0;
    rr.suppress_all_ts = rr.suppress_text = 0;
    rr.ts_floor = -1;
    if (R.ts_begin >= 0 && nsamp > 0) {
      const bool last_ts = row_tok[pos] >= R.ts_begin;
      const bool pen_ts = nsamp < 2 || row_tok[pos - 1] >= R.ts_begin;
      if (last_ts) {
        if (pen_ts) rr.suppress_all_ts = 1;
        else rr.suppress_text = 1;
      }
      if (last_ts_pos >= 0) {
        const int last_stamp = row_tok[last_ts_pos];
        rr.ts_floor = (last_ts && !pen_ts) ? last_stamp : last_stamp + 1;
      }
    }
  }
  __syncthreads();
  const RowRules rl = rr;
  const float* L = logits + (int64_t)b * V;

  // pass 1: maxima (all allowed, text, timestamps)
  float m_all = -INFINITY, m_text = -INFINITY, m_ts = -INFINITY;
  for (int t = tid; t < V; t += 256) {
    if (!allowed(t, smask, R, rl, false)) continue;
    const float v = L[t];
    m_all = fmaxf(m_all, v);
    if (R.ts_begin >= 0 && t >= R.ts_begin) m_ts = fmaxf(m_ts, v);
    else m_text = fmaxf(m_text, v);
  }
  auto fmax_op = [](float a, float c) { return fmaxf(a, c); };
  auto add_op = [](float a, float c) { return a + c; };
  m_all = block_reduce(m_all, red, fmax_op);
  m_text = block_reduce(m_text, red, fmax_op);
  m_ts = block_reduce(m_ts, red, fmax_op);
  // pass 2: partition sums
  float s_all = 0.f, s_ts = 0.f;
  for (int t = tid; t < V; t += 256) {
    if (!allowed(t, smask, R, rl, false)) continue;
    const float v = L[t];
    s_all += __expf(v - m_all);
    if (R.ts_begin >= 0 && t >= R.ts_begin) s_ts += __expf(v - m_ts);
  }
  s_all = block_reduce(s_all, red, add_op);
  s_ts = block_reduce(s_ts, red, add_op);
  const float lse_all = m_all + __logf(s_all);
  bool ban_text = false;
  float lse_final = lse_all;
  if (R.ts_begin >= 0 && m_ts > -INFINITY) {
    const float ts_lp = m_ts + __logf(s_ts) - lse_all;   // logsumexp of timestamp logprobs
    const float text_lp = m_text - lse_all;              // max text-token logprob
    if (ts_lp > text_lp) {
      ban_text = true;
      lse_final = m_ts + __logf(s_ts);
    }
  }
  // pass 3: argmax (first index on ties)
  unsigned long long key = 0ull;
  for (int t = tid; t < V; t += 256) {
    if (!allowed(t, smask, R, rl, ban_text)) continue;
    const uint32_t u = __float_as_uint(L[t]);
    const uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    const unsigned long long k = ((unsigned long long)ord << 32) | (uint32_t)(0xffffffffu - t);
    key = k > key ? k : key;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(key, o);
    key = other > key ? other : key;
  }
  if ((tid & 63) == 0) atomicMax(&best, key);
  __syncthreads();
  if (tid == 0) {
    const int next = (int)(0xffffffffu - (uint32_t)(best & 0xffffffffu));
    row_tok[pos + 1] = next;
    sum_lp[b] += L[next] - lse_final;
    n_tok[b] += 1;
    if (next == R.eot) done[b] = 1;
  }
}

void select_launch(const float* logits, int V, const DecodeRules& R, const uint8_t* smask,
                   int32_t* tokens, int ld, int pos, int sample_begin_pos, int32_t* done,
                   float* sum_lp, int32_t* n_tok, int B, hipStream_t s) {
  select_kernel<<<B, 256, 0, s>>>(logits, V, R, smask, tokens, ld, pos, sample_begin_pos, done,
                                  sum_lp, n_tok);
  JANUS_LAUNCH_CHECK();
}

__global__ void build_mask_kernel(const int32_t* __restrict__ list, int n, uint8_t* __restrict__ mask,
                                  int V) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && list[i] >= 0 && list[i] < V) mask[list[i]] = 1;
}

void build_mask_launch(const int32_t* list, int n, uint8_t* mask, int V, hipStream_t s) {
  JANUS_HIP(hipMemsetAsync(mask, 0, V, s));
  if (n > 0) {
    build_mask_kernel<<<(n + 255) / 256, 256, 0, s>>>(list, n, mask, V);
    JANUS_LAUNCH_CHECK();
  }
}

}  // namespace janus

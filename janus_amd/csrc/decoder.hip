#include <algorithm>
// Small kernels of the greedy Whisper decoder loop (batched over utterances, one
// token per step) and of the encoder/decoder glue.
//
// The token selector restates the logit filters faster-whisper's greedy path applies
// (transcribe(beam_size=1, language='en'), transcriber.py:53-57; CTranslate2
// Whisper generate with the OpenAI decoding rules: SuppressBlank, SuppressTokens,
// ApplyTimestampRules incl. max_initial_timestamp, then argmax) and accumulates the
// chosen token's log-probability (avg_logprob).
#include <cfloat>
#include <cstdlib>
#ifdef JANUS_DEBUG_ASSERT
#include <cassert>
#endif
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
// 16-column LayerNorm piece (sum, M2 about the piece mean) of 16 values spread two per
// lane over 8 aligned lanes; every lane of the group returns it.
__device__ __forceinline__ float2 ln_piece8x2(float v0, float v1) {
  float s = v0 + v1;
  s += xshfl<1>(s);
  s += xshfl<2>(s);
  s += xshfl<4>(s);
  const float m = s * (1.0f / 16.0f);
  float q = (v0 - m) * (v0 - m) + (v1 - m) * (v1 - m);
  q += xshfl<1>(q);
  q += xshfl<2>(q);
  q += xshfl<4>(q);
  return make_float2(s, q);
}

// row b's embedding at position pos (token tok) -> x[b] (+ LayerNorm pieces / the first
// layer's LayerNorm of the row); 256 threads
__device__ __forceinline__ void embed_row(const _Float16* __restrict__ tok_emb,
                                          const float* __restrict__ pos_emb, int tok, int b,
                                          int pos, int d, float* __restrict__ x,
                                          float2* __restrict__ part, const float* __restrict__ ln_g,
                                          const float* __restrict__ ln_b,
                                          _Float16* __restrict__ ln_out) {
  __shared__ float red[2][4];
  // every token read here was written by a selection or the prompt: the context rejects a
  // staggered row continued past where its slot stands (janus_whisper_decode_stand), so
  // the -1 fill is never embedded (JANUS_DEBUG_ASSERT builds check it). Release builds
  // still clamp: a path that missed the host check embeds token 0 (wrong text, no fault)
  // instead of reading before tok_emb
#ifdef JANUS_DEBUG_ASSERT
  assert(tok >= 0);
#endif
  tok = max(tok, 0);
  float v0 = 0.f, v1 = 0.f;
  for (int base = 0; base < d; base += 512) {
    const int col = base + 2 * threadIdx.x;   // 8 lanes = one 16-column piece
    v0 = 0.f; v1 = 0.f;
    if (col < d) {
      v0 = (float)tok_emb[(int64_t)tok * d + col] + pos_emb[(int64_t)pos * d + col];
      v1 = (float)tok_emb[(int64_t)tok * d + col + 1] + pos_emb[(int64_t)pos * d + col + 1];
      *reinterpret_cast<float2*>(x + (int64_t)b * d + col) = make_float2(v0, v1);
    }
    if (part) {
      const float2 pc = ln_piece8x2(v0, v1);
      if (col < d && (threadIdx.x & 7) == 0) part[(int64_t)b * (d / 16) + col / 16] = pc;
    }
  }
  if (ln_out) {  // the first layer's LayerNorm of this row (d <= 512: one pass above)
    const int col = 2 * threadIdx.x, wv = threadIdx.x >> 6;
    const bool ok = col < d;
    float s = v0 + v1;
    s = wave_sum_f32(s);
    if ((threadIdx.x & 63) == 0) red[0][wv] = s;
    __syncthreads();
    const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / d;
    float q = ok ? (v0 - mean) * (v0 - mean) + (v1 - mean) * (v1 - mean) : 0.f;
    q = wave_sum_f32(q);
    if ((threadIdx.x & 63) == 0) red[1][wv] = q;
    __syncthreads();
    const float rstd = rsqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / d + 1e-5f);
    if (ok) {
      ln_out[(int64_t)b * d + col] = (_Float16)((v0 - mean) * rstd * ln_g[col] + ln_b[col]);
      ln_out[(int64_t)b * d + col + 1] = (_Float16)((v1 - mean) * rstd * ln_g[col + 1] + ln_b[col + 1]);
    }
  }
}

__global__ __launch_bounds__(256) void embed_kernel(const _Float16* __restrict__ tok_emb,
                                                    const float* __restrict__ pos_emb,
                                                    const int32_t* __restrict__ tokens,
                                                    int ld_tokens, int pos, int d,
                                                    float* __restrict__ x,
                                                    float2* __restrict__ part,
                                                    const float* __restrict__ ln_g,
                                                    const float* __restrict__ ln_b,
                                                    _Float16* __restrict__ ln_out,
                                                    const int32_t* __restrict__ roff) {
  const int b = blockIdx.x;
  const int pb = pos + (roff ? roff[b] : 0);  // the row's own position (staggered rows)
  embed_row(tok_emb, pos_emb, tokens[(int64_t)b * ld_tokens + pb], b, pb, d, x, part, ln_g, ln_b,
            ln_out);
}

void embed_launch(const _Float16* tok_emb, const float* pos_emb, const int32_t* tokens,
                  int ld_tokens, int pos, int d, float* x, float2* part, int B, hipStream_t s,
                  const float* ln_g, const float* ln_b, _Float16* ln_out, const int32_t* roff) {
  JANUS_CHECK(d % 16 == 0, "embed: d % 16 != 0");
  JANUS_CHECK(!ln_out || d <= 512, "embed: fused LayerNorm needs d <= 512");
  embed_kernel<<<B, 256, 0, s>>>(tok_emb, pos_emb, tokens, ld_tokens, pos, d, x, part, ln_g, ln_b,
                                 ln_out, roff);
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

__global__ void init_counters_kernel(int32_t* done, float* sum_lp, int32_t* n_tok, float* nsp, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  done[b] = 0;
  sum_lp[b] = 0.f;
  n_tok[b] = 0;
  if (nsp) nsp[b] = 0.f;
}

void init_counters_launch(int32_t* done, float* sum_lp, int32_t* n_tok, float* nsp, int B,
                          hipStream_t s) {
  init_counters_kernel<<<(B + 63) / 64, 64, 0, s>>>(done, sum_lp, n_tok, nsp, B);
  JANUS_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ select
// the rules past the suppress mask, for a token whose mask byte is already in a register
__device__ __forceinline__ bool allowed_unmasked(int t, const DecodeRules& R, const RowRules& rr,
                                                 bool ban_all_text);

__device__ __forceinline__ bool allowed(int t, const uint8_t* smask, const DecodeRules& R,
                                        const RowRules& rr, bool ban_all_text) {
  if (smask[t]) return false;
  return allowed_unmasked(t, R, rr, ban_all_text);
}

__device__ __forceinline__ bool allowed_unmasked(int t, const DecodeRules& R, const RowRules& rr,
                                                 bool ban_all_text) {
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
  v = op(v, xshfl<32>(v)); v = op(v, xshfl<16>(v)); v = op(v, xshfl<8>(v));
  v = op(v, xshfl<4>(v)); v = op(v, xshfl<2>(v)); v = op(v, xshfl<1>(v));
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
    rr.last_stamp = -1;
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


// ------------------------------------------------------- fused logits path
__global__ void rules_init_kernel(RowRules* rules, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  RowRules r;
  r.sample_begin = 1;
  r.suppress_all_ts = r.suppress_text = 0;
  r.ts_floor = -1;
  r.last_stamp = -1;
  r.pad[0] = r.pad[1] = r.pad[2] = 0;
  rules[b] = r;
}

void rules_init_launch(RowRules* rules, int B, hipStream_t s) {
  rules_init_kernel<<<(B + 63) / 64, 64, 0, s>>>(rules, B);
  JANUS_LAUNCH_CHECK();
}

// one merged partial per (row, block): the grid of logits_partial_kernel
// waves per logits block (16 waves — about one tile per wave — measured 4x slower:
// 114.7 vs 28.8 us per launch)
constexpr int lg_waves(int /*K*/) { return 8; }
int logits_partial_blocks(int V, int K, int max_blocks) {
  const int cap = max_blocks > 0 ? max_blocks : 256;  // one per CU of a whole MI355X
  return std::max(1, std::min(cap, ((V + 15) / 16 + lg_waves(K) - 1) / lg_waves(K)));
}

__device__ __forceinline__ float lse_merge(float m1, float s1, float m2, float s2, float* mo) {
  const float m = fmaxf(m1, m2);
  *mo = m;
  if (m == -INFINITY) return 0.f;
  return s1 * __expf(m1 - m) + s2 * __expf(m2 - m);
}

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  return v > bv || (v == bv && i < bi);
}

// Vocabulary projection + rule-filtered statistics: logits = A[B<=64][K] . W[V][K]^T
// (W = the token embedding, tied). The 53 MB weight read once per step is the cost: each
// block stages A (all rows) in LDS once, then its 8 waves walk 16-column tiles
// independently with the next tile's weight fragments (K/32 x 16 B per lane) and its 16
// suppress-mask bytes in flight during the current tile's epilogue (the first tile's
// during the A staging). A tile's 64 x 16 logits go through a wave-private LDS patch so
// lane = row folds its 16 columns (rule filter, maxima, partition sums, argmaxes) into
// running per-row statistics without shuffles; at the end the 8 waves' statistics are
// merged per row (wave order) into ONE partial per (row, block) for the selector.

// NB: weight tiles in flight per wave (2: two register sets, the tile two strides ahead is
// issued after this tile's MFMAs, so each load has two tile-times to land)
// SAMPLE (decode at temperature > 0, faster-whisper's fallback): the argmaxes are taken
// over the perturbed keys logit * inv_temp + Gumbel noise (Gumbel-max: a draw from
// softmax(logits / T) over the same rule-filtered set), the chosen logit carried beside
// the key for the log-probability; everything else as in the greedy kernel.
template <int NKS, int NB, bool SAMPLE>  // K / 32
__global__ __launch_bounds__(lg_waves(NKS * 32) * 64) void logits_partial_kernel(
    const _Float16* __restrict__ A, int lda, const _Float16* __restrict__ W, int V, int B,
    DecodeRules R, const uint8_t* __restrict__ smask, const RowRules* __restrict__ rules,
    LogitPart* __restrict__ parts, int ntiles, const float* __restrict__ lnx, int ldx,
    const float* __restrict__ ln_g, const float* __restrict__ ln_b, int rot,
    const uint32_t* __restrict__ seeds, int pos, const float* __restrict__ rinv) {
  extern __shared__ __attribute__((aligned(16))) _Float16 lg_smem[];
  JANUS_DEC_WAVE_PRIO();
  // row group blockIdx.y: rows [64 y, 64 y + 64) of the call (one launch for every group:
  // a group's blocks start while the previous group's last blocks drain)
  {
    const int r0 = (int)blockIdx.y * 64;
    A += (int64_t)r0 * lda;
    rules += r0;
    parts += (int64_t)r0 * gridDim.x;
    if (lnx) lnx += (int64_t)r0 * ldx;
    if (seeds) seeds += r0;
    if (rinv) rinv += r0;
    B = min(64, B - r0);
  }
  constexpr int K = NKS * 32;
  constexpr int kLgWaves = lg_waves(K);
  constexpr int AP = K + 16;  // row pitch (halves): 16*AP bytes with AP/8 % 4 == 2 -> conflict-free
  _Float16* sA = lg_smem;                                            // [64][AP]
  float* sT = reinterpret_cast<float*>(sA + 64 * AP);                // [waves][64][17]
  RowRules* sR = reinterpret_cast<RowRules*>(sT + kLgWaves * 64 * 17);  // [64]
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  // the first tile's weights and suppress-mask bytes are issued before A is staged (they
  // do not depend on it); later tiles' loads are issued before the previous epilogue
  half8 bw[NB][NKS];
  uint4 sm16[NB];
#if defined(JANUS_W_NT) || defined(JANUS_LG_NT)  // A/B: token-embedding stream past the caches
#define LG_WLD(P) ([&]() { const uint4 u_ = ld_nt(P); return *reinterpret_cast<const half8*>(&u_); }())
#else
#define LG_WLD(P) (*reinterpret_cast<const half8*>(P))
#endif
  // logical tile t -> physical tile (t + rot) mod ntiles (see logits_partial_launch)
  auto phys = [&](int t) { const int q = t + rot; return q >= ntiles ? q - ntiles : q; };
#define LG_LOAD(BUF, TILE)                                                                    \
  do {                                                                                        \
    const int bcol_ = min(phys(TILE) * 16 + (lane & 15), V - 1);                              \
    const _Float16* wrow_ = W + (int64_t)bcol_ * K + 8 * (lane >> 4);                         \
    _Pragma("unroll") for (int ks = 0; ks < NKS; ++ks)                                        \
      bw[BUF][ks] = LG_WLD(wrow_ + 32 * ks);                                                  \
    /* 16 mask bytes per tile (the mask buffer is padded to a multiple of 16) */             \
    sm16[BUF] = *reinterpret_cast<const uint4*>(smask + phys(TILE) * 16);                     \
  } while (0)
  const int tile0 = blockIdx.x * kLgWaves + w;
  const int stride = gridDim.x * kLgWaves;
#pragma unroll
  for (int u = 0; u < NB; ++u)
    if (tile0 + u * stride < ntiles) LG_LOAD(u, tile0 + u * stride);
  if (lnx) {  // A = the decoder's final LayerNorm of x, computed here (one wave per row)
    // wave w: rows w + 8j (j < 8), all loads up front
    ln_rows_wave<(K + 255) / 256, 64 / kLgWaves>(lnx, ldx, w, kLgWaves, B, ln_g, ln_b, sA, w, AP, K,
                                                 1e-5f, lane);
  } else {
    for (int i = tid; i < 64 * (K / 8); i += kLgWaves * 64) {
      const int r = i / (K / 8), c8 = (i % (K / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r < B) v = *reinterpret_cast<const uint4*>(A + (int64_t)r * lda + c8);
      *reinterpret_cast<uint4*>(sA + r * AP + c8) = v;
    }
  }
  if (tid < 64) {
    RowRules rr;
    if (tid < B) rr = rules[tid];
    else { rr.sample_begin = 0; rr.suppress_all_ts = rr.suppress_text = 0; rr.ts_floor = -1; rr.last_stamp = -1; }
    sR[tid] = rr;
  }
  __syncthreads();
  float* patch = sT + w * 64 * 17;
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  RowRules rr;  // lane = row in the statistics pass (fields copied: no scratch for pad[])
  rr.sample_begin = sR[lane].sample_begin; rr.suppress_all_ts = sR[lane].suppress_all_ts;
  rr.suppress_text = sR[lane].suppress_text; rr.ts_floor = sR[lane].ts_floor;
  // this row's 1 / T (sampling): per row when the call mixes temperatures; 0 = a greedy
  // row (key = logit, as the greedy kernel)
  const float inv_t = SAMPLE && rinv ? rinv[min(lane, B - 1)] : R.inv_temp;
  // running statistics of this wave's tiles for row = lane
  float m_all = -INFINITY, s_all = 0.f, m_text = -INFINITY, m_ts = -INFINITY, s_ts = 0.f;
  float ba_v = -INFINITY, bt_v = -INFINITY;
  int ba_i = 0x7fffffff, bt_i = 0x7fffffff;
  float m_raw = -INFINITY, s_raw = 0.f, t_v = -INFINITY;  // unfiltered softmax, target logit
  float ba_r = -INFINITY, bt_r = -INFINITY;                // logits of the sampled argmaxes
  uint32_t nb = 0;                                         // row's noise base at this position
  if constexpr (SAMPLE) nb = noise_base(lane < B ? seeds[lane] : 0u, pos);
  for (int tb = tile0; tb < ntiles; tb += NB * stride) {
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int tile = tb + u * stride;
    if (tile >= ntiles) break;  // wave-uniform
    const int col0 = phys(tile) * 16;
    f32x4 acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = zero_f32x4();
    // A fragments of k-step ks+1 read while k-step ks's MFMAs run (left to the compiler,
    // every ds_read was followed by an lgkmcnt(0) wait and one MFMA: 64 exposed LDS round
    // trips per tile)
    half8 af[2][4];
#pragma unroll
    for (int m = 0; m < 4; ++m) af[0][m] = *reinterpret_cast<const half8*>(sA + (16 * m + lr) * AP + kc8);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks + 1 < NKS) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
          af[(ks + 1) & 1][m] = *reinterpret_cast<const half8*>(sA + (16 * m + lr) * AP + 32 * (ks + 1) + kc8);
      }
      // keep the reads above the MFMAs (the scheduler otherwise sinks each read to just
      // before its MFMA to save registers, re-serialising the loop)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mfma16(af[ks & 1][m], bw[u][ks], acc[m]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) patch[(16 * m + 4 * (lane >> 4) + r) * 17 + lr] = acc[m][r];
    const uint4 smc = sm16[u];
    // the tile NB strides ahead into the registers just consumed, during the epilogue
    if (tile + NB * stride < ntiles) LG_LOAD(u, tile + NB * stride);
    // wave-private patch: the wave's own stores are visible to its loads in order
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    const int row = lane;
    float t_all = -INFINITY, t_text = -INFINITY, t_ts = -INFINITY, t_raw = -INFINITY;
    float vals[16];
    unsigned okm = 0;
    float u_all = 0.f, u_ts = 0.f, u_raw = 0.f;
    auto in_tile = [&](int t) { return t >= col0 && t < col0 + 16; };
    // Plain tile (wave-uniform): 16 in-vocabulary text or special tokens, none of blank /
    // eot / no_timestamps, no timestamp: the rules then give one verdict per row for the
    // whole tile (allowed_unmasked reduces to the row flags below), and when every column
    // is allowed the filtered softmax sum IS the raw one (same maximum, same terms in the
    // same order) — half the exponentials. Bit-identical to the general path.
    const bool plain = col0 + 16 <= V && (R.ts_begin < 0 || col0 + 16 <= R.ts_begin) &&
                       !in_tile(R.blank) && !in_tile(R.eot) && !in_tile(R.no_timestamps);
    if (plain) {
      const bool row_ok = row < B && !(R.ts_begin >= 0 && ((rr.suppress_text && col0 < R.eot) || rr.sample_begin));
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float v = patch[row * 17 + c];
        vals[c] = v;
        t_raw = fmaxf(t_raw, v);
        if (col0 + c == R.target) t_v = v;
        const unsigned smw = c < 4 ? smc.x : c < 8 ? smc.y : c < 12 ? smc.z : smc.w;
        const bool ok = row_ok && !((smw >> (8 * (c & 3))) & 0xffu);
        okm |= (unsigned)ok << c;
        if (ok) t_all = fmaxf(t_all, v);
      }
      t_text = t_all;
#pragma unroll
      for (int c = 0; c < 16; ++c) u_raw += __expf(vals[c] - t_raw);
      if (okm == 0xffffu) {
        u_all = u_raw;
      } else {
#pragma unroll
        for (int c = 0; c < 16; ++c)
          if ((okm >> c) & 1u) u_all += __expf(vals[c] - t_all);
      }
      if constexpr (SAMPLE) {
        for (int c = 0; c < 16; ++c) {
          if (!((okm >> c) & 1u)) continue;
          const float key = inv_t > 0.f ? vals[c] * inv_t + sample_gumbel(nb, col0 + c) : vals[c];
          if (better(key, col0 + c, ba_v, ba_i)) { ba_v = key; ba_i = col0 + c; ba_r = vals[c]; }
        }
      } else {
#pragma unroll
        for (int c = 0; c < 16; ++c)
          if (((okm >> c) & 1u) && better(vals[c], col0 + c, ba_v, ba_i)) { ba_v = vals[c]; ba_i = col0 + c; }
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int t = col0 + c;
        const float v = patch[row * 17 + c];
        vals[c] = v;
        if (t < V) t_raw = fmaxf(t_raw, v);
        if (t == R.target) t_v = v;
        const unsigned smw = c < 4 ? smc.x : c < 8 ? smc.y : c < 12 ? smc.z : smc.w;
        const bool masked = (smw >> (8 * (c & 3))) & 0xffu;
        const bool ok = row < B && t < V && !masked && allowed_unmasked(t, R, rr, false);
        okm |= (unsigned)ok << c;
        if (ok) {
          t_all = fmaxf(t_all, v);
          if (R.ts_begin >= 0 && t >= R.ts_begin) t_ts = fmaxf(t_ts, v);
          else t_text = fmaxf(t_text, v);
        }
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) u_raw += (col0 + c < V) ? __expf(vals[c] - t_raw) : 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!((okm >> c) & 1u)) continue;
        const int t = col0 + c;
        const float v = vals[c];
        u_all += __expf(v - t_all);
        // sampling: the key (perturbed logit) is compared, the logit kept beside it
        const float key = SAMPLE && inv_t > 0.f ? v * inv_t + sample_gumbel(nb, t) : v;
        if (better(key, t, ba_v, ba_i)) { ba_v = key; ba_i = t; ba_r = v; }
        if (R.ts_begin >= 0 && t >= R.ts_begin) {
          u_ts += __expf(v - t_ts);
          if (better(key, t, bt_v, bt_i)) { bt_v = key; bt_i = t; bt_r = v; }
        }
      }
    }
    float mo;
    s_all = lse_merge(m_all, s_all, t_all, u_all, &mo); m_all = mo;
    s_ts = lse_merge(m_ts, s_ts, t_ts, u_ts, &mo); m_ts = mo;
    s_raw = lse_merge(m_raw, s_raw, t_raw, u_raw, &mo); m_raw = mo;
    m_text = fmaxf(m_text, t_text);
  }
  }
  // merge the 8 waves' statistics per row (wave order), one partial per (row, block)
  __syncthreads();  // every wave is done with its patch: reuse sT for the wave partials
  LogitPart* wp = reinterpret_cast<LogitPart*>(sT);  // [kLgWaves][64]
  {
    LogitPart p;
    p.m_all = m_all; p.s_all = s_all; p.m_text = m_text; p.m_ts = m_ts; p.s_ts = s_ts;
    p.b_all_v = ba_v; p.b_all_i = ba_i; p.b_ts_v = bt_v; p.b_ts_i = bt_i;
    p.b_all_r = SAMPLE ? ba_r : ba_v; p.b_ts_r = SAMPLE ? bt_r : bt_v;
    p.t_v = t_v; p.m_raw = m_raw; p.s_raw = s_raw;
    wp[w * 64 + lane] = p;
  }
  __syncthreads();
  if (w == 0 && lane < B) {
    LogitPart q = wp[lane];
    for (int k = 1; k < kLgWaves; ++k) {
      const LogitPart p = wp[k * 64 + lane];
      float mo;
      q.s_all = lse_merge(q.m_all, q.s_all, p.m_all, p.s_all, &mo); q.m_all = mo;
      q.s_ts = lse_merge(q.m_ts, q.s_ts, p.m_ts, p.s_ts, &mo); q.m_ts = mo;
      q.m_text = fmaxf(q.m_text, p.m_text);
      if (better(p.b_all_v, p.b_all_i, q.b_all_v, q.b_all_i)) { q.b_all_v = p.b_all_v; q.b_all_i = p.b_all_i; q.b_all_r = p.b_all_r; }
      if (better(p.b_ts_v, p.b_ts_i, q.b_ts_v, q.b_ts_i)) { q.b_ts_v = p.b_ts_v; q.b_ts_i = p.b_ts_i; q.b_ts_r = p.b_ts_r; }
      q.s_raw = lse_merge(q.m_raw, q.s_raw, p.m_raw, p.s_raw, &mo); q.m_raw = mo;
      q.t_v = fmaxf(q.t_v, p.t_v);
    }
    parts[(int64_t)lane * gridDim.x + blockIdx.x] = q;
  }
}
#undef LG_LOAD
#undef LG_WLD

void logits_partial_launch(const _Float16* A, int lda, const _Float16* W, int K, int V, int B,
                           const DecodeRules& R, const uint8_t* smask, const RowRules* rules,
                           LogitPart* parts, hipStream_t s, const float* lnx, int ldx,
                           const float* ln_g, const float* ln_b, int max_blocks,
                           const uint32_t* seeds, int pos, const float* row_inv_temp) {
  JANUS_CHECK(K == 384 || K == 512 || K == 768, "logits: K (d_model) must be 384, 512 or 768");
  const bool sample = R.inv_temp > 0.f;
  JANUS_CHECK(!sample || seeds, "logits: sampling needs per-row seeds");
  const int ntiles = (V + 15) / 16;
  const int nw = lg_waves(K);
  const size_t lds = (size_t)64 * (K + 16) * 2 + (size_t)nw * 64 * 17 * 4 + 64 * sizeof(RowRules);
  // weight tiles in flight per wave (JANUS_LG_DEPTH=2: two)
  static const int depth = ab_env("JANUS_LG_DEPTH") ? std::atoi(ab_env("JANUS_LG_DEPTH")) : 1;
  auto kern = sample ? (K == 384 ? logits_partial_kernel<12, 1, true> : K == 512 ? logits_partial_kernel<16, 1, true>
                                                                          : logits_partial_kernel<24, 1, true>)
              : depth > 1 ? (K == 384 ? logits_partial_kernel<12, 2, false> : K == 512 ? logits_partial_kernel<16, 2, false>
                                                                            : logits_partial_kernel<24, 1, false>)
                        : (K == 384 ? logits_partial_kernel<12, 1, false> : K == 512 ? logits_partial_kernel<16, 1, false>
                                                                            : logits_partial_kernel<24, 1, false>);
  static bool attr[9] = {false, false, false, false, false, false, false, false, false};
  const int ai = (K == 384 ? 0 : K == 512 ? 1 : 2) + (sample ? 6 : depth > 1 ? 3 : 0);
  if (!attr[ai]) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
    attr[ai] = true;
  }
  const int grid = logits_partial_blocks(V, K, max_blocks);
  // Tile rotation: waves take tiles t, t + stride, ...; the first ntiles % stride waves get
  // one tile more and set the kernel's length. The special tiles (eot / no_timestamps /
  // timestamps at the top of the vocabulary, and the blank token's tile) run the general
  // rule-filter epilogue, several times a plain tile's VALU work; rotated so they land in
  // the first round of the waves with one tile fewer. Order-dependent only in the last
  // bits of the softmax sums (the argmax ties break by index either way).
  static const bool no_rot = ab_env("JANUS_LG_NO_ROT") != nullptr;
  int rot = 0;
  {
    const int stride = grid * nw, rem = ntiles % stride;
    int s0 = ntiles;
    for (int t : {R.eot, R.no_timestamps, R.ts_begin})
      if (t >= 0 && t < V) s0 = std::min(s0, t / 16);
    const int nspec = ntiles - s0;
    if (!no_rot && rem > 0 && nspec > 0 && rem + nspec + (R.blank >= 0 ? 1 + R.blank / 16 : 0) <= stride)
      rot = ((s0 - rem) % ntiles + ntiles) % ntiles;
  }
  // 64 rows per row group (blockIdx.y), every group in one launch
  kern<<<dim3(grid, (B + 63) / 64), nw * 64, lds, s>>>(A, lda, W, V, B, R, smask, rules, parts, ntiles, lnx, ldx,
                                                      ln_g, ln_b, rot, seeds, pos,
                                                      sample ? row_inv_temp : nullptr);
  JANUS_LAUNCH_CHECK();
}


// One block per row: reduce the partials, apply the timestamp-probability rule, pick
// the token, accumulate its log-probability and derive the next step's row rules.
// Row b's selection at position pos; returns (in thread 0) the row's token at pos + 1:
// the selected one, eot for a finished row, the forced one inside the row's prompt.
// roff (nullable): per-row position offsets (staggered rows, janus_decode_rows.pos_offset):
// row b is at position pos + roff[b]; a row whose next position would pass the token
// buffer (pos + 1 >= ld) has finished and writes nothing (returns -1).
__device__ __forceinline__ int select_row(
    const LogitPart* __restrict__ parts, int nblk, const DecodeRules& R, RowRules* __restrict__ rules,
    int32_t* __restrict__ tokens, int ld, int pos, int32_t* __restrict__ done,
    float* __restrict__ sum_lp, int32_t* __restrict__ n_tok, const int32_t* __restrict__ plen,
    float* __restrict__ nsp, const int32_t* __restrict__ roff = nullptr) {
  __shared__ LogitPart sh[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id();
  if (roff) {
    pos += roff[b];
    if (pos + 1 >= ld) return -1;  // block-uniform
  }
  int32_t* row_tok = tokens + (int64_t)b * ld;
  const int pl = plen ? plen[b] : 1;
  if (pos + 1 < pl) return row_tok[pos + 1];  // inside this row's prompt: the forced token stays
  if (done[b]) {
    if (tid == 0) row_tok[pos + 1] = R.eot;
    return R.eot;
  }
  float m_all = -INFINITY, s_all = 0.f, m_text = -INFINITY, m_ts = -INFINITY, s_ts = 0.f;
  float ba_v = -INFINITY, bt_v = -INFINITY;
  int ba_i = 0x7fffffff, bt_i = 0x7fffffff;
  float m_raw = -INFINITY, s_raw = 0.f, t_v = -INFINITY;
  float ba_r = -INFINITY, bt_r = -INFINITY;
  const LogitPart* pr = parts + (int64_t)b * nblk;
  for (int i = tid; i < nblk; i += 256) {
    const LogitPart p = pr[i];
    float mo;
    s_all = lse_merge(m_all, s_all, p.m_all, p.s_all, &mo); m_all = mo;
    s_ts = lse_merge(m_ts, s_ts, p.m_ts, p.s_ts, &mo); m_ts = mo;
    s_raw = lse_merge(m_raw, s_raw, p.m_raw, p.s_raw, &mo); m_raw = mo;
    m_text = fmaxf(m_text, p.m_text);
    t_v = fmaxf(t_v, p.t_v);
    if (better(p.b_all_v, p.b_all_i, ba_v, ba_i)) { ba_v = p.b_all_v; ba_i = p.b_all_i; ba_r = p.b_all_r; }
    if (better(p.b_ts_v, p.b_ts_i, bt_v, bt_i)) { bt_v = p.b_ts_v; bt_i = p.b_ts_i; bt_r = p.b_ts_r; }
  }
  // butterfly over the wave (xshfl: the partner lane's values as __shfl_xor, no LDS trip)
  auto level = [&](auto shf, auto shi) __attribute__((always_inline)) {
    float mo;
    const float om = shf(m_all), os = shf(s_all);
    s_all = lse_merge(m_all, s_all, om, os, &mo); m_all = mo;
    const float tm = shf(m_ts), ts = shf(s_ts);
    s_ts = lse_merge(m_ts, s_ts, tm, ts, &mo); m_ts = mo;
    const float rm = shf(m_raw), rs = shf(s_raw);
    s_raw = lse_merge(m_raw, s_raw, rm, rs, &mo); m_raw = mo;
    m_text = fmaxf(m_text, shf(m_text));
    t_v = fmaxf(t_v, shf(t_v));
    const float av = shf(ba_v); const int ai = shi(ba_i);
    const float ar = shf(ba_r);
    if (better(av, ai, ba_v, ba_i)) { ba_v = av; ba_i = ai; ba_r = ar; }
    const float tv = shf(bt_v); const int ti = shi(bt_i);
    const float tr = shf(bt_r);
    if (better(tv, ti, bt_v, bt_i)) { bt_v = tv; bt_i = ti; bt_r = tr; }
  };
  level([](float x) { return xshfl<32>(x); }, [](int x) { return xshfl_i<32>(x); });
  level([](float x) { return xshfl<16>(x); }, [](int x) { return xshfl_i<16>(x); });
  level([](float x) { return xshfl<8>(x); }, [](int x) { return xshfl_i<8>(x); });
  level([](float x) { return xshfl<4>(x); }, [](int x) { return xshfl_i<4>(x); });
  level([](float x) { return xshfl<2>(x); }, [](int x) { return xshfl_i<2>(x); });
  level([](float x) { return xshfl<1>(x); }, [](int x) { return xshfl_i<1>(x); });
  if (lane == 0) {
    LogitPart p;
    p.m_all = m_all; p.s_all = s_all; p.m_text = m_text; p.m_ts = m_ts; p.s_ts = s_ts;
    p.b_all_v = ba_v; p.b_all_i = ba_i; p.b_ts_v = bt_v; p.b_ts_i = bt_i;
    p.t_v = t_v; p.m_raw = m_raw; p.s_raw = s_raw; p.b_all_r = ba_r; p.b_ts_r = bt_r;
    sh[w] = p;
  }
  __syncthreads();
  if (tid != 0) return -1;
  for (int k = 1; k < 4; ++k) {
    const LogitPart& p = sh[k];
    float mo;
    s_all = lse_merge(m_all, s_all, p.m_all, p.s_all, &mo); m_all = mo;
    s_ts = lse_merge(m_ts, s_ts, p.m_ts, p.s_ts, &mo); m_ts = mo;
    s_raw = lse_merge(m_raw, s_raw, p.m_raw, p.s_raw, &mo); m_raw = mo;
    m_text = fmaxf(m_text, p.m_text);
    t_v = fmaxf(t_v, p.t_v);
    if (better(p.b_all_v, p.b_all_i, ba_v, ba_i)) { ba_v = p.b_all_v; ba_i = p.b_all_i; ba_r = p.b_all_r; }
    if (better(p.b_ts_v, p.b_ts_i, bt_v, bt_i)) { bt_v = p.b_ts_v; bt_i = p.b_ts_i; bt_r = p.b_ts_r; }
  }
  // no_speech_prob: the raw softmax probability of the target token at the row's first
  // sampled step (logits at the <|startoftranscript|> position, before any filter)
  if (nsp && pos + 1 == pl) nsp[b] = R.target >= 0 ? __expf(t_v - (m_raw + __logf(s_raw))) : 0.f;
  const float lse_all = m_all + __logf(s_all);
  // the chosen token's log-probability uses its logit (b_*_r; = the key when greedy)
  int next = ba_i;
  float lp = ba_r - lse_all;
  if (R.ts_begin >= 0 && m_ts > -INFINITY) {
    const float lse_ts = m_ts + __logf(s_ts);
    if (lse_ts - lse_all > m_text - lse_all) {  // timestamp mass beats every text token
      next = bt_i;
      lp = bt_r - lse_ts;
    }
  }
  row_tok[pos + 1] = next;
  sum_lp[b] += lp;
  n_tok[b] += 1;
  if (next == R.eot) done[b] = 1;
  // rules for the next step
  RowRules r = rules[b];
  const bool last_ts = R.ts_begin >= 0 && next >= R.ts_begin;
  const bool pen_ts = r.sample_begin || (R.ts_begin >= 0 && row_tok[pos] >= R.ts_begin);
  r.sample_begin = 0;
  r.suppress_all_ts = last_ts && pen_ts;
  r.suppress_text = last_ts && !pen_ts;
  if (last_ts) r.last_stamp = next;
  r.ts_floor = r.last_stamp >= 0 ? ((last_ts && !pen_ts) ? r.last_stamp : r.last_stamp + 1) : -1;
  rules[b] = r;
  return next;
}

__global__ __launch_bounds__(256) void select_partials_kernel(
    const LogitPart* __restrict__ parts, int nblk, DecodeRules R, RowRules* __restrict__ rules,
    int32_t* __restrict__ tokens, int ld, int pos, int32_t* __restrict__ done,
    float* __restrict__ sum_lp, int32_t* __restrict__ n_tok, const int32_t* __restrict__ plen,
    float* __restrict__ nsp, const int32_t* __restrict__ roff) {
  (void)select_row(parts, nblk, R, rules, tokens, ld, pos, done, sum_lp, n_tok, plen, nsp, roff);
}

// The selection at position pos and the embedding of the chosen token at pos + 1 in one
// launch (both are per row: one block per utterance): one launch per position fewer.
// Bit-identical to select_partials_kernel followed by embed_kernel at pos + 1.
__global__ __launch_bounds__(256) void select_embed_kernel(
    const LogitPart* __restrict__ parts, int nblk, DecodeRules R, RowRules* __restrict__ rules,
    int32_t* __restrict__ tokens, int ld, int pos, int32_t* __restrict__ done,
    float* __restrict__ sum_lp, int32_t* __restrict__ n_tok, const int32_t* __restrict__ plen,
    float* __restrict__ nsp, const _Float16* __restrict__ tok_emb, const float* __restrict__ pos_emb,
    int d, float* __restrict__ x, float2* __restrict__ part, const float* __restrict__ ln_g,
    const float* __restrict__ ln_b, _Float16* __restrict__ ln_out, const int32_t* __restrict__ roff) {
  __shared__ int s_tok;
  JANUS_DEC_WAVE_PRIO();
  const int t = select_row(parts, nblk, R, rules, tokens, ld, pos, done, sum_lp, n_tok, plen, nsp, roff);
  const int pb = pos + (roff ? roff[blockIdx.x] : 0);
  if (pb + 1 >= ld) return;  // a staggered row past its last position: nothing to embed
  if (threadIdx.x == 0) s_tok = t;
  __syncthreads();
  embed_row(tok_emb, pos_emb, s_tok, blockIdx.x, pb + 1, d, x, part, ln_g, ln_b, ln_out);
}

void select_embed_launch(const LogitPart* parts, int nblk, const DecodeRules& R, RowRules* rules,
                         int32_t* tokens, int ld, int pos, int32_t* done, float* sum_lp,
                         int32_t* n_tok, int B, hipStream_t s, const int32_t* plen, float* nsp,
                         const _Float16* tok_emb, const float* pos_emb, int d, float* x,
                         float2* part, const float* ln_g, const float* ln_b, _Float16* ln_out,
                         const int32_t* roff) {
  JANUS_CHECK(d % 16 == 0, "embed: d % 16 != 0");
  JANUS_CHECK(!ln_out || d <= 512, "embed: fused LayerNorm needs d <= 512");
  select_embed_kernel<<<B, 256, 0, s>>>(parts, nblk, R, rules, tokens, ld, pos, done, sum_lp, n_tok,
                                        plen, nsp, tok_emb, pos_emb, d, x, part, ln_g, ln_b, ln_out,
                                        roff);
  JANUS_LAUNCH_CHECK();
}

void select_partials_launch(const LogitPart* parts, int nblk, const DecodeRules& R,
                            RowRules* rules, int32_t* tokens, int ld, int pos, int32_t* done,
                            float* sum_lp, int32_t* n_tok, int B, hipStream_t s,
                            const int32_t* plen, float* nsp, const int32_t* roff) {
  select_partials_kernel<<<B, 256, 0, s>>>(parts, nblk, R, rules, tokens, ld, pos, done, sum_lp,
                                           n_tok, plen, nsp, roff);
  JANUS_LAUNCH_CHECK();
}

// The sampling noise the SAMPLE logits kernel adds, written out (kernel-level ABI
// janus_sample_gumbel_f32: the CPU oracle's restatement is checked against it)
__global__ void sample_gumbel_kernel(const uint32_t* __restrict__ seeds, int pos, int V,
                                     float* __restrict__ out) {
  const int b = blockIdx.y, t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < V) out[(int64_t)b * V + t] = sample_gumbel(noise_base(seeds[b], pos), t);
}

void sample_gumbel_launch(const uint32_t* seeds, int B, int pos, int V, float* out, hipStream_t s) {
  JANUS_CHECK(B >= 1 && V >= 1, "sample_gumbel: empty shape");
  sample_gumbel_kernel<<<dim3((unsigned)cdiv(V, 256), (unsigned)B), 256, 0, s>>>(seeds, pos, V, out);
  JANUS_LAUNCH_CHECK();
}

void build_mask_launch(const int32_t* list, int n, uint8_t* mask, int V, hipStream_t s) {
  JANUS_HIP(hipMemsetAsync(mask, 0, V, s));
  if (n > 0) {
    build_mask_kernel<<<(n + 255) / 256, 256, 0, s>>>(list, n, mask, V);
    JANUS_LAUNCH_CHECK();
  }
}

}  // namespace janus

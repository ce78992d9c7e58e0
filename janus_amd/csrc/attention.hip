// Attention for the Whisper encoder (non-causal, T = 1500, head_dim 64) and decoder
// (one query per step against a K/V cache).
//
// Encoder: flash-style, fp16 MFMA 16x16x32 with fp32 online softmax (exp2 domain).
// Block = 4 waves = 64 query rows of one (b, h); each wave owns 16 rows. Q fragments
// stay in registers; 64-key K and V tiles are staged in LDS (V transposed on the way
// in so P·V reads 16-byte B fragments); P goes through a per-wave LDS tile to become
// the A operand. The S = QK^T score matrix is never materialised in HBM.
#include <cstdlib>
#include <type_traits>
#include "mfma.h"
#include "kernels.h"

namespace janus {

constexpr int kHd = 64;        // Whisper head_dim (all model sizes)
constexpr int kQT = 64;        // query rows per block
constexpr int kKT = 64;        // keys per tile
constexpr int kLS = kHd + 8;   // LDS row stride (halves): 144 B, 16-B aligned, odd x16

__global__ __launch_bounds__(256) void attention_kernel(const _Float16* __restrict__ qkv,
                                                        _Float16* __restrict__ out, int T, int H,
                                                        float scale_log2) {
  __shared__ __attribute__((aligned(16))) _Float16 sK[kKT * kLS];
  __shared__ __attribute__((aligned(16))) _Float16 sVt[kHd * kLS];
  __shared__ __attribute__((aligned(16))) _Float16 sP[4][16 * kLS];

  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int d = H * kHd;
  const int64_t ld = 3 * (int64_t)d;
  const _Float16* base = qkv + (int64_t)b * T * ld;
  const int q0 = blockIdx.x * kQT + w * 16;

  // Q fragments (A operand): row q0 + (lane&15), dims ks*32 + 8*(lane>>4) .. +7
  half8 aq[2];
  {
    const int qr = q0 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      aq[ks] = qr < T ? *reinterpret_cast<const half8*>(base + (int64_t)qr * ld + h * kHd + ks * 32 + 8 * (lane >> 4))
                      : zero_half8();
  }
  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = zero_f32x4();
  float mrow[4], lrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mrow[r] = -INFINITY; lrow[r] = 0.f; }

  for (int k0 = 0; k0 < T; k0 += kKT) {
    __syncthreads();
    // stage K tile [key][dim] and V^T tile [dim][key]; 64 keys x 8 chunks of 16 B each
    for (int idx = tid; idx < kKT * 8; idx += 256) {
      const int key = idx >> 3, c = idx & 7;
      const int kr = k0 + key;
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (kr < T) {
        const _Float16* rowp = base + (int64_t)kr * ld + h * kHd + c * 8;
        kv = *reinterpret_cast<const uint4*>(rowp + d);
        vv = *reinterpret_cast<const uint4*>(rowp + 2 * d);
      }
      *reinterpret_cast<uint4*>(sK + key * kLS + c * 8) = kv;
      const _Float16* vh = reinterpret_cast<const _Float16*>(&vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) sVt[(c * 8 + j) * kLS + key] = vh[j];
    }
    __syncthreads();

    // S = Q K^T for 4 key tiles of 16
    f32x4 s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = zero_f32x4();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const half8 bk = *reinterpret_cast<const half8*>(sK + (n * 16 + (lane & 15)) * kLS + ks * 32 + 8 * (lane >> 4));
        s[n] = mfma16(aq[ks], bk, s[n]);
      }
    }
    // scale (log2 domain), mask the tail, row max over this tile
    float tmax[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) tmax[r] = -INFINITY;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bool valid = (k0 + n * 16 + (lane & 15)) < T;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = valid ? s[n][r] * scale_log2 : -INFINITY;
        s[n][r] = v;
        tmax[r] = fmaxf(tmax[r], v);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) tmax[r] = fmaxf(tmax[r], __shfl_xor(tmax[r], off));
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(mrow[r], tmax[r]);
      alpha[r] = exp2f(mrow[r] - mn);  // mrow = -inf on the first tile -> 0
      mrow[r] = mn;
      lrow[r] *= alpha[r];
    }
    _Float16* pw = sP[w];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = exp2f(s[n][r] - mrow[r]);
        lrow[r] += pv;
        pw[(4 * (lane >> 4) + r) * kLS + n * 16 + (lane & 15)] = (_Float16)pv;
      }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[n][r] *= alpha[r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): P stores visible to this wave
    __builtin_amdgcn_wave_barrier();
    half8 ap[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      ap[ks] = *reinterpret_cast<const half8*>(pw + (lane & 15) * kLS + ks * 32 + 8 * (lane >> 4));
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const half8 bv = *reinterpret_cast<const half8*>(sVt + (n * 16 + (lane & 15)) * kLS + ks * 32 + 8 * (lane >> 4));
        o[n] = mfma16(ap[ks], bv, o[n]);
      }
    }
  }
  // row sums live spread over the 16 lanes of each row group
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) lrow[r] += __shfl_xor(lrow[r], off);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + 4 * (lane >> 4) + r;
    if (qr >= T) continue;
    const float inv = 1.0f / lrow[r];
    _Float16* orow = out + ((int64_t)b * T + qr) * d + h * kHd;
#pragma unroll
    for (int n = 0; n < 4; ++n) orow[n * 16 + (lane & 15)] = (_Float16)(o[n][r] * inv);
  }
}

// Encoder attention, transposed-score form. Each wave owns 32 queries (two 16-query
// groups) and computes S^T = K Q^T, so the MFMA output puts one query per lane (column
// l & 15) and 16 keys per lane (rows 4(l>>4) + r of the 4 key tiles): the online softmax
// needs two cross-lane shuffles per tile instead of four per row, and the exponentials
// feed O^T += V^T P^T straight from registers — lane l's own 8 probabilities of a 32-key
// chunk ARE its B fragment, under the key order k = 8g + j <-> key 16(2c + j/4) + 4g + j%4
// (g = l >> 4); the V^T A fragments are read from LDS in that same order (two 8-byte
// reads). No P round trip through LDS. K / V^T tiles are double-buffered in LDS with the
// next tile's global loads in flight during this tile's MFMAs (one barrier per tile);
// each thread stages key pairs so the transposed V writes are 4-byte and conflict-free.
constexpr int kSQW = 32;            // queries per wave
constexpr int kSQB = 4 * kSQW;      // queries per block
constexpr int kSKT = 64;            // keys per tile
constexpr int kSLK = kHd + 8;       // sK pitch (halves): 36 dwords, conflict-free 16-B reads
constexpr int kSLV = kSKT + 8;      // sVt pitch (halves): 36 dwords

// Grid: one block per (query block, head, utterance), flattened; with remap the blocks
// that share one (utterance, head) — and so read the same 384 KB of keys and values — run
// on one XCD (xcd_remap gives each XCD a contiguous run of work items), so those rows are
// fetched into one L2 instead of into every XCD's.
// JANUS_ATTN_MINB: blocks per CU the register budget is sized for (3: 168 VGPRs, no
// spills; left free the kernel takes 174 and runs 2 blocks per CU; 4 spills)
#ifndef JANUS_ATTN_MINB
#define JANUS_ATTN_MINB 3
#endif
__global__ __launch_bounds__(256, JANUS_ATTN_MINB) void attention_st_kernel(const _Float16* __restrict__ qkv,
                                                           _Float16* __restrict__ out, int T,
                                                           int H, float scale_log2, int nqb,
                                                           int remap) {
  __shared__ __attribute__((aligned(16))) _Float16 sK[2][kSKT * kSLK];
  __shared__ __attribute__((aligned(16))) _Float16 sVt[2][kHd * kSLV];

  const int item = remap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int qblk = item % nqb, h = (item / nqb) % H, b = item / (nqb * H);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, lr = lane & 15;
  const int d = H * kHd;
  const int64_t ld = 3 * (int64_t)d;
  const _Float16* base = qkv + (int64_t)b * T * ld + h * kHd;
  const int q0 = qblk * kSQB + w * kSQW;

  // Q^T B fragments: query q0 + 16 qg + lr, dims 32 ks + 8 g .. +7
  half8 qb[2][2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int qr = q0 + 16 * qg + lr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qb[qg][ks] = qr < T ? *reinterpret_cast<const half8*>(base + (int64_t)qr * ld + ks * 32 + 8 * g)
                          : zero_half8();
  }

  // staging: thread -> (16-byte dim chunk sc, key pair kp); keys 2kp, 2kp + 1
  const int sc = tid >> 5, kp = tid & 31;
  uint4 pk[2], pv[2];
  // GUARD: the tile may run past T (the last tile only; full tiles load unguarded)
  auto load_tile = [&](int k0, auto guard_c) {
    constexpr bool GUARD = decltype(guard_c)::value;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int kr = k0 + 2 * kp + e;
      const bool ok = !GUARD || kr < T;
      const _Float16* rowp = base + (int64_t)(ok ? kr : 0) * ld + sc * 8;
      pk[e] = ok ? *reinterpret_cast<const uint4*>(rowp + d) : make_uint4(0, 0, 0, 0);
      pv[e] = ok ? *reinterpret_cast<const uint4*>(rowp + 2 * d) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
      *reinterpret_cast<uint4*>(&sK[buf][(2 * kp + e) * kSLK + sc * 8]) = pk[e];
    const _Float16* v0 = reinterpret_cast<const _Float16*>(&pv[0]);
    const _Float16* v1 = reinterpret_cast<const _Float16*>(&pv[1]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __attribute__((ext_vector_type(2))) _Float16 pr = {v0[j], v1[j]};
      *reinterpret_cast<decltype(pr)*>(&sVt[buf][(sc * 8 + j) * kSLV + 2 * kp]) = pr;
    }
  };

  f32x4 o[2][4];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
#pragma unroll
    for (int m = 0; m < 4; ++m) o[qg][m] = zero_f32x4();
  float mq[2] = {-INFINITY, -INFINITY}, lq[2] = {0.f, 0.f};

  const int ntiles = (T + kSKT - 1) / kSKT;
  using False = std::false_type;
  using True = std::true_type;
  auto load_any = [&](int k0) {  // block-uniform choice
    if (k0 + kSKT <= T) load_tile(k0, False{});
    else load_tile(k0, True{});
  };
  load_any(0);
  store_tile(0);
  __syncthreads();
  // TAIL: the last, partial tile masks the keys past T (peeled, so the full tiles carry no
  // per-key compares or selects)
  auto tile_step = [&](int t, auto tail_c) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail_c)::value;
    const int buf = t & 1, k0 = t * kSKT;
    if (t + 1 < ntiles) load_any(k0 + kSKT);  // in flight during this tile
    const _Float16* K = sK[buf];
    const _Float16* Vt = sVt[buf];

    // S^T tiles: rows = keys 16n + 4g + r, column = query lr
    f32x4 st[2][4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const half8 ka0 = *reinterpret_cast<const half8*>(K + (16 * n + lr) * kSLK + 8 * g);
      const half8 ka1 = *reinterpret_cast<const half8*>(K + (16 * n + lr) * kSLK + 32 + 8 * g);
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) {
        st[qg][n] = mfma16(ka0, qb[qg][0], zero_f32x4());
        st[qg][n] = mfma16(ka1, qb[qg][1], st[qg][n]);
      }
    }
    // V^T A fragments for dim tile m, chunk c (keys in the B-fragment order)
    half8 va[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const _Float16* vr = Vt + (16 * m + lr) * kSLV + 32 * c + 4 * g;
        const half4 lo = *reinterpret_cast<const half4*>(vr);
        const half4 hi = *reinterpret_cast<const half4*>(vr + 16);
        va[m][c] = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }

    if constexpr (TAIL) {
#pragma unroll
      for (int qg = 0; qg < 2; ++qg)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (k0 + 16 * n + 4 * g + r >= T) st[qg][n][r] = -INFINITY;
    }
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      // max on raw scores (the scale is positive); p = exp2(s * scale - m) as one fma
      float tmax = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, st[qg][n][r]);
      // ds_bpermute here, not xshfl: this loop is VALU-bound and the LDS crossbar is idle
      // (the permlane form measured 490 vs 475 us per launch)
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float mn = fmaxf(mq[qg], tmax * scale_log2);
      const float alpha = __builtin_amdgcn_exp2f(mq[qg] - mn);  // mq = -inf on the first tile -> 0
      mq[qg] = mn;
      float ls = 0.f;
      half8 pb[2];
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv_ = __builtin_amdgcn_exp2f(fmaf(st[qg][n][r], scale_log2, -mn));
          ls += pv_;
          pb[n >> 1][4 * (n & 1) + r] = (_Float16)pv_;
        }
      lq[qg] = lq[qg] * alpha + ls;
      // once no query's running maximum moved (alpha == 1 exactly in every lane, the
      // common case after the first tiles) the rescale is a multiply by 1: skipped
      if (!__all(alpha == 1.0f)) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[qg][m][r] *= alpha;
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        o[qg][m] = mfma16(va[m][0], pb[0], o[qg][m]);
        o[qg][m] = mfma16(va[m][1], pb[1], o[qg][m]);
      }
    }
    if (t + 1 < ntiles) store_tile(buf ^ 1);  // its readers finished before the last barrier
    __syncthreads();
  };
  for (int t = 0; t + 1 < ntiles; ++t) tile_step(t, False{});
  if (ntiles * kSKT > T) tile_step(ntiles - 1, True{});
  else tile_step(ntiles - 1, False{});

#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    float l = lq[qg];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const int qr = q0 + 16 * qg + lr;
    if (qr >= T) continue;
    const float inv = 1.0f / l;
    _Float16* orow = out + ((int64_t)b * T + qr) * d + h * kHd;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const half4 hv = {(_Float16)(o[qg][m][0] * inv), (_Float16)(o[qg][m][1] * inv),
                        (_Float16)(o[qg][m][2] * inv), (_Float16)(o[qg][m][3] * inv)};
      *reinterpret_cast<half4*>(orow + 16 * m + 4 * g) = hv;
    }
  }
}

void attention_launch(const _Float16* qkv, _Float16* out, int B, int T, int H, float scale,
                      hipStream_t s) {
  if (B <= 0 || T <= 0) return;
  // JANUS_ATTN_V1: the first form (P through LDS, one query row per 4 lanes' registers)
  static const bool v1 = ab_env("JANUS_ATTN_V1") != nullptr;
  if (v1) {
    dim3 grid((T + kQT - 1) / kQT, H, B);
    attention_kernel<<<grid, 256, 0, s>>>(qkv, out, T, H, scale * 1.4426950408889634f);
  } else {
    // JANUS_ATTN_NO_REMAP: dispatch order (blocks of one head spread over all XCDs)
    static const int remap = ab_env("JANUS_ATTN_NO_REMAP") ? 0 : 1;
    const int nqb = (T + kSQB - 1) / kSQB;
    const int64_t nblk = (int64_t)nqb * H * B;
    JANUS_CHECK(nblk < (1ll << 31), "attention: grid too large");
    attention_st_kernel<<<(unsigned)nblk, 256, 0, s>>>(qkv, out, T, H, scale * 1.4426950408889634f,
                                                      nqb, remap);
  }
  JANUS_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- decode
// One block per (h, b): scores for all cached keys into LDS, block softmax, then
// 4 key-groups x 64 dims accumulate P·V with coalesced 128-byte V rows.
constexpr int kMaxKv = 2048;

__global__ __launch_bounds__(256) void decode_attention_kernel(
    const _Float16* __restrict__ q, int64_t q_bs, const _Float16* __restrict__ k,
    const _Float16* __restrict__ v, int64_t kv_bs, int64_t kv_rs, int Tkv,
    const int32_t* __restrict__ tkv, _Float16* __restrict__ out, int64_t o_bs, float scale) {
  __shared__ float sq[kHd];
  __shared__ float sp[kMaxKv];
  __shared__ float red[8];
  __shared__ float acc[4][kHd];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int T = tkv ? tkv[b] : Tkv;
  if (tid < kHd) sq[tid] = (float)q[(int64_t)b * q_bs + h * kHd + tid];
  __syncthreads();
  const _Float16* kb = k + (int64_t)b * kv_bs + h * kHd;
  const _Float16* vb = v + (int64_t)b * kv_bs + h * kHd;
  float mx = -INFINITY;
  for (int t = tid; t < T; t += 256) {
    const uint4* kr = reinterpret_cast<const uint4*>(kb + (int64_t)t * kv_rs);
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 u = kr[c];
      const _Float16* hh = reinterpret_cast<const _Float16*>(&u);
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += (float)hh[j] * sq[c * 8 + j];
    }
    dot *= scale;
    sp[t] = dot;
    mx = fmaxf(mx, dot);
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
  for (int t = tid; t < T; t += 256) {
    const float e = __expf(sp[t] - mx);
    sp[t] = e;
    sum += e;
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  __syncthreads();
  if ((tid & 63) == 0) red[4 + (tid >> 6)] = sum;
  __syncthreads();
  const float inv = 1.0f / (red[4] + red[5] + red[6] + red[7]);
  const int grp = tid >> 6, dd = tid & 63;
  float a = 0.f;
  for (int t = grp; t < T; t += 4) a += sp[t] * (float)vb[(int64_t)t * kv_rs + dd];
  acc[grp][dd] = a;
  __syncthreads();
  if (tid < kHd) {
    const float r = (acc[0][tid] + acc[1][tid] + acc[2][tid] + acc[3][tid]) * inv;
    out[(int64_t)b * o_bs + h * kHd + tid] = (_Float16)r;
  }
}

void decode_attention_launch(const _Float16* q, int64_t q_bs, const _Float16* k, const _Float16* v,
                             int64_t kv_bs, int64_t kv_rs, int Tkv, const int32_t* tkv,
                             _Float16* out, int64_t o_bs, int B, int H, float scale,
                             hipStream_t s) {
  JANUS_CHECK(Tkv <= kMaxKv, "decode attention: too many keys");
  if (B <= 0) return;
  decode_attention_kernel<<<dim3(H, B), 256, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, tkv, out,
                                                     o_bs, scale);
  JANUS_LAUNCH_CHECK();
}


// ------------------------------------------------------- split-key decode
// Flash-decoding for one query per (b, h): a block owns (b, key split) for ALL heads, so
// every cached key/value row (H*64 fp16 = 1 KB at d = 512) is read by one wave as one
// 16-byte-per-lane coalesced load; lane l holds dims 8l..8l+7 (head l/8). Partial
// (max, sum, unnormalised P·V) per split go to a small fp32 workspace and a second
// kernel combines the splits. HBM-bound on the K/V stream.
constexpr int kSplitKeys = 64;   // keys per split (target)
constexpr int kMaxHeads = 8;     // d <= 512

__global__ __launch_bounds__(256) void decode_split_kernel(
    const _Float16* __restrict__ q, int64_t q_bs, const _Float16* __restrict__ k,
    const _Float16* __restrict__ v, int64_t kv_bs, int64_t kv_rs, int Tkv, int H, int chunk,
    float scale_log2, float* __restrict__ part_o, float* __restrict__ part_ml) {
  __shared__ float sc[kSplitKeys * 2][kMaxHeads];
  __shared__ float acc_s[4][kMaxHeads * kHd];
  __shared__ float mh[kMaxHeads], lh[kMaxHeads];
  const int s = blockIdx.x, b = blockIdx.y, nsplit = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int d = H * kHd;
  const bool active = lane * 8 < d;
  const int head = lane >> 3;
  const int t0 = s * chunk, t1 = min(Tkv, t0 + chunk);
  float qv[8];
  {
    uint4 u = active ? *reinterpret_cast<const uint4*>(q + (int64_t)b * q_bs + lane * 8) : make_uint4(0, 0, 0, 0);
    const _Float16* h8 = reinterpret_cast<const _Float16*>(&u);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[j] = (float)h8[j] * scale_log2;
  }
  const _Float16* kb = k + (int64_t)b * kv_bs;
  const _Float16* vb = v + (int64_t)b * kv_bs;
  // issue every K and V row load of this wave before any use (<= 16 keys per wave):
  // 32 x 16 B per lane in flight hides the HBM latency of the once-read cache
  constexpr int KPW = kSplitKeys / 4;
  uint4 kr[KPW], vr[KPW];
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int t = t0 + w + 4 * i;
    kr[i] = (active && t < t1) ? *reinterpret_cast<const uint4*>(kb + (int64_t)t * kv_rs + lane * 8)
                               : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int t = t0 + w + 4 * i;
    vr[i] = (active && t < t1) ? *reinterpret_cast<const uint4*>(vb + (int64_t)t * kv_rs + lane * 8)
                               : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int t = t0 + w + 4 * i;
    const _Float16* h8 = reinterpret_cast<const _Float16*>(&kr[i]);
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dot += (float)h8[j] * qv[j];
    dot += __shfl_xor(dot, 1);
    dot += __shfl_xor(dot, 2);
    dot += __shfl_xor(dot, 4);
    if ((lane & 7) == 0 && active && t < t1) sc[t - t0][head] = dot;
  }
  __syncthreads();
  // per-head max / exp / sum over this split: wave w handles heads w, w+4
  const int nk = t1 - t0;
  for (int h = w; h < H; h += 4) {
    float m = -INFINITY;
    for (int t = lane; t < nk; t += 64) m = fmaxf(m, sc[t][h]);
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    float l = 0.f;
    for (int t = lane; t < nk; t += 64) {
      const float p = exp2f(sc[t][h] - m);
      sc[t][h] = p;
      l += p;
    }
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);
    if (lane == 0) { mh[h] = m; lh[h] = l; }
  }
  __syncthreads();
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int t = t0 + w + 4 * i;
    const _Float16* h8 = reinterpret_cast<const _Float16*>(&vr[i]);
    const float p = (active && t < t1) ? sc[t - t0][head] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += p * (float)h8[j];
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc_s[w][lane * 8 + j] = a[j];
  }
  __syncthreads();
  float* po = part_o + ((int64_t)b * nsplit + s) * d;
  for (int i = tid; i < d; i += 256) po[i] = acc_s[0][i] + acc_s[1][i] + acc_s[2][i] + acc_s[3][i];
  if (tid < H) {
    float* pm = part_ml + (((int64_t)b * nsplit + s) * H + tid) * 2;
    pm[0] = nk > 0 ? mh[tid] : -INFINITY;
    pm[1] = nk > 0 ? lh[tid] : 0.f;
  }
}

__global__ __launch_bounds__(512) void decode_combine_kernel(const float* __restrict__ part_o,
                                                             const float* __restrict__ part_ml,
                                                             int nsplit, int H,
                                                             _Float16* __restrict__ out,
                                                             int64_t o_bs) {
  __shared__ float sm[64][kMaxHeads], sl[64][kMaxHeads];
  const int b = blockIdx.x, i = threadIdx.x;  // i < d
  const int d = H * kHd;
  const float* pml = part_ml + (int64_t)b * nsplit * H * 2;
  for (int j = i; j < nsplit * H; j += blockDim.x) {
    sm[j / H][j % H] = pml[2 * j];
    sl[j / H][j % H] = pml[2 * j + 1];
  }
  __syncthreads();
  if (i >= d) return;
  const int h = i / kHd;
  float m = -INFINITY;
  for (int s = 0; s < nsplit; ++s) m = fmaxf(m, sm[s][h]);
  float l = 0.f, o = 0.f;
  const float* po = part_o + (int64_t)b * nsplit * d + i;
#pragma unroll 8
  for (int s = 0; s < nsplit; ++s) {
    const float f = exp2f(sm[s][h] - m);
    l += sl[s][h] * f;
    o += po[(int64_t)s * d] * f;
  }
  out[(int64_t)b * o_bs + i] = (_Float16)(o / l);
}

// nsplit <= 8 (self-attention up to 512 cached keys): each thread's split partials and
// the (m, l) pairs are loaded up front (one memory latency instead of two dependent ones)
constexpr int kCombRegs = 8;
__global__ __launch_bounds__(512) void decode_combine_reg_kernel(const float* __restrict__ part_o,
                                                                 const float* __restrict__ part_ml,
                                                                 int nsplit, int H,
                                                                 _Float16* __restrict__ out,
                                                                 int64_t o_bs) {
  const int b = blockIdx.x, i = threadIdx.x;
  const int d = H * kHd;
  if (i >= d) return;
  const int h = i / kHd;
  const float* pml = part_ml + (int64_t)b * nsplit * H * 2;
  const float* po = part_o + (int64_t)b * nsplit * d + i;
  float2 ml[kCombRegs];
  float ov[kCombRegs];
#pragma unroll
  for (int s = 0; s < kCombRegs; ++s) {
    if (s < nsplit) {
      ml[s] = *reinterpret_cast<const float2*>(pml + ((int64_t)s * H + h) * 2);
      ov[s] = po[(int64_t)s * d];
    }
  }
  float m = -INFINITY;
#pragma unroll
  for (int s = 0; s < kCombRegs; ++s)
    if (s < nsplit) m = fmaxf(m, ml[s].x);
  float l = 0.f, o = 0.f;
#pragma unroll
  for (int s = 0; s < kCombRegs; ++s) {
    if (s < nsplit) {
      const float f = exp2f(ml[s].x - m);
      l += ml[s].y * f;
      o += ov[s] * f;
    }
  }
  out[(int64_t)b * o_bs + i] = (_Float16)(o / l);
}

// -------------------------------------------------------- per-head decode
// Self-attention over a KV cache of at most kHeadKeys keys: one block per (head,
// utterance), so the B*H blocks fill the chip without splitting keys and no combine
// launch follows. A wave-instruction reads 8 keys x one head's 128-byte row segment
// (lane l: key l>>3, dims 8(l&7)..+7); every K and V load of the wave is issued up front
// (<= 8 + 8 x 16 B per lane). Each wave keeps its own (max, sum, P.V) and the 8 waves
// merge through LDS at the end.
constexpr int kHeadWaves = 8;
constexpr int kHeadRounds = 8;                               // key groups per wave
constexpr int kHeadKeys = 8 * kHeadWaves * kHeadRounds;      // 512

// NR: key rounds actually holding keys (ceil(Tkv / 64)): the rounds past the cache end
// only loaded the clamped last row and added p = 0 — dropping them changes no bit.
template <int NR>
__global__ __launch_bounds__(512) void decode_head_kernel(
    const _Float16* __restrict__ q, int64_t q_bs, const _Float16* __restrict__ k,
    const _Float16* __restrict__ v, int64_t kv_bs, int64_t kv_rs, int Tkv0, float scale_log2,
    _Float16* __restrict__ out, int64_t o_bs, const int32_t* __restrict__ roff) {
  __shared__ float wo[kHeadWaves][kHd];
  __shared__ float wm[kHeadWaves], wl[kHeadWaves];
  const int h = blockIdx.x, b = blockIdx.y;
  // staggered rows (roff): row b attends over its own Tkv0 + roff[b] keys; NR covers the
  // longest row, a shorter row's extra rounds load its clamped last key at weight 0
  const int Tkv = Tkv0 + (roff ? roff[b] : 0);
  const int lane = threadIdx.x & 63, w = wave_id();
  const int kg = lane >> 3, dg = lane & 7;
  float qv[8];
  {
    const uint4 u = *reinterpret_cast<const uint4*>(q + (int64_t)b * q_bs + h * kHd + dg * 8);
    const _Float16* h8 = reinterpret_cast<const _Float16*>(&u);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[j] = (float)h8[j] * scale_log2;
  }
  const _Float16* kb = k + (int64_t)b * kv_bs + h * kHd + dg * 8;
  const _Float16* vb = v + (int64_t)b * kv_bs + h * kHd + dg * 8;
  // key of round i: 8 (i * kHeadWaves + w) + kg; rows past the cache clamp to its last
  // row (finite values, weight 0) so every load is unconditional. The cache rows are read
  // non-temporal (r03 v3; JANUS_KV_PLAIN for A/B): the Infinity Cache is better spent on
  // the encoder output the cross-attention re-reads 6x per position and on the weights —
  // same-box pairs 286.8-295.6 vs 294.8-301.8 ms per step, decoder side -6 to -11 ms
  const int tl = Tkv - 1;
  uint4 kr[NR], vr[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = min(8 * (i * kHeadWaves + w) + kg, tl);
#ifndef JANUS_KV_PLAIN
    kr[i] = ld_nt(kb + (int64_t)t * kv_rs);
#else
    kr[i] = *reinterpret_cast<const uint4*>(kb + (int64_t)t * kv_rs);
#endif
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = min(8 * (i * kHeadWaves + w) + kg, tl);
#ifndef JANUS_KV_PLAIN
    vr[i] = ld_nt(vb + (int64_t)t * kv_rs);
#else
    vr[i] = *reinterpret_cast<const uint4*>(vb + (int64_t)t * kv_rs);
#endif
  }
  float sc[NR];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const _Float16* h8 = reinterpret_cast<const _Float16*>(&kr[i]);
    // explicit fmaf (here and below): left to the compiler, the contraction of these
    // sums into fma / pk_mul + add differed between NR instantiations, so a row's result
    // depended on the LONGEST row of its launch (staggered rows) in the last bits
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dot = fmaf((float)h8[j], qv[j], dot);
    dot += xshfl<1>(dot);
    dot += xshfl<2>(dot);
    dot += xshfl<4>(dot);
    const bool ok = 8 * (i * kHeadWaves + w) + kg < Tkv;
    sc[i] = ok ? dot : -INFINITY;
    m = fmaxf(m, sc[i]);
  }
  m = fmaxf(m, xshfl<8>(m));
  m = fmaxf(m, xshfl<16>(m));
  m = fmaxf(m, xshfl<32>(m));
  float l = 0.f, a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  if (m != -INFINITY) {  // wave-uniform: this wave holds at least one key
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const float p = exp2f(sc[i] - m);  // -inf -> 0
      l += p;
      const _Float16* h8 = reinterpret_cast<const _Float16*>(&vr[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = fmaf(p, (float)h8[j], a[j]);
    }
  }
  // sum over the 8 key groups (lanes sharing dg); l is replicated over dg
  auto merge = [&](auto sh) __attribute__((always_inline)) {
    l += sh(l);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += sh(a[j]);
  };
  merge([](float x) { return xshfl<8>(x); });
  merge([](float x) { return xshfl<16>(x); });
  merge([](float x) { return xshfl<32>(x); });
  if (kg == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) wo[w][dg * 8 + j] = a[j];
  }
  if (lane == 0) { wm[w] = m; wl[w] = l; }
  __syncthreads();
  if (threadIdx.x < kHd) {
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < kHeadWaves; ++i) M = fmaxf(M, wm[i]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int i = 0; i < kHeadWaves; ++i) {
      const float f = exp2f(wm[i] - M);  // empty wave: -inf -> 0
      L = fmaf(wl[i], f, L);
      O = fmaf(wo[i][threadIdx.x], f, O);
    }
    out[(int64_t)b * o_bs + h * kHd + threadIdx.x] = (_Float16)(O / L);
  }
}

int decode_split_count(int Tkv) {
  int n = (Tkv + kSplitKeys - 1) / kSplitKeys;
  return n < 1 ? 1 : n;
}

void decode_attention_split_launch(const _Float16* q, int64_t q_bs, const _Float16* k,
                                   const _Float16* v, int64_t kv_bs, int64_t kv_rs, int Tkv,
                                   _Float16* out, int64_t o_bs, int B, int H, float scale,
                                   float* part_o, float* part_ml, hipStream_t s,
                                   const int32_t* roff, int max_roff) {
  JANUS_CHECK(H <= kMaxHeads, "split decode attention: at most 8 heads (d <= 512)");
  if (B <= 0 || Tkv <= 0) return;
  static const bool force_split = ab_env("JANUS_DEC_SPLIT") != nullptr;
  const int tmax = Tkv + (roff ? max_roff : 0);
  JANUS_CHECK(!roff || tmax <= kHeadKeys, "decode attention: staggered rows need <= 512 keys");
  if (tmax <= kHeadKeys && (!force_split || part_o == nullptr || roff)) {
    static const bool all_rounds = ab_env("JANUS_HEAD_ALL_ROUNDS") != nullptr;
    const int nr = all_rounds ? kHeadRounds : (tmax + 8 * kHeadWaves - 1) / (8 * kHeadWaves);
    const float sl = scale * 1.4426950408889634f;
    const dim3 grid(H, B), blk(64 * kHeadWaves);
    switch (nr) {
      case 1: decode_head_kernel<1><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
      case 2: decode_head_kernel<2><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
      case 3: decode_head_kernel<3><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
      case 4: decode_head_kernel<4><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
      case 5: decode_head_kernel<5><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
      case 6: decode_head_kernel<6><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
      case 7: decode_head_kernel<7><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
      default: decode_head_kernel<kHeadRounds><<<grid, blk, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, sl, out, o_bs, roff); break;
    }
    JANUS_LAUNCH_CHECK();
    return;
  }
  const int nsplit = decode_split_count(Tkv);
  const int chunk = (Tkv + nsplit - 1) / nsplit;
  JANUS_CHECK(chunk <= kSplitKeys && nsplit <= 64, "split decode attention: too many keys");
  JANUS_CHECK(part_o != nullptr && part_ml != nullptr, "split decode attention: scratch missing");
  decode_split_kernel<<<dim3(nsplit, B), 256, 0, s>>>(q, q_bs, k, v, kv_bs, kv_rs, Tkv, H, chunk,
                                                      scale * 1.4426950408889634f, part_o, part_ml);
  JANUS_LAUNCH_CHECK();
  if (nsplit <= kCombRegs)
    decode_combine_reg_kernel<<<B, H * kHd, 0, s>>>(part_o, part_ml, nsplit, H, out, o_bs);
  else
    decode_combine_kernel<<<B, H * kHd, 0, s>>>(part_o, part_ml, nsplit, H, out, o_bs);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

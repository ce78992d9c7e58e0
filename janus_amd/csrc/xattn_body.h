// Absorbed cross-attention over the encoder output: the per-block body of xattn_kernel
// (xattn.hip has the derivation), shared with the decoder layer kernel (dec_persist.hip),
// which runs the one-split form as its last phase.
#pragma once
#include "mfma.h"

namespace janus {

typedef short short4v __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------ attention over enc
// Contraction order of a chunk's 32 keys in the P.E product: MFMA k index
// k = 8g + 4hf + q (g = lane>>4, hf = which of the two transposed reads, q = row in
// the read) takes key kappa(k) = 16(g>>1) + 8hf + 4(g&1) + q, so the 8 rows one
// 32-lane half reads per ds_read_b64_tr_b16 are distinct mod 8 — with a row pitch of
// D+16 halves (8 banks mod 64 per row) the half touches all 64 banks once.
__device__ __forceinline__ int xkappa(int k) {
  const int g = k >> 3, hf = (k >> 2) & 1, q = k & 3;
  return 16 * (g >> 1) + 8 * hf + 4 * (g & 1) + q;
}
__device__ __forceinline__ int xkappa_inv(int key) {
  const int g2 = key >> 4, hf = (key >> 3) & 1, g1 = (key >> 2) & 1, q = key & 3;
  return 8 * (2 * g2 + g1) + 4 * hf + q;
}

template <int D, int CH>
struct XGeo {
  static constexpr int NW = CH / 8;          // waves: CH / 16 key tiles x 2 dim halves
  static constexpr int NKT = CH / 16;        // S-phase key tiles
  static constexpr int QP = D + 16;          // sE row pitch (halves)
  static constexpr int PP = CH + 16;         // sP pitch (halves): frag_pitch(CH)
  static constexpr int KH = D / 2;           // dims per S-phase k-half
  static constexpr int KS = KH / 32;         // S-phase k-steps per wave
  static constexpr int NT = D / (16 * NW);   // C-phase 16-col tiles per wave
  static constexpr int HPW = 16 / NW;        // softmax heads per wave
  static constexpr int LDS = (CH * QP + 16 * PP) * 2 + 2 * 16 * CH * 4 + 16 * 4;
};

// CH keys per chunk: 32 (4 waves, three blocks per CU) or 64 (8 waves: half the serial
// chunk steps per split at the same registers per wave).
// PAIR (shared encoder output, r04): the block's 16 MFMA rows hold the heads of TWO decoder
// rows that attend to the same encoder output (faster-whisper's best_of hypotheses of one
// window): rows 0-7 are row b0's heads, rows 8-15 row b1's (H <= 8; b1 < 0: none), and
// the block reads encoder row e once for both — where the one-row form pads 8 heads to 16
// MFMA rows and reads E once per decoder row. pairs[blockIdx.y] = {b0, b1, e, -}.
// DIRECT (one key split, r05): the block holds the whole softmax of its row, so it writes
// c[b][h*D + j] = C / l in fp16 itself (the merge's arithmetic at one split: weight
// exp2(m - m) = 1, L = l, c = C * (1 / L)) and no merge launch follows.
// PF2 (DIRECT, r05): two chunks in flight per wave — chunk c + 2's E fragments load while
// chunk c + 1's are already in flight, so each block streams at twice the bytes per round
// trip (one block per CU on the staggered decoder's partition streams at the per-CU
// latency rate: ≈ 24 GB/s with one 64 KB chunk in flight). Same chunk order and
// arithmetic: bit-identical to the one-deep form. 32 more VGPRs: one block per CU.
// The block's work as a device function (xattn_kernel; the decoder layer kernel runs it as
// a phase, dec_persist.hip): split s of nsplit, MFMA-row group by (the utterance, or
// pairs[by]), LDS at smem (XGeo::LDS bytes). SC1Q: the query rows were written by other
// workgroups of the same launch — read them agent-coherent (sc1), not through a stale L2.
// ROWLD (DIRECT, D = 512, CH = 64): each wave loads whole 1 KB key rows (8 keys of the
// chunk, lane = 16-byte column) straight into their sE rows, and the S phase reads its B
// fragments back from sE — the fragment-pattern loads touch 16 keys x 64 B per instruction
// and stream ≈ 20 % slower per CU (tools/stream_probe.hip). One more barrier per chunk.
template <int D, int CH, bool PAIR, bool DIRECT, bool PF2, bool SC1Q = false, bool ROWLD = false>
__device__ __forceinline__ void xattn_body(
    const _Float16* __restrict__ qk, const _Float16* __restrict__ enc, int Te, int H, int kps,
    float* __restrict__ part_c, float* __restrict__ part_ml, const int4* __restrict__ pairs,
    _Float16* __restrict__ out, int s, int nsplit, int by, _Float16* smem, bool rev = false) {
  using G = XGeo<D, CH>;
  constexpr int QP = G::QP, PP = G::PP, KH = G::KH, KS = G::KS, NT = G::NT, NW = G::NW,
                NKT = G::NKT, HPW = G::HPW;
  _Float16* sE = smem;                         // [CH][QP] keys x dims
  _Float16* sP = sE + CH * QP;                 // [16][PP] heads x (permuted) keys
  float* sS = reinterpret_cast<float*>(sP + 16 * PP);  // [2][16][CH] partial scores
  float* sA = sS + 2 * 16 * CH;                // [16] rescale factors

  int b = by, b1 = -1, e = by;
  if constexpr (PAIR) {
    const int4 q = pairs[by];
    b = __builtin_amdgcn_readfirstlane(q.x);
    b1 = __builtin_amdgcn_readfirstlane(q.y);
    e = __builtin_amdgcn_readfirstlane(q.z);
  }
  // MFMA row r <-> (decoder row, head): one-row form (b, r) for r < H; PAIR (b, r) for
  // r < 8, (b1, r - 8) above
  auto row_b = [&](int r) { return (PAIR && r >= 8) ? b1 : b; };
  auto row_h = [&](int r) { return PAIR ? (r & 7) : r; };
  auto row_ok = [&](int r) { return PAIR ? ((r & 7) < H && (r < 8 || b1 >= 0)) : r < H; };
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int t0 = s * kps, t1 = min(Te, t0 + kps);
  const _Float16* eb = enc + (int64_t)e * Te * D;

  // S-phase role: key tile nt (16 keys), dims half kh; the wave's Qk fragments (rows =
  // heads, zero rows >= H) stay in registers for the whole split
  const int nt = w % NKT, kh = w / NKT;
  const int lr = lane & 15, lg = lane >> 4;
  half8 qa[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int64_t qo = ((int64_t)row_b(lr) * H + row_h(lr)) * D + kh * KH + 32 * ks + 8 * lg;
    if constexpr (SC1Q) {
      const auto rq = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(qk), 0, 0x7fffffff, 0x00020000);
      qa[ks] = row_ok(lr) ? __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rq, (uint32_t)(qo * 2), 0, 16))
                          : zero_half8();
    } else {
      qa[ks] = row_ok(lr) ? *reinterpret_cast<const half8*>(qk + qo) : zero_half8();
    }
  }
  for (int i = tid; i < 16 * PP; i += NW * 64) sP[i] = (_Float16)0.0f;  // P rows >= H stay zero

  static_assert(!ROWLD || (D == 512 && CH == 64 && DIRECT && !PAIR && KS == CH / NW),
                "row loads: one 1 KB key row per register slot");
  half8 ef[KS], eg[KS];  // eg: the second chunk in flight (PF2)
  auto load_to = [&](half8 (&dst)[KS], int t) __attribute__((always_inline)) {
    if constexpr (ROWLD) {
#pragma unroll
      for (int i = 0; i < KS; ++i) {
        const int key = min(t + (CH / NW) * w + i, t1 - 1);  // past the end: a finite row, masked
        dst[i] = *reinterpret_cast<const half8*>(eb + (int64_t)key * D + 8 * lane);
      }
      return;
    }
    // PF2: keys past the split's end load its last key instead (no branch around the loads,
    // so the wait before a chunk's first MFMA counts only the other chunk's loads as still
    // in flight); their scores are masked (-inf) and their P entries are 0, so those finite
    // rows add exact zeros to C, as the zero rows of the one-deep form do
    const int key = PF2 ? min(t + 16 * nt + lr, t1 - 1) : t + 16 * nt + lr;
    const bool ok = PF2 || key < t1;
    const _Float16* src = eb + (int64_t)key * D + kh * KH + 8 * lg;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#ifdef JANUS_XATTN_NT
    {
      const uint4 u = ok ? ld_nt(src + 32 * ks) : make_uint4(0, 0, 0, 0);
      dst[ks] = *reinterpret_cast<const half8*>(&u);
    }
#else
      dst[ks] = ok ? *reinterpret_cast<const half8*>(src + 32 * ks) : zero_half8();
#endif
  };

  f32x4 accc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) accc[n] = zero_f32x4();
  float m_run[HPW], l_run[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) { m_run[i] = -INFINITY; l_run[i] = 0.f; }

  // rev (row loads, one chunk in flight): the chunks last to first — a decoder layer whose
  // predecessor swept the encoder output forwards starts on the chunks it read last, still in
  // the Infinity Cache (the 256-row call's 393 MB per layer do not fit it)
  const int tl = t0 + ((t1 - t0 - 1) / CH) * CH;   // the last chunk's first key
  const bool rv = ROWLD && !PF2 && rev;
  const int tfirst = rv ? tl : t0, dt = rv ? -CH : CH;
  if (PF2 || t0 < t1) load_to(ef, tfirst);
  if (PF2) load_to(eg, t0 + CH);
  __syncthreads();
  // one chunk of CH keys whose E fragments are in `cur`; `cur` is refilled with the chunk
  // `ahead` chunks on (1, or 2 with PF2) once its rows are in LDS
  auto chunk = [&](int t, half8 (&cur)[KS]) __attribute__((always_inline)) {
    // ---- S partial: rows = heads, cols = keys 16nt.., k = dims of half kh
    f32x4 accs = zero_f32x4();
    if constexpr (ROWLD) {
      // the wave's 8 key rows -> sE, the next chunk's rows in flight, then the S fragments
      // from sE once every wave's rows are in
#pragma unroll
      for (int i = 0; i < KS; ++i)
        *reinterpret_cast<half8*>(sE + ((CH / NW) * w + i) * QP + 8 * lane) = cur[i];
      // (PF2: the chunk two ahead — the other register set holds the next one's rows)
      if constexpr (PF2) load_to(cur, t + 2 * CH);
      else if (t + dt < t1 && t + dt >= t0) load_to(cur, t + dt);
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        accs = mfma16(qa[ks], *reinterpret_cast<const half8*>(sE + (16 * nt + lr) * QP + kh * KH + 32 * ks + 8 * lg),
                      accs);
    } else {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) accs = mfma16(qa[ks], cur[ks], accs);
      // E rows -> LDS (row-major) for the P.E product
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        *reinterpret_cast<half8*>(sE + (16 * nt + lr) * QP + kh * KH + 32 * ks + 8 * lg) = cur[ks];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sS[(kh * 16 + 4 * lg + r) * CH + 16 * nt + lr] = accs[r];
    if constexpr (!ROWLD) {
      if constexpr (PF2) load_to(cur, t + 2 * CH);        // in flight during the next chunk
      else if (t + CH < t1) load_to(cur, t + CH);          // in flight during softmax + P.E
    }
    __syncthreads();

    // ---- online softmax: wave w owns heads w, w + NW, ...; lane = key (lanes < CH)
    const int nk = min(CH, t1 - t);
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int h = w + NW * i;  // MFMA row
      if constexpr (PAIR) {
        if (!row_ok(h)) continue;  // wave-uniform
      } else {
        if (h >= H) break;  // wave-uniform
      }
      const bool valid = lane < nk;
      const float sc = valid ? sS[h * CH + lane] + sS[(16 + h) * CH + lane] : -INFINITY;
      const float mc = wave_max_f32(sc);
      const float m_new = fmaxf(m_run[i], mc);
      const float alpha = exp2f(m_run[i] - m_new);  // 0 on the first chunk
      const float p = valid ? exp2f(sc - m_new) : 0.f;
      const float ps = wave_sum_f32(p);
      l_run[i] = l_run[i] * alpha + ps;
      m_run[i] = m_new;
      if (lane < CH) sP[h * PP + (lane & ~31) + xkappa_inv(lane & 31)] = (_Float16)p;
      if (lane == 0) sA[h] = alpha;
    }
    __syncthreads();

    // ---- C += P . E over this chunk; wave w owns dims [w*D/NW, (w+1)*D/NW)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * lg + r;
      const float al = row_ok(row) ? sA[row] : 0.f;
#pragma unroll
      for (int n = 0; n < NT; ++n) accc[n][r] *= al;
    }
    const int q = lr >> 2, pcol = 4 * (lr & 3);
    const int row0 = 16 * (lg >> 1) + 4 * (lg & 1) + q;  // kappa(8lg + q), hf = 0
#pragma unroll
    for (int kk = 0; kk < CH / 32; ++kk) {
      const half8 pa = *reinterpret_cast<const half8*>(sP + lr * PP + 32 * kk + 8 * lg);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int c0 = w * (D / NW) + 16 * n + pcol;
        const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) short4v*)(sE + (32 * kk + row0) * QP + c0));
        const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) short4v*)(sE + (32 * kk + row0 + 8) * QP + c0));
        half8 bv;
        const _Float16* l4 = reinterpret_cast<const _Float16*>(&lo);
        const _Float16* h4 = reinterpret_cast<const _Float16*>(&hi);
#pragma unroll
        for (int j = 0; j < 4; ++j) { bv[j] = l4[j]; bv[4 + j] = h4[j]; }
        accc[n] = mfma16(pa, bv, accc[n]);
      }
    }
    __syncthreads();  // sE / sS / sP are rewritten by the next chunk
  };
  if constexpr (PF2) {
    // both chunks of a pair run unconditionally inside the loop, so on every path into the
    // loop head ef's loads are the older ones (the wait before its first MFMA leaves eg's
    // eight in flight); an odd last chunk runs after it
    int t = t0;
    for (; t + CH < t1; t += 2 * CH) {
      chunk(t, ef);
      chunk(t + CH, eg);
    }
    if (t < t1) chunk(t, ef);
  } else {
    for (int t = tfirst; t < t1 && t >= t0; t += dt) chunk(t, ef);
  }

  if constexpr (DIRECT) {
    // 1 / l per head through LDS (the softmax waves own the heads), then c = C * (1 / l)
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < HPW; ++i) {
        const int h = w + NW * i;
        if (h < H) sA[h] = 1.0f / fmaf(1.0f, l_run[i], 0.0f);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * lg + r;
      if (row >= H) continue;
      const float il = sA[row];
      _Float16* o = out + ((int64_t)b * H + row) * D;
#pragma unroll
      for (int n = 0; n < NT; ++n) o[w * (D / NW) + 16 * n + lr] = (_Float16)(fmaf(1.0f, accc[n][r], 0.0f) * il);
    }
    return;
  }
  // ---- per-split partials: C of the valid rows (fp32), (m, l) per head
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * lg + r;
    if (!row_ok(row)) continue;
    float* pc = part_c + (((int64_t)row_b(row) * nsplit + s) * H + row_h(row)) * D;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#ifndef JANUS_XPART_PLAIN  // partials written / read past the caches (r03 v4; A/B switch)
      __builtin_nontemporal_store(accc[n][r], &pc[w * (D / NW) + 16 * n + lr]);
#else
      pc[w * (D / NW) + 16 * n + lr] = accc[n][r];
#endif
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int h = w + NW * i;  // MFMA row
      if (row_ok(h)) {
        float* pm = part_ml + (((int64_t)row_b(h) * nsplit + s) * H + row_h(h)) * 2;
        pm[0] = m_run[i];
        pm[1] = l_run[i];
      }
    }
  }
}


}  // namespace janus

// Decoder cross-attention over the encoder output with the K/V projections absorbed.
//
// Whisper's cross-attention for head h (faster-whisper / CTranslate2 decoder,
// transcriber.py:23-27 -> model.transcribe) is
//   q_h = LN2(x) Wq_h^T + bq_h,  K_h = enc Wk_h^T,  V_h = enc Wv_h^T + bv_h,
//   o_h = softmax(q_h K_h^T / 8) V_h,  x += concat_h(o_h) Wo^T + bo.
// Re-associating the score side (k_proj has no bias) and the value side:
//   q_h K_h^T = (q_h Wk_h) enc^T = qk_h enc^T          (qk_h: a D-vector per head)
//   o_h = p_h V_h = (p_h enc) Wv_h^T + bv_h             (p_h sums to 1)
// so per token the decoder streams the encoder output itself — D values per key shared by
// all heads — instead of per-layer K and V: half the bytes per layer, one tensor for all
// layers, and no per-window K/V projection GEMMs. The absorbed query weights
//   Wqk[h*D + j][i] = s * sum_c Wq[h*64+c][i] Wk[h*64+c][j],  bqk[h*D + j] likewise from bq
// (s = log2(e)/8: scores arrive in the exp2 domain) are built once on the device in fp32
// and stored fp16; qk = LN2(x) Wqk^T + bqk runs on the skinny GEMM, and the value side is
// the block-diagonal (per-head) skinny GEMM o = c Wv^T + bv followed by the usual
// x += o Wo^T + bo. (Folding Wv into Wo as well measured slower: a K = H*D GEMM.)
//
// xattn_kernel: block = (key split, utterance), 4 waves, chunks of 32 keys:
//   S[16 x 32]  = Qk[16 x D] . E^T        MFMA; heads padded to 16 rows; E fragments
//                                           straight from HBM into registers
//   online softmax per head (exp2), P -> fp16 LDS in a key order chosen so the
//   transposed reads below are bank-conflict-free
//   C[16 x D]  += P[16 x 32] . E[32 x D]   MFMA; E^T fragments by ds_read_b64_tr_b16
// then per-split partial (C, m, l) in fp32; xattn_combine merges the splits into
// c[b][h*D + j] fp16, the A operand of the per-head Wv GEMM.
#include "mfma.h"
#include <cstdlib>
#include "kernels.h"
#include "xattn_body.h"

namespace janus {


// ------------------------------------------------------------ weight absorption
__global__ void absorb_qk_kernel(const float* __restrict__ wq, const float* __restrict__ bq,
                                 const float* __restrict__ wk, int D, int H, float s,
                                 _Float16* __restrict__ wqk, float* __restrict__ bqk) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over H*D*D
  const int64_t total = (int64_t)H * D * D;
  if (idx < total) {
    const int i = (int)(idx % D);
    const int64_t rj = idx / D;  // h*D + j
    const int j = (int)(rj % D), h = (int)(rj / D);
    float acc = 0.f;
    for (int c = 0; c < 64; ++c)
      acc += wq[(int64_t)(h * 64 + c) * D + i] * wk[(int64_t)(h * 64 + c) * D + j];
    wqk[idx] = (_Float16)(acc * s);
  }
  if (idx < (int64_t)H * D) {
    const int j = (int)(idx % D), h = (int)(idx / D);
    float acc = 0.f;
    if (bq)
      for (int c = 0; c < 64; ++c) acc += bq[h * 64 + c] * wk[(int64_t)(h * 64 + c) * D + j];
    bqk[idx] = acc * s;
  }
}

void xattn_absorb(const float* wq, const float* bq, const float* wk, int D, int H,
                  _Float16* wqk, float* bqk, hipStream_t s) {
  JANUS_CHECK(H * 64 == D, "xattn: head_dim must be 64");
  const int64_t n = (int64_t)H * D * D;
  const float sc = 1.4426950408889634f / 8.0f;  // log2(e) / sqrt(64)
  absorb_qk_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(wq, bq, wk, D, H, sc, wqk, bqk);
  JANUS_LAUNCH_CHECK();
}

template <int D, int CH, bool PAIR = false, bool DIRECT = false, bool PF2 = false, bool ROWLD = false>
__global__ __launch_bounds__(CH * 8, (PF2 && !ROWLD) ? 1 : (CH == 32 ? (D > 512 ? 2 : 3) : 2)) void xattn_kernel(
    const _Float16* __restrict__ qk, const _Float16* __restrict__ enc, int Te, int H, int kps,
    float* __restrict__ part_c, float* __restrict__ part_ml, const int4* __restrict__ pairs,
    _Float16* __restrict__ out = nullptr, int rev = 0) {
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  JANUS_DEC_WAVE_PRIO();
  xattn_body<D, CH, PAIR, DIRECT, PF2, false, ROWLD>(qk, enc, Te, H, kps, part_c, part_ml, pairs, out,
                                                     blockIdx.x, gridDim.x, blockIdx.y, smem, rev != 0);
}

// GROUP (r04): up to 2*NMT decoder rows attending to the same encoder row — the best_of = 5
// sampled hypotheses of one window (faster-whisper's generate_with_fallback) — in ONE
// block: NMT m-tiles of 16 MFMA rows (8 per decoder row, H <= 8), so the block reads the
// window's encoder output ONCE for all of them and each E fragment (S phase) and each
// transposed E read (C phase) feeds NMT MFMAs. Per row the same MFMA k-sequence, softmax
// and merge arithmetic as xattn_kernel, so every row's partials are bit-identical to its
// one-row (or PAIR) computation. groups[g][8] = {e, row_0 .. row_{2 NMT - 1} (-1: none), -}.
// One block per CU (NMT = 3: ~220 VGPRs).
template <int D, int CH, int NMT>
__global__ __launch_bounds__(CH * 8, 1) void xattn_group_kernel(
    const _Float16* __restrict__ qk, const _Float16* __restrict__ enc, int Te, int H, int kps,
    float* __restrict__ part_c, float* __restrict__ part_ml, const int* __restrict__ groups) {
  using G = XGeo<D, CH>;
  constexpr int QP = G::QP, PP = G::PP, KH = G::KH, KS = G::KS, NT = G::NT, NW = G::NW,
                NKT = G::NKT;
  constexpr int R16 = 16 * NMT;        // MFMA rows
  constexpr int HPW = R16 / NW;        // softmax rows per wave
  constexpr int NR = 2 * NMT;          // decoder rows per group
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  _Float16* sE = smem;                          // [CH][QP] keys x dims
  _Float16* sP = sE + CH * QP;                  // [R16][PP] rows x (permuted) keys
  float* sS = reinterpret_cast<float*>(sP + R16 * PP);  // [2][R16][CH] partial scores
  float* sA = sS + 2 * R16 * CH;                // [R16] rescale factors
  // NMT = 3: the query fragments of m-tiles 1.. live in LDS (registers: m-tile 0 only), as
  // 256 VGPRs would not hold all three: sQ [NMT-1][16][D]
  constexpr int QR = NMT >= 3 ? 1 : NMT;        // m-tiles with register query fragments
  _Float16* sQ = reinterpret_cast<_Float16*>(sA + R16);

  const int s = blockIdx.x, nsplit = gridDim.x;
  const int* gp = groups + (int64_t)blockIdx.y * 8;
  const int e = __builtin_amdgcn_readfirstlane(gp[0]);
  int rb[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) rb[j] = __builtin_amdgcn_readfirstlane(gp[1 + j]);
  // MFMA row r (0 .. R16-1) <-> decoder row rb[r >> 3], head r & 7
  auto row_b = [&](int r) {
    int v = rb[0];
#pragma unroll
    for (int j = 1; j < NR; ++j) v = (r >> 3) == j ? rb[j] : v;
    return v;
  };
  auto row_ok = [&](int r) { return (r & 7) < H && row_b(r) >= 0; };
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int t0 = s * kps, t1 = min(Te, t0 + kps);
  const _Float16* eb = enc + (int64_t)e * Te * D;

  const int nt = w % NKT, kh = w / NKT;
  const int lr = lane & 15, lg = lane >> 4;
  half8 qa[QR][KS];
#pragma unroll
  for (int t = 0; t < QR; ++t) {
    const int r = 16 * t + lr;
    const bool ok = row_ok(r);
    const int qb = ok ? row_b(r) : 0;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qa[t][ks] = ok ? *reinterpret_cast<const half8*>(qk + ((int64_t)qb * H + (r & 7)) * D + kh * KH +
                                                        32 * ks + 8 * lg)
                     : zero_half8();
  }
  if constexpr (QR < NMT) {  // rows of m-tiles QR.. -> sQ, 8 halves per thread-step
    for (int i = tid; i < (NMT - QR) * 16 * (D / 8); i += NW * 64) {
      const int rr = i / (D / 8), c8 = (i % (D / 8)) * 8;
      const int r = 16 * QR + rr;
      const bool ok = row_ok(r);
      const int qb = ok ? row_b(r) : 0;
      *reinterpret_cast<half8*>(sQ + rr * D + c8) =
          ok ? *reinterpret_cast<const half8*>(qk + ((int64_t)qb * H + (r & 7)) * D + c8) : zero_half8();
    }
  }
  for (int i = tid; i < R16 * PP; i += NW * 64) sP[i] = (_Float16)0.0f;  // invalid rows stay zero

  half8 ef[KS];
  auto load_e = [&](int t) {
    const int key = t + 16 * nt + lr;
    const bool ok = key < t1;
    const _Float16* src = eb + (int64_t)key * D + kh * KH + 8 * lg;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) ef[ks] = ok ? *reinterpret_cast<const half8*>(src + 32 * ks) : zero_half8();
  };

  f32x4 accc[NMT][NT];
#pragma unroll
  for (int t = 0; t < NMT; ++t)
#pragma unroll
    for (int n = 0; n < NT; ++n) accc[t][n] = zero_f32x4();
  float m_run[HPW], l_run[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) { m_run[i] = -INFINITY; l_run[i] = 0.f; }

  if (t0 < t1) load_e(t0);
  __syncthreads();
  for (int t = t0; t < t1; t += CH) {
    // ---- S partials of every m-tile from the same E fragments
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) {
      f32x4 accs = zero_f32x4();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        half8 qf;
        if (mt < QR) qf = qa[mt < QR ? mt : 0][ks];
        else qf = *reinterpret_cast<const half8*>(sQ + ((mt - QR) * 16 + lr) * D + kh * KH + 32 * ks + 8 * lg);
        accs = mfma16(qf, ef[ks], accs);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sS[(kh * R16 + 16 * mt + 4 * lg + r) * CH + 16 * nt + lr] = accs[r];
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      *reinterpret_cast<half8*>(sE + (16 * nt + lr) * QP + kh * KH + 32 * ks + 8 * lg) = ef[ks];
    if (t + CH < t1) load_e(t + CH);
    __syncthreads();

    // ---- online softmax: wave w owns MFMA rows w, w + NW, ...; lane = key
    const int nk = min(CH, t1 - t);
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int h = w + NW * i;  // MFMA row
      if (!row_ok(h)) continue;  // wave-uniform
      const bool valid = lane < nk;
      const float sc = valid ? sS[h * CH + lane] + sS[(R16 + h) * CH + lane] : -INFINITY;
      const float mc = wave_max_f32(sc);  // the same reductions as xattn_kernel
      const float m_new = fmaxf(m_run[i], mc);
      const float alpha = exp2f(m_run[i] - m_new);
      const float p = valid ? exp2f(sc - m_new) : 0.f;
      const float ps = wave_sum_f32(p);
      l_run[i] = l_run[i] * alpha + ps;
      m_run[i] = m_new;
      if (lane < CH) sP[h * PP + (lane & ~31) + xkappa_inv(lane & 31)] = (_Float16)p;
      if (lane == 0) sA[h] = alpha;
    }
    __syncthreads();

    // ---- C += P . E: each transposed E read feeds the NMT m-tiles
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + 4 * lg + r;
        const float al = row_ok(row) ? sA[row] : 0.f;
#pragma unroll
        for (int n = 0; n < NT; ++n) accc[mt][n][r] *= al;
      }
    const int q = lr >> 2, pcol = 4 * (lr & 3);
    const int row0 = 16 * (lg >> 1) + 4 * (lg & 1) + q;
#pragma unroll
    for (int kk = 0; kk < CH / 32; ++kk) {
      half8 pa[NMT];
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt)
        pa[mt] = *reinterpret_cast<const half8*>(sP + (16 * mt + lr) * PP + 32 * kk + 8 * lg);
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
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt) accc[mt][n] = mfma16(pa[mt], bv, accc[mt][n]);
      }
    }
    __syncthreads();
  }

#pragma unroll
  for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * mt + 4 * lg + r;
      if (!row_ok(row)) continue;
      float* pc = part_c + (((int64_t)row_b(row) * nsplit + s) * H + (row & 7)) * D;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#ifndef JANUS_XPART_PLAIN
        __builtin_nontemporal_store(accc[mt][n][r], &pc[w * (D / NW) + 16 * n + lr]);
#else
        pc[w * (D / NW) + 16 * n + lr] = accc[mt][n][r];
#endif
    }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int h = w + NW * i;
      if (row_ok(h)) {
        float* pm = part_ml + (((int64_t)row_b(h) * nsplit + s) * H + (h & 7)) * 2;
        pm[0] = m_run[i];
        pm[1] = l_run[i];
      }
    }
  }
}

template <int D, int CH, int NMT>
static void xattn_group_cfg(const _Float16* qk, const _Float16* enc, int Te, int H, int nsplit,
                            float* part_c, float* part_ml, hipStream_t s, const int* groups, int ngroups) {
  const int chunks = (Te + CH - 1) / CH;
  const int kps = (chunks + nsplit - 1) / nsplit * CH;
  using G = XGeo<D, CH>;
  constexpr int R16 = 16 * NMT;
  constexpr int QR = NMT >= 3 ? 1 : NMT;
  constexpr size_t lds = (size_t)(CH * G::QP + R16 * G::PP) * 2 + (size_t)2 * R16 * CH * 4 + R16 * 4 +
                         (size_t)(NMT - QR) * 16 * D * 2;
  auto kern = xattn_group_kernel<D, CH, NMT>;
  static bool attr = false;
  if (!attr) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  kern<<<dim3(nsplit, ngroups), CH * 8, lds, s>>>(qk, enc, Te, H, kps, part_c, part_ml, groups);
  JANUS_LAUNCH_CHECK();
}

void xattn_group_launch(const _Float16* qk, const _Float16* enc, int Te, int D, int H, int nsplit,
                        float* part_c, float* part_ml, hipStream_t s, const int* groups, int ngroups,
                        int rows_per_group) {
  JANUS_CHECK(H <= 8 && (D == 384 || D == 512) && H * 64 == D, "xattn groups: H <= 8, D in {384, 512}");
  JANUS_CHECK(rows_per_group >= 1 && rows_per_group <= 6, "xattn groups: 1..6 rows per group");
  JANUS_CHECK(nsplit >= 1 && nsplit <= 63, "xattn: 1..63 key splits");
  if (ngroups <= 0 || Te <= 0) return;
  const int nmt = (rows_per_group + 1) / 2;
  if (D == 512) {
    if (nmt == 1) xattn_group_cfg<512, 64, 1>(qk, enc, Te, H, nsplit, part_c, part_ml, s, groups, ngroups);
    else if (nmt == 2) xattn_group_cfg<512, 64, 2>(qk, enc, Te, H, nsplit, part_c, part_ml, s, groups, ngroups);
    else xattn_group_cfg<512, 64, 3>(qk, enc, Te, H, nsplit, part_c, part_ml, s, groups, ngroups);
  } else {
    if (nmt == 1) xattn_group_cfg<384, 64, 1>(qk, enc, Te, H, nsplit, part_c, part_ml, s, groups, ngroups);
    else if (nmt == 2) xattn_group_cfg<384, 64, 2>(qk, enc, Te, H, nsplit, part_c, part_ml, s, groups, ngroups);
    else xattn_group_cfg<384, 64, 3>(qk, enc, Te, H, nsplit, part_c, part_ml, s, groups, ngroups);
  }
}

// c[b][h*D + j] = sum_s 2^(m_s - M) C_s[h][j] / sum_s 2^(m_s - M) l_s   (fp16)
__global__ __launch_bounds__(256) void xattn_combine_kernel(const float* __restrict__ part_c,
                                                            const float* __restrict__ part_ml,
                                                            int nsplit, int H, int D,
                                                            _Float16* __restrict__ out) {
  __shared__ float sw[16][64];  // per (head, split) weight, then 1/L in [h][63]... (nsplit <= 63)
  __shared__ float sinv[16];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* pml = part_ml + (int64_t)b * nsplit * H * 2;
  if (tid < H) {
    float M = -INFINITY;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, pml[(s * H + tid) * 2]);
    float L = 0.f;
    for (int s = 0; s < nsplit; ++s) {
      const float wgt = exp2f(pml[(s * H + tid) * 2] - M);  // empty split: m = -inf -> 0
      sw[tid][s] = wgt;
      L += wgt * pml[(s * H + tid) * 2 + 1];
    }
    sinv[tid] = 1.0f / L;
  }
  __syncthreads();
  const float* pc = part_c + (int64_t)b * nsplit * H * D;
  const int HD = H * D;
  for (int e = tid * 4; e < HD; e += 256 * 4) {
    const int h = e / D;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < nsplit; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(pc + (int64_t)s * HD + e);
      const float wgt = sw[h][s];
      acc.x += wgt * v.x; acc.y += wgt * v.y; acc.z += wgt * v.z; acc.w += wgt * v.w;
    }
    const float il = sinv[h];
    _Float16* o = out + (int64_t)b * HD + e;
    o[0] = (_Float16)(acc.x * il); o[1] = (_Float16)(acc.y * il);
    o[2] = (_Float16)(acc.z * il); o[3] = (_Float16)(acc.w * il);
  }
}

// Same merge, one block per (head, utterance) and every load issued up front: each
// thread holds its float4 of all (<= 16) split partials plus the head's (m, l) pairs, so
// the merge pays one memory latency, spread over B*H blocks instead of B.
constexpr int kXCombMax = 16;
__global__ __launch_bounds__(128) void xattn_combine_wide_kernel(const float* __restrict__ part_c,
                                                                 const float* __restrict__ part_ml,
                                                                 int nsplit, int H, int D,
                                                                 _Float16* __restrict__ out) {
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int HD = H * D;
  const float* pml = part_ml + (int64_t)b * nsplit * H * 2;
  const float* pc = part_c + (int64_t)b * nsplit * HD + (int64_t)h * D;
  float2 ml[kXCombMax];
  float4 v[kXCombMax];
  const int e = tid * 4;  // D <= 512: 128 threads x 4 dims
#pragma unroll
  for (int s = 0; s < kXCombMax; ++s) {
    if (s < nsplit) {
      ml[s] = *reinterpret_cast<const float2*>(pml + ((int64_t)s * H + h) * 2);
      v[s] = e < D ? *reinterpret_cast<const float4*>(pc + (int64_t)s * HD + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < kXCombMax; ++s)
    if (s < nsplit) M = fmaxf(M, ml[s].x);
  float L = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int s = 0; s < kXCombMax; ++s) {
    if (s < nsplit) {
      const float wgt = exp2f(ml[s].x - M);  // empty split: m = -inf -> 0
      // explicit fmaf: the fused merge + value projection below rounds identically
      L = fmaf(wgt, ml[s].y, L);
      acc.x = fmaf(wgt, v[s].x, acc.x); acc.y = fmaf(wgt, v[s].y, acc.y);
      acc.z = fmaf(wgt, v[s].z, acc.z); acc.w = fmaf(wgt, v[s].w, acc.w);
    }
  }
  if (e >= D) return;
  const float il = 1.0f / L;
  half4 o = {(_Float16)(acc.x * il), (_Float16)(acc.y * il), (_Float16)(acc.z * il), (_Float16)(acc.w * il)};
  *reinterpret_cast<half4*>(out + (int64_t)b * HD + (int64_t)h * D + e) = o;
}

// Split merge + per-head value projection in ONE launch: block = (head h, 4 rows); phase
// 1 merges the rows' split partials of head h (xattn_combine_wide_kernel's arithmetic) into
// an fp16 LDS tile, phase 2 is the block-diagonal projection o[r][64h + j] = c[r][h] .
// Wv[64h + j]^T + bv (gemm_skinny_kernel's arithmetic: 16 waves, one 32-deep k-step each,
// partials summed as (p_0 + p_8) + ... + (p_7 + p_15)) — bit-identical to the two launches
// it replaces. Each block reads its rows' partials once (4 x nsplit x D fp32) and the
// head's 64 x D weight slice.
constexpr int kCvpRows = 4;
template <int D>
__global__ __launch_bounds__(1024) void xattn_combine_vproj_kernel(
    const float* __restrict__ part_c, const float* __restrict__ part_ml, int nsplit, int H, int B,
    const _Float16* __restrict__ wv, const float* __restrict__ bv, _Float16* __restrict__ out,
    int64_t ldo) {
  constexpr int AP = frag_pitch(D);
  constexpr int KS = D / 32;  // k-steps (<= 16: one per wave)
  static_assert(KS <= 16, "D <= 512");
  __shared__ __attribute__((aligned(16))) _Float16 sA[16 * AP];
  __shared__ float red[4][8][16][17];
  const int h = blockIdx.x, r0 = blockIdx.y * kCvpRows;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int HD = H * D;
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  // weight fragments of this wave's k-step for the head's 4 column tiles: in flight first
  half8 bw[4];
  const bool kok = w < KS;  // wave-uniform
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const _Float16* wr = wv + (int64_t)(h * 64 + 16 * t + lr) * D + 32 * w + kc8;
    bw[t] = kok ? *reinterpret_cast<const half8*>(wr) : zero_half8();
  }
  const int ecol = tid & 63, erow = tid >> 6;  // epilogue: rows < kCvpRows, 64 columns
  const float e_add = (erow < kCvpRows && bv) ? bv[h * 64 + ecol] : 0.0f;
  // phase 1: merge, 2 dims per thread (rows r0 + tid / (D/2))
  for (int i = tid; i < 16 * (D / 2); i += 1024) {
    const int rr = i / (D / 2), e = (i % (D / 2)) * 2;
    const int b = r0 + rr;
    half2v o = {(_Float16)0.0f, (_Float16)0.0f};
    if (rr < kCvpRows && b < B) {
      const float* pml = part_ml + (int64_t)b * nsplit * H * 2;
      const float* pc = part_c + (int64_t)b * nsplit * HD + (int64_t)h * D + e;
      float2 ml[kXCombMax], v[kXCombMax];
#pragma unroll
      for (int s = 0; s < kXCombMax; ++s) {
        if (s < nsplit) {
          ml[s] = *reinterpret_cast<const float2*>(pml + ((int64_t)s * H + h) * 2);
#ifndef JANUS_XPART_PLAIN
        {
          typedef float f2v __attribute__((ext_vector_type(2)));
          const f2v t = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(pc + (int64_t)s * HD));
          v[s] = make_float2(t.x, t.y);
        }
#else
          v[s] = *reinterpret_cast<const float2*>(pc + (int64_t)s * HD);
#endif
        }
      }
      float M = -INFINITY;
#pragma unroll
      for (int s = 0; s < kXCombMax; ++s)
        if (s < nsplit) M = fmaxf(M, ml[s].x);
      float L = 0.f, a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int s = 0; s < kXCombMax; ++s) {
        if (s < nsplit) {
          const float wgt = exp2f(ml[s].x - M);
          L = fmaf(wgt, ml[s].y, L);
          a0 = fmaf(wgt, v[s].x, a0);
          a1 = fmaf(wgt, v[s].y, a1);
        }
      }
      const float il = 1.0f / L;
      o = half2v{(_Float16)(a0 * il), (_Float16)(a1 * il)};
    }
    *reinterpret_cast<half2v*>(sA + rr * AP + e) = o;
  }
  __syncthreads();
  // phase 2: one k-step per wave, four column tiles
  f32x4 acc[4];
  {
    const half8 af = kok ? *reinterpret_cast<const half8*>(sA + lr * AP + 32 * w + kc8) : zero_half8();
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = mfma16(af, bw[t], zero_f32x4());
  }
  if (w < 8) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[t][w][4 * (lane >> 4) + r][lr] = acc[t][r];
  }
  __syncthreads();
  if (w >= 8) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[t][w - 8][4 * (lane >> 4) + r][lr] += acc[t][r];
  }
  __syncthreads();
  if (erow < kCvpRows && r0 + erow < B) {
    const int t = ecol >> 4, c = ecol & 15;
    float v = e_add;
#pragma unroll
    for (int i = 0; i < 8; ++i) v += red[t][i][erow][c];
    out[(int64_t)(r0 + erow) * ldo + h * 64 + ecol] = (_Float16)v;
  }
}

bool xattn_cvp_supported(int D, int H) { return H * 64 == D && (D == 384 || D == 512); }

void xattn_combine_vproj_launch(const float* part_c, const float* part_ml, int nsplit, int B, int H,
                                int D, const _Float16* wv, const float* bv, _Float16* out, int64_t ldo,
                                hipStream_t s) {
  JANUS_CHECK(xattn_cvp_supported(D, H), "xattn combine+vproj: D = 64 H in {384, 512}");
  JANUS_CHECK(nsplit >= 1 && nsplit <= kXCombMax, "xattn combine+vproj: 1..16 key splits");
  if (B <= 0) return;
  const dim3 grid(H, (B + kCvpRows - 1) / kCvpRows);
  if (D == 512)
    xattn_combine_vproj_kernel<512><<<grid, 1024, 0, s>>>(part_c, part_ml, nsplit, H, B, wv, bv, out, ldo);
  else
    xattn_combine_vproj_kernel<384><<<grid, 1024, 0, s>>>(part_c, part_ml, nsplit, H, B, wv, bv, out, ldo);
  JANUS_LAUNCH_CHECK();
}

int xattn_split_count(int Te, int requested) {
  int n = requested > 0 ? requested : 8;  // 512 blocks at batch 64 (bench sweep: 8 < 6, 10, 12)
  n = std::min(n, 63);
  n = std::min(n, (Te + 63) / 64);  // at least one 64-key chunk per split
  return std::max(n, 1);
}

#ifndef JANUS_XATTN_FRAG
constexpr bool kXattnRow = true;   // one-split D = 512: whole-row loads (ROWLD)
#else
constexpr bool kXattnRow = false;  // A/B build: the fragment-pattern loads
#endif
// one-split row loads with two chunks in flight per wave (two register sets of 8 rows):
// 158 VGPRs, one block per CU — measured slower at 256 rows (decoder 1539 vs 1444 us per
// position in the staggered step, profiles/r06_xattn_ab.txt); A/B build only
#ifdef JANUS_XATTN_ROW2
constexpr bool kXattnRowPF2 = true;
#else
constexpr bool kXattnRowPF2 = false;
#endif
#ifndef JANUS_XATTN_PF1
constexpr bool kXattnPF2 = true;
#else
constexpr bool kXattnPF2 = false;  // A/B build: one chunk in flight
#endif
template <int D, int CH>
static void xattn_cfg(const _Float16* qk, const _Float16* enc, int B, int Te, int H, int nsplit,
                      float* part_c, float* part_ml, hipStream_t s, const int4* pairs, int npairs,
                      _Float16* out = nullptr, bool rev = false) {
  const int chunks = (Te + CH - 1) / CH;
  const int kps = (chunks + nsplit - 1) / nsplit * CH;
  const bool direct = out != nullptr;
  constexpr bool row = kXattnRow && D == 512 && CH == 64;
  decltype(&xattn_kernel<D, CH, false>) kern;
  if (direct) {
    if constexpr (row) kern = kXattnRowPF2 ? xattn_kernel<D, CH, false, true, true, true>
                                           : xattn_kernel<D, CH, false, true, false, true>;
    else kern = xattn_kernel<D, CH, false, true, kXattnPF2>;
  } else {
    kern = pairs ? xattn_kernel<D, CH, true> : xattn_kernel<D, CH, false>;
  }
  const int ai = direct ? 2 : pairs != nullptr;
  static bool attr[3] = {false, false, false};
  if (!attr[ai]) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
    attr[ai] = true;
  }
  kern<<<dim3(nsplit, pairs ? npairs : B), CH * 8, XGeo<D, CH>::LDS, s>>>(qk, enc, Te, H, kps, part_c,
                                                                         part_ml, pairs, out, rev ? 1 : 0);
  JANUS_LAUNCH_CHECK();
}

bool xattn_supported(int D, int H) {
  return H * 64 == D && H <= 16 && (D == 384 || D == 512 || D == 768);
}

void xattn_launch(const _Float16* qk, const _Float16* enc, int B, int Te, int D, int H,
                  int nsplit, float* part_c, float* part_ml, _Float16* out, hipStream_t s,
                  bool combine, const int4* pairs, int npairs, bool rev) {
  JANUS_CHECK(xattn_supported(D, H), "xattn: need D = 64 H in {384, 512, 768}");
  if (B <= 0 || Te <= 0) return;
  JANUS_CHECK(nsplit >= 1 && nsplit <= 63, "xattn: 1..63 key splits");
  JANUS_CHECK(!pairs || (H <= 8 && npairs >= 1 && D <= 512), "xattn: row pairs need H <= 8, D <= 512");
  // 64-key chunks (8 waves) unless JANUS_XATTN_CH32
  static const bool ch32 = ab_env("JANUS_XATTN_CH32") != nullptr;
  // one key split with the merge requested: the kernel writes c itself (DIRECT), no merge
  if (combine && nsplit == 1 && !pairs && !ch32 && D <= 512) {
    if (D == 384) xattn_cfg<384, 64>(qk, enc, B, Te, H, 1, part_c, part_ml, s, nullptr, 0, out);
    else xattn_cfg<512, 64>(qk, enc, B, Te, H, 1, part_c, part_ml, s, nullptr, 0, out, rev);
    return;
  }
  if (D == 384) {
    if (ch32) xattn_cfg<384, 32>(qk, enc, B, Te, H, nsplit, part_c, part_ml, s, pairs, npairs);
    else xattn_cfg<384, 64>(qk, enc, B, Te, H, nsplit, part_c, part_ml, s, pairs, npairs);
  } else if (D == 512) {
    if (ch32) xattn_cfg<512, 32>(qk, enc, B, Te, H, nsplit, part_c, part_ml, s, pairs, npairs);
    else xattn_cfg<512, 64>(qk, enc, B, Te, H, nsplit, part_c, part_ml, s, pairs, npairs);
  } else {
    xattn_cfg<768, 32>(qk, enc, B, Te, H, nsplit, part_c, part_ml, s, nullptr, 0);
  }
  if (!combine) return;  // the caller merges (xattn_combine_vproj_launch)
  if (nsplit <= kXCombMax && D <= 512)
    xattn_combine_wide_kernel<<<dim3(H, B), 128, 0, s>>>(part_c, part_ml, nsplit, H, D, out);
  else
    xattn_combine_kernel<<<B, 256, 0, s>>>(part_c, part_ml, nsplit, H, D, out);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

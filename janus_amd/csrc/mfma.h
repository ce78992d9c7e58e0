// MFMA fragment helpers for gfx950 (CDNA4): v_mfma_f32_16x16x32_f16.
//
// Lane maps (cdna_hip_programming.md §3): lane l holds A[row l&15][k 8(l>>4)+j] and
// B[k 8(l>>4)+j][col l&15], j = 0..7 (16 B per lane); C/D: col l&15,
// row 4(l>>4)+r, r = 0..3.
#pragma once
#include "common.h"

namespace janus {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(const half8& a, const half8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the fp16 rounding of
// every consumer): branchless, one v_rcp and one v_exp, where the library erff's
// piecewise polynomial diverges within a wave. The encoder's fc1 epilogue evaluates it
// on 2048 columns of every row.
__device__ __forceinline__ float erf_fast(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float e = __builtin_amdgcn_exp2f(-a * a * 1.4426950408889634f);
  return copysignf(fmaf(-y, e, 1.0f), x);
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}

// __shfl_xor(v, O) over a full wave without the LDS crossbar: the partner lane's value,
// bit for bit, so every butterfly reduction keeps its association. O = 1, 2: quad_perm;
// 8: row_ror:8; 4: row_shl:4 / row_shr:4 and a select; 16, 32: v_permlane16_swap /
// v_permlane32_swap (gfx950) and a select. Each is a few VALU cycles where a ds_bpermute
// is an LDS round trip, and reductions chain six of them (a softmax's max and sum, a
// LayerNorm's two moments). All 64 lanes must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int O>
__device__ __forceinline__ float xshfl(float v) {
  static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16 || O == 32, "xor offset");
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if constexpr (O == 1) return dpp_f32<0xB1>(v);        // quad_perm [1, 0, 3, 2]
  else if constexpr (O == 2) return dpp_f32<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  else if constexpr (O == 8) return dpp_f32<0x128>(v);  // row_ror:8
  else if constexpr (O == 4) {
    const float up = dpp_f32<0x104>(v), dn = dpp_f32<0x114>(v);  // row_shl:4 / row_shr:4
    return (lane & 4) ? dn : up;
  } else if constexpr (O == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v),
                                                    __builtin_bit_cast(unsigned, v), false, false);
    return __builtin_bit_cast(float, (unsigned)((lane & 16) ? r[0] : r[1]));
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v),
                                                    __builtin_bit_cast(unsigned, v), false, false);
    return __builtin_bit_cast(float, (unsigned)((lane & 32) ? r[0] : r[1]));
  }
}
// Wave priority of the decoder's kernels: the YIN blocks that share the decoder's CUs keep
// priority 0, so the latency-bound decoder phases win the issue arbitration on a shared
// SIMD and YIN takes the cycles they leave (decoder side -4 to -5 ms per step at the same
// YIN share; with a sixth packet of vocoder work moved to it, 241.4-241.7 vs 243.6-244.0 ms
// per step, profiles/r05_dec_prio_ab.txt). -DJANUS_DEC_PRIO=0 builds the old order.
#ifndef JANUS_DEC_PRIO
#define JANUS_DEC_PRIO 3
#endif
#define JANUS_DEC_WAVE_PRIO() __builtin_amdgcn_s_setprio(JANUS_DEC_PRIO)

template <int O>
__device__ __forceinline__ int xshfl_i(int v) {
  return __builtin_bit_cast(int, xshfl<O>(__builtin_bit_cast(float, v)));  // moves only: bits kept
}
// butterfly sum / max over the whole wave (the __shfl_xor 32, 16, ..., 1 order)
__device__ __forceinline__ float wave_sum_f32(float v) {
  v += xshfl<32>(v); v += xshfl<16>(v); v += xshfl<8>(v);
  v += xshfl<4>(v); v += xshfl<2>(v); v += xshfl<1>(v);
  return v;
}
__device__ __forceinline__ float wave_max_f32(float v) {
  v = fmaxf(v, xshfl<32>(v)); v = fmaxf(v, xshfl<16>(v)); v = fmaxf(v, xshfl<8>(v));
  v = fmaxf(v, xshfl<4>(v)); v = fmaxf(v, xshfl<2>(v)); v = fmaxf(v, xshfl<1>(v));
  return v;
}

// x * sigmoid(x) with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of the
// ~10-instruction IEEE division: SiLU runs on every staged vocoder activation.
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}

// SiLU of 8 staged fp16 activations. Default: each through fp32 (silu above) and rounded
// once. JANUS_SILU_F16: fp16 arithmetic (v_exp_f16 / v_rcp_f16, packed multiplies), no
// conversions — a few fp16 ulps instead of half of one.
__device__ __forceinline__ half8 silu_h8(half8 v) {
#ifdef JANUS_SILU_F16
  const half8 t = v * (_Float16)(-1.4426950408889634f);
  half8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = __builtin_amdgcn_rcph((_Float16)1.0f + __builtin_elementwise_exp2(t[j]));
  return v * r;
#else
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (_Float16)silu((float)v[j]);
  return v;
#endif
}

// Streaming activation traffic of the vocoder (tiles read once per unit, outputs written
// once): with JANUS_ACT_NT the accesses carry the non-temporal hint, so the multi-GB
// vocoder stream does not displace what the concurrently running decoder re-reads
// (encoder output, weights) from the caches.
// Measured (overlapped bench step, r02): non-temporal OUTPUT stores — 324.3 -> 319.3 ms,
// both sides faster (decoder -5.5 ms: its re-read encoder output and weights survive in
// the caches; vocoder -3 ms); non-temporal loads as well then cost the vocoder +4.5 ms
// (the tile's halo / residual re-reads missed) for a -3 ms decoder. r03 v3: with the wide
// units' residual resident and the vocoder side ~11 ms shorter than the decoder's, every
// activation access is non-temporal by default: decoder side 278.4 -> 275.7 ms, vocoder
// side +2 ms, step 289.6-290.7 -> 287.2-287.9 ms (A/B on one box; the staging loads alone
// change nothing, the gain is the residual / accumulator re-reads).
// Switches for A/B builds: JANUS_ACT_LD_PLAIN (plain loads), or JANUS_ACT_NT_LD /
// JANUS_ACT_NT_RES alone (tile staging loads / epilogue re-reads); JANUS_ACT_ST_PLAIN
// (plain stores).
#ifndef JANUS_ACT_LD_PLAIN
#ifndef JANUS_ACT_NT_LD
#define JANUS_ACT_NT_LD
#endif
#ifndef JANUS_ACT_NT_RES
#define JANUS_ACT_NT_RES
#endif
#endif
#ifndef JANUS_ACT_ST_PLAIN
#define JANUS_ACT_NT_ST
#endif
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const _Float16* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ld_act(const _Float16* p) {  // tile staging
#ifdef JANUS_ACT_NT_LD
  return ld_nt(p);
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}
// Tile staging with the halo rows a neighbouring tile re-reads kept in L2 (r04): a row read
// by two tiles (the (k-1)d + halo-recompute rows at either end of a tile's window) is
// loaded with the default policy so the neighbour (same XCD: tile_remap) finds it in L2;
// rows only this tile reads stay non-temporal. `keep` must be wave-uniform (one load form
// per wave, no exec-masked pair). JANUS_HALO_NT: every staging load non-temporal (r03).
// Default since r04 (staggered step): the C = 64 / 32 callers keep EVERY staged row (their
// epilogues re-read the body rows as the residual): traffic 1.26 / 1.36x -> 1.00 / 1.00x of
// the algorithmic bytes, step level-to-better in two same-box pairs (266.2 / 266.9 vs 266.6
// / 267.7 ms). JANUS_STAGE_HALO_ONLY (A/B build): only the halo rows kept, as r04 v2.
#ifdef JANUS_STAGE_HALO_ONLY
#define JANUS_STAGE_KEEP_ALL 0
#else
#define JANUS_STAGE_KEEP_ALL 1
#endif
__device__ __forceinline__ uint4 ld_act_halo(const _Float16* p, bool keep) {
#if defined(JANUS_ACT_NT_LD) && !defined(JANUS_HALO_NT)
  if (keep) return *reinterpret_cast<const uint4*>(p);
  return ld_nt(p);
#else
  (void)keep;
  return ld_act(p);
#endif
}
__device__ __forceinline__ uint4 ld_res(const _Float16* p) {  // epilogue re-reads
#ifdef JANUS_ACT_NT_RES
  return ld_nt(p);
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}
// Write-through (sc1) vector stores: the line leaves the XCD's L2 with the store, so no
// dirty vocoder line is left for a kernel-boundary L2 writeback to flush (the greedy
// decoder beside the vocoder shares every XCD's L2 and ends ~68 kernels per position).
// Plain / nt stores KEEP the line dirty in L2 (MI355X_MICROARCH.md, store flavours).
// Inline asm: hipcc counts no asm store; s_endpgm waits for them, and nothing in the
// kernel re-reads a stored activation.
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_wt16(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_wt8(void* p, u32x2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_act(_Float16* p, const half8& v) {
#if defined(JANUS_ACT_WT)
  st_wt16(p, __builtin_bit_cast(u32x4, v));
#elif defined(JANUS_ACT_NT_ST)
  __builtin_nontemporal_store(v, reinterpret_cast<half8*>(p));
#else
  *reinterpret_cast<half8*>(p) = v;
#endif
}

__device__ __forceinline__ half8 zero_half8() {
  half8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (_Float16)0.0f;
  return z;
}

// Wave index within the block as a wave-uniform (SGPR) value: tid >> 6 alone is a VGPR
// to the compiler, so branches on it (m-tile / head ownership) became exec-masked
// branches with accumulators shuttled through VGPRs around every MFMA.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ f32x4 zero_f32x4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// LDS row pitch (in halves) for tiles read as MFMA fragments with ds_read_b128: a pitch
// of 16*P bytes with P % 4 == 2 puts the 16 lanes of every gfx950 b128 lane group
// ({0-3,12-15,20-27}, ...: rows r, r+12.. of one 16-B column chunk and rows r+4.. of the
// next) on 16 distinct 4-bank slots — conflict-free. (P % 4 == 1, e.g. the classic
// "+8 halves" pad of a 64-half row, is 2-way.)
__host__ __device__ constexpr int frag_pitch(int min_halves) {
  int p = (min_halves + 7) / 8;
  while (p % 4 != 2) ++p;
  return p * 8;
}

// XCD-aware remap of a 1-D block index (bijective; MI355X deals blocks round-robin
// over 8 XCDs, so consecutive logical tiles are placed on one XCD's L2).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  constexpr int kXcd = 8;
  if (nblocks < kXcd) return bid;
  const int q = nblocks / kXcd, r = nblocks % kXcd;
  const int xcd = bid % kXcd, idx = bid / kXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// The vocoder kernels' tile order (JANUS_NO_TILE_REMAP: plain dispatch order, for A/B
// builds). Remapped, the standalone vocoder's L2->fabric traffic fell from 1.42x to
// 1.19x the algorithmic bytes (profiles/traffic_r02.json).
__device__ __forceinline__ int tile_remap(int bid, int nblocks) {
#ifdef JANUS_NO_TILE_REMAP
  return bid;
#else
  return xcd_remap(bid, nblocks);
#endif
}

// Store an MFMA output fragment (lane = column col = tile column (lane & 15), rows row0 + rr,
// rr < 4, row0 = m*16 + 4*(lane >> 4)) as fp16 into an LDS tile with 4-byte stores: lanes
// l and l^1 trade two packed halves (one DPP quad_perm move), then the even lane writes rows
// 0-1 and the odd lane rows 2-3 of the column pair (col & ~1, col | 1): half the store
// instructions of per-element 2-byte stores. Opt-in build switch JANUS_C1_PAIRS: measured
// slower (standalone 64 x 30 s vocoder 154.0 vs 151.9 ms), so the LDS bank conflicts of
// the wide units do not come from these stores; the default is the 2-byte form.
__device__ __forceinline__ void st_frag_f16_pairs(_Float16* tile, int ld, int row0, int col,
                                                  const float (&v)[4], int lane) {
#ifndef JANUS_C1_PAIRS
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) tile[(row0 + rr) * ld + col] = (_Float16)v[rr];
#else
  const bool odd = lane & 1;
  const half2v mine_lo = {(_Float16)v[0], (_Float16)v[1]}, mine_hi = {(_Float16)v[2], (_Float16)v[3]};
  const half2v send = odd ? mine_lo : mine_hi;
  const int got_i = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send), 0xB1 /* quad_perm [1,0,3,2] */,
                                                0xF, 0xF, false);
  const half2v got = __builtin_bit_cast(half2v, got_i);
  half2v ra, rb;
  if (odd) {  // rows 2, 3: (partner's column, mine)
    ra = half2v{got[0], mine_hi[0]};
    rb = half2v{got[1], mine_hi[1]};
  } else {    // rows 0, 1: (mine, partner's column)
    ra = half2v{mine_lo[0], got[0]};
    rb = half2v{mine_lo[1], got[1]};
  }
  const int r = row0 + (odd ? 2 : 0), c0 = col & ~1;
  *reinterpret_cast<half2v*>(tile + r * ld + c0) = ra;
  *reinterpret_cast<half2v*>(tile + (r + 1) * ld + c0) = rb;
#endif
}

// LayerNorm arithmetic shared by layernorm_kernel and resid_ln_kernel (gemm.hip), written
// with explicit fmaf and no other contraction so the two kernels round alike: left to the
// compiler, a*a + b*b may become fma(a, a, b*b) in one kernel and fma(b, b, a*a) in the
// other.
__device__ __forceinline__ float ln_sum4(const float4& v) {
#pragma clang fp contract(off)
  return ((v.x + v.y) + v.z) + v.w;
}
__device__ __forceinline__ float ln_sq4(const float4& v, float mean) {
#pragma clang fp contract(off)
  const float a = v.x - mean, b = v.y - mean, c = v.z - mean, e = v.w - mean;
  return fmaf(e, e, fmaf(c, c, fmaf(b, b, a * a)));
}
__device__ __forceinline__ half4 ln_norm4(const float4& v, float mean, float rstd, const float4& g,
                                          const float4& b) {
#pragma clang fp contract(off)
  return half4{(_Float16)fmaf((v.x - mean) * rstd, g.x, b.x), (_Float16)fmaf((v.y - mean) * rstd, g.y, b.y),
               (_Float16)fmaf((v.z - mean) * rstd, g.z, b.z), (_Float16)fmaf((v.w - mean) * rstd, g.w, b.w)};
}

// LayerNorm of R fp32 rows by one wave (rows row0 + j*rstep, j < R; d <= 256*MAXV, d % 4
// == 0): every row, gamma and beta load is issued before the first use (one memory round
// trip for all R rows); fp16 out rows at out + (lrow0 + j*rstep)*ldo, ALL R of them written
// (rows >= nrows as zeros: out must hold R rows, e.g. an LDS tile).
// Two-pass mean / variance in fp32 as layernorm_kernel. MAXV sized to d keeps the register
// footprint small enough not to cost the caller occupancy; the loads are unconditional
// (clamped index) — guarded vector loads are split into branchy dword loads by the
// compiler, which measured 3x slower in the GEMM prologue.
template <int MAXV, int R>
__device__ __forceinline__ void ln_rows_wave(const float* x, int64_t ldx, int row0, int rstep,
                                             int nrows, const float* __restrict__ g,
                                             const float* __restrict__ b, _Float16* out,
                                             int lrow0, int ldo, int d, float eps, int lane) {
  const int nv = d >> 2;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  float4 v[R][MAXV], gg[MAXV], bb[MAXV];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int r = row0 + j * rstep;
    const float4* x4 = reinterpret_cast<const float4*>(x + (int64_t)min(r, nrows - 1) * ldx);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int i = lane + 64 * k;
      // unconditional 16-byte loads (clamped index; values past d are masked below)
      v[j][k] = x4[min(i, nv - 1)];
    }
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int i = min(lane + 64 * k, nv - 1);
    gg[k] = g4[i];
    bb[k] = b4[i];
  }
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
      if (lane + 64 * k >= nv) v[j][k] = z;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    // layernorm_kernel's arithmetic (ln_sum4 / ln_sq4 / ln_norm4): a LayerNorm in a GEMM
    // prologue rounds exactly as the separate LayerNorm launch it replaces
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) s += ln_sum4(v[j][k]);
    s = wave_sum_f32(s);
    const float mean = s / d;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
      if (lane + 64 * k < nv) q += ln_sq4(v[j][k], mean);
    q = wave_sum_f32(q);
    const float rstd = rsqrtf(q / d + eps);
    const bool rok = row0 + j * rstep < nrows;
    _Float16* orow = out + (int64_t)(lrow0 + j * rstep) * ldo;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int i = lane + 64 * k;
      if (i < nv) {
        half4 h = ln_norm4(v[j][k], mean, rstd, gg[k], bb[k]);
        if (!rok) h = half4{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
        *reinterpret_cast<half4*>(orow + 4 * i) = h;
      }
    }
  }
}

// LayerNorm of one fp32 row of d <= 1024 columns by one wave (two-pass mean / variance
// in fp32, as layernorm_kernel), fp16 out. SC1: read the row with agent-scope relaxed
// (sc1) loads — for rows other workgroups of the same launch have just stored sc1.
template <bool SC1>
__device__ __forceinline__ void ln_row_wave(const float* xr, const float* __restrict__ g,
                                            const float* __restrict__ b, _Float16* out, int d,
                                            float eps, int lane) {
  if constexpr (SC1) {
    float v[16];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = lane + 64 * i;
      const float t = c < d ? __hip_atomic_load(xr + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
      v[i] = t;
      s += t;
    }
    s = wave_sum_f32(s);
    const float mean = s / d;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = lane + 64 * i;
      if (c < d) q += (v[i] - mean) * (v[i] - mean);
    }
    q = wave_sum_f32(q);
    const float rstd = rsqrtf(q / d + eps);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = lane + 64 * i;
      if (c < d) out[c] = (_Float16)((v[i] - mean) * rstd * g[c] + b[c]);
    }
  } else {
    ln_rows_wave<4, 1>(xr, 0, 0, 1, 1, g, b, out, 0, 0, d, eps, lane);
  }
}

}  // namespace janus

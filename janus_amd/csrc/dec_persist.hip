// Persistent decoder segments (r05): the greedy decoder's small launches between the two
// attention kernels of a layer, as two resident-grid launches with grid barriers.
//
// Whisper's decoder layer (faster-whisper / CTranslate2 greedy step, transcriber.py:53-57;
// the absorbed cross-attention of xattn.hip) per position, rows = the decode batch:
//   self-attention launch -> o
//   SEGMENT A:  x += o Wo^T + bo                      (split-K GEMM, residual epilogue)
//               | grid barrier
//               xqk = LN2(x) Wqk^T + bqk              (LayerNorm in the block + GEMM)
//   cross-attention launch (one key split: writes c = softmax(qk enc^T) enc itself)
//   SEGMENT B:  o' = c_h Wv_h^T + bv  (per head)      (split-K, block-diagonal A)
//               | x += o' Wo_c^T + bo_c               (split-K, residual)
//               | f = gelu(LN3(x) W1^T + b1)          (LayerNorm + GEMM)
//               | x += f W2^T + b2                    (split-K, K = 4d)
//               | [next layer] q, K/V[pos] = LN1(x) Wqkv^T + bqkv   (LayerNorm + GEMM)
// which replaces ten launches per layer (O, LN2, qk, value projection, cross O, LN3, fc1,
// fc2, LN1, QKV) by two: 75 -> 29 launches per position at base.en.
//
// What a resident grid buys over launch boundaries (MI355X_MICROARCH.md price list,
// phase-in-launch / prefetch-credit): no per-launch fill and drain, and each phase's WEIGHT
// fragments (independent of the activations) are loaded into registers while the previous
// phase finishes, so after the barrier a phase waits only for its (small, L2/MALL-served)
// activation rows. Hand-offs follow the guide's R1 form (cdna_hip_programming.md §6
// Guideline 16): every handed-off byte is stored write-through (sc1 buffer stores), every
// storing wave drains (s_waitcnt vmcnt(0)) before its block arrives at the barrier, and
// every load of a handed-off byte is an sc1 load. The barrier is two-level (one arrival
// counter per XCD group on its own 64-byte line, the group's last arriver bumps the top
// counter; one lane polls the top counter relaxed with s_sleep), spins are bounded (a
// timeout sets the error word and the kernel runs to its end), and the last block to leave
// zeroes every counter for the next launch (self-cleaning: nothing to memset per call).
//
// Numerics: LayerNorm with layernorm_kernel's arithmetic (ln_sum4 / ln_sq4 / ln_norm4);
// split-K partials summed in a fixed order ((k0 + k1) + k2) + k3 independent of the grid
// and of the rows' neighbours, so a row's result does not depend on the batch it rides in
// (the staggered decode's bit-identity). The GEMMs' k order differs from the launch path's
// 16-wave split (gemm_skinny_kernel), so the two paths agree to fp32 rounding, not bits.
#include "mfma.h"
#include "kernels.h"
#include "dec_persist.h"
#include "xattn_body.h"
#include <algorithm>
#include <cstdlib>

namespace janus {

namespace {

constexpr int kD = 512;            // d_model (base.en); LayerNorm / residual width
constexpr int kNT = 512;           // threads per block: 8 waves
constexpr int kAP = frag_pitch(kD);  // LDS row pitch of the normalised A tile (halves)
constexpr unsigned kSpinLimit = 1u << 22;  // ~0.5 s of s_sleep polls before giving up

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  // raw buffer: out-of-range loads return 0 and out-of-range stores are dropped, so rows
  // past the batch need no guards
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
// sc1: agent-coherent, L1-bypassing (write-through stores) — the R1 hand-off flavour
__device__ __forceinline__ u32x4v ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ void st_sc1(u32x4v v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
__device__ __forceinline__ void st_sc1_8(u32x2v v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 16);
}
__device__ __forceinline__ half8 as_h8(u32x4v v) { return __builtin_bit_cast(half8, v); }
// an opaque copy of a value: the compiler cannot prove two phases' copies equal, so it
// recomputes per-phase addresses instead of keeping them live across the whole launch
template <class T>
__device__ __forceinline__ T opaque(T v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ float4 as_f4(u32x4v v) { return __builtin_bit_cast(float4, v); }

// Grid barrier `epoch` (1, 2, ... within the launch). Every wave drains its stores first
// (the sc1 payload is in memory), then lane 0 of the block arrives on its XCD group's
// counter; the group's last arriver bumps the top counter; lane 0 polls the top counter.
// bar: [0] top, [16 * (1 + g)] group g (g < 8), [16 * 9] exit — 64-byte lines.
// Phase stamps (JANUS_PHASE_PROF builds): thread 0 of every block writes the real-time
// clock (100 MHz) at kernel start [0], at each barrier's arrival [2e - 1] (every wave
// drained) and release [2e] (e <= 7), before the exit [15]; [16] HW_ID, [17] XCC_ID; inside
// phase p (1-based, segment kernels) wave 0's progress at [18 + 3 (p - 1) + i] (split-K:
// MFMAs done, reduction synced; LayerNorm GEMM: LayerNorm synced, first tile's MFMAs done,
// its stores issued). 48 slots per block.
#ifdef JANUS_PHASE_PROF
#define SEG_STAMP(ST, I) do { if ((ST) && threadIdx.x == 0) (ST)[I] = (long long)wall_clock64(); } while (0)
#define SEG_END(ST) do { __syncthreads(); SEG_STAMP(ST, 15); } while (0)
#else
#define SEG_STAMP(ST, I) do { (void)(ST); } while (0)
#define SEG_END(ST) do { (void)(ST); } while (0)
#endif

// Memory-model invariant (the barrier itself carries no acquire / release fence, which on
// gfx950 would write back and invalidate the L2 at every barrier): EVERY byte handed off
// between phases is stored with st_sc1 / st_sc1_8 and loaded with ld_sc1 (or the sc1
// arguments of the raw buffer builtins), so it goes to and comes from the coherent level
// whatever XCD the other block ran on; the s_waitcnt vmcnt(0) below retires the stores
// before the arrival, and the asm memory clobbers keep the compiler from moving loads above
// the poll. A phase that reads a handed-off buffer with a plain load would see stale L2 data
// from another XCD: new phases must use ld_sc1 for such reads.
__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned epoch, unsigned* err,
                                             long long* st = nullptr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  SEG_STAMP(st, 2 * epoch - 1);
  if (threadIdx.x == 0) {
    const unsigned G = gridDim.x, g = blockIdx.x & 7;
    const unsigned ng = G < 8 ? G : 8;
    const unsigned gsz = G / 8 + (g < G % 8 ? 1u : 0u);
    const unsigned old = __hip_atomic_fetch_add(bar + 16 * (1 + g), 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old == epoch * gsz - 1)
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch * ng) {
      __builtin_amdgcn_s_sleep(2);
      // a block never arrived: give up and flag it; once flagged (this launch or an
      // earlier one of the call) nobody waits again, so a broken call ends quickly
      if (++spins > kSpinLimit ||
          ((spins & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  SEG_STAMP(st, 2 * epoch);
  __syncthreads();
}

// The last block to leave zeroes the counters (every block has passed every wait by then).
__device__ __forceinline__ void grid_exit(unsigned* bar) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(bar + 16 * 9, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int g = 0; g < 8; ++g)
        __hip_atomic_store(bar + 16 * (1 + g), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(bar + 16 * 9, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------ L2 touch
// The weight slabs a block reads in a phase come from HBM (the encoder-output and KV-cache
// streams of the other launches keep them out of the Infinity Cache): a LayerNorm GEMM
// phase waited ≈5 µs for its first 128 KB per block (tools/seg_prof.py). So at the START
// of each phase, before its own loads, every block touches the NEXT phase's slab — one
// dword per 128-byte line of its share (the blocks that read the same slab split its
// lines) — and the next phase's fragment loads then hit the XCD's L2. The touched dwords
// land during the phase (issued first, they retire in order ahead of the phase's own
// loads at about the same latency) and are folded into a sink after the next barrier;
// no result depends on them.
__device__ __forceinline__ uint32_t l2_touch(const _Float16* base, uint32_t bytes, int slice,
                                             int nslices) {
  const uint32_t lines = bytes >> 7;
  const uint32_t per = (lines + nslices - 1) / nslices;
  const uint32_t l0 = min(lines, (uint32_t)slice * per);
  const uint32_t n = min(per, lines - l0);  // <= kNT at the shapes dec_seg_grid admits
  const auto r = rsrc(reinterpret_cast<const char*>(base) + (size_t)l0 * 128, n * 128);
  const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(r, threadIdx.x * 128, 0, 0);
  __builtin_amdgcn_sched_barrier(0);  // issued here, ahead of the phase's own loads
  return v;
}

// two m-tiles per block for a LayerNorm GEMM phase of N columns when one per block would
// leave a wave more than one 16-column tile (uniform over the grid)
__device__ __forceinline__ bool dec_seg_mb2(int N, int MT) {
  return MT % 2 == 0 && (N / 16) / ((int)gridDim.x / MT) > 8;
}

// the slab of a LayerNorm GEMM phase: the block's column group, split over the blocks of
// its m-groups (lng_tiles<MB>)
template <int MB = 1>
__device__ __forceinline__ uint32_t touch_lng(const _Float16* wt, int N, int MT) {
  const int b = blockIdx.x, G = gridDim.x;
  const int j = b >> 3, xcd = b & 7;
  const int MG = MT / MB;
  const int npg = (N / 16) / (G / MG), g = xcd + 8 * (j / MG);
  return l2_touch(wt + (int64_t)16 * g * npg * kD, (uint32_t)npg * 16 * kD * 2, j % MG, MG);
}

// the slab of a split-K phase: the rows of the pair's column tile(s), split over the
// pairs that share them
__device__ __forceinline__ uint32_t touch_splitk(const _Float16* wt, int K, int MT) {
  const int p = blockIdx.x;
  if (p >= 16 * MT) return 0u;
  const int n0 = (2 * p) / MT, n1 = (2 * p + 1) / MT;
  const int share = MT >= 2 ? MT / 2 : 1;
  return l2_touch(wt + (int64_t)16 * n0 * K, (uint32_t)(n1 - n0 + 1) * 16 * K * 2, p % share, share);
}

// 256 rows on the 128-block grid (BIG): block b = xcd + 8 j takes column tile
// n = xcd + 8 (j / 4) and the m-tiles 4 (j % 4) .. + 3 of it, so the four blocks of a column
// tile sit on one XCD (its weights come into that XCD's L2 once) and each block reads its
// weight fragments once for four m-tiles
__device__ __forceinline__ int quad_col() { return (int)(blockIdx.x & 7) + 8 * ((int)(blockIdx.x >> 3) >> 2); }
__device__ __forceinline__ int quad_m0() { return 4 * (((int)blockIdx.x >> 3) & 3); }
__device__ __forceinline__ uint32_t touch_quad(const _Float16* wt, int K) {
  return l2_touch(wt + (int64_t)16 * quad_col() * K, (uint32_t)16 * K * 2, ((int)blockIdx.x >> 3) & 3, 4);
}

// ------------------------------------------------------------------ split-K phase
// out[R][512] from A[R][K] . W[512][K]^T: tiles of 16 rows x 16 columns, each over K in
// four quarters (one wave per quarter), two tiles per block (8 waves); pair p of the
// phase: tiles 2p, 2p + 1, tile t -> (m = t % MT, n = t / MT). KSW = k-steps per quarter.
// GROUP: block-diagonal A (output columns [64h, 64h + 64) read A columns [512h, 512h + 512):
// the per-head value projection).
template <int KSW>
struct SplitW {
  half8 w[KSW];
};

template <int KSW>
__device__ __forceinline__ void splitk_prefetch(SplitW<KSW>& W, const _Float16* wt, int K,
                                                int pair, int MT, int lane, int wv, bool quad = false) {
  const int t = 2 * pair + (wv >> 2), kp = wv & 3;
  const int n = quad ? quad_col() : t / MT;
  const _Float16* wr = wt + (int64_t)(16 * n + (lane & 15)) * K + kp * (K / 4) + 8 * (lane >> 4);
#pragma unroll
  for (int s = 0; s < KSW; ++s) W.w[s] = *reinterpret_cast<const half8*>(wr + 32 * s);
  // every weight fragment in flight before the phase's activation loads (left alone, the
  // scheduler issued the later k-steps' weights after the first MFMA: a second round trip)
  __builtin_amdgcn_sched_barrier(0);
}

enum SegEpi { SE_RESID = 0, SE_F16_SC1 = 1 };

// one pair of tiles: the waves' products, the fixed-order reduction, the epilogue. pre():
// the NEXT phase's weight loads, issued right after this pair's MFMAs so they are in
// flight during the reduction and the epilogue (the barrier's drain then finds them done)
template <int KSW, int EPI, bool GROUP, class Pre>
__device__ __forceinline__ void splitk_pair(const SplitW<KSW>& W, int pair, int MT, int K,
                                            __amdgpu_buffer_rsrc_t ra, int lda,
                                            const float* bias,
                                            __amdgpu_buffer_rsrc_t rx,  // SE_RESID: x [B][512] f32
                                            __amdgpu_buffer_rsrc_t ro,  // SE_F16_SC1: out [B][512]
                                            float* red, int lane, int wv, bool last, Pre&& pre,
                                            long long* st = nullptr, int si = 0) {
  const int tsub = wv >> 2, kp = wv & 3;
  const int t = 2 * pair + tsub;
  const int m = t % MT, n = t / MT;
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  const int acol = (GROUP ? (16 * n / 64) * kD : 0) + kp * (K / 4) + kc8;
  const uint32_t abase = (uint32_t)(((16 * m + lr) * lda + acol) * 2);
  f32x4 acc = zero_f32x4();
  // A in halves of at most 8 k-steps (K = 4d: 64 + 32 registers, not 64 + 64)
  constexpr int H = KSW > 8 ? 8 : KSW;
#pragma unroll
  for (int h0 = 0; h0 < KSW; h0 += H) {
    half8 a[H];
#pragma unroll
    for (int s = 0; s < H; ++s) a[s] = as_h8(ld_sc1(ra, abase + 64 * (h0 + s)));
#pragma unroll
    for (int s = 0; s < H; ++s) acc = mfma16(a[s], W.w[h0 + s], acc);
    // the second half's loads stay below the first half's MFMAs (hoisted, all 16 A
    // fragments plus the 16 weight fragments would need 128 registers)
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the next phase's loads below the MFMAs
  if (last) pre();
  __builtin_amdgcn_sched_barrier(0);
  // red[tsub][kp][16][17]
  float* rp = red + (tsub * 4 + kp) * 16 * 17;
#pragma unroll
  for (int r = 0; r < 4; ++r) rp[(4 * (lane >> 4) + r) * 17 + lr] = acc[r];
  SEG_STAMP(st, si);
  __syncthreads();
  SEG_STAMP(st, si + 1);
  const int tid = threadIdx.x;
  if (tid < 128) {
    const int es = tid >> 6, q = tid & 63;
    const int et = 2 * pair + es;
    const int em = et % MT, en = et / MT;
    const int row = q >> 2, c4 = 4 * (q & 3);
    const float* r0 = red + (es * 4) * 16 * 17 + row * 17 + c4;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = r0[i] + r0[16 * 17 + i];
      s += r0[2 * 16 * 17 + i];
      s += r0[3 * 16 * 17 + i];
      v[i] = s + bias[16 * en + c4 + i];
    }
    const uint32_t eoff = (uint32_t)((16 * em + row) * kD + 16 * en + c4);
    if constexpr (EPI == SE_RESID) {
      const float4 xv = as_f4(ld_sc1(rx, eoff * 4));
      const float4 y = make_float4(xv.x + v[0], xv.y + v[1], xv.z + v[2], xv.w + v[3]);
      st_sc1(__builtin_bit_cast(u32x4v, y), rx, eoff * 4);
    } else {
      const half4 h = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
      st_sc1_8(__builtin_bit_cast(u32x2v, h), ro, eoff * 2);
    }
  }
  __syncthreads();  // red is reused by the next pair
}

// ------------------------------------------------------------ LayerNorm + GEMM phase
// out[R][N] = epi(LN(x) W[N][512]^T + b): block -> (m-tile, group of NPG 16-column tiles);
// the block normalises its 16 rows into LDS (layernorm_kernel's arithmetic), each wave
// computes whole-K tiles of the group (up to two prefetched).
struct LngW {
  half8 w[16];
};

// MB m-tiles per block (MB = 2: the block's 32 rows share each weight fragment, so a block
// reads half the weight bytes of MB = 1 for the same columns): block -> (m-group of MB
// tiles, column group), the blocks of one column group on one XCD (its L2 serves them)
template <int MB = 1>
__device__ __forceinline__ void lng_tiles(int N, int MT, int& m, int& nt0, int& npg) {
  const int b = blockIdx.x, G = gridDim.x;
  const int j = b >> 3, xcd = b & 7;
  const int MG = MT / MB;
  const int NG = G / MG;
  m = (j % MG) * MB;  // first m-tile
  const int g = xcd + 8 * (j / MG);
  npg = (N / 16) / NG;
  nt0 = g * npg;
}

__device__ __forceinline__ void lng_load(half8 (&w)[16], const _Float16* wt, int nt, int lane) {
  const _Float16* wr = wt + (int64_t)(16 * nt + (lane & 15)) * kD + 8 * (lane >> 4);
#pragma unroll
  for (int s = 0; s < 16; ++s) w[s] = *reinterpret_cast<const half8*>(wr + 32 * s);
}

// the wave's first tile of the phase (the rest are loaded during the phase)
__device__ __forceinline__ void lng_prefetch(LngW& W, const _Float16* wt, int N, int MT,
                                             int lane, int wv) {
  int m, nt0, npg;
  lng_tiles(N, MT, m, nt0, npg);
  if (wv < npg) lng_load(W.w, wt, nt0 + wv, lane);  // wave-uniform
  __builtin_amdgcn_sched_barrier(0);
}

enum LngEpi { LE_F16 = 0, LE_GELU_SC1 = 1, LE_QKV = 2 };

struct LngOut {
  _Float16* out; int ldo;                  // LE_F16 / LE_GELU_SC1 / q part of LE_QKV
  _Float16* kc; _Float16* vc; int pos, n_ctx; const int32_t* roff;  // LE_QKV
};

template <int EPI, int MB = 1, class Pre>
__device__ __forceinline__ void lng_phase(LngW& W, const _Float16* wt, int N, int MT,
                                          int B, __amdgpu_buffer_rsrc_t rx, const float* g,
                                          const float* bt, const float* bias,
                                          const LngOut& o, _Float16* sA, float* patch_all, int lane,
                                          int wv, Pre&& pre, long long* st = nullptr, int si = 0) {
  int m, nt0, npg;
  lng_tiles<MB>(N, MT, m, nt0, npg);
  constexpr int RW = 2 * MB;  // LayerNorm rows per wave
  // ---- LayerNorm of rows 16m + 2wv, 16m + 2wv + 1 (sc1 loads: x was just handed off).
  // Issue order: both rows and gamma / beta first, THEN the phase's weight fragments, so
  // the LayerNorm waits only for its own loads (vector loads retire in issue order: with
  // the weights issued first it waited for all 16 of them) while the weights stream in
  float4 v[RW][2], gg[2], bb[2];
#pragma unroll
  for (int j = 0; j < RW; ++j)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      v[j][k] = as_f4(ld_sc1(rx, (uint32_t)(((16 * m + RW * wv + j) * kD + 4 * (lane + 64 * k)) * 4)));
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    gg[k] = reinterpret_cast<const float4*>(g)[lane + 64 * k];
    bb[k] = reinterpret_cast<const float4*>(bt)[lane + 64 * k];
  }
  __builtin_amdgcn_sched_barrier(0);
  // unconditional (a wave without a tile re-reads the group's first, unused): behind a
  // branch the wait-count pass merged the paths and the LayerNorm waited for the weights.
  // MB = 2 (four rows in flight) issues the first 8 k-steps here and the rest after the
  // LayerNorm: all 16 beside the rows would spill
  const _Float16* wrow = wt + (int64_t)(16 * (nt0 + (wv < npg ? wv : 0)) + (lane & 15)) * kD + 8 * (lane >> 4);
  constexpr int WH = MB == 1 ? 16 : 8;
#pragma unroll
  for (int k = 0; k < WH; ++k) W.w[k] = *reinterpret_cast<const half8*>(wrow + 32 * k);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int lrow = RW * wv + j;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 2; ++k) s += ln_sum4(v[j][k]);
    s = wave_sum_f32(s);
    const float mean = s / kD;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 2; ++k) q += ln_sq4(v[j][k], mean);
    q = wave_sum_f32(q);
    const float rstd = rsqrtf(q / kD + 1e-5f);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      *reinterpret_cast<half4*>(sA + lrow * kAP + 4 * (lane + 64 * k)) = ln_norm4(v[j][k], mean, rstd, gg[k], bb[k]);
  }
  if constexpr (WH < 16) {
#pragma unroll
    for (int k = WH; k < 16; ++k) W.w[k] = *reinterpret_cast<const half8*>(wrow + 32 * k);
  }
  __syncthreads();
  SEG_STAMP(st, si);
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  float* patch = patch_all + wv * 16 * 17;
  // the wave's tiles li = wv, wv + 8, ...; the last one peeled so pre() (the next phase's
  // weights) sits after the loop in straight-line code: inside it, its registers would be
  // live across every iteration
  const int ntile = wv < npg ? (npg - wv + 7) / 8 : 0;
  auto tile = [&](int li, bool last) __attribute__((always_inline)) {
    const int nt = nt0 + li;
    // the tile's bias now: loaded in the epilogue it would queue behind the next tile's
    // weight loads issued there (vector loads retire in order)
    const float4 bias4 = *reinterpret_cast<const float4*>(bias + 16 * nt + 4 * (lane & 3));
    f32x4 acc[MB];
#pragma unroll
    for (int u = 0; u < MB; ++u) acc[u] = zero_f32x4();
    half8 a[2][MB];
#pragma unroll
    for (int u = 0; u < MB; ++u) a[0][u] = *reinterpret_cast<const half8*>(sA + (16 * u + lr) * kAP + kc8);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + 1 < 16)
#pragma unroll
        for (int u = 0; u < MB; ++u)
          a[(s + 1) & 1][u] = *reinterpret_cast<const half8*>(sA + (16 * u + lr) * kAP + 32 * (s + 1) + kc8);
#pragma unroll
      for (int u = 0; u < MB; ++u) acc[u] = mfma16(a[s & 1][u], W.w[s], acc[u]);
    }
    if (li == wv) SEG_STAMP(st, si + 1);
    // the next tile's weights (or the next phase's) in flight during this epilogue
    // (scheduling barriers: hoisted above the MFMAs, the loads' registers would overlap
    // this tile's weights)
    __builtin_amdgcn_sched_barrier(0);
    if (!last) lng_load(W.w, wt, nt + 8, lane);
    else pre();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < MB; ++u) {
#pragma unroll
    for (int r = 0; r < 4; ++r) patch[(4 * (lane >> 4) + r) * 17 + lr] = acc[u][r];
    // wave-private patch: own stores visible to own loads in order
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    const int row = lane >> 2, c4 = 4 * (lane & 3);
    const int grow = 16 * (m + u) + row, col = 16 * nt + c4;
    float v[4];
    v[0] = patch[row * 17 + c4 + 0] + bias4.x;
    v[1] = patch[row * 17 + c4 + 1] + bias4.y;
    v[2] = patch[row * 17 + c4 + 2] + bias4.z;
    v[3] = patch[row * 17 + c4 + 3] + bias4.w;
    if (grow < B) {
      if constexpr (EPI == LE_GELU_SC1) {
        const half4 h = {(_Float16)gelu_erf(v[0]), (_Float16)gelu_erf(v[1]), (_Float16)gelu_erf(v[2]),
                         (_Float16)gelu_erf(v[3])};
        st_sc1_8(__builtin_bit_cast(u32x2v, h), rsrc(o.out, (uint32_t)B * o.ldo * 2),
                 (uint32_t)((grow * o.ldo + col) * 2));
      } else {
        const half4 h = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        if constexpr (EPI == LE_QKV) {
          // write-through: the layer kernel's self-attention phase reads q and the new K/V
          // rows in the same launch (the 16-column tile is in one of q / K / V: uniform)
          if (col < kD) {
            st_sc1_8(__builtin_bit_cast(u32x2v, h), rsrc(o.out, (uint32_t)B * o.ldo * 2),
                     (uint32_t)((grow * o.ldo + col) * 2));
          } else {
            _Float16* cache = col < 2 * kD ? o.kc : o.vc;
            const int cpos = o.pos + (o.roff ? o.roff[grow] : 0);
            st_sc1_8(__builtin_bit_cast(u32x2v, h), rsrc(cache, (uint32_t)B * o.n_ctx * kD * 2),
                     (uint32_t)(((grow * o.n_ctx + cpos) * kD + (col % kD)) * 2));
          }
        } else {
          // write-through: the layer kernel's cross-attention phase reads xqk in the launch
          st_sc1_8(__builtin_bit_cast(u32x2v, h), rsrc(o.out, (uint32_t)B * o.ldo * 2),
                   (uint32_t)((grow * o.ldo + col) * 2));
        }
      }
    }
    if (li == wv) SEG_STAMP(st, si + 2);
    }  // u: the patch is reused by the next m-tile (one wave's LDS operations run in order)
    // the patch is rewritten by the next tile: LDS operations of one wave run in order
  };
  for (int i = 0; i + 1 < ntile; ++i) tile(wv + 8 * i, false);
  if (ntile > 0) tile(wv + 8 * (ntile - 1), true);
  else pre();  // no tile for this wave
  (void)N;
}

// K = 4d (fc2) with both tiles of the pair in the same column tile (MT even): every wave
// takes one eighth of K for BOTH tiles — its 8 weight fragments shared by the two m-tiles,
// 2 x 8 activation fragments — so all of a wave's loads go out in one round trip (the
// quarter split needed 16 weight + 2 x 8 activation fragments per wave and issued the
// second activation half after the first half's MFMAs: two round trips); the 8 partials
// per output are summed in a fixed order
__device__ __forceinline__ void splitk8_pair(const _Float16* wt, int pair, int MT,
                                             __amdgpu_buffer_rsrc_t ra, const float* bias,
                                             __amdgpu_buffer_rsrc_t rx, float* red, int lane, int wv,
                                             long long* st, int si) {
  constexpr int K = 4 * kD, KS = K / 8 / 32;  // 8 k-steps per wave
  const int t0 = 2 * pair;
  const int m0 = t0 % MT, n = t0 / MT;
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  const int k0 = wv * (K / 8) + kc8;
  half8 w[KS], a0[KS], a1[KS];
  const _Float16* wr = wt + (int64_t)(16 * n + lr) * K + k0;
#pragma unroll
  for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const half8*>(wr + 32 * s);
  const uint32_t ab0 = (uint32_t)(((16 * m0 + lr) * K + k0) * 2);
  const uint32_t ab1 = ab0 + (uint32_t)(16 * K * 2);
#pragma unroll
  for (int s = 0; s < KS; ++s) a0[s] = as_h8(ld_sc1(ra, ab0 + 64 * s));
#pragma unroll
  for (int s = 0; s < KS; ++s) a1[s] = as_h8(ld_sc1(ra, ab1 + 64 * s));
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc0 = zero_f32x4(), acc1 = zero_f32x4();
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    acc0 = mfma16(a0[s], w[s], acc0);
    acc1 = mfma16(a1[s], w[s], acc1);
  }
  // red[tile][wave][16][17]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[((0 * 8 + wv) * 16 + 4 * (lane >> 4) + r) * 17 + lr] = acc0[r];
    red[((1 * 8 + wv) * 16 + 4 * (lane >> 4) + r) * 17 + lr] = acc1[r];
  }
  SEG_STAMP(st, si);
  __syncthreads();
  SEG_STAMP(st, si + 1);
  const int tid = threadIdx.x;
  if (tid < 128) {
    const int es = tid >> 6, q = tid & 63;
    const int em = m0 + es;
    const int row = q >> 2, c4 = 4 * (q & 3);
    const float* r0 = red + (es * 8) * 16 * 17 + row * 17 + c4;
    const float4 b4 = *reinterpret_cast<const float4*>(bias + 16 * n + c4);
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float sum = r0[i];
#pragma unroll
      for (int k = 1; k < 8; ++k) sum += r0[k * 16 * 17 + i];
      v[i] = sum;
    }
    v[0] += b4.x; v[1] += b4.y; v[2] += b4.z; v[3] += b4.w;
    const uint32_t eoff = (uint32_t)((16 * em + row) * kD + 16 * n + c4);
    const float4 xv = as_f4(ld_sc1(rx, eoff * 4));
    const float4 y = make_float4(xv.x + v[0], xv.y + v[1], xv.z + v[2], xv.w + v[3]);
    st_sc1(__builtin_bit_cast(u32x4v, y), rx, eoff * 4);
  }
}

// BIG (MT = 16 on the 128-block grid): the block's four m-tiles of its column tile (quad_col,
// quad_m0), wave (tsub, kp) computing k-quarter kp of m-tiles m0 + tsub and m0 + 2 + tsub
// with ONE set of weight fragments; every load of the phase out before the MFMAs, one
// reduction of the four tiles. Each tile's arithmetic (k-quarter products, the fixed-order
// sum ((k0 + k1) + k2) + k3, bias, epilogue) is splitk_pair's.
template <int KSW, int EPI, bool GROUP, class Pre>
__device__ __forceinline__ void splitk_quad(const SplitW<KSW>& W, int K, __amdgpu_buffer_rsrc_t ra, int lda,
                                            const float* bias, __amdgpu_buffer_rsrc_t rx,
                                            __amdgpu_buffer_rsrc_t ro, float* red, int lane, int wv,
                                            Pre&& pre, long long* st, int si) {
  static_assert(KSW <= 8, "quad split-K: A of both m-tiles in registers");
  const int tsub = wv >> 2, kp = wv & 3;
  const int n = quad_col(), mq = quad_m0();
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  const int acol = (GROUP ? (16 * n / 64) * kD : 0) + kp * (K / 4) + kc8;
  half8 a[2][KSW];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const uint32_t ab = (uint32_t)(((16 * (mq + 2 * v + tsub) + lr) * lda + acol) * 2);
#pragma unroll
    for (int s = 0; s < KSW; ++s) a[v][s] = as_h8(ld_sc1(ra, ab + 64 * s));
  }
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[2] = {zero_f32x4(), zero_f32x4()};
#pragma unroll
  for (int s = 0; s < KSW; ++s)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[v] = mfma16(a[v][s], W.w[s], acc[v]);
  __builtin_amdgcn_sched_barrier(0);  // keep the next phase's loads below the MFMAs
  pre();
  __builtin_amdgcn_sched_barrier(0);
  // red[tile 2v + tsub][kp][16][17]
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    float* rp = red + ((2 * v + tsub) * 4 + kp) * 16 * 17;
#pragma unroll
    for (int r = 0; r < 4; ++r) rp[(4 * (lane >> 4) + r) * 17 + lr] = acc[v][r];
  }
  SEG_STAMP(st, si);
  __syncthreads();
  SEG_STAMP(st, si + 1);
  const int tid = threadIdx.x;
  if (tid < 256) {
    const int es = tid >> 6, q = tid & 63;   // tile es = m-tile mq + es
    const int em = mq + es;
    const int row = q >> 2, c4 = 4 * (q & 3);
    const float* r0 = red + (es * 4) * 16 * 17 + row * 17 + c4;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = r0[i] + r0[16 * 17 + i];
      s += r0[2 * 16 * 17 + i];
      s += r0[3 * 16 * 17 + i];
      v[i] = s + bias[16 * n + c4 + i];
    }
    const uint32_t eoff = (uint32_t)((16 * em + row) * kD + 16 * n + c4);
    if constexpr (EPI == SE_RESID) {
      const float4 xv = as_f4(ld_sc1(rx, eoff * 4));
      const float4 y = make_float4(xv.x + v[0], xv.y + v[1], xv.z + v[2], xv.w + v[3]);
      st_sc1(__builtin_bit_cast(u32x4v, y), rx, eoff * 4);
    } else {
      const half4 h = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
      st_sc1_8(__builtin_bit_cast(u32x2v, h), ro, eoff * 2);
    }
  }
  __syncthreads();  // red is reused by the next phase
}

// fc2 (K = 4d) on the quads: splitk8_pair's arithmetic for the m-tile pairs (m0, m0 + 1) and
// (m0 + 2, m0 + 3) of the block's column tile, the weight fragments loaded once; the second
// pair's activation fragments are issued right after the first pair's MFMAs, in flight during
// its reduction and epilogue
template <bool PREV>
__device__ __forceinline__ void splitk8_quad(const _Float16* wt, __amdgpu_buffer_rsrc_t ra, const float* bias,
                                             __amdgpu_buffer_rsrc_t rx, float* red, int lane, int wv,
                                             long long* st, int si) {
  constexpr int K = 4 * kD, KS = K / 8 / 32;  // 8 k-steps per wave
  const int n = quad_col(), mq = quad_m0();
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  const int k0 = wv * (K / 8) + kc8;
  half8 w[KS], a0[KS], a1[KS];
  const _Float16* wr = wt + (int64_t)(16 * n + lr) * K + k0;
#pragma unroll
  for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const half8*>(wr + 32 * s);
  const int tid = threadIdx.x;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int m0 = mq + 2 * v;
    const uint32_t ab0 = (uint32_t)(((16 * m0 + lr) * K + k0) * 2);
    const uint32_t ab1 = ab0 + (uint32_t)(16 * K * 2);
    if (v == 0 || !PREV) {
#pragma unroll
      for (int s = 0; s < KS; ++s) a0[s] = as_h8(ld_sc1(ra, ab0 + 64 * s));
#pragma unroll
      for (int s = 0; s < KS; ++s) a1[s] = as_h8(ld_sc1(ra, ab1 + 64 * s));
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc0 = zero_f32x4(), acc1 = zero_f32x4();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      acc0 = mfma16(a0[s], w[s], acc0);
      acc1 = mfma16(a1[s], w[s], acc1);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (v == 0 && PREV) {  // the second pair's rows, during this pair's reduction
      const uint32_t nb0 = ab0 + (uint32_t)(2 * 16 * K * 2), nb1 = nb0 + (uint32_t)(16 * K * 2);
#pragma unroll
      for (int s = 0; s < KS; ++s) a0[s] = as_h8(ld_sc1(ra, nb0 + 64 * s));
#pragma unroll
      for (int s = 0; s < KS; ++s) a1[s] = as_h8(ld_sc1(ra, nb1 + 64 * s));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (v == 1) __syncthreads();  // red of the first pair read
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[((0 * 8 + wv) * 16 + 4 * (lane >> 4) + r) * 17 + lr] = acc0[r];
      red[((1 * 8 + wv) * 16 + 4 * (lane >> 4) + r) * 17 + lr] = acc1[r];
    }
    SEG_STAMP(st, si);
    __syncthreads();
    SEG_STAMP(st, si + 1);
    if (tid < 128) {
      const int es = tid >> 6, q = tid & 63;
      const int em = m0 + es;
      const int row = q >> 2, c4 = 4 * (q & 3);
      const float* r0 = red + (es * 8) * 16 * 17 + row * 17 + c4;
      const float4 b4 = *reinterpret_cast<const float4*>(bias + 16 * n + c4);
      float vv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float sum = r0[i];
#pragma unroll
        for (int k = 1; k < 8; ++k) sum += r0[k * 16 * 17 + i];
        vv[i] = sum;
      }
      vv[0] += b4.x; vv[1] += b4.y; vv[2] += b4.z; vv[3] += b4.w;
      const uint32_t eoff = (uint32_t)((16 * em + row) * kD + 16 * n + c4);
      const float4 xv = as_f4(ld_sc1(rx, eoff * 4));
      const float4 y = make_float4(xv.x + vv[0], xv.y + vv[1], xv.z + vv[2], xv.w + vv[3]);
      st_sc1(__builtin_bit_cast(u32x4v, y), rx, eoff * 4);
    }
  }
}

// one pair per block while the grid has at least 16 * MT blocks; BIG (MT = 16 on a
// 128-block grid, dec_seg_grid): the block's column quad (splitk_quad). Each tile's
// arithmetic is the one-pair form's, so a row's result does not depend on how many rows the
// call carries.
template <int KSW, int EPI, bool GROUP, bool BIG, class Pre>
__device__ __forceinline__ void splitk_phase(const SplitW<KSW>& W, const _Float16* wt, int K,
                                             int MT, __amdgpu_buffer_rsrc_t ra, int lda,
                                             const float* bias, __amdgpu_buffer_rsrc_t rx,
                                             __amdgpu_buffer_rsrc_t ro, float* red, int lane, int wv,
                                             Pre&& pre, long long* st = nullptr, int si = 0) {
  if constexpr (BIG) {
    splitk_quad<KSW, EPI, GROUP>(W, K, ra, lda, bias, rx, ro, red, lane, wv, pre, st, si);
  } else {
    const int p0 = blockIdx.x;
    if (p0 >= 16 * MT) { pre(); return; }  // 32 column tiles x MT row tiles / 2
    splitk_pair<KSW, EPI, GROUP>(W, p0, MT, K, ra, lda, bias, rx, ro, red, lane, wv, true, pre, st, si);
  }
  (void)wt;
}

}  // namespace

// LDS: split-K reduction [2][4][16][17] f32 | LN tile [16][kAP] f16 | wave patches [8][16][17]
constexpr int kRedF = 2 * 8 * 16 * 17;  // [2 tiles][8 k-parts][16][17] (the quarter split uses half)
constexpr int kPatchF = 8 * 16 * 17;
constexpr int kSegRows = 32;            // LayerNorm rows per block (MB = 2)
constexpr size_t kSegLds = (size_t)kRedF * 4 + (size_t)kSegRows * kAP * 2 + (size_t)kPatchF * 4;

// 128 VGPRs (four waves per SIMD): two blocks fit a CU, so a CU already holding other
// blocks (the YIN grid beside the decoder) still takes one and the grid stays co-resident.
// Each phase issues its weight loads first, right after the barrier, so they are in flight
// together with the phase's activation loads (sc1) — carrying them ACROSS the barrier in
// registers measured no faster in this shape (the activation round trip follows the
// barrier anyway) and cost the register budget.
__device__ __forceinline__ long long* seg_stamps(long long* prof, int k) {
#ifdef JANUS_PHASE_PROF
  if (prof) {
    long long* st = prof + ((int64_t)k * 256 + blockIdx.x) * 48;
    if (threadIdx.x == 0) {
      st[0] = (long long)wall_clock64();
      st[16] = (long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
      st[17] = (long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
    }
    return st;
  }
#endif
  (void)prof; (void)k;
  return nullptr;
}

// Segment A after barrier epoch e0: x += o Wo^T + bo | barrier e0 + 1 | xqk = LN2(x) Wqk^T +
// bqk. touched: the previous phase's L2 touch (folded into sink here, after the barrier that
// ended that phase); pst: in-phase stamps (stand-alone kernels only).
template <bool BIG>
__device__ __forceinline__ void seg_a_body(const DecSegArgs& a, float* seg_smem, long long* st,
                                           long long* pst, unsigned e0, uint32_t& touched,
                                           uint32_t& sink) {
  float* red = seg_smem;
  _Float16* sA = reinterpret_cast<_Float16*>(seg_smem + kRedF);
  float* patch = reinterpret_cast<float*>(sA + kSegRows * kAP);
  const int lane = threadIdx.x & 63, wv = wave_id();
  const int B = a.B, MT = a.MT;
  const auto rx = rsrc(a.x, (uint32_t)B * kD * 4);
  const bool first = (int)blockIdx.x < 16 * MT;
  // the qk projection (N = 8d) at two m-tiles per block where one would leave a wave two
  // weight tiles in a row (dec_seg_mb2): one weight round trip instead of two
  const bool mb2 = BIG || dec_seg_mb2(8 * kD, MT);
  sink ^= touched;
  touched = mb2 ? touch_lng<2>(a.wqk, 8 * kD, MT) : touch_lng<1>(a.wqk, 8 * kD, MT);
  // phase 1: x += o Wo^T + bo (o from the self-attention launch / phase)
  {
    SplitW<4> w;
    if (first) splitk_prefetch<4>(w, a.wo, kD, blockIdx.x, MT, lane, wv, BIG);
    splitk_phase<4, SE_RESID, false, BIG>(w, a.wo, kD, MT, rsrc(a.o, (uint32_t)B * kD * 2), kD, a.bo, rx, rx,
                                     red, lane, wv, [] {}, pst, 18);
  }
  grid_barrier(a.bar, e0 + 1, a.err, st);
  sink ^= touched;
  touched = 0u;
  // phase 2: xqk = LN2(x) Wqk^T + bqk (read by the cross-attention launch)
  {
    LngW w;
    LngOut o{a.xqk, 8 * kD, nullptr, nullptr, 0, 0, nullptr};
    if (mb2)
      lng_phase<LE_F16, 2>(w, a.wqk, 8 * kD, MT, B, rx, a.ln2g, a.ln2b, a.bqk, o, sA, patch, lane, wv, [] {}, pst, 21);
    else
      lng_phase<LE_F16, 1>(w, a.wqk, 8 * kD, MT, B, rx, a.ln2g, a.ln2b, a.bqk, o, sA, patch, lane, wv, [] {}, pst, 21);
  }
}

// Segment B after barrier epoch e0 (phases 1-4, barriers e0 + 1 .. e0 + 3, and with the next
// layer's weights phase 5 behind barrier e0 + 4).
template <bool BIG>
__device__ __forceinline__ void seg_b_body(const DecSegArgs& a, float* seg_smem, long long* st,
                                           long long* pst, unsigned e0, uint32_t& touched,
                                           uint32_t& sink) {
  float* red = seg_smem;
  _Float16* sA = reinterpret_cast<_Float16*>(seg_smem + kRedF);
  float* patch = reinterpret_cast<float*>(sA + kSegRows * kAP);
  const int lane = threadIdx.x & 63, wv = wave_id();
  const int B = a.B, MT = a.MT;
  const auto rx = rsrc(a.x, (uint32_t)B * kD * 4);
  const auto rom = rsrc(a.omid, (uint32_t)B * kD * 2);
  const bool first = (int)blockIdx.x < 16 * MT;
  sink ^= touched;
  touched = BIG ? touch_quad(a.woc, kD) : touch_splitk(a.woc, kD, MT);
  // phase 1: o' = c_h Wv_h^T + bv (c from the cross-attention launch), sc1 out
  {
    SplitW<4> w;
    if (first) splitk_prefetch<4>(w, a.wv, kD, blockIdx.x, MT, lane, wv, BIG);
    splitk_phase<4, SE_F16_SC1, true, BIG>(w, a.wv, kD, MT, rsrc(a.xc, (uint32_t)B * 8 * kD * 2), 8 * kD, a.bv,
                                      rx, rom, red, lane, wv, [] {}, pst, 18);
  }
  grid_barrier(a.bar, e0 + 1, a.err, st);
  sink ^= touched;
  touched = BIG ? touch_lng<2>(a.w1, 4 * kD, MT) : touch_lng<1>(a.w1, 4 * kD, MT);
  // phase 2: x += o' Wo_c^T + bo_c
  {
    SplitW<4> w;
    if (first) splitk_prefetch<4>(w, a.woc, kD, blockIdx.x, MT, lane, wv, BIG);
    splitk_phase<4, SE_RESID, false, BIG>(w, a.woc, kD, MT, rom, kD, a.boc, rx, rx, red, lane, wv, [] {}, pst, 21);
  }
  grid_barrier(a.bar, e0 + 2, a.err, st);
  sink ^= touched;
  touched = BIG ? touch_quad(a.w2, 4 * kD) : touch_splitk(a.w2, 4 * kD, MT);
  // phase 3: f = gelu(LN3(x) W1^T + b1), sc1 out
  {
    LngW w;
    LngOut o{a.f, 4 * kD, nullptr, nullptr, 0, 0, nullptr};
    if constexpr (BIG)
      lng_phase<LE_GELU_SC1, 2>(w, a.w1, 4 * kD, MT, B, rx, a.ln3g, a.ln3b, a.b1, o, sA, patch, lane, wv, [] {}, pst, 24);
    else
      lng_phase<LE_GELU_SC1>(w, a.w1, 4 * kD, MT, B, rx, a.ln3g, a.ln3b, a.b1, o, sA, patch, lane, wv, [] {}, pst, 24);
  }
  grid_barrier(a.bar, e0 + 3, a.err, st);
  sink ^= touched;
  touched = !a.wqkv ? 0u : BIG ? touch_lng<2>(a.wqkv, 3 * kD, MT) : touch_lng<1>(a.wqkv, 3 * kD, MT);
  // phase 4: x += f W2^T + b2 (K = 4d: eighths of K shared by the pair's two tiles, or
  // 16 k-steps per quarter when the pair spans two column tiles, MT = 1)
  if (MT % 2 == 0) {
    if constexpr (BIG) {
      splitk8_quad<false>(a.w2, rsrc(a.f, (uint32_t)B * 4 * kD * 2), a.b2, rx, red, lane, wv, pst, 27);
    } else if (first) {
      splitk8_pair(a.w2, blockIdx.x, MT, rsrc(a.f, (uint32_t)B * 4 * kD * 2), a.b2, rx, red, lane, wv, pst, 27);
    }
  } else {
    SplitW<16> w;
    if (first) splitk_prefetch<16>(w, a.w2, 4 * kD, blockIdx.x, MT, lane, wv);
    splitk_phase<16, SE_RESID, false, false>(w, a.w2, 4 * kD, MT, rsrc(a.f, (uint32_t)B * 4 * kD * 2), 4 * kD, a.b2,
                                      rx, rx, red, lane, wv, [] {}, pst, 27);
  }
  // phase 5 (all but the last layer): the next layer's q and K/V cache rows (write-through)
  if (a.wqkv) {
    grid_barrier(a.bar, e0 + 4, a.err, st);
    sink ^= touched;
    touched = 0u;
    LngW w;
    LngOut o{a.qkv, 3 * kD, a.kc, a.vc, a.pos, a.n_ctx, a.roff};
    if constexpr (BIG)
      lng_phase<LE_QKV, 2>(w, a.wqkv, 3 * kD, MT, B, rx, a.ln1g, a.ln1b, a.bqkv, o, sA, patch, lane, wv, [] {}, pst, 30);
    else
      lng_phase<LE_QKV>(w, a.wqkv, 3 * kD, MT, B, rx, a.ln1g, a.ln1b, a.bqkv, o, sA, patch, lane, wv, [] {}, pst, 30);
  } else if (a.fin_out) {
    // phase 5 of the last layer: the decoder's final LayerNorm, one wave per row, with
    // layernorm_kernel's arithmetic (ln_sum4 / ln_sq4 / ln_norm4, butterfly sums), x read
    // sc1 (rows other blocks' phase 4 just wrote)
    grid_barrier(a.bar, e0 + 4, a.err, st);
    sink ^= touched;
    touched = 0u;
    const int row = (int)blockIdx.x * (kNT / 64) + wv;
    if (row < B) {  // wave-uniform
      float4 v[2], gg[2], bb[2];
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = lane + 64 * k;
        v[k] = as_f4(ld_sc1(rx, (uint32_t)(row * kD + 4 * c) * 4));
        gg[k] = reinterpret_cast<const float4*>(a.fing)[c];
        bb[k] = reinterpret_cast<const float4*>(a.finb)[c];
        s += ln_sum4(v[k]);
      }
      s = wave_sum_f32(s);
      const float mean = s / kD;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) q += ln_sq4(v[k], mean);
      q = wave_sum_f32(q);
      const float rstd = rsqrtf(q / kD + 1e-5f);
#pragma unroll
      for (int k = 0; k < 2; ++k)
        reinterpret_cast<half4*>(a.fin_out + (int64_t)row * kD)[lane + 64 * k] =
            ln_norm4(v[k], mean, rstd, gg[k], bb[k]);
    }
  }
}

// Self-attention phase of the layer kernel: decode_head_kernel's lane layout (lane: key
// 8r + (lane >> 3) of a round, dims 8 (lane & 7) ..) over 64-key chunks, all 16 K / V loads
// of a chunk in flight, online softmax across chunks (exp2 domain, explicit fmaf), the 8
// key groups summed by shuffles. Cache rows below a row's position come from earlier
// launches (loaded non-temporal, as the launch path does); the chunk holding the newest
// row — written by phase 5 of this launch — is loaded sc1, as is q.
struct AttnState {
  float m, l, acc[8];
};

__device__ __forceinline__ void attn_init(AttnState& t) {
  t.m = -INFINITY;
  t.l = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) t.acc[j] = 0.f;
}

__device__ __forceinline__ void attn_q(const DecSegArgs& g, int b, int h, int dg, float (&qv)[8]) {
  constexpr float kScaleLog2 = 0.125f * 1.4426950408889634f;  // 1 / sqrt(64), exp2 domain
  const half8 qh = as_h8(ld_sc1(rsrc(g.qkv, (uint32_t)g.B * 3 * kD * 2),
                                (uint32_t)((b * 3 * kD + h * 64 + dg * 8) * 2)));
#pragma unroll
  for (int j = 0; j < 8; ++j) qv[j] = (float)qh[j] * kScaleLog2;
}

// keys [k0, k1) (k0 a multiple of 64, k1 <= cpos + 1) of row b, head h into the state
__device__ __forceinline__ void attn_keys(const DecSegArgs& g, int b, int h, int k0, int k1, int cpos,
                                          const float (&qv)[8], AttnState& t, int lane) {
  const int kg = lane >> 3, dg = lane & 7;
  const uint32_t kvbytes = (uint32_t)g.B * g.n_ctx * kD * 2;
  const auto rk = rsrc(g.kc, kvbytes), rv = rsrc(g.vc, kvbytes);
  const uint32_t rowoff = (uint32_t)(((b * g.n_ctx) * kD + h * 64 + dg * 8) * 2);
  for (int c0 = k0; c0 < k1; c0 += 64) {
    u32x4v kr[8], vr[8];
    if (c0 + 64 > cpos) {  // wave-uniform: the chunk holding the newest row
#pragma unroll
      for (int r = 0; r < 8; ++r)
        kr[r] = ld_sc1(rk, rowoff + (uint32_t)min(c0 + 8 * r + kg, cpos) * (kD * 2));
#pragma unroll
      for (int r = 0; r < 8; ++r)
        vr[r] = ld_sc1(rv, rowoff + (uint32_t)min(c0 + 8 * r + kg, cpos) * (kD * 2));
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        kr[r] = __builtin_amdgcn_raw_buffer_load_b128(rk, rowoff + (uint32_t)(c0 + 8 * r + kg) * (kD * 2), 0, 2);
#pragma unroll
      for (int r = 0; r < 8; ++r)
        vr[r] = __builtin_amdgcn_raw_buffer_load_b128(rv, rowoff + (uint32_t)(c0 + 8 * r + kg) * (kD * 2), 0, 2);
    }
    float sc[8], cm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const half8 k8 = as_h8(kr[r]);
      float dot = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) dot = fmaf((float)k8[j], qv[j], dot);
      dot += xshfl<1>(dot);
      dot += xshfl<2>(dot);
      dot += xshfl<4>(dot);
      sc[r] = c0 + 8 * r + kg < k1 ? dot : -INFINITY;
      cm = fmaxf(cm, sc[r]);
    }
    cm = fmaxf(cm, xshfl<8>(cm));
    cm = fmaxf(cm, xshfl<16>(cm));
    cm = fmaxf(cm, xshfl<32>(cm));
    const float m_new = fmaxf(t.m, cm);  // finite: every chunk holds key c0 < k1
    const float alpha = exp2f(t.m - m_new);
    t.l *= alpha;
#pragma unroll
    for (int j = 0; j < 8; ++j) t.acc[j] *= alpha;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float p = exp2f(sc[r] - m_new);  // -inf -> 0
      t.l += p;
      const half8 v8 = as_h8(vr[r]);
#pragma unroll
      for (int j = 0; j < 8; ++j) t.acc[j] = fmaf(p, (float)v8[j], t.acc[j]);
    }
    t.m = m_new;
  }
  // the 8 key groups (lanes sharing dg) share m: plain sums
  auto merge = [&](auto sh) __attribute__((always_inline)) {
    t.l += sh(t.l);
#pragma unroll
    for (int j = 0; j < 8; ++j) t.acc[j] += sh(t.acc[j]);
  };
  merge([](float x) { return xshfl<8>(x); });
  merge([](float x) { return xshfl<16>(x); });
  merge([](float x) { return xshfl<32>(x); });
}

__device__ __forceinline__ void attn_store(const DecSegArgs& g, int b, int h, const AttnState& t, int lane) {
  if ((lane >> 3) == 0) {
    const float il = 1.0f / t.l;
    half8 o8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o8[j] = (_Float16)(t.acc[j] * il);
    st_sc1(__builtin_bit_cast(u32x4v, o8), rsrc(g.o, (uint32_t)g.B * kD * 2),
           (uint32_t)((b * kD + h * 64 + (lane & 7) * 8) * 2));
  }
}

// Work split. Every row's keys are cut in two parts by its own length only (the first
// s(n) = 64 ceil(n / 128) keys and the rest), so a row's arithmetic — part one, part two,
// merged in that order — does not depend on the rows beside it (staggered bit-identity).
// Block j takes head group 4 (j >= H2) .. + 3 of rows a = j mod H2 and b = a + H2 (H2 =
// ceil(B / 2): in the staggered call one row of each slot set, S positions apart); waves w
// and w + 4 share head h: wave w runs a's first part and b's second, wave w + 4 b's first
// and a's second — about the same keys on every wave whatever the two rows' lengths (one
// (row, head) per wave left the longest rows' waves with three times the shortest's keys)
// — and each finishes its first-part row with the partner's second part through LDS.
__device__ __forceinline__ int attn_split(int n) { return min(n, 64 * ((n + 127) / 128)); }

__device__ __forceinline__ void attn_block(const DecSegArgs& g, float* lds, int lane, int wv, int j) {
  const int B = g.B, H2 = (B + 1) >> 1;
  const int p = j % H2;
  const int h = (j >= H2 ? 4 : 0) + (wv & 3);
  const bool hasb = p + H2 < B;
  // this wave's first-part row r1 and second-part row r2
  const int r1 = wv < 4 ? p : p + H2, r2 = wv < 4 ? p + H2 : p;
  const bool has1 = wv < 4 || hasb, has2 = wv < 4 ? hasb : true;
  float qv[8];
  // second part first, straight to the partner's LDS slot (one state live at a time)
  float* mine = lds + ((wv & 3) * 2 + (wv >> 2)) * 80;       // [8 lanes][8 acc] + [m, l]
  const float* other = lds + ((wv & 3) * 2 + 1 - (wv >> 2)) * 80;
  {
    AttnState t2;
    attn_init(t2);
    if (has2) {
      const int c2 = g.pos + (g.roff ? g.roff[r2] : 0);
      const int s2 = attn_split(c2 + 1);
      if (s2 < c2 + 1) {
        attn_q(g, r2, h, lane & 7, qv);
        attn_keys(g, r2, h, s2, c2 + 1, c2, qv, t2, lane);
      }
    }
    if (lane < 8) {
#pragma unroll
      for (int q = 0; q < 8; ++q) mine[lane * 8 + q] = t2.acc[q];
      if (lane == 0) { mine[64] = t2.m; mine[65] = t2.l; }
    }
  }
  AttnState t1;
  attn_init(t1);
  if (has1) {
    const int c1 = g.pos + (g.roff ? g.roff[r1] : 0);
    attn_q(g, r1, h, lane & 7, qv);
    attn_keys(g, r1, h, 0, attn_split(c1 + 1), c1, qv, t1, lane);
  }
  __syncthreads();
  if (has1) {
    const float m2 = other[64], l2 = other[65];
    if (m2 != -INFINITY) {  // the row has a second part (block-uniform per pair)
      const float M = fmaxf(t1.m, m2);
      const float f1 = exp2f(t1.m - M), f2 = exp2f(m2 - M);
      t1.l = t1.l * f1 + l2 * f2;
      if (lane < 8) {
#pragma unroll
        for (int q = 0; q < 8; ++q) t1.acc[q] = t1.acc[q] * f1 + other[lane * 8 + q] * f2;
      }
    }
    attn_store(g, r1, h, t1, lane);
  }
}

// blocks j < 2 ceil(B / 2); at 256 rows on a 128-block grid each block takes j and j + G (the
// LDS hand-off slots are reused: a barrier between the two)
template <bool BIG>
__device__ __forceinline__ void attn_phase(const DecSegArgs& g, float* lds, int lane, int wv) {
  const int n = 2 * ((g.B + 1) >> 1);
  if constexpr (!BIG) {
    if ((int)blockIdx.x < n) attn_block(g, lds, lane, wv, blockIdx.x);  // block-uniform
  } else {
    for (int j = blockIdx.x; j < n; j += gridDim.x) {  // block-uniform
      if (j != (int)blockIdx.x) __syncthreads();
      attn_block(g, lds, lane, wv, j);
    }
  }
}

// Cross-attention phase (layer / head kernel, after segment A): block b takes row b with
// xattn_kernel's one-split body (xattn_body.h), its query rows read sc1 (written by this
// launch's segment A), c written to xc for the next launch's segment B.
constexpr int kXattnLds = XGeo<kD, 64>::LDS;
template <bool BIG>
__device__ __forceinline__ void xattn_phase(const DecSegArgs& g, float* lds) {
  if constexpr (!BIG) {
    const int b = blockIdx.x;
    if (b >= g.B) return;  // block-uniform
    xattn_body<kD, 64, false, true, false, true>(g.xqk, g.enc, g.Te, 8, (g.Te + 63) / 64 * 64, nullptr, nullptr,
                                                 nullptr, const_cast<_Float16*>(g.xc), 0, 1, b,
                                                 reinterpret_cast<_Float16*>(lds));
  } else {
    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {  // block-uniform
      if (b != (int)blockIdx.x) __syncthreads();
      xattn_body<kD, 64, false, true, false, true>(g.xqk, g.enc, g.Te, 8, (g.Te + 63) / 64 * 64, nullptr, nullptr,
                                                   nullptr, const_cast<_Float16*>(g.xc), 0, 1, b,
                                                   reinterpret_cast<_Float16*>(lds));
    }
  }
}

// the touched dwords feed a store no reader looks at (word 150 of the counter block is
// unused), taken with probability 2^-32: the loads cannot be dropped
#define SEG_SINK(A, T, S) do { if (((S) ^ (T)) == 0x5eed5eedu) (A).bar[150] = 1u; } while (0)

template <bool BIG>
__global__ __launch_bounds__(kNT, 4) void dec_seg_a_kernel(DecSegArgs a) {
  JANUS_DEC_WAVE_PRIO();
  extern __shared__ __attribute__((aligned(16))) float seg_smem[];
  long long* st = seg_stamps(a.prof, 0);
  uint32_t touched = 0u, sink = 0u;
  seg_a_body<BIG>(a, seg_smem, st, st, 0, touched, sink);
  SEG_SINK(a, touched, sink);
  SEG_END(st);
  grid_exit(a.bar);
}

template <bool BIG>
__global__ __launch_bounds__(kNT, 4) void dec_seg_b_kernel(DecSegArgs a) {
  JANUS_DEC_WAVE_PRIO();
  extern __shared__ __attribute__((aligned(16))) float seg_smem[];
  long long* st = seg_stamps(a.prof, 1);
  uint32_t touched = 0u, sink = 0u;
  seg_b_body<BIG>(a, seg_smem, st, st, 0, touched, sink);
  SEG_SINK(a, touched, sink);
  SEG_END(st);
  grid_exit(a.bar);
}

// One launch per layer step (r05): segment B of layer l (its phase 5 writes layer l + 1's q
// and K/V rows write-through) | barrier 5 | the self-attention of layer l + 1 | barrier 6 |
// segment A of layer l + 1 — the launches between two cross-attentions as one grid.
template <bool BIG>
__global__ __launch_bounds__(kNT, 4) void dec_layer_kernel(DecSegArgs bsg, DecSegNext nx) {
  JANUS_DEC_WAVE_PRIO();
  extern __shared__ __attribute__((aligned(16))) float seg_smem[];
  long long* st = seg_stamps(bsg.prof, 2);
  const int lane = threadIdx.x & 63, wv = wave_id();
  uint32_t touched = 0u, sink = 0u;
  seg_b_body<BIG>(bsg, seg_smem, st, nullptr, 0, touched, sink);
  grid_barrier(bsg.bar, 5, bsg.err, st);
  sink ^= touched;
  touched = BIG ? touch_quad(nx.wo, kD) : touch_splitk(nx.wo, kD, bsg.MT);
  attn_phase<BIG>(bsg, seg_smem, lane, wv);
  grid_barrier(bsg.bar, 6, bsg.err, st);
  DecSegArgs asg = bsg;
  asg.wo = nx.wo; asg.bo = nx.bo; asg.ln2g = nx.ln2g; asg.ln2b = nx.ln2b; asg.wqk = nx.wqk; asg.bqk = nx.bqk;
  seg_a_body<BIG>(asg, seg_smem, st, nullptr, 6, touched, sink);
  if (bsg.enc) {
    grid_barrier(bsg.bar, 8, bsg.err, st);
    xattn_phase<BIG>(asg, seg_smem);
  }
  SEG_SINK(bsg, touched, sink);
  SEG_END(st);
  grid_exit(bsg.bar);
}

// Layer 0's head: the QKV projection of layer 0 (segment B's phase 5 over the embedded
// rows) | barrier 1 | the self-attention | barrier 2 | segment A of layer 0 — the three
// launches before the first cross-attention as one grid.
template <bool BIG>
__global__ __launch_bounds__(kNT, 4) void dec_head_kernel(DecSegArgs g) {
  JANUS_DEC_WAVE_PRIO();
  extern __shared__ __attribute__((aligned(16))) float seg_smem[];
  long long* st = seg_stamps(g.prof, 0);
  const int lane = threadIdx.x & 63, wv = wave_id();
  uint32_t touched = 0u, sink = 0u;
  {
    _Float16* sA = reinterpret_cast<_Float16*>(seg_smem + kRedF);
    float* patch = reinterpret_cast<float*>(sA + kSegRows * kAP);
    LngW w;
    LngOut o{g.qkv, 3 * kD, g.kc, g.vc, g.pos, g.n_ctx, g.roff};
    const auto rx0 = rsrc(g.x, (uint32_t)g.B * kD * 4);
    if constexpr (BIG)
      lng_phase<LE_QKV, 2>(w, g.wqkv, 3 * kD, g.MT, g.B, rx0, g.ln1g, g.ln1b, g.bqkv, o, sA, patch, lane, wv,
                           [] {}, nullptr, 30);
    else
      lng_phase<LE_QKV>(w, g.wqkv, 3 * kD, g.MT, g.B, rx0, g.ln1g, g.ln1b, g.bqkv, o, sA, patch, lane, wv,
                        [] {}, nullptr, 30);
  }
  grid_barrier(g.bar, 1, g.err, st);
  touched = BIG ? touch_quad(g.wo, kD) : touch_splitk(g.wo, kD, g.MT);
  attn_phase<BIG>(g, seg_smem, lane, wv);
  grid_barrier(g.bar, 2, g.err, st);
  seg_a_body<BIG>(g, seg_smem, st, nullptr, 2, touched, sink);
  if (g.enc) {
    grid_barrier(g.bar, 4, g.err, st);
    xattn_phase<BIG>(g, seg_smem);
  }
  SEG_SINK(g, touched, sink);
  SEG_END(st);
  grid_exit(g.bar);
}

static int seg_per_cu();

int dec_seg_grid(int B, int cus, bool two_per_cu) {
  // rows in 16-row tiles, rounded to a power of two (<= 8); groups of 16-column tiles per
  // m-tile NG in {32, 16} (a divisor of 96, 128 and 256 tiles: QKV, fc1, qk) with
  // MT * NG <= the partition's CUs: one block per CU, every block co-resident
  const int MT = dec_seg_mtiles(B);
  if (MT <= 0) return 0;
  // NG >= 16: at least 16 * MT blocks, one split-K tile pair each
  for (int ng : {32, 16})
    if (MT * ng <= cus) return MT * ng;
  if (MT == 16) {
    // 256 rows on a half-chip partition: 128 blocks taking two split-K pairs / attention
    // blocks each, the LayerNorm GEMM phases at two m-tiles per block (1452 us per position
    // in the staggered step); or (two_per_cu) 256 blocks, two per CU (the segment kernels'
    // 128 VGPRs and LDS admit two: 16 waves per CU), each with the 128-row grid's one-pair
    // work (1492 us; profiles/r06_seg_grid_ab.txt)
    if (two_per_cu && 16 * MT <= 2 * cus && seg_per_cu() >= 2) return 16 * MT;
    if (8 * MT <= cus) return 8 * MT;
  }
  return 0;
}

int dec_seg_mtiles(int B) {
  if (B <= 0 || B > 256) return 0;
  int mt = 1;
  while (mt * 16 < B) mt *= 2;
  return mt;
}

bool dec_seg_supported(int d, int H, int B, int cus) {
  return d == kD && H == 8 && dec_seg_grid(B, cus) > 0;
}

static void seg_attr(const void* k, size_t lds = kSegLds) {
  JANUS_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
}

bool dec_seg_resident(int grid, int cus) { return (int64_t)seg_per_cu() * cus >= grid; }

// co-resident blocks per CU of the segment kernels: the most demanding launch, the layer
// kernel with the cross-attention's LDS tile
static int seg_per_cu() {
  static int per_cu = -1;
  if (per_cu < 0) {
    const size_t lds = std::max(kSegLds, (size_t)kXattnLds);
    int a = 0, b = 0;
    seg_attr((const void*)dec_layer_kernel<false>, lds);
    seg_attr((const void*)dec_layer_kernel<true>, lds);
    JANUS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, dec_layer_kernel<false>, kNT, lds));
    JANUS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, dec_layer_kernel<true>, kNT, lds));
    per_cu = std::min(a, b);
  }
  return per_cu;
}
// the layer and head kernels with the cross-attention phase: its LDS tile on top
static size_t layer_lds(const DecSegArgs& a) {
  return a.enc ? std::max(kSegLds, (size_t)kXattnLds) : kSegLds;
}

// BIG: 256 rows on a 128-block grid (two split-K pairs / attention blocks per block)
static bool seg_big(const DecSegArgs& a, int grid) { return grid < 16 * a.MT; }

template <bool BIG>
static void seg_a_go(const DecSegArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) { seg_attr((const void*)dec_seg_a_kernel<BIG>); attr = true; }
  dec_seg_a_kernel<BIG><<<grid, kNT, kSegLds, s>>>(a);
  JANUS_LAUNCH_CHECK();
}
void dec_seg_a_launch(const DecSegArgs& a, int grid, hipStream_t s) {
  if (seg_big(a, grid)) seg_a_go<true>(a, grid, s);
  else seg_a_go<false>(a, grid, s);
}

template <bool BIG>
static void seg_b_go(const DecSegArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) { seg_attr((const void*)dec_seg_b_kernel<BIG>); attr = true; }
  dec_seg_b_kernel<BIG><<<grid, kNT, kSegLds, s>>>(a);
  JANUS_LAUNCH_CHECK();
}
void dec_seg_b_launch(const DecSegArgs& a, int grid, hipStream_t s) {
  if (seg_big(a, grid)) seg_b_go<true>(a, grid, s);
  else seg_b_go<false>(a, grid, s);
}

template <bool BIG>
static void layer_go(const DecSegArgs& b, const DecSegNext& nx, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) { seg_attr((const void*)dec_layer_kernel<BIG>, std::max(kSegLds, (size_t)kXattnLds)); attr = true; }
  dec_layer_kernel<BIG><<<grid, kNT, layer_lds(b), s>>>(b, nx);
  JANUS_LAUNCH_CHECK();
}
void dec_layer_launch(const DecSegArgs& b, const DecSegNext& nx, int grid, hipStream_t s) {
  const bool big = seg_big(b, grid);
  const int cover = big ? 2 * grid : grid;
  JANUS_CHECK(2 * ((b.B + 1) / 2) <= cover && b.wqkv != nullptr && b.qkv != nullptr,
              "decoder layer kernel: a block per row pair and head group, and a next layer");
  JANUS_CHECK(!b.enc || (b.B <= cover && b.Te > 0), "decoder layer kernel: a block per row for the cross-attention");
  if (big) layer_go<true>(b, nx, grid, s);
  else layer_go<false>(b, nx, grid, s);
}

template <bool BIG>
static void head_go(const DecSegArgs& g, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) { seg_attr((const void*)dec_head_kernel<BIG>, std::max(kSegLds, (size_t)kXattnLds)); attr = true; }
  dec_head_kernel<BIG><<<grid, kNT, layer_lds(g), s>>>(g);
  JANUS_LAUNCH_CHECK();
}
void dec_head_launch(const DecSegArgs& g, int grid, hipStream_t s) {
  const bool big = seg_big(g, grid);
  const int cover = big ? 2 * grid : grid;
  JANUS_CHECK(2 * ((g.B + 1) / 2) <= cover && g.wqkv != nullptr && g.qkv != nullptr,
              "decoder head kernel: a block per row pair and head group, and layer 0's QKV");
  JANUS_CHECK(!g.enc || (g.B <= cover && g.Te > 0), "decoder head kernel: a block per row for the cross-attention");
  if (big) head_go<true>(g, grid, s);
  else head_go<false>(g, grid, s);
}

#ifdef JANUS_PHASE_PROF
// JANUS_SEG_PROF=l: every seg_a / seg_b / layer launch of layer l stamps into one buffer
// (graph replays included), so it holds the last such launch of the run
__device__ long long g_seg_prof[3 * 256 * 48];  // a device global: no allocation under capture
long long* dec_seg_prof_target(int l) {
  static const int want = std::getenv("JANUS_SEG_PROF") ? std::atoi(std::getenv("JANUS_SEG_PROF")) : -1;
  if (l != want) return nullptr;
  void* p = nullptr;
  JANUS_HIP(hipGetSymbolAddress(&p, HIP_SYMBOL(g_seg_prof)));
  return static_cast<long long*>(p);
}
}  // namespace janus
extern "C" int janus_debug_seg_read(long long* dst, int cap) {
  const int n = std::min(cap, 3 * 256);
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(janus::g_seg_prof), sizeof(long long) * 48 * (size_t)n, 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}
namespace janus {
#else
long long* dec_seg_prof_target(int) { return nullptr; }
#endif

}  // namespace janus

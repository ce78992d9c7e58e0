// Fused ResBlock1 unit for the MFMA-width Firefly-GAN stages (C = 64, 128, 256):
//   y = x + c2( silu( c1( silu(x) ) + b1 ) ) + b2 ;  out = (accumulate ? out : 0) + scale * y
// (fish-speech ResBlock1.forward, one (convs1[m], convs2[m]) pair; same contract as the
// narrow-stage kernel in resunit.hip).
//
// Why fused: run as two conv launches, a C = 128 unit moves ~1.3 KB of HBM per time row
// (x read, intermediate written and re-read, residual read, output written) for
// 4*C*C*k FLOP, which leaves the k = 3 / 7 units HBM-bound and the intermediate
// round trip costs a launch boundary per conv. Here one block owns BM output rows:
//   1. stage silu(x) rows [t0 - p2 - p1, t0 + MT1*16 - p2 + (k-1)d) for ALL C channels
//      in LDS (every load of the tile in flight before the first store);
//   2. c1 over MT1*16 rows (>= BM + k - 1: c2's halo) -> silu(. + b1) written as fp16
//      into LDS over the dead sX tile (zero outside [0, T): c2's zero padding);
//   3. c2 over BM rows from that LDS tile; the residual x and the ParallelBlock
//      accumulator rows are loaded into registers at c2's start;
//   4. epilogue through an fp32 LDS tile, 16-byte coalesced loads/stores.
// HBM per unit and time row: read x (+ residual re-read, L2-hot), write out (+ the
// accumulator read on the last unit of a ResBlock1) = 2-3 x C x 2 B.
//
// Both convs are implicit GEMMs on v_mfma_f32_16x16x32_f16 with K = k*C ordered
// tap-major: each 32-wide k-step lies inside one tap, so the A fragment is the LDS tile
// row (m*16 + lane%16 + tap*dil) at channel offset ci. B (weights, packed
// [k-step][Cout][32] so one n-tile fragment is 1 KB contiguous) streams from L2
// straight into registers through an NPB-deep per-wave ring: the K loops carry no LDS
// weight stores and no barriers. Every wave of a block owns distinct output columns
// (WN) or distinct m-tiles (WM); weights are re-read per tile from L2 (~C*k*C*4 B per
// tile, far below the L2's rate at the MFMA pace).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include "mfma.h"
#include "kernels.h"

namespace janus {

// packed[(ks*C + co)*32 + j] = w[co][ci][tap] with kk = ks*32 + j, tap = kk / C, ci = kk % C
__global__ void resunit_wide_pack_kernel(const float* __restrict__ w, _Float16* __restrict__ out,
                                         int C, int k) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)k * C * C;
  if (idx >= total) return;
  const int j = (int)(idx % 32);
  const int co = (int)((idx / 32) % C);
  const int ks = (int)(idx / (32 * (int64_t)C));
  const int kk = ks * 32 + j;
  const int tap = kk / C, ci = kk % C;
  out[idx] = (_Float16)w[((int64_t)co * C + ci) * k + tap];
}

// Phase profile (JANUS_PHASE_PROF builds only, tools/phase_prof.py): thread 0 of every
// block of one chosen unit launch records the shader clock at each phase boundary plus the
// real-time clock and its hardware slot (HW_ID, XCC_ID), 16 values per block.
#ifdef JANUS_PHASE_PROF
#define JANUS_PROF(I)                                                                    \
  do {                                                                                  \
    if (prof && threadIdx.x == 0) prof[(int64_t)blockIdx.x * 16 + (I)] = (long long)clock64(); \
  } while (0)
#else
#define JANUS_PROF(I) do { } while (0)
#endif

#ifdef JANUS_ABL_NOSILU  // timing ablation only (wrong results)
#define WSILU(x) (x)
#else
#define WSILU(x) silu(x)
#endif

template <int C, int V = 0> struct WideCfg;
// BM output rows per block, WM x WN waves (wave tile: every WM-th m-tile x C/WN columns),
// NPB = weight k-steps in flight per wave (divides the k-step count k*C/32).
// EPF: residual / accumulator rows loaded before c2 (in flight during it) where the
// registers allow, else after it.
// NP: epilogue passes (the fp32 tile in NP row slices so the block fits 3 per CU)
template <> struct WideCfg<128> { static constexpr int BM = 112, WM = 1, WN = 4, NPB = 4, NP = 2; static constexpr bool EPF = false, AROT = false; };
// 8 waves (2 x 4): half the m-tiles per wave, so fewer registers per wave and two 8-wave
// blocks per CU (16 waves) instead of three 4-wave blocks (JANUS_WIDE128_CFG=1).
// Measured slower (64 x 30 s, whole GPU: C = 128 units 47.5 -> 59.6 ms): each weight
// fragment is now fetched by two waves; kept as an A/B switch.
// ring depth 2 (the default, JANUS_WIDE128_CFG=2): 16 fewer VGPRs, three blocks per CU
template <> struct WideCfg<128, 2> { static constexpr int BM = 112, WM = 1, WN = 4, NPB = 2, NP = 2; static constexpr bool EPF = false, AROT = true; };
template <> struct WideCfg<128, 1> { static constexpr int BM = 112, WM = 2, WN = 4, NPB = 4, NP = 1; static constexpr bool EPF = false, AROT = false; };
// C = 256 on the register ring (JANUS_WIDE256_CFG=ring): 8 waves x 32 columns over all
// m-tiles, weights from L2 into registers. Per block k-step: A-fragment LDS reads 64 KB
// (512 clocks at 128 B/clock), weight fragments 16 KB over the L1 path (256 clocks), MFMA
// 512 clocks per SIMD — against the LDS-staged form's 80 KB of LDS traffic (640 clocks).
template <> struct WideCfg<256, 3> { static constexpr int BM = 112, WM = 1, WN = 8, NPB = 2, NP = 2; static constexpr bool EPF = false, AROT = false; };
// C = 64 on the register ring (JANUS_WIDE64_CFG=ring): 2 x 2 waves of 32 columns x 6
// m-tiles; per block k-step A-fragment LDS reads 24 KB and weight fragments 8 KB from L2
// (three blocks per CU: 576 / 384 clocks against 576 of MFMA), where the LDS-staged form
// moves 32 KB through LDS (768 clocks). Measured slower all the same (standalone 64 x 30 s,
// C = 64 units 30.9-31.1 vs 30.2 ms): kept as an A/B switch.
template <> struct WideCfg<64, 5> { static constexpr int BM = 176, WM = 2, WN = 2, NPB = 2, NP = 1; static constexpr bool EPF = false, AROT = false; };
// the same with the weight ring 4 deep (the default; one block per CU either way)
template <> struct WideCfg<256, 4> { static constexpr int BM = 112, WM = 1, WN = 8, NPB = 4, NP = 2; static constexpr bool EPF = false, AROT = false; };

template <int C, int V = 0>
struct WideGeo {
  using Cfg = WideCfg<C, V>;
  static constexpr int BM = Cfg::BM, WM = Cfg::WM, WN = Cfg::WN, NPB = Cfg::NPB;
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int LI = frag_pitch(C);        // activation row pitch (halves)
  static constexpr int CPR = C / 8;               // 16-byte chunks per activation row
  static constexpr int MT1 = (BM + 10 + 15) / 16; // c1 m-tiles (k <= 11)
  static constexpr int MT2 = BM / 16;             // c2 m-tiles
  static constexpr int MW1 = (MT1 + WM - 1) / WM; // c1 m-tiles per wave
  static constexpr int MW2 = (MT2 + WM - 1) / WM; // c2 m-tiles per wave
  static constexpr int NTW = C / 16 / WN;         // n-tiles per wave
  static constexpr int R0MAX = MT1 * 16 + 50;     // staged x rows, (k-1)*d <= 50
  static constexpr int NLD = (R0MAX * CPR + NT - 1) / NT;
  static constexpr int ES = C + 4;                // fp32 epilogue row pitch
  static constexpr int NE = (BM * CPR + NT - 1) / NT;
  static constexpr int NP = Cfg::NP;
  static constexpr int RP = 16 * WM * ((MW2 + NP - 1) / NP);  // rows per epilogue pass
  static constexpr int ACT = std::max(R0MAX * LI, MT1 * 16 * LI);
  static constexpr size_t LDS = std::max((size_t)ACT * 2, (size_t)RP * ES * 4);
  // blocks per CU the register budget is sized for (C = 256: one 8-wave block, 256 VGPRs)
  static constexpr int MINB = C == 256 ? 1 : (C == 64 || Cfg::NPB == 2 ? 3 : 2);
  static_assert(BM % 16 == 0 && C % (16 * WN) == 0 && C % 32 == 0, "tiling");
};

// A wave past the last m-tile of a conv recomputes its own last tile (result dropped in
// the epilogue): no branch around an MFMA (branches there made the compiler shuttle
// accumulators between AGPRs; see resunit.hip).
template <int MT, int WM>
__device__ __forceinline__ int own_tile(int j, int wm) {
  if (j < MT / WM) return j;
  return wm + j * WM < MT ? j : (MT - 1 - wm) / WM;
}

template <int C, int MW, int MT, class G, bool AROT = false>
__device__ __forceinline__ void wide_conv(f32x4 (&acc)[MW][G::NTW], const _Float16* __restrict__ wp,
                                          const _Float16* src, int dil, int nks, int wm,
                                          int a_lane, int b_lane) {
  constexpr int NTW = G::NTW, NPB = G::NPB, LI = G::LI, WM = G::WM;
  // at least one ring turn (k*C/32 >= NPB, checked at launch): without it the compiler
  // guards the loop and sinks the ring preload into the guard, out of ring order
  __builtin_assume(nks >= NPB);
  if constexpr (AROT) {
    // A fragments in ONE register set, refilled per m-tile: m-tile j's fragment for step
    // ks+1 is read as soon as step ks's MFMAs on it are issued, so it has the other MW-1
    // m-tiles' MFMAs to land (half the A registers of the double-buffered form below).
#pragma unroll
    for (int j = 0; j < MW; ++j)
#pragma unroll
      for (int n = 0; n < NTW; ++n) acc[j][n] = zero_f32x4();
    half8 bq[NPB][NTW];
    const _Float16* wl = wp + b_lane;
    // slots issued in ring order (the loop's vmcnt for slot s counts on it: loaded out of
    // order, the merged loop-header state made every k-step wait for the whole ring)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < NPB; ++s) {
#pragma unroll
      for (int n = 0; n < NTW; ++n)
        bq[s][n] = *reinterpret_cast<const half8*>(wl + ((int64_t)s * C + n * 16) * 32);
      __builtin_amdgcn_sched_barrier(0);
    }
    auto a_addr = [&](int ks) __attribute__((always_inline)) {
      const int kk = ks * 32;  // wave-uniform: one tap
      return src + a_lane + (kk / C) * dil * LI + kk % C;
    };
    half8 av[MW];
    {
      const _Float16* ap = a_addr(0);
#pragma unroll
      for (int j = 0; j < MW; ++j)
        av[j] = *reinterpret_cast<const half8*>(ap + own_tile<MT, WM>(j, wm) * WM * 16 * LI);
    }
#pragma nounroll
    for (int ks0 = 0; ks0 < nks; ks0 += NPB) {
#pragma unroll
      for (int s = 0; s < NPB; ++s) {
        const int ks = ks0 + s;
        const _Float16* ap = a_addr(min(ks + 1, nks - 1));
#pragma unroll
        for (int j = 0; j < MW; ++j) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int n = 0; n < NTW; ++n) acc[j][n] = mfma16(av[j], bq[s][n], acc[j][n]);
          av[j] = *reinterpret_cast<const half8*>(ap + own_tile<MT, WM>(j, wm) * WM * 16 * LI);
        }
        __builtin_amdgcn_sched_barrier(0);
        const int nx = min(ks + NPB, nks - 1);
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          bq[s][n] = *reinterpret_cast<const half8*>(wl + ((int64_t)nx * C + n * 16) * 32);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < MW; ++j)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[j][n] = zero_f32x4();
  // B ring: slot s holds k-step (ks0 + s); loads are unconditional (clamped index) so the
  // compiler's vmcnt for a slot never has to cover younger slots' loads
  half8 bq[NPB][NTW];
  const _Float16* wl = wp + b_lane;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < NPB; ++s) {
#pragma unroll
    for (int n = 0; n < NTW; ++n)
      bq[s][n] = *reinterpret_cast<const half8*>(wl + ((int64_t)s * C + n * 16) * 32);
    __builtin_amdgcn_sched_barrier(0);
  }
  // A fragments double-buffered across k-steps: step ks+1's LDS reads are issued before
  // step ks's MFMAs (NPB even keeps the buffer index static)
  static_assert(NPB % 2 == 0, "even ring depth");
  half8 av[2][MW];
  auto a_addr = [&](int ks) __attribute__((always_inline)) {
    const int kk = ks * 32;  // wave-uniform: one tap
    return src + a_lane + (kk / C) * dil * LI + kk % C;
  };
  {
    const _Float16* ap = a_addr(0);
#pragma unroll
    for (int j = 0; j < MW; ++j)
      av[0][j] = *reinterpret_cast<const half8*>(ap + own_tile<MT, WM>(j, wm) * WM * 16 * LI);
  }
  for (int ks0 = 0; ks0 < nks; ks0 += NPB) {
#pragma unroll
    for (int s = 0; s < NPB; ++s) {
      const int ks = ks0 + s;
      const _Float16* ap = a_addr(min(ks + 1, nks - 1));
#pragma unroll
      for (int j = 0; j < MW; ++j)
        av[(s + 1) & 1][j] = *reinterpret_cast<const half8*>(ap + own_tile<MT, WM>(j, wm) * WM * 16 * LI);
      // sched barriers pin the issue order: next A reads, this step's MFMAs, then the
      // ring refill. Without them the scheduler sank every weight load to just before its
      // use (s_waitcnt vmcnt(0) ahead of the MFMA: one exposed L2 round trip per k-step)
      // and the A reads likewise.
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < MW; ++j)
#pragma unroll
        for (int n = 0; n < NTW; ++n) acc[j][n] = mfma16(av[s & 1][j], bq[s][n], acc[j][n]);
      __builtin_amdgcn_sched_barrier(0);
      const int nx = min(ks + NPB, nks - 1);
#pragma unroll
      for (int n = 0; n < NTW; ++n)
        bq[s][n] = *reinterpret_cast<const half8*>(wl + ((int64_t)nx * C + n * 16) * 32);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// KC, DC > 0: the unit's kernel size and dilation at compile time. The stage loop then
// walks rows relative to the tile's first output row, so stage slots [0, BM*CPR/NT) of
// every thread are exactly the residual rows [t0, t0 + BM) in the epilogue's thread
// mapping: those slots stay in registers through c1 and c2 (raw x; the LDS tile holds
// silu(x)) instead of being re-read from HBM after c2 (the 1.4-1.6x traffic of the
// re-reading form). KC = 0: (k, d) at run time, residual re-read after c2.
template <int C, int V, int KC = 0, int DC = 0>
__global__ __launch_bounds__((WideGeo<C, V>::NT), (WideGeo<C, V>::MINB)) void resunit_wide_kernel(ResUnitArgs a,
                                                                         int tiles_per_utt,
                                                                         long long* prof) {
  using G = WideGeo<C, V>;
  constexpr int BM = G::BM, WM = G::WM, NT = G::NT, LI = G::LI;
  constexpr int CPR = G::CPR, MT1 = G::MT1, MT2 = G::MT2, MW1 = G::MW1, MW2 = G::MW2;
  constexpr int NTW = G::NTW, ES = G::ES;
  constexpr bool RES = KC > 0;
  constexpr bool AROT = RES && G::Cfg::AROT;
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  _Float16* sX = smem;                         // [R0][LI] silu(x)
  _Float16* sS = smem;                         // [MT1*16][LI] silu(c1 + b1) (over sX)
  float* sE = reinterpret_cast<float*>(smem);  // [BM][ES] epilogue (over sS)

#ifdef JANUS_PHASE_PROF
  if (prof && threadIdx.x == 0) {
    prof[(int64_t)blockIdx.x * 16 + 8] = (long long)wall_clock64();
    prof[(int64_t)blockIdx.x * 16 + 10] = (long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
    prof[(int64_t)blockIdx.x * 16 + 11] = (long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
  }
#endif
  JANUS_PROF(0);
  const int k = RES ? KC : a.k, d = RES ? DC : a.d, T = a.T;
  const int p1 = d * (k - 1) / 2, p2 = (k - 1) / 2;
  const int R1 = BM + 2 * p2;                  // c1 rows c2 reads
  const int R0 = MT1 * 16 + (k - 1) * d;       // x rows c1 reads
  // consecutive tiles on one XCD: a tile's halo rows are its neighbour's, staged through
  // the same L2
  const int tile = tile_remap(blockIdx.x, gridDim.x);
  const int b = tile / tiles_per_utt, t0 = (tile % tiles_per_utt) * BM;
  const int tid = threadIdx.x, lane = tid & 63, wid = wave_id();
  const int wm = wid % WM, wn = wid / WM;
  const _Float16* xb = a.x + (int64_t)b * T * C;
  _Float16* ob = a.out + (int64_t)b * T * C;
  const int nks = k * C / 32;

  // residual rows x[t0 + r] of this thread's epilogue chunks (RES: kept from the stage)
  constexpr int NR = RES ? BM * CPR / NT : 1;
  static_assert(!RES || (NT % CPR == 0 && (BM * CPR) % NT == 0 && NR == G::NE),
                "resident residual: stage slots = epilogue chunks");
  uint4 rx[NR];
  // ---- 1. stage silu(x): all loads in flight, then convert + store
  if constexpr (RES) {
    constexpr int P = (KC - 1) / 2 + DC * (KC - 1) / 2;  // rows left of t0: p2 + p1
    constexpr int RPI = NT / CPR;                        // rows per stage slot
    constexpr int ILO = -((P + RPI - 1) / RPI);          // first slot (left halo)
    constexpr int R0C = MT1 * 16 + (KC - 1) * DC;        // staged rows
    constexpr int IHI = (R0C - P + RPI - 1) / RPI;       // one past the last slot
    constexpr int NS = IHI - ILO;
    static_assert(ILO <= 0 && IHI >= NR, "stage slots cover the residual rows");
    uint4 pf[NS];
    const int rr0 = tid / CPR, cc = tid % CPR;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int rl = (ILO + i) * RPI + rr0;  // row relative to t0
      const int t = t0 + rl;
      const int tc = min(max(t, 0), T - 1);
#ifdef JANUS_ABL_NOSTAGE  // timing ablation only (wrong results)
      pf[i] = make_uint4(tc, 0, 0, 0);
#else
      pf[i] = ld_act(xb + (int64_t)tc * C + cc * 8);
#endif
      if (!(rl >= -P && rl < R0C - P && t >= 0 && t < T)) pf[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int rl = (ILO + i) * RPI + rr0;
      if (rl >= -P && rl < R0C - P) {
        half8 v = *reinterpret_cast<const half8*>(&pf[i]);
#ifdef JANUS_ABL_NOSILU
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)WSILU((float)v[j]);
#else
        v = silu_h8(v);
#endif
        *reinterpret_cast<half8*>(sX + (rl + P) * LI + cc * 8) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) rx[i] = pf[i - ILO];
  } else {
    const int xbase = t0 - p2 - p1;
    uint4 pf[G::NLD];
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cc = idx % CPR;
      const int t = xbase + r;
      // unconditional load of a clamped row, zeroed below (no branch per load)
      const int tc = min(max(t, 0), T - 1);
#ifdef JANUS_ABL_NOSTAGE  // timing ablation only (wrong results)
      pf[i] = make_uint4(tc, 0, 0, 0);
#else
      pf[i] = ld_act(xb + (int64_t)tc * C + cc * 8);
#endif
      if (!(r < R0 && t >= 0 && t < T)) pf[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cc = idx % CPR;
      if (r < R0) {
        half8 v = *reinterpret_cast<const half8*>(&pf[i]);
#ifdef JANUS_ABL_NOSILU
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)WSILU((float)v[j]);
#else
        v = silu_h8(v);
#endif
        *reinterpret_cast<half8*>(sX + r * LI + cc * 8) = v;
      }
    }
  }
  __syncthreads();

  JANUS_PROF(1);
  const int arow = lane & 15, kq = 8 * (lane >> 4);
  const int a_lane = (wm * 16 + arow) * LI + kq;                 // A: row, k chunk
  const int b_lane = ((wn * NTW) * 16 + arow) * 32 + kq;         // B: column, k chunk

  // ---- 2. c1 over MT1*16 rows (row r <-> time t0 - p2 + r): A = sX[r + tap*d]
  {
    f32x4 acc[MW1][NTW];
    wide_conv<C, MW1, MT1, G, AROT>(acc, a.w1, sX, d, nks, wm, a_lane, b_lane);
    JANUS_PROF(2);
    __syncthreads();  // every wave is done reading sX: write silu(c1 + b1) over it
    JANUS_PROF(3);
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int co = (wn * NTW + n) * 16 + arow;
      const float bias = a.b1[co];
#pragma unroll
      for (int j = 0; j < MW1; ++j) {
        const int m = wm + j * WM;
        if (j >= MT1 / WM && m >= MT1) break;
        float v[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = m * 16 + 4 * (lane >> 4) + rr;
          const int t = t0 - p2 + r;
          // c2 zero-pads its input outside [0, T): a 0/1 factor, not a branch per element
          v[rr] = WSILU(acc[j][n][rr] + bias) * ((r < R1 && t >= 0 && t < T) ? 1.0f : 0.0f);
        }
        st_frag_f16_pairs(sS, LI, m * 16 + 4 * (lane >> 4), co, v, lane);
      }
    }
  }
  __syncthreads();

  // residual x and accumulator rows of this tile (before c2 when Cfg::EPF)
  uint4 rq[G::NE], pq[G::NE];
  auto epi_load = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < G::NE; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cg = (idx % CPR) * 8;
      const bool ok = r < BM && t0 + r < T;
      const int64_t o = (int64_t)(t0 + r) * C + cg;
#ifdef JANUS_ABL_NORES  // timing ablation only (wrong results)
      rq[i] = make_uint4(o, 0, 0, 0);
      pq[i] = make_uint4(ok, 0, 0, 0);
#else
      if constexpr (RES) rq[i] = rx[i];
      else rq[i] = ok ? ld_res(xb + o) : make_uint4(0, 0, 0, 0);
      pq[i] = (ok && a.accumulate) ? ld_res(ob + o) : make_uint4(0, 0, 0, 0);
#endif
    }
  };
  JANUS_PROF(4);
  if constexpr (G::Cfg::EPF) epi_load();

  // ---- 3. c2 over BM rows (row r <-> time t0 + r): A = sS[r + tap]
  f32x4 acc2[MW2][NTW];
  wide_conv<C, MW2, MT2, G, AROT>(acc2, a.w2, sS, 1, nks, wm, a_lane, b_lane);
  JANUS_PROF(5);
  if constexpr (!G::Cfg::EPF) epi_load();
  __syncthreads();  // sS dead: the fp32 epilogue tile takes its place
  JANUS_PROF(6);

  // ---- 4. epilogue in NP row passes (WM == 1: every wave owns all m-tiles): c2 + b2 ->
  // fp32 LDS tile of RP rows, then 16-byte row chunks
  static_assert(G::NP == 1 || WM == 1, "multi-pass epilogue needs WM == 1");
#pragma unroll
  for (int p = 0; p < G::NP; ++p) {
    if (p > 0) __syncthreads();  // the previous pass's sE reads are done
    constexpr int JP = (MW2 + G::NP - 1) / G::NP;  // m-tiles per pass
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int co = (wn * NTW + n) * 16 + arow;
      const float bias = a.b2[co];
#pragma unroll
      for (int j = p * JP; j < (p + 1) * JP && j < MW2; ++j) {
        const int m = wm + j * WM;
        if (j >= MT2 / WM && m >= MT2) break;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          sE[(m * 16 - p * G::RP + 4 * (lane >> 4) + rr) * ES + co] = acc2[j][n][rr] + bias;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < G::NE; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cg = (idx % CPR) * 8;
      if (r < p * G::RP || r >= (p + 1) * G::RP) continue;  // compile-time per (i, p)
      if (r >= BM || t0 + r >= T) continue;
      const int rl = r - p * G::RP;
      const float4 v0 = *reinterpret_cast<const float4*>(sE + rl * ES + cg);
      const float4 v1 = *reinterpret_cast<const float4*>(sE + rl * ES + cg + 4);
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      const half8 xv = *reinterpret_cast<const half8*>(&rq[i]);
      const half8 pv = *reinterpret_cast<const half8*>(&pq[i]);
      half8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[j] = (_Float16)((v[j] + (float)xv[j]) * a.scale + (float)pv[j]);
      if (a.post_silu) {  // block-uniform
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = (_Float16)silu((v[j] + (float)xv[j]) * a.scale + (float)pv[j]);
      }
      st_act(ob + (int64_t)(t0 + r) * C + cg, hv);
    }
  }
  JANUS_PROF(7);
#ifdef JANUS_PHASE_PROF
  if (prof && threadIdx.x == 0) prof[(int64_t)blockIdx.x * 16 + 9] = (long long)wall_clock64();
#endif
}

#ifdef JANUS_PHASE_PROF
// JANUS_PHASE_PROF=C,k,d: the first launch of that unit records into a device buffer
static long long* g_prof = nullptr;
static int g_prof_blocks = 0;
static bool g_prof_done = false;
static long long* phase_prof_target(int C, int k, int d, int blocks) {
  const char* e = std::getenv("JANUS_PHASE_PROF");
  if (!e || g_prof_done) return nullptr;
  int pc = 0, pk = 0, pd = 0;
  if (std::sscanf(e, "%d,%d,%d", &pc, &pk, &pd) != 3 || pc != C || pk != k || pd != d) return nullptr;
  g_prof_done = true;
  g_prof_blocks = blocks;
  JANUS_HIP(hipMalloc(&g_prof, sizeof(long long) * 16 * (size_t)blocks));
  JANUS_HIP(hipMemset(g_prof, 0, sizeof(long long) * 16 * (size_t)blocks));
  return g_prof;
}
}  // namespace janus
extern "C" int janus_debug_phase_read(long long* dst, int cap) {
  if (!janus::g_prof) return 0;
  const int n = std::min(cap, janus::g_prof_blocks);
  if (hipMemcpy(dst, janus::g_prof, sizeof(long long) * 16 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return n;
}
namespace janus {
#endif

template <int C, int V, int KC, int DC>
static void wide_go(const ResUnitArgs& a, hipStream_t s) {
  using G = WideGeo<C, V>;
  static_assert(G::LDS <= 160 * 1024, "LDS");
  auto kern = resunit_wide_kernel<C, V, KC, DC>;
  static bool attr = false;
  if (!attr) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)G::LDS));
    attr = true;
  }
  const int tiles_per_utt = (a.T + G::BM - 1) / G::BM;
  long long* prof = nullptr;
#ifdef JANUS_PHASE_PROF
  prof = phase_prof_target(C, a.k, a.d, tiles_per_utt * a.B);
#endif
  kern<<<(unsigned)(tiles_per_utt * a.B), G::NT, G::LDS, s>>>(a, tiles_per_utt, prof);
  JANUS_LAUNCH_CHECK();
}

template <int C, int V>
static void wide_cfg(const ResUnitArgs& a, hipStream_t s) {
  using G = WideGeo<C, V>;
  JANUS_CHECK((a.k - 1) * a.d <= 50 && a.k <= 11, "resunit (wide): (k-1)*d must be <= 50, k <= 11");
  JANUS_CHECK((a.k * C / 32) % G::NPB == 0, "resunit (wide): k-step count vs ring depth");
  // Firefly-GAN's ResBlock1 geometry (k in {3, 7, 11} x d in {1, 3, 5}) at compile time with
  // the residual kept resident; JANUS_WIDE_RES=0 (A/B) or any other (k, d): run-time form
  static const bool res = [] { const char* e = ab_env("JANUS_WIDE_RES"); return e ? std::atoi(e) != 0 : true; }();
  constexpr bool fits = G::NT % G::CPR == 0 && (G::BM * G::CPR) % G::NT == 0 &&
                        G::BM * G::CPR / G::NT == G::NE;
  if constexpr (fits) {
    if (res) {
#define JANUS_WIDE_KD(K_, D_) \
    if (a.k == K_ && a.d == D_) return wide_go<C, V, K_, D_>(a, s);
    JANUS_WIDE_KD(3, 1) JANUS_WIDE_KD(3, 3) JANUS_WIDE_KD(3, 5)
    JANUS_WIDE_KD(7, 1) JANUS_WIDE_KD(7, 3) JANUS_WIDE_KD(7, 5)
    JANUS_WIDE_KD(11, 1) JANUS_WIDE_KD(11, 3) JANUS_WIDE_KD(11, 5)
#undef JANUS_WIDE_KD
    }
  }
  wide_go<C, V, 0, 0>(a, s);
}

template <int C, int V = 0> struct LdsCfg;
// ---------------------------------------------------------------------------------
// Variant with the weights staged through LDS (one copy per block, double-buffered,
// each k-block's loads issued two k-blocks ahead into registers): measured faster where
// all waves share the weight columns (C = 64: 4 waves x 64 columns) or where the per-wave
// column slice is wide (C = 256), i.e. where direct per-wave B loads would exceed the
// L2 -> CU rate. Same packed layout ([k-step][Cout][32]).
// BM output rows per block, WM x WN waves, KB = K per weight k-block.
template <> struct LdsCfg<64> { static constexpr int BM = 176, WM = 4, WN = 1, KB = 32; };
template <> struct LdsCfg<256> { static constexpr int BM = 112, WM = 2, WN = 4, KB = 32; };
// twice the waves per block (JANUS_WIDE64_WAVES=8 / JANUS_WIDE256_WAVES=16): fewer m-tiles
// or n-tiles per wave, fewer registers, more waves per SIMD to hide the block's phases.
// Measured (64 x 30 s, whole GPU): C = 64 30.4 -> 34.5 ms, C = 256 level (28.4); the
// narrow units' gain from more waves (resunit.hip) does not carry over to these
// MFMA-heavier tiles. A/B switches only.
template <> struct LdsCfg<64, 1> { static constexpr int BM = 176, WM = 4, WN = 2, KB = 32; };
template <> struct LdsCfg<256, 1> { static constexpr int BM = 112, WM = 4, WN = 4, KB = 32; };

template <int C, int V = 0>
struct LdsGeo {
  using Cfg = LdsCfg<C, V>;
  static constexpr int BM = Cfg::BM, WM = Cfg::WM, WN = Cfg::WN, KB = Cfg::KB;
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int LI = frag_pitch(C);        // activation row pitch (halves)
  static constexpr int LW = frag_pitch(KB);       // weight row pitch (halves)
  static constexpr int CPR = C / 8;               // 16-byte chunks per activation row
  static constexpr int MT1 = (BM + 10 + 15) / 16; // c1 m-tiles (k <= 11)
  static constexpr int MT2 = BM / 16;             // c2 m-tiles
  static constexpr int MW1 = (MT1 + WM - 1) / WM; // c1 m-tiles per wave
  static constexpr int MW2 = (MT2 + WM - 1) / WM; // c2 m-tiles per wave
  static constexpr int NTW = C / 16 / WN;         // n-tiles per wave
  static constexpr int R0MAX = MT1 * 16 + 50;     // staged x rows, (k-1)*d <= 50
  static constexpr int NLD = (R0MAX * CPR + NT - 1) / NT;
  static constexpr int ES = C + 4;                // fp32 epilogue row pitch
  static constexpr int NE = (BM * CPR + NT - 1) / NT;
  // weight uint4 per thread per k-block (WCH 0: fewer chunks than threads, the first
  // C*KB/8 threads carry one each)
  static constexpr int WCH = C * KB / 8 / NT;
  static constexpr int WACT = C * KB / 8;         // weight chunks per k-block
  static constexpr int ACT = std::max(R0MAX * LI, MT1 * 16 * LI);
  static constexpr int ACT_H = (ACT + 7) / 8 * 8; // halves
  // the fp32 epilogue tile spans the activation AND weight regions (both dead by then)
  static constexpr size_t LDS = std::max(((size_t)ACT_H + 2 * (size_t)C * LW) * 2,
                                         (size_t)BM * ES * 4);
  static_assert(BM % 16 == 0 && C % (16 * WN) == 0, "tiling");
  static_assert(C * KB / 8 % NT == 0 || NT % (C * KB / 8) == 0, "weight k-block split");
  static_assert(KB <= C && C % KB == 0 && KB % 32 == 0, "k-block inside one tap");
  static_assert((C / KB) % 2 == 0, "even k-block count (two register slots)");
};

// EPF: load the residual / accumulator rows at c2's start (in flight during its MFMAs)
// instead of after its last k-block (costs 2*NE*4 VGPRs across the c2 loop).
// KC / DC: the unit's (k, d) at compile time (0: run-time a.k / a.d) — Firefly's nine
// ResBlock1 geometries get constant tap offsets, k-block counts and staged-row counts
template <int C, bool EPF, int V, int KC = 0, int DC = 0>
__global__ __launch_bounds__((LdsGeo<C, V>::NT), 3) void resunit_wide_lds_kernel(ResUnitArgs a,
                                                                         int tiles_per_utt) {
  using G = LdsGeo<C, V>;
  constexpr int BM = G::BM, WM = G::WM, KB = G::KB, NT = G::NT, LI = G::LI, LW = G::LW;
  constexpr int CPR = G::CPR, MT1 = G::MT1, MT2 = G::MT2, MW1 = G::MW1, MW2 = G::MW2;
  constexpr int NTW = G::NTW, ES = G::ES;
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  _Float16* sX = smem;                         // [R0][LI] silu(x)
  _Float16* sS = smem;                         // [MT1*16][LI] silu(c1 + b1) (over sX)
  float* sE = reinterpret_cast<float*>(smem);  // [BM][ES] epilogue (over sS and sW)
  _Float16* sW = smem + G::ACT_H;              // [2][C][LW]

  const int k = KC ? KC : a.k, d = DC ? DC : a.d, T = a.T;
  const int p1 = d * (k - 1) / 2, p2 = (k - 1) / 2;
  const int R1 = BM + 2 * p2;                  // c1 rows c2 reads
  const int R0 = MT1 * 16 + (k - 1) * d;       // x rows c1 reads
  // consecutive tiles on one XCD: a tile's halo rows are its neighbour's, staged through
  // the same L2
  const int tile = tile_remap(blockIdx.x, gridDim.x);
  const int b = tile / tiles_per_utt, t0 = (tile % tiles_per_utt) * BM;
  const int tid = threadIdx.x, lane = tid & 63, wid = wave_id();
  const int wm = wid % WM, wn = wid / WM;
  const _Float16* xb = a.x + (int64_t)b * T * C;
  _Float16* ob = a.out + (int64_t)b * T * C;
  const int nkb = k * C / KB;

  // weight k-blocks: two register slots, each load issued two k-blocks before its LDS
  // store (an L2 round trip is longer than one k-block of MFMAs at KB = 32). Plain
  // locals + macros: captured by reference in lambdas they were left in scratch memory.
  static_assert(G::WCH <= 2, "weight slot width");
  const int wt = min(tid, G::WACT - 1);  // WCH 0: threads past WACT repeat a chunk, store none
  const bool wst = G::WCH > 0 || tid < G::WACT;
  const int wsrc0 = (wt / (KB / 8)) * KB + (wt % (KB / 8)) * 8;
  const int wdst0 = (wt / (KB / 8)) * LW + (wt % (KB / 8)) * 8;
  const int wsrc1 = ((tid + NT) / (KB / 8)) * KB + ((tid + NT) % (KB / 8)) * 8;
  const int wdst1 = ((tid + NT) / (KB / 8)) * LW + ((tid + NT) % (KB / 8)) * 8;
  uint4 rwA0, rwA1, rwB0, rwB1;
#define WIDE_WLOAD(R0_, R1_, WP, KBI)                                                   \
  do {                                                                                  \
    const _Float16* src_ = (WP) + (int64_t)(KBI) * C * KB;                              \
    R0_ = *reinterpret_cast<const uint4*>(src_ + wsrc0);                                \
    if constexpr (G::WCH == 2) R1_ = *reinterpret_cast<const uint4*>(src_ + wsrc1);      \
  } while (0)
#define WIDE_WSTORE(R0_, R1_, BUF)                                                      \
  do {                                                                                  \
    _Float16* dst_ = sW + (BUF) * C * LW;                                               \
    if (wst) *reinterpret_cast<uint4*>(dst_ + wdst0) = R0_;                             \
    if constexpr (G::WCH == 2) *reinterpret_cast<uint4*>(dst_ + wdst1) = R1_;            \
  } while (0)

  // ---- 1. stage silu(x): all loads in flight, then convert + store
  {
    const int xbase = t0 - p2 - p1;
    // window rows [0, R0 - BM) are the previous tile's, [BM, R0) the next tile's: those
    // stay in L2 for the neighbour (per wave: any of its rows shared)
    const int wr0 = wid * 64 / CPR;  // first window row of this wave at i = 0
    uint4 pf[G::NLD];
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cc = idx % CPR;
      const int t = xbase + r;
      const int rw = wr0 + i * (NT / CPR);  // wave-uniform
      const bool keep = JANUS_STAGE_KEEP_ALL || rw < R0 - BM || rw + 64 / CPR > BM;
      // unconditional load of a clamped row, zeroed below (no branch per load)
      const int tc = min(max(t, 0), T - 1);
      pf[i] = ld_act_halo(xb + (int64_t)tc * C + cc * 8, keep);
      if (!(r < R0 && t >= 0 && t < T)) pf[i] = make_uint4(0, 0, 0, 0);
    }
    WIDE_WLOAD(rwA0, rwA1, a.w1, 0);
    WIDE_WLOAD(rwB0, rwB1, a.w1, 1);
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cc = idx % CPR;
      if (r < R0) {
        half8 v = *reinterpret_cast<const half8*>(&pf[i]);
#ifdef JANUS_ABL_NOSILU
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)WSILU((float)v[j]);
#else
        v = silu_h8(v);
#endif
        *reinterpret_cast<half8*>(sX + r * LI + cc * 8) = v;
      }
    }
    WIDE_WSTORE(rwA0, rwA1, 0);
  }
  __syncthreads();

  const int kq = 8 * (lane >> 4);
  const int arow = lane & 15;
  const _Float16* bbase = sW + (wn * NTW * 16 + arow) * LW + kq;

  // one k-block of MFMAs: A rows (m*16 + lane%16 + tap*dil) of src, B from weight buffer buf
  auto mma = [&](auto& acc, auto mw_tag, auto mt_tag, const _Float16* src, int dil, int kb,
                 int buf) __attribute__((always_inline)) {
    constexpr int MW = decltype(mw_tag)::value, MT = decltype(mt_tag)::value;
    const _Float16* wb = bbase + buf * C * LW;
#pragma unroll
    for (int ks = 0; ks < KB / 32; ++ks) {
      const int kk = kb * KB + ks * 32;  // wave-uniform: one tap
      const int tap = kk / C, ci = kk % C;
      half8 bw[NTW];
#pragma unroll
      for (int n = 0; n < NTW; ++n) bw[n] = *reinterpret_cast<const half8*>(wb + n * 16 * LW + ks * 32);
      const _Float16* ap = src + (wm * 16 + arow + tap * dil) * LI + ci + kq;
#pragma unroll
      for (int j = 0; j < MW; ++j) {
        // a wave past the last m-tile recomputes it (dropped in the epilogue): no branch
        // around the MFMA (see resunit.hip)
        const int jj = (j < MT / WM) ? j : (wm + j * WM < MT ? j : (MT - 1 - wm) / WM);
        const half8 av = *reinterpret_cast<const half8*>(ap + jj * WM * 16 * LI);
#pragma unroll
        for (int n = 0; n < NTW; ++n) acc[j][n] = mfma16(av, bw[n], acc[j][n]);
      }
    }
  };
  // the K loop of one conv; on entry buffer 0 holds k-block 0 and slot B k-block 1
  // (nkb = k*C/KB is even: two k-blocks per trip keep the register slots static; the
  // loads are unconditional (clamped index) so the compiler's vmcnt for slot B never
  // has to cover slot A's younger loads)
// (sched barriers pin each weight load ahead of the MFMAs it is meant to overlap: left
// free, the scheduler sank the loads past the next k-block's MFMAs, one k-block of cover
// instead of two)
#define WIDE_KLOOP(ACC, MWT, MTT, WP, SRC, DIL)                                         \
  for (int kb = 0; kb < nkb; kb += 2) {                                                 \
    WIDE_WLOAD(rwA0, rwA1, WP, min(kb + 2, nkb - 1));                                   \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    mma(ACC, MWT{}, MTT{}, SRC, DIL, kb, 0);                                            \
    WIDE_WSTORE(rwB0, rwB1, 1);                                                         \
    __syncthreads();                                                                    \
    WIDE_WLOAD(rwB0, rwB1, WP, min(kb + 3, nkb - 1));                                   \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    mma(ACC, MWT{}, MTT{}, SRC, DIL, kb + 1, 1);                                        \
    if (kb + 2 < nkb) WIDE_WSTORE(rwA0, rwA1, 0);                                       \
    __syncthreads();                                                                    \
  }
  using MW1T = std::integral_constant<int, MW1>;
  using MT1T = std::integral_constant<int, MT1>;
  using MW2T = std::integral_constant<int, MW2>;
  using MT2T = std::integral_constant<int, MT2>;

  // ---- 2. c1 over MT1*16 rows (row r <-> time t0 - p2 + r): A = sX[r + tap*d]
  {
    f32x4 acc[MW1][NTW];
#pragma unroll
    for (int j = 0; j < MW1; ++j)
#pragma unroll
      for (int n = 0; n < NTW; ++n) acc[j][n] = zero_f32x4();
    WIDE_KLOOP(acc, MW1T, MT1T, a.w1, sX, d);
    // sX is dead (last barrier of the loop): write silu(c1 + b1) over it
    WIDE_WLOAD(rwA0, rwA1, a.w2, 0);
    WIDE_WLOAD(rwB0, rwB1, a.w2, 1);
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int co = (wn * NTW + n) * 16 + arow;
      const float bias = a.b1[co];
#pragma unroll
      for (int j = 0; j < MW1; ++j) {
        const int m = wm + j * WM;
        if (j >= MT1 / WM && m >= MT1) break;
        float v[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = m * 16 + 4 * (lane >> 4) + rr;
          const int t = t0 - p2 + r;
          // c2 zero-pads its input outside [0, T): a 0/1 factor, not a branch per element
          v[rr] = WSILU(acc[j][n][rr] + bias) * ((r < R1 && t >= 0 && t < T) ? 1.0f : 0.0f);
        }
        st_frag_f16_pairs(sS, LI, m * 16 + 4 * (lane >> 4), co, v, lane);
      }
    }
    WIDE_WSTORE(rwA0, rwA1, 0);
  }
  __syncthreads();

  // residual x and accumulator rows of this tile
  uint4 rq[G::NE], pq[G::NE];
  auto epi_load = [&]() {
#pragma unroll
    for (int i = 0; i < G::NE; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cg = (idx % CPR) * 8;
      const bool ok = r < BM && t0 + r < T;
      const int64_t o = (int64_t)(t0 + r) * C + cg;
      rq[i] = ok ? ld_res(xb + o) : make_uint4(0, 0, 0, 0);
      pq[i] = (ok && a.accumulate) ? ld_res(ob + o) : make_uint4(0, 0, 0, 0);
    }
  };
  if constexpr (EPF) epi_load();

  // ---- 3. c2 over BM rows (row r <-> time t0 + r): A = sS[r + tap]
  f32x4 acc2[MW2][NTW];
#pragma unroll
  for (int j = 0; j < MW2; ++j)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc2[j][n] = zero_f32x4();
  WIDE_KLOOP(acc2, MW2T, MT2T, a.w2, sS, 1);
  if constexpr (!EPF) epi_load();

  // ---- 4. epilogue: c2 + b2 -> fp32 LDS tile (sS dead), then 16-byte row chunks
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    const int co = (wn * NTW + n) * 16 + arow;
    const float bias = a.b2[co];
#pragma unroll
    for (int j = 0; j < MW2; ++j) {
      const int m = wm + j * WM;
      if (j >= MT2 / WM && m >= MT2) break;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) sE[(m * 16 + 4 * (lane >> 4) + rr) * ES + co] = acc2[j][n][rr] + bias;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < G::NE; ++i) {
    const int idx = tid + i * NT;
    const int r = idx / CPR, cg = (idx % CPR) * 8;
    if (r >= BM || t0 + r >= T) continue;
    const float4 v0 = *reinterpret_cast<const float4*>(sE + r * ES + cg);
    const float4 v1 = *reinterpret_cast<const float4*>(sE + r * ES + cg + 4);
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const half8 xv = *reinterpret_cast<const half8*>(&rq[i]);
    const half8 pv = *reinterpret_cast<const half8*>(&pq[i]);
    half8 hv;
#pragma unroll
    for (int j = 0; j < 8; ++j) hv[j] = (_Float16)((v[j] + (float)xv[j]) * a.scale + (float)pv[j]);
      if (a.post_silu) {  // block-uniform
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = (_Float16)silu((v[j] + (float)xv[j]) * a.scale + (float)pv[j]);
      }
    st_act(ob + (int64_t)(t0 + r) * C + cg, hv);
  }
}

#undef WIDE_WLOAD
#undef WIDE_WSTORE
#undef WIDE_KLOOP

template <int C, bool EPF, int V, int KC, int DC>
static void lds_go(const ResUnitArgs& a, hipStream_t s) {
  using G = LdsGeo<C, V>;
  static_assert(G::LDS <= 160 * 1024, "LDS");
  auto kern = resunit_wide_lds_kernel<C, EPF, V, KC, DC>;
  static bool attr = false;
  if (!attr) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)G::LDS));
    attr = true;
  }
  const int tiles_per_utt = (a.T + G::BM - 1) / G::BM;
  kern<<<(unsigned)(tiles_per_utt * a.B), G::NT, G::LDS, s>>>(a, tiles_per_utt);
  JANUS_LAUNCH_CHECK();
}

template <int C, bool EPF, int V>
static void lds_cfg(const ResUnitArgs& a, hipStream_t s) {
  JANUS_CHECK((a.k - 1) * a.d <= 50 && a.k <= 11, "resunit (wide): (k-1)*d must be <= 50, k <= 11");
  // Firefly-GAN's ResBlock1 geometry (k in {3, 7, 11} x d in {1, 3, 5}) compiled per (k, d)
  // for C = 64 (r05; JANUS_WIDE_LDS_RT=1: the run-time form, A/B): standalone 64 x 30 s
  // forward, C = 64 units 29.7-29.8 vs 30.7 ms; step 250.3-251.2 vs 251.5-251.9 ms
  // (profiles/r05_c64_kd_ab.txt); any other (k, d) and C run the run-time form
  static const bool rt = ab_env("JANUS_WIDE_LDS_RT") != nullptr;
  if constexpr (C == 64 && V == 0) {
    if (!rt) {
#define JANUS_LDS_KD(K_, D_) \
      if (a.k == K_ && a.d == D_) return lds_go<C, EPF, V, K_, D_>(a, s);
      JANUS_LDS_KD(3, 1) JANUS_LDS_KD(3, 3) JANUS_LDS_KD(3, 5)
      JANUS_LDS_KD(7, 1) JANUS_LDS_KD(7, 3) JANUS_LDS_KD(7, 5)
      JANUS_LDS_KD(11, 1) JANUS_LDS_KD(11, 3) JANUS_LDS_KD(11, 5)
#undef JANUS_LDS_KD
    }
  }
  lds_go<C, EPF, V, 0, 0>(a, s);
}

bool resunit_wide_supported(int C, int k, int d) {
  static const bool off = ab_env("JANUS_NO_WIDE_UNITS") != nullptr;
  return !off && (C == 64 || C == 128 || C == 256) && k >= 1 && k <= 11 && (k & 1) &&
         (k - 1) * d <= 50;
}

void resunit_wide_pack(const float* w, _Float16* out, int C, int k, hipStream_t s) {
  const int64_t total = (int64_t)k * C * C;
  resunit_wide_pack_kernel<<<(unsigned)cdiv(total, 256), 256, 0, s>>>(w, out, C, k);
  JANUS_LAUNCH_CHECK();
}

void resunit_wide_launch(const ResUnitArgs& a, hipStream_t s) {
  static const int epf = [] { const char* e = ab_env("JANUS_WIDE_EPF"); return e ? std::atoi(e) : 1; }();
  static const int w64 = ab_env("JANUS_WIDE64_WAVES") ? std::atoi(ab_env("JANUS_WIDE64_WAVES")) : 4;
  static const int w256 = ab_env("JANUS_WIDE256_WAVES") ? std::atoi(ab_env("JANUS_WIDE256_WAVES")) : 8;
  if (a.C == 64) {
    static const std::string c64 = ab_env("JANUS_WIDE64_CFG") ? ab_env("JANUS_WIDE64_CFG") : "lds";
    if (c64 == "ring") wide_cfg<64, 5>(a, s);
    else if (w64 == 8) epf ? lds_cfg<64, true, 1>(a, s) : lds_cfg<64, false, 1>(a, s);
    else epf ? lds_cfg<64, true, 0>(a, s) : lds_cfg<64, false, 0>(a, s);
  }
  else if (a.C == 128) {
    // JANUS_WIDE128_CFG: 2 (default) = 4 waves, weight ring 2 deep (166 VGPRs, three blocks
    // per CU); 0 = ring 4 deep (178 VGPRs, two blocks); 1 = 8 waves. Standalone 64 x 30 s,
    // C = 128 units: 45.4 / 49.0 / 59.6 ms (46.5 before the issue order was pinned)
    static const int c128 = ab_env("JANUS_WIDE128_CFG") ? std::atoi(ab_env("JANUS_WIDE128_CFG")) : 2;
    if (c128 == 1) wide_cfg<128, 1>(a, s);
    else if (c128 == 0) wide_cfg<128, 0>(a, s);
    else wide_cfg<128, 2>(a, s);
  }
  else if (a.C == 256) {
    // JANUS_WIDE256_CFG: ring4 (default: weights from L2 into a per-wave register ring 4
    // deep, 8 waves x 32 columns; standalone 64 x 30 s, C = 256 units 27.0 -> 22.3 ms;
    // overlapped step, vocoder side 289 -> 282 ms), ring (2 deep: 22.8 ms), lds (weights
    // staged through LDS, the r01 form)
    static const std::string c256 = ab_env("JANUS_WIDE256_CFG") ? ab_env("JANUS_WIDE256_CFG") : "ring4";
    if (c256 == "ring") wide_cfg<256, 3>(a, s);
    else if (c256 == "ring4") wide_cfg<256, 4>(a, s);
    else if (w256 == 16) epf ? lds_cfg<256, true, 1>(a, s) : lds_cfg<256, false, 1>(a, s);
    else epf ? lds_cfg<256, true, 0>(a, s) : lds_cfg<256, false, 0>(a, s);
  }
  else throw Error("resunit (wide): C must be 64, 128 or 256");
}

}  // namespace janus

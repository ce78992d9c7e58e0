// Fused ResBlock1 unit for the narrow (16/32-channel) Firefly-GAN stages:
//   y = x + c2( silu( c1( silu(x) ) + b1 ) ) + b2 ;  out = (accumulate ? out : 0) + scale * y
// c1: Conv1d(C, C, k, dilation d, padding d(k-1)/2); c2: Conv1d(C, C, k, padding (k-1)/2).
// (fish-speech ResBlock1.forward, one (convs1[m], convs2[m]) pair.)
//
// At C <= 32 each conv alone is HBM-bound (≈0.5 kFLOP per byte moved), so the pair runs
// in ONE kernel: the block stages silu(x) rows [t0 - p2 - p1, t0 + BM + p2 + p1) in LDS,
// computes c1 for rows [t0 - p2, t0 + BM + p2) into an LDS tile (never HBM), then c2 for
// its BM rows, adds the raw-x residual and writes with 16-byte stores. Both weight
// matrices stay in LDS for the block. HBM traffic per unit: read x once (+ the residual
// re-read, L2-hot), write out once — half of two separate conv launches.
#include <algorithm>
#include <cstdlib>
#include "mfma.h"
#include "kernels.h"

namespace janus {

__global__ void resunit_pack_kernel(const float* __restrict__ w, _Float16* __restrict__ out, int C,
                                    int k, int KP) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * KP) return;
  const int co = idx / KP, kk = idx % KP;
  const int tap = kk / C, ci = kk % C;
  out[idx] = tap < k ? (_Float16)w[((int64_t)co * C + ci) * k + tap] : (_Float16)0.0f;
}

int resunit_kp(int C, int k) { return (k * C + 31) / 32 * 32; }

bool resunit_wide_supported(int C, int k, int d);
void resunit_wide_pack(const float* w, _Float16* out, int C, int k, hipStream_t s);
void resunit_wide_launch(const ResUnitArgs& a, hipStream_t s);

void resunit_pack(const float* w, _Float16* out, int C, int k, hipStream_t s) {
  if (C >= 64) {  // resunit_wide.hip layout [kb][Cout][KB]
    resunit_wide_pack(w, out, C, k, s);
    return;
  }
  const int KP = resunit_kp(C, k);
  resunit_pack_kernel<<<(C * KP + 255) / 256, 256, 0, s>>>(w, out, C, k, KP);
  JANUS_LAUNCH_CHECK();
}

// Compile-time geometry: C channels, K taps, dilation D, BM output rows per tile.
// c1 covers M1 = BM + 16 rows (>= BM + K - 1, c2's halo); a 16x16x32 MFMA k-step spans
// TPK = 32 / C taps, so K rounds up to TP taps with zero weights on the padding tap;
// every row a padding tap touches is staged (and finite), so the MFMA loop has no guards.
template <int C, int K, int D, int BM, int NW = 4>
struct NarrowGeo {
  static constexpr int NT = 64 * NW;                    // NW waves per block
  static constexpr int TPK = 32 / C;                    // taps per k-step
  static constexpr int KS = (K + TPK - 1) / TPK;        // k-steps per conv
  static constexpr int KP = KS * 32;                    // packed K (resunit_kp)
  static constexpr int TP = KS * TPK;                   // taps incl. padding
  static constexpr int P1 = D * (K - 1) / 2, P2 = (K - 1) / 2;
  static constexpr int LI = frag_pitch(C);              // activation pitch (halves)
  static constexpr int LW = frag_pitch(KP);             // weight pitch (halves)
  static constexpr int CPR = C / 8;                     // 16-byte chunks per row
  static constexpr int MT1 = BM / 16 + 1, M1 = MT1 * 16;
  static constexpr int MT2 = BM / 16;
  static constexpr int MW1 = (MT1 + NW - 1) / NW, MW2 = (MT2 + NW - 1) / NW;
  static constexpr int NTL = C / 16;                    // n-tiles (all per wave)
  static constexpr int R0 = M1 + (TP - 1) * D;          // staged x rows
  static constexpr int NPF = (R0 * CPR + NT - 1) / NT;  // prefetch uint4 per thread
  static constexpr int ES = C + 4;                      // fp32 epilogue pitch
  static constexpr int NE = (BM * CPR + NT - 1) / NT;   // epilogue uint4 per thread
  // epilogue passes: at C = 32 the fp32 tile goes out in two row halves so that the
  // block fits in 80 KB of LDS (two blocks per CU)
  // (C = 16 too: the half-size fp32 tile brings its block to 31 KB of LDS, four blocks
  // per CU instead of three; JANUS_NARROW16_NP=1 builds the single-pass form)
#ifndef JANUS_NARROW16_NP
#define JANUS_NARROW16_NP 2
#endif
  static constexpr int NP =
      C == 32 ? 2 : (NE % JANUS_NARROW16_NP == 0 && MW2 % JANUS_NARROW16_NP == 0 ? JANUS_NARROW16_NP : 1);
  static constexpr int RP = 16 * NW * (MW2 / NP);       // rows per epilogue pass
  // the residual x rows: kept from the staging in an LDS tile where LDS allows (C = 16),
  // else re-read from global memory (L2-hot) into registers during the convs
  static constexpr bool RES_LDS = C == 16;
  // LDS (halves): [sX | sS | sE alias] [sR] [sW1] [sW2]
  static constexpr int ACT = std::max(std::max(R0 * LI, M1 * LI), RP * ES * 2);
  static constexpr int ACT_H = (ACT + 7) / 8 * 8;
  static constexpr int RES_H = RES_LDS ? BM * LI : 0;
  static constexpr int LDS_H = ACT_H + RES_H + 2 * C * LW;
  static constexpr size_t LDS = (size_t)LDS_H * 2;
  static_assert(KP == (K * C + 31) / 32 * 32, "matches resunit_kp");
  static_assert(BM % 16 == 0 && M1 >= BM + K - 1 && M1 >= BM + TP - 1, "c2 halo");
  static_assert(MW2 % NP == 0 && NE % NP == 0 && NE * NT / CPR / NP == RP, "epilogue passes");
};

// Persistent: weights staged once; per tile the next tile's x rows are loaded into
// registers while this tile computes. Edge tiles (the first and last of an utterance)
// take the guarded epilogue path; interior tiles run unguarded.
template <int C, int K, int D, int BM, int NW>
__global__ __launch_bounds__(64 * NW) void resunit_kernel(ResUnitArgs a, int tiles_per_utt, int n_tiles) {
  using G = NarrowGeo<C, K, D, BM, NW>;
  constexpr int NT = G::NT;
  constexpr int LI = G::LI, LW = G::LW, CPR = G::CPR, ES = G::ES, NTL = G::NTL;
  constexpr int MT1 = G::MT1, MT2 = G::MT2, MW1 = G::MW1, MW2 = G::MW2, M1 = G::M1;
  constexpr int P1 = G::P1, P2 = G::P2, R0 = G::R0, KS = G::KS, KP = G::KP;
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  _Float16* sX = smem;                        // [R0][LI]  silu(x)
  _Float16* sS = smem;                        // [M1][LI]  silu(c1 + b1), over dead sX
  float* sE = reinterpret_cast<float*>(smem); // [RP][ES]  c2 + b2, over dead sS
  _Float16* sR = smem + G::ACT_H;             // [BM][LI]  raw x (RES_LDS only)
  _Float16* sW1 = sR + G::RES_H;              // [C][LW]
  _Float16* sW2 = sW1 + C * LW;               // [C][LW]
  const int T = a.T;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();

  for (int idx = tid; idx < C * (KP / 8); idx += NT) {
    const int co = idx / (KP / 8), cc = idx % (KP / 8);
    *reinterpret_cast<uint4*>(sW1 + co * LW + cc * 8) =
        *reinterpret_cast<const uint4*>(a.w1 + (int64_t)co * KP + cc * 8);
    *reinterpret_cast<uint4*>(sW2 + co * LW + cc * 8) =
        *reinterpret_cast<const uint4*>(a.w2 + (int64_t)co * KP + cc * 8);
  }
  // per-lane bias of the lane's output column (one per n-tile)
  float bias1[NTL], bias2[NTL];
#pragma unroll
  for (int n = 0; n < NTL; ++n) {
    bias1[n] = a.b1[n * 16 + (lane & 15)];
    bias2[n] = a.b2[n * 16 + (lane & 15)];
  }

  uint4 pf[G::NPF];
#define NARROW_PREFETCH(TILE)                                                               \
  do {                                                                                      \
    const int L_ = (TILE);                                                                  \
    const int tl_ = L_ < n_tiles ? tile_of(L_) : 0;                                         \
    const int b_ = tl_ / tiles_per_utt, t0_ = (tl_ % tiles_per_utt) * BM;                   \
    const _Float16* xb_ = a.x + (int64_t)b_ * T * C;                                        \
    _Pragma("unroll") for (int i = 0; i < G::NPF; ++i) {                                    \
      const int idx = tid + i * NT;                                                         \
      const int r = idx / CPR, cc = idx % CPR;                                              \
      const int t = t0_ - P2 - P1 + r;                                                      \
      const int rw_ = w * (64 / CPR) + i * (NT / CPR);                                      \
      pf[i] = (L_ < n_tiles && r < R0  && t >= 0 && t < T)                                 \
                  ? ld_act_halo(xb_ + (int64_t)t * C + cc * 8,                              \
                                C == 32 && (JANUS_STAGE_KEEP_ALL || rw_ < R0 - BM ||        \
                                            rw_ + 64 / CPR > BM))                           \
                  : make_uint4(0, 0, 0, 0);                                                 \
    }                                                                                       \
  } while (0)
  // the grid's blocks walk logical tiles L = blockIdx.x + i * gridDim.x; with gridDim.x % 8
  // == 0 block b stays on one XCD, and xcd_remap gives that XCD a contiguous run of tiles,
  // so the blocks in flight there stage neighbouring tiles (shared halo rows hit its L2)
  // (C = 32 only: it reads 1.10x -> 1.01x its algorithmic bytes at equal time; C = 16
  // compiled with the remap ran 2 ms per step slower, remapped or not)
  const bool xm = C == 32 && (gridDim.x & 7) == 0;
  auto tile_of = [=](int L) {
    if constexpr (C == 32) return xm ? tile_remap(L, n_tiles) : L;
    else return L;
  };
  NARROW_PREFETCH(blockIdx.x);

  // fragment addressing: lane row (lane & 15); k chunk 8*(lane >> 4) -> tap / channel
  const int arow = lane & 15;
  const int kq = 8 * (lane >> 4);
  const int ltap = kq / C, lci = kq % C;      // tap offset and channel of this lane's chunk
  const int a1_off = arow * LI + ltap * D * LI + lci;  // + (m*16 + 2*ks*D... ) below
  const int a2_off = arow * LI + ltap * LI + lci;
  const int b_off = arow * LW + kq;

  for (int L = blockIdx.x; L < n_tiles; L += gridDim.x) {
    const int tile = tile_of(L);
    const int b = tile / tiles_per_utt, t0 = (tile % tiles_per_utt) * BM;
    const bool edge = (t0 - P2 < 0) || (t0 - P2 + M1 > T) || (t0 + BM > T);
    __syncthreads();  // previous tile's epilogue is done with sE / sR
#pragma unroll
    for (int i = 0; i < G::NPF; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cc = idx % CPR;
      if (r < R0) {
        half8 v = *reinterpret_cast<const half8*>(&pf[i]);
        if constexpr (G::RES_LDS) {
          const int rr = r - P2 - P1;
          if (rr >= 0 && rr < BM) *reinterpret_cast<half8*>(sR + rr * LI + cc * 8) = v;
        }
        v = silu_h8(v);
        *reinterpret_cast<half8*>(sX + r * LI + cc * 8) = v;
      }
    }
    __syncthreads();
    NARROW_PREFETCH(L + gridDim.x);  // in flight during this tile's compute
    _Float16* ob = a.out + (int64_t)b * T * C;
    // the residual x rows (re-read: L2-hot since this tile's prefetch) and the
    // accumulator rows, in flight during the convs
    const _Float16* xb = a.x + (int64_t)b * T * C;
    uint4 xres[G::NE], acc_in[G::NE];
#pragma unroll
    for (int i = 0; i < G::NE; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / CPR, cg = (idx % CPR) * 8;
      const bool ok = r < BM && t0 + r < T;
      if constexpr (!G::RES_LDS)
        xres[i] = ok ? ld_res(xb + (int64_t)(t0 + r) * C + cg)
                     : make_uint4(0, 0, 0, 0);
      acc_in[i] = (a.accumulate && ok)
                      ? ld_res(ob + (int64_t)(t0 + r) * C + cg)
                      : make_uint4(0, 0, 0, 0);
    }

    // ---- c1 over M1 rows (row r <-> time t0 - P2 + r): A = sX[r + tap*D]
    {
      f32x4 acc[MW1][NTL];
#pragma unroll
      for (int j = 0; j < MW1; ++j)
#pragma unroll
        for (int n = 0; n < NTL; ++n) acc[j][n] = zero_f32x4();
      // fragments double-buffered across k-steps: step ks+1's LDS reads are issued before
      // step ks's MFMAs. (Left to the compiler, each A read was followed by an
      // lgkmcnt(0) wait and two MFMAs: the LDS latency, not the MFMA, paced the loop —
      // 26 % matrix-core busy on C = 32, k = 11.)
      half8 bw[2][NTL], av[2][MW1];
      auto ld1 = [&](int ks, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int n = 0; n < NTL; ++n)
          bw[buf][n] = *reinterpret_cast<const half8*>(sW1 + b_off + n * 16 * LW + ks * 32);
#pragma unroll
        for (int j = 0; j < MW1; ++j) {
          // a wave past the last m-tile recomputes it (result dropped in the epilogue):
          // no branch around the MFMA — branches there made the compiler shuttle
          // accumulators between AGPRs and overwrite a pending MFMA's srcC (gfx950)
          const int m = min(w + NW * j, MT1 - 1);
          av[buf][j] = *reinterpret_cast<const half8*>(sX + a1_off + (m * 16 + ks * G::TPK * D) * LI);
        }
      };
      ld1(0, 0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) ld1(ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);  // reads stay above the MFMAs (see logits)
#pragma unroll
        for (int j = 0; j < MW1; ++j)
#pragma unroll
          for (int n = 0; n < NTL; ++n) acc[j][n] = mfma16(av[ks & 1][j], bw[ks & 1][n], acc[j][n]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();  // every wave is done reading sX
#pragma unroll
      for (int j = 0; j < MW1; ++j) {
        const int m = w + NW * j;
        if (j >= MT1 / NW && m >= MT1) continue;
#pragma unroll
        for (int n = 0; n < NTL; ++n) {
          const int co = n * 16 + arow;
          float v[4];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int r = m * 16 + 4 * (lane >> 4) + rr;
            v[rr] = silu(acc[j][n][rr] + bias1[n]);
            if (edge) {  // c2 zero-pads its input outside [0, T)
              const int t = t0 - P2 + r;
              v[rr] = (t >= 0 && t < T) ? v[rr] : 0.0f;
            }
          }
          st_frag_f16_pairs(sS, LI, m * 16 + 4 * (lane >> 4), co, v, lane);
        }
      }
    }
    __syncthreads();

    // ---- c2 over BM rows (row r <-> time t0 + r): A = sS[r + tap]
    f32x4 acc2[MW2][NTL];
#pragma unroll
    for (int j = 0; j < MW2; ++j)
#pragma unroll
      for (int n = 0; n < NTL; ++n) acc2[j][n] = zero_f32x4();
    {
      half8 bw[2][NTL], av[2][MW2];  // double-buffered as in c1
      auto ld2 = [&](int ks, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int n = 0; n < NTL; ++n)
          bw[buf][n] = *reinterpret_cast<const half8*>(sW2 + b_off + n * 16 * LW + ks * 32);
#pragma unroll
        for (int j = 0; j < MW2; ++j) {
          const int m = min(w + NW * j, MT2 - 1);  // see c1
          av[buf][j] = *reinterpret_cast<const half8*>(sS + a2_off + (m * 16 + ks * G::TPK) * LI);
        }
      };
      ld2(0, 0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) ld2(ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < MW2; ++j)
#pragma unroll
          for (int n = 0; n < NTL; ++n) acc2[j][n] = mfma16(av[ks & 1][j], bw[ks & 1][n], acc2[j][n]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- epilogue in NP row passes: c2 + b2 -> fp32 LDS (over dead sS), then 16-byte
    // row chunks out = (accumulate ? out : 0) + scale * (conv + x)
#pragma unroll
    for (int p = 0; p < G::NP; ++p) {
      __syncthreads();  // sS reads (p = 0) / the previous pass's sE reads are done
#pragma unroll
      for (int j = p * (MW2 / G::NP); j < (p + 1) * (MW2 / G::NP); ++j) {
        const int m = w + NW * j;
        if (j >= MT2 / NW && m >= MT2) continue;
#pragma unroll
        for (int n = 0; n < NTL; ++n)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            sE[(m * 16 - p * G::RP + 4 * (lane >> 4) + rr) * ES + n * 16 + arow] = acc2[j][n][rr] + bias2[n];
      }
      __syncthreads();
#pragma unroll
      for (int i = p * (G::NE / G::NP); i < (p + 1) * (G::NE / G::NP); ++i) {
        const int idx = tid + i * NT;
        const int r = idx / CPR, cg = (idx % CPR) * 8;
        if (r >= BM || t0 + r >= T) continue;
        const int rl = r - p * G::RP;
        const float4 v0 = *reinterpret_cast<const float4*>(sE + rl * ES + cg);
        const float4 v1 = *reinterpret_cast<const float4*>(sE + rl * ES + cg + 4);
        const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        const half8 xv = G::RES_LDS ? *reinterpret_cast<const half8*>(sR + r * LI + cg)
                                    : *reinterpret_cast<const half8*>(&xres[i]);
        const half8 pv = *reinterpret_cast<const half8*>(&acc_in[i]);
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
  }
#undef NARROW_PREFETCH
}

template <int C, int K, int D, int BM, int NW>
static void narrow_cfg(const ResUnitArgs& a, hipStream_t s) {
  using G = NarrowGeo<C, K, D, BM, NW>;
  static_assert(G::LDS <= 160 * 1024, "LDS");
  auto kern = resunit_kernel<C, K, D, BM, NW>;
  static bool attr = false;
  if (!attr) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)G::LDS));
    attr = true;
  }
  const int tiles_per_utt = (a.T + BM - 1) / BM;
  const int n_tiles = tiles_per_utt * a.B;
  const int per_cu = std::max(1, std::min(4, (int)((160 * 1024) / G::LDS)));
  // persistent grid: 1024 x blocks-per-CU — on the vocoder's 128-CU partition that is
  // eight rounds of short tile stripes, which balances the uneven tile costs (edge tiles,
  // HBM contention with the decoder) better than fewer, longer stripes. Sweep (vocoder
  // side per step): 128 -> +3 ms, 256 -> 315.6, 512 -> 313.5, 1024 -> 312.2, 2048 -> 313,
  // one block per tile -> 327.7 ms. JANUS_NARROW_GRID_CUS overrides the 1024.
  static const int gcu = ab_env("JANUS_NARROW_GRID_CUS") ? std::atoi(ab_env("JANUS_NARROW_GRID_CUS")) : 1024;
  const int grid = std::min(n_tiles, std::max(1, gcu) * per_cu);
  kern<<<grid, G::NT, G::LDS, s>>>(a, tiles_per_utt, n_tiles);
  JANUS_LAUNCH_CHECK();
}

#ifndef JANUS_NARROW16_BM
#define JANUS_NARROW16_BM 240
#endif
#ifndef JANUS_NARROW32_BM
#define JANUS_NARROW32_BM 240
#endif
template <int C, int K, int NW>
static void narrow_dw(const ResUnitArgs& a, hipStream_t s) {
  constexpr int BM = C == 16 ? JANUS_NARROW16_BM : JANUS_NARROW32_BM;  // output rows per tile
  if (a.d == 1) narrow_cfg<C, K, 1, BM, NW>(a, s);
  else if (a.d == 3) narrow_cfg<C, K, 3, BM, NW>(a, s);
  else if (a.d == 5) narrow_cfg<C, K, 5, BM, NW>(a, s);
  else throw Error("resunit: dilation must be 1, 3 or 5");
}

// waves per block (JANUS_NARROW_WAVES: 4 or 8). C = 32 runs 8 waves: its blocks (76 KB of
// LDS, 2 per CU) gave each SIMD only 2 waves to hide the staging, SiLU and epilogue phases
// behind the other block's MFMAs (overlapped step: C = 32 units 39.7 -> 34.0 ms); C = 16
// (3 blocks per CU already) is level-to-slower at 8 (29.9 -> 30.4 ms).
template <int C, int K>
static void narrow_d(const ResUnitArgs& a, hipStream_t s) {
  static const int nw = ab_env("JANUS_NARROW_WAVES") ? std::atoi(ab_env("JANUS_NARROW_WAVES"))
                                                          : (C == 32 ? 8 : 4);
  if constexpr (C == 16 && JANUS_NARROW16_BM != 240) narrow_dw<C, K, 4>(a, s);  // BM A/B builds
  else if (nw == 8) narrow_dw<C, K, 8>(a, s);
  else narrow_dw<C, K, 4>(a, s);
}

template <int C>
static void narrow_k(const ResUnitArgs& a, hipStream_t s) {
  if (a.k == 3) narrow_d<C, 3>(a, s);
  else if (a.k == 7) narrow_d<C, 7>(a, s);
  else if (a.k == 11) narrow_d<C, 11>(a, s);
  else throw Error("resunit: k must be 3, 7 or 11 for C <= 32");
}

bool resunit_supported(int C, int k) {
  if (C >= 64) return resunit_wide_supported(C, k, 5);
  return (C == 16 || C == 32) && (k == 3 || k == 7 || k == 11);
}

void resunit_launch(const ResUnitArgs& a, hipStream_t s) {
  JANUS_CHECK(resunit_supported(a.C, a.k), "resunit: C must be 16, 32, 64, 128 or 256, k odd <= 11");
  JANUS_CHECK(a.x != a.out, "resunit: out must not alias x");
  if (a.B <= 0 || a.T <= 0) return;
  if (a.C >= 64) {
    resunit_wide_launch(a, s);
    return;
  }
  if (a.C == 16) narrow_k<16>(a, s);
  else narrow_k<32>(a, s);
}

}  // namespace janus

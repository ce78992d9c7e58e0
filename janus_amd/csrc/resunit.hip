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

template <int C, int BM>
struct ResUnitGeo {
  // halves per activation row: conflict-free fragment pitch for C = 32; C = 16 keeps the
  // 48-B pitch (its sS/sX store pattern measured 10% faster than the 32-B one)
  static constexpr int LI = C == 16 ? 24 : frag_pitch(C);
  static constexpr int CPR = C / 8;                         // 16-byte chunks per row
  static constexpr int R0MAX = BM + 10 + 50;                // k <= 11, d <= 5
  static constexpr int NPF = (R0MAX * CPR + 255) / 256;     // prefetch uint4 per thread
  static constexpr int MT1 = ((BM + 10 + 15) / 16 + 3) / 4; // c1 M-tiles per wave
  static constexpr int MT2 = BM / 64;                       // c2 M-tiles per wave
  static constexpr int ES = C + 4;                          // fp32 epilogue row stride
  static constexpr int NE = BM * CPR / 256;                 // epilogue uint4 per thread
};

// Persistent: each block loads both weight matrices into LDS once, then walks tiles
// (b, 16*BM-row blocks) with the next tile's input rows prefetched into registers
// while the current tile computes, so HBM latency overlaps the MFMA/LDS work.
template <int C, int BM>
__global__ __launch_bounds__(256) void resunit_kernel(ResUnitArgs a, int KP, int tiles_per_utt,
                                                      int n_tiles, int act_halves) {
  using G = ResUnitGeo<C, BM>;
  constexpr int LI = G::LI, CPR = G::CPR, NT = C / 16, MT1 = G::MT1, MT2 = G::MT2, ES = G::ES;
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  const int k = a.k, d = a.d, T = a.T;
  const int p1 = d * (k - 1) / 2, p2 = (k - 1) / 2;
  const int R1 = BM + 2 * p2, R0 = R1 + 2 * p1;
  const int LW = frag_pitch(KP);
  _Float16* sX = smem;                        // [R0][LI]   silu(x)
  _Float16* sS = sX + R0 * LI;                // [R1p][LI]  silu(c1(.) + b1)
  float* sE = reinterpret_cast<float*>(smem); // [BM][ES] epilogue tile (aliases sX/sS)
  _Float16* sR = smem + act_halves;           // [BM][LI]   raw x (the unit's residual)
  _Float16* sW1 = sR + BM * LI;               // [C][LW]
  _Float16* sW2 = sW1 + C * LW;               // [C][LW]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  for (int idx = tid; idx < C * (KP / 8); idx += 256) {
    const int co = idx / (KP / 8), cc = idx % (KP / 8);
    *reinterpret_cast<uint4*>(sW1 + co * LW + cc * 8) =
        *reinterpret_cast<const uint4*>(a.w1 + (int64_t)co * KP + cc * 8);
    *reinterpret_cast<uint4*>(sW2 + co * LW + cc * 8) =
        *reinterpret_cast<const uint4*>(a.w2 + (int64_t)co * KP + cc * 8);
  }

  uint4 pf[G::NPF];
  auto prefetch = [&](int tile) {
    const int b = tile / tiles_per_utt, t0 = (tile % tiles_per_utt) * BM;
    const _Float16* xb = a.x + (int64_t)b * T * C;
    const int xbase = t0 - p2 - p1;
#pragma unroll
    for (int i = 0; i < G::NPF; ++i) {
      const int idx = tid + i * 256;
      const int r = idx / CPR, cc = idx % CPR;
      const int t = xbase + r;
      pf[i] = (tile < n_tiles && r < R0 && t >= 0 && t < T)
                  ? *reinterpret_cast<const uint4*>(xb + (int64_t)t * C + cc * 8)
                  : make_uint4(0, 0, 0, 0);
    }
  };
  prefetch(blockIdx.x);

  for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int b = tile / tiles_per_utt, t0 = (tile % tiles_per_utt) * BM;
    __syncthreads();  // previous tile's epilogue reads of sE are done (and W staged)
#pragma unroll
    for (int i = 0; i < G::NPF; ++i) {
      const int idx = tid + i * 256;
      const int r = idx / CPR, cc = idx % CPR;
      if (r < R0) {
        half8 v = *reinterpret_cast<const half8*>(&pf[i]);
        const int rr = r - p2 - p1;
        if (rr >= 0 && rr < BM) *reinterpret_cast<half8*>(sR + rr * LI + cc * 8) = v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)silu((float)v[j]);
        *reinterpret_cast<half8*>(sX + r * LI + cc * 8) = v;
      }
    }
    __syncthreads();
    prefetch(tile + gridDim.x);  // in flight during this tile's compute
    _Float16* ob = a.out + (int64_t)b * T * C;
    uint4 acc_in[G::NE];         // accumulate target, also in flight during compute
    if (a.accumulate) {
#pragma unroll
      for (int i = 0; i < G::NE; ++i) {
        const int idx = tid + i * 256;
        const int r = idx / CPR, cg = (idx % CPR) * 8;
        acc_in[i] = t0 + r < T ? *reinterpret_cast<const uint4*>(ob + (int64_t)(t0 + r) * C + cg)
                               : make_uint4(0, 0, 0, 0);
      }
    }

    // ---- c1 over R1 rows (c1 row r <-> time t0 - p2 + r): A = sX[r + tap*d]
    {
      f32x4 acc[MT1][NT];
#pragma unroll
      for (int j = 0; j < MT1; ++j)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[j][n] = zero_f32x4();
      for (int ks = 0; ks < KP / 32; ++ks) {
        const int kk = ks * 32 + 8 * (lane >> 4);
        const int tap = kk / C, ci = kk % C;
        const bool ok = tap < k;
        half8 bw[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n)
          bw[n] = *reinterpret_cast<const half8*>(sW1 + (n * 16 + (lane & 15)) * LW + kk);
#pragma unroll
        for (int j = 0; j < MT1; ++j) {
          const int m = w + 4 * j;
          if (m * 16 >= R1) break;
          const int r = m * 16 + (lane & 15);
          half8 av = zero_half8();
          if (ok && r < R1) av = *reinterpret_cast<const half8*>(sX + (r + tap * d) * LI + ci);
#pragma unroll
          for (int n = 0; n < NT; ++n) acc[j][n] = mfma16(av, bw[n], acc[j][n]);
        }
      }
#pragma unroll
      for (int j = 0; j < MT1; ++j) {
        const int m = w + 4 * j;
        if (m * 16 >= R1) break;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int co = n * 16 + (lane & 15);
          const float bias = a.b1[co];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int r = m * 16 + 4 * (lane >> 4) + rr;
            const int t = t0 - p2 + r;
            const float v = (r < R1 && t >= 0 && t < T) ? silu(acc[j][n][rr] + bias) : 0.0f;
            sS[r * LI + co] = (_Float16)v;  // c2 zero-pads its input outside [0, T)
          }
        }
      }
    }
    __syncthreads();

    // ---- c2 over BM rows (row r <-> time t0 + r): A = sS[r + tap]
    f32x4 acc2[MT2][NT];
#pragma unroll
    for (int j = 0; j < MT2; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc2[j][n] = zero_f32x4();
    for (int ks = 0; ks < KP / 32; ++ks) {
      const int kk = ks * 32 + 8 * (lane >> 4);
      const int tap = kk / C, ci = kk % C;
      const bool ok = tap < k;
      half8 bw[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n)
        bw[n] = *reinterpret_cast<const half8*>(sW2 + (n * 16 + (lane & 15)) * LW + kk);
#pragma unroll
      for (int j = 0; j < MT2; ++j) {
        const int r = (w * MT2 + j) * 16 + (lane & 15);
        const half8 av = ok ? *reinterpret_cast<const half8*>(sS + (r + tap) * LI + ci) : zero_half8();
#pragma unroll
        for (int n = 0; n < NT; ++n) acc2[j][n] = mfma16(av, bw[n], acc2[j][n]);
      }
    }
    __syncthreads();  // sX/sS dead: sE takes their place
#pragma unroll
    for (int j = 0; j < MT2; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int co = n * 16 + (lane & 15);
        const float bias = a.b2[co];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = (w * MT2 + j) * 16 + 4 * (lane >> 4) + rr;
          sE[r * ES + co] = acc2[j][n][rr] + bias;
        }
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < G::NE; ++i) {
      const int idx = tid + i * 256;
      const int r = idx / CPR, cg = (idx % CPR) * 8;
      const int t = t0 + r;
      if (t >= T) continue;
      const int64_t o = (int64_t)t * C + cg;
      const half8 xv = *reinterpret_cast<const half8*>(sR + r * LI + cg);
      const float4 v0 = *reinterpret_cast<const float4*>(sE + r * ES + cg);
      const float4 v1 = *reinterpret_cast<const float4*>(sE + r * ES + cg + 4);
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      const half8 pv = *reinterpret_cast<const half8*>(&acc_in[i]);
      half8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float y = (v[j] + (float)xv[j]) * a.scale;
        if (a.accumulate) y += (float)pv[j];
        hv[j] = (_Float16)y;
      }
      *reinterpret_cast<half8*>(ob + o) = hv;
    }
  }
}

template <int C, int BM>
static void resunit_cfg(const ResUnitArgs& a, hipStream_t s) {
  using G = ResUnitGeo<C, BM>;
  const int KP = resunit_kp(C, a.k);
  const int p1 = a.d * (a.k - 1) / 2, p2 = (a.k - 1) / 2;
  const int R1 = BM + 2 * p2, R0 = R1 + 2 * p1, R1p = (R1 + 15) / 16 * 16;
  JANUS_CHECK(R0 <= G::R0MAX, "resunit: (k-1)*(d+1) exceeds the prefetch budget");
  const int act = std::max((R0 + R1p) * G::LI, BM * G::ES * 2);  // halves
  const int act_halves = (act + 7) / 8 * 8;
  const size_t lds = ((size_t)act_halves + (size_t)BM * G::LI + 2 * (size_t)C * frag_pitch(KP)) * 2;
  JANUS_CHECK(lds <= 160 * 1024, "resunit: LDS tile too large");
  auto kern = resunit_kernel<C, BM>;
  static bool attr = false;
  if (!attr) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
    attr = true;
  }
  const int tiles_per_utt = (a.T + BM - 1) / BM;
  const int n_tiles = tiles_per_utt * a.B;
  const int per_cu = std::max(1, std::min(4, (int)((160 * 1024) / lds)));
  const int grid = std::min(n_tiles, 256 * per_cu);
  kern<<<grid, 256, lds, s>>>(a, KP, tiles_per_utt, n_tiles, act_halves);
  JANUS_LAUNCH_CHECK();
}

bool resunit_supported(int C, int k) {
  if (C >= 64) return resunit_wide_supported(C, k, 5);
  return (C == 16 || C == 32) && k >= 1 && k <= 11 && (k & 1);
}

void resunit_launch(const ResUnitArgs& a, hipStream_t s) {
  JANUS_CHECK(resunit_supported(a.C, a.k), "resunit: C must be 16, 32, 64, 128 or 256, k odd <= 11");
  JANUS_CHECK(a.x != a.out, "resunit: out must not alias x");
  if (a.B <= 0 || a.T <= 0) return;
  if (a.C >= 64) {
    resunit_wide_launch(a, s);
    return;
  }
  // tile rows per block (JANUS_RU_BM overrides, for tuning sweeps)
  static const int bm = [] { const char* e = std::getenv("JANUS_RU_BM"); return e ? std::atoi(e) : 0; }();
  // measured (B=16, 30 s, accumulate): C16 BM 256 beats 512 by 1.8x (3 blocks/CU vs 2);
  // C32 k<=7 is best at BM 128, k 11 at BM 64 (1.84 vs 2.23 ms)
  if (a.C == 16) {
    if (bm == 512) resunit_cfg<16, 512>(a, s);
    else resunit_cfg<16, 256>(a, s);
  } else {
    if (bm == 256) resunit_cfg<32, 256>(a, s);
    else if (bm == 64 || (bm == 0 && a.k > 7)) resunit_cfg<32, 64>(a, s);
    else resunit_cfg<32, 128>(a, s);
  }
}

}  // namespace janus

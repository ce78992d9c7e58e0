// Large-M fp16 "NT" GEMM on MFMA for the Whisper encoder's projections (QKV, attention
// output, fc1, fc2 at M = B x 1500 rows; transcriber.py:53-57 -> the CTranslate2 encoder):
//   C[M,N] = epi( A[M,K] · W[N,K]^T + bias[N] ),  epi: fp16 | exact-erf GELU -> fp16 |
//   fp32 residual add (C = R + ..., in place) | fp32.
//
// Geometry: 256 x 256 x 64 block tile, 8 waves (2 along M x 4 along N, 128 x 64 outputs
// each = 8 x 4 tiles of v_mfma_f32_16x16x32_f16), one block per CU (128 KB of staging).
// Staging: global_load_lds (16 B per lane, LDS-DMA, no VGPR round trip) into two LDS
// buffers — the next k-tile's loads are issued before the current k-tile's MFMAs, one
// vmcnt(0) + barrier per 64-deep k-tile.
// LDS image: rows of 64 halves (128 B = 8 chunks of 16 B), chunk c of row r stored at
// c ^ ((r >> 1) & 7). The fragment reads (lane l: row l & 15, chunk 4s + (l >> 4)) then put
// the 16 lanes of every ds_read_b128 lane group ({0-3,12-15,20-27}, ...) on 16 distinct
// 16-B bank slots: conflict-free. The DMA writes lane-linear, so the swizzle is applied to
// the per-lane SOURCE address (the chunk a lane fetches), and the same XOR on the read.
// Tiles are dealt XCD-aware (consecutive tiles of one A row panel on one L2).
// Epilogue: the accumulators of each half of a wave's rows go through the (free) staging
// LDS, then 8 consecutive columns per lane: bias, GELU or residual in fp32, 16-B stores.
//
// Accumulation order: one fp32 accumulator per output, k-steps of 32 in order — the same
// MFMA sequence per output as gemm_nt_kernel (gemm.hip), so the two are bit-identical.
#include <cstring>

#include "common.h"
#include "mfma.h"
#include "kernels.h"

namespace janus {

namespace {
constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kThreads = 512;                   // 8 waves
constexpr int kWMT = 8, kWNT = 4;               // 16x16 tiles per wave (128 x 64)
constexpr int kStageHalves = (kBM + kBN) * kBK; // one buffer: A tile then B tile
constexpr int kEP = 68;                         // epilogue fp32 pitch (64 + 4)
constexpr int kEpWave = 64 * kEP;               // floats per wave in the epilogue image
constexpr int kSmemBytes = 8 * kEpWave * 4 > 2 * kStageHalves * 2 ? 8 * kEpWave * 4 : 2 * kStageHalves * 2;
constexpr bool kGemmBigPhased = false;          // the default schedule (A/B: JANUS_GEMM_BIG)
constexpr bool kGemmBigTwo = false;
constexpr int kEpiNone = 99;                    // A/B timing builds: no epilogue (wrong output)
}  // namespace

// DMA one 8-row x 128-B piece per wave-instruction: lane l -> row (l >> 3) of the piece,
// physical chunk l & 7, fetching logical chunk (l & 7) ^ ((row >> 1) & 7).
__device__ __forceinline__ void glds_rows8(const _Float16* __restrict__ src, int64_t ld, int row_g,
                                           int row_l, int max_row, int k0, _Float16* lds_piece, int lane) {
  const int r = row_l + (lane >> 3);
  const int c = (lane & 7) ^ ((r >> 1) & 7);
  const int gr = min(row_g + (lane >> 3), max_row);
  const _Float16* g = src + (int64_t)gr * ld + k0 + 8 * c;
  typedef __attribute__((address_space(3))) void lds_void;
  __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)lds_piece, 16, 0, 0);
}

// The epilogue of one wave's 128 x 64 outputs (rows rbase + [0, 128), columns cbase +
// [0, 64); acc[m][n] = 16x16 tile (m, n)): two passes of 64 rows through the wave's own LDS
// image sC (64 x kEP floats), then 8 consecutive columns per lane: bias, GELU or residual
// in fp32, 16-B stores.
template <int EPI>
__device__ __forceinline__ void epilogue_wave(const GemmArgs& p, f32x4 (&acc)[kWMT][kWNT], float* sC,
                                              int rbase, int cbase, int lane) {
  const int M = p.M, fr = lane & 15;
  const int er = lane >> 3, ec = (lane & 7) * 8;           // 8 rows x 8 lanes per pass step
  const int gcol = cbase + ec;
  float bias[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias[j] = p.bias ? p.bias[gcol + j] : 0.0f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < kWNT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sC[(m * 16 + (lane >> 4) * 4 + r) * kEP + n * 16 + fr] = acc[4 * h + m][n][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's stores land before its reads
    __builtin_amdgcn_wave_barrier();
    // RESID: the pass's residual rows are loaded before any of its stores (vmcnt retires in
    // issue order, so a residual load issued behind a store waits for that store)
    float4 res[8][2];
    if constexpr (EPI == EPI_RESID_F32) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = min(rbase + h * 64 + it * 8 + er, M - 1);
        res[it][0] = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + gcol);
        res[it][1] = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + gcol + 4);
      }
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int lr = it * 8 + er;
      const int row = rbase + h * 64 + lr;
      const float4 lo = *reinterpret_cast<const float4*>(sC + lr * kEP + ec);
      const float4 hi = *reinterpret_cast<const float4*>(sC + lr * kEP + ec + 4);
      float v[8] = {lo.x + bias[0], lo.y + bias[1], lo.z + bias[2], lo.w + bias[3],
                    hi.x + bias[4], hi.y + bias[5], hi.z + bias[6], hi.w + bias[7]};
      if (row < M) {
        if constexpr (EPI == EPI_F16 || EPI == EPI_GELU_F16) {
          half8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (_Float16)(EPI == EPI_GELU_F16 ? gelu_erf(v[j]) : v[j]);
          *reinterpret_cast<half8*>(static_cast<_Float16*>(p.C) + (int64_t)row * p.ldc + gcol) = o;
        } else {
          float* c = static_cast<float*>(p.C) + (int64_t)row * p.ldc + gcol;
          if constexpr (EPI == EPI_RESID_F32) {
            v[0] += res[it][0].x; v[1] += res[it][0].y; v[2] += res[it][0].z; v[3] += res[it][0].w;
            v[4] += res[it][1].x; v[5] += res[it][1].y; v[6] += res[it][1].z; v[7] += res[it][1].w;
          }
          *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();       // the next pass overwrites the image
  }
}

template <int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm_big_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[kSmemBytes];
  _Float16* smem = reinterpret_cast<_Float16*>(smem_raw);

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / kBN, nbm = (M + kBM - 1) / kBM;
  const int bid = xcd_remap(blockIdx.x, nbm * nbn);
  const int bm = bid / nbn, bn = bid % nbn;
  const int row0 = bm * kBM, col0 = bn * kBN;
  const int lane = threadIdx.x & 63, wid = wave_id();
  const int wm = wid >> 2, wn = wid & 3;

  // stage k-tile kt into buffer b: wave w DMAs rows [32w, 32w + 32) of the A tile and of
  // the B tile, four 8-row pieces each
  auto stage = [&](int kt, int b) {
    _Float16* sA = smem + b * kStageHalves;
    _Float16* sB = sA + kBM * kBK;
    const int k0 = kt * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = wid * 32 + i * 8;
      glds_rows8(p.A, p.lda, row0 + rl, rl, M - 1, k0, sA + rl * kBK, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = wid * 32 + i * 8;
      glds_rows8(p.W, p.ldw, col0 + rl, rl, N - 1, k0, sB + rl * kBK, lane);
    }
  };

  f32x4 acc[kWMT][kWNT];
#pragma unroll
  for (int m = 0; m < kWMT; ++m)
#pragma unroll
    for (int n = 0; n < kWNT; ++n) acc[m][n] = zero_f32x4();

  // per-lane fragment offsets (halves): row lane & 15 of each 16-row tile, swizzled chunk
  const int fr = lane & 15, sw = fr >> 1;
  const int a_off = (wm * 128 + fr) * kBK, b_off = kBM * kBK + (wn * 64 + fr) * kBK;

  const int nk = K / kBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const _Float16* buf = smem + cur * kStageHalves;
#pragma unroll
    for (int s = 0; s < kBK / 32; ++s) {
      const int ch = ((4 * s + (lane >> 4)) ^ sw) * 8;
      half8 a[kWMT], b[kWNT];
#pragma unroll
      for (int n = 0; n < kWNT; ++n) b[n] = *reinterpret_cast<const half8*>(buf + b_off + n * 16 * kBK + ch);
#pragma unroll
      for (int m = 0; m < kWMT; ++m) a[m] = *reinterpret_cast<const half8*>(buf + a_off + m * 16 * kBK + ch);
#pragma unroll
      for (int m = 0; m < kWMT; ++m)
#pragma unroll
        for (int n = 0; n < kWNT; ++n) acc[m][n] = mfma16(a[m], b[n], acc[m][n]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if constexpr (EPI == kEpiNone) {   // timing ablation: keep the accumulators alive only
    float t = 0.0f;
#pragma unroll
    for (int m = 0; m < kWMT; ++m)
#pragma unroll
      for (int n = 0; n < kWNT; ++n) t += acc[m][n][0] + acc[m][n][3];
    if (t == 1234.5f) static_cast<float*>(p.C)[threadIdx.x] = t;
    return;
  }
  // epilogue, two passes of 64 rows per wave through the wave's own LDS image
  epilogue_wave<EPI>(p, acc, reinterpret_cast<float*>(smem_raw) + wid * kEpWave, row0 + wm * 128,
                     col0 + wn * 64, lane);
}

// ---------------------------------------------------------------------------------------
// Phased schedule (r06, A/B builds only: bit-identical, level with gemm_big_kernel — the
// staging is not what bounds it, DESIGN.md §7 r06 encoder GEMM): the same 256 x 256 x 64 tiles, MFMA sequence per output and
// epilogue, but the 128 KB of LDS is eight 16-KB HALF-TILE slots (A rows 0-127 / 128-255,
// W rows 0-127 / 128-255 of one k-tile; k-tile t in slots 4 (t & 1) + h) and each k-tile is
// three phases, so a slot is restaged for k-tile t + 2 as soon as its last fragment read
// of k-tile t has retired — not after the whole k-tile. Wave (wr, wc) owns rows
// mh·128 + wr·64 + [0, 64) and columns nh·128 + wc·32 + [0, 32) (mh, nh in {0, 1}), so
// output quadrant (mh, nh) of every wave reads A half mh and W half nh only:
//   phase 0: read A0, W0 -> quadrant (0, 0);  issue A1(t + 1)
//   phase 1: read W1      -> quadrant (0, 1);  issue A0(t + 2), W0(t + 2)
//   phase 2: read A1      -> quadrants (1, 1), (1, 0) (W0 still in registers);  issue W1(t + 2)
// Every half-tile is DMA'd 4-7 phases ahead of its first read (≈ 80-112 KB in flight per
// CU instead of one 64 KB k-tile drained to zero at every k-tile), retired by a counted
// vmcnt before the raw s_barrier that ends the phase ahead of its first read. A slot's
// restage is issued after the barrier that follows its last read (every fragment read of a
// phase is consumed by that phase's MFMAs, so the reads have retired at the barrier).
// The per-output k order is unchanged: bit-identical to gemm_big_kernel / gemm_nt_kernel.
namespace {
constexpr int kHalf = 128 * kBK;   // halves per slot
}

template <int N_>
__device__ __forceinline__ void vm_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N_) : "memory");   // + this wave's reads
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int EPI, bool PRIO>
__global__ __launch_bounds__(kThreads, 1) void gemm_big_phased_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[kSmemBytes];
  _Float16* smem = reinterpret_cast<_Float16*>(smem_raw);

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / kBN, nbm = (M + kBM - 1) / kBM;
  const int bid = xcd_remap(blockIdx.x, nbm * nbn);
  const int bm = bid / nbn, bn = bid % nbn;
  const int row0 = bm * kBM, col0 = bn * kBN;
  const int lane = threadIdx.x & 63, wid = wave_id();
  const int wr = wid >> 2, wc = wid & 3;

  // DMA half h of k-tile t into its slot: wave w takes rows [16w, 16w + 16) of the half
  auto stage = [&](int t, int h) {
    _Float16* dst = smem + ((t & 1) * 4 + h) * kHalf;
    const bool a = h < 2;
    const int base = (a ? row0 : col0) + (h & 1) * 128, lim = (a ? M : N) - 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rl = wid * 16 + i * 8;
      glds_rows8(a ? p.A : p.W, a ? p.lda : p.ldw, base + rl, rl, lim, t * kBK, dst + rl * kBK, lane);
    }
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[i][j][m][n] = zero_f32x4();

  const int fr = lane & 15, sw = fr >> 1;
  const int a_off = (wr * 64 + fr) * kBK, b_off = (wc * 32 + fr) * kBK;
  half8 fa[4][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](const _Float16* slot) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = ((4 * s + (lane >> 4)) ^ sw) * 8;
#pragma unroll
      for (int m = 0; m < 4; ++m) fa[m][s] = *reinterpret_cast<const half8*>(slot + a_off + m * 16 * kBK + ch);
    }
  };
  auto read_b = [&](const _Float16* slot, half8 (&fb)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = ((4 * s + (lane >> 4)) ^ sw) * 8;
#pragma unroll
      for (int n = 0; n < 2; ++n) fb[n][s] = *reinterpret_cast<const half8*>(slot + b_off + n * 16 * kBK + ch);
    }
  };
  auto quad = [&](f32x4 (&c)[4][2], half8 (&fb)[2][2]) {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) c[m][n] = mfma16(fa[m][s], fb[n][s], c[m][n]);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  const int nk = K / kBK;
  // prologue: k-tile 0 whole, then A0 W0 W1 of k-tile 1 (its A1 goes out in k-tile 0's
  // phase 0); wait for A0(0), W0(0)
  stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
  if (nk > 1) {
    stage(1, 0); stage(1, 2); stage(1, 3);
    vm_wait_barrier<10>();
  } else {
    vm_wait_barrier<4>();
  }
  for (int t = 0; t < nk; ++t) {
    const _Float16* sl = smem + (t & 1) * 4 * kHalf;
    const bool more1 = t + 1 < nk, more2 = t + 2 < nk;
    // phase 0
    if (more1) stage(t + 1, 1);
    read_a(sl);
    read_b(sl + 2 * kHalf, fb0);
    quad(acc[0][0], fb0);
    if (more1) vm_wait_barrier<10>(); else vm_wait_barrier<2>();   // W1(t)
    // phase 1
    if (more2) { stage(t + 2, 0); stage(t + 2, 2); }
    read_b(sl + 3 * kHalf, fb1);
    quad(acc[0][1], fb1);
    if (more2) vm_wait_barrier<12>(); else if (more1) vm_wait_barrier<8>(); else vm_wait_barrier<0>();  // A1(t)
    // phase 2
    if (more2) stage(t + 2, 3);
    read_a(sl + kHalf);
    quad(acc[1][1], fb1);
    quad(acc[1][0], fb0);
    if (more2) vm_wait_barrier<10>(); else if (more1) vm_wait_barrier<4>(); else vm_wait_barrier<0>();  // A0, W0(t + 1)
  }

  if constexpr (EPI == kEpiNone) {
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) t += acc[i][j][m][n][0] + acc[i][j][m][n][3];
    if (t == 1234.5f) static_cast<float*>(p.C)[threadIdx.x] = t;
    return;
  }
  // epilogue (the staging image is free: every DMA retired, every read consumed), two
  // passes (mh) of 64 rows per wave; image column v < 32 is the wave's nh = 0 group,
  // v >= 32 its nh = 1 group
  float* sC = reinterpret_cast<float*>(smem_raw) + wid * kEpWave;
  const int er = lane >> 3, ec = (lane & 7) * 8;
  const int gcol = col0 + (ec >> 5) * 128 + wc * 32 + (ec & 31);
  float bias[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias[j] = p.bias ? p.bias[gcol + j] : 0.0f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sC[(m * 16 + (lane >> 4) * 4 + r) * kEP + nh * 32 + n * 16 + fr] = acc[h][nh][m][n][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    float4 res[8][2];
    if constexpr (EPI == EPI_RESID_F32) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = min(row0 + h * 128 + wr * 64 + it * 8 + er, M - 1);
        res[it][0] = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + gcol);
        res[it][1] = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + gcol + 4);
      }
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int lr = it * 8 + er;
      const int row = row0 + h * 128 + wr * 64 + lr;
      const float4 lo = *reinterpret_cast<const float4*>(sC + lr * kEP + ec);
      const float4 hi = *reinterpret_cast<const float4*>(sC + lr * kEP + ec + 4);
      float v[8] = {lo.x + bias[0], lo.y + bias[1], lo.z + bias[2], lo.w + bias[3],
                    hi.x + bias[4], hi.y + bias[5], hi.z + bias[6], hi.w + bias[7]};
      if (row < M) {
        if constexpr (EPI == EPI_F16 || EPI == EPI_GELU_F16) {
          half8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (_Float16)(EPI == EPI_GELU_F16 ? gelu_erf(v[j]) : v[j]);
          *reinterpret_cast<half8*>(static_cast<_Float16*>(p.C) + (int64_t)row * p.ldc + gcol) = o;
        } else {
          float* c = static_cast<float*>(p.C) + (int64_t)row * p.ldc + gcol;
          if constexpr (EPI == EPI_RESID_F32) {
            v[0] += res[it][0].x; v[1] += res[it][0].y; v[2] += res[it][0].z; v[3] += res[it][0].w;
            v[4] += res[it][1].x; v[5] += res[it][1].y; v[6] += res[it][1].z; v[7] += res[it][1].w;
          }
          *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------------------
// Two blocks per CU (r06, A/B builds only: bit-identical, measured slower — DESIGN.md §7
// r06 encoder GEMM): 256 x 128 tiles, 4 waves (2 x 2, the same 128 x 64
// outputs and 8 x 4 16x16x32 MFMA tiles per wave as gemm_big_kernel), k-tiles of 32 in a
// 3-slot LDS ring (24 KB each: A 256 x 32 then W 128 x 32 halves, two k-tiles in flight,
// counted vmcnt + raw s_barrier), 72 KB per block. With one block per CU the whole CU
// waits for a block's epilogue (the LDS transposition, bias / GELU / residual, the stores:
// 30-60 % of gemm_big_kernel's time, `profiles/r06_gemm_ab.txt`); the idea was that the
// other block's MFMAs fill it. They did not: the epilogue's output bytes cost the same.
// LDS rows are 64 B (4 chunks of 16 B); chunk c of row r sits at c ^ g[(r >> 2) & 3],
// g = {0, 2, 3, 1}: the ds_read_b128 lane groups of the fragment reads (rows fr = lane & 15,
// chunk lane >> 4) then cover 16 distinct 16-B bank slots. The DMA writes lane-linear, so
// the XOR goes on the per-lane source address. Per output the k-steps run in order: the
// MFMA sequence of gemm_big_kernel / gemm_nt_kernel, bit-identical.
namespace {
constexpr int k2BM = 256, k2BN = 128, k2BK = 32, k2Threads = 256, k2Slots = 3;
constexpr int k2SlotHalves = (k2BM + k2BN) * k2BK;           // 24 KB
constexpr int k2Smem = k2Slots * k2SlotHalves * 2 > 4 * kEpWave * 4 ? k2Slots * k2SlotHalves * 2
                                                                     : 4 * kEpWave * 4;
}  // namespace

__device__ __forceinline__ int sw64(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }

// DMA one 16-row x 64-B piece per wave-instruction: lane l -> row (l >> 2) of the piece,
// physical chunk l & 3 holding logical chunk (l & 3) ^ g[(row >> 2) & 3]
__device__ __forceinline__ void glds_rows16(const _Float16* __restrict__ src, int64_t ld, int row_g,
                                            int row_l, int max_row, int k0, _Float16* lds_piece, int lane) {
  const int r = row_l + (lane >> 2);
  const int c = (lane & 3) ^ sw64(r);
  const int gr = min(row_g + (lane >> 2), max_row);
  const _Float16* g = src + (int64_t)gr * ld + k0 + 8 * c;
  typedef __attribute__((address_space(3))) void lds_void;
  __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)lds_piece, 16, 0, 0);
}

template <int EPI>
__global__ __launch_bounds__(k2Threads, 2) void gemm_big2_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[k2Smem];
  _Float16* smem = reinterpret_cast<_Float16*>(smem_raw);

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / k2BN, nbm = (M + k2BM - 1) / k2BM;
  const int bid = xcd_remap(blockIdx.x, nbm * nbn);
  const int bm = bid / nbn, bn = bid % nbn;
  const int row0 = bm * k2BM, col0 = bn * k2BN;
  const int lane = threadIdx.x & 63, wid = wave_id();
  const int wm = wid >> 1, wn = wid & 1;

  // stage k-tile kt into slot kt % 3: wave w DMAs A rows [64w, 64w + 64) and W rows
  // [32w, 32w + 32), 16-row pieces (6 DMA instructions per lane)
  auto stage = [&](int kt, int slot) {
    _Float16* sA = smem + slot * k2SlotHalves;
    _Float16* sB = sA + k2BM * k2BK;
    const int k0 = kt * k2BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = wid * 64 + i * 16;
      glds_rows16(p.A, p.lda, row0 + rl, rl, M - 1, k0, sA + rl * k2BK, lane);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rl = wid * 32 + i * 16;
      glds_rows16(p.W, p.ldw, col0 + rl, rl, N - 1, k0, sB + rl * k2BK, lane);
    }
  };

  f32x4 acc[kWMT][kWNT];
#pragma unroll
  for (int m = 0; m < kWMT; ++m)
#pragma unroll
    for (int n = 0; n < kWNT; ++n) acc[m][n] = zero_f32x4();

  const int fr = lane & 15;
  const int ch = ((lane >> 4) ^ sw64(fr)) * 8;
  const int a_off = (wm * 128 + fr) * k2BK + ch, b_off = k2BM * k2BK + (wn * 64 + fr) * k2BK + ch;

  const int nk = K / k2BK;
  stage(0, 0);
  if (nk > 1) stage(1, 1);
  int slot = 0, slot2 = 2;   // slot of k-tile kt, of kt + 2
  for (int kt = 0; kt < nk; ++kt) {
    // k-tile kt landed for every wave, and every wave is done reading k-tile kt - 1 (the
    // slot k-tile kt + 2 goes to)
    if (kt + 1 < nk) vm_wait_barrier<6>(); else vm_wait_barrier<0>();
    if (kt + 2 < nk) stage(kt + 2, slot2);
    const _Float16* buf = smem + slot * k2SlotHalves;
    half8 a[kWMT], b[kWNT];
#pragma unroll
    for (int n = 0; n < kWNT; ++n) b[n] = *reinterpret_cast<const half8*>(buf + b_off + n * 16 * k2BK);
#pragma unroll
    for (int m = 0; m < kWMT; ++m) a[m] = *reinterpret_cast<const half8*>(buf + a_off + m * 16 * k2BK);
#pragma unroll
    for (int m = 0; m < kWMT; ++m)
#pragma unroll
      for (int n = 0; n < kWNT; ++n) acc[m][n] = mfma16(a[m], b[n], acc[m][n]);
    slot = slot == 2 ? 0 : slot + 1;
    slot2 = slot2 == 2 ? 0 : slot2 + 1;
  }
  if constexpr (EPI == kEpiNone) {
    float t = 0.0f;
#pragma unroll
    for (int m = 0; m < kWMT; ++m)
#pragma unroll
      for (int n = 0; n < kWNT; ++n) t += acc[m][n][0] + acc[m][n][3];
    if (t == 1234.5f) static_cast<float*>(p.C)[threadIdx.x] = t;
    return;
  }
  vm_wait_barrier<0>();   // every wave's last fragment reads retired: the ring is free
  epilogue_wave<EPI>(p, acc, reinterpret_cast<float*>(smem_raw) + wid * kEpWave, row0 + wm * 128,
                     col0 + wn * 64, lane);
}

bool gemm_big_supported(int epi, const GemmArgs& p) {
  if (!(epi == EPI_F16 || epi == EPI_GELU_F16 || epi == EPI_RESID_F32 || epi == EPI_F32)) return false;
  if (p.M < kBM || p.N % kBN != 0 || p.K % kBK != 0 || p.K < kBK) return false;
  if (p.lda % 8 || p.ldw % 8 || p.ldc % 8) return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.W & 15) || ((uintptr_t)p.C & 15)) return false;
  if (epi == EPI_RESID_F32 && (!p.R || p.ldr % 4 || ((uintptr_t)p.R & 15))) return false;
  if (p.kc || p.ln_part || p.a_group_cols || p.ln_out || p.lnin_x) return false;
  return (int64_t)cdiv(p.M, kBM) * (p.N / kBN) < (1ll << 31);
}

void gemm_big_launch(int epi, const GemmArgs& p, hipStream_t s) {
  JANUS_CHECK(gemm_big_supported(epi, p), "gemm_big: unsupported shape / layout");
  const unsigned blocks = (unsigned)(cdiv(p.M, kBM) * (p.N / kBN));
  const char* v = ab_env("JANUS_GEMM_BIG");   // A/B builds: dbuf | phased | phased_prio | two [_noepi]
  const bool two = v ? std::strncmp(v, "two", 3) == 0 : kGemmBigTwo;
  if (two) {
    const unsigned blocks2 = (unsigned)(cdiv(p.M, k2BM) * (p.N / k2BN));
    if (v && std::strstr(v, "_noepi")) {
      gemm_big2_kernel<kEpiNone><<<blocks2, k2Threads, 0, s>>>(p);
    } else {
      switch (epi) {
        case EPI_F16: gemm_big2_kernel<EPI_F16><<<blocks2, k2Threads, 0, s>>>(p); break;
        case EPI_GELU_F16: gemm_big2_kernel<EPI_GELU_F16><<<blocks2, k2Threads, 0, s>>>(p); break;
        case EPI_RESID_F32: gemm_big2_kernel<EPI_RESID_F32><<<blocks2, k2Threads, 0, s>>>(p); break;
        default: gemm_big2_kernel<EPI_F32><<<blocks2, k2Threads, 0, s>>>(p); break;
      }
    }
    JANUS_LAUNCH_CHECK();
    return;
  }
  const bool phased = v ? std::strncmp(v, "phased", 6) == 0 : kGemmBigPhased;
  if (v && std::strstr(v, "_noepi")) {
    if (!phased) gemm_big_kernel<kEpiNone><<<blocks, kThreads, 0, s>>>(p);
    else gemm_big_phased_kernel<kEpiNone, false><<<blocks, kThreads, 0, s>>>(p);
    JANUS_LAUNCH_CHECK();
    return;
  }
  if (phased) {
    const bool prio = v && std::strcmp(v, "phased_prio") == 0;
    switch (epi) {
      case EPI_F16:
        if (prio) gemm_big_phased_kernel<EPI_F16, true><<<blocks, kThreads, 0, s>>>(p);
        else gemm_big_phased_kernel<EPI_F16, false><<<blocks, kThreads, 0, s>>>(p);
        break;
      case EPI_GELU_F16:
        if (prio) gemm_big_phased_kernel<EPI_GELU_F16, true><<<blocks, kThreads, 0, s>>>(p);
        else gemm_big_phased_kernel<EPI_GELU_F16, false><<<blocks, kThreads, 0, s>>>(p);
        break;
      case EPI_RESID_F32:
        if (prio) gemm_big_phased_kernel<EPI_RESID_F32, true><<<blocks, kThreads, 0, s>>>(p);
        else gemm_big_phased_kernel<EPI_RESID_F32, false><<<blocks, kThreads, 0, s>>>(p);
        break;
      default:
        if (prio) gemm_big_phased_kernel<EPI_F32, true><<<blocks, kThreads, 0, s>>>(p);
        else gemm_big_phased_kernel<EPI_F32, false><<<blocks, kThreads, 0, s>>>(p);
        break;
    }
    JANUS_LAUNCH_CHECK();
    return;
  }
  switch (epi) {
    case EPI_F16: gemm_big_kernel<EPI_F16><<<blocks, kThreads, 0, s>>>(p); break;
    case EPI_GELU_F16: gemm_big_kernel<EPI_GELU_F16><<<blocks, kThreads, 0, s>>>(p); break;
    case EPI_RESID_F32: gemm_big_kernel<EPI_RESID_F32><<<blocks, kThreads, 0, s>>>(p); break;
    default: gemm_big_kernel<EPI_F32><<<blocks, kThreads, 0, s>>>(p); break;
  }
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

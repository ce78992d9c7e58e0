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
#include <algorithm>
#include <cstdlib>
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

  // epilogue, two passes of 64 rows per wave through the wave's own LDS image
  float* sC = reinterpret_cast<float*>(smem_raw) + wid * kEpWave;
  const int er = lane >> 3, ec = (lane & 7) * 8;           // 8 rows x 8 lanes per pass step
  const int gcol = col0 + wn * 64 + ec;
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
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int lr = it * 8 + er;
      const int row = row0 + wm * 128 + h * 64 + lr;
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
            const float4 r0 = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + gcol);
            const float4 r1 = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + gcol + 4);
            v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
            v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
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

// ---------------------------------------------------------------- persistent form
// One block per CU walks tiles t = blockIdx.x, + gridDim.x, ... (XCD-aware order as above).
// The product is computed transposed, D = W_frag · A_frag^T (the W fragment as the MFMA's
// A operand): a lane then holds 4 consecutive OUTPUT COLUMNS of one output row, so the
// epilogue stores straight from the accumulators (no LDS image) and the staging buffers
// stay free for the next tile: its first k-tile is DMA'd during this tile's last k-step
// and lands while this tile's epilogue runs. The B tile's LDS rows are gathered so that
// the two n-tiles j = 2p, 2p + 1 of a wave put 8 consecutive columns on each lane (one
// 16-B fp16 store, or two 16-B fp32 stores): LDS row 64 wn + 16 j + i holds W row
// col0 + 64 wn + 32 (j >> 1) + 8 (i >> 2) + 4 (j & 1) + (i & 3).
__device__ __forceinline__ int bcol_perm(int R) {
  const int j = (R >> 4) & 3, i = R & 15;
  return (R & ~63) + 32 * (j >> 1) + 8 * (i >> 2) + 4 * (j & 1) + (i & 3);
}

template <int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm_big_persist_kernel(GemmArgs p) {
  // staging buffers, then the tile's bias [256] f32 (one array: a second __shared__ object
  // can make hipcc drain the LDS-DMA before every ds_read)
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * kStageHalves + 2 * kBN];
  float* sBias = reinterpret_cast<float*>(smem + 2 * kStageHalves);
  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / kBN, nbm = (M + kBM - 1) / kBM, ntiles = nbm * nbn;
  const int tid = threadIdx.x;
  const int lane = threadIdx.x & 63, wid = wave_id();
  const int wm = wid >> 2, wn = wid & 3;
  const int nk = K / kBK;
  typedef __attribute__((address_space(3))) void lds_void;

  auto tile_origin = [&](int t, int& row0, int& col0) {
    const int bid = xcd_remap(t, ntiles);
    row0 = (bid / nbn) * kBM;
    col0 = (bid % nbn) * kBN;
  };
  // stage k-tile kt of the tile at (row0, col0) into buffer b (8 LDS-DMA per wave)
  auto stage = [&](int row0, int col0, int kt, int b) {
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
      const int r = rl + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const _Float16* g = p.W + (int64_t)(col0 + bcol_perm(r)) * p.ldw + k0 + 8 * c;
      __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(sB + rl * kBK), 16, 0, 0);
    }
  };

  const int fr = lane & 15, sw = fr >> 1, g4 = lane >> 4;
  const int a_off = (wm * 128 + fr) * kBK, b_off = kBM * kBK + (wn * 64 + fr) * kBK;

  int t = blockIdx.x;
  if (t >= ntiles) return;
  int row0, col0;
  tile_origin(t, row0, col0);
  stage(row0, col0, 0, 0);
  // a tile's bias goes to LDS: loaded together with its first k-tile, stored after the
  // barrier that retires it (a plain load waited for later would wait for every DMA
  // issued after it: vmcnt retires in issue order)
  float nb = (tid < kBN && p.bias) ? p.bias[col0 + tid] : 0.0f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < kBN) sBias[tid] = nb;
  int it = 0;  // k-tiles consumed by this block (buffer parity)
  for (; t < ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    int nrow0 = 0, ncol0 = 0;
    if (tn < ntiles) tile_origin(tn, nrow0, ncol0);
    f32x4 acc[kWMT][kWNT];
#pragma unroll
    for (int m = 0; m < kWMT; ++m)
#pragma unroll
      for (int n = 0; n < kWNT; ++n) acc[m][n] = zero_f32x4();
    for (int kt = 0; kt < nk; ++kt, ++it) {
      const int cur = it & 1;
      if (kt + 1 < nk) {
        stage(row0, col0, kt + 1, cur ^ 1);
      } else if (tn < ntiles) {
        stage(nrow0, ncol0, 0, cur ^ 1);
        nb = (tid < kBN && p.bias) ? p.bias[ncol0 + tid] : 0.0f;
      }
      asm volatile("" ::: "memory");
      const _Float16* buf = smem + cur * kStageHalves;
#pragma unroll
      for (int s = 0; s < kBK / 32; ++s) {
        const int ch = ((4 * s + g4) ^ sw) * 8;
        half8 a[kWMT], b[kWNT];
#pragma unroll
        for (int n = 0; n < kWNT; ++n) b[n] = *reinterpret_cast<const half8*>(buf + b_off + n * 16 * kBK + ch);
#pragma unroll
        for (int m = 0; m < kWMT; ++m) a[m] = *reinterpret_cast<const half8*>(buf + a_off + m * 16 * kBK + ch);
#pragma unroll
        for (int m = 0; m < kWMT; ++m)
#pragma unroll
          for (int n = 0; n < kWNT; ++n) acc[m][n] = mfma16(b[n], a[m], acc[m][n]);
      }
      if (kt + 1 < nk || nk == 1) {   // (nk == 1: the barrier that publishes sBias)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
    // epilogue straight from the accumulators: lane -> row fr of each m-tile, columns
    // 32 p + 8 g4 + [0, 8) of the wave's 64
    const int cbase = col0 + wn * 64 + 8 * g4;
    float bias[2][8];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const float4 b0 = *reinterpret_cast<const float4*>(sBias + wn * 64 + 8 * g4 + 32 * pp);
      const float4 b1 = *reinterpret_cast<const float4*>(sBias + wn * 64 + 8 * g4 + 32 * pp + 4);
      bias[pp][0] = b0.x; bias[pp][1] = b0.y; bias[pp][2] = b0.z; bias[pp][3] = b0.w;
      bias[pp][4] = b1.x; bias[pp][5] = b1.y; bias[pp][6] = b1.z; bias[pp][7] = b1.w;
    }
#pragma unroll
    for (int m = 0; m < kWMT; ++m) {
      const int row = row0 + wm * 128 + m * 16 + fr;
      if (row >= M) continue;
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int col = cbase + 32 * pp;
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = acc[m][2 * pp][q] + bias[pp][q];
          v[4 + q] = acc[m][2 * pp + 1][q] + bias[pp][4 + q];
        }
        if constexpr (EPI == EPI_F16 || EPI == EPI_GELU_F16) {
          half8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (_Float16)(EPI == EPI_GELU_F16 ? gelu_erf(v[q]) : v[q]);
          *reinterpret_cast<half8*>(static_cast<_Float16*>(p.C) + (int64_t)row * p.ldc + col) = o;
        } else {
          float* c = static_cast<float*>(p.C) + (int64_t)row * p.ldc + col;
          if constexpr (EPI == EPI_RESID_F32) {
            const float4 r0 = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + col);
            const float4 r1 = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + col + 4);
            v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
            v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
          }
          *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
    // the next tile's first k-tile (DMA'd during the last k-step) has landed everywhere,
    // and every wave is done with this tile's bias
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < kBN) sBias[tid] = nb;
    row0 = nrow0;
    col0 = ncol0;
  }
}

// ---------------------------------------------------------------- ring form (v3)
// The persistent transposed-output kernel above keeps one 64-deep k-tile (64 KB per CU) in
// flight: PMC on the QKV shape showed the waves waiting ~40 % of the time with the MFMA
// pipes 32 % busy — one k-tile of DMA does not cover the L2 latency at the rate the MFMAs
// consume it. Here the staging is a ring of four 32-deep slots (32 KB each): three slots
// are in flight while one is consumed, the wait at each step's end is a counted
// vmcnt(2 x 4) (the two younger slots stay in flight) and the barrier is a raw s_barrier
// (__syncthreads would drain the LDS-DMA). The ring runs across tiles: the first slots of
// the next tile are issued during the last steps of the current one and land while its
// epilogue stores. LDS image rows are 64 B (4 chunks); chunk c of row r is stored at
// c ^ g[(r >> 2) & 3], g = {0, 3, 2, 1}: the 16 lanes of each ds_read_b128 group then hit
// 16 distinct 16-B slots.
constexpr int kRBK = 32, kRSlots = 4;
constexpr int kRSlotHalves = (kBM + kBN) * kRBK;   // 16 K halves = 32 KB

__device__ __forceinline__ int ring_swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

// ds_read_b128 of 4 floats the compiler does not see as an LDS read: hipcc waits
// vmcnt(0) before any LDS read that may alias a pending LDS-DMA, which here would drain
// the next tile's slots in flight. Safe because the bias DMA it reads was retired by an
// earlier counted vmcnt + barrier.
__device__ __forceinline__ float4 lds_read4_asm(const float* p) {
  typedef __attribute__((address_space(3))) const float lds_float;
  const uint32_t a = (uint32_t)(uintptr_t)(lds_float*)p;
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return make_float4(v[0], v[1], v[2], v[3]);
}

template <int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm_big_ring_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) _Float16 smem[kRSlots * kRSlotHalves + 2 * 2 * kBN];
  float* sBias = reinterpret_cast<float*>(smem + kRSlots * kRSlotHalves);   // [2][256]
  const int M = p.M, N = p.N, K = p.K;
  const int nbn = N / kBN, nbm = (M + kBM - 1) / kBM, ntiles = nbm * nbn;
  const int tid = threadIdx.x, lane = tid & 63, wid = wave_id();
  const int wm = wid >> 2, wn = wid & 3;
  const int nks = K / kRBK;                                   // steps per tile (>= 3)
  typedef __attribute__((address_space(3))) void lds_void;
  const int G = gridDim.x;
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / G + 1 : 0;
  const int total_steps = my_tiles * nks;

  auto tile_origin = [&](int local, int& row0, int& col0) {
    const int bid = xcd_remap(blockIdx.x + local * G, ntiles);
    row0 = (bid / nbn) * kBM;
    col0 = (bid % nbn) * kBN;
  };
  // producer: DMA global step q (tile q / nks, k-step q % nks) into slot q % 4; wave w
  // moves rows [32w, 32w + 32) of the A slot and of the B slot, 16 rows of 64 B per
  // instruction: lane l -> row l >> 2, physical chunk l & 3
  auto produce = [&](int q) {
    int r0, c0;
    tile_origin(q / nks, r0, c0);
    const int k0 = (q % nks) * kRBK;
    _Float16* sA = smem + (q % kRSlots) * kRSlotHalves;
    _Float16* sB = sA + kBM * kRBK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rl = wid * 32 + i * 16;
      const int r = rl + (lane >> 2);
      const int c = (lane & 3) ^ ring_swz(r);
      const _Float16* ga = p.A + (int64_t)min(r0 + r, M - 1) * p.lda + k0 + 8 * c;
      __builtin_amdgcn_global_load_lds((const void*)ga, (lds_void*)(sA + rl * kRBK), 16, 0, 0);
      const _Float16* gb = p.W + (int64_t)(c0 + bcol_perm(r)) * p.ldw + k0 + 8 * c;
      __builtin_amdgcn_global_load_lds((const void*)gb, (lds_void*)(sB + rl * kRBK), 16, 0, 0);
    }
    // a tile's bias rides with its first slot: LDS-DMA of 4 B per lane by waves 0-3 into
    // sBias[tile & 1] (a plain load into a register would be waited for with vmcnt(0))
    if (q % nks == 0 && p.bias != nullptr && wid < kBN / 64) {
      __builtin_amdgcn_global_load_lds((const void*)(p.bias + c0 + wid * 64 + lane),
                                       (lds_void*)(sBias + ((q / nks) & 1) * kBN + wid * 64), 4, 0, 0);
    }
  };

  if (my_tiles == 0) return;
  if (p.bias == nullptr) {
    for (int i = tid; i < 2 * kBN; i += kThreads) sBias[i] = 0.0f;
  }
  const int fr = lane & 15, g4 = lane >> 4;
  const int pch = (g4 ^ ring_swz(fr)) * 8;                     // this lane's chunk (halves)
  const int a_off = (wm * 128 + fr) * kRBK + pch;
  const int b_off = kBM * kRBK + (wn * 64 + fr) * kRBK + pch;

  // prologue: three slots in flight, the first landed
  produce(0);
  if (total_steps > 1) produce(1);
  if (total_steps > 2) produce(2);
  if (total_steps > 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (total_steps > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  f32x4 acc[kWMT][kWNT];
  int row0 = 0, col0 = 0;
  for (int c = 0; c < total_steps; ++c) {
    const int kstep = c % nks, tl = c / nks;
    if (kstep == 0) {
      tile_origin(tl, row0, col0);
#pragma unroll
      for (int m = 0; m < kWMT; ++m)
#pragma unroll
        for (int n = 0; n < kWNT; ++n) acc[m][n] = zero_f32x4();
    }
    if (c + 3 < total_steps) produce(c + 3);   // into the slot step c - 1 freed
    asm volatile("" ::: "memory");
    const _Float16* buf = smem + (c % kRSlots) * kRSlotHalves;
    {
      half8 a[kWMT], b[kWNT];
#pragma unroll
      for (int n = 0; n < kWNT; ++n) b[n] = *reinterpret_cast<const half8*>(buf + b_off + n * 16 * kRBK);
#pragma unroll
      for (int m = 0; m < kWMT; ++m) a[m] = *reinterpret_cast<const half8*>(buf + a_off + m * 16 * kRBK);
#pragma unroll
      for (int m = 0; m < kWMT; ++m)
#pragma unroll
        for (int n = 0; n < kWNT; ++n) acc[m][n] = mfma16(b[n], a[m], acc[m][n]);
    }
    if (kstep == nks - 1) {
      // epilogue straight from the accumulators (rows fr of each m-tile, columns
      // 32 p + 8 g4 + [0, 8) of the wave's 64); the next tile's slots are landing meanwhile
      const float* bt = sBias + (tl & 1) * kBN + wn * 64 + 8 * g4;
      float4 bias4[2][2];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
#pragma unroll
        for (int h = 0; h < 2; ++h) bias4[pp][h] = lds_read4_asm(bt + 32 * pp + 4 * h);
      const int cbase = col0 + wn * 64 + 8 * g4;
#pragma unroll
      for (int m = 0; m < kWMT; ++m) {
        const int row = row0 + wm * 128 + m * 16 + fr;
        if (row >= M) continue;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int col = cbase + 32 * pp;
          const float4 b0 = bias4[pp][0], b1 = bias4[pp][1];
          float v[8] = {acc[m][2 * pp][0] + b0.x, acc[m][2 * pp][1] + b0.y,
                        acc[m][2 * pp][2] + b0.z, acc[m][2 * pp][3] + b0.w,
                        acc[m][2 * pp + 1][0] + b1.x, acc[m][2 * pp + 1][1] + b1.y,
                        acc[m][2 * pp + 1][2] + b1.z, acc[m][2 * pp + 1][3] + b1.w};
          if constexpr (EPI == EPI_F16 || EPI == EPI_GELU_F16) {
            half8 o;
#pragma unroll
            for (int q = 0; q < 8; ++q) o[q] = (_Float16)(EPI == EPI_GELU_F16 ? gelu_erf(v[q]) : v[q]);
            *reinterpret_cast<half8*>(static_cast<_Float16*>(p.C) + (int64_t)row * p.ldc + col) = o;
          } else {
            float* cp = static_cast<float*>(p.C) + (int64_t)row * p.ldc + col;
            if constexpr (EPI == EPI_RESID_F32) {
              const float4 r0 = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + col);
              const float4 r1 = *reinterpret_cast<const float4*>(p.R + (int64_t)row * p.ldr + col + 4);
              v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
              v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
            }
            *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
          }
        }
      }
    }
    // step c + 1's slot has landed (only the two younger slots may still be in flight:
    // vmcnt retires in issue order, so any younger epilogue stores only add to the wait),
    // and every wave is done reading slot c % 4 before it is refilled at step c + 1
    if (c + 1 < total_steps) {
      const int ahead = min(2, total_steps - (c + 2));
      if (ahead == 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
}

bool gemm_big_supported(int epi, const GemmArgs& p) {
  if (!(epi == EPI_F16 || epi == EPI_GELU_F16 || epi == EPI_RESID_F32 || epi == EPI_F32)) return false;
  if (p.M < kBM || p.N % kBN != 0 || p.K % kBK != 0 || p.K < 2 * kBK) return false;
  if (p.lda % 8 || p.ldw % 8 || p.ldc % 8) return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.W & 15) || ((uintptr_t)p.C & 15)) return false;
  if (epi == EPI_RESID_F32 && (!p.R || p.ldr % 4 || ((uintptr_t)p.R & 15))) return false;
  if (p.kc || p.ln_part || p.a_group_cols || p.ln_out || p.lnin_x) return false;
  return (int64_t)cdiv(p.M, kBM) * (p.N / kBN) < (1ll << 31);
}

void gemm_big_launch(int epi, const GemmArgs& p, hipStream_t s) {
  JANUS_CHECK(gemm_big_supported(epi, p), "gemm_big: unsupported shape / layout");
  const unsigned blocks = (unsigned)(cdiv(p.M, kBM) * (p.N / kBN));
  static const int variant = std::getenv("JANUS_GEMM_BIG_V") ? std::atoi(std::getenv("JANUS_GEMM_BIG_V")) : 3;
  if (variant == 3) {
    const unsigned grid = std::min<unsigned>(blocks, (unsigned)stream_cu_count(s));
    switch (epi) {
      case EPI_F16: gemm_big_ring_kernel<EPI_F16><<<grid, kThreads, 0, s>>>(p); break;
      case EPI_GELU_F16: gemm_big_ring_kernel<EPI_GELU_F16><<<grid, kThreads, 0, s>>>(p); break;
      case EPI_RESID_F32: gemm_big_ring_kernel<EPI_RESID_F32><<<grid, kThreads, 0, s>>>(p); break;
      default: gemm_big_ring_kernel<EPI_F32><<<grid, kThreads, 0, s>>>(p); break;
    }
    JANUS_LAUNCH_CHECK();
    return;
  }
  if (variant == 2) {
    const unsigned grid = std::min<unsigned>(blocks, (unsigned)stream_cu_count(s));
    switch (epi) {
      case EPI_F16: gemm_big_persist_kernel<EPI_F16><<<grid, kThreads, 0, s>>>(p); break;
      case EPI_GELU_F16: gemm_big_persist_kernel<EPI_GELU_F16><<<grid, kThreads, 0, s>>>(p); break;
      case EPI_RESID_F32: gemm_big_persist_kernel<EPI_RESID_F32><<<grid, kThreads, 0, s>>>(p); break;
      default: gemm_big_persist_kernel<EPI_F32><<<grid, kThreads, 0, s>>>(p); break;
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

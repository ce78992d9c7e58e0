// fp16 "NT" GEMM on MFMA (v_mfma_f32_16x16x32_f16, fp32 accumulate) with fused
// epilogues, for the Whisper encoder/decoder projections:
//   C[M,N] = epi( A[M,K] · W[N,K]^T + bias[N] )
// A row-major (K contiguous), W in nn.Linear layout [out][in] (K contiguous), so both
// operands feed MFMA fragments as 16-byte LDS reads with no transpose.
// Epilogues: store fp16 | erf-GELU -> fp16 | fp32 residual add (x += ...) | store fp32.
//
// Tiling: BMxBNx64 block tile, 4 waves (each WMT x WNT 16x16 tiles), register-staged
// double-buffered LDS (one barrier per 64-deep K step; next tile's global loads issued
// before the current tile's MFMAs), rows padded to a 160-B pitch so the ds_read_b128
// lane groups are conflict-free (frag_pitch), XCD-aware tile order (blocks sharing an A panel on one L2).
#include <cstdlib>
#include "mfma.h"
#include "kernels.h"

namespace janus {

template <int BM, int BN, int WMT, int WNT, int EPI>
__global__ __launch_bounds__(256) void gemm_nt_kernel(GemmArgs p) {
  constexpr int BK = 64, LS = frag_pitch(BK);  // LDS row stride (conflict-free b128 reads)
  constexpr int WN = BN / (16 * WNT);
  static_assert((BM / (16 * WMT)) * WN == 4, "4 waves per block");
  constexpr int KC = BK / 8;                  // 16-byte chunks per tile row
  constexpr int A_CH = BM * KC / 256, B_CH = BN * KC / 256;
  static_assert(A_CH * 256 == BM * KC && B_CH * 256 == BN * KC, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * (BM + BN) * LS];

  const int M = p.M, N = p.N, K = p.K;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, nbm * nbn);
  const int bm = bid / nbn, bn = bid % nbn;
  const int row0 = bm * BM, col0 = bn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = wave_id();
  const int wm = wid / WN, wn = wid % WN;

  uint4 ra[A_CH], rb[B_CH];
  // unconditional loads of clamped addresses, zeroed after (a guarded load compiles to a
  // branch per 16-byte chunk)
  auto gload = [&](int k0) {
#pragma unroll
    for (int c = 0; c < A_CH; ++c) {
      const int idx = tid + c * 256, r = idx / KC, kc = idx % KC;
      const int gr = row0 + r, gk = k0 + kc * 8;
      ra[c] = *reinterpret_cast<const uint4*>(p.A + (int64_t)min(gr, M - 1) * p.lda + min(gk, K - 8));
      if (!(gr < M && gk < K)) ra[c] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < B_CH; ++c) {
      const int idx = tid + c * 256, r = idx / KC, kc = idx % KC;
      const int gr = col0 + r, gk = k0 + kc * 8;
      rb[c] = *reinterpret_cast<const uint4*>(p.W + (int64_t)min(gr, N - 1) * p.ldw + min(gk, K - 8));
      if (!(gr < N && gk < K)) rb[c] = make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
    _Float16* sA = smem + buf * (BM + BN) * LS;
    _Float16* sB = sA + BM * LS;
#pragma unroll
    for (int c = 0; c < A_CH; ++c) {
      const int idx = tid + c * 256, r = idx / KC, kc = idx % KC;
      *reinterpret_cast<uint4*>(sA + r * LS + kc * 8) = ra[c];
    }
#pragma unroll
    for (int c = 0; c < B_CH; ++c) {
      const int idx = tid + c * 256, r = idx / KC, kc = idx % KC;
      *reinterpret_cast<uint4*>(sB + r * LS + kc * 8) = rb[c];
    }
  };

  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int m = 0; m < WMT; ++m)
#pragma unroll
    for (int n = 0; n < WNT; ++n) acc[m][n] = zero_f32x4();

  const int nk = (K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const _Float16* sA = smem + cur * (BM + BN) * LS;
    const _Float16* sB = sA + BM * LS;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      half8 a[WMT], b[WNT];
      const int ko = ks * 32 + 8 * (lane >> 4);
#pragma unroll
      for (int m = 0; m < WMT; ++m)
        a[m] = *reinterpret_cast<const half8*>(sA + (wm * WMT * 16 + m * 16 + (lane & 15)) * LS + ko);
#pragma unroll
      for (int n = 0; n < WNT; ++n)
        b[n] = *reinterpret_cast<const half8*>(sB + (wn * WNT * 16 + n * 16 + (lane & 15)) * LS + ko);
#pragma unroll
      for (int m = 0; m < WMT; ++m)
#pragma unroll
        for (int n = 0; n < WNT; ++n) acc[m][n] = mfma16(a[m], b[n], acc[m][n]);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue through LDS (the loop's last barrier freed it): the fp32 tile, then 8
  // consecutive columns per thread -> bias / activation / residual -> 16-byte stores
  constexpr int EP = BN + 4;  // fp32 pitch: the 4 row groups of a fragment store hit distinct banks
  static_assert((size_t)BM * EP * 4 <= sizeof(smem), "epilogue tile must fit the staging LDS");
  float* sC = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int m = 0; m < WMT; ++m)
#pragma unroll
    for (int n = 0; n < WNT; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sC[(wm * WMT * 16 + m * 16 + (lane >> 4) * 4 + r) * EP + wn * WNT * 16 + n * 16 + (lane & 15)] =
            acc[m][n][r];
  __syncthreads();
  constexpr int CPR8 = BN / 8;  // 8-column chunks per tile row
  const bool vec = (N % 8) == 0 && (p.ldc % 8) == 0 && (EPI != EPI_RESID_F32 || (p.ldr % 4) == 0);
#pragma unroll 2
  for (int idx = tid; idx < BM * CPR8; idx += 256) {
    const int r = idx / CPR8, c8 = (idx % CPR8) * 8;
    const int row = row0 + r, col = col0 + c8;
    if (row >= M || col >= N) continue;
    const float4 lo = *reinterpret_cast<const float4*>(sC + r * EP + c8);
    const float4 hi = *reinterpret_cast<const float4*>(sC + r * EP + c8 + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += p.bias[min(col + j, N - 1)];
    }
    if (vec) {
      if constexpr (EPI == EPI_F16 || EPI == EPI_GELU_F16) {
        half8 h;
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = (_Float16)(EPI == EPI_GELU_F16 ? gelu_erf(v[j]) : v[j]);
        *reinterpret_cast<half8*>(static_cast<_Float16*>(p.C) + (int64_t)row * p.ldc + col) = h;
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
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (col + j >= N) break;
        if constexpr (EPI == EPI_F16) {
          static_cast<_Float16*>(p.C)[(int64_t)row * p.ldc + col + j] = (_Float16)v[j];
        } else if constexpr (EPI == EPI_GELU_F16) {
          static_cast<_Float16*>(p.C)[(int64_t)row * p.ldc + col + j] = (_Float16)gelu_erf(v[j]);
        } else if constexpr (EPI == EPI_RESID_F32) {
          float* c = static_cast<float*>(p.C) + (int64_t)row * p.ldc + col + j;
          *c = p.R[(int64_t)row * p.ldr + col + j] + v[j];
        } else {
          static_cast<float*>(p.C)[(int64_t)row * p.ldc + col + j] = v[j];
        }
      }
    }
  }
}

template <int BM, int BN, int WMT, int WNT>
static void launch_cfg(int epi, const GemmArgs& p, hipStream_t s) {
  const int blocks = (int)(cdiv(p.M, BM) * cdiv(p.N, BN));
  switch (epi) {
    case EPI_F16: gemm_nt_kernel<BM, BN, WMT, WNT, EPI_F16><<<blocks, 256, 0, s>>>(p); break;
    case EPI_GELU_F16: gemm_nt_kernel<BM, BN, WMT, WNT, EPI_GELU_F16><<<blocks, 256, 0, s>>>(p); break;
    case EPI_RESID_F32: gemm_nt_kernel<BM, BN, WMT, WNT, EPI_RESID_F32><<<blocks, 256, 0, s>>>(p); break;
    case EPI_F32: gemm_nt_kernel<BM, BN, WMT, WNT, EPI_F32><<<blocks, 256, 0, s>>>(p); break;
    default: throw Error("bad gemm epilogue");
  }
  JANUS_LAUNCH_CHECK();
}


// ---------------------------------------------------------------- skinny M
// M <= 64 (decoder steps: one row per utterance). These GEMMs are latency-bound (0.5-2 MB
// of weights, 64 rows), so the design minimises dependent memory round trips: a block is
// all 64 rows x 16 columns with 16 waves splitting K (an N = 512 projection still spreads
// over 32 blocks and every weight byte is read once per step); each wave issues the loads
// of up to G k-steps before its first MFMA (one k-step per wave at K = 512), the epilogue's
// residual / bias loads are issued at kernel entry, and the 16 partial products are
// reduced through LDS. LNA: A is the fp32 residual stream, LayerNorm-ed on load from the
// row-statistic pieces its producer wrote (SkinnyLnArgs).
struct SkinnyArgs {
  const _Float16* A; int64_t lda;
  const float* x; int64_t ldx; const float2* part; const float* gamma; const float* beta;
  float eps;
  const _Float16* W; int64_t ldw;
  const float* bias;
  void* C; int64_t ldc;
  const float* R; int64_t ldr;
  int M, N, K;
  _Float16* kc; _Float16* vc; int pos, n_ctx, qkv_d;
  float2* ln_part;
  int a_group_cols;
  int msplit_n;
  const float* ln_g; const float* ln_b; float ln_eps; _Float16* ln_out; int* ln_cnt;
  const float* lnin_g; const float* lnin_b;  // AM_LNX: A = LayerNorm(x) computed in-block
  const int32_t* roff;  // EPI_QKV: per-row position offsets (row r's cache row pos + roff[r])
};

// A operand modes: fp16 from global memory; LayerNorm-on-load from producer pieces
// (JANUS_FUSED_LN); LayerNorm of the block's fp32 rows computed in the block's prologue
// into an fp16 LDS tile (no separate LayerNorm launch).
enum SkinnyAMode { AM_F16 = 0, AM_LNA = 1, AM_LNX = 2 };

constexpr int kSkWaves = 16;

// MTB: 16-row m-tiles per block (4: all 64 rows; 1: rows split over gridDim.y, for narrow
// outputs whose N / 16 column tiles alone would leave most CUs idle).
// K1: K <= 16 waves x 32, one k-step per wave: G = 1 keeps the all-rows form (MTB = 4)
// under 64 VGPRs, two 16-wave blocks per CU (the 4096-wide absorbed query projection's 256
// blocks in one round on a 128-CU partition instead of two: 91 VGPRs admitted one).
template <int EPI, int AM, int MTB, bool K1 = false>
__global__ __launch_bounds__(1024) void gemm_skinny_kernel(SkinnyArgs p) {
  constexpr bool LNA = AM == AM_LNA, LNX = AM == AM_LNX;
  // k-steps in flight per wave (128-VGPR budget at 1024 threads; the LayerNorm modes run
  // K <= 512, one k-step per wave)
  constexpr int G = (LNA || LNX || K1) ? 1 : 2;
  extern __shared__ __attribute__((aligned(16))) _Float16 sk_smem[];  // LNX: [16*MTB][AP]
  __shared__ float red[8][16 * MTB][17];
  __shared__ float s_mean[64], s_rstd[64];
  const int M = p.M, N = p.N, K = p.K;
  const int col0 = blockIdx.x * 16, r0 = blockIdx.y * 16 * MTB;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int kq = ((K + kSkWaves - 1) / kSkWaves + 31) / 32 * 32;
  const int kbeg = w * kq, kend = min(K, kbeg + kq);
  const int bcol = col0 + (lane & 15);
  const _Float16* wrow = p.W + (int64_t)min(bcol, N - 1) * p.ldw;
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  const _Float16* Ab = p.A;
  if constexpr (AM == AM_F16) {
    if (p.a_group_cols > 0) Ab += (int64_t)(col0 / p.a_group_cols) * K;  // block-diagonal
  }
  const int AP = frag_pitch(K);  // LNX tile pitch (halves)

  // epilogue operands independent of the product, in flight from the start
  const int elr = tid >> 4, erow = r0 + elr, ec = tid & 15, ecol = col0 + ec;
  const bool eok = elr < 16 * MTB && erow < M && ecol < N;
  float e_add = (p.bias && eok) ? p.bias[ecol] : 0.0f;
  if constexpr (EPI == EPI_RESID_F32) e_add += eok ? p.R[(int64_t)erow * p.ldr + ecol] : 0.0f;

  half8 bw[G];
  half8 ah[LNA ? 1 : G][MTB];
  float4 ax[LNA ? G : 1][4][2];
  auto load = [&](int k0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int kk = k0 + 32 * g + kc8;
      const bool ok = kk < kend;
#ifdef JANUS_W_NT
      {
        const uint4 u = (ok && bcol < N) ? ld_nt(wrow + kk) : make_uint4(0, 0, 0, 0);
        bw[g] = *reinterpret_cast<const half8*>(&u);
      }
#else
      bw[g] = (ok && bcol < N) ? *reinterpret_cast<const half8*>(wrow + kk) : zero_half8();
#endif
#pragma unroll
      for (int m = 0; m < MTB; ++m) {
        const int r = r0 + m * 16 + lr;
        if constexpr (LNA) {
          const float* xr = p.x + (int64_t)r * p.ldx + kk;
          const bool rok = ok && r < M;
          ax[g][m][0] = rok ? *reinterpret_cast<const float4*>(xr) : make_float4(0.f, 0.f, 0.f, 0.f);
          ax[g][m][1] = rok ? *reinterpret_cast<const float4*>(xr + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        } else if constexpr (!LNX) {
          ah[g][m] = (ok && r < M) ? *reinterpret_cast<const half8*>(Ab + (int64_t)r * p.lda + kk)
                                   : zero_half8();
        }
      }
    }
  };
  load(kbeg);

  if constexpr (LNX) {
    // this block's rows of LN(x) -> fp16 LDS tile: wave w normalises rows w + 16j (j < MTB),
    // all loads in one round trip behind the weights already in flight
    ln_rows_wave<2, MTB>(p.x, p.ldx, r0 + w, kSkWaves, M, p.lnin_g, p.lnin_b, sk_smem, w, AP, K, p.eps, lane);
    __syncthreads();
  }

  if constexpr (LNA) {
    // row statistics from the producer's pieces: waves 0-3, thread = (row, quarter)
    if (tid < 64 * MTB) {
      const int r = tid >> 2, qd = tid & 3, np = K / 16;  // r: local row
      const int gr = r0 + r;
      constexpr int NPQ = 12;  // pieces per thread held in registers (K <= 768)
      float2 pc[NPQ];
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < NPQ; ++j) {
        const int g = qd + 4 * j;
        pc[j] = (gr < M && g < np) ? p.part[(int64_t)gr * np + g] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < NPQ; ++j) sm += pc[j].x;
      for (int g = qd + 4 * NPQ; g < np; g += 4) sm += (gr < M) ? p.part[(int64_t)gr * np + g].x : 0.f;
      sm += __shfl_xor(sm, 1);
      sm += __shfl_xor(sm, 2);
      const float mean = sm / K;
      float m2 = 0.f;
#pragma unroll
      for (int j = 0; j < NPQ; ++j) {
        if (qd + 4 * j < np) {
          const float dm = pc[j].x * (1.0f / 16.0f) - mean;
          m2 += pc[j].y + 16.0f * dm * dm;
        }
      }
      for (int g = qd + 4 * NPQ; g < np; g += 4) {
        const float2 q = (gr < M) ? p.part[(int64_t)gr * np + g] : make_float2(0.f, 0.f);
        const float dm = q.x * (1.0f / 16.0f) - mean;
        m2 += q.y + 16.0f * dm * dm;
      }
      m2 += __shfl_xor(m2, 1);
      m2 += __shfl_xor(m2, 2);
      if (qd == 0) { s_mean[r] = mean; s_rstd[r] = rsqrtf(m2 / K + p.eps); }
    }
    __syncthreads();
  }

  f32x4 acc[MTB];
#pragma unroll
  for (int m = 0; m < MTB; ++m) acc[m] = zero_f32x4();
  for (int k0 = kbeg; k0 < kend; k0 += 32 * G) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int kk = k0 + 32 * g + kc8;
      if (k0 + 32 * g >= kend) break;  // wave-uniform
      half8 af[MTB];
      if constexpr (LNA) {
        const bool ok = kk < kend;
        float ga[8], be[8];
        {
          const float4 g0 = ok ? *reinterpret_cast<const float4*>(p.gamma + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 g1 = ok ? *reinterpret_cast<const float4*>(p.gamma + kk + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 b0 = ok ? *reinterpret_cast<const float4*>(p.beta + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 b1 = ok ? *reinterpret_cast<const float4*>(p.beta + kk + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
          ga[0] = g0.x; ga[1] = g0.y; ga[2] = g0.z; ga[3] = g0.w; ga[4] = g1.x; ga[5] = g1.y; ga[6] = g1.z; ga[7] = g1.w;
          be[0] = b0.x; be[1] = b0.y; be[2] = b0.z; be[3] = b0.w; be[4] = b1.x; be[5] = b1.y; be[6] = b1.z; be[7] = b1.w;
        }
#pragma unroll
        for (int m = 0; m < MTB; ++m) {
          const int r = m * 16 + lr;
          const float mean = s_mean[r], rstd = s_rstd[r];
          const float xv[8] = {ax[g][m][0].x, ax[g][m][0].y, ax[g][m][0].z, ax[g][m][0].w,
                               ax[g][m][1].x, ax[g][m][1].y, ax[g][m][1].z, ax[g][m][1].w};
#pragma unroll
          for (int j = 0; j < 8; ++j)
            af[m][j] = (ok && r0 + r < M) ? (_Float16)((xv[j] - mean) * rstd * ga[j] + be[j]) : (_Float16)0.0f;
        }
      } else if constexpr (LNX) {
        const bool ok = kk < kend;
#pragma unroll
        for (int m = 0; m < MTB; ++m)
          af[m] = ok ? *reinterpret_cast<const half8*>(sk_smem + (m * 16 + lr) * AP + kk) : zero_half8();
      } else {
#pragma unroll
        for (int m = 0; m < MTB; ++m) af[m] = ah[g][m];
      }
#pragma unroll
      for (int m = 0; m < MTB; ++m) acc[m] = mfma16(af[m], bw[g], acc[m]);
    }
    if (k0 + 32 * G < kend) load(k0 + 32 * G);
  }

  // 16 partials -> LDS: waves 0-7 store, waves 8-15 add, then one output per thread
  if (w < 8) {
#pragma unroll
    for (int m = 0; m < MTB; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][m * 16 + 4 * (lane >> 4) + r][lane & 15] = acc[m][r];
  }
  __syncthreads();
  if (w >= 8) {
#pragma unroll
    for (int m = 0; m < MTB; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w - 8][m * 16 + 4 * (lane >> 4) + r][lane & 15] += acc[m][r];
  }
  __syncthreads();
  float v = e_add;
  if (elr < 16 * MTB) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v += red[i][elr][ec];
  }
  // thread -> (row tid>>4, col col0 + (tid&15)): 16 aligned lanes hold one row's columns
  if constexpr (EPI == EPI_RESID_F32) {
    if (p.ln_out) {  // block-uniform: fused LayerNorm of the new rows (GemmArgs::ln_out)
      __shared__ int s_last;
      if (eok) __hip_atomic_store(static_cast<float*>(p.C) + (int64_t)erow * p.ldc + ecol, v,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores drained
      __syncthreads();                                   // ... and every other wave's
      // one counter per row block: the last of its gridDim.x column blocks to arrive
      // normalises the block's rows (one row per wave), in parallel over row blocks
      int* cnt = p.ln_cnt + blockIdx.y;
      if (tid == 0)
        s_last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 (int)gridDim.x - 1;
      __syncthreads();
      if (!s_last) return;
      for (int r = r0 + w; r < min(M, r0 + 16 * MTB); r += kSkWaves)
        ln_row_wave<true>(static_cast<const float*>(p.C) + (int64_t)r * p.ldc, p.ln_g, p.ln_b,
                          p.ln_out + (int64_t)r * N, N, p.ln_eps, lane);
      if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (eok) static_cast<float*>(p.C)[(int64_t)erow * p.ldc + ecol] = v;
    if (p.ln_part) {  // block-uniform
      const float y = eok ? v : 0.0f;
      float sm = y;
      sm += __shfl_xor(sm, 1); sm += __shfl_xor(sm, 2);
      sm += __shfl_xor(sm, 4); sm += __shfl_xor(sm, 8);
      const float mu = sm * (1.0f / 16.0f);
      float q = (y - mu) * (y - mu);
      q += __shfl_xor(q, 1); q += __shfl_xor(q, 2);
      q += __shfl_xor(q, 4); q += __shfl_xor(q, 8);
      if (ec == 0 && eok) p.ln_part[(int64_t)erow * (N / 16) + col0 / 16] = make_float2(sm, q);
    }
    return;
  }
  if (!eok) return;
  if constexpr (EPI == EPI_F16) {
    static_cast<_Float16*>(p.C)[(int64_t)erow * p.ldc + ecol] = (_Float16)v;
  } else if constexpr (EPI == EPI_GELU_F16) {
    static_cast<_Float16*>(p.C)[(int64_t)erow * p.ldc + ecol] = (_Float16)gelu_erf(v);
  } else if constexpr (EPI == EPI_QKV) {
    // q -> C; k, v -> cache rows (row * n_ctx + pos)
    const int dq = p.qkv_d;
    if (ecol < dq) {
      static_cast<_Float16*>(p.C)[(int64_t)erow * p.ldc + ecol] = (_Float16)v;
    } else {
      _Float16* cache = ecol < 2 * dq ? p.kc : p.vc;
      const int cpos = p.pos + (p.roff ? p.roff[erow] : 0);
      cache[((int64_t)erow * p.n_ctx + cpos) * dq + (ecol % dq)] = (_Float16)v;
    }
  } else {
    static_cast<float*>(p.C)[(int64_t)erow * p.ldc + ecol] = v;
  }
}

// 64 rows x 32 columns per block (two 16-column tiles per wave), 16 waves split K at one
// 32-deep k-step each (K <= 512): for plain fp16 projections wider than one 16-column tile
// per CU (the decoder's 4096-wide absorbed query projection), one block per CU with half
// the A re-reads of the 16-column form. Bit-identical to gemm_skinny_kernel<EPI_F16,
// AM_F16, 4, K1> (same single-k-step MFMA per wave, same reduction order).
// LNX: A = LayerNorm(x) of all 64 rows computed in the block's prologue into an fp16 LDS
// tile (ln_rows_wave: layernorm_kernel's arithmetic, so bit-identical to a LayerNorm launch
// followed by the plain form).
template <bool LNX>
__global__ __launch_bounds__(1024) void gemm_skinny2_kernel(SkinnyArgs p) {
  __shared__ float red[2][8][64][17];
  extern __shared__ __attribute__((aligned(16))) _Float16 s2_smem[];  // LNX: [64][AP]
  const int M = p.M, N = p.N, K = p.K;
  const int col0 = blockIdx.x * 32;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int kbeg = w * 32;
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);
  const bool kok = kbeg + kc8 < K;  // this lane's 8 halves (K % 8 == 0)
  half8 bw[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int bcol = col0 + 16 * t + lr;
    const _Float16* wrow = p.W + (int64_t)min(bcol, N - 1) * p.ldw;
    bw[t] = (kok && bcol < N) ? *reinterpret_cast<const half8*>(wrow + kbeg + kc8) : zero_half8();
  }
  half8 ah[4];
  if constexpr (LNX) {
    const int AP = frag_pitch(K);
    // wave w normalises rows w + 16j (j < 4), all loads in one round trip
    ln_rows_wave<2, 4>(p.x, p.ldx, w, kSkWaves, M, p.lnin_g, p.lnin_b, s2_smem, w, AP, K, p.eps, lane);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 4; ++m)
      ah[m] = kok ? *reinterpret_cast<const half8*>(s2_smem + (m * 16 + lr) * AP + kbeg + kc8) : zero_half8();
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int r = m * 16 + lr;
      ah[m] = (kok && r < M) ? *reinterpret_cast<const half8*>(p.A + (int64_t)r * p.lda + kbeg + kc8)
                             : zero_half8();
    }
  }
  const int elr = tid >> 4, ec = tid & 15;
  float e_add[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ecol = col0 + 16 * t + ec;
    e_add[t] = (p.bias && elr < M && ecol < N) ? p.bias[ecol] : 0.0f;
  }
  f32x4 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[m][t] = mfma16(ah[m], bw[t], zero_f32x4());
  if (w < 8) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[t][w][m * 16 + 4 * (lane >> 4) + r][lr] = acc[m][t][r];
  }
  __syncthreads();
  if (w >= 8) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[t][w - 8][m * 16 + 4 * (lane >> 4) + r][lr] += acc[m][t][r];
  }
  __syncthreads();
  if (elr >= M) return;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ecol = col0 + 16 * t + ec;
    float v = e_add[t];
#pragma unroll
    for (int i = 0; i < 8; ++i) v += red[t][i][elr][ec];
    if (ecol < N) static_cast<_Float16*>(p.C)[(int64_t)elr * p.ldc + ecol] = (_Float16)v;
  }
}

template <int AM, int EPI, int MTB>
static void skinny_go(const SkinnyArgs& p, dim3 grid, hipStream_t s) {
  auto kern = gemm_skinny_kernel<EPI, AM, MTB>;
  if constexpr (AM == AM_F16 && MTB == 4) {
    if (p.K <= kSkWaves * 32 && ab_env("JANUS_SKINNY_NO_K1") == nullptr)
      kern = gemm_skinny_kernel<EPI, AM, MTB, true>;
  }
  size_t lds = 0;
  if constexpr (AM == AM_LNX) {
    lds = (size_t)16 * MTB * frag_pitch(p.K) * 2;
    static bool attr = false;
    if (!attr) {
      JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    100 * 1024));
      attr = true;
    }
  }
  kern<<<grid, 1024, lds, s>>>(p);
}

template <int AM, int MTB>
static void launch_skinny_m(int epi, const SkinnyArgs& p, hipStream_t s) {
  const dim3 grid((p.N + 15) / 16, (p.M + 16 * MTB - 1) / (16 * MTB));
  switch (epi) {
    case EPI_F16: skinny_go<AM, EPI_F16, MTB>(p, grid, s); break;
    case EPI_GELU_F16: skinny_go<AM, EPI_GELU_F16, MTB>(p, grid, s); break;
    case EPI_QKV: skinny_go<AM, EPI_QKV, MTB>(p, grid, s); break;
    case EPI_RESID_F32:
      if constexpr (AM == AM_F16) { skinny_go<AM, EPI_RESID_F32, MTB>(p, grid, s); break; }
      else throw Error("skinny LN gemm: bad epilogue");
    case EPI_F32:
      if constexpr (AM == AM_F16) { skinny_go<AM, EPI_F32, MTB>(p, grid, s); break; }
      else throw Error("skinny LN gemm: bad epilogue");
    default: throw Error("bad gemm epilogue");
  }
  JANUS_LAUNCH_CHECK();
}

template <int AM>
static void launch_skinny_t(int epi, const SkinnyArgs& p, hipStream_t s) {
  // plain fp16 outputs wider than 2048 columns (more 16-column tiles than a 128-CU
  // partition holds in one round) at K <= 512: 32 columns per block
  static const bool nct2 = ab_env("JANUS_SKINNY_NO_NCT2") == nullptr;
  if constexpr (AM == AM_F16 || AM == AM_LNX) {
    if (nct2 && epi == EPI_F16 && p.N > 2048 && p.K <= kSkWaves * 32 && p.a_group_cols == 0 && p.M <= 64) {
      if constexpr (AM == AM_LNX) {
        auto kern = gemm_skinny2_kernel<true>;
        static bool attr = false;
        if (!attr) {
          JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        88 * 1024));
          attr = true;
        }
        kern<<<(p.N + 31) / 32, 1024, (size_t)64 * frag_pitch(p.K) * 2, s>>>(p);
      } else {
        gemm_skinny2_kernel<false><<<(p.N + 31) / 32, 1024, 0, s>>>(p);
      }
      JANUS_LAUNCH_CHECK();
      return;
    }
  }
  // narrow outputs (N <= JANUS_SKINNY_MSPLIT_N, default 2048: <= 128 column tiles) split the
  // rows over 16-row blocks as well, so 4x as many CUs share the latency-bound product
  static const int msplit_n = [] {
    const char* e = ab_env("JANUS_SKINNY_MSPLIT_N");
    return e ? std::atoi(e) : 2048;
  }();
  if (p.N <= (p.msplit_n > 0 ? p.msplit_n : msplit_n)) { launch_skinny_m<AM, 1>(epi, p, s); return; }
  launch_skinny_m<AM, 4>(epi, p, s);
}

static void launch_skinny(int epi, const GemmArgs& g, hipStream_t s) {
  SkinnyArgs p{};
  p.A = g.A; p.lda = g.lda; p.W = g.W; p.ldw = g.ldw; p.bias = g.bias; p.C = g.C; p.ldc = g.ldc;
  p.R = g.R; p.ldr = g.ldr; p.M = g.M; p.N = g.N; p.K = g.K;
  p.kc = g.kc; p.vc = g.vc; p.pos = g.pos; p.n_ctx = g.n_ctx; p.qkv_d = g.qkv_d;
  p.roff = g.roff;
  p.ln_part = g.ln_part;
  p.a_group_cols = g.a_group_cols;
  p.msplit_n = g.msplit_n;
  p.ln_g = g.ln_g; p.ln_b = g.ln_b; p.ln_eps = g.ln_eps; p.ln_out = g.ln_out; p.ln_cnt = g.ln_cnt;
  if (g.lnin_x) {  // A = LayerNorm(x) in the block's prologue (K <= 512)
    JANUS_CHECK(g.K <= 512 && g.K % 4 == 0, "skinny LayerNorm prologue: K <= 512, K % 4 == 0");
    p.x = g.lnin_x; p.ldx = g.lnin_ldx; p.lnin_g = g.lnin_g; p.lnin_b = g.lnin_b; p.eps = g.lnin_eps;
    launch_skinny_t<AM_LNX>(epi, p, s);
    return;
  }
  launch_skinny_t<AM_F16>(epi, p, s);
}

void gemm_skinny_ln_launch(int epi, const SkinnyLnArgs& g, hipStream_t s) {
  JANUS_CHECK(g.M <= 64 && g.K % 16 == 0 && g.ldx % 4 == 0 && g.part,
              "skinny LN gemm: M <= 64, K % 16 == 0, LayerNorm pieces required");
  if (g.M <= 0 || g.N <= 0) return;
  SkinnyArgs p{};
  p.x = g.x; p.ldx = g.ldx; p.part = g.part; p.gamma = g.gamma; p.beta = g.beta; p.eps = g.eps;
  p.W = g.W; p.ldw = g.ldw; p.bias = g.bias; p.C = g.C; p.ldc = g.ldc; p.M = g.M; p.N = g.N; p.K = g.K;
  p.kc = g.kc; p.vc = g.vc; p.pos = g.pos; p.n_ctx = g.n_ctx; p.qkv_d = g.qkv_d;
  launch_skinny_t<AM_LNA>(epi, p, s);
}

void gemm_launch(int epi, const GemmArgs& p, hipStream_t s) {
  JANUS_CHECK(p.K % 8 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0, "gemm: K/lda/ldw must be multiples of 8");
  JANUS_CHECK(((uintptr_t)p.A & 15) == 0 && ((uintptr_t)p.W & 15) == 0, "gemm: A/W must be 16-byte aligned");
  if (p.M <= 0 || p.N <= 0) return;
  // decoder batches above 64 rows (faster-whisper's best_of hypotheses of many windows in
  // one sampled decode) stay on the skinny kernel: its blocks split the rows as well
  JANUS_CHECK(p.M <= kSkinnyMaxRows || epi != EPI_QKV,
              "gemm: the KV-cache epilogue needs M <= kSkinnyMaxRows");
  JANUS_CHECK(p.M <= 64 || !p.ln_part, "gemm: the LayerNorm-piece epilogue needs M <= 64");
  JANUS_CHECK(p.a_group_cols == 0 || (p.M <= kSkinnyMaxRows && p.a_group_cols % 16 == 0),
              "gemm: grouped A needs M <= kSkinnyMaxRows and 16-column groups");
  JANUS_CHECK(!p.ln_part || (epi == EPI_RESID_F32 && p.N % 16 == 0),
              "gemm: LayerNorm pieces come from a RESID epilogue with N % 16 == 0");
  JANUS_CHECK(!p.lnin_x || (p.M <= kSkinnyMaxRows && p.K <= 1024 && p.K % 32 == 0 && p.a_group_cols == 0 &&
                            p.lnin_g && p.lnin_b && epi != EPI_RESID_F32 && epi != EPI_F32),
              "gemm: LayerNorm-prologue A needs M <= kSkinnyMaxRows, K <= 1024 (multiple of 32), no groups");
  JANUS_CHECK(!p.ln_out || (epi == EPI_RESID_F32 && p.M <= 64 && p.N <= 512 && p.N % 4 == 0 && p.ln_cnt &&
                            p.ln_g && p.ln_b && p.ldc == p.N),
              "gemm: fused LayerNorm needs a RESID epilogue, M <= 64, N <= 512, ldc == N");
  JANUS_CHECK(p.M <= 64 || p.decode_rows || (epi != EPI_QKV && !p.lnin_x && p.a_group_cols == 0),
              "gemm: KV-cache / LayerNorm-prologue / grouped products above 64 rows are decoder steps "
              "(GemmArgs::decode_rows)");
  if (p.M <= 64 || (p.decode_rows && p.M <= kSkinnyMaxRows)) launch_skinny(epi, p, s);
  else if (gemm_big_supported(epi, p)) gemm_big_launch(epi, p, s);
  else launch_cfg<128, 128, 4, 4>(epi, p, s);
}

void gemm_nt128_launch(int epi, const GemmArgs& p, hipStream_t s) {
  JANUS_CHECK(p.K % 8 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0, "gemm: K/lda/ldw must be multiples of 8");
  JANUS_CHECK(((uintptr_t)p.A & 15) == 0 && ((uintptr_t)p.W & 15) == 0, "gemm: A/W must be 16-byte aligned");
  JANUS_CHECK(epi >= EPI_F16 && epi <= EPI_F32, "gemm_nt128: plain epilogues only");
  if (p.M <= 0 || p.N <= 0) return;
  launch_cfg<128, 128, 4, 4>(epi, p, s);
}

// exact-erf GELU in place, 8 halves per thread (the library GEMM's fc1 epilogue)
__global__ void gelu_inplace_f16_kernel(_Float16* __restrict__ x, int64_t ld, int M, int N8) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N8) return;
  const int64_t r = i / N8, c = (i % N8) * 8;
  half8* p = reinterpret_cast<half8*>(x + r * ld + c);
  half8 v = *p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (_Float16)gelu_erf((float)v[j]);
  *p = v;
}

void gelu_inplace_f16_launch(_Float16* x, int64_t ld, int M, int N, hipStream_t s) {
  JANUS_CHECK(N % 8 == 0 && ld % 8 == 0, "gelu_inplace: N and ld must be multiples of 8");
  const int64_t n = (int64_t)M * (N / 8);
  if (n == 0) return;
  gelu_inplace_f16_kernel<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(x, ld, M, N / 8);
  JANUS_LAUNCH_CHECK();
}

// ------------------------------------------------------------ residual projection + LayerNorm
// x[r] += A[r] W^T + bias (fp32 residual, in place) and out[r] = LayerNorm(x[r]) (fp16),
// 16 rows per block over ALL N = 32 * NW columns, so the block owns whole rows and the
// LayerNorm needs no second launch and no cross-block hand-off (decoder: the self- and
// cross-attention output projections, each followed by LN2 / LN3; d = 512: 16 waves).
// Wave w owns columns [32w, 32w + 32) over the full K; the block streams all of W
// (0.5 MB at d = 512) through one CU, which a separate LayerNorm launch (≈ 5 µs) more
// than pays for.
// Bit-identical to gemm_skinny_kernel<EPI_RESID_F32> (+ layernorm_kernel): that kernel
// gives each of its 16 waves one 32-deep k-step, p_i = mfma(a_i, b_i, 0), and sums
// v = (bias + R) + (p_0 + p_8) + (p_1 + p_9) + ... + (p_7 + p_15); here a wave walks its
// k-steps in the order 0, 8, 1, 9, ... and adds the pairs in the same order. The
// LayerNorm is layernorm_kernel's arithmetic (lane = float4 column groups, sequential
// per-lane sums, xor-shuffle trees, two-pass variance).
template <int NW, int K>
__global__ __launch_bounds__(NW * 64) void resid_ln_kernel(ResidLnArgs p) {
  constexpr int N = 32 * NW, NV = N / 4, MAXV = (NV + 63) / 64;
  constexpr int KS = K / 32, AP = frag_pitch(K);
  extern __shared__ __attribute__((aligned(16))) unsigned char rl_smem[];
  _Float16* sA = reinterpret_cast<_Float16*>(rl_smem);                  // [16][AP]
  float* sX = reinterpret_cast<float*>(rl_smem + 16 * AP * 2);          // [16][N]
  float* sG = sX + 16 * N;                                              // [N] gamma
  float* sB = sG + N;                                                   // [N] beta
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int r0 = blockIdx.x * 16, M = p.M;
  const int lr = lane & 15, kc8 = 8 * (lane >> 4);

  // k-step of sequence position j: 0, 8, 1, 9, ... (pairs (i, i + 8) adjacent)
  auto kstep = [](int j) { return (j & 1) * 8 + (j >> 1); };
  const _Float16* wr0 = p.W + (int64_t)(32 * w + lr) * p.ldw + kc8;
  const _Float16* wr1 = wr0 + 16 * p.ldw;
  constexpr int RING = 4;  // sequence positions in flight (2 x 16 B per lane each)
  half8 wb[RING][2];
#pragma unroll
  for (int j = 0; j < RING; ++j) {
    const int ks = kstep(j);
    wb[j][0] = ks < KS ? *reinterpret_cast<const half8*>(wr0 + 32 * ks) : zero_half8();
    wb[j][1] = ks < KS ? *reinterpret_cast<const half8*>(wr1 + 32 * ks) : zero_half8();
  }
  // epilogue operands: bias + residual of this lane's 4 rows x 2 columns
  float e[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = 32 * w + 16 * t + lr;
    const float bs = p.bias ? p.bias[col] : 0.0f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * (lane >> 4) + r;
      e[t][r] = bs + (row < M ? p.x[(int64_t)row * p.ldx + col] : 0.0f);
    }
  }
  // A rows and gamma / beta -> LDS
  for (int i = tid; i < 16 * (K / 8); i += NW * 64) {
    const int rr = i / (K / 8), c8 = (i % (K / 8)) * 8;
    const int row = min(r0 + rr, M - 1);
    *reinterpret_cast<half8*>(sA + rr * AP + c8) =
        *reinterpret_cast<const half8*>(p.A + (int64_t)row * p.lda + c8);
  }
  for (int i = tid; i < NV; i += NW * 64) {
    reinterpret_cast<float4*>(sG)[i] = reinterpret_cast<const float4*>(p.g)[i];
    reinterpret_cast<float4*>(sB)[i] = reinterpret_cast<const float4*>(p.b)[i];
  }
  __syncthreads();

  f32x4 v[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) v[t] = f32x4{e[t][0], e[t][1], e[t][2], e[t][3]};
  f32x4 pl[2];
#pragma unroll
  for (int j = 0; j < 2 * 8; ++j) {
    // keep each refill at its iteration: hoisted, all 32 weight loads of the wave would be
    // live at once (164 VGPRs; spills under the 16-wave 128-VGPR budget)
    __builtin_amdgcn_sched_barrier(0);
    const int ks = kstep(j);
    const int slot = j % RING;
    half8 af = ks < KS ? *reinterpret_cast<const half8*>(sA + lr * AP + 32 * ks + kc8) : zero_half8();
    f32x4 pc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) pc[t] = mfma16(af, wb[slot][t], zero_f32x4());
    // refill the slot with sequence position j + RING
    if (j + RING < 16) {
      const int kn = kstep(j + RING);
      wb[slot][0] = kn < KS ? *reinterpret_cast<const half8*>(wr0 + 32 * kn) : zero_half8();
      wb[slot][1] = kn < KS ? *reinterpret_cast<const half8*>(wr1 + 32 * kn) : zero_half8();
    }
    if ((j & 1) == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) pl[t] = pc[t];
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) v[t] += pl[t] + pc[t];
    }
  }
  // new residual rows -> global (fp32) and LDS
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = 32 * w + 16 * t + lr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * (lane >> 4) + r;
      sX[rr * N + col] = v[t][r];
      if (r0 + rr < M) p.x[(int64_t)(r0 + rr) * p.ldx + col] = v[t][r];
    }
  }
  __syncthreads();
  // LayerNorm, one wave per row (layernorm_kernel's arithmetic)
  for (int rr = w; rr < 16; rr += NW) {
    if (r0 + rr >= M) break;
    const float4* xr = reinterpret_cast<const float4*>(sX + rr * N);
    float4 xv[MAXV];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int i = lane + k * 64;
      xv[k] = i < NV ? xr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      s += ln_sum4(xv[k]);
    }
    s = wave_sum_f32(s);
    const float mean = s / (float)N;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int i = lane + k * 64;
      if (i < NV) q += ln_sq4(xv[k], mean);
    }
    q = wave_sum_f32(q);
    const float rstd = rsqrtf(q / (float)N + p.eps);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int i = lane + k * 64;
      if (i >= NV) continue;
      const float4 gg = reinterpret_cast<const float4*>(sG)[i];
      const float4 bb = reinterpret_cast<const float4*>(sB)[i];
      reinterpret_cast<half4*>(p.out + (int64_t)(r0 + rr) * N)[i] = ln_norm4(xv[k], mean, rstd, gg, bb);
    }
  }
}

template <int NW, int K>
static void resid_ln_go(const ResidLnArgs& p, hipStream_t s) {
  auto kern = resid_ln_kernel<NW, K>;
  const size_t lds = (size_t)16 * frag_pitch(p.K) * 2 + (size_t)(16 + 2) * 32 * NW * 4;
  static bool attr = false;
  if (!attr) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
    attr = true;
  }
  kern<<<(p.M + 15) / 16, NW * 64, lds, s>>>(p);
}

bool resid_ln_supported(int N, int K) { return (N == 384 || N == 512) && K == N; }

void resid_ln_launch(const ResidLnArgs& p, hipStream_t s) {
  JANUS_CHECK(resid_ln_supported(p.N, p.K), "resid_ln: N = K in {384, 512}");
  JANUS_CHECK(p.ldx == p.N && p.lda % 8 == 0 && p.ldw % 8 == 0, "resid_ln: ldx == N, lda / ldw % 8 == 0");
  JANUS_CHECK(((uintptr_t)p.A & 15) == 0 && ((uintptr_t)p.W & 15) == 0 && ((uintptr_t)p.x & 15) == 0 &&
                  ((uintptr_t)p.g & 15) == 0 && ((uintptr_t)p.b & 15) == 0 && ((uintptr_t)p.out & 7) == 0,
              "resid_ln: operands must be aligned");
  if (p.M <= 0) return;
  if (p.N == 512) resid_ln_go<16, 512>(p, s);
  else resid_ln_go<12, 384>(p, s);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

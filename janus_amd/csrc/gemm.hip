// fp16 "NT" GEMM on MFMA (v_mfma_f32_16x16x32_f16, fp32 accumulate) with fused
// epilogues, for the Whisper encoder/decoder projections:
//   C[M,N] = epi( A[M,K] · W[N,K]^T + bias[N] )
// A row-major (K contiguous), W in nn.Linear layout [out][in] (K contiguous), so both
// operands feed MFMA fragments as 16-byte LDS reads with no transpose.
// Epilogues: store fp16 | erf-GELU -> fp16 | fp32 residual add (x += ...) | store fp32.
//
// Tiling: BMxBNx64 block tile, 4 waves (each WMT x WNT 16x16 tiles), register-staged
// double-buffered LDS (one barrier per 64-deep K step; next tile's global loads issued
// before the current tile's MFMAs), rows padded by 16 B so the 16-lane ds_read_b128
// groups are conflict-free, XCD-aware tile order (blocks sharing an A panel on one L2).
#include "mfma.h"
#include "kernels.h"

namespace janus {

template <int BM, int BN, int WMT, int WNT, int EPI>
__global__ __launch_bounds__(256) void gemm_nt_kernel(GemmArgs p) {
  constexpr int BK = 64, LS = BK + 8;  // LDS row stride in halves (144 B = 16 B * 9)
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
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  uint4 ra[A_CH], rb[B_CH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int c = 0; c < A_CH; ++c) {
      const int idx = tid + c * 256, r = idx / KC, kc = idx % KC;
      const int gr = row0 + r, gk = k0 + kc * 8;
      ra[c] = (gr < M && gk < K) ? *reinterpret_cast<const uint4*>(p.A + (int64_t)gr * p.lda + gk)
                                 : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < B_CH; ++c) {
      const int idx = tid + c * 256, r = idx / KC, kc = idx % KC;
      const int gr = col0 + r, gk = k0 + kc * 8;
      rb[c] = (gr < N && gk < K) ? *reinterpret_cast<const uint4*>(p.W + (int64_t)gr * p.ldw + gk)
                                 : make_uint4(0, 0, 0, 0);
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

#pragma unroll
  for (int n = 0; n < WNT; ++n) {
    const int col = col0 + wn * WNT * 16 + n * 16 + (lane & 15);
    if (col >= N) continue;
    const float bv = p.bias ? p.bias[col] : 0.0f;
#pragma unroll
    for (int m = 0; m < WMT; ++m) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * WMT * 16 + m * 16 + (lane >> 4) * 4 + r;
        if (row >= M) continue;
        float v = acc[m][n][r] + bv;
        if constexpr (EPI == EPI_F16) {
          static_cast<_Float16*>(p.C)[(int64_t)row * p.ldc + col] = (_Float16)v;
        } else if constexpr (EPI == EPI_GELU_F16) {
          static_cast<_Float16*>(p.C)[(int64_t)row * p.ldc + col] = (_Float16)gelu_erf(v);
        } else if constexpr (EPI == EPI_RESID_F32) {
          float* c = static_cast<float*>(p.C) + (int64_t)row * p.ldc + col;
          *c = p.R[(int64_t)row * p.ldr + col] + v;
        } else {
          static_cast<float*>(p.C)[(int64_t)row * p.ldc + col] = v;
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
// M <= 64 (decoder steps: one row per utterance). Block = all 64 rows x 16 columns;
// the 4 waves split K and reduce through LDS, so an N = 512 projection still spreads
// over 32 blocks and every weight byte is read once per step (weight-streaming bound).
template <int EPI>
__device__ __forceinline__ void skinny_epilogue(const GemmArgs& p, float (*red)[64][17], int col0,
                                                int M, int N);

template <int EPI>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(GemmArgs p) {
  __shared__ float red[4][64][17];
  const int M = p.M, N = p.N, K = p.K;
  const int col0 = blockIdx.x * 16;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kq = ((K + 3) / 4 + 31) / 32 * 32;  // per-wave K slice, multiple of 32
  const int kbeg = w * kq, kend = min(K, kbeg + kq);
  f32x4 acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) acc[m] = zero_f32x4();
  const int bcol = col0 + (lane & 15);
  const _Float16* wrow = p.W + (int64_t)min(bcol, N - 1) * p.ldw;

  for (int k0 = kbeg; k0 < kend; k0 += 32) {
    const int kk = k0 + 8 * (lane >> 4);
    const bool kok = kk < kend;
    const half8 b = (kok && bcol < N) ? *reinterpret_cast<const half8*>(wrow + kk) : zero_half8();
    half8 a[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int r = m * 16 + (lane & 15);
      a[m] = (kok && r < M) ? *reinterpret_cast<const half8*>(p.A + (int64_t)r * p.lda + kk) : zero_half8();
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = mfma16(a[m], b, acc[m]);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][m * 16 + 4 * (lane >> 4) + r][lane & 15] = acc[m][r];
  __syncthreads();
  skinny_epilogue<EPI>(p, red, col0, M, N);
}

// Shared epilogue of the skinny kernels: thread i -> (row i>>4, col col0 + (i&15)), so
// the 16 lanes of an aligned group hold one row's 16 columns (LayerNorm pieces).
template <int EPI>
__device__ __forceinline__ void skinny_epilogue(const GemmArgs& p, float (*red)[64][17], int col0,
                                                int M, int N) {
  const int tid = threadIdx.x;
  for (int i = tid; i < 64 * 16; i += 256) {
    const int row = i >> 4, c = i & 15, col = col0 + c;
    const bool ok = row < M && col < N;
    float v = red[0][row][c] + red[1][row][c] + red[2][row][c] + red[3][row][c];
    v += (p.bias && ok) ? p.bias[col] : 0.0f;
    if constexpr (EPI == EPI_RESID_F32) {
      const float y = ok ? p.R[(int64_t)row * p.ldr + col] + v : 0.0f;
      if (ok) static_cast<float*>(p.C)[(int64_t)row * p.ldc + col] = y;
      if (p.ln_part) {  // uniform branch: all 16 lanes of the row group take part
        float sm = y;
        sm += __shfl_xor(sm, 1); sm += __shfl_xor(sm, 2);
        sm += __shfl_xor(sm, 4); sm += __shfl_xor(sm, 8);
        const float mu = sm * (1.0f / 16.0f);
        float q = (y - mu) * (y - mu);
        q += __shfl_xor(q, 1); q += __shfl_xor(q, 2);
        q += __shfl_xor(q, 4); q += __shfl_xor(q, 8);
        if (c == 0 && row < M) p.ln_part[(int64_t)row * (N / 16) + col0 / 16] = make_float2(sm, q);
      }
      continue;
    }
    if (!ok) continue;
    if constexpr (EPI == EPI_F16) {
      static_cast<_Float16*>(p.C)[(int64_t)row * p.ldc + col] = (_Float16)v;
    } else if constexpr (EPI == EPI_GELU_F16) {
      static_cast<_Float16*>(p.C)[(int64_t)row * p.ldc + col] = (_Float16)gelu_erf(v);
    } else if constexpr (EPI == EPI_QKV) {
      // q -> C; k, v -> cache rows (row * n_ctx + pos); R/ldr carry the cache pointers
      const int dq = p.qkv_d;
      if (col < dq) {
        static_cast<_Float16*>(p.C)[(int64_t)row * p.ldc + col] = (_Float16)v;
      } else {
        _Float16* cache = col < 2 * dq ? p.kc : p.vc;
        cache[((int64_t)row * p.n_ctx + p.pos) * dq + (col % dq)] = (_Float16)v;
      }
    } else {
      static_cast<float*>(p.C)[(int64_t)row * p.ldc + col] = v;
    }
  }
}

static void launch_skinny(int epi, const GemmArgs& p, hipStream_t s) {
  const int blocks = (p.N + 15) / 16;
  switch (epi) {
    case EPI_F16: gemm_skinny_kernel<EPI_F16><<<blocks, 256, 0, s>>>(p); break;
    case EPI_GELU_F16: gemm_skinny_kernel<EPI_GELU_F16><<<blocks, 256, 0, s>>>(p); break;
    case EPI_RESID_F32: gemm_skinny_kernel<EPI_RESID_F32><<<blocks, 256, 0, s>>>(p); break;
    case EPI_F32: gemm_skinny_kernel<EPI_F32><<<blocks, 256, 0, s>>>(p); break;
    case EPI_QKV: gemm_skinny_kernel<EPI_QKV><<<blocks, 256, 0, s>>>(p); break;
    default: throw Error("bad gemm epilogue");
  }
  JANUS_LAUNCH_CHECK();
}

// ------------------------------------------------------- skinny M + fused LN
// C = epi( LN(x)[M,K] · W[N,K]^T + bias ), M <= 64, x fp32 (the residual stream). The
// row statistics come from the K/16 LayerNorm pieces its producer wrote (SkinnyLnArgs):
// thread (row tid/4, quarter tid%4) combines a quarter of the pieces, four lanes finish
// the row (Chan: M2 = sum M2_i + 16 * sum (mu_i - mean)^2). A fragments are normalised
// on load. Replaces the LayerNorm launch in front of every decoder projection.
template <int EPI>
__global__ __launch_bounds__(256) void gemm_skinny_ln_kernel(SkinnyLnArgs p) {
  __shared__ float red[4][64][17];
  __shared__ float s_mean[64], s_rstd[64];
  const int M = p.M, N = p.N, K = p.K;
  const int col0 = blockIdx.x * 16;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kq = ((K + 3) / 4 + 31) / 32 * 32;
  const int kbeg = w * kq, kend = min(K, kbeg + kq);
  const int bcol = col0 + (lane & 15);
  const _Float16* wrow = p.W + (int64_t)min(bcol, N - 1) * p.ldw;
  // the first weight fragment does not depend on the statistics: start it now
  half8 b_next = (kbeg + 8 * (lane >> 4) < kend && bcol < N)
                     ? *reinterpret_cast<const half8*>(wrow + kbeg + 8 * (lane >> 4)) : zero_half8();
  {
    const int r = tid >> 2, qd = tid & 3, np = K / 16;
    float2 pc[8];
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int g = qd + 4 * j;
      pc[j] = (r < M && g < np) ? p.part[(int64_t)r * np + g] : make_float2(0.f, 0.f);
      sm += pc[j].x;
    }
    for (int g = qd + 32; g < np; g += 4) sm += (r < M) ? p.part[(int64_t)r * np + g].x : 0.f;
    sm += __shfl_xor(sm, 1);
    sm += __shfl_xor(sm, 2);
    const float mean = sm / K;
    float m2 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int g = qd + 4 * j;
      if (g < np) {
        const float dm = pc[j].x * (1.0f / 16.0f) - mean;
        m2 += pc[j].y + 16.0f * dm * dm;
      }
    }
    for (int g = qd + 32; g < np; g += 4) {
      const float2 q = (r < M) ? p.part[(int64_t)r * np + g] : make_float2(0.f, 0.f);
      const float dm = q.x * (1.0f / 16.0f) - mean;
      m2 += q.y + 16.0f * dm * dm;
    }
    m2 += __shfl_xor(m2, 1);
    m2 += __shfl_xor(m2, 2);
    if (qd == 0) { s_mean[r] = mean; s_rstd[r] = rsqrtf(m2 / K + p.eps); }
  }
  __syncthreads();
  f32x4 acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) acc[m] = zero_f32x4();
  for (int k0 = kbeg; k0 < kend; k0 += 32) {
    const int kk = k0 + 8 * (lane >> 4);
    const bool kok = kk < kend;
    const half8 b = b_next;
    const int kn = kk + 32;
    b_next = (kn < kend && bcol < N) ? *reinterpret_cast<const half8*>(wrow + kn) : zero_half8();
    float g[8], be[8];
    if (kok) {
      const float4 g0 = *reinterpret_cast<const float4*>(p.gamma + kk);
      const float4 g1 = *reinterpret_cast<const float4*>(p.gamma + kk + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(p.beta + kk);
      const float4 b1 = *reinterpret_cast<const float4*>(p.beta + kk + 4);
      g[0] = g0.x; g[1] = g0.y; g[2] = g0.z; g[3] = g0.w; g[4] = g1.x; g[5] = g1.y; g[6] = g1.z; g[7] = g1.w;
      be[0] = b0.x; be[1] = b0.y; be[2] = b0.z; be[3] = b0.w; be[4] = b1.x; be[5] = b1.y; be[6] = b1.z; be[7] = b1.w;
    }
    half8 a[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int r = m * 16 + (lane & 15);
      a[m] = zero_half8();
      if (kok && r < M) {
        const float* xr = p.x + (int64_t)r * p.ldx + kk;
        const float4 x0 = *reinterpret_cast<const float4*>(xr);
        const float4 x1 = *reinterpret_cast<const float4*>(xr + 4);
        const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const float mean = s_mean[r], rstd = s_rstd[r];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[m][j] = (_Float16)((xv[j] - mean) * rstd * g[j] + be[j]);
      }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = mfma16(a[m], b, acc[m]);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][m * 16 + 4 * (lane >> 4) + r][lane & 15] = acc[m][r];
  __syncthreads();
  GemmArgs q{};
  q.bias = p.bias; q.C = p.C; q.ldc = p.ldc;
  q.kc = p.kc; q.vc = p.vc; q.pos = p.pos; q.n_ctx = p.n_ctx; q.qkv_d = p.qkv_d;
  skinny_epilogue<EPI>(q, red, col0, M, N);
}

void gemm_skinny_ln_launch(int epi, const SkinnyLnArgs& p, hipStream_t s) {
  JANUS_CHECK(p.M <= 64 && p.K % 16 == 0 && p.K <= 2048 && p.ldx % 4 == 0 && p.part,
              "skinny LN gemm: M <= 64, K % 16 == 0, K <= 2048, LayerNorm pieces required");
  if (p.M <= 0 || p.N <= 0) return;
  const int blocks = (p.N + 15) / 16;
  switch (epi) {
    case EPI_F16: gemm_skinny_ln_kernel<EPI_F16><<<blocks, 256, 0, s>>>(p); break;
    case EPI_GELU_F16: gemm_skinny_ln_kernel<EPI_GELU_F16><<<blocks, 256, 0, s>>>(p); break;
    case EPI_QKV: gemm_skinny_ln_kernel<EPI_QKV><<<blocks, 256, 0, s>>>(p); break;
    default: throw Error("skinny LN gemm: bad epilogue");
  }
  JANUS_LAUNCH_CHECK();
}

void gemm_launch(int epi, const GemmArgs& p, hipStream_t s) {
  JANUS_CHECK(p.K % 8 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0, "gemm: K/lda/ldw must be multiples of 8");
  JANUS_CHECK(((uintptr_t)p.A & 15) == 0 && ((uintptr_t)p.W & 15) == 0, "gemm: A/W must be 16-byte aligned");
  if (p.M <= 0 || p.N <= 0) return;
  JANUS_CHECK(p.M <= 64 || (epi != EPI_QKV && !p.ln_part),
              "gemm: the KV-cache and LayerNorm-piece epilogues need M <= 64");
  JANUS_CHECK(!p.ln_part || (epi == EPI_RESID_F32 && p.N % 16 == 0),
              "gemm: LayerNorm pieces come from a RESID epilogue with N % 16 == 0");
  if (p.M <= 64) launch_skinny(epi, p, s);
  else launch_cfg<128, 128, 4, 4>(epi, p, s);
}

}  // namespace janus

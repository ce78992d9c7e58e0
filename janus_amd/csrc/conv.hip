// Implicit-GEMM 1-D convolution / transposed convolution on MFMA (fp16 in, fp32 acc).
//
// Used by the Whisper encoder stem (conv1 80->d k3 p1 + GELU; conv2 d->d k3 s2 p1 +
// GELU + positional embedding) and by every layer of the Firefly-GAN generator
// (conv_pre k13, ConvTranspose upsamplers, residual dilated ResBlock1 convs with
// fused pre-SiLU, post-SiLU, residual add and the ParallelBlock 1/3-mean).
//
// Layout: activations are time-major [B][T][C] fp16, so output row t of a conv is a
// GEMM row whose K = taps x Cin operand is the same input tile shifted by tap*dil
// rows. A block stages an input tile of (BM-1)*stride + (taps-1)*|dil| + 1 rows x CK
// channels in LDS ONCE per channel chunk and every tap reads it at a row offset (no
// im2col in HBM). Weights are pre-packed into contiguous [BN x 64] k-blocks
// (chunk, tap-group) and double-buffered in LDS. Pre-activation (SiLU) is applied
// while staging; bias, post-activation, residual and scaled accumulation in the
// epilogue. ConvTranspose1d(stride u, kernel 2u) runs as u phases of a 2-tap conv.
// Roofline: MFMA-bound for C >= 64; HBM-bound for the 16/32-channel tail stages.
#include <cstdlib>
#include "mfma.h"
#include "kernels.h"

namespace janus {

constexpr int kConvKB = 64;  // K per k-block (two 16x16x32 MFMA k-steps)

ConvPack conv_pack_geometry(int Cin, int Cout, int taps) {
  ConvPack g;
  g.ck = (Cin % 64 == 0) ? 64 : (Cin % 32 == 0) ? 32 : 16;
  g.kb = kConvKB;
  const int tpg = g.kb / g.ck;
  g.chunks = Cin / g.ck;
  g.groups = (taps + tpg - 1) / tpg;
  g.phase_elems = (int64_t)g.chunks * g.groups * Cout * g.kb;
  return g;
}

__global__ void conv_pack_kernel(const float* __restrict__ w, _Float16* __restrict__ packed, int Cin,
                                 int Cout, int taps, int transposed, int u, int ck, int chunks,
                                 int groups, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int kb = kConvKB, tpg = kb / ck;
  int64_t t = idx;
  const int kk = (int)(t % kb); t /= kb;
  const int co = (int)(t % Cout); t /= Cout;
  const int g = (int)(t % groups); t /= groups;
  const int c = (int)(t % chunks); t /= chunks;
  const int ph = (int)t;
  const int tap = g * tpg + kk / ck;
  const int ci = c * ck + kk % ck;
  float v = 0.0f;
  if (tap < taps) {
    if (!transposed) {
      v = w[((int64_t)co * Cin + ci) * taps + tap];
    } else {
      // ConvTranspose1d weight [Cin][Cout][2u]; phase ph uses kernel index ph (input q)
      // and ph + u (input q - 1).
      const int j = tap == 0 ? ph : ph + u;
      v = w[((int64_t)ci * Cout + co) * (2 * u) + j];
    }
  }
  packed[idx] = (_Float16)v;
}

void conv_pack_weights(const float* w, _Float16* packed, int Cin, int Cout, int taps,
                       int transposed, int u, hipStream_t s) {
  const int real_taps = transposed ? 2 : taps;
  const int phases = transposed ? u : 1;
  const ConvPack g = conv_pack_geometry(Cin, Cout, real_taps);
  const int64_t total = g.phase_elems * phases;
  conv_pack_kernel<<<(unsigned)cdiv(total, 256), 256, 0, s>>>(w, packed, Cin, Cout, real_taps,
                                                               transposed, u, g.ck, g.chunks,
                                                               g.groups, total);
  JANUS_LAUNCH_CHECK();
}

template <int ACT>
__device__ __forceinline__ float act_apply(float x) {
  if constexpr (ACT == ACT_SILU) return silu(x);
  else if constexpr (ACT == ACT_GELU) return gelu_erf(x);
  else if constexpr (ACT == ACT_TANH) return tanhf(x);
  else return x;
}


// PRE / POST: compile-time activations (ACT_*), so staging and epilogue carry no
// per-element dispatch.
template <int BM, int BN, int WMT, int WNT, int CK, int PRE, int POST>
__global__ __launch_bounds__(256) void conv_kernel(ConvArgs a, int rows_max) {
  constexpr int KB = kConvKB, TPG = KB / CK;
  constexpr int LI = frag_pitch(CK);   // input row stride in halves (conflict-free b128)
  constexpr int LW = frag_pitch(KB);   // weight row stride
  constexpr int WN = BN / (16 * WNT);
  static_assert((BM / (16 * WMT)) * WN == 4, "4 waves");
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  _Float16* sIn = smem;
  _Float16* sW = smem + rows_max * LI;  // [2][BN][LW]

  const int nbn = (a.Cout + BN - 1) / BN, nbm = (a.n_rows + BM - 1) / BM;
  // tile order (a.remap): 3 = phase-fastest XCD runs (below); 2 = XCD-aware over the whole grid (blocks are dealt to XCDs in
  // linear order, x fastest: each XCD gets a contiguous run of (utterance, phase,
  // row-block) tiles); 1 = over blockIdx.x only; 0 = dispatch order
  const int gx = gridDim.x, gxy = gx * gridDim.y;
  int bid = blockIdx.x, ph = blockIdx.y, b = blockIdx.z;
  if (a.remap == 2) {
    const int lin = xcd_remap(blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z), gxy * gridDim.z);
    bid = lin % gx;
    ph = (lin / gx) % gridDim.y;
    b = lin / gxy;
  } else if (a.remap == 3) {  // as 2 with the phases of one row block adjacent (they
                              // read the same input rows)
    const int lin = xcd_remap(blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z), gxy * gridDim.z);
    ph = lin % gridDim.y;
    bid = (lin / gridDim.y) % gx;
    b = lin / gxy;
  } else if (a.remap == 1) {
    bid = xcd_remap(blockIdx.x, gx);
  }
  const int bm = bid / nbn, bn = bid % nbn;
  const int r0 = bm * BM, co0 = bn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = wave_id();
  const int wm = wid / WN, wn = wid % WN;

  const int lo_tap = min(0, (a.taps - 1) * a.dil);
  const int row_base = r0 * a.in_stride + a.in_off + lo_tap;   // global input row of LDS row 0
  // rows staged: every tap of every k-group, including the zero-weight padding taps of
  // the last group (TPG > 1), so fragment reads need no per-tap guard (host checks that
  // transposed convs, dil < 0, have no padding taps)
  const int nrows = (BM - 1) * a.in_stride +
                    abs(((a.taps + TPG - 1) / TPG * TPG - 1) * a.dil) + 1;
  const int chunks = a.Cin / CK, groups = (a.taps + TPG - 1) / TPG;
  const _Float16* inb = a.in + (int64_t)b * a.in_bs;
  const _Float16* wph = a.w + (int64_t)ph * chunks * groups * a.Cout * KB;

  constexpr int W_CH = (BN * KB / 8 + 255) / 256;
  uint4 rw[W_CH];
  auto wload = [&](int c, int g) {
    const _Float16* src = wph + ((int64_t)(c * groups + g) * a.Cout + co0) * KB;
#pragma unroll
    for (int k = 0; k < W_CH; ++k) {
      const int idx = tid + k * 256;
      const int row = idx / (KB / 8), cc = idx % (KB / 8);
      rw[k] = (idx < BN * KB / 8 && co0 + row < a.Cout)
                  ? *reinterpret_cast<const uint4*>(src + (int64_t)row * KB + cc * 8)
                  : make_uint4(0, 0, 0, 0);
    }
  };
  auto wstore = [&](int buf) {
    _Float16* dst = sW + buf * BN * LW;
#pragma unroll
    for (int k = 0; k < W_CH; ++k) {
      const int idx = tid + k * 256;
      if (idx < BN * KB / 8) {
        const int row = idx / (KB / 8), cc = idx % (KB / 8);
        *reinterpret_cast<uint4*>(dst + row * LW + cc * 8) = rw[k];
      }
    }
  };
  // Input staging: every thread issues all of its loads for a channel chunk before any
  // LDS store (NLD 16-byte loads in flight), so one HBM latency is paid per chunk instead
  // of one per row group. With several chunks the next chunk's rows are loaded into
  // registers while the current chunk computes.
  constexpr int PER_ROW = CK / 8;
  constexpr int NLD = ((BM + 64) * PER_ROW + 255) / 256;
  const bool batched = nrows * PER_ROW <= NLD * 256;
  uint4 pf[NLD];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / PER_ROW, cc = idx % PER_ROW;
      const int gr = row_base + row;
      pf[i] = (row < nrows && gr >= 0 && gr < a.T_in)
                  ? ld_act(inb + (int64_t)gr * a.Cin + c * CK + cc * 8)
                  : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / PER_ROW, cc = idx % PER_ROW;
      if (row < nrows) {
        uint4 v = pf[i];
        if constexpr (PRE != ACT_NONE) {
          _Float16* hv = reinterpret_cast<_Float16*>(&v);
#pragma unroll
          for (int j = 0; j < 8; ++j) hv[j] = (_Float16)act_apply<PRE>((float)hv[j]);
        }
        *reinterpret_cast<uint4*>(sIn + row * LI + cc * 8) = v;
      }
    }
  };
  auto stage_input = [&](int c) {
    const int per_row = CK / 8;
    for (int idx = tid; idx < nrows * per_row; idx += 256) {
      const int row = idx / per_row, cc = idx % per_row;
      const int gr = row_base + row;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gr >= 0 && gr < a.T_in) {
        v = ld_act(inb + (int64_t)gr * a.Cin + c * CK + cc * 8);
        if constexpr (PRE != ACT_NONE) {
          _Float16* hv = reinterpret_cast<_Float16*>(&v);
#pragma unroll
          for (int j = 0; j < 8; ++j) hv[j] = (_Float16)act_apply<PRE>((float)hv[j]);
        }
      }
      *reinterpret_cast<uint4*>(sIn + row * LI + cc * 8) = v;
    }
  };

  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int m = 0; m < WMT; ++m)
#pragma unroll
    for (int n = 0; n < WNT; ++n) acc[m][n] = zero_f32x4();

  // per-thread fragment addressing (lane -> row lane&15, k chunk 8*(lane>>4))
  const int kq = 8 * (lane >> 4);
  const int a_mstep = a.in_stride * LI;                              // one output row
  const int a_off = (wm * WMT * 16 + (lane & 15)) * a_mstep;
  const int b_off = (wn * WNT * 16 + (lane & 15)) * LW;
  const int nkb = chunks * groups;
  if (batched) load_chunk(0);
  wload(0, 0);
  wstore(0);
  for (int kbi = 0; kbi < nkb; ++kbi) {
    const int c = kbi / groups, g = kbi % groups;
    if (g == 0) {
      __syncthreads();  // previous chunk's input tile fully consumed
      if (batched) store_chunk();
      else stage_input(c);
    }
    __syncthreads();    // input tile + weights[kbi&1] visible
    if (batched && g == 0 && c + 1 < chunks) load_chunk(c + 1);  // lands during this chunk
    if (kbi + 1 < nkb) wload((kbi + 1) / groups, (kbi + 1) % groups);
    const _Float16* w_cur = sW + (kbi & 1) * BN * LW + b_off;
#pragma unroll
    for (int ks = 0; ks < KB / 32; ++ks) {
      const int kk = ks * 32 + kq;
      const int tap = g * TPG + kk / CK;
      const _Float16* ap = sIn + a_off + (tap * a.dil - lo_tap) * LI + kk % CK;
      half8 av[WMT], bv[WNT];
#pragma unroll
      for (int m = 0; m < WMT; ++m)
        av[m] = *reinterpret_cast<const half8*>(ap + m * 16 * a_mstep);
#pragma unroll
      for (int n = 0; n < WNT; ++n)
        bv[n] = *reinterpret_cast<const half8*>(w_cur + n * 16 * LW + kk);
#pragma unroll
      for (int m = 0; m < WMT; ++m)
#pragma unroll
        for (int n = 0; n < WNT; ++n) acc[m][n] = mfma16(av[m], bv[n], acc[m][n]);
    }
    if (kbi + 1 < nkb) wstore((kbi + 1) & 1);
  }

  // epilogue: bias + post-activation into an fp32 LDS tile (reusing the staging
  // buffers), then every thread moves 16-byte row chunks: residual and accumulate reads
  // and the fp16 store are full-width, coalesced accesses.
  constexpr int ES = BN + 4;  // fp32 row stride
  float* sE = reinterpret_cast<float*>(smem);
  __syncthreads();
#pragma unroll
  for (int n = 0; n < WNT; ++n) {
    const int cl = wn * WNT * 16 + n * 16 + (lane & 15);
    const int co = co0 + cl;
    const float bias = (a.bias && co < a.Cout) ? a.bias[co] : 0.0f;
#pragma unroll
    for (int m = 0; m < WMT; ++m)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int rl = wm * WMT * 16 + m * 16 + (lane >> 4) * 4 + rr;
        sE[rl * ES + cl] = act_apply<POST>(acc[m][n][rr] + bias);
      }
  }
  __syncthreads();
  _Float16* outb = a.out + (int64_t)b * a.out_bs;
  const _Float16* resb = a.res ? a.res + (int64_t)b * a.res_bs : nullptr;
  constexpr int CPR = BN / 8;  // 16-byte chunks per tile row
  constexpr int NE = BM * CPR / 256;
  static_assert(BM * CPR % 256 == 0, "epilogue chunks");
  // all residual / accumulate loads of the thread first (one latency), then the math
  uint4 rq[NE], pq[NE];
  int64_t oo[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int idx = tid + i * 256;
    const int rl = idx / CPR, cg = (idx % CPR) * 8;
    const int r = r0 + rl, co = co0 + cg;
    const int t = r * a.out_stride + a.out_off + ph;
    const bool ok = r < a.n_rows && co < a.Cout && t >= 0 && t < a.T_out;
    oo[i] = ok ? (int64_t)t * a.Cout + co : -1;
    rq[i] = (ok && resb) ? ld_res(resb + oo[i]) : make_uint4(0, 0, 0, 0);
    pq[i] = (ok && a.accumulate) ? ld_res(outb + oo[i])
                                 : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    if (oo[i] < 0) continue;
    const int idx = tid + i * 256;
    const int rl = idx / CPR, cg = (idx % CPR) * 8;
    const float4 v0 = *reinterpret_cast<const float4*>(sE + rl * ES + cg);
    const float4 v1 = *reinterpret_cast<const float4*>(sE + rl * ES + cg + 4);
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const half8 rv = *reinterpret_cast<const half8*>(&rq[i]);
    const half8 pv = *reinterpret_cast<const half8*>(&pq[i]);
    half8 hv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // y = scale * (conv + res) (+ out): res/pv are zero when absent
      hv[j] = (_Float16)((v[j] + (float)rv[j]) * a.out_scale + (float)pv[j]);
    }
    if (a.post_acc_silu) {  // block-uniform
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[j] = (_Float16)silu((v[j] + (float)rv[j]) * a.out_scale + (float)pv[j]);
    }
    st_act(outb + oo[i], hv);
  }
}

template <int BM, int BN, int WMT, int WNT, int CK, int PRE, int POST>
static void conv_cfg(const ConvArgs& a, hipStream_t s) {
  constexpr int LI = frag_pitch(CK), LW = frag_pitch(kConvKB);
  constexpr int TPG = kConvKB / CK;
  const int taps_padded = (a.taps + TPG - 1) / TPG * TPG;
  JANUS_CHECK(a.dil > 0 || taps_padded == a.taps,
              "conv: transposed conv with padding taps (Cin % 32 != 0) unsupported");
  const int rows_max = (BM - 1) * a.in_stride + std::abs((taps_padded - 1) * a.dil) + 1;
  const size_t lds_loop = (size_t)rows_max * LI * 2 + 2 * (size_t)BN * LW * 2;
  const size_t lds_epi = (size_t)BM * (BN + 4) * 4;
  const size_t lds = lds_loop > lds_epi ? lds_loop : lds_epi;
  JANUS_CHECK(lds <= 160 * 1024, "conv: LDS tile too large (" + std::to_string(lds) + " B)");
  const int blocks = (int)(cdiv(a.n_rows, BM) * cdiv(a.Cout, BN));
  auto kern = conv_kernel<BM, BN, WMT, WNT, CK, PRE, POST>;
  static bool attr_set = false;
  if (!attr_set) {
    JANUS_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
    attr_set = true;
  }
  kern<<<dim3(blocks, a.phases, a.B), 256, lds, s>>>(a, rows_max);
  JANUS_LAUNCH_CHECK();
}

template <int BM, int BN, int WMT, int WNT, int CK>
static void conv_act(const ConvArgs& a, hipStream_t s) {
  // the (pre, post) pairs the Whisper stem and the Firefly-GAN generator use
  if (a.pre_act == ACT_NONE && a.post_act == ACT_NONE) conv_cfg<BM, BN, WMT, WNT, CK, ACT_NONE, ACT_NONE>(a, s);
  else if (a.pre_act == ACT_SILU && a.post_act == ACT_NONE) conv_cfg<BM, BN, WMT, WNT, CK, ACT_SILU, ACT_NONE>(a, s);
  else if (a.pre_act == ACT_NONE && a.post_act == ACT_SILU) conv_cfg<BM, BN, WMT, WNT, CK, ACT_NONE, ACT_SILU>(a, s);
  else if (a.pre_act == ACT_SILU && a.post_act == ACT_SILU) conv_cfg<BM, BN, WMT, WNT, CK, ACT_SILU, ACT_SILU>(a, s);
  else if (a.pre_act == ACT_NONE && a.post_act == ACT_GELU) conv_cfg<BM, BN, WMT, WNT, CK, ACT_NONE, ACT_GELU>(a, s);
  else throw Error("conv: unsupported (pre_act, post_act) = (" + std::to_string(a.pre_act) + ", " +
                   std::to_string(a.post_act) + ")");
}

template <int BM, int BN, int WMT, int WNT>
static void conv_ck(const ConvArgs& a, hipStream_t s) {
  const ConvPack g = conv_pack_geometry(a.Cin, a.Cout, a.taps);
  if (g.ck == 64) conv_act<BM, BN, WMT, WNT, 64>(a, s);
  else if (g.ck == 32) conv_act<BM, BN, WMT, WNT, 32>(a, s);
  else conv_act<BM, BN, WMT, WNT, 16>(a, s);
}

void conv_launch(const ConvArgs& args, hipStream_t s) {
  // tile order: phase-fastest XCD runs (3) fetch 1.21x the algorithmic bytes against
  // 1.84x for runs of row blocks per phase (1): the u phases of an upsampler read the same
  // input rows; in the overlapped step 3 costs ~0.9 ms of conv time against 1 (19.9 vs
  // 19.0 ms), at equal step time. JANUS_CONV_REMAP overrides
  static const int remap_env = ab_env("JANUS_CONV_REMAP") ? std::atoi(ab_env("JANUS_CONV_REMAP")) : 3;
  ConvArgs a = args;
  if (a.remap < 0) a.remap = remap_env;
  JANUS_CHECK(a.Cin % 16 == 0, "conv: Cin must be a multiple of 16");
  JANUS_CHECK(a.Cout % 16 == 0, "conv: Cout must be a multiple of 16");
  JANUS_CHECK(a.in_stride >= 1 && a.taps >= 1 && a.phases >= 1, "conv: bad geometry");
  if (a.B <= 0 || a.n_rows <= 0) return;
  if (a.Cout >= 128) conv_ck<128, 128, 4, 4>(a, s);
  else if (a.Cout == 64) conv_ck<256, 64, 4, 4>(a, s);
  else if (a.Cout == 32) conv_ck<256, 32, 4, 2>(a, s);
  else if (a.Cout == 16) conv_ck<256, 16, 4, 1>(a, s);
  else throw Error("conv: unsupported Cout " + std::to_string(a.Cout));
}

}  // namespace janus

// Kernel-level C-ABI (include/janus_kernels.h): thin wrappers over the launchers.
#include "kernels.h"
#include "decoder.h"
#include "../../include/janus_kernels.h"

namespace janus {

// Shared by janus_conv1d_f16 and the vocoder: PyTorch conv hyper-parameters ->
// the implicit-GEMM row mapping of ConvArgs.
ConvArgs conv_args_torch(const _Float16* in, int B, int T_in, int Cin, const _Float16* packed,
                         const float* bias, _Float16* out, int T_out, int Cout, int taps,
                         int stride, int padding, int dilation, int transposed, int pre_act,
                         int post_act, const _Float16* res, int64_t res_bs, float scale,
                         int accumulate) {
  ConvArgs a{};
  a.in = in; a.in_bs = (int64_t)T_in * Cin; a.T_in = T_in; a.Cin = Cin;
  a.w = packed; a.bias = bias;
  a.out = out; a.out_bs = (int64_t)T_out * Cout; a.T_out = T_out; a.Cout = Cout;
  a.res = res; a.res_bs = res_bs;
  a.pre_act = pre_act; a.post_act = post_act; a.out_scale = scale; a.accumulate = accumulate;
  a.B = B;
  if (!transposed) {
    a.taps = taps; a.dil = dilation; a.in_stride = stride; a.in_off = -padding;
    a.out_stride = 1; a.out_off = 0; a.n_rows = T_out; a.phases = 1;
  } else {
    // ConvTranspose1d(k = 2u, stride u, padding p): output t = q*u + ph - p reads input
    // rows q (kernel index ph) and q-1 (kernel index ph+u).
    const int u = stride;
    a.taps = 2; a.dil = -1; a.in_stride = 1; a.in_off = 0;
    a.out_stride = u; a.out_off = -padding; a.phases = u;
    a.n_rows = (T_out + padding) / u + 1;
  }
  return a;
}

}  // namespace janus

using namespace janus;

extern "C" int janus_gemm_f16(int epi, const uint16_t* A, int64_t lda, const uint16_t* W,
                              int64_t ldw, const float* bias, void* C, int64_t ldc, const float* R,
                              int64_t ldr, int M, int N, int K, void* stream) {
  return guarded([&] {
    GemmArgs g;
    g.A = reinterpret_cast<const _Float16*>(A); g.lda = lda;
    g.W = reinterpret_cast<const _Float16*>(W); g.ldw = ldw;
    g.bias = bias; g.C = C; g.ldc = ldc; g.R = R; g.ldr = ldr; g.M = M; g.N = N; g.K = K;
    gemm_launch(epi, g, (hipStream_t)stream);
  });
}

extern "C" int janus_gemm_nt128_f16(int epi, const uint16_t* A, int64_t lda, const uint16_t* W,
                                    int64_t ldw, const float* bias, void* C, int64_t ldc,
                                    const float* R, int64_t ldr, int M, int N, int K, void* stream) {
  return guarded([&] {
    GemmArgs g;
    g.A = reinterpret_cast<const _Float16*>(A); g.lda = lda;
    g.W = reinterpret_cast<const _Float16*>(W); g.ldw = ldw;
    g.bias = bias; g.C = C; g.ldc = ldc; g.R = R; g.ldr = ldr; g.M = M; g.N = N; g.K = K;
    gemm_nt128_launch(epi, g, (hipStream_t)stream);
  });
}

extern "C" int janus_gemm_lt_f16(int epi, const uint16_t* A, int64_t lda, const uint16_t* W,
                                 int64_t ldw, const float* bias, void* C, int64_t ldc,
                                 const float* R, int64_t ldr, int M, int N, int K, void* stream) {
  return guarded([&] {
    GemmArgs g;
    g.A = reinterpret_cast<const _Float16*>(A); g.lda = lda;
    g.W = reinterpret_cast<const _Float16*>(W); g.ldw = ldw;
    g.bias = bias; g.C = C; g.ldc = ldc; g.R = R; g.ldr = ldr; g.M = M; g.N = N; g.K = K;
    JANUS_CHECK(gemm_lt_launch(epi, g, (hipStream_t)stream),
                "gemm_lt: no hipBLASLt plan for this shape / epilogue");
  });
}

extern "C" int janus_gemm_ln_f16(int epi, const float* x, int64_t ldx, const float* gamma,
                                 const float* beta, float eps, const uint16_t* W, int64_t ldw,
                                 const float* bias, void* C, int64_t ldc, int M, int N, int K,
                                 void* stream) {
  return guarded([&] {
    JANUS_CHECK(M <= 64 && K <= 512 && K % 32 == 0, "gemm_ln: M <= 64, K <= 512 (multiple of 32)");
    GemmArgs g;
    g.A = nullptr; g.lda = K; g.R = nullptr; g.ldr = 0;
    g.W = reinterpret_cast<const _Float16*>(W); g.ldw = ldw;
    g.bias = bias; g.C = C; g.ldc = ldc; g.M = M; g.N = N; g.K = K;
    g.lnin_x = x; g.lnin_ldx = ldx; g.lnin_g = gamma; g.lnin_b = beta; g.lnin_eps = eps;
    gemm_launch(epi, g, (hipStream_t)stream);
  });
}

extern "C" int janus_resid_ln_f16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                                  const float* bias, float* x, const float* gamma, const float* beta,
                                  float eps, uint16_t* out, int M, int N, int K, void* stream) {
  return guarded([&] {
    JANUS_CHECK(A && W && x && gamma && beta && out, "resid_ln: null argument");
    ResidLnArgs p;
    p.A = reinterpret_cast<const _Float16*>(A); p.lda = lda;
    p.W = reinterpret_cast<const _Float16*>(W); p.ldw = ldw;
    p.bias = bias; p.x = x; p.ldx = N; p.g = gamma; p.b = beta; p.eps = eps;
    p.out = reinterpret_cast<_Float16*>(out); p.M = M; p.N = N; p.K = K;
    resid_ln_launch(p, (hipStream_t)stream);
  });
}

extern "C" int janus_layernorm_f16(const float* x, const float* gamma, const float* beta,
                                   uint16_t* out, int rows, int d, float eps, void* stream) {
  return guarded([&] {
    layernorm_launch(x, gamma, beta, reinterpret_cast<_Float16*>(out), rows, d, eps,
                     (hipStream_t)stream);
  });
}

extern "C" int janus_wave_xor_f32(const float* in, float* out, int n_waves, void* stream) {
  return guarded([&] {
    JANUS_CHECK(in && out, "null argument");
    wave_xor_launch(in, out, n_waves, (hipStream_t)stream);
  });
}

extern "C" int janus_attention_f16(const uint16_t* qkv, uint16_t* out, int batch, int T, int H,
                                   float scale, void* stream) {
  return guarded([&] {
    attention_launch(reinterpret_cast<const _Float16*>(qkv), reinterpret_cast<_Float16*>(out),
                     batch, T, H, scale, (hipStream_t)stream);
  });
}

extern "C" int64_t janus_conv1d_packed_size(int Cin, int Cout, int taps, int transposed,
                                            int stride) {
  const ConvPack g = conv_pack_geometry(Cin, Cout, transposed ? 2 : taps);
  return g.phase_elems * (transposed ? stride : 1);
}

extern "C" int janus_conv1d_pack(const float* w, uint16_t* packed, int Cin, int Cout, int taps,
                                 int transposed, int stride, void* stream) {
  return guarded([&] {
    conv_pack_weights(w, reinterpret_cast<_Float16*>(packed), Cin, Cout, taps, transposed, stride,
                      (hipStream_t)stream);
  });
}

extern "C" int janus_conv1d_f16(const uint16_t* in, int batch, int T_in, int Cin,
                                const uint16_t* packed, const float* bias, uint16_t* out, int T_out,
                                int Cout, int taps, int stride, int padding, int dilation,
                                int transposed, int pre_act, int post_act, const uint16_t* res,
                                int64_t res_bs, float scale, int accumulate, void* stream) {
  return guarded([&] {
    ConvArgs a = conv_args_torch(
        reinterpret_cast<const _Float16*>(in), batch, T_in, Cin,
        reinterpret_cast<const _Float16*>(packed), bias, reinterpret_cast<_Float16*>(out), T_out,
        Cout, taps, stride, padding, dilation, transposed, pre_act, post_act,
        reinterpret_cast<const _Float16*>(res), res_bs, scale, accumulate);
    conv_launch(a, (hipStream_t)stream);
  });
}

extern "C" int janus_resunit_packed_size(int C, int k) { return resunit_kp(C, k) * C; }

extern "C" int janus_resunit_pack(const float* w, uint16_t* packed, int C, int k, void* stream) {
  return guarded([&] {
    resunit_pack(w, reinterpret_cast<_Float16*>(packed), C, k, (hipStream_t)stream);
  });
}

extern "C" int janus_resunit_f16(const uint16_t* x, uint16_t* out, const uint16_t* w1,
                                 const float* b1, const uint16_t* w2, const float* b2, int batch,
                                 int T, int C, int k, int dilation, float scale, int accumulate,
                                 void* stream) {
  return guarded([&] {
    ResUnitArgs a;
    a.x = reinterpret_cast<const _Float16*>(x); a.out = reinterpret_cast<_Float16*>(out);
    a.w1 = reinterpret_cast<const _Float16*>(w1); a.b1 = b1;
    a.w2 = reinterpret_cast<const _Float16*>(w2); a.b2 = b2;
    a.B = batch; a.T = T; a.C = C; a.k = k; a.d = dilation; a.scale = scale;
    a.accumulate = accumulate;
    resunit_launch(a, (hipStream_t)stream);
  });
}

extern "C" int janus_cross_attention_f16(const uint16_t* qk, const uint16_t* enc, int batch,
                                         int Te, int D, int H, int nsplit, float* part_c,
                                         float* part_ml, uint16_t* out, void* stream) {
  return guarded([&] {
    xattn_launch(reinterpret_cast<const _Float16*>(qk), reinterpret_cast<const _Float16*>(enc),
                 batch, Te, D, H, nsplit, part_c, part_ml, reinterpret_cast<_Float16*>(out),
                 (hipStream_t)stream);
  });
}

extern "C" int janus_decode_attention_f16(const uint16_t* q, int64_t q_bs, const uint16_t* k,
                                          const uint16_t* v, int64_t kv_bs, int64_t kv_rs,
                                          int Tkv, uint16_t* out, int64_t o_bs, int batch, int H,
                                          float scale, float* part_o, float* part_ml,
                                          void* stream) {
  return guarded([&] {
    JANUS_CHECK(Tkv <= 512 || (part_o && part_ml), "decode attention: scratch needed past 512 keys");
    decode_attention_split_launch(reinterpret_cast<const _Float16*>(q), q_bs,
                                  reinterpret_cast<const _Float16*>(k),
                                  reinterpret_cast<const _Float16*>(v), kv_bs, kv_rs, Tkv,
                                  reinterpret_cast<_Float16*>(out), o_bs, batch, H, scale, part_o,
                                  part_ml, (hipStream_t)stream);
  });
}

extern "C" int janus_sample_gumbel_f32(const uint32_t* seeds, int batch, int pos, int V, float* out,
                                       void* stream) {
  return guarded([&] {
    JANUS_CHECK(seeds && out, "null argument");
    sample_gumbel_launch(seeds, batch, pos, V, out, (hipStream_t)stream);
  });
}

/*
 * janus_kernels.h — kernel-level C-ABI of libjanus_hip.so (gfx950).
 *
 * The building blocks the whisper / vocoder entry points of janus.h are made of,
 * exposed for parity tests and for callers that orchestrate their own graphs. All
 * pointers are [device]; fp16 tensors are uint16_t (binary16 bits); all calls are
 * asynchronous on `stream`. Return 0 on success (janus_last_error() otherwise).
 */
#ifndef JANUS_KERNELS_H_
#define JANUS_KERNELS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Epilogues of janus_gemm_f16 */
enum { JANUS_EPI_F16 = 0, JANUS_EPI_GELU_F16 = 1, JANUS_EPI_RESID_F32 = 2, JANUS_EPI_F32 = 3 };
/* Activations of janus_conv1d_f16 */
enum { JANUS_ACT_NONE = 0, JANUS_ACT_SILU = 1, JANUS_ACT_GELU = 2, JANUS_ACT_TANH = 3 };

/*
 * C[M,N] = epi(A[M,K] · W[N,K]^T + bias[N]); A, W fp16 (K contiguous, K % 8 == 0);
 * C fp16 or fp32 by epilogue; JANUS_EPI_RESID_F32: C = R + (A·W^T + bias) in fp32.
 * Replaces the dense projections inside CTranslate2's Whisper (transcriber.py:23-27).
 */
int janus_gemm_f16(int epi, const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                   const float* bias, void* C, int64_t ldc, const float* R, int64_t ldr, int M,
                   int N, int K, void* stream);

/* The same product on the general 128 x 128-tile kernel (any N, K % 8 == 0). janus_gemm_f16
 * dispatches M > 64 products with N % 256 == 0 and K % 64 == 0 to the 256 x 256-tile
 * kernel (gemm_big.hip, the encoder's projections); both accumulate each output over the
 * same k-steps in the same order, so their results are bit-identical. */
int janus_gemm_nt128_f16(int epi, const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                         const float* bias, void* C, int64_t ldc, const float* R, int64_t ldr, int M,
                         int N, int K, void* stream);

/* The same product on hipBLASLt — a comparison point for the hand-written kernels
 * (tools/gemm_big_probe.py); no product path calls it. epi F16 / F32 / RESID_F32 (C == R
 * in place) / GELU_F16 (bias epilogue, then an exact-erf GELU pass); bias required;
 * workspace-free plans only. Error when the library has no such plan for the shape. */
int janus_gemm_lt_f16(int epi, const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                      const float* bias, void* C, int64_t ldc, const float* R, int64_t ldr, int M,
                      int N, int K, void* stream);

/* LayerNorm rows of an fp32 [rows][d] tensor into fp16 (eps as given). */
/* C = epilogue(LayerNorm(x) W^T + bias) for M <= 64 rows: the LayerNorm of each block's
 * rows (fp32 x, row stride ldx; gamma/beta f32 [K]; two-pass fp32 statistics) is computed in
 * the GEMM's prologue instead of a separate janus_layernorm_f16 launch. K <= 512, K % 4 == 0;
 * epi one of EPI_F16 / EPI_GELU_F16. The decoder's pre-LN projections (transcriber.py:53-57
 * -> Whisper decoder layers). */
int janus_gemm_ln_f16(int epi, const float* x, int64_t ldx, const float* gamma, const float* beta,
                      float eps, const uint16_t* W, int64_t ldw, const float* bias, void* C,
                      int64_t ldc, int M, int N, int K, void* stream);
int janus_layernorm_f16(const float* x, const float* gamma, const float* beta, uint16_t* out,
                        int rows, int d, float eps, void* stream);

/* The cross-lane moves every wave reduction of the library uses (DPP / v_permlane swaps in
 * place of ds_bpermute): in [device] f32 [n_waves][64] -> out [device] f32 [n_waves][6][64],
 * out[w][k][l] = in[w][l ^ (1 << k)] when they are right. Test entry. */
int janus_wave_xor_f32(const float* in, float* out, int n_waves, void* stream);

/* x[M][N] += A[M][K] W[N][K]^T + bias (fp32 residual, in place), then out[M][N] =
 * LayerNorm(x) fp16 (gamma/beta f32 [N], eps) in ONE launch: 16 rows per workgroup over
 * all N columns. N = K in {384, 512} (tiny.en / base.en d_model). Bit-identical to
 * janus_gemm_f16(JANUS_EPI_RESID_F32) at M <= 64 followed by janus_layernorm_f16. The
 * decoder's attention output projections and the LayerNorm after them
 * (transcriber.py:53-57 -> Whisper decoder layers: self_attn.out_proj + encoder_attn_layer_norm,
 * encoder_attn.out_proj + final_layer_norm). */
int janus_resid_ln_f16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                       const float* bias, float* x, const float* gamma, const float* beta,
                       float eps, uint16_t* out, int M, int N, int K, void* stream);

/* Non-causal multi-head attention, head_dim 64: qkv fp16 [B*T][3*H*64] -> out fp16 [B*T][H*64]. */
int janus_attention_f16(const uint16_t* qkv, uint16_t* out, int batch, int T, int H, float scale,
                        void* stream);

/* Size in fp16 elements of the packed weight buffer janus_conv1d_pack expects/produces. */
int64_t janus_conv1d_packed_size(int Cin, int Cout, int taps, int transposed, int stride);
/*
 * Pack fp32 PyTorch conv weights for janus_conv1d_f16: Conv1d [Cout][Cin][taps]
 * (transposed=0) or ConvTranspose1d [Cin][Cout][2*stride] (transposed=1).
 */
int janus_conv1d_pack(const float* w, uint16_t* packed, int Cin, int Cout, int taps,
                      int transposed, int stride, void* stream);
/*
 * Time-major 1-D convolution on MFMA: in [B][T_in][Cin], out [B][T_out][Cout] (fp16).
 * transposed=0: PyTorch Conv1d(Cin, Cout, taps, stride, padding, dilation)
 * transposed=1: ConvTranspose1d(Cin, Cout, 2*stride, stride, padding) (taps ignored).
 * y = post_act(conv(pre_act(x)) + bias); y += res (fp16 [B][T_out][Cout], may be NULL,
 * res_bs = batch stride in elements, 0 to broadcast); out = (accumulate ? out : 0) + scale*y.
 * (pre_act, post_act) is one of (NONE, NONE), (SILU, NONE), (SILU, SILU), (NONE, GELU) —
 * the pairs of the Whisper stem and the generator, compiled in; others return an error.
 */
int janus_conv1d_f16(const uint16_t* in, int batch, int T_in, int Cin, const uint16_t* packed,
                     const float* bias, uint16_t* out, int T_out, int Cout, int taps, int stride,
                     int padding, int dilation, int transposed, int pre_act, int post_act,
                     const uint16_t* res, int64_t res_bs, float scale, int accumulate,
                     void* stream);

/*
 * Fused fish-speech ResBlock1 unit for narrow stages (C = 16 or 32, odd k <= 11):
 * out = (accumulate ? out : 0) + scale * (x + c2(silu(c1(silu(x)) + b1)) + b2), with
 * c1 = Conv1d(C, C, k, dilation, padding dilation*(k-1)/2), c2 = Conv1d(C, C, k,
 * padding (k-1)/2); x/out fp16 [B][T][C] (must not alias); weights packed by
 * janus_resunit_pack from PyTorch [C][C][k] fp32 into janus_resunit_packed_size halves.
 */
int janus_resunit_packed_size(int C, int k);
int janus_resunit_pack(const float* w, uint16_t* packed, int C, int k, void* stream);
int janus_resunit_f16(const uint16_t* x, uint16_t* out, const uint16_t* w1, const float* b1,
                      const uint16_t* w2, const float* b2, int batch, int T, int C, int k,
                      int dilation, float scale, int accumulate, void* stream);

/*
 * Decoder cross-attention over the encoder output with absorbed K/V projections:
 * for every utterance b and head h (H * 64 == D, D in {384, 512, 768}),
 *   p = softmax_2(qk[b][h] . enc[b]^T)   (base-2 softmax: qk carries log2(e)/8),
 *   out[b][h*D:(h+1)*D] = p . enc[b]
 * qk fp16 [B][H*D], enc fp16 [B][Te][D], out fp16 [B][H*D]; nsplit key splits
 * (1..63) with scratch part_c f32 [B][nsplit][H][D] and part_ml f32 [B][nsplit][H][2].
 * Replaces the cross-attention K/V projections + attention of the Whisper decoder
 * (transcriber.py:23-27); see janus_amd/csrc/xattn.hip for the re-association.
 */
int janus_cross_attention_f16(const uint16_t* qk, const uint16_t* enc, int batch, int Te, int D,
                              int H, int nsplit, float* part_c, float* part_ml, uint16_t* out,
                              void* stream);

/* Decoder self-attention, one query per (utterance, head) against a KV cache:
 *   out[b][h*64:(h+1)*64] = softmax(q_h . K_h[0:Tkv]^T * scale) . V_h[0:Tkv]
 * q fp16 rows of stride q_bs; k/v fp16 [B][>=Tkv][H*64] with batch stride kv_bs and row
 * stride kv_rs (elements); out fp16 rows of stride o_bs. Tkv <= 512 runs one block per
 * (head, utterance); longer caches split keys over blocks with scratch part_o f32
 * [B][ceil(Tkv/64)][H*64] and part_ml f32 [B][ceil(Tkv/64)][H][2] (may be NULL when
 * Tkv <= 512). The per-step self-attention of the greedy decoder (transcriber.py:53-57
 * -> model.transcribe, CTranslate2 decoder with KV cache). */
int janus_decode_attention_f16(const uint16_t* q, int64_t q_bs, const uint16_t* k,
                               const uint16_t* v, int64_t kv_bs, int64_t kv_rs, int Tkv,
                               uint16_t* out, int64_t o_bs, int batch, int H, float scale,
                               float* part_o, float* part_ml, void* stream);

/* Per segment b of a flat f32 array (offsets[B+1], int64): the count of values > 0 and
 * np.mean of those values in order, numpy float32 bit for bit (float32 pairwise sums over
 * 8192-element buffers, float64 divide by the count, 0 when none). The voiced-f0 mean of
 * janus_prosody_analyze (backend/services/prosody.py:86-90: pitch_values.append(pitch) for
 * pitch > 0, np.mean(pitch_values)) exposed for edge tests. */
int janus_np_voiced_mean_f32(const float* values, const int64_t* offsets, int batch,
                             float* mean_out, int32_t* count_out, void* stream);

/*
 * The decoder's sampling noise (janus_whisper_decode_sample_ex): out [batch][V] f32 =
 * Gumbel(0, 1) draw of token t for row b at position pos, -log(-log u) with u an odd
 * multiple of 2^-24 from a murmur3-finalised hash of (seeds[b] [device uint32], pos, t).
 * Lets tests pin the CPU oracle's noise to the device's.
 */
int janus_sample_gumbel_f32(const uint32_t* seeds, int batch, int pos, int V, float* out,
                            void* stream);

#ifdef __cplusplus
}
#endif
#endif /* JANUS_KERNELS_H_ */

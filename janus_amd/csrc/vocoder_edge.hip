// Vocoder edge kernels: the text+emotion -> latent front end and the fused
// SiLU -> conv_post(16->1, k13) -> tanh -> f32 waveform + int16 PCM tail.
//
// Front end (build-defined; the reference's decode is a cloud call,
// synthesizer.py:191-203): latent[b][f][:] = E_text[prompt_byte(b, f)] + E_emo[emo(b)],
// prompt_byte(b, f) = byte floor(f * n_b / F) of the "(emotion) text" prompt the
// reference sends to Fish (synthesizer.py:151-177); HBM-bound gather.
#include "mfma.h"
#include "kernels.h"
#include "vocoder.h"

namespace janus {

__global__ void frontend_kernel(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ boff,
                                const int32_t* __restrict__ emo, const float* __restrict__ e_text,
                                const float* __restrict__ e_emo, int F, int C,
                                _Float16* __restrict__ lat) {
  const int f = blockIdx.x, b = blockIdx.y;
  const int64_t n = boff[b + 1] - boff[b];
  const float* et = nullptr;
  if (n > 0) {
    const int64_t j = (int64_t)f * n / F;
    et = e_text + (int64_t)bytes[boff[b] + j] * C;
  }
  const float* ee = e_emo + (int64_t)emo[b] * C;
  _Float16* o = lat + ((int64_t)b * F + f) * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) o[c] = (_Float16)((et ? et[c] : 0.0f) + ee[c]);
}

void frontend_launch(const uint8_t* bytes, const int64_t* boff, const int32_t* emo,
                     const float* e_text, const float* e_emo, int B, int F, int C, _Float16* lat,
                     hipStream_t s) {
  if (B <= 0 || F <= 0) return;
  frontend_kernel<<<dim3(F, B), 256, 0, s>>>(bytes, boff, emo, e_text, e_emo, F, C, lat);
  JANUS_LAUNCH_CHECK();
}

// conv_post: y[t] = tanh(b + sum_{c,j} w[c][j] * silu(x[t + j - 6][c])), x fp16 [B][T][16]
// (pre_silu = 0: x already holds silu(x), stored by the last ResBlock unit)
constexpr int kPostC = 16, kPostK = 13, kPostT = 256;

__global__ __launch_bounds__(kPostT) void conv_post_kernel(const _Float16* __restrict__ x, int T,
                                                           const float* __restrict__ w, float bias,
                                                           float* __restrict__ wav,
                                                           int16_t* __restrict__ pcm, int pre_silu) {
  __shared__ float xs[(kPostT + kPostK - 1) * (kPostC + 1)];
  __shared__ float ws[kPostC * kPostK];
  const int b = blockIdx.y, t0 = blockIdx.x * kPostT;
  const _Float16* xb = x + (int64_t)b * T * kPostC;
  for (int i = threadIdx.x; i < kPostC * kPostK; i += kPostT) ws[i] = w[i];
  // stage rows t0-6 .. t0+255+6, 16 channels each (one 32-byte row = 2 x 16 B)
  for (int i = threadIdx.x; i < (kPostT + kPostK - 1) * 2; i += kPostT) {
    const int r = i >> 1, half = i & 1;
    const int t = t0 - kPostK / 2 + r;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t >= 0 && t < T) v = *reinterpret_cast<const uint4*>(xb + (int64_t)t * kPostC + half * 8);
    const _Float16* h = reinterpret_cast<const _Float16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) xs[r * (kPostC + 1) + half * 8 + j] = pre_silu ? silu((float)h[j]) : (float)h[j];
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  float acc = bias;
#pragma unroll
  for (int j = 0; j < kPostK; ++j)
#pragma unroll
    for (int c = 0; c < kPostC; ++c) acc += ws[c * kPostK + j] * xs[(threadIdx.x + j) * (kPostC + 1) + c];
  const float y = tanhf(acc);
  wav[(int64_t)b * T + t] = y;
  if (pcm) {
    float q = rintf(y * 32767.0f);
    q = fminf(fmaxf(q, -32768.0f), 32767.0f);
    pcm[(int64_t)b * T + t] = (int16_t)q;
  }
}

void conv_post_launch(const _Float16* x, int B, int T, const float* w, float bias, float* wav,
                      int16_t* pcm, hipStream_t s, int pre_silu) {
  if (B <= 0 || T <= 0) return;
  conv_post_kernel<<<dim3((T + kPostT - 1) / kPostT, B), kPostT, 0, s>>>(x, T, w, bias, wav, pcm,
                                                                         pre_silu);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

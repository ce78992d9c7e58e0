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
                                const float* __restrict__ e_emo, const float* __restrict__ spk,
                                int F, int C, _Float16* __restrict__ lat) {
  const int f = blockIdx.x, b = blockIdx.y;
  const int64_t n = boff[b + 1] - boff[b];
  const float* et = nullptr;
  if (n > 0) {
    const int64_t j = (int64_t)f * n / F;
    et = e_text + (int64_t)bytes[boff[b] + j] * C;
  }
  const float* ee = e_emo + (int64_t)emo[b] * C;
  const float* sp = spk ? spk + (int64_t)b * C : nullptr;
  _Float16* o = lat + ((int64_t)b * F + f) * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    o[c] = (_Float16)(((et ? et[c] : 0.0f) + ee[c]) + (sp ? sp[c] : 0.0f));
}

void frontend_launch(const uint8_t* bytes, const int64_t* boff, const int32_t* emo,
                     const float* e_text, const float* e_emo, const float* spk, int B, int F, int C,
                     _Float16* lat, hipStream_t s) {
  if (B <= 0 || F <= 0) return;
  frontend_kernel<<<dim3(F, B), 256, 0, s>>>(bytes, boff, emo, e_text, e_emo, spk, F, C, lat);
  JANUS_LAUNCH_CHECK();
}

// Speaker (voice-cloning) conditioning, build-defined: the reference hands its reference
// recording to the cloud TTS as references=[ReferenceAudio(audio, text="")]
// (synthesizer.py:183-200). Locally the recording's Whisper log-mel (mel_kernel, 16 kHz)
// is averaged over the frames that hold audio and projected to the latent width:
//   spk[b][c] = bias[c] + sum_m P[c][m] * mean_f norm(logmel[b][f][m]),
//   norm(v) = (max(v, gmax_b - 8) + 4) / 4  (the encoder's own normalisation).
// One block per clip; HBM/latency-bound (<= 3000 x 80 floats read).
__global__ __launch_bounds__(256) void speaker_kernel(const float* __restrict__ logmel,
                                                      const uint32_t* __restrict__ maxkey,
                                                      const int64_t* __restrict__ offsets,
                                                      int frames, const float* __restrict__ P,
                                                      const float* __restrict__ bias, int C,
                                                      float* __restrict__ spk) {
  constexpr int kM = 80, kPh = 3;  // 240 threads: (frame phase, mel bin)
  __shared__ float part[kPh][kM];
  __shared__ float mean[kM];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int64_t len = offsets[b + 1] - offsets[b];
  const int nf = (int)max((int64_t)1, min((int64_t)frames, (len + 159) / 160));
  const uint32_t k = maxkey[b];
  const float gmax = __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
  if (tid < kPh * kM) {
    const int ph = tid / kM, m = tid % kM;
    float s = 0.f;
    for (int f = ph; f < nf; f += kPh)
      s += (fmaxf(logmel[((int64_t)b * frames + f) * kM + m], gmax - 8.0f) + 4.0f) * 0.25f;
    part[ph][m] = s;
  }
  __syncthreads();
  if (tid < kM) mean[tid] = (part[0][tid] + part[1][tid] + part[2][tid]) / (float)nf;
  __syncthreads();
  for (int c = tid; c < C; c += blockDim.x) {
    float acc = bias ? bias[c] : 0.f;
    const float* pr = P + (int64_t)c * kM;
#pragma unroll 8
    for (int m = 0; m < kM; ++m) acc = fmaf(pr[m], mean[m], acc);
    spk[(int64_t)b * C + c] = acc;
  }
}

void speaker_launch(const float* logmel, const uint32_t* maxkey, const int64_t* offsets, int B,
                    int frames, const float* P, const float* bias, int C, float* spk,
                    hipStream_t s) {
  if (B <= 0) return;
  speaker_kernel<<<B, 256, 0, s>>>(logmel, maxkey, offsets, frames, P, bias, C, spk);
  JANUS_LAUNCH_CHECK();
}

// conv_post: y[t] = tanh(b + sum_{c,j} w[c][j] * silu(x[t + j - 6][c])), x fp16 [B][T][16]
// (pre_silu = 0: x already holds silu(x), stored by the last ResBlock unit).
// A block covers kPostT = 1024 samples of one utterance; the input rows are staged
// channel-major (xs[c][row]) so a thread's 16-row window of one channel is four 16-byte
// LDS reads, shared by its kPostR = 4 consecutive outputs (52 FMAs per channel window);
// the waveform goes out as one float4 and the PCM as one 8-byte store per thread.
constexpr int kPostC = 16, kPostK = 13, kPostR = 4, kPostThreads = 256;
constexpr int kPostT = kPostThreads * kPostR;                   // samples per block
constexpr int kPostRows = kPostT + 16;                          // staged rows (>= T + K - 1), 16-B rows
constexpr size_t kPostLds = (size_t)(kPostC * kPostRows + kPostC * 16) * sizeof(float);

__global__ __launch_bounds__(kPostThreads) void conv_post_kernel(const _Float16* __restrict__ x, int T,
                                                                 const float* __restrict__ w, float bias,
                                                                 float* __restrict__ wav,
                                                                 int16_t* __restrict__ pcm, int pre_silu,
                                                                 float* __restrict__ pre_tanh) {
  extern __shared__ __attribute__((aligned(16))) float post_smem[];
  float* xs = post_smem;                        // [kPostC][kPostRows]
  float* ws = post_smem + kPostC * kPostRows;   // [kPostC][16] (taps padded to 16)
  const int b = blockIdx.y, t0 = blockIdx.x * kPostT, tid = threadIdx.x;
  const _Float16* xb = x + (int64_t)b * T * kPostC;
  // stage rows t0-6 .. t0+kPostT+9 (16 channels = two 16-byte halves per row): every load
  // of the tile in flight before the first convert/store (one memory latency per block;
  // a load-store loop paid one per iteration: 1.9 ms for the 64 x 30 s pass)
  constexpr int NPL = (kPostRows * 2 + kPostThreads - 1) / kPostThreads;
  uint4 pv[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int i = tid + k * kPostThreads;
    const int t = t0 - kPostK / 2 + (i >> 1);
    pv[k] = (i < kPostRows * 2 && t >= 0 && t < T)
                ? ld_act(xb + (int64_t)t * kPostC + (i & 1) * 8)  // non-temporal (mfma.h)
                : make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < kPostC * 16; i += kPostThreads) {
    const int c = i >> 4, j = i & 15;
    ws[i] = j < kPostK ? w[c * kPostK + j] : 0.0f;
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int i = tid + k * kPostThreads;
    if (i >= kPostRows * 2) break;
    const int r = i >> 1, half = i & 1;
    const _Float16* h = reinterpret_cast<const _Float16*>(&pv[k]);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      xs[(half * 8 + j) * kPostRows + r] = pre_silu ? silu((float)h[j]) : (float)h[j];
  }
  __syncthreads();
  float acc[kPostR];
#pragma unroll
  for (int o = 0; o < kPostR; ++o) acc[o] = bias;
#pragma unroll 4
  for (int c = 0; c < kPostC; ++c) {
    float xv[16], wv[16];
    const float4* xr = reinterpret_cast<const float4*>(xs + c * kPostRows + kPostR * tid);
    const float4* wr = reinterpret_cast<const float4*>(ws + c * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a4 = xr[q], w4 = wr[q];
      xv[4 * q] = a4.x; xv[4 * q + 1] = a4.y; xv[4 * q + 2] = a4.z; xv[4 * q + 3] = a4.w;
      wv[4 * q] = w4.x; wv[4 * q + 1] = w4.y; wv[4 * q + 2] = w4.z; wv[4 * q + 3] = w4.w;
    }
#pragma unroll
    for (int j = 0; j < kPostK; ++j)
#pragma unroll
      for (int o = 0; o < kPostR; ++o) acc[o] += wv[j] * xv[o + j];
  }
  const int t = t0 + kPostR * tid;
  float y[kPostR];
  int16_t q16[kPostR];
#pragma unroll
  for (int o = 0; o < kPostR; ++o) {
    y[o] = tanhf(acc[o]);
    const float q = fminf(fmaxf(rintf(y[o] * 32767.0f), -32768.0f), 32767.0f);
    q16[o] = (int16_t)q;
  }
  float* wo = wav + (int64_t)b * T + t;
  int16_t* po = pcm ? pcm + (int64_t)b * T + t : nullptr;
  if (pre_tanh) {  // conv_post output before tanh (parity checks upstream of saturation)
#pragma unroll
    for (int o = 0; o < kPostR; ++o)
      if (t + o < T) pre_tanh[(int64_t)b * T + t + o] = acc[o];
  }
  if (t + kPostR <= T && (T & 3) == 0) {  // aligned full group: vector stores, non-temporal
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef short s4v __attribute__((ext_vector_type(4)));
#ifdef JANUS_ACT_WT
    {
      const f4v yv{y[0], y[1], y[2], y[3]};
      st_wt16(wo, __builtin_bit_cast(u32x4, yv));
      if (po) {
        const s4v qv{q16[0], q16[1], q16[2], q16[3]};
        st_wt8(po, __builtin_bit_cast(u32x2, qv));
      }
    }
#else
    __builtin_nontemporal_store(f4v{y[0], y[1], y[2], y[3]}, reinterpret_cast<f4v*>(wo));
    if (po) __builtin_nontemporal_store(s4v{q16[0], q16[1], q16[2], q16[3]}, reinterpret_cast<s4v*>(po));
#endif
  } else {
#pragma unroll
    for (int o = 0; o < kPostR; ++o) {
      if (t + o < T) {
        wo[o] = y[o];
        if (po) po[o] = q16[o];
      }
    }
  }
}

void conv_post_launch(const _Float16* x, int B, int T, const float* w, float bias, float* wav,
                      int16_t* pcm, hipStream_t s, int pre_silu, float* pre_tanh) {
  if (B <= 0 || T <= 0) return;
  static bool attr = false;
  if (!attr) {
    JANUS_HIP(hipFuncSetAttribute((const void*)conv_post_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPostLds));
    attr = true;
  }
  conv_post_kernel<<<dim3((T + kPostT - 1) / kPostT, B), kPostThreads, kPostLds, s>>>(
      x, T, w, bias, wav, pcm, pre_silu, pre_tanh);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

// Edge kernels of the streaming engine and the receiver:
//
// * duck_pcm16_kernel — the receiver's playback ducking, engine.py:94-134
//   (apply_ducking_if_needed): while the local user talks, int16 playback samples are
//   scaled by ducking_level: np.clip(s.astype(float32) * level, -32768, 32767).astype(int16).
//   Restated exactly: float32 product, float32 clip, C truncation toward zero. In place on
//   the vocoder's int16 PCM, so a batch of received utterances is ducked where it was made.
//
// * vad_energy_kernel — the speech gate in front of phrase segmentation (engine.py:474,
//   vad.py:40-77: chunk[::3] -> silero -> prob > threshold). silero's weights are a remote
//   torch.hub download (unavailable offline), so the gate is a documented deterministic
//   stand-in on the same 512-sample 16 kHz view of each 1536-sample chunk:
//   prob = 1 / (1 + exp(-(level_dB - center_db) / width_db)), level_dB = 10 log10(mean x^2).
//   One wave per chunk, HBM-bound (6 KB read per chunk, stride-3 view).
#include "mfma.h"
#include "kernels.h"

namespace janus {

__global__ void duck_pcm16_kernel(int16_t* __restrict__ pcm, int64_t n, float level) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i8 = i * 8;
  if (i8 >= n) return;
  if (i8 + 8 <= n && ((reinterpret_cast<uintptr_t>(pcm) & 15) == 0)) {
    uint4 v = *reinterpret_cast<const uint4*>(pcm + i8);
    int16_t* s = reinterpret_cast<int16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = __fmul_rn((float)s[j], level);
      f = fminf(fmaxf(f, -32768.0f), 32767.0f);
      s[j] = (int16_t)f;  // truncation toward zero, as numpy's astype(int16)
    }
    *reinterpret_cast<uint4*>(pcm + i8) = v;
  } else {
    for (int64_t k = i8; k < n && k < i8 + 8; ++k) {
      float f = __fmul_rn((float)pcm[k], level);
      f = fminf(fmaxf(f, -32768.0f), 32767.0f);
      pcm[k] = (int16_t)f;
    }
  }
}

void duck_pcm16_launch(int16_t* pcm, int64_t n, float level, hipStream_t s) {
  if (n <= 0) return;
  const int64_t threads = (n + 7) / 8;
  duck_pcm16_kernel<<<(unsigned)cdiv(threads, 256), 256, 0, s>>>(pcm, n, level);
  JANUS_LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void vad_energy_kernel(const float* __restrict__ pcm, int64_t n_chunks,
                                                         int chunk_len, int decim, float center_db,
                                                         float width_db, float* __restrict__ prob) {
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= n_chunks) return;
  const float* x = pcm + c * chunk_len;
  const int m = (chunk_len + decim - 1) / decim;  // samples of x[::decim]
  float e = 0.f;
  for (int j = lane; j < m; j += 64) {
    const float v = x[(int64_t)j * decim];
    e += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o);
  if (lane == 0) {
    const float db = 10.0f * log10f(e / (float)m + 1e-12f);
    prob[c] = 1.0f / (1.0f + __expf(-(db - center_db) / width_db));
  }
}

void vad_energy_launch(const float* pcm, int64_t n_chunks, int chunk_len, int decim,
                       float center_db, float width_db, float* prob, hipStream_t s) {
  if (n_chunks <= 0) return;
  vad_energy_kernel<<<(unsigned)cdiv(n_chunks, 4), 256, 0, s>>>(pcm, n_chunks, chunk_len, decim,
                                                                center_db, width_db, prob);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

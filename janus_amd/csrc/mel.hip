// Whisper log-mel front end (faster-whisper FeatureExtractor semantics; same math as
// transformers' WhisperFeatureExtractor._np_extract_fbank_features):
//   x16 = x48[::3]                        (transcriber.py:51, fused as a strided read)
//   frames: n_fft 400, hop 160, center=True (reflect), periodic Hann; the waveform is
//           zero-padded on the right (faster-whisper pads 30 s of zeros)
//   P = |rFFT|^2 (201 bins), mel = P @ filters[201x80] (slaney), log10(max(mel,1e-10))
//   then (in mel_normalize) max(x, global_max - 8), (x + 4) / 4.
// The 400-point DFT is a GEMM [frames x 400] x [400 x 416] (Hann folded into a
// cos|sin basis) on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32, fp32 accumulate);
// the mel projection is a second f32 MFMA GEMM from LDS. One block = 64 frames of one
// utterance; the 10.5k-sample window is staged once in LDS with a 162-float row
// pitch (per 160-sample hop) so the 16 frames of an MFMA A-fragment hit distinct banks.
#include "mfma.h"
#include "kernels.h"

namespace janus {

constexpr int kNfft = 400, kHop = 160, kBins = 201;
constexpr int kBinPad = 208;                 // 13 tiles of 16
constexpr int kNB = 2 * kBinPad;             // basis columns: cos | sin
constexpr int kMels = 80;
constexpr int kFT = 64;                      // frames per block
constexpr int kXRow = 162;                   // LDS pitch per hop of samples
constexpr int kXRows = (kFT * kHop + kNfft - kHop) / kHop + 1;  // 66 rows
constexpr int kPS = 210;                     // LDS pitch of the power tile

__device__ __forceinline__ f32x4 mfma_f32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t ordered_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// LDS: the sample window (xs) and, once every wave is done with it, the power tile (ps) in
// the same 53.8 KB, so three blocks fit per CU (the DFT's basis loads come from L2: the
// other blocks' waves cover their latency)
constexpr int kMelLds = (kXRows * kXRow > kFT * kPS) ? kXRows * kXRow : kFT * kPS;
constexpr int kKG = 10;                      // DFT k-steps per basis prefetch group
constexpr int kNG = kNfft / 4 / kKG;         // 10 groups
static_assert(kNG * kKG * 4 == kNfft && kNG % 2 == 0, "basis prefetch groups");

__global__ __launch_bounds__(256, 3) void mel_kernel(const float* __restrict__ pcm,
                                                  const int64_t* __restrict__ offsets,
                                                  const float* __restrict__ basis,
                                                  const float* __restrict__ filtT,
                                                  float* __restrict__ logmel,
                                                  uint32_t* __restrict__ maxkey, int n_frames_out,
                                                  int n_frames_max, int decim) {
  __shared__ float smem[kMelLds];
  __shared__ float redmax[4];
  float* xs = smem;  // [kXRows][kXRow] samples
  float* ps = smem;  // [kFT][kPS] power, after the DFT
  const int b = blockIdx.y, f0 = blockIdx.x * kFT;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int64_t base = offsets[b];
  const int64_t n16 = (offsets[b + 1] - base + decim - 1) / decim;  // len(x[::decim])
  const float* x = pcm + base;

  // stage samples p = f0*160 - 200 + off, off in [0, 64*160 + 240)
  const int64_t s0 = (int64_t)f0 * kHop - kNfft / 2;
  for (int off = tid; off < kFT * kHop + kNfft - kHop; off += 256) {
    int64_t p = s0 + off;
    if (p < 0) p = -p;  // reflect (numpy 'reflect': edge not repeated)
    const float v = p < n16 ? x[p * decim] : 0.0f;
    xs[(off / kHop) * kXRow + off % kHop] = v;
  }
  __syncthreads();

  // DFT power: wave w owns bin tiles w, w+4, w+8 (and 12 for w == 0). The basis values
  // of kKG k-steps are loaded a group ahead (two register sets), and the power values
  // stay in registers until every wave is done with xs.
  float pw[4][4][4];  // [tile j][m][r]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int bt = w + 4 * j;
    if (bt >= kBinPad / 16) break;  // wave-uniform
    f32x4 re[4], im[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) { re[m] = zero_f32x4(); im[m] = zero_f32x4(); }
    const int col = bt * 16 + (lane & 15);
    const float* bp = basis + (lane >> 4) * kNB + col;  // basis row n = 4 kk + (lane >> 4)
    float cA[kKG], sA[kKG], cB[kKG], sB[kKG];
    auto ldg = [&](float (&c)[kKG], float (&sn)[kKG], int g) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < kKG; ++q) {
        const int kk = g * kKG + q;
        c[q] = bp[kk * 4 * kNB];
        sn[q] = bp[kk * 4 * kNB + kBinPad];
      }
    };
    auto run = [&](const float (&c)[kKG], const float (&sn)[kKG], int g) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < kKG; ++q) {
        const int n = (g * kKG + q) * 4 + (lane >> 4);
        const int hr = n / kHop, hc = n % kHop;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int i = m * 16 + (lane & 15);
          const float av = xs[(i + hr) * kXRow + hc];
          re[m] = mfma_f32(av, c[q], re[m]);
          im[m] = mfma_f32(av, sn[q], im[m]);
        }
      }
    };
    ldg(cA, sA, 0);
    for (int g = 0; g < kNG; g += 2) {
      ldg(cB, sB, g + 1);
      run(cA, sA, g);
      if (g + 2 < kNG) ldg(cA, sA, g + 2);
      run(cB, sB, g + 1);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) pw[j][m][r] = re[m][r] * re[m][r] + im[m][r] * im[m][r];
  }
  __syncthreads();  // every wave is done with xs: ps over it
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int bt = w + 4 * j;
    if (bt >= kBinPad / 16) break;
    const int col = bt * 16 + (lane & 15);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) ps[(m * 16 + 4 * (lane >> 4) + r) * kPS + col] = pw[j][m][r];
  }
  __syncthreads();

  // mel projection: wave w -> frames 16w..16w+15, all 5 mel tiles
  f32x4 mel[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) mel[t] = zero_f32x4();
  for (int kk = 0; kk < kBinPad / 4; ++kk) {
    const int bin = kk * 4 + (lane >> 4);
    const float av = ps[(w * 16 + (lane & 15)) * kPS + bin];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const float bv = filtT[bin * kMels + t * 16 + (lane & 15)];
      mel[t] = mfma_f32(av, bv, mel[t]);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int fr = f0 + w * 16 + 4 * (lane >> 4) + r;
      const int mb = t * 16 + (lane & 15);
      const float v = log10f(fmaxf(mel[t][r], 1e-10f));
      if (fr < n_frames_max) mx = fmaxf(mx, v);
      if (fr < n_frames_out) logmel[((int64_t)b * n_frames_out + fr) * kMels + mb] = v;
    }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) redmax[w] = mx;
  __syncthreads();
  if (tid == 0) {
    const float m = fmaxf(fmaxf(redmax[0], redmax[1]), fmaxf(redmax[2], redmax[3]));
    atomicMax(&maxkey[b], ordered_key(m));
  }
}

// max(x, global_max - 8), (x + 4) / 4 for the content frames of each utterance; frames at
// and beyond content = len(x16) // 160 are 0.0. faster-whisper slices every 30 s window out
// of the whole clip's log-mel (content frames only: segment_size = min(3000,
// content_frames - seek)) and pads it to 3000 frames with zeros (pad_or_trim), so a window
// past the end of the audio holds 0.0 there, not the log-mel of silence.
__global__ void mel_normalize_kernel(const float* __restrict__ logmel,
                                     const uint32_t* __restrict__ maxkey, _Float16* __restrict__ out,
                                     const int64_t* __restrict__ offsets, int decim,
                                     int frames, int out_ld, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int mb = (int)(idx % kMels);
  const int64_t row = idx / kMels;  // b*frames + f
  const int b = (int)(row / frames);
  const int f = (int)(row - (int64_t)b * frames);
  const int64_t n16 = (offsets[b + 1] - offsets[b] + decim - 1) / decim;
  const uint32_t k = maxkey[b];
  const float gmax = __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
  float v = fmaxf(logmel[idx], gmax - 8.0f);
  out[row * out_ld + mb] = f < n16 / kHop ? (_Float16)((v + 4.0f) / 4.0f) : (_Float16)0.0f;
}

void mel_launch(const float* pcm, const int64_t* offsets, int B, const float* basis,
                const float* filters, float* logmel, uint32_t* maxkey, int n_frames_out,
                int decim, hipStream_t s) {
  JANUS_CHECK(decim >= 1, "mel: decimation must be >= 1");
  if (B <= 0) return;
  // frames whose window reaches audio: up to index 3001 for a 30 s input
  const int n_frames_max = n_frames_out + 2;
  JANUS_HIP(hipMemsetAsync(maxkey, 0, sizeof(uint32_t) * B, s));
  dim3 grid((n_frames_max + kFT - 1) / kFT, B);
  mel_kernel<<<grid, 256, 0, s>>>(pcm, offsets, basis, filters, logmel, maxkey, n_frames_out,
                                  n_frames_max, decim);
  JANUS_LAUNCH_CHECK();
}

void mel_normalize_launch(const float* logmel, const uint32_t* maxkey, _Float16* out,
                          const int64_t* offsets, int decim, int B, int frames, int n_mels,
                          int out_ld, hipStream_t s) {
  JANUS_CHECK(n_mels == kMels, "mel: 80 bins only");
  const int64_t total = (int64_t)B * frames * kMels;
  if (total == 0) return;
  mel_normalize_kernel<<<(unsigned)cdiv(total, 256), 256, 0, s>>>(logmel, maxkey, out, offsets,
                                                                   decim, frames, out_ld, total);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

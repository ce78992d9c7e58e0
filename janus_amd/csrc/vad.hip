// Silero-style neural speech gate on gfx950: the local-weights replacement for the
// reference's VoiceActivityDetector (backend/services/vad.py:10-88), which loads
// silero-vad from torch.hub (remote) and calls model(chunk[::3], 16000) per 1536-sample
// 48 kHz capture chunk (vad.py:52-77; engine.py:474). The model object is stateful across
// calls (64-sample context + LSTM state) and the reference never resets it (vad.py:79-88).
//
// Per 512-sample 16 kHz chunk (silero-vad v5 16 kHz graph, as published):
//   x = [context(64) | chunk(512)]            576 samples; context <- x[512:576]
//   STFT: reflect-pad 64 on the right (640), frames of 256 at hop 128 (4 frames),
//         magnitude of the 129-bin basis projection  -> mag [129][4]
//   encoder: 4 x (Conv1d k3 p1 + ReLU): 129->128 s1, 128->64 s2, 64->64 s2, 64->128 s1
//            -> [128][1]
//   decoder: LSTMCell(128, 128) on the carried (h, c) -> ReLU -> Conv1d(128, 1, 1)
//            -> sigmoid = speech probability
// One 256-thread block per channel walks that channel's chunks in order (the LSTM is
// sequential in time; channels are independent). ~0.7 M MAC per chunk from L2-resident
// fp32 weights (~0.9 MB): latency-bound, one launch per block of chunks for all channels.
#include "mfma.h"
#include "kernels.h"

namespace janus {


constexpr int kVadChunk = 512, kVadCtx = 64, kVadIn = kVadChunk + kVadCtx, kVadPadded = kVadIn + 64;
constexpr int kVadBins = 129, kVadFrames = 4, kVadH = 128;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

// conv1d k3 p1 over T_in frames with stride st: out[co][t] = relu(b + sum w[co][ci][k] in[ci][t*st+k-1])
__device__ __forceinline__ void vad_conv(const float* __restrict__ w, const float* __restrict__ b,
                                         const float* in, int Cin, int Tin, float* out, int Cout,
                                         int st) {
  const int Tout = (Tin + 2 - 3) / st + 1;
  for (int o = threadIdx.x; o < Cout * Tout; o += blockDim.x) {
    const int co = o / Tout, t = o % Tout;
    float acc = b[co];
    const float* wr = w + (int64_t)co * Cin * 3;
    for (int k = 0; k < 3; ++k) {
      const int p = t * st + k - 1;
      if (p < 0 || p >= Tin) continue;
      for (int ci = 0; ci < Cin; ++ci) acc = fmaf(wr[ci * 3 + k], in[ci * Tin + p], acc);
    }
    out[co * Tout + t] = fmaxf(acc, 0.0f);
  }
}

__global__ __launch_bounds__(256) void silero_vad_kernel(const float* __restrict__ pcm, int n_chunks,
                                                          int chunk_len, int decim, VadWeights W,
                                                          float* __restrict__ ctx_state,
                                                          float* __restrict__ hc_state,
                                                          float* __restrict__ prob) {
  __shared__ float x[kVadPadded];
  __shared__ float mag[kVadBins * kVadFrames];
  __shared__ float e0[128 * 4], e1[64 * 2], e2[64], e3[128];
  __shared__ float h[kVadH], c[kVadH], gates[4 * kVadH];
  __shared__ float red[4];
  const int s = blockIdx.x, tid = threadIdx.x;
  float* ctx = ctx_state + (int64_t)s * kVadCtx;
  float* hc = hc_state + (int64_t)s * 2 * kVadH;
  if (tid < kVadH) { h[tid] = hc[tid]; c[tid] = hc[kVadH + tid]; }
  if (tid < kVadCtx) x[tid] = ctx[tid];
  for (int j = 0; j < n_chunks; ++j) {
    const float* src = pcm + ((int64_t)s * n_chunks + j) * chunk_len;
    for (int i = tid; i < kVadChunk; i += blockDim.x) x[kVadCtx + i] = src[(int64_t)i * decim];
    __syncthreads();
    if (tid < 64) x[kVadIn + tid] = x[kVadIn - 2 - tid];   // reflect pad (edge excluded)
    __syncthreads();
    // STFT magnitude: 4 frames x 129 bins (real rows 0..128, imaginary rows 129..257)
    for (int o = tid; o < kVadBins * kVadFrames; o += blockDim.x) {
      const int bin = o / kVadFrames, f = o % kVadFrames;
      const float* br = W.basis + (int64_t)bin * 256;
      const float* bi = W.basis + (int64_t)(bin + kVadBins) * 256;
      const float* xf = x + f * 128;
      float re = 0.f, im = 0.f;
      for (int k = 0; k < 256; ++k) {
        re = fmaf(br[k], xf[k], re);
        im = fmaf(bi[k], xf[k], im);
      }
      mag[bin * kVadFrames + f] = sqrtf(re * re + im * im);
    }
    __syncthreads();
    vad_conv(W.w0, W.b0, mag, kVadBins, 4, e0, 128, 1);
    __syncthreads();
    vad_conv(W.w1, W.b1, e0, 128, 4, e1, 64, 2);
    __syncthreads();
    vad_conv(W.w2, W.b2, e1, 64, 2, e2, 64, 2);
    __syncthreads();
    vad_conv(W.w3, W.b3, e2, 64, 1, e3, 128, 1);
    __syncthreads();
    // LSTMCell: gates (i, f, g, o) = W_ih e3 + b_ih + W_hh h + b_hh
    for (int g = tid; g < 4 * kVadH; g += blockDim.x) {
      float acc = W.bih[g] + W.bhh[g];
      const float* wi = W.wih + (int64_t)g * kVadH;
      const float* wh = W.whh + (int64_t)g * kVadH;
      for (int k = 0; k < kVadH; ++k) acc = fmaf(wi[k], e3[k], fmaf(wh[k], h[k], acc));
      gates[g] = acc;
    }
    __syncthreads();
    float contrib = 0.f;
    if (tid < kVadH) {
      const float ig = sigm(gates[tid]), fg = sigm(gates[kVadH + tid]);
      const float gg = tanhf(gates[2 * kVadH + tid]), og = sigm(gates[3 * kVadH + tid]);
      const float cn = fg * c[tid] + ig * gg;
      const float hn = og * tanhf(cn);
      c[tid] = cn;
      h[tid] = hn;
      contrib = W.wo[tid] * fmaxf(hn, 0.0f);
    }
    for (int o = 32; o > 0; o >>= 1) contrib += __shfl_xor(contrib, o);
    if ((tid & 63) == 0) red[tid >> 6] = contrib;
    __syncthreads();
    if (tid == 0) prob[(int64_t)s * n_chunks + j] = sigm(W.bo[0] + ((red[0] + red[1]) + (red[2] + red[3])));
    // next chunk's context: the last 64 input samples of this one
    float keep = 0.f;
    if (tid < kVadCtx) keep = x[kVadChunk + tid];
    __syncthreads();
    if (tid < kVadCtx) x[tid] = keep;
  }
  __syncthreads();
  if (tid < kVadH) { hc[tid] = h[tid]; hc[kVadH + tid] = c[tid]; }
  if (tid < kVadCtx) ctx[tid] = x[tid];
}

void silero_vad_launch(const float* pcm, int n_streams, int n_chunks, int chunk_len, int decim,
                       const VadWeights& W, float* ctx_state, float* hc_state, float* prob,
                       hipStream_t s) {
  JANUS_CHECK(chunk_len >= kVadChunk * decim, "vad: a chunk must hold 512 samples after decimation");
  if (n_streams <= 0 || n_chunks <= 0) return;
  silero_vad_kernel<<<n_streams, 256, 0, s>>>(pcm, n_chunks, chunk_len, decim, W, ctx_state,
                                              hc_state, prob);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

// LayerNorm over the fp32 residual stream (Whisper pre-LN blocks, eps 1e-5), one
// wavefront per row; two-pass mean/variance from registers, wave-shuffle reductions,
// 16-byte loads/stores. HBM-bound: 4·d B read + 2·d B written per row. The fp16 path's
// arithmetic is mfma.h's ln_sum4 / ln_sq4 / ln_norm4 (shared with resid_ln_kernel).
#include "mfma.h"
#include "kernels.h"

namespace janus {

template <int MAXV, bool F32OUT>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ b, void* out,
                                                        int rows, int d, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = d / 4;
  const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)row * d);
  // gamma / beta are independent of the row: in flight with it (one memory latency)
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  float4 gg[MAXV], bb[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int i = lane + k * 64;
    gg[k] = i < nv ? g4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    bb[k] = i < nv ? b4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 v[MAXV];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int i = lane + k * 64;
    v[k] = i < nv ? xr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += ln_sum4(v[k]);
  }
  s = wave_sum_f32(s);
  const float mean = s / d;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int i = lane + k * 64;
    if (i < nv) q += ln_sq4(v[k], mean);
  }
  q = wave_sum_f32(q);
  const float rstd = rsqrtf(q / d + eps);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int i = lane + k * 64;
    if (i >= nv) continue;
    if constexpr (F32OUT) {
      float4 y;
      y.x = (v[k].x - mean) * rstd * gg[k].x + bb[k].x;
      y.y = (v[k].y - mean) * rstd * gg[k].y + bb[k].y;
      y.z = (v[k].z - mean) * rstd * gg[k].z + bb[k].z;
      y.w = (v[k].w - mean) * rstd * gg[k].w + bb[k].w;
      reinterpret_cast<float4*>(static_cast<float*>(out) + (int64_t)row * d)[i] = y;
    } else {
      reinterpret_cast<half4*>(static_cast<_Float16*>(out) + (int64_t)row * d)[i] =
          ln_norm4(v[k], mean, rstd, gg[k], bb[k]);
    }
  }
}

template <bool F32OUT>
static void ln_dispatch(const float* x, const float* g, const float* b, void* out, int rows, int d,
                        float eps, hipStream_t s) {
  JANUS_CHECK(d % 4 == 0 && d <= 2048, "layernorm: d must be a multiple of 4 and <= 2048");
  if (rows <= 0) return;
  const int grid = (rows + 3) / 4;
  if (d <= 256) layernorm_kernel<1, F32OUT><<<grid, 256, 0, s>>>(x, g, b, out, rows, d, eps);
  else if (d <= 512) layernorm_kernel<2, F32OUT><<<grid, 256, 0, s>>>(x, g, b, out, rows, d, eps);
  else if (d <= 1024) layernorm_kernel<4, F32OUT><<<grid, 256, 0, s>>>(x, g, b, out, rows, d, eps);
  else layernorm_kernel<8, F32OUT><<<grid, 256, 0, s>>>(x, g, b, out, rows, d, eps);
  JANUS_LAUNCH_CHECK();
}

void layernorm_launch(const float* x, const float* g, const float* b, _Float16* out, int rows,
                      int d, float eps, hipStream_t s) {
  ln_dispatch<false>(x, g, b, out, rows, d, eps, s);
}

void layernorm_f32_launch(const float* x, const float* g, const float* b, float* out, int rows,
                          int d, float eps, hipStream_t s) {
  ln_dispatch<true>(x, g, b, out, rows, d, eps, s);
}

// The wave shuffles of mfma.h (xshfl<O>, 64 lanes) against the lane permutation they stand
// for: out[w][k][lane] = xshfl<2^k>(in[w][lane]), k = 0..5 (janus_wave_xor_f32, a kernel
// test entry).
__global__ __launch_bounds__(64) void wave_xor_kernel(const float* __restrict__ in, float* __restrict__ out) {
  const int lane = threadIdx.x;
  const float v = in[blockIdx.x * 64 + lane];
  float* o = out + (int64_t)blockIdx.x * 6 * 64 + lane;
  o[0] = xshfl<1>(v);
  o[64] = xshfl<2>(v);
  o[128] = xshfl<4>(v);
  o[192] = xshfl<8>(v);
  o[256] = xshfl<16>(v);
  o[320] = xshfl<32>(v);
}

void wave_xor_launch(const float* in, float* out, int n_waves, hipStream_t s) {
  if (n_waves <= 0) return;
  wave_xor_kernel<<<n_waves, 64, 0, s>>>(in, out);
  JANUS_LAUNCH_CHECK();
}

}  // namespace janus

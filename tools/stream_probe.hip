// Per-CU streaming rate of the cross-attention's encoder reads on gfx950: one block (8
// waves) per decoder row streams that row's encoder output (1500 keys x 512 fp16 = 1.5 MB)
// in 64-key chunks, as xattn_kernel does, with the loaded data folded into a checksum
// (no math), so only the access pattern differs between variants:
//   frag : the MFMA B-fragment pattern of xattn_kernel (lane = key lr, 16 B at dim group
//          lg; 8 loads per chunk per wave, each instruction touching 16 keys x 64 B)
//   row  : whole key rows (each load instruction one contiguous 1 KB row; 8 per wave)
// DEPTH chunks in flight per wave (1 or 2). Question: is the ~24-29 GB/s per CU the
// xattn kernel reaches set by the access pattern, by bytes in flight, or by neither?
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
// run:   tools/stream_probe [rows=64] [reps=20]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int kTe = 1500, kD = 512, kCH = 64;

template <bool ROW, int DEPTH>
__global__ __launch_bounds__(512) void stream_kernel(const uint4* __restrict__ enc, uint32_t* __restrict__ out) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint4* eb = enc + (size_t)b * kTe * kD / 8;
  uint4 buf[DEPTH][8];
  auto load = [&](uint4 (&dst)[8], int t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int key, c;  // key and 16-byte column of this lane's i-th load
      if constexpr (ROW) {
        key = t + 8 * w + i;          // wave w: keys 8w .. 8w+7 of the chunk, one row per load
        c = lane;                     // 64 lanes x 16 B = the row
      } else {
        const int nt = w % 4, kh = w / 4, lr = lane & 15, lg = lane >> 4;
        key = t + 16 * nt + lr;       // xattn_kernel: key tile nt, dim half kh
        c = (kh * 256 + 8 * lg + 32 * i) / 8;
      }
      key = key < kTe ? key : kTe - 1;
      dst[i] = eb[(size_t)key * (kD / 8) + c];
    }
  };
  uint32_t acc = 0;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(buf[d], d * kCH);
  for (int t = 0; t < kTe; t += DEPTH * kCH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= buf[d][i].x ^ buf[d][i].y ^ buf[d][i].z ^ buf[d][i].w;
      load(buf[d], t + (d + DEPTH) * kCH);
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= buf[d][i].x;
  out[(size_t)b * 512 + tid] = acc;
}

template <bool ROW, int DEPTH>
static void run(const char* name, const uint4* enc, uint32_t* out, int rows, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  stream_kernel<ROW, DEPTH><<<rows, 512>>>(enc, out);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) stream_kernel<ROW, DEPTH><<<rows, 512>>>(enc, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / reps;
  const double bytes = (double)rows * kTe * kD * 2;
  std::printf("{\"variant\": \"%s\", \"depth\": %d, \"rows\": %d, \"us\": %.1f, \"GBps\": %.0f, \"GBps_per_block\": %.1f}\n",
              name, DEPTH, rows, us, bytes / us / 1e3, bytes / rows / us / 1e3);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? std::atoi(argv[1]) : 64;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  if (rows < 1 || rows > 256 || reps < 1) return 2;
  uint4* enc = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&enc, (size_t)rows * kTe * kD * 2));
  CK(hipMalloc(&out, (size_t)rows * 512 * 4));
  CK(hipMemset(enc, 0x3c, (size_t)rows * kTe * kD * 2));
  for (int k = 0; k < 2; ++k) {
    run<false, 1>("frag", enc, out, rows, reps);
    run<false, 2>("frag", enc, out, rows, reps);
    run<true, 1>("row", enc, out, rows, reps);
    run<true, 2>("row", enc, out, rows, reps);
  }
  CK(hipFree(enc));
  CK(hipFree(out));
  return 0;
}

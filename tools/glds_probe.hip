// L2 -> LDS staging rate of the encoder GEMM's operand pattern on gfx950 (no math): every
// block of the QKV shape (M = 96 000, N = 1536, K = 512, 256 x 256 tiles, XCD-aware order)
// DMAs its A and W k-slices with global_load_lds 16 B per lane in 8-row x 128-B pieces, as
// gemm_big_kernel does, and only the schedule differs:
//   depth 0 : the shipped one — a whole 64 KB k-tile issued, vmcnt(0) + barrier
//   depth D : 16 KB half-tiles (128 rows of A or W), one issued per step, counted
//             vmcnt(2 (D - 1)) + raw s_barrier, so D - 1 half-tiles stay in flight
// Question: is gemm_big's staging rate set by bytes in flight (latency) or by a per-CU
// throughput ceiling? (DESIGN.md §7, r06 encoder GEMM.)
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/glds_probe tools/glds_probe.hip
// run:   tools/glds_probe [reps=20] [K=512] [N=1536]
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

constexpr int kBM = 256, kBK = 64;

__device__ __forceinline__ int remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ void piece(const _Float16* src, int ld, int row_g, int max_row, int k0,
                                      _Float16* lds, int lane) {
  const int r = lane >> 3;
  const int c = (lane & 7) ^ ((r >> 1) & 7);
  const int gr = min(row_g + r, max_row);
  typedef __attribute__((address_space(3))) void lds_void;
  __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)gr * ld + k0 + 8 * c), (lds_void*)lds, 16, 0, 0);
}

template <int DEPTH>
__global__ __launch_bounds__(512, 1) void stage_kernel(const _Float16* A, const _Float16* W, int M, int N, int K,
                                                       int* out) {
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * 2 * kBM * kBK];   // 128 KB
  const int nbn = N / 256, nbm = (M + kBM - 1) / kBM;
  const int bid = remap(blockIdx.x, nbm * nbn);
  const int row0 = (bid / nbn) * kBM, col0 = (bid % nbn) * 256;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nk = K / kBK;
  // half-tile h of k-tile t: 0 = A rows 0-127, 1 = A 128-255, 2 = W 0-127, 3 = W 128-255;
  // each wave DMAs two 8-row pieces of it
  auto half = [&](int s) {
    const int t = s >> 2, h = s & 3;
    _Float16* dst = smem + (s & 7) * 128 * kBK;
    const _Float16* src = h < 2 ? A : W;
    const int base = (h < 2 ? row0 : col0) + (h & 1) * 128, lim = (h < 2 ? M : N) - 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rl = wid * 16 + i * 8;
      piece(src, K, base + rl, lim, t * kBK, dst + rl * kBK, lane);
    }
  };
  if constexpr (DEPTH == 0) {
    for (int t = 0; t < nk; ++t) {
      for (int h = 0; h < 4; ++h) half(4 * t + h);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    const int ns = 4 * nk;
    for (int s = 0; s < DEPTH - 1 && s < ns; ++s) half(s);
    for (int s = 0; s < ns; ++s) {
      if (s + DEPTH - 1 < ns) {
        half(s + DEPTH - 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DEPTH - 1)) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
    }
  }
  if (threadIdx.x == 0 && smem[lane] == (_Float16)12345.0f) out[blockIdx.x] = 1;   // keep the DMAs
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const int K = argc > 2 ? std::atoi(argv[2]) : 512;
  const int N = argc > 3 ? std::atoi(argv[3]) : 1536;
  const int M = 96000;
  _Float16 *A, *W;
  int* out;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&W, (size_t)N * K * 2));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(A, 0, (size_t)M * K * 2));
  CK(hipMemset(W, 0, (size_t)N * K * 2));
  const int blocks = ((M + kBM - 1) / kBM) * (N / 256);
  const double bytes = (double)blocks * (K / kBK) * 64.0 * 1024.0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int d) {
    switch (d) {
      case 0: stage_kernel<0><<<blocks, 512>>>(A, W, M, N, K, out); break;
      case 2: stage_kernel<2><<<blocks, 512>>>(A, W, M, N, K, out); break;
      case 3: stage_kernel<3><<<blocks, 512>>>(A, W, M, N, K, out); break;
      case 4: stage_kernel<4><<<blocks, 512>>>(A, W, M, N, K, out); break;
      case 6: stage_kernel<6><<<blocks, 512>>>(A, W, M, N, K, out); break;
      default: stage_kernel<8><<<blocks, 512>>>(A, W, M, N, K, out); break;
    }
  };
  const int depths[] = {0, 2, 3, 4, 6, 8};
  for (int d : depths) run(d);
  CK(hipDeviceSynchronize());
  for (int round = 0; round < 2; ++round)
    for (int d : depths) {
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) run(d);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1000.0 * ms / reps;
      std::printf("{\"K\": %d, \"N\": %d, \"depth\": %d, \"in_flight_kb\": %d, \"us\": %.1f, \"staged_tb_s\": %.2f}\n",
                  K, N, d, d == 0 ? 64 : 16 * (d - 1), us, bytes / us * 1e-6);
    }
  CK(hipFree(A));
  CK(hipFree(W));
  CK(hipFree(out));
  return 0;
}

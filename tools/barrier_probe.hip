// Grid barrier vs kernel boundary on gfx950: what one dependent hand-off between all blocks
// costs inside a persistent kernel, against one launch boundary in a HIP graph. This decides
// whether the greedy decoder (~67 dependent launches per position, ~5 us each inside the
// overlapped step) can gain from a persistent layer-step kernel.
//
// Every hand-off moves data like the decoder does: each of G blocks writes 1 KB (its rows),
// and after the hand-off reads the 1 KB another block wrote (on another XCD), checking the
// values. Variants:
//   graph   : N dependent launches of the exchange kernel captured in one HIP graph
//   bar_ar  : one launch, N barriers; agent-scope release add + acquire poll (the compiler's
//             fences: L2 writeback before arrival, L2 invalidate after)
//   bar_uc  : same exchange in uncached device memory (hipDeviceMallocUncached) with
//             relaxed atomics and a plain vmcnt drain before arrival: no L2 maintenance
//   bar_h   : bar_uc with a two-level arrival (8 group counters on separate 256-B lines, the
//             last arriver of a group bumps the top counter) so no one address takes all
//             128 atomics
// Each runs on a CU-masked stream of `per_xcd` CUs per XCD, alone (busy 0) and with a
// streaming copy kernel on the other CUs (the vocoder's HBM traffic beside the decoder):
// ordinary stores (busy 1) or non-temporal stores (busy 2).
// Spins are bounded: a barrier that does not complete within ~1 s sets an error flag and
// the kernel exits (no hang if blocks are not co-resident).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/barrier_probe tools/barrier_probe.hip
// run:   tools/barrier_probe [per_xcd=16] [N=2000]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int NT = 256;     // threads per block
constexpr int W = 256;      // floats per block per hand-off (1 KB)
constexpr long SPIN = 1L << 22;

__device__ __forceinline__ void write_rows(float* buf, int it, int blk) {
  float* p = buf + ((size_t)(it & 1) * gridDim.x + blk) * W;
  p[threadIdx.x] = (float)(it * 4096 + blk) + 0.25f * threadIdx.x;
}

__device__ __forceinline__ int read_check(const float* buf, int it, int blk) {
  const int src = (blk + gridDim.x / 2 + 1) % gridDim.x;  // another XCD
  const float* p = buf + ((size_t)(it & 1) * gridDim.x + src) * W;
  const float v = __builtin_nontemporal_load(p + threadIdx.x);
  return v != (float)(it * 4096 + src) + 0.25f * threadIdx.x;
}

// one hand-off per launch: read what the previous launch wrote, write this launch's rows
__global__ void exchange_kernel(float* buf, int it, int* err) {
  const int blk = blockIdx.x;
  if (it > 0 && read_check(buf, it - 1, blk)) atomicAdd(err, 1);
  write_rows(buf, it, blk);
}

template <bool UC, bool HIER = false>
__global__ void persistent_kernel(float* buf, int* cnt, int n, int* err) {
  const int blk = blockIdx.x;
  __shared__ int bad;
  for (int it = 0; it < n; ++it) {
    write_rows(buf, it, blk);
    __syncthreads();
    if (threadIdx.x == 0) {
      const int target = (it + 1) * gridDim.x;
      if (HIER) {
        __builtin_amdgcn_s_waitcnt(0);
        const int grp = blk & 7, gsz = gridDim.x / 8;
        const int old = __hip_atomic_fetch_add(cnt + 64 * (1 + grp), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (it + 1) * gsz - 1) __hip_atomic_fetch_add(cnt, gsz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (UC) {
        __builtin_amdgcn_s_waitcnt(0);  // stores of this thread done (uncached: in memory)
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      long s = 0;
      bad = 0;
      while (__hip_atomic_load(cnt, UC ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++s > SPIN) { bad = 1; break; }
      }
    }
    __syncthreads();
    if (bad) { if (threadIdx.x == 0) atomicAdd(err + 1, 1); return; }
    if (read_check(buf, it, blk)) atomicAdd(err, 1);
  }
}

// the vocoder stand-in: streaming copy, `reps` passes; NT: non-temporal stores (busy = 2)
template <bool NTS>
__global__ void copy_kernel(const float4* __restrict__ a, float4* __restrict__ b, size_t n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      const float4 v = a[i] + make_float4(1.f, 1.f, 1.f, 1.f);
      typedef float vf4 __attribute__((ext_vector_type(4)));
      if (NTS) __builtin_nontemporal_store(vf4{v.x, v.y, v.z, v.w}, reinterpret_cast<vf4*>(b + i));
      else b[i] = v;
    }
}

static void masks(int ncu, int per_xcd, std::vector<uint32_t>& a, std::vector<uint32_t>& b) {
  const int words = (ncu + 31) / 32;
  a.assign(words, 0);
  b.assign(words, 0);
  for (int i = 0; i < ncu; ++i) ((i / 8) < per_xcd ? a : b)[i / 32] |= 1u << (i % 32);
}

int main(int argc, char** argv) {
  const int per_xcd = argc > 1 ? atoi(argv[1]) : 16;
  const int N = argc > 2 ? atoi(argv[2]) : 2000;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  std::vector<uint32_t> ma, mb;
  masks(ncu, per_xcd, ma, mb);
  hipStream_t sd, sv;
  CK(hipExtStreamCreateWithCUMask(&sd, (uint32_t)ma.size(), ma.data()));
  CK(hipExtStreamCreateWithCUMask(&sv, (uint32_t)mb.size(), mb.data()));
  const int G = 8 * per_xcd;  // one block per CU of the partition

  float *buf, *ubuf;
  int *cnt, *err;
  CK(hipMalloc(&buf, sizeof(float) * 2 * G * W));
  CK(hipExtMallocWithFlags((void**)&ubuf, sizeof(float) * 2 * G * W, hipDeviceMallocUncached));
  CK(hipMalloc(&cnt, 64 * 9 * sizeof(int)));
  CK(hipMalloc(&err, 2 * sizeof(int)));
  const size_t cn = (size_t)1 << 26;  // 1 GB per array
  float4 *ca, *cb;
  CK(hipMalloc(&ca, cn * sizeof(float4)));
  CK(hipMalloc(&cb, cn * sizeof(float4)));
  CK(hipMemset(ca, 0, cn * sizeof(float4)));

  // graph of N dependent exchange launches
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(sd, hipStreamCaptureModeThreadLocal));
  for (int it = 0; it < N; ++it) exchange_kernel<<<G, NT, 0, sd>>>(buf, it, err);
  CK(hipStreamEndCapture(sd, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[4] = {"graph", "bar_ar", "bar_uc", "bar_h"};
  for (int busy = 0; busy < 3; ++busy) {
    for (int v = 0; v < 4; ++v) {
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemsetAsync(err, 0, 2 * sizeof(int), sd));
        CK(hipMemsetAsync(cnt, 0, 64 * 9 * sizeof(int), sd));
        CK(hipStreamSynchronize(sd));
        if (busy) {
          if (busy == 1) copy_kernel<false><<<8 * (ncu / 8 - per_xcd) * 8, 256, 0, sv>>>(ca, cb, cn, 40);
          else copy_kernel<true><<<8 * (ncu / 8 - per_xcd) * 8, 256, 0, sv>>>(ca, cb, cn, 40);
          CK(hipGetLastError());
        }
        CK(hipEventRecord(e0, sd));
        if (v == 0) CK(hipGraphLaunch(ge, sd));
        else if (v == 1) persistent_kernel<false><<<G, NT, 0, sd>>>(buf, cnt, N, err);
        else if (v == 2) persistent_kernel<true><<<G, NT, 0, sd>>>(ubuf, cnt, N, err);
        else persistent_kernel<true, true><<<G, NT, 0, sd>>>(ubuf, cnt, N, err);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, sd));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        int herr[2];
        CK(hipMemcpy(herr, err, sizeof(herr), hipMemcpyDeviceToHost));
        CK(hipStreamSynchronize(sv));
        printf("{\"variant\": \"%s\", \"busy\": %d, \"rep\": %d, \"G\": %d, \"N\": %d, \"us_per_handoff\": %.3f, "
               "\"bad_reads\": %d, \"timeouts\": %d}\n",
               names[v], busy, rep, G, N, 1000.0 * ms / N, herr[0], herr[1]);
        fflush(stdout);
        if (herr[1]) return 2;
      }
    }
  }
  return 0;
}

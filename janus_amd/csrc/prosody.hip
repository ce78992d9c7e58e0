// Prosody hot path: per-hop YIN pitch (aubio 'yin', buf 4096) + RMS energy, batched
// over a ragged set of utterances (one stream each).
//
// Replaces, for the reference's ProsodyExtractor (backend/services/prosody.py):
//   :32-34  aubio.pitch('yin', 4096, hop, sr), unit Hz, tolerance 0.8  (one stateful detector)
//   :67     rms = sqrt(mean(x**2))
//   :78-87  per-hop loop: zero-pad last hop to `hop`, pitch = detector(chunk)[0], keep > 0
//   :90     mean of voiced pitches
// aubio 0.4.9 is a third-party C library absent from this container; its published
// algorithm (src/pitch/pitch.c aubio_pitch_do / aubio_pitch_do_yin / slideblock,
// src/pitch/pitchyin.c aubio_pitchyin_do, src/mathutils.c aubio_quadratic_peak_pos /
// fvec_min_elem / aubio_level_lin / aubio_db_spl) is restated here and in
// oracle/yin_oracle.c. The arithmetic below keeps aubio's float rounding order
// (sequential j-sum, separate mul/add, sequential tau running sum, float divide),
// so per-hop f0 is bit-identical to the sequential C restatement.
//
// Layout in HBM: pcm is one flat f32 array of all utterances back to back
// (sample_offsets[B+1]); hops are numbered globally (hop_offsets[B+1]); per-stream
// detector state is the 4096-sample aubio buffer, [B][4096] f32.
//
// Roofline: VALU-bound (fp32 non-contracted sub/mul/add), ≈3·2048 flop per tau,
// up to 2047 taus per hop; HBM traffic is 16 KB window per hop (L2-served overlap).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include "common.h"

namespace janus {

constexpr int kYinBuf = 4096;          // aubio pitch buffer (prosody.py:32)
constexpr int kYinLen = kYinBuf / 2;   // yin fvec length
// Block = NT threads, each lane owns 2 consecutive taus, so one pass covers 2·NT taus.
// NT = 128 (256-tau passes, the default for an uncapped grid): a voiced hop stops within
// 256 taus of its period; NT = 64 / 256 (128- / 512-tau passes) by JANUS_YIN_THREADS; 256
// for a grid capped beside the decoder.

__device__ __forceinline__ int find_utt(const int64_t* offs, int B, int64_t g) {
  // largest b with offs[b] <= g (offs is non-decreasing, offs[0]=0, offs[B]=total)
  int lo = 0, hi = B;  // invariant: offs[lo] <= g < offs[hi]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (offs[mid] <= g) lo = mid; else hi = mid;
  }
  return lo;
}

// Window sample k (0..4095) of hop i of stream b: the aubio buffer after sliding
// hop i in (prosody.py:81-84, aubio_pitch_slideblock).
__device__ __forceinline__ float window_sample(const float* pcm, int64_t base, int64_t n,
                                               const float* state, int64_t i, int hop, int k) {
  int64_t p = (i + 1) * (int64_t)hop - kYinBuf + k;
  if (p < 0) return state ? state[kYinBuf + p] : 0.0f;
  return p < n ? pcm[base + p] : 0.0f;
}

template <int kYinThreads>
__global__ __launch_bounds__(kYinThreads) void yin_hops_kernel(
    const float* __restrict__ pcm, const int64_t* __restrict__ sample_off,
    const int64_t* __restrict__ hop_off, int B, int hop, const float* __restrict__ state_in,
    float tol, float silence_db, float level_thr, unsigned sample_rate,
    float* __restrict__ f0_out, int64_t total_hops) {
  __shared__ __attribute__((aligned(16))) float w[kYinBuf];
  __shared__ __attribute__((aligned(16))) float dd[kYinLen];   // d(tau), then yin(tau)
  constexpr int kTauChunk = kYinThreads * 2;
  constexpr int kWaves = kYinThreads / 64;
  __shared__ __attribute__((aligned(16))) float cum[kTauChunk];                           // running sum (tmp2) of a chunk
  __shared__ int s_found;
  __shared__ float s_level;
  __shared__ unsigned long long s_best;  // argmin key

  const int tid = threadIdx.x;
  for (int64_t g = blockIdx.x; g < total_hops; g += gridDim.x) {
    const int b = find_utt(hop_off, B, g);
    const int64_t i = g - hop_off[b];
    const int64_t base = sample_off[b];
    const int64_t n = sample_off[b + 1] - base;
    const float* st = state_in ? state_in + (int64_t)b * kYinBuf : nullptr;

    {
      // all of this thread's window loads in flight at once (a load -> wait -> LDS store
      // per sample serialised 32 global round trips per hop): clamped addresses, no
      // branches, out-of-range samples zeroed after the load
      constexpr int kPer = kYinBuf / kYinThreads;
      const int64_t p0 = (i + 1) * (int64_t)hop - kYinBuf;
      float v[kPer];
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int64_t p = p0 + tid + u * kYinThreads;
        const bool in_pcm = p >= 0 && p < n;
        const bool in_st = p < 0 && st != nullptr;
        const float* src = in_pcm ? pcm + base + p : (in_st ? st + kYinBuf + p : pcm);
#ifdef JANUS_YIN_NT  // A/B: the window stream past the caches (YIN runs beside the decoder)
        v[u] = __builtin_nontemporal_load(src);
#else
        v[u] = *src;
#endif
        v[u] = (in_pcm || in_st) ? v[u] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kPer; ++u) w[tid + u * kYinThreads] = v[u];
    }
    if (tid == 0) s_found = 0x7fffffff;
    __syncthreads();

    // Silent hop: aubio_pitch_do forces f0 = 0 when the new hop's level is under the
    // silence threshold, whatever YIN found, so YIN is skipped. The decision uses a
    // parallel (reordered) level sum with a 1 dB margin, far outside float rounding: the
    // sequential aubio level below then agrees (digital silence gives exactly 0 = -inf dB).
    {
      float e = 0.0f;
      for (int j = kYinBuf - hop + tid; j < kYinBuf; j += kYinThreads) e += w[j] * w[j];
      for (int off = 32; off > 0; off >>= 1) e += __shfl_xor(e, off);
      if ((tid & 63) == 0) cum[tid >> 6] = e;
      __syncthreads();
      float ps = 0.0f;
#pragma unroll
      for (int k = 0; k < kWaves; ++k) ps += cum[k];
      const float pe = ps / (float)hop;
      const bool silent = 10.0f * log10f(pe) < silence_db - 1.0f;
      __syncthreads();  // cum[0..kWaves) read by all before the tau passes reuse it
      if (silent) {
        if (tid == 0) f0_out[g] = 0.0f;
        continue;
      }
    }

    // aubio_level_lin on the new hop (sequential float sum, as aubio).
    if (tid == kYinThreads - 1) {
      float e = 0.0f;
      for (int j = kYinBuf - hop; j < kYinBuf; ++j) e = __fadd_rn(e, __fmul_rn(w[j], w[j]));
      s_level = __fdiv_rn(e, (float)hop);
    }

    float running = 0.0f;  // tmp2, carried across chunks (only lane 0 uses it)
    int found = 0x7fffffff;
    for (int chunk = 0; chunk < kYinLen / kTauChunk; ++chunk) {
      const int tau0 = chunk * kTauChunk + 2 * tid;
      // the lane's two taus as one packed pair: v_pk_add_f32 / v_pk_mul_f32 do the two
      // taus' sub, square and add in one instruction each (IEEE single ops, no
      // contraction: this file builds with -ffp-contract=off), half the VALU issue of
      // scalar code; the same per-tau j order as aubio
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      f32x2 acc = {0.f, 0.f};
#pragma unroll 4
      for (int j = 0; j < kYinLen; j += 4) {
        const float4 a = *reinterpret_cast<const float4*>(&w[j]);
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const f32x2 bv = {w[j + tau0 + jj], w[j + tau0 + jj + 1]};
          const f32x2 aa = {av[jj], av[jj]};
          const f32x2 t = aa - bv;
          acc = acc + t * t;
        }
      }
      dd[tau0 + 0] = acc.x;
      dd[tau0 + 1] = acc.y;
      __syncthreads();
      // tmp2 += yin[tau] in tau order (pitchyin.c), one lane. 16 taus per batch through
      // 16-byte LDS reads / writes: the add chain stays sequential (bit-exact), but one LDS
      // round trip now serves 16 adds instead of one (the per-tau read->add->write loop
      // was latency-bound at ~100 cycles a tau). tau = 0 adds nothing (cum[0] unread).
      if (tid == 0) {
        const float4* d4 = reinterpret_cast<const float4*>(dd + chunk * kTauChunk);
        float4* c4 = reinterpret_cast<float4*>(cum);
        float4 nxt[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) nxt[q] = d4[q];
        for (int bt = 0; bt < kTauChunk / 16; ++bt) {
          float4 cur[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
          if (bt + 1 < kTauChunk / 16) {
#pragma unroll
            for (int q = 0; q < 4; ++q) nxt[q] = d4[4 * (bt + 1) + q];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float4 o;
            running = (chunk == 0 && bt == 0 && q == 0) ? running : __fadd_rn(running, cur[q].x);
            o.x = running;
            running = __fadd_rn(running, cur[q].y);
            o.y = running;
            running = __fadd_rn(running, cur[q].z);
            o.z = running;
            running = __fadd_rn(running, cur[q].w);
            o.w = running;
            c4[4 * bt + q] = o;
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int t = tau0 + m;
        float y;
        if (t == 0) y = 1.0f;
        else {
          const float s = cum[t - chunk * kTauChunk];
          y = (s != 0.0f) ? __fmul_rn(dd[t], __fdiv_rn((float)t, s)) : 1.0f;
        }
        dd[t] = y;
      }
      __syncthreads();
      // Early exit: first period p in [2, 2044] (tau = p+3 computed) with
      // yin[p] < tol && yin[p] < yin[p+1]. Periods whose p+1 lies in the next chunk wait.
      const int p_hi = min((chunk + 1) * kTauChunk - 2, kYinLen - 4);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int p = tau0 + m - (chunk == 0 ? 0 : 1);  // chunk>0 also re-checks its first-1
        if (p >= 2 && p <= p_hi && p >= chunk * kTauChunk - 1) {
          const float yp = dd[p];
          if (yp < tol && yp < dd[p + 1]) atomicMin(&s_found, p);
        }
      }
      __syncthreads();
      found = s_found;
      if (found != 0x7fffffff) break;
    }

    int pos;
    if (found != 0x7fffffff) {
      pos = found;
    } else {
      // fvec_min_elem: smallest value, ties -> LAST index.
      if (tid == 0) s_best = ~0ull;
      __syncthreads();
      unsigned long long best = ~0ull;
      for (int t = tid; t < kYinLen; t += kYinThreads) {
        // yin >= 0, so the float bit pattern orders like the value; invert index for ties.
        const unsigned long long key =
            ((unsigned long long)__float_as_uint(dd[t]) << 32) | (unsigned)(kYinLen - 1 - t);
        best = key < best ? key : best;
      }
      for (int off = 32; off > 0; off >>= 1) {
        unsigned long long o = __shfl_xor(best, off);
        best = o < best ? o : best;
      }
      if ((tid & 63) == 0) atomicMin(&s_best, best);
      __syncthreads();
      pos = kYinLen - 1 - (int)(s_best & 0xffffffffu);
    }

    if (tid == 0) {
      // aubio_quadratic_peak_pos
      float period;
      if (pos == 0 || pos == kYinLen - 1) {
        period = (float)pos;
      } else {
        const float s0 = dd[pos - 1], s1 = dd[pos], s2 = dd[pos + 1];
        const float num = __fmul_rn(0.5f, __fsub_rn(s0, s2));
        const float den = __fadd_rn(__fsub_rn(s0, __fmul_rn(2.0f, s1)), s2);
        period = __fadd_rn((float)pos, __fdiv_rn(num, den));
      }
      // aubio_pitch_do_yin: samplerate / (pitch + 0.) in double, stored as float.
      float f0 = period > 0.0f ? (float)((double)sample_rate / (double)period) : 0.0f;
      // aubio_silence_detection(ibuf, silence): (float)(10 * log10f(level)) < silence -> 0,
      // decided as level < level_thr: the host found the float where the C library's
      // log10f crosses the threshold (silence_level_threshold), so the gate follows the
      // CPU's log10f rounding bit for bit, not the device log10f's
      if (s_level < level_thr) f0 = 0.0f;
      f0_out[g] = f0;
    }
    __syncthreads();
  }
}

// ---- numpy float32 reductions, bit for bit -------------------------------------------
// rms = np.sqrt(np.mean(x ** 2)) (prosody.py:67) and np.mean(pitch_values) (:90) are float32
// np.add.reduce followed by a float64 divide by the np.intp count (numpy/_core/_methods.py
// _mean: ret.dtype.type(ret / rcount)). np.add.reduce over a contiguous float32 array:
//   * the reduction iterator hands the inner loop buffers of NPY_BUFSIZE = 8192 elements,
//     whose sums accumulate SEQUENTIALLY into the identity 0.0f (out += pairwise(buffer));
//   * each buffer is summed by pairwise_sum (numpy/_core/src/umath/loops_utils.h.src):
//     n < 8 -> sequential from 0; n <= 128 -> 8 accumulators seeded with a[0..7], stepped
//     by 8, combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), remainder added in order;
//     else split at n2 = n/2 - (n/2)%8 and return pairwise(a, n2) + pairwise(a+n2, n-n2).
// Pinned against numpy 2.2 on random sizes (tests/test_oracle_prosody.py).
// The split tree depends on the buffer length only. A buffer <= 8192 has its leaves at depth
// <= 7, so it maps onto 128 slots: slot t walks the splits by the bits of t (msb first);
// a leaf reached at depth l belongs to the slot whose low 7-l bits are zero, the others
// hold 0.0f. The perfect binary tree over the slots then adds exactly the pairs numpy adds
// (x + 0.0f == x for every x >= 0 and NaN/inf alike), so a 7-level xor-shuffle tree gives
// numpy's value bit for bit.
constexpr int kNpBuf = 8192;    // NPY_BUFSIZE
constexpr int kPwBlock = 128;   // PW_BLOCKSIZE
constexpr int kPwDepth = 7;     // slots = 2^7 cover every buffer <= 8192 (host test)
constexpr int kPwSlots = 1 << kPwDepth;

__device__ __forceinline__ bool pw_slot(int m, int t, int& off, int& len) {
  off = 0;
  len = m;
#pragma unroll
  for (int l = 0; l < kPwDepth; ++l) {
    if (len <= kPwBlock) return (t & ((1 << (kPwDepth - l)) - 1)) == 0;
    int n2 = len >> 1;
    n2 -= n2 & 7;
    if ((t >> (kPwDepth - 1 - l)) & 1) { off += n2; len -= n2; }
    else len = n2;
  }
  return true;
}

// pairwise_sum leaf over ld(off .. off+len), len <= 128
template <class Ld>
__device__ __forceinline__ float pw_leaf(const Ld& ld, int off, int len) {
  if (len < 8) {
    float r = 0.0f;
    for (int i = 0; i < len; ++i) r = __fadd_rn(r, ld(off + i));
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = ld(off + j);
  const int end = len - (len & 7);
  int i = 8;
  for (; i < end; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], ld(off + i + j));
  }
  float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                        __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
  for (; i < len; ++i) res = __fadd_rn(res, ld(off + i));
  return res;
}

// Tree over the 128 slots of one buffer: slot t lives in lane t & 63 of wave (t >> 6) of a
// 2-wave group; the root is the two waves' sums added (through LDS by the caller).
__device__ __forceinline__ float pw_wave_tree(float v) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) v = __fadd_rn(v, __shfl_xor(v, off));
  return v;
}

// Squares of leaf i of one full 8192-element buffer (the 128 elements at 128 i): 16-byte
// loads when x is 16-byte aligned.
__device__ __forceinline__ float sq_leaf_full(const float* x, int leaf) {
  const float* a = x + kPwBlock * leaf;
  float r[8];
  if (((uintptr_t)a & 15) == 0) {
    // two halves of 16 loads in flight (the 8-accumulator order is sequential in i, so
    // the split changes nothing): 64 VGPRs of loads fit the 1024-thread block's budget
    const float4* a4 = reinterpret_cast<const float4*>(a);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = a4[16 * h + q];
      int q0 = 0;
      if (h == 0) {
        r[0] = __fmul_rn(v[0].x, v[0].x); r[1] = __fmul_rn(v[0].y, v[0].y);
        r[2] = __fmul_rn(v[0].z, v[0].z); r[3] = __fmul_rn(v[0].w, v[0].w);
        r[4] = __fmul_rn(v[1].x, v[1].x); r[5] = __fmul_rn(v[1].y, v[1].y);
        r[6] = __fmul_rn(v[1].z, v[1].z); r[7] = __fmul_rn(v[1].w, v[1].w);
        q0 = 2;
      }
#pragma unroll
      for (int q = q0; q < 16; q += 2) {
        r[0] = __fadd_rn(r[0], __fmul_rn(v[q].x, v[q].x));
        r[1] = __fadd_rn(r[1], __fmul_rn(v[q].y, v[q].y));
        r[2] = __fadd_rn(r[2], __fmul_rn(v[q].z, v[q].z));
        r[3] = __fadd_rn(r[3], __fmul_rn(v[q].w, v[q].w));
        r[4] = __fadd_rn(r[4], __fmul_rn(v[q + 1].x, v[q + 1].x));
        r[5] = __fadd_rn(r[5], __fmul_rn(v[q + 1].y, v[q + 1].y));
        r[6] = __fadd_rn(r[6], __fmul_rn(v[q + 1].z, v[q + 1].z));
        r[7] = __fadd_rn(r[7], __fmul_rn(v[q + 1].w, v[q + 1].w));
      }
    }
    return __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                     __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
  }
  auto ld = [&](int i) { return __fmul_rn(a[i], a[i]); };
  return pw_leaf(ld, 0, kPwBlock);
}

constexpr int kReduceThreads = 1024;                       // 8 buffers per pass
constexpr int kReduceGroups = kReduceThreads / kPwSlots;

// Per utterance: rms = np.sqrt(np.mean(x ** 2)) (prosody.py:67) and the count and
// np.mean of the voiced f0 values in hop order (:86-90), numpy float32 bit for bit.
// pcm == nullptr skips the energy half (kernel-level janus_np_voiced_mean_f32).
__global__ __launch_bounds__(kReduceThreads) void prosody_reduce_kernel(
    const float* __restrict__ pcm, const int64_t* __restrict__ sample_off,
    const int64_t* __restrict__ hop_off, const float* __restrict__ f0, float* __restrict__ rms_out,
    float* __restrict__ mean_f0_out, int32_t* __restrict__ n_voiced_out) {
  __shared__ float s_wave[kReduceThreads / 64];
  __shared__ int s_cnt[kReduceThreads / 64];
  __shared__ float s_comp[kNpBuf];   // the voiced values of one numpy buffer, compacted
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = tid / kPwSlots, slot = tid % kPwSlots;

  if (pcm != nullptr) {
    const int64_t base = sample_off[b], n = sample_off[b + 1] - base;
    const float* x = pcm + base;
    const int64_t nbuf = (n + kNpBuf - 1) / kNpBuf;
    float total = 0.0f;   // out = identity; out += pairwise(buffer) in buffer order (tid 0)
    for (int64_t c0 = 0; c0 < nbuf; c0 += kReduceGroups) {
      const int64_t c = c0 + grp;
      float v = 0.0f;
      if (c < nbuf) {
        const float* xb = x + c * kNpBuf;
        const int m = (int)min<int64_t>(kNpBuf, n - c * kNpBuf);
        if (m == kNpBuf) {
          // a full buffer's 64 leaves of 128 sit at depth 6: slot 2i owns leaf i
          // (pw_slot(8192, 2i) = (128 i, 128), tests/test_oracle_prosody.py)
          if ((slot & 1) == 0) v = sq_leaf_full(xb, slot >> 1);
        } else {
          int off, len;
          if (pw_slot(m, slot, off, len)) {
            auto ld = [&](int i) { return __fmul_rn(xb[i], xb[i]); };
            v = pw_leaf(ld, off, len);
          }
        }
      }
      v = pw_wave_tree(v);
      if (lane == 0) s_wave[wid] = v;
      __syncthreads();
      if (tid == 0) {
        for (int g = 0; g < kReduceGroups && c0 + g < nbuf; ++g)
          total = __fadd_rn(total, __fadd_rn(s_wave[2 * g], s_wave[2 * g + 1]));
      }
      __syncthreads();
    }
    if (tid == 0)
      // np.sqrt of the float32 mean, correctly rounded: v_sqrt_f32 (what sqrtf / __fsqrt_rn
      // compile to here) is 1-ulp approximate, the f64 square root is correctly rounded,
      // and rounding it to float is the correctly rounded float root (53 >= 2 * 24 + 2)
      rms_out[b] = n > 0 ? (float)sqrt((double)(float)((double)total / (double)n))
                         : __int_as_float(0x7fc00000);  // mean([]) = nan
  }

  // voiced f0: count, then per numpy buffer of compacted values, gather + pairwise
  const int64_t h0 = hop_off[b], nh = hop_off[b + 1] - h0;
  int cnt = 0;
  for (int64_t k = tid; k < nh; k += kReduceThreads) cnt += f0[h0 + k] > 0.0f;
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (lane == 0) s_cnt[wid] = cnt;
  __syncthreads();
  int nv = 0;
#pragma unroll
  for (int w = 0; w < kReduceThreads / 64; ++w) nv += s_cnt[w];
  __syncthreads();
  float fsum = 0.0f;
  for (int64_t cb = 0; cb < nv; cb += kNpBuf) {
    // compact hops in order: block-wide exclusive scan of the voiced flags per 1024 hops
    int64_t before = 0;
    for (int64_t k0 = 0; k0 < nh; k0 += kReduceThreads) {
      const int64_t k = k0 + tid;
      const float v = k < nh ? f0[h0 + k] : 0.0f;
      const bool voiced = v > 0.0f;
      const unsigned long long m = __ballot(voiced);
      const int in_wave = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) s_cnt[wid] = __popcll(m);
      __syncthreads();
      int64_t pos = before + in_wave;
      int64_t seg = 0;
#pragma unroll
      for (int w = 0; w < kReduceThreads / 64; ++w) {
        pos += w < wid ? s_cnt[w] : 0;
        seg += s_cnt[w];
      }
      if (voiced && pos >= cb && pos < cb + kNpBuf) s_comp[pos - cb] = v;
      before += seg;
      __syncthreads();
    }
    const int m = (int)min<int64_t>(kNpBuf, nv - cb);
    if (tid < kPwSlots) {
      float v = 0.0f;
      int off, len;
      if (pw_slot(m, slot, off, len)) {
        auto ld = [&](int i) { return s_comp[i]; };
        v = pw_leaf(ld, off, len);
      }
      v = pw_wave_tree(v);
      if (lane == 0) s_wave[wid] = v;
    }
    __syncthreads();
    if (tid == 0) fsum = __fadd_rn(fsum, __fadd_rn(s_wave[0], s_wave[1]));
    __syncthreads();
  }
  if (tid == 0) {
    mean_f0_out[b] = nv > 0 ? (float)((double)fsum / (double)nv) : 0.0f;
    n_voiced_out[b] = nv;
  }
}

void np_voiced_mean_launch(const float* vals, const int64_t* offsets, int B, float* mean_out,
                           int32_t* n_out, hipStream_t stream) {
  JANUS_CHECK(B >= 0, "batch must be >= 0");
  if (B == 0) return;
  prosody_reduce_kernel<<<dim3(B), dim3(kReduceThreads), 0, stream>>>(
      nullptr, nullptr, offsets, vals, nullptr, mean_out, n_out);
  JANUS_LAUNCH_CHECK();
}

// Detector state after the call = the aubio buffer after the last hop.
__global__ void prosody_state_kernel(const float* __restrict__ pcm, const int64_t* __restrict__ sample_off,
                                     const int64_t* __restrict__ hop_off, int hop,
                                     const float* __restrict__ state_in, float* __restrict__ state_out) {
  const int b = blockIdx.x;
  const int64_t base = sample_off[b], n = sample_off[b + 1] - base;
  const int64_t nh = hop_off[b + 1] - hop_off[b];
  const float* st = state_in ? state_in + (int64_t)b * kYinBuf : nullptr;
  for (int k = threadIdx.x; k < kYinBuf; k += blockDim.x) {
    float v;
    if (nh == 0) v = st ? st[k] : 0.0f;
    else v = window_sample(pcm, base, n, st, nh - 1, hop, k);
    state_out[(int64_t)b * kYinBuf + k] = v;
  }
}

// Smallest float level L with (float)(10.0 * log10f(L)) >= silence_db (aubio's level is
// not silent from there up), by bisection over the ordered bit patterns of [0, +inf]
// with the host C library's log10f — the one aubio (and the oracle) call. Assumes only
// that log10f is monotone.
static float silence_level_threshold(float silence_db) {
  auto silent = [&](uint32_t bits) {
    float L;
    std::memcpy(&L, &bits, 4);
    return (float)(10.0 * (double)log10f(L)) < silence_db;
  };
  uint32_t lo = 0u, hi = 0x7f800000u;  // 0.0f (-inf dB: silent) .. +inf (never silent)
  if (!silent(lo)) return 0.0f;         // silence_db = -inf: nothing is silent
  while (hi - lo > 1u) {
    const uint32_t mid = lo + (hi - lo) / 2u;
    if (silent(mid)) lo = mid;
    else hi = mid;
  }
  float thr;
  std::memcpy(&thr, &hi, 4);
  return thr;
}

void prosody_launch(const float* pcm, const int64_t* sample_off, const int64_t* hop_off, int B,
                    int64_t total_hops, int sample_rate, int hop, float tol, float silence_db,
                    const float* state_in, float* state_out, float* f0_out, float* rms_out,
                    float* mean_f0_out, int32_t* n_voiced_out, hipStream_t stream,
                    int max_blocks) {
  JANUS_CHECK(B >= 0, "batch must be >= 0");
  JANUS_CHECK(hop > 0 && hop <= kYinBuf, "hop_size must be in [1, 4096]");
  JANUS_CHECK(sample_rate > 0, "sample_rate must be > 0");
  if (B == 0) return;
  JANUS_CHECK(state_in != state_out || state_in == nullptr, "state_in and state_out must not alias");
  if (total_hops > 0) {
    const float level_thr = silence_level_threshold(silence_db);
    // max_blocks > 0 caps the grid (blocks loop over hops): the pipeline runs prosody
    // beside the latency-bound decoder with one block per CU, leaving it room to dispatch
    const int64_t cap = max_blocks > 0 ? max_blocks : (1ll << 30);
    const int64_t grid = std::min<int64_t>(total_hops, cap);
    // two-wave blocks (256-tau passes) for an uncapped grid on its own CUs: with the packed
    // difference loop (LDS-latency-bound at one wave per 24.5 KB block) the second wave
    // per block pays for the coarser early exit (r02 v49: 56 x 30 s 11.86 vs 12.63 ms
    // standalone, 302.0-302.2 vs 304.7-305.1 ms per step; with the scalar loop one-wave
    // blocks had been 1.6 ms per step faster); a capped grid beside the greedy decoder
    // keeps the 256-thread blocks (back-to-back step: 422 vs 449 ms per step with 128)
    static const int nt_env = ab_env("JANUS_YIN_THREADS") ? std::atoi(ab_env("JANUS_YIN_THREADS")) : 0;
    const int nt = nt_env > 0 ? nt_env : (max_blocks > 0 ? 256 : 128);
    if (nt == 256)
      yin_hops_kernel<256><<<dim3((unsigned)grid), dim3(256), 0, stream>>>(
          pcm, sample_off, hop_off, B, hop, state_in, tol, silence_db, level_thr, (unsigned)sample_rate,
          f0_out, total_hops);
    else if (nt == 64)  // 128-tau passes
      yin_hops_kernel<64><<<dim3((unsigned)grid), dim3(64), 0, stream>>>(
          pcm, sample_off, hop_off, B, hop, state_in, tol, silence_db, level_thr, (unsigned)sample_rate,
          f0_out, total_hops);
    else
      yin_hops_kernel<128><<<dim3((unsigned)grid), dim3(128), 0, stream>>>(
          pcm, sample_off, hop_off, B, hop, state_in, tol, silence_db, level_thr, (unsigned)sample_rate,
          f0_out, total_hops);
    JANUS_LAUNCH_CHECK();
  }
  prosody_reduce_kernel<<<dim3(B), dim3(kReduceThreads), 0, stream>>>(pcm, sample_off, hop_off, f0_out, rms_out,
                                                           mean_f0_out, n_voiced_out);
  JANUS_LAUNCH_CHECK();
  if (state_out) {
    prosody_state_kernel<<<dim3(B), dim3(256), 0, stream>>>(pcm, sample_off, hop_off, hop, state_in,
                                                            state_out);
    JANUS_LAUNCH_CHECK();
  }
}

}  // namespace janus

// C-ABI glue: error slot, version, thin extern "C" wrappers over the launchers.
#include <map>
#include <mutex>
#include "common.h"
#include "../../include/janus.h"

namespace janus {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// Not cached: a destroyed CU-masked stream's handle can be reused by a new stream with a
// different mask, and the query is cheap next to a decode.
int stream_cu_count(hipStream_t s) {
  uint32_t mask[32] = {};
  int n = 0;
  if (hipExtStreamGetCUMask(s, 32, mask) == hipSuccess)
    for (uint32_t m : mask) n += __builtin_popcount(m);
  if (n <= 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            ? prop.multiProcessorCount : 256;
  }
  return n;
}

void prosody_launch(const float* pcm, const int64_t* sample_off, const int64_t* hop_off, int B,
                    int64_t total_hops, int sample_rate, int hop, float tol, float silence_db,
                    const float* state_in, float* state_out, float* f0_out, float* rms_out,
                    float* mean_f0_out, int32_t* n_voiced_out, hipStream_t stream,
                    int max_blocks = 0);

void np_voiced_mean_launch(const float* vals, const int64_t* offsets, int B, float* mean_out,
                           int32_t* n_out, hipStream_t stream);
void duck_pcm16_launch(int16_t* pcm, int64_t n, float level, hipStream_t s);
void vad_energy_launch(const float* pcm, int64_t n_chunks, int chunk_len, int decim,
                       float center_db, float width_db, float* prob, hipStream_t s);

}  // namespace janus

using namespace janus;

extern "C" const char* janus_last_error(void) { return g_last_error.c_str(); }

extern "C" int janus_version(void) { return 100; }

extern "C" int janus_stream_create_cu_mask(const uint32_t* cu_mask, int words, void** out) {
  return guarded([&] {
    JANUS_CHECK(cu_mask && out && words > 0, "bad argument");
    hipStream_t st = nullptr;
    JANUS_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)words, cu_mask));
    *out = st;
  });
}

extern "C" int janus_stream_destroy(void* stream) {
  return guarded([&] {
    if (stream) JANUS_HIP(hipStreamDestroy((hipStream_t)stream));
  });
}

extern "C" int janus_prosody_analyze(const float* pcm, const int64_t* sample_offsets,
                                     const int64_t* hop_offsets, int batch, int64_t total_hops,
                                     int sample_rate, int hop_size, float tolerance,
                                     float silence_db, const float* state_in, float* state_out,
                                     float* f0_out, float* rms_out, float* mean_f0_out,
                                     int32_t* n_voiced_out, void* stream) {
  return guarded([&] {
    prosody_launch(pcm, sample_offsets, hop_offsets, batch, total_hops, sample_rate, hop_size,
                   tolerance, silence_db, state_in, state_out, f0_out, rms_out, mean_f0_out,
                   n_voiced_out, (hipStream_t)stream);
  });
}

extern "C" int janus_prosody_analyze_ex(const float* pcm, const int64_t* sample_offsets,
                                        const int64_t* hop_offsets, int batch, int64_t total_hops,
                                        int sample_rate, int hop_size, float tolerance,
                                        float silence_db, const float* state_in, float* state_out,
                                        float* f0_out, float* rms_out, float* mean_f0_out,
                                        int32_t* n_voiced_out, int max_blocks, void* stream) {
  return guarded([&] {
    JANUS_CHECK(max_blocks >= 0, "max_blocks must be >= 0");
    prosody_launch(pcm, sample_offsets, hop_offsets, batch, total_hops, sample_rate, hop_size,
                   tolerance, silence_db, state_in, state_out, f0_out, rms_out, mean_f0_out,
                   n_voiced_out, (hipStream_t)stream, max_blocks);
  });
}

extern "C" int janus_np_voiced_mean_f32(const float* values, const int64_t* offsets, int batch,
                                        float* mean_out, int32_t* count_out, void* stream) {
  return guarded([&] {
    JANUS_CHECK(batch >= 0 && (batch == 0 || (offsets && mean_out && count_out)), "bad argument");
    np_voiced_mean_launch(values, offsets, batch, mean_out, count_out, (hipStream_t)stream);
  });
}

extern "C" int janus_duck_pcm16(int16_t* pcm, int64_t n, float level, void* stream) {
  return guarded([&] {
    JANUS_CHECK(pcm || n == 0, "null argument");
    JANUS_CHECK(level >= 0.0f && level < 1.0f, "ducking level must be in [0, 1) (callers skip 1.0)");
    duck_pcm16_launch(pcm, n, level, (hipStream_t)stream);
  });
}

extern "C" int janus_vad_energy(const float* pcm, int64_t n_chunks, int chunk_len, int decim,
                                float center_db, float width_db, float* prob_out, void* stream) {
  return guarded([&] {
    JANUS_CHECK((pcm && prob_out) || n_chunks == 0, "null argument");
    JANUS_CHECK(chunk_len > 0 && decim > 0 && width_db > 0.0f, "bad VAD geometry");
    vad_energy_launch(pcm, n_chunks, chunk_len, decim, center_db, width_db, prob_out,
                      (hipStream_t)stream);
  });
}

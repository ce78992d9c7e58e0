// Vocoder edge kernels (vocoder.hip).
#pragma once
#include "common.h"

namespace janus {

void frontend_launch(const uint8_t* bytes, const int64_t* boff, const int32_t* emo,
                     const float* e_text, const float* e_emo, const float* spk, int B, int F, int C,
                     _Float16* lat, hipStream_t s);
void speaker_launch(const float* logmel, const uint32_t* maxkey, const int64_t* offsets, int B,
                    int frames, const float* P, const float* bias, int C, float* spk,
                    hipStream_t s);
void conv_post_launch(const _Float16* x, int B, int T, const float* w, float bias, float* wav,
                      int16_t* pcm, hipStream_t s, int pre_silu = 1, float* pre_tanh = nullptr);

}  // namespace janus

// Vocoder edge kernels (vocoder.hip).
#pragma once
#include "common.h"

namespace janus {

void frontend_launch(const uint8_t* bytes, const int64_t* boff, const int32_t* emo,
                     const float* e_text, const float* e_emo, int B, int F, int C, _Float16* lat,
                     hipStream_t s);
void conv_post_launch(const _Float16* x, int B, int T, const float* w, float bias, float* wav,
                      int16_t* pcm, hipStream_t s, int pre_silu = 1);

}  // namespace janus

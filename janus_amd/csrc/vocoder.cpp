// Firefly-GAN (fish-speech HiFiGANGenerator) decoder on gfx950: the local stand-in for
// the reference's Fish Audio cloud TTS (backend/services/synthesizer.py:133-207,
// client.tts.convert at :202), which returns speech for an "(emotion) text" prompt.
//
//   latents [B][F][512] -> conv_pre(k13) -> 5 x { SiLU -> ConvTranspose(u, 2u)
//   -> ParallelBlock(mean of ResBlock1 k in {3,7,11}, dilations {1,3,5}) }
//   -> SiLU -> conv_post(k13, ->1) -> tanh -> f32 waveform @ 44.1 kHz (+ int16 PCM)
//
// Every conv is the implicit-GEMM MFMA kernel (conv.hip) on time-major fp16
// activations with SiLU fused into operand staging and bias / SiLU / residual /
// 1/3-mean fused into the epilogue, so each ResBlock1 conv pair costs two launches and
// no elementwise passes. Optional per-conv HIP-event timing feeds bench.py's roofline.
#include <cstdlib>
#include <mutex>
#include <vector>
#include "devmem.h"
#include "kernels.h"
#include "vocoder.h"
#include "../../include/janus.h"

namespace janus {
ConvArgs conv_args_torch(const _Float16* in, int B, int T_in, int Cin, const _Float16* packed,
                         const float* bias, _Float16* out, int T_out, int Cout, int taps,
                         int stride, int padding, int dilation, int transposed, int pre_act,
                         int post_act, const _Float16* res, int64_t res_bs, float scale,
                         int accumulate);
void cast_f32_f16_launch(const float* in, _Float16* out, int64_t n, hipStream_t s);

struct VConv {
  DevMem packed;
  const float* bias = nullptr;
  int cin = 0, cout = 0, taps = 0, stride = 1, pad = 0, dil = 1, transposed = 0;
};
struct VUnit {  // fused (convs1[m], convs2[m]) pair for narrow stages
  DevMem w1, w2;
  const float *b1 = nullptr, *b2 = nullptr;
  int c = 0, k = 0, d = 1;
};
struct TimedLaunch {
  hipEvent_t a, b;
  double flops, bytes;  // algorithmic: MFMA FLOPs, fp16 activation bytes read once / written once
  int fam;              // channel width of a fused ResBlock1 unit, 0 for the conv kernel
};
// per-family accumulators (index by slot: 0 conv, then C = 16 .. 512)
struct FamStat { int fam = -1; double flops = 0, bytes = 0, ms = 0; int64_t launches = 0; };
}  // namespace janus

struct janus_vocoder {
  janus_vocoder_config cfg;
  janus::ParamStore params;
  bool prepared = false;
  std::mutex mu;
  janus::VConv pre;
  std::vector<janus::VConv> ups;
  std::vector<janus::VConv> rb;  // [stage][kernel][dilation][conv1|conv2]
  std::vector<janus::VUnit> units;  // same indexing / 2, fused path (C <= 32)
  bool fuse = true;
  const float* post_w = nullptr;
  float post_b = 0.f;
  janus::DevMem buf[5];
  janus::DevMem spk_logmel, spk_maxkey;  // speaker-conditioning workspace
  // timing
  bool timing = false;
  std::vector<janus::TimedLaunch> pending;
  std::vector<hipEvent_t> pool;
  double t_flops = 0, t_ms = 0;
  int64_t t_launches = 0;
  janus::FamStat fam[8];
};

namespace janus {

static int rb_index(const janus_vocoder_config& c, int stage, int kj, int m, int which) {
  return ((stage * c.n_kernels + kj) * c.n_dilations + m) * 2 + which;
}

static void make_conv(janus_vocoder* v, VConv& cv, const std::string& name, int cin, int cout,
                      int taps, int stride, int pad, int dil, int transposed, hipStream_t s) {
  cv.cin = cin; cv.cout = cout; cv.taps = taps; cv.stride = stride; cv.pad = pad; cv.dil = dil;
  cv.transposed = transposed;
  const int64_t wn = transposed ? (int64_t)cin * cout * 2 * stride : (int64_t)cout * cin * taps;
  const float* w = v->params.get(name + ".weight", wn);
  cv.bias = v->params.get(name + ".bias", cout);
  const ConvPack g = conv_pack_geometry(cin, cout, transposed ? 2 : taps);
  cv.packed.ensure(sizeof(_Float16) * g.phase_elems * (transposed ? stride : 1));
  conv_pack_weights(w, cv.packed.as<_Float16>(), cin, cout, taps, transposed, stride, s);
}

static void prepare(janus_vocoder* v, hipStream_t s) {
  if (v->prepared) return;
  const auto& c = v->cfg;
  make_conv(v, v->pre, "conv_pre", c.latent_dim, c.channels, c.pre_kernel, 1,
            (c.pre_kernel - 1) / 2, 1, 0, s);
  v->ups.clear();
  v->ups.resize(c.n_ups);
  v->rb.clear();
  v->rb.resize((size_t)c.n_ups * c.n_kernels * c.n_dilations * 2);
  v->units.clear();
  v->units.resize((size_t)c.n_ups * c.n_kernels * c.n_dilations);
  int ch = c.channels;
  for (int i = 0; i < c.n_ups; ++i) {
    const int u = c.up_rates[i];
    make_conv(v, v->ups[i], "ups." + std::to_string(i), ch, ch / 2, 0, u, u / 2, 1, 1, s);
    ch /= 2;
    for (int kj = 0; kj < c.n_kernels; ++kj) {
      const int k = c.rb_kernels[kj];
      for (int m = 0; m < c.n_dilations; ++m) {
        const int d = c.rb_dilations[m];
        const std::string p = "resblocks." + std::to_string(i) + ".blocks." + std::to_string(kj);
        make_conv(v, v->rb[rb_index(c, i, kj, m, 0)], p + ".convs1." + std::to_string(m), ch, ch,
                  k, 1, d * (k - 1) / 2, d, 0, s);
        make_conv(v, v->rb[rb_index(c, i, kj, m, 1)], p + ".convs2." + std::to_string(m), ch, ch,
                  k, 1, (k - 1) / 2, 1, 0, s);
        if (resunit_supported(ch, k)) {
          VUnit& U = v->units[rb_index(c, i, kj, m, 0) / 2];
          U.c = ch; U.k = k; U.d = d;
          const int64_t n = (int64_t)resunit_kp(ch, k) * ch;
          U.w1.ensure(sizeof(_Float16) * n);
          U.w2.ensure(sizeof(_Float16) * n);
          resunit_pack(v->params.get(p + ".convs1." + std::to_string(m) + ".weight", (int64_t)ch * ch * k),
                       U.w1.as<_Float16>(), ch, k, s);
          resunit_pack(v->params.get(p + ".convs2." + std::to_string(m) + ".weight", (int64_t)ch * ch * k),
                       U.w2.as<_Float16>(), ch, k, s);
          U.b1 = v->params.get(p + ".convs1." + std::to_string(m) + ".bias", ch);
          U.b2 = v->params.get(p + ".convs2." + std::to_string(m) + ".bias", ch);
        }
      }
    }
  }
  JANUS_CHECK(ch == 16, "vocoder: conv_post expects 16 channels after the upsamplers");
  v->post_w = v->params.get("conv_post.weight", (int64_t)ch * c.post_kernel);
  JANUS_CHECK(c.post_kernel == 13, "vocoder: conv_post kernel 13 supported");
  JANUS_HIP(hipMemcpy(&v->post_b, v->params.get("conv_post.bias", 1), sizeof(float),
                      hipMemcpyDeviceToHost));
  JANUS_HIP(hipStreamSynchronize(s));
  v->prepared = true;
}

static hipEvent_t take_event(janus_vocoder* v) {
  if (v->pool.empty()) {
    hipEvent_t e;
    JANUS_HIP(hipEventCreate(&e));
    return e;
  }
  hipEvent_t e = v->pool.back();
  v->pool.pop_back();
  return e;
}

static void run_conv(janus_vocoder* v, const VConv& cv, const _Float16* in, int B, int T_in,
                     _Float16* out, int T_out, int pre, int post, const _Float16* res, float scale,
                     int acc, hipStream_t s, int post_acc_silu = 0) {
  ConvArgs a = conv_args_torch(in, B, T_in, cv.cin, cv.packed.as<_Float16>(), cv.bias, out, T_out,
                               cv.cout, cv.taps, cv.stride, cv.pad, cv.dil, cv.transposed, pre,
                               post, res, (int64_t)T_out * cv.cout, scale, acc);
  a.post_acc_silu = post_acc_silu;
  if (v->timing) {
    TimedLaunch t;
    t.a = take_event(v);
    t.b = take_event(v);
    const int taps = cv.transposed ? 2 : cv.taps;
    t.flops = 2.0 * cv.cin * cv.cout * taps * (double)T_out * B;
    t.bytes = 2.0 * B * ((double)T_in * cv.cin + (double)T_out * cv.cout * (1 + (res ? 1 : 0) + (acc ? 1 : 0)));
    t.fam = 0;
    JANUS_HIP(hipEventRecord(t.a, s));
    conv_launch(a, s);
    JANUS_HIP(hipEventRecord(t.b, s));
    v->pending.push_back(t);
  } else {
    conv_launch(a, s);
  }
}

static void run_unit(janus_vocoder* v, const VUnit& U, const _Float16* x, _Float16* out, int B,
                     int T, float scale, int acc, hipStream_t s, int post_silu = 0) {
  ResUnitArgs a;
  a.x = x; a.out = out; a.w1 = U.w1.as<_Float16>(); a.b1 = U.b1; a.w2 = U.w2.as<_Float16>();
  a.b2 = U.b2; a.B = B; a.T = T; a.C = U.c; a.k = U.k; a.d = U.d; a.scale = scale;
  a.accumulate = acc; a.post_silu = post_silu;
  if (v->timing) {
    TimedLaunch t;
    t.a = take_event(v);
    t.b = take_event(v);
    t.flops = 2.0 * 2.0 * U.c * U.c * U.k * (double)T * B;
    t.bytes = 2.0 * B * (double)T * U.c * (2 + (acc ? 1 : 0));
    t.fam = U.c;
    JANUS_HIP(hipEventRecord(t.a, s));
    resunit_launch(a, s);
    JANUS_HIP(hipEventRecord(t.b, s));
    v->pending.push_back(t);
  } else {
    resunit_launch(a, s);
  }
}

static void forward(janus_vocoder* v, const _Float16* lat, int B, int F, float* wav, int16_t* pcm,
                    float* pre_tanh, hipStream_t s) {
  const auto& c = v->cfg;
  int64_t maxel = (int64_t)F * c.channels;
  {
    int64_t T = F;
    int ch = c.channels;
    for (int i = 0; i < c.n_ups; ++i) {
      T *= c.up_rates[i];
      ch /= 2;
      maxel = std::max(maxel, T * ch);
    }
  }
  for (auto& b : v->buf) b.ensure(sizeof(_Float16) * maxel * B);
  _Float16* H = v->buf[0].as<_Float16>();
  _Float16* U = v->buf[1].as<_Float16>();
  _Float16* S = v->buf[2].as<_Float16>();
  _Float16* X[2] = {v->buf[3].as<_Float16>(), v->buf[4].as<_Float16>()};
  int T = F;
  // H only feeds the next upsampler or conv_post, which both take silu(H): every producer
  // of H's final value (conv_pre, the last unit of each ParallelBlock) stores silu(H)
  // instead, so the SiLU runs once per element rather than once per upsampler phase
  run_conv(v, v->pre, lat, B, F, H, F, ACT_NONE, ACT_SILU, nullptr, 1.0f, 0, s);
  const float inv_k = 1.0f / c.n_kernels;
  for (int i = 0; i < c.n_ups; ++i) {
    const int Tn = T * c.up_rates[i];
    run_conv(v, v->ups[i], H, B, T, U, Tn, ACT_NONE, ACT_NONE, nullptr, 1.0f, 0, s);
    T = Tn;
    for (int kj = 0; kj < c.n_kernels; ++kj) {
      const _Float16* x = U;
      for (int m = 0; m < c.n_dilations; ++m) {
        const VUnit& U = v->units[rb_index(c, i, kj, m, 0) / 2];
        if (v->fuse && U.c > 0) {
          if (m + 1 < c.n_dilations) {
            _Float16* xn = X[m & 1];
            run_unit(v, U, x, xn, B, T, 1.0f, 0, s);
            x = xn;
          } else {
            run_unit(v, U, x, H, B, T, inv_k, kj > 0 ? 1 : 0, s, kj + 1 == c.n_kernels);
          }
          continue;
        }
        const VConv& c1 = v->rb[rb_index(c, i, kj, m, 0)];
        const VConv& c2 = v->rb[rb_index(c, i, kj, m, 1)];
        run_conv(v, c1, x, B, T, S, T, ACT_SILU, ACT_SILU, nullptr, 1.0f, 0, s);
        if (m + 1 < c.n_dilations) {
          _Float16* xn = X[m & 1];
          run_conv(v, c2, S, B, T, xn, T, ACT_NONE, ACT_NONE, x, 1.0f, 0, s);
          x = xn;
        } else {
          run_conv(v, c2, S, B, T, H, T, ACT_NONE, ACT_NONE, x, inv_k, kj > 0 ? 1 : 0, s,
                   kj + 1 == c.n_kernels);
        }
      }
    }
  }
  conv_post_launch(H, B, T, v->post_w, v->post_b, wav, pcm, s, /*pre_silu=*/0, pre_tanh);
}

static void collect_timing(janus_vocoder* v) {
  for (auto& t : v->pending) {
    JANUS_HIP(hipEventSynchronize(t.b));
    float ms = 0.f;
    JANUS_HIP(hipEventElapsedTime(&ms, t.a, t.b));
    v->t_ms += ms;
    v->t_flops += t.flops;
    v->t_launches += 1;
    for (auto& f : v->fam) {
      if (f.fam != t.fam && f.fam != -1) continue;
      f.fam = t.fam;
      f.flops += t.flops; f.bytes += t.bytes; f.ms += ms; f.launches += 1;
      break;
    }
    v->pool.push_back(t.a);
    v->pool.push_back(t.b);
  }
  v->pending.clear();
}

}  // namespace janus

using namespace janus;

extern "C" int janus_vocoder_create(const janus_vocoder_config* cfg, janus_vocoder** out) {
  return guarded([&] {
    JANUS_CHECK(cfg && out, "null argument");
    JANUS_CHECK(cfg->n_ups >= 1 && cfg->n_ups <= 8 && cfg->n_kernels >= 1 && cfg->n_kernels <= 4 &&
                    cfg->n_dilations >= 1 && cfg->n_dilations <= 4,
                "vocoder: bad config");
    auto* v = new janus_vocoder();
    v->cfg = *cfg;
    v->fuse = ab_env("JANUS_NO_FUSE") == nullptr;
    *out = v;
  });
}

extern "C" int janus_vocoder_destroy(janus_vocoder* v) {
  return guarded([&] {
    if (!v) return;
    (void)hipDeviceSynchronize();
    for (auto& t : v->pending) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
    for (auto e : v->pool) (void)hipEventDestroy(e);
    delete v;
  });
}

extern "C" int janus_vocoder_set_tensor(janus_vocoder* v, const char* name, const float* host,
                                        int64_t numel) {
  return guarded([&] {
    JANUS_CHECK(v && name && host && numel > 0, "bad argument");
    std::lock_guard<std::mutex> lk(v->mu);
    v->params.set(name, host, numel);
    v->prepared = false;
  });
}

extern "C" int janus_vocoder_frontend_ex(janus_vocoder* v, const uint8_t* bytes,
                                         const int64_t* byte_offsets, const int32_t* emotion_ids,
                                         const float* speaker, int batch, int frames,
                                         uint16_t* latents, void* stream) {
  return guarded([&] {
    JANUS_CHECK(v && byte_offsets && emotion_ids && latents, "null argument");
    std::lock_guard<std::mutex> lk(v->mu);
    const auto& c = v->cfg;
    frontend_launch(bytes, byte_offsets, emotion_ids,
                    v->params.get("frontend.text_embed", 256 * (int64_t)c.latent_dim),
                    v->params.get("frontend.emotion_embed", (int64_t)c.n_emotions * c.latent_dim),
                    speaker, batch, frames, c.latent_dim, reinterpret_cast<_Float16*>(latents),
                    (hipStream_t)stream);
  });
}

extern "C" int janus_vocoder_frontend(janus_vocoder* v, const uint8_t* bytes,
                                      const int64_t* byte_offsets, const int32_t* emotion_ids,
                                      int batch, int frames, uint16_t* latents, void* stream) {
  return janus_vocoder_frontend_ex(v, bytes, byte_offsets, emotion_ids, nullptr, batch, frames,
                                   latents, stream);
}

extern "C" int janus_vocoder_speaker(janus_vocoder* v, const float* pcm16k, const int64_t* offsets,
                                     int batch, float* speaker_out, void* stream) {
  return guarded([&] {
    JANUS_CHECK(v && pcm16k && offsets && speaker_out, "null argument");
    JANUS_CHECK(batch >= 1, "speaker: batch must be >= 1");
    std::lock_guard<std::mutex> lk(v->mu);
    const auto& c = v->cfg;
    hipStream_t s = (hipStream_t)stream;
    constexpr int kFrames = 3000;  // one 30 s Whisper window at 16 kHz
    v->spk_logmel.ensure(sizeof(float) * (int64_t)batch * kFrames * 80);
    v->spk_maxkey.ensure(sizeof(uint32_t) * batch);
    mel_launch(pcm16k, offsets, batch, v->params.get("mel.basis", 400 * 416),
               v->params.get("mel.filters", 208 * 80), v->spk_logmel.as<float>(),
               v->spk_maxkey.as<uint32_t>(), kFrames, 1, s);
    speaker_launch(v->spk_logmel.as<float>(), v->spk_maxkey.as<uint32_t>(), offsets, batch, kFrames,
                   v->params.get("frontend.speaker_proj", (int64_t)c.latent_dim * 80),
                   v->params.get("frontend.speaker_bias", c.latent_dim), c.latent_dim, speaker_out,
                   s);
  });
}

extern "C" int janus_vocoder_forward_ex(janus_vocoder* v, const uint16_t* latents, int batch,
                                        int frames, float* wav, int16_t* pcm, float* pre_tanh,
                                        void* stream) {
  return guarded([&] {
    JANUS_CHECK(v && latents && wav, "null argument");
    std::lock_guard<std::mutex> lk(v->mu);
    hipStream_t s = (hipStream_t)stream;
    prepare(v, s);
    if (batch <= 0 || frames <= 0) return;
    forward(v, reinterpret_cast<const _Float16*>(latents), batch, frames, wav, pcm, pre_tanh, s);
  });
}

extern "C" int janus_vocoder_forward(janus_vocoder* v, const uint16_t* latents, int batch,
                                     int frames, float* wav, int16_t* pcm, void* stream) {
  return janus_vocoder_forward_ex(v, latents, batch, frames, wav, pcm, nullptr, stream);
}

extern "C" int janus_vocoder_set_timing(janus_vocoder* v, int on) {
  return guarded([&] {
    JANUS_CHECK(v, "null argument");
    std::lock_guard<std::mutex> lk(v->mu);
    v->timing = on != 0;
  });
}

extern "C" int janus_vocoder_conv_stats(janus_vocoder* v, double* flops, double* ms,
                                        int64_t* launches, int reset) {
  return guarded([&] {
    JANUS_CHECK(v && flops && ms && launches, "null argument");
    std::lock_guard<std::mutex> lk(v->mu);
    collect_timing(v);
    *flops = v->t_flops;
    *ms = v->t_ms;
    *launches = v->t_launches;
    if (reset) { v->t_flops = 0; v->t_ms = 0; v->t_launches = 0; for (auto& f : v->fam) f = FamStat(); }
  });
}

extern "C" int janus_vocoder_family_stats(janus_vocoder* v, int cap, int* fam, double* flops,
                                          double* bytes, double* ms, int64_t* launches, int* n,
                                          int reset) {
  return guarded([&] {
    JANUS_CHECK(v && fam && flops && bytes && ms && launches && n && cap > 0, "null argument");
    std::lock_guard<std::mutex> lk(v->mu);
    collect_timing(v);
    int k = 0;
    for (auto& f : v->fam) {
      if (f.fam < 0 || k >= cap) continue;
      fam[k] = f.fam; flops[k] = f.flops; bytes[k] = f.bytes; ms[k] = f.ms; launches[k] = f.launches;
      ++k;
    }
    *n = k;
    if (reset) { v->t_flops = 0; v->t_ms = 0; v->t_launches = 0; for (auto& f : v->fam) f = FamStat(); }
  });
}

// C-ABI of the neural speech gate (vad.hip): a parameter context holding the silero-vad
// v5 16 kHz weights by their published state-dict names; per-channel state lives in
// caller buffers so one context serves any number of channels.
#include <mutex>
#include "devmem.h"
#include "kernels.h"
#include "../../include/janus.h"


struct janus_vad {
  janus::ParamStore params;
  std::mutex mu;
};

using namespace janus;

extern "C" int janus_vad_create(janus_vad** out) {
  return guarded([&] {
    JANUS_CHECK(out, "null argument");
    *out = new janus_vad();
  });
}

extern "C" int janus_vad_destroy(janus_vad* v) {
  return guarded([&] {
    if (v) {
      (void)hipDeviceSynchronize();
      delete v;
    }
  });
}

extern "C" int janus_vad_set_tensor(janus_vad* v, const char* name, const float* host, int64_t numel) {
  return guarded([&] {
    JANUS_CHECK(v && name && host && numel > 0, "bad argument");
    std::lock_guard<std::mutex> lk(v->mu);
    v->params.set(name, host, numel);
  });
}

extern "C" int janus_vad_run(janus_vad* v, const float* pcm, int n_streams, int n_chunks,
                             int chunk_len, int decim, float* ctx_state, float* hc_state,
                             float* prob, void* stream) {
  return guarded([&] {
    JANUS_CHECK(v && (pcm || n_streams * n_chunks == 0) && ctx_state && hc_state && prob,
                "null argument");
    JANUS_CHECK(n_streams >= 0 && n_chunks >= 0 && decim >= 1, "bad VAD geometry");
    std::lock_guard<std::mutex> lk(v->mu);
    const ParamStore& P = v->params;
    const std::string m = "_model.";
    VadWeights W;
    W.basis = P.get(m + "stft.forward_basis_buffer", 258 * 256);
    W.w0 = P.get(m + "encoder.0.reparam_conv.weight", 128 * 129 * 3);
    W.b0 = P.get(m + "encoder.0.reparam_conv.bias", 128);
    W.w1 = P.get(m + "encoder.1.reparam_conv.weight", 64 * 128 * 3);
    W.b1 = P.get(m + "encoder.1.reparam_conv.bias", 64);
    W.w2 = P.get(m + "encoder.2.reparam_conv.weight", 64 * 64 * 3);
    W.b2 = P.get(m + "encoder.2.reparam_conv.bias", 64);
    W.w3 = P.get(m + "encoder.3.reparam_conv.weight", 128 * 64 * 3);
    W.b3 = P.get(m + "encoder.3.reparam_conv.bias", 128);
    W.wih = P.get(m + "decoder.rnn.weight_ih", 512 * 128);
    W.whh = P.get(m + "decoder.rnn.weight_hh", 512 * 128);
    W.bih = P.get(m + "decoder.rnn.bias_ih", 512);
    W.bhh = P.get(m + "decoder.rnn.bias_hh", 512);
    W.wo = P.get(m + "decoder.decoder.2.weight", 128);
    W.bo = P.get(m + "decoder.decoder.2.bias", 1);
    silero_vad_launch(pcm, n_streams, n_chunks, chunk_len, decim, W, ctx_state, hc_state, prob,
                      (hipStream_t)stream);
  });
}

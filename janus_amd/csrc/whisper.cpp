// Whisper STT on gfx950: log-mel -> encoder -> batched greedy decoder.
//
// Replaces faster-whisper's WhisperModel (CTranslate2, int8 on CPU) as driven by
// Transcriber.transcribe_buffer (backend/services/transcriber.py:29-64):
// model.transcribe(audio[::3], beam_size=1, language='en') for one 30 s window.
// Weights arrive by name (HF Whisper checkpoint naming) as fp32 and are re-laid out
// on the device: fused fp16 QKV, packed conv weights, fp16 embeddings; the residual
// stream stays fp32, GEMM/attention operands are fp16 on MFMA with fp32 accumulation.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <cstring>
#include "devmem.h"
#include "kernels.h"
#include "decoder.h"
#include "dec_persist.h"
#include "../../include/janus.h"

namespace janus {

struct EncLayer {
  DevMem wqkv, bqkv, wo, w1, w2;  // fp16 weights / fp32 fused bias
  const float *bo, *b1, *b2, *ln1g, *ln1b, *ln2g, *ln2b;
};
struct DecLayer {
  DevMem wqkv, bqkv, wo, wq_c, wk_c, wv_c, wo_c, w1, w2;
  DevMem wqk, bqk;  // absorbed cross-attention query weights (xattn.hip)
  const float *bo, *bq_c, *bv_c, *bo_c, *b1, *b2;
  const float *ln1g, *ln1b, *ln2g, *ln2b, *ln3g, *ln3b;
};

// Lanes allocate their workspaces (hipMalloc / hipFree) before any of them starts a graph
// capture: every lane arrives here after its allocations, and captures once all have.
struct LaneLatch {
  std::mutex m;
  std::condition_variable cv;
  int left = 0;
  void arrive(bool wait) {
    std::unique_lock<std::mutex> lk(m);
    if (--left == 0) cv.notify_all();
    if (wait) cv.wait(lk, [&] { return left <= 0; });
  }
};
struct LaneArrival {
  LaneLatch* l;
  bool done = false;
  explicit LaneArrival(LaneLatch* latch) : l(latch) {}
  void now() {
    if (l && !done) l->arrive(true);
    done = true;
  }
  ~LaneArrival() {
    if (l && !done) l->arrive(false);  // a lane that failed early must not stall the others
  }
};

// One decoder lane: the per-step workspaces, KV caches and captured decode graphs for one
// slice of the batch, plus the stream it runs on. Independent lanes run concurrently
// (one host thread and one HIP stream each): every decoder launch is latency-bound at
// B <= 64, so two half-batch chains overlap their launch and memory round trips.
struct DecLane {
  DevMem d_x, d_a, d_qkv, d_o, d_q2, d_f, d_kc, d_vc, d_ck, d_cv, d_smask, d_done, d_prompt, d_nsp,
      d_supp, d_part_o, d_part_ml, d_parts, d_rules, d_tok, d_ntok, d_slp, d_lnp, d_lncnt, d_xqk,
      d_xc, d_xpc, d_xpml, d_enc, d_seed, d_xpairs, d_xgroups, d_roff, d_omid, d_segbar, d_segerr,
      d_itemp;
  std::vector<float> h_itemp;    // per-row 1 / T of the last call (source of an async copy)
  std::map<std::vector<int64_t>, hipGraphExec_t> graphs;
  std::map<std::vector<int64_t>, size_t> graph_nodes;  // kernel nodes per captured graph
  int last_positions = 0;        // positions the last decode stepped
  int64_t last_launches = 0;     // kernel launches those positions issued (graph nodes)
  // where each row slot stands after the last call (positions whose KV rows and next
  // tokens are written): a staggered call may continue row b only from an offset <=
  // stand[b], with the same batch size and max_length. Empty: nothing to continue (no call
  // yet, or the last one failed).
  std::vector<int32_t> stand;
  int stand_maxlen = 0;
  hipStream_t stream = nullptr;  // graph capture needs a non-null stream
  std::vector<uint32_t> stream_mask;  // CU mask the lane stream was created with (empty: none)
  hipEvent_t ev_done = nullptr;
  // a call without early-exit polling (check_every 0) returns without waiting for its
  // stream: its persistent segments' barrier-timeout flag is copied to pinned h_segerr
  // behind it and checked by janus_whisper_decode_check (or at this lane's next call)
  uint32_t* h_segerr = nullptr;
  hipEvent_t ev_segerr = nullptr;
  bool segerr_pending = false;
  DecLane() = default;
  DecLane(const DecLane&) = delete;
  DecLane& operator=(const DecLane&) = delete;
  ~DecLane() {
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
    if (stream) (void)hipStreamDestroy(stream);
    if (ev_done) (void)hipEventDestroy(ev_done);
    if (ev_segerr) (void)hipEventDestroy(ev_segerr);
    if (h_segerr) (void)hipHostFree(h_segerr);
  }
};

}  // namespace janus

struct janus_whisper {
  janus_whisper_config cfg;
  janus::ParamStore params;
  bool prepared = false;
  std::mutex mu;
  // device-side prepared weights
  janus::DevMem conv1p, conv2p, pos16, tok16;
  std::vector<janus::EncLayer> enc;
  std::vector<janus::DecLayer> dec;
  // workspaces
  janus::DevMem ws_x1, ws_x2, ws_r, ws_a, ws_qkv, ws_o, ws_f, ws_logmel, ws_maxkey;
  // decoder lanes: each owns the workspaces, captured graphs and stream of one batch slice
  std::vector<std::unique_ptr<janus::DecLane>> lanes;
  int last_slot = 0;  // state slot of the last decode call (decode_info reports it)
  hipEvent_t ev_in = nullptr;
  ~janus_whisper() {
    if (ev_in) (void)hipEventDestroy(ev_in);
  }
};

namespace janus {

static _Float16* to_f16(const float* src, int64_t n, DevMem& dst, hipStream_t s) {
  dst.ensure(sizeof(_Float16) * n);
  cast_f32_f16_launch(src, dst.as<_Float16>(), n, s);
  return dst.as<_Float16>();
}

// concat rows of fp32 matrices into one fp16 matrix (missing name => zeros)
static void fuse_f16(const ParamStore& P, const std::vector<std::string>& names, int64_t each,
                     DevMem& dst, hipStream_t s) {
  dst.ensure(sizeof(_Float16) * each * names.size());
  for (size_t i = 0; i < names.size(); ++i) {
    _Float16* d = dst.as<_Float16>() + i * each;
    if (P.has(names[i])) cast_f32_f16_launch(P.get(names[i], each), d, each, s);
    else JANUS_HIP(hipMemsetAsync(d, 0, sizeof(_Float16) * each, s));
  }
}

static void fuse_f32(const ParamStore& P, const std::vector<std::string>& names, int64_t each,
                     DevMem& dst, hipStream_t s) {
  dst.ensure(sizeof(float) * each * names.size());
  for (size_t i = 0; i < names.size(); ++i) {
    float* d = dst.as<float>() + i * each;
    if (P.has(names[i]))
      JANUS_HIP(hipMemcpyAsync(d, P.get(names[i], each), sizeof(float) * each,
                               hipMemcpyDeviceToDevice, s));
    else JANUS_HIP(hipMemsetAsync(d, 0, sizeof(float) * each, s));
  }
}

static void prepare(janus_whisper* w, hipStream_t s) {
  if (w->prepared) return;
  // the captured decode graphs bake in the device weight pointers that are re-allocated
  // below: drop them (a set_tensor after a decode must not replay freed weights)
  JANUS_HIP(hipDeviceSynchronize());
  for (auto& lane : w->lanes) {
    for (auto& kv : lane->graphs) (void)hipGraphExecDestroy(kv.second);
    lane->graphs.clear();
    lane->graph_nodes.clear();
  }
  const auto& c = w->cfg;
  const int d = c.d_model, ff = 4 * d;
  const ParamStore& P = w->params;
  auto pk = [&](const std::string& name, int cin, DevMem& dst) {
    const float* src = P.get(name, (int64_t)d * cin * 3);
    const ConvPack g = conv_pack_geometry(cin, d, 3);
    dst.ensure(sizeof(_Float16) * g.phase_elems);
    conv_pack_weights(src, dst.as<_Float16>(), cin, d, 3, 0, 1, s);
  };
  pk("encoder.conv1.weight", c.n_mels, w->conv1p);
  pk("encoder.conv2.weight", d, w->conv2p);
  to_f16(P.get("encoder.embed_positions.weight", (int64_t)c.n_audio_ctx * d),
         (int64_t)c.n_audio_ctx * d, w->pos16, s);
  to_f16(P.get("decoder.embed_tokens.weight", (int64_t)c.n_vocab * d), (int64_t)c.n_vocab * d,
         w->tok16, s);
  const int64_t dd = (int64_t)d * d, fd = (int64_t)ff * d;
  w->enc.clear();
  w->enc.resize(c.enc_layers);
  for (int l = 0; l < c.enc_layers; ++l) {
    const std::string p = "encoder.layers." + std::to_string(l) + ".";
    EncLayer& L = w->enc[l];
    fuse_f16(P, {p + "self_attn.q_proj.weight", p + "self_attn.k_proj.weight", p + "self_attn.v_proj.weight"}, dd, L.wqkv, s);
    fuse_f32(P, {p + "self_attn.q_proj.bias", p + "self_attn.k_proj.bias", p + "self_attn.v_proj.bias"}, d, L.bqkv, s);
    to_f16(P.get(p + "self_attn.out_proj.weight", dd), dd, L.wo, s);
    to_f16(P.get(p + "fc1.weight", fd), fd, L.w1, s);
    to_f16(P.get(p + "fc2.weight", fd), fd, L.w2, s);
    L.bo = P.get(p + "self_attn.out_proj.bias", d);
    L.b1 = P.get(p + "fc1.bias", ff);
    L.b2 = P.get(p + "fc2.bias", d);
    L.ln1g = P.get(p + "self_attn_layer_norm.weight", d);
    L.ln1b = P.get(p + "self_attn_layer_norm.bias", d);
    L.ln2g = P.get(p + "final_layer_norm.weight", d);
    L.ln2b = P.get(p + "final_layer_norm.bias", d);
  }
  w->dec.clear();
  w->dec.resize(c.dec_layers);
  for (int l = 0; l < c.dec_layers; ++l) {
    const std::string p = "decoder.layers." + std::to_string(l) + ".";
    DecLayer& L = w->dec[l];
    fuse_f16(P, {p + "self_attn.q_proj.weight", p + "self_attn.k_proj.weight", p + "self_attn.v_proj.weight"}, dd, L.wqkv, s);
    fuse_f32(P, {p + "self_attn.q_proj.bias", p + "self_attn.k_proj.bias", p + "self_attn.v_proj.bias"}, d, L.bqkv, s);
    to_f16(P.get(p + "self_attn.out_proj.weight", dd), dd, L.wo, s);
    to_f16(P.get(p + "encoder_attn.q_proj.weight", dd), dd, L.wq_c, s);
    to_f16(P.get(p + "encoder_attn.k_proj.weight", dd), dd, L.wk_c, s);
    to_f16(P.get(p + "encoder_attn.v_proj.weight", dd), dd, L.wv_c, s);
    to_f16(P.get(p + "encoder_attn.out_proj.weight", dd), dd, L.wo_c, s);
    to_f16(P.get(p + "fc1.weight", fd), fd, L.w1, s);
    to_f16(P.get(p + "fc2.weight", fd), fd, L.w2, s);
    L.bo = P.get(p + "self_attn.out_proj.bias", d);
    L.bq_c = P.get(p + "encoder_attn.q_proj.bias", d);
    L.bv_c = P.get(p + "encoder_attn.v_proj.bias", d);
    L.bo_c = P.get(p + "encoder_attn.out_proj.bias", d);
    L.b1 = P.get(p + "fc1.bias", ff);
    L.b2 = P.get(p + "fc2.bias", d);
    L.ln1g = P.get(p + "self_attn_layer_norm.weight", d);
    L.ln1b = P.get(p + "self_attn_layer_norm.bias", d);
    L.ln2g = P.get(p + "encoder_attn_layer_norm.weight", d);
    L.ln2b = P.get(p + "encoder_attn_layer_norm.bias", d);
    L.ln3g = P.get(p + "final_layer_norm.weight", d);
    L.ln3b = P.get(p + "final_layer_norm.bias", d);
    if (xattn_supported(d, c.n_heads)) {
      const int64_t hd = (int64_t)c.n_heads * d;
      L.wqk.ensure(sizeof(_Float16) * hd * d);
      L.bqk.ensure(sizeof(float) * hd);
      const std::string e = p + "encoder_attn.";
      xattn_absorb(P.get(e + "q_proj.weight", dd), P.has(e + "q_proj.bias") ? P.get(e + "q_proj.bias", d) : nullptr,
                   P.get(e + "k_proj.weight", dd), d, c.n_heads, L.wqk.as<_Float16>(), L.bqk.as<float>(), s);
    }
  }
  JANUS_HIP(hipStreamSynchronize(s));
  w->prepared = true;
}

// The encoder's projections (M = B * 1500 rows): gemm_launch dispatches them to the
// 256 x 256-tile LDS-DMA kernel (gemm_big.hip) when N % 256 == 0 (base.en: every one).
static void enc_gemm(int epi, const GemmArgs& g, hipStream_t s) { gemm_launch(epi, g, s); }

static GemmArgs gargs(const _Float16* A, int64_t lda, const _Float16* W, int64_t ldw,
                      const float* bias, void* C, int64_t ldc, int M, int N, int K,
                      const float* R = nullptr, int64_t ldr = 0) {
  GemmArgs g;
  g.A = A; g.lda = lda; g.W = W; g.ldw = ldw; g.bias = bias; g.C = C; g.ldc = ldc;
  g.R = R; g.ldr = ldr; g.M = M; g.N = N; g.K = K;
  return g;
}

static void encode(janus_whisper* w, const _Float16* mel, int B, _Float16* out, hipStream_t s) {
  const auto& c = w->cfg;
  const int d = c.d_model, H = c.n_heads, Tm = 2 * c.n_audio_ctx, Te = c.n_audio_ctx;
  const int64_t M = (int64_t)B * Te;
  JANUS_CHECK(M < (1ll << 31), "encode: batch too large");
  w->ws_x1.ensure(sizeof(_Float16) * B * Tm * d);
  w->ws_x2.ensure(sizeof(_Float16) * M * d);
  w->ws_r.ensure(sizeof(float) * M * d);
  w->ws_a.ensure(sizeof(_Float16) * M * d);
  w->ws_qkv.ensure(sizeof(_Float16) * M * 3 * d);
  w->ws_o.ensure(sizeof(_Float16) * M * d);
  w->ws_f.ensure(sizeof(_Float16) * M * 4 * d);
  _Float16 *x1 = w->ws_x1.as<_Float16>(), *x2 = w->ws_x2.as<_Float16>();
  float* r = w->ws_r.as<float>();
  _Float16 *a = w->ws_a.as<_Float16>(), *qkv = w->ws_qkv.as<_Float16>(), *o = w->ws_o.as<_Float16>(),
           *f = w->ws_f.as<_Float16>();

  ConvArgs ca{};
  ca.in = mel; ca.in_bs = (int64_t)Tm * c.n_mels; ca.T_in = Tm; ca.Cin = c.n_mels;
  ca.w = w->conv1p.as<_Float16>(); ca.bias = w->params.get("encoder.conv1.bias", d);
  ca.out = x1; ca.out_bs = (int64_t)Tm * d; ca.T_out = Tm; ca.Cout = d;
  ca.res = nullptr; ca.res_bs = 0;
  ca.taps = 3; ca.dil = 1; ca.in_stride = 1; ca.in_off = -1; ca.out_stride = 1; ca.out_off = 0;
  ca.n_rows = Tm; ca.phases = 1; ca.pre_act = ACT_NONE; ca.post_act = ACT_GELU;
  ca.out_scale = 1.0f; ca.accumulate = 0; ca.B = B;
  conv_launch(ca, s);
  ConvArgs cb = ca;
  cb.in = x1; cb.in_bs = (int64_t)Tm * d; cb.T_in = Tm; cb.Cin = d;
  cb.w = w->conv2p.as<_Float16>(); cb.bias = w->params.get("encoder.conv2.bias", d);
  cb.out = x2; cb.out_bs = (int64_t)Te * d; cb.T_out = Te; cb.n_rows = Te; cb.in_stride = 2;
  cb.res = w->pos16.as<_Float16>(); cb.res_bs = 0;
  conv_launch(cb, s);
  cast_f16_f32_launch(x2, r, M * d, s);

  const float scale = 0.125f;  // head_dim 64 ** -0.5
  for (int l = 0; l < c.enc_layers; ++l) {
    EncLayer& L = w->enc[l];
    layernorm_launch(r, L.ln1g, L.ln1b, a, (int)M, d, 1e-5f, s);
    enc_gemm(EPI_F16, gargs(a, d, L.wqkv.as<_Float16>(), d, L.bqkv.as<float>(), qkv, 3 * d, (int)M, 3 * d, d), s);
    attention_launch(qkv, o, B, Te, H, scale, s);
    enc_gemm(EPI_RESID_F32, gargs(o, d, L.wo.as<_Float16>(), d, L.bo, r, d, (int)M, d, d, r, d), s);
    layernorm_launch(r, L.ln2g, L.ln2b, a, (int)M, d, 1e-5f, s);
    enc_gemm(EPI_GELU_F16, gargs(a, d, L.w1.as<_Float16>(), d, L.b1, f, 4 * d, (int)M, 4 * d, d), s);
    enc_gemm(EPI_RESID_F32, gargs(f, 4 * d, L.w2.as<_Float16>(), 4 * d, L.b2, r, d, (int)M, d, 4 * d, r, d), s);
  }
  layernorm_launch(r, w->params.get("encoder.layer_norm.weight", d),
                   w->params.get("encoder.layer_norm.bias", d), out, (int)M, d, 1e-5f, s);
}

static uint32_t float_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, sizeof(u));
  return u;
}

// Sampling (faster-whisper's temperature fallback, CTranslate2 generate(sampling_temperature=
// T, sampling_topk=0)): temperature > 0 draws each token from softmax(filtered logits / T)
// by Gumbel-max with per-row counter-based noise (seeds [host] uint32 [B]); null = greedy.
struct DecodeSampling {
  float temperature;
  const uint32_t* seeds;
  const float* temps = nullptr;   // host [B], per-row temperatures (overrides temperature)
};

// The deferred barrier-timeout check of the lane's last non-polling call (check_every 0):
// waits for that call's flag copy and throws if a persistent segment gave up at a barrier.
static void lane_check(DecLane& Z) {
  if (!Z.segerr_pending) return;
  Z.segerr_pending = false;
  JANUS_HIP(hipEventSynchronize(Z.ev_segerr));
  if (*Z.h_segerr) {
    *Z.h_segerr = 0;
    JANUS_HIP(hipMemset(Z.d_segbar.p, 0, sizeof(unsigned) * 256));
    JANUS_HIP(hipMemset(Z.d_segerr.p, 0, 256));
    throw Error("decode: a persistent decoder segment timed out at a grid barrier (grid not co-resident)");
  }
}

static void decode_greedy(janus_whisper* w, DecLane& Z, const _Float16* enc_in, int B, const janus_decode_options* opt,
                          const janus_decode_rows* rows, int32_t* tokens_out, int32_t* n_tokens_out,
                          float* sum_lp_out, float* nsp_out, hipStream_t s, LaneLatch* latch,
                          const DecodeSampling* smp = nullptr) {
  lane_check(Z);   // the previous non-polling call's flag first
  LaneArrival arrival(latch);
  const auto& c = w->cfg;
  const int d = c.d_model, H = c.n_heads, Te = c.n_audio_ctx, V = c.n_vocab, NC = c.n_text_ctx;
  // alternative paths (janus_decode_options.path_flags, 0 = the measured default)
  const uint32_t pf = opt->path_flags;
  auto path = [pf](uint32_t f) { return (pf & f) != 0; };
  // shared encoder rows (janus_decode_rows::enc_index): row b attends to enc_in row
  // enc_index[b] of n_enc; the absorbed cross-attention then reads each shared row once per
  // pair of decoder rows (xattn PAIR blocks), other paths get a per-row gathered copy
  const bool shared = rows && rows->enc_index;
  const int n_enc = shared ? rows->n_enc : B;
  std::vector<int4> h_pairs;
  if (shared) {
    JANUS_CHECK(n_enc >= 1, "decode: enc_index needs n_enc >= 1");
    for (int b = 0; b < B; ++b)
      JANUS_CHECK(rows->enc_index[b] >= 0 && rows->enc_index[b] < n_enc, "decode: enc_index out of range");
  }
  const bool pair_ok = shared && xattn_supported(d, H) && H <= 8 && d <= 512 && B <= kSkinnyMaxRows &&
                       !path(JANUS_DEC_PATH_NO_XABSORB) && !path(JANUS_DEC_PATH_NO_XPAIR);
  // rows sharing an encoder row (best_of = 5 hypotheses of a window): PAIR blocks
  // (xattn_kernel<PAIR>, two blocks per CU, the window's output read once per two rows).
  // GROUP blocks of up to 6 rows (xattn_group_kernel: one read for all hypotheses) are
  // opt-in, JANUS_XGROUP=1: measured slower in the fallback step (4 810 vs 4 380 ms per
  // step, two same-box pairs, profiles/r04_lanes_sweep_fallback_ab.json) — one block per
  // CU with three m-tiles of queries staged through LDS loses more than the reads it saves
  std::vector<int> h_groups;
  int grp_rows = 0;
  if (pair_ok) {
    std::vector<std::vector<int>> grp(n_enc);
    for (int b = 0; b < B; ++b) grp[rows->enc_index[b]].push_back(b);
    size_t maxg = 0;
    for (auto& g : grp) maxg = std::max(maxg, g.size());
    if (maxg > 2 && path(JANUS_DEC_PATH_XGROUP)) {
      grp_rows = (int)std::min<size_t>(6, maxg);
      for (int e = 0; e < n_enc; ++e)
        for (size_t i = 0; i < grp[e].size(); i += grp_rows) {
          h_groups.push_back(e);
          for (int j = 0; j < 7; ++j)
            h_groups.push_back(j < grp_rows && i + j < grp[e].size() ? grp[e][i + j] : -1);
        }
    } else {
      // rows grouped by encoder row, paired in row order within a group
      for (int e = 0; e < n_enc; ++e)
        for (size_t i = 0; i < grp[e].size(); i += 2)
          h_pairs.push_back(make_int4(grp[e][i], i + 1 < grp[e].size() ? grp[e][i + 1] : -1, e, 0));
    }
  }
  // the captured decode graphs bake in every pointer they read: the encoder output goes
  // to a context-owned buffer first (one ~0.1 ms device copy) so the graphs are reused
  // whatever buffer the caller's allocator handed out this time
  const int enc_rows = pair_ok ? n_enc : B;
  const int64_t erow = (int64_t)Te * d;
  Z.d_enc.ensure(sizeof(_Float16) * (int64_t)enc_rows * erow);
  if (shared && !pair_ok) {
    for (int b = 0; b < B; ++b)
      JANUS_HIP(hipMemcpyAsync(Z.d_enc.as<_Float16>() + (int64_t)b * erow, enc_in + (int64_t)rows->enc_index[b] * erow,
                               sizeof(_Float16) * erow, hipMemcpyDeviceToDevice, s));
  } else {
    JANUS_HIP(hipMemcpyAsync(Z.d_enc.p, enc_in, sizeof(_Float16) * (int64_t)enc_rows * erow,
                             hipMemcpyDeviceToDevice, s));
  }
  const _Float16* enc = Z.d_enc.as<_Float16>();
  const int npairs = (int)h_pairs.size();
  if (npairs > 0) {
    Z.d_xpairs.ensure(sizeof(int4) * npairs);
    JANUS_HIP(hipMemcpyAsync(Z.d_xpairs.p, h_pairs.data(), sizeof(int4) * npairs, hipMemcpyHostToDevice, s));
  }
  const int4* xpairs = npairs > 0 ? Z.d_xpairs.as<int4>() : nullptr;
  const int ngroups = (int)h_groups.size() / 8;
  if (ngroups > 0) {
    Z.d_xgroups.ensure(sizeof(int) * h_groups.size());
    JANUS_HIP(hipMemcpyAsync(Z.d_xgroups.p, h_groups.data(), sizeof(int) * h_groups.size(),
                             hipMemcpyHostToDevice, s));
  }
  const int* xgroups = ngroups > 0 ? Z.d_xgroups.as<int>() : nullptr;
  const int maxlen = opt->max_length;
  // per-row prompts (janus_decode_rows): row b samples from position plen[b]; all rows step
  // together from position 0, rows still inside their prompt keep the forced token
  const bool per_row = rows && rows->prompts;
  std::vector<int32_t> h_plen(B, opt->prompt_len);
  std::vector<int32_t> h_init((size_t)B * maxlen, -1);
  if (per_row) {
    JANUS_CHECK(rows->prompt_lens && rows->stride >= 1, "decode: per-row prompts need lengths and a stride");
    for (int b = 0; b < B; ++b) {
      h_plen[b] = rows->prompt_lens[b];
      JANUS_CHECK(h_plen[b] >= 1 && h_plen[b] <= rows->stride && h_plen[b] < maxlen,
                  "decode: per-row prompt length out of range");
      for (int i = 0; i < h_plen[b]; ++i) h_init[(size_t)b * maxlen + i] = rows->prompts[(size_t)b * rows->stride + i];
    }
  } else {
    JANUS_CHECK(opt->prompt && opt->prompt_len >= 1, "decode: missing prompt");
    for (int b = 0; b < B; ++b)
      for (int i = 0; i < opt->prompt_len; ++i) h_init[(size_t)b * maxlen + i] = opt->prompt[i];
  }
  // staggered rows (janus_decode_rows.pos_offset): rows with an offset > 0 continue the
  // previous call's state in the same slots (tokens, KV cache, counters, rule state); rows
  // with 0 start fresh and must be one contiguous range [f0, f1). Every row runs `steps`
  // positions from its own offset.
  const bool stagger = rows && rows->pos_offset;
  int f0 = 0, f1 = B, max_roff = 0;
  std::vector<int32_t> h_roff;
  if (stagger) {
    JANUS_CHECK(!shared && !(smp && smp->temperature > 0.f), "decode: staggered rows are greedy, unshared");
    h_roff.assign(rows->pos_offset, rows->pos_offset + B);
    f0 = B; f1 = 0;
    for (int b = 0; b < B; ++b) {
      JANUS_CHECK(h_roff[b] >= 0 && h_roff[b] < maxlen, "decode: pos_offset out of range");
      max_roff = std::max(max_roff, h_roff[b]);
      if (h_roff[b] == 0) { f0 = std::min(f0, b); f1 = std::max(f1, b + 1); }
    }
    if (f1 <= f0) f0 = f1 = 0;
    for (int b = f0; b < f1; ++b) JANUS_CHECK(h_roff[b] == 0, "decode: fresh rows must be contiguous");
  }
  JANUS_CHECK(!stagger || rows->steps >= 0, "decode: steps must be >= 0");
  const int steps = (stagger && rows->steps > 0) ? rows->steps : maxlen - 1;
  JANUS_CHECK(!stagger || max_roff + steps <= maxlen, "decode: pos_offset + steps > max_length");
  // a continuing row reads the tokens and KV rows its slot holds: only up to where the
  // previous calls left it (a larger offset would read unwritten tokens / KV rows)
  if (stagger) {
    for (int b = 0; b < B; ++b) {
      if (h_roff[b] == 0) continue;
      JANUS_CHECK((int)Z.stand.size() == B && Z.stand_maxlen == maxlen,
                  "decode: continuing rows need the previous call's batch size and max_length");
      JANUS_CHECK(h_roff[b] <= Z.stand[b],
                  "decode: row " + std::to_string(b) + " continues at pos_offset " + std::to_string(h_roff[b]) +
                      " but its slot stands at " + std::to_string(Z.stand[b]));
    }
  }
  // until this call completes, nothing may be continued (a failed call leaves stand empty)
  Z.stand.clear();
  const int min_plen = f1 > f0 ? *std::min_element(h_plen.begin() + f0, h_plen.begin() + f1) : 1;
  const int max_plen = f1 > f0 ? *std::max_element(h_plen.begin() + f0, h_plen.begin() + f1) : 1;
  JANUS_CHECK(min_plen >= 1 && max_plen < maxlen && maxlen <= NC,
              "decode: need 1 <= prompt_len < max_length <= n_text_ctx");
  const int64_t Me = (int64_t)B * Te;
  const int nl = c.dec_layers;
  Z.d_x.ensure(sizeof(float) * B * d);
  Z.d_a.ensure(sizeof(_Float16) * B * d);
  Z.d_qkv.ensure(sizeof(_Float16) * B * 3 * d);
  Z.d_o.ensure(sizeof(_Float16) * B * d);
  Z.d_q2.ensure(sizeof(_Float16) * B * d);
  Z.d_f.ensure(sizeof(_Float16) * B * 4 * d);
  Z.d_kc.ensure(sizeof(_Float16) * (int64_t)nl * B * NC * d);
  Z.d_vc.ensure(sizeof(_Float16) * (int64_t)nl * B * NC * d);

  Z.d_smask.ensure((V + 15) / 16 * 16);  // logits_partial_kernel reads 16 mask bytes per tile
  const int max_split = std::max(decode_split_count(Te), decode_split_count(NC));
  Z.d_part_o.ensure(sizeof(float) * (int64_t)B * max_split * d);
  Z.d_part_ml.ensure(sizeof(float) * (int64_t)B * max_split * H * 2);
  // cu_count: the CUs the caller's stream may use (a CU-masked partition); 0 = read it
  // from the stream's CU mask
  // (a caller's cu_count larger than its stream's CU mask is clamped to the mask)
  const int cus = opt->cu_count > 0 ? std::min(opt->cu_count, stream_cu_count(s)) : stream_cu_count(s);
  // launch geometry from the options (janus_decode_options.logits_blocks / msplit_rows_n;
  // measured defaults: DESIGN.md §5b / §5d)
  const int lg_cap = opt->logits_blocks > 0 ? opt->logits_blocks : cus;
  const int msplit_n = opt->msplit_rows_n > 0 ? opt->msplit_rows_n
                       : opt->msplit_rows_n < 0 ? 0 : (cus <= 128 ? 1024 : 0);
  auto dgargs = [&](auto&&... args) {
    GemmArgs g = gargs(args...);
    g.msplit_n = msplit_n;
    g.decode_rows = true;
    return g;
  };
  const int nblk = logits_partial_blocks(V, d, lg_cap);
  Z.d_parts.ensure(sizeof(LogitPart) * (int64_t)B * nblk);
  Z.d_rules.ensure(sizeof(RowRules) * B);
  float* part_o = Z.d_part_o.as<float>();
  float* part_ml = Z.d_part_ml.as<float>();
  Z.d_done.ensure(sizeof(int32_t) * B);
  Z.d_prompt.ensure(sizeof(int32_t) * B);   // per-row prompt lengths
  Z.d_tok.ensure(sizeof(int32_t) * (int64_t)B * maxlen);
  Z.d_ntok.ensure(sizeof(int32_t) * B);
  Z.d_slp.ensure(sizeof(float) * B);
  Z.d_nsp.ensure(sizeof(float) * B);
  int32_t* tokens = Z.d_tok.as<int32_t>();
  int32_t* n_tokens = Z.d_ntok.as<int32_t>();
  float* sum_lp = Z.d_slp.as<float>();
  Z.d_supp.ensure(sizeof(int32_t) * (opt->n_suppress > 0 ? opt->n_suppress : 1));
  float* x = Z.d_x.as<float>();
  _Float16 *a = Z.d_a.as<_Float16>(), *qkv = Z.d_qkv.as<_Float16>(), *o = Z.d_o.as<_Float16>(),
           *q2 = Z.d_q2.as<_Float16>(), *f = Z.d_f.as<_Float16>();
  int32_t* done = Z.d_done.as<int32_t>();

  // synchronous uploads: the host vectors die with this call (staggered: fresh rows only)
  if (f1 > f0) {
    JANUS_HIP(hipMemcpyAsync(Z.d_prompt.as<int32_t>() + f0, h_plen.data() + f0, sizeof(int32_t) * (f1 - f0),
                             hipMemcpyHostToDevice, s));
    JANUS_HIP(hipMemcpyAsync(tokens + (int64_t)f0 * maxlen, h_init.data() + (size_t)f0 * maxlen,
                             sizeof(int32_t) * (size_t)(f1 - f0) * maxlen, hipMemcpyHostToDevice, s));
  }
  Z.d_roff.ensure(sizeof(int32_t) * B);
  if (stagger)
    JANUS_HIP(hipMemcpyAsync(Z.d_roff.p, h_roff.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice, s));
  const int32_t* roff = stagger ? Z.d_roff.as<int32_t>() : nullptr;
  const bool sampling = smp && smp->temperature > 0.f;
  Z.d_seed.ensure(sizeof(uint32_t) * B);
  if (sampling) {
    JANUS_CHECK(smp->seeds, "decode: sampling needs per-row seeds");
    JANUS_HIP(hipMemcpyAsync(Z.d_seed.p, smp->seeds, sizeof(uint32_t) * B, hipMemcpyHostToDevice, s));
  }
  const bool row_temps = sampling && smp->temps;
  if (row_temps) {
    Z.h_itemp.resize(B);
    for (int b = 0; b < B; ++b) {
      JANUS_CHECK(smp->temps[b] >= 0.f, "decode: per-row temperatures must be >= 0");
      Z.h_itemp[b] = smp->temps[b] > 0.f ? 1.0f / smp->temps[b] : 0.f;   // 0: a greedy row
    }
    Z.d_itemp.ensure(sizeof(float) * B);
    JANUS_HIP(hipMemcpyAsync(Z.d_itemp.p, Z.h_itemp.data(), sizeof(float) * B, hipMemcpyHostToDevice, s));
  }
  if (opt->n_suppress > 0)
    JANUS_HIP(hipMemcpyAsync(Z.d_supp.p, opt->suppress, sizeof(int32_t) * opt->n_suppress,
                             hipMemcpyHostToDevice, s));
  JANUS_HIP(hipStreamSynchronize(s));
  build_mask_launch(Z.d_supp.as<int32_t>(), opt->n_suppress, Z.d_smask.as<uint8_t>(), V, s);
  if (f1 > f0) {
    init_counters_launch(done + f0, sum_lp + f0, n_tokens + f0, Z.d_nsp.as<float>() + f0, f1 - f0, s);
    rules_init_launch(Z.d_rules.as<RowRules>() + f0, f1 - f0, s);
  }

  // cross-attention: absorbed (stream enc itself, JANUS_DEC_PATH_NO_XABSORB restores per-layer K/V)
  const bool xabs = xattn_supported(d, H) && B <= kSkinnyMaxRows && !path(JANUS_DEC_PATH_NO_XABSORB);
  const int xsplit = xattn_split_count(Te, opt->xattn_splits);
  if (xabs) {
    Z.d_xqk.ensure(sizeof(_Float16) * B * H * d);
    Z.d_xc.ensure(sizeof(_Float16) * B * H * d);
    Z.d_xpc.ensure(sizeof(float) * (int64_t)B * xsplit * H * d);
    Z.d_xpml.ensure(sizeof(float) * (int64_t)B * xsplit * H * 2);
  }
  // cross-attention keys/values, once per window
  if (!xabs) {
    Z.d_ck.ensure(sizeof(_Float16) * (int64_t)nl * Me * d);
    Z.d_cv.ensure(sizeof(_Float16) * (int64_t)nl * Me * d);
  }
  for (int l = 0; l < nl && !xabs; ++l) {
    DecLayer& L = w->dec[l];
    _Float16* ck = Z.d_ck.as<_Float16>() + (int64_t)l * Me * d;
    _Float16* cv = Z.d_cv.as<_Float16>() + (int64_t)l * Me * d;
    gemm_launch(EPI_F16, dgargs(enc, d, L.wk_c.as<_Float16>(), d, nullptr, ck, d, (int)Me, d, d), s);
    gemm_launch(EPI_F16, dgargs(enc, d, L.wv_c.as<_Float16>(), d, L.bv_c, cv, d, (int)Me, d, d), s);
  }

  DecodeRules R;
  R.eot = opt->eot;
  R.suppress_blank = opt->suppress_blank;
  R.blank = opt->blank_token;
  R.ts_begin = opt->timestamp_begin;
  R.no_timestamps = opt->no_timestamps;
  R.max_initial_ts = opt->max_initial_timestamp_index;
  R.target = rows ? rows->no_speech_token : -1;
  // per-row temperatures: R.inv_temp only selects the sampling kernel (rows read their own)
  R.inv_temp = !sampling ? 0.f : smp->temps ? 1.0f : 1.0f / smp->temperature;
  const float scale = 0.125f;
  const float* pos_emb = w->params.get("decoder.embed_positions.weight", (int64_t)NC * d);
  std::vector<int32_t> h_done(B);
  // index of the first sampled token (earliest row); staggered continuing rows sample from
  // the first step on
  const int sample_begin = (stagger && f1 - f0 < B) ? 0 : min_plen;
  // JANUS_DEC_PATH_FUSED_LN (B <= 64): LayerNorm rides on the projections (row-statistic pieces
  // written by the producer of each residual row, normalised on load by the consumer).
  // Opt-in: with the 16-wave skinny GEMM the separate LayerNorm launch measured faster
  // (637.7 vs 660.8 ms per bench step) — the consumer ingests A as fp32.
  const bool fused_ln = B <= 64 && path(JANUS_DEC_PATH_FUSED_LN);
  Z.d_lnp.ensure(sizeof(float2) * B * (d / 16));
  float2* lnp = Z.d_lnp.as<float2>();
  auto lnargs = [&](const float* g, const float* bta, const _Float16* W, const float* bias,
                    void* C, int64_t ldc, int N, _Float16* kcp, _Float16* vcp, int pos) {
    SkinnyLnArgs p;
    p.x = x; p.ldx = d; p.part = lnp; p.gamma = g; p.beta = bta; p.eps = 1e-5f; p.W = W; p.ldw = d;
    p.bias = bias; p.C = C; p.ldc = ldc; p.M = B; p.N = N; p.K = d;
    p.kc = kcp; p.vc = vcp; p.pos = pos; p.n_ctx = NC; p.qkv_d = d;
    return p;
  };
  // JANUS_DEC_PATH_LN_FUSE (opt-in, B <= 64): LayerNorm handed off inside the producing kernel —
  // the residual GEMM's last block normalises the new rows (GemmArgs::ln_out, sc1 stores
  // + arrival counter), the embedding kernel normalises its row; no LayerNorm launches.
  // Measured slower than the separate launches (616.8 vs 536.5 ms per bench step): the
  // write-through stores and the serial tail cost more than the launch they save.
  const bool ln_fuse = B <= 64 && !fused_ln && d <= 512 && path(JANUS_DEC_PATH_LN_FUSE);
  // LayerNorm in the consuming projection's prologue (GemmArgs::lnin_x: each block
  // normalises its rows of x into an fp16 LDS tile; the vocabulary projection the final
  // LayerNorm) instead of a LayerNorm launch.
  // Per LayerNorm (bit mask, JANUS_DEC_PATH_LN_MASK(m) overrides): 1 = LN1 into the QKV
  // projection, 2 = LN2 into the absorbed query projection, 4 = LN3 into fc1, 8 = the final
  // LayerNorm into the vocabulary projection. Measured per kernel, decoder alone on 16 CUs
  // per XCD: QKV 9.2 us vs 5.6 + 5.1 (LayerNorm launch), fc1 8.6 vs 5.2 + 5.1, logits 49.4
  // vs 47.3 + 5.1 — but the absorbed query projection 16.1 vs 9.2 + 5.1 us: its 256
  // 64-row blocks would each normalise all 64 rows. Beside the vocoder (overlapped
  // step, decoder side): mask 0 303.5-308.7, 13 305.1-306.8, 9 304.0-304.2, 5 306.6-306.9
  // ms — within the box's noise; 9 (LN1 + final) is the default up to 64 rows. Above (the
  // staggered 2 x 64 rows) every LayerNorm is its own launch: decoder side 230-234 ms with
  // mask 0 against 235-241 (9), 245-249 (13), 265-269 (15) on one box
  // (profiles/r04_decoder_knobs.json): each prologue normalises its block's rows again.
  const int ln_pro_mask = (B <= kSkinnyMaxRows && d <= 512 && !fused_ln && !ln_fuse)
                              ? (path(JANUS_DEC_PATH_LN_PROLOGUE) ? (int)((pf >> 12) & 15u)
                                                                  : (B <= 64 ? 9 : 0))
                              : 0;
  // the embedding kernel owns whole rows (one block per utterance): it also writes the
  // first layer's LayerNorm of its row, one launch fewer per position
  // (JANUS_NO_EMBED_LN restores the separate launch)
  const bool embed_ln = !fused_ln && !ln_fuse && d <= 512 && !path(JANUS_DEC_PATH_NO_EMBED_LN);
  auto with_ln = [&](GemmArgs g, const float* lg, const float* lb, bool on) {
    if (on) { g.lnin_x = x; g.lnin_ldx = d; g.lnin_g = lg; g.lnin_b = lb; g.lnin_eps = 1e-5f; }
    return g;
  };
  const bool lnp2 = ln_pro_mask & 2, lnp3 = ln_pro_mask & 4, lnp_fin = ln_pro_mask & 8;
  // Opt-in (JANUS_DEC_PATH_RESID_LN): the attention output projections and the LayerNorm after
  // them (LN2 / LN3) in one launch (resid_ln_kernel: 16 rows per block over all d columns,
  // bit-identical to the residual GEMM + LayerNorm pair). Measured 72 ms per step SLOWER
  // on the decoder side (361 vs 289 ms): at B = 64 only 4 blocks stream the 0.5 MB weight
  // each, at ~25 GB/s per CU (≈ 24 µs per launch against 5.6 + 5.0 µs for the pair).
  const bool rln = B <= 64 && !fused_ln && !ln_fuse && resid_ln_supported(d, d) &&
                   path(JANUS_DEC_PATH_RESID_LN);
  const bool rln2 = rln && !lnp2, rln3 = rln && !lnp3;
  // the split merge fused into the per-head value projection (one launch) up to 64 rows;
  // above (the staggered 2 x 64 rows) the merge in the cross-attention's last split block
  // and a block-diagonal skinny projection measured faster (decoder side -1.5 / -2.9 ms
  // per step on two boxes, profiles/r04_decoder_knobs.json); bit-identical either way
  // (xattn_combine_vproj_kernel; JANUS_DEC_PATH_NO_CVP / _CVP force either form)
  const bool cvp = xattn_cvp_supported(d, H) && xsplit <= 16 && !path(JANUS_DEC_PATH_NO_CVP) &&
                   (B <= 64 || ngroups > 0 || path(JANUS_DEC_PATH_CVP));
  Z.d_lncnt.ensure(sizeof(int) * 64);  // one arrival counter per 16-row block (JANUS_DEC_PATH_LN_FUSE)
  JANUS_HIP(hipMemsetAsync(Z.d_lncnt.p, 0, sizeof(int) * 64, s));
  const float* fin_g = w->params.get("decoder.layer_norm.weight", d);
  const float* fin_b = w->params.get("decoder.layer_norm.bias", d);
  auto resid = [&](const _Float16* A, int K, const DevMem& W, const float* bias, const float* ng,
                   const float* nb) {
    GemmArgs g = dgargs(A, K, W.as<_Float16>(), K, bias, x, d, B, d, K, x, d);
    if (fused_ln) g.ln_part = lnp;
    if (ln_fuse) { g.ln_g = ng; g.ln_b = nb; g.ln_out = a; g.ln_cnt = Z.d_lncnt.as<int>(); }
    gemm_launch(EPI_RESID_F32, g, s);
  };
  auto resid_ln = [&](const _Float16* A, const DevMem& W, const float* bias, const float* ng,
                      const float* nb) {
    ResidLnArgs p;
    p.A = A; p.lda = d; p.W = W.as<_Float16>(); p.ldw = d; p.bias = bias;
    p.x = x; p.ldx = d; p.g = ng; p.b = nb; p.eps = 1e-5f; p.out = a;
    p.M = B; p.N = d; p.K = d;
    resid_ln_launch(p, s);
  };
  // the selection at pos and the embedding at pos + 1 in one launch (select_embed_kernel,
  // bit-identical; JANUS_DEC_PATH_NO_SEL_EMBED restores the two launches): a step from the first
  // sampled position on finds its row already embedded by the previous step's selection
  const bool fuse_se = !path(JANUS_DEC_PATH_NO_SEL_EMBED);
  JANUS_CHECK(!stagger || (!fused_ln && !ln_fuse && !rln && xabs),
              "decode: staggered rows run the default decoder kernels only");
  // persistent segments (dec_persist.hip, janus_decode_options.persistent): per layer the
  // launches between the self-attention and the cross-attention (O + residual, LN2, the
  // absorbed query projection) and between the cross-attention and the next layer's
  // self-attention (value projection, cross O + residual, LN3, fc1, fc2 + residual, LN1,
  // QKV) as two resident grids; the cross-attention then runs at one key split (its
  // output written directly). Shapes it does not cover keep the launch path.
  // (resident grids need every block co-resident: the kernels' occupancy must admit one
  // block per CU of the partition, and a multi-lane call, whose lanes run concurrently on
  // the same CUs, keeps the launch path)
  const int seg_grid = opt->persistent && latch == nullptr ? dec_seg_grid(B, cus, path(JANUS_DEC_PATH_SEG_2CU)) : 0;
  const bool persist = seg_grid > 0 && dec_seg_supported(d, H, B, cus) && dec_seg_resident(seg_grid, cus) &&
                       xabs && !shared && !fused_ln && !ln_fuse && !rln && ngroups == 0 && npairs == 0;
  // persistent = 2: segment B of layer l, the self-attention of l + 1 and its segment A as
  // ONE launch per layer step (dec_layer_kernel): 29 -> 19 launches per position; layer
  // 0's QKV, self-attention and segment A as one head kernel and the final LayerNorm as the
  // last segment B's phase: 16
  const bool layerk = persist && opt->persistent >= 2 && 2 * ((B + 1) / 2) <= 2 * seg_grid;
  // persistent = 3: the cross-attention as the head / layer kernel's last phase (10 launches
  // per position); the decoder side measured level with 16 (369.1-369.3 vs 368.4-369.4 ms
  // over 447 positions, profiles/r05_xattn_phase_ab.txt): a grid barrier costs what the
  // launch boundary it replaces did
  const bool xfuse = layerk && opt->persistent >= 3 && B <= 2 * seg_grid;
  // odd layers' cross-attention sweeps the encoder output's key chunks last to first, so it
  // starts on what the layer before it read last, still in the Infinity Cache (at 256 rows a
  // layer reads 393 MB, past its 256 MB): decoder 1472 -> 1394 us per position in the
  // staggered step (profiles/r06_xattn_ab.txt); JANUS_DEC_PATH_XFWD keeps every sweep forwards
  const bool xrev = !path(JANUS_DEC_PATH_XFWD);
  if (persist) {
    Z.d_omid.ensure(sizeof(_Float16) * B * d);
    if (!Z.d_segbar.p) {  // barrier counters start at zero; the kernels leave them zeroed
      Z.d_segbar.ensure(sizeof(unsigned) * 256);
      JANUS_HIP(hipMemsetAsync(Z.d_segbar.p, 0, sizeof(unsigned) * 256, s));
    }
    if (!Z.d_segerr.p) {
      Z.d_segerr.ensure(256);
      JANUS_HIP(hipMemsetAsync(Z.d_segerr.p, 0, 256, s));
    }
  }
  auto seg_args = [&](int l, int pos) {
    DecLayer& L = w->dec[l];
    DecSegArgs g{};
    g.B = B; g.MT = dec_seg_mtiles(B); g.x = x;
    g.o = o; g.wo = L.wo.as<_Float16>(); g.bo = L.bo; g.ln2g = L.ln2g; g.ln2b = L.ln2b;
    g.wqk = L.wqk.as<_Float16>(); g.bqk = L.bqk.as<float>(); g.xqk = Z.d_xqk.as<_Float16>();
    g.xc = Z.d_xc.as<_Float16>(); g.wv = L.wv_c.as<_Float16>(); g.bv = L.bv_c; g.omid = Z.d_omid.as<_Float16>();
    g.woc = L.wo_c.as<_Float16>(); g.boc = L.bo_c; g.ln3g = L.ln3g; g.ln3b = L.ln3b;
    g.w1 = L.w1.as<_Float16>(); g.b1 = L.b1; g.f = f; g.w2 = L.w2.as<_Float16>(); g.b2 = L.b2;
    if (l + 1 < nl) {
      DecLayer& N = w->dec[l + 1];
      g.ln1g = N.ln1g; g.ln1b = N.ln1b; g.wqkv = N.wqkv.as<_Float16>(); g.bqkv = N.bqkv.as<float>();
      g.qkv = qkv;
      g.kc = Z.d_kc.as<_Float16>() + (int64_t)(l + 1) * B * NC * d;
      g.vc = Z.d_vc.as<_Float16>() + (int64_t)(l + 1) * B * NC * d;
    }
    g.pos = pos; g.n_ctx = NC; g.roff = roff;
    g.bar = Z.d_segbar.as<unsigned>(); g.err = Z.d_segerr.as<unsigned>();
    g.prof = dec_seg_prof_target(l);
    if (layerk && l + 1 == nl && !lnp_fin) {  // the final LayerNorm as the last segment's phase
      g.fing = fin_g; g.finb = fin_b; g.fin_out = a;
    }
    if (xfuse) { g.enc = enc; g.Te = Te; }  // the cross-attention as the layer / head kernel's last phase
    return g;
  };
  // layer 0's head kernel: segment A args of layer 0 with layer 0's own LN1 / QKV / cache
  auto head_args = [&](int pos) {
    DecSegArgs g = seg_args(0, pos);
    DecLayer& L0 = w->dec[0];
    g.ln1g = L0.ln1g; g.ln1b = L0.ln1b; g.wqkv = L0.wqkv.as<_Float16>(); g.bqkv = L0.bqkv.as<float>();
    g.qkv = qkv; g.kc = Z.d_kc.as<_Float16>(); g.vc = Z.d_vc.as<_Float16>();
    g.fing = nullptr; g.finb = nullptr; g.fin_out = nullptr;
    return g;
  };
  auto step = [&](int pos) {
    if (!(fuse_se && pos >= sample_begin && pos > 0))
      embed_launch(w->tok16.as<_Float16>(), pos_emb, tokens, maxlen, pos, d, x,
                   fused_ln ? lnp : nullptr, B, s, w->dec[0].ln1g, w->dec[0].ln1b,
                   (ln_fuse || (embed_ln && !layerk)) ? a : nullptr, roff);
    for (int l = 0; l < nl; ++l) {
      DecLayer& L = w->dec[l];
      _Float16* kc = Z.d_kc.as<_Float16>() + (int64_t)l * B * NC * d;
      _Float16* vc = Z.d_vc.as<_Float16>() + (int64_t)l * B * NC * d;
      _Float16* ck = Z.d_ck.as<_Float16>() + (int64_t)l * Me * d;
      _Float16* cv = Z.d_cv.as<_Float16>() + (int64_t)l * Me * d;
      if (persist && (l > 0 || layerk)) {
        // q and this layer's K/V cache row came from the previous layer's segment B (layer
        // 0 with the layer kernel: from the head kernel below)
      } else if (fused_ln) {
        gemm_skinny_ln_launch(EPI_QKV, lnargs(L.ln1g, L.ln1b, L.wqkv.as<_Float16>(), L.bqkv.as<float>(),
                                              qkv, 3 * d, 3 * d, kc, vc, pos), s);
      } else {
        // layer 0's LN1 comes from the embedding kernel when embed_ln
        const bool lnp1 = (ln_pro_mask & 1) && !(embed_ln && l == 0);
        if (!ln_fuse && !lnp1 && !(embed_ln && l == 0))
          layernorm_launch(x, L.ln1g, L.ln1b, a, B, d, 1e-5f, s);
        if (B <= kSkinnyMaxRows) {
          GemmArgs g = with_ln(dgargs(a, d, L.wqkv.as<_Float16>(), d, L.bqkv.as<float>(), qkv, 3 * d, B, 3 * d, d),
                               L.ln1g, L.ln1b, lnp1);
          g.kc = kc; g.vc = vc; g.pos = pos; g.n_ctx = NC; g.qkv_d = d;
          g.roff = roff;
          gemm_launch(EPI_QKV, g, s);
        } else {
          JANUS_CHECK(!stagger, "decode: staggered rows need B <= kSkinnyMaxRows");
          gemm_launch(EPI_F16, dgargs(a, d, L.wqkv.as<_Float16>(), d, L.bqkv.as<float>(), qkv, 3 * d, B, 3 * d, d), s);
          kv_store_launch(qkv, d, pos, NC, kc, vc, B, s);
        }
      }
      // (layer kernel: layers > 0 got their self-attention and segment A in the previous
      // layer's launch)
      if (!layerk)
        decode_attention_split_launch(qkv, 3 * d, kc, vc, (int64_t)NC * d, d, pos + 1, o, d, B, H, scale,
                                      part_o, part_ml, s, roff, max_roff);
      if (persist) {
        const DecSegArgs g = seg_args(l, pos);
        if (!layerk) dec_seg_a_launch(g, seg_grid, s);
        else if (l == 0) dec_head_launch(head_args(pos), seg_grid, s);
        if (!xfuse)  // (persistent 3: the cross-attention ran as the head / layer kernel's last phase)
          xattn_launch(g.xqk, enc, B, Te, d, H, 1, Z.d_xpc.as<float>(), Z.d_xpml.as<float>(), Z.d_xc.as<_Float16>(),
                       s, true, nullptr, 0, xrev && (l & 1));
        if (layerk && l + 1 < nl) {
          DecLayer& N = w->dec[l + 1];
          const DecSegNext nx{N.wo.as<_Float16>(), N.bo, N.ln2g, N.ln2b, N.wqk.as<_Float16>(), N.bqk.as<float>()};
          dec_layer_launch(g, nx, seg_grid, s);
        } else {
          dec_seg_b_launch(g, seg_grid, s);
        }
        continue;
      }
      if (rln2) resid_ln(o, L.wo, L.bo, L.ln2g, L.ln2b);
      else resid(o, d, L.wo, L.bo, L.ln2g, L.ln2b);
      if (xabs) {
        const int hd = H * d;
        _Float16* xqk = Z.d_xqk.as<_Float16>();
        _Float16* xc = Z.d_xc.as<_Float16>();
        if (fused_ln) {
          gemm_skinny_ln_launch(EPI_F16, lnargs(L.ln2g, L.ln2b, L.wqk.as<_Float16>(), L.bqk.as<float>(),
                                                xqk, hd, hd, nullptr, nullptr, pos), s);
        } else {
          if (!ln_fuse && !lnp2 && !rln2) layernorm_launch(x, L.ln2g, L.ln2b, a, B, d, 1e-5f, s);
          gemm_launch(EPI_F16, with_ln(dgargs(a, d, L.wqk.as<_Float16>(), d, L.bqk.as<float>(), xqk, hd, B, hd, d),
                                       L.ln2g, L.ln2b, lnp2), s);
        }
        // o_h = c_h Wv_h^T + bv_h (block-diagonal over heads), then x += o Wo^T + bo; the
        // split merge and the value projection in one launch (cvp) where supported
        JANUS_CHECK(!xgroups || cvp, "decode: shared-encoder groups need the fused merge (no JANUS_DEC_PATH_NO_CVP)");
        if (xgroups)
          xattn_group_launch(xqk, enc, Te, d, H, xsplit, Z.d_xpc.as<float>(), Z.d_xpml.as<float>(), s,
                             xgroups, ngroups, grp_rows);
        else
          xattn_launch(xqk, enc, B, Te, d, H, xsplit, Z.d_xpc.as<float>(), Z.d_xpml.as<float>(), xc, s,
                       !cvp, xpairs, npairs);
        if (cvp) {
          xattn_combine_vproj_launch(Z.d_xpc.as<float>(), Z.d_xpml.as<float>(), xsplit, B, H, d,
                                     L.wv_c.as<_Float16>(), L.bv_c, o, d, s);
        } else {
          GemmArgs gv = dgargs(xc, hd, L.wv_c.as<_Float16>(), d, L.bv_c, o, d, B, d, d);
          gv.a_group_cols = 64;
          gemm_launch(EPI_F16, gv, s);
        }
        if (rln3) resid_ln(o, L.wo_c, L.bo_c, L.ln3g, L.ln3b);
        else resid(o, d, L.wo_c, L.bo_c, L.ln3g, L.ln3b);
      } else {
        if (fused_ln) {
          gemm_skinny_ln_launch(EPI_F16, lnargs(L.ln2g, L.ln2b, L.wq_c.as<_Float16>(), L.bq_c, q2, d, d,
                                                nullptr, nullptr, pos), s);
        } else {
          if (!ln_fuse && !lnp2 && !rln2) layernorm_launch(x, L.ln2g, L.ln2b, a, B, d, 1e-5f, s);
          gemm_launch(EPI_F16, with_ln(dgargs(a, d, L.wq_c.as<_Float16>(), d, L.bq_c, q2, d, B, d, d),
                                       L.ln2g, L.ln2b, lnp2), s);
        }
        decode_attention_split_launch(q2, d, ck, cv, (int64_t)Te * d, d, Te, o, d, B, H, scale, part_o,
                                      part_ml, s);
        if (rln3) resid_ln(o, L.wo_c, L.bo_c, L.ln3g, L.ln3b);
        else resid(o, d, L.wo_c, L.bo_c, L.ln3g, L.ln3b);
      }
      if (fused_ln) {
        gemm_skinny_ln_launch(EPI_GELU_F16, lnargs(L.ln3g, L.ln3b, L.w1.as<_Float16>(), L.b1, f, 4 * d,
                                                   4 * d, nullptr, nullptr, pos), s);
      } else {
        if (!ln_fuse && !lnp3 && !rln3) layernorm_launch(x, L.ln3g, L.ln3b, a, B, d, 1e-5f, s);
        gemm_launch(EPI_GELU_F16, with_ln(dgargs(a, d, L.w1.as<_Float16>(), d, L.b1, f, 4 * d, B, 4 * d, d),
                                          L.ln3g, L.ln3b, lnp3), s);
      }
      // next LayerNorm: the following layer's LN1, or the decoder's final LN
      resid(f, 4 * d, L.w2, L.b2, l + 1 < nl ? w->dec[l + 1].ln1g : fin_g,
            l + 1 < nl ? w->dec[l + 1].ln1b : fin_b);
    }
    if (pos + 1 < sample_begin) return;  // still inside the prompt
    if (!ln_fuse && !lnp_fin && !layerk) layernorm_launch(x, fin_g, fin_b, a, B, d, 1e-5f, s);
    logits_partial_launch(a, d, w->tok16.as<_Float16>(), d, V, B, R, Z.d_smask.as<uint8_t>(),
                          Z.d_rules.as<RowRules>(), Z.d_parts.as<LogitPart>(), s,
                          lnp_fin ? x : nullptr, d, fin_g, fin_b, lg_cap,
                          sampling ? Z.d_seed.as<uint32_t>() : nullptr, pos,
                          row_temps ? Z.d_itemp.as<float>() : nullptr);
    if (fuse_se && pos + 1 < maxlen - 1)
      select_embed_launch(Z.d_parts.as<LogitPart>(), nblk, R, Z.d_rules.as<RowRules>(), tokens,
                          maxlen, pos, done, sum_lp, n_tokens, B, s, Z.d_prompt.as<int32_t>(),
                          Z.d_nsp.as<float>(), w->tok16.as<_Float16>(), pos_emb, d, x,
                          fused_ln ? lnp : nullptr, w->dec[0].ln1g, w->dec[0].ln1b,
                          (ln_fuse || (embed_ln && !layerk)) ? a : nullptr, roff);
    else
      select_partials_launch(Z.d_parts.as<LogitPart>(), nblk, R, Z.d_rules.as<RowRules>(), tokens,
                             maxlen, pos, done, sum_lp, n_tokens, B, s, Z.d_prompt.as<int32_t>(),
                             Z.d_nsp.as<float>(), roff);
  };
  const bool use_graph = !path(JANUS_DEC_PATH_NO_GRAPH);
  const int chunk = opt->check_every > 0 ? opt->check_every : 16;
  // every device pointer a captured kernel touches, plus the shape: the graph cache key
  const std::vector<int64_t> base_key = {
      B, maxlen, sample_begin, chunk, (int64_t)x, (int64_t)a, (int64_t)qkv, (int64_t)o,
      (int64_t)q2, (int64_t)f, (int64_t)Z.d_kc.p, (int64_t)Z.d_vc.p, (int64_t)Z.d_ck.p,
      (int64_t)Z.d_cv.p, (int64_t)part_o, (int64_t)part_ml, (int64_t)Z.d_parts.p,
      (int64_t)Z.d_rules.p, (int64_t)Z.d_lnp.p, (int64_t)fused_ln, (int64_t)ln_fuse, (int64_t)ln_pro_mask, (int64_t)embed_ln, (int64_t)rln, (int64_t)cvp, (int64_t)fuse_se, (int64_t)nblk, (int64_t)msplit_n, (int64_t)Z.d_lncnt.p, (int64_t)xabs, (int64_t)xsplit, (int64_t)Z.d_xqk.p,
      (int64_t)Z.d_xc.p, (int64_t)Z.d_xpc.p, (int64_t)Z.d_xpml.p, (int64_t)enc, (int64_t)tokens, (int64_t)done, (int64_t)sum_lp,
      (int64_t)n_tokens, (int64_t)Z.d_smask.p, R.eot, R.ts_begin, R.suppress_blank, R.blank,
      R.no_timestamps, R.max_initial_ts, R.target, (int64_t)Z.d_prompt.p, (int64_t)Z.d_nsp.p,
      (int64_t)sampling, (int64_t)float_bits(R.inv_temp), (int64_t)Z.d_seed.p, (int64_t)row_temps,
      (int64_t)Z.d_itemp.p, (int64_t)xpairs,
      (int64_t)npairs, (int64_t)xgroups, (int64_t)ngroups, (int64_t)grp_rows, (int64_t)roff,
      (int64_t)max_roff, (int64_t)persist + (int64_t)layerk + (int64_t)xfuse, (int64_t)seg_grid, (int64_t)Z.d_omid.p, (int64_t)Z.d_segbar.p,
      (int64_t)Z.d_segerr.p};
  arrival.now();  // all lanes' allocations done: captures may start
  if (Z.graphs.size() > 512) {
    for (auto& kv : Z.graphs) (void)hipGraphExecDestroy(kv.second);
    Z.graphs.clear();
    Z.graph_nodes.clear();
  }
  Z.last_positions = 0;
  Z.last_launches = 0;
  for (int p0 = 0; p0 < steps; p0 += chunk) {
    const int n = std::min(chunk, steps - p0);
    Z.last_positions += n;
    if (use_graph) {
      std::vector<int64_t> key = base_key;
      key.push_back(p0);
      key.push_back(n);
      auto it = Z.graphs.find(key);
      if (it == Z.graphs.end()) {
        hipGraph_t g;
        JANUS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        try {
          for (int pos = p0; pos < p0 + n; ++pos) step(pos);
        } catch (...) {
          hipGraph_t dead;
          (void)hipStreamEndCapture(s, &dead);
          if (dead) (void)hipGraphDestroy(dead);
          throw;
        }
        JANUS_HIP(hipStreamEndCapture(s, &g));
        size_t nodes = 0;
        JANUS_HIP(hipGraphGetNodes(g, nullptr, &nodes));
        hipGraphExec_t ge;
        JANUS_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        JANUS_HIP(hipGraphDestroy(g));
        it = Z.graphs.emplace(key, ge).first;
        Z.graph_nodes[key] = nodes;
      }
      JANUS_HIP(hipGraphLaunch(it->second, s));
      Z.last_launches += (int64_t)Z.graph_nodes[key];
    } else {
      for (int pos = p0; pos < p0 + n; ++pos) step(pos);
    }
    if (opt->check_every > 0 && p0 + n >= sample_begin) {
      JANUS_HIP(hipMemcpyAsync(h_done.data(), done, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
      JANUS_HIP(hipStreamSynchronize(s));
      bool all = true;
      for (int b = 0; b < B; ++b) all = all && h_done[b];
      if (all) break;  // remaining positions keep -1; callers stop at the first eot
    }
  }
  if (persist && opt->check_every <= 0) {   // the check deferred: the call does not wait
    if (!Z.h_segerr) JANUS_HIP(hipHostMalloc((void**)&Z.h_segerr, sizeof(uint32_t), hipHostMallocDefault));
    if (!Z.ev_segerr) JANUS_HIP(hipEventCreateWithFlags(&Z.ev_segerr, hipEventDisableTiming));
    JANUS_HIP(hipMemcpyAsync(Z.h_segerr, Z.d_segerr.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    JANUS_HIP(hipEventRecord(Z.ev_segerr, s));
    Z.segerr_pending = true;
  } else if (persist) {  // a segment whose grid never became co-resident gave up at a barrier
    uint32_t herr = 0;
    JANUS_HIP(hipMemcpyAsync(&herr, Z.d_segerr.p, sizeof(herr), hipMemcpyDeviceToHost, s));
    JANUS_HIP(hipStreamSynchronize(s));
    if (herr) {
      JANUS_HIP(hipMemsetAsync(Z.d_segbar.p, 0, sizeof(unsigned) * 256, s));
      JANUS_HIP(hipMemsetAsync(Z.d_segerr.p, 0, 256, s));
      JANUS_HIP(hipStreamSynchronize(s));
      throw Error("decode: a persistent decoder segment timed out at a grid barrier (grid not co-resident)");
    }
  }
  // every row ran Z.last_positions positions from its offset (the early exit stops all rows
  // together); janus_whisper_decode_stand reports it, stagger plans continue from there
  Z.stand.assign(B, 0);
  for (int b = 0; b < B; ++b) Z.stand[b] = (stagger ? h_roff[b] : 0) + Z.last_positions;
  Z.stand_maxlen = maxlen;
  JANUS_HIP(hipMemcpyAsync(tokens_out, tokens, sizeof(int32_t) * (int64_t)B * maxlen,
                           hipMemcpyDeviceToDevice, s));
  JANUS_HIP(hipMemcpyAsync(n_tokens_out, n_tokens, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s));
  JANUS_HIP(hipMemcpyAsync(sum_lp_out, sum_lp, sizeof(float) * B, hipMemcpyDeviceToDevice, s));
  if (nsp_out)
    JANUS_HIP(hipMemcpyAsync(nsp_out, Z.d_nsp.p, sizeof(float) * B, hipMemcpyDeviceToDevice, s));
}

}  // namespace janus

using namespace janus;

extern "C" int janus_whisper_create(const janus_whisper_config* cfg, janus_whisper** out) {
  return guarded([&] {
    JANUS_CHECK(cfg && out, "null argument");
    JANUS_CHECK(cfg->d_model % 64 == 0 && cfg->n_heads * 64 == cfg->d_model,
                "whisper: head_dim must be 64");
    JANUS_CHECK(cfg->n_mels == 80, "whisper: 80 mel bins supported");
    auto* w = new janus_whisper();
    w->cfg = *cfg;
    *out = w;
  });
}

extern "C" int janus_whisper_destroy(janus_whisper* w) {
  return guarded([&] {
    if (w) {
      (void)hipDeviceSynchronize();
      delete w;
    }
  });
}

extern "C" int janus_whisper_set_tensor(janus_whisper* w, const char* name, const float* host,
                                        int64_t numel) {
  return guarded([&] {
    JANUS_CHECK(w && name && host && numel > 0, "bad argument");
    std::lock_guard<std::mutex> lk(w->mu);
    w->params.set(name, host, numel);
    w->prepared = false;
  });
}

static void logmel_frames(janus_whisper* w, const float* pcm, const int64_t* offsets, int batch,
                          int decim, int frames, float* logmel, uint16_t* mel, hipStream_t s) {
  float* lm = logmel;
  if (!lm) {
    w->ws_logmel.ensure(sizeof(float) * (int64_t)batch * frames * 80);
    lm = w->ws_logmel.as<float>();
  }
  w->ws_maxkey.ensure(sizeof(uint32_t) * (batch > 0 ? batch : 1));
  mel_launch(pcm, offsets, batch, w->params.get("mel.basis", 400 * 416),
             w->params.get("mel.filters", 208 * 80), lm, w->ws_maxkey.as<uint32_t>(), frames,
             decim, s);
  mel_normalize_launch(lm, w->ws_maxkey.as<uint32_t>(), reinterpret_cast<_Float16*>(mel), offsets,
                       decim, batch, frames, 80, 80, s);
}

extern "C" int janus_whisper_logmel(janus_whisper* w, const float* pcm, const int64_t* offsets,
                                    int batch, int decim, float* logmel, uint16_t* mel,
                                    void* stream) {
  return guarded([&] {
    JANUS_CHECK(w && pcm && offsets && mel, "null argument");
    std::lock_guard<std::mutex> lk(w->mu);
    logmel_frames(w, pcm, offsets, batch, decim, 2 * w->cfg.n_audio_ctx, logmel, mel,
                  (hipStream_t)stream);
  });
}

extern "C" int janus_whisper_logmel_frames(janus_whisper* w, const float* pcm,
                                           const int64_t* offsets, int batch, int decim,
                                           int frames, uint16_t* mel, void* stream) {
  return guarded([&] {
    JANUS_CHECK(w && pcm && offsets && mel, "null argument");
    JANUS_CHECK(frames >= 1 && (int64_t)batch * frames * 80 < (1ll << 40), "bad frame count");
    std::lock_guard<std::mutex> lk(w->mu);
    logmel_frames(w, pcm, offsets, batch, decim, frames, nullptr, mel, (hipStream_t)stream);
  });
}

extern "C" int janus_whisper_encode(janus_whisper* w, const uint16_t* mel, int batch, uint16_t* enc,
                                    void* stream) {
  return guarded([&] {
    JANUS_CHECK(w && mel && enc, "null argument");
    std::lock_guard<std::mutex> lk(w->mu);
    hipStream_t s = (hipStream_t)stream;
    prepare(w, s);
    encode(w, reinterpret_cast<const _Float16*>(mel), batch, reinterpret_cast<_Float16*>(enc), s);
  });
}

extern "C" int janus_whisper_decode_greedy(janus_whisper* w, const uint16_t* enc, int batch,
                                           const janus_decode_options* opt, int32_t* tokens,
                                           int32_t* n_tokens, float* sum_logprob, void* stream) {
  return janus_whisper_decode_greedy_ex(w, enc, batch, opt, nullptr, tokens, n_tokens, sum_logprob,
                                        nullptr, stream);
}

static int decode_entry(janus_whisper* w, const uint16_t* enc, int batch,
                        const janus_decode_options* opt, const janus_decode_rows* rows,
                        int32_t* tokens, int32_t* n_tokens, float* sum_logprob,
                        float* no_speech_prob, void* stream, const DecodeSampling* smp);

extern "C" int janus_whisper_decode_greedy_ex(janus_whisper* w, const uint16_t* enc, int batch,
                                              const janus_decode_options* opt,
                                              const janus_decode_rows* rows, int32_t* tokens,
                                              int32_t* n_tokens, float* sum_logprob,
                                              float* no_speech_prob, void* stream) {
  return decode_entry(w, enc, batch, opt, rows, tokens, n_tokens, sum_logprob, no_speech_prob, stream,
                      nullptr);
}

extern "C" int janus_whisper_decode_sample_ex(janus_whisper* w, const uint16_t* enc, int batch,
                                              const janus_decode_options* opt,
                                              const janus_decode_rows* rows, float temperature,
                                              const uint32_t* seeds, int32_t* tokens,
                                              int32_t* n_tokens, float* sum_logprob,
                                              float* no_speech_prob, void* stream) {
  if (!(temperature > 0.f) || !seeds) {
    set_error("decode_sample: temperature must be > 0 and seeds non-null");
    return -1;
  }
  const DecodeSampling smp{temperature, seeds};
  return decode_entry(w, enc, batch, opt, rows, tokens, n_tokens, sum_logprob, no_speech_prob, stream,
                      &smp);
}

extern "C" int janus_whisper_decode_sample_rows_ex(janus_whisper* w, const uint16_t* enc, int batch,
                                                   const janus_decode_options* opt,
                                                   const janus_decode_rows* rows, const float* temperatures,
                                                   const uint32_t* seeds, int32_t* tokens,
                                                   int32_t* n_tokens, float* sum_logprob,
                                                   float* no_speech_prob, void* stream) {
  if (!temperatures || !seeds || batch <= 0) {
    set_error("decode_sample_rows: temperatures and seeds must be non-null");
    return -1;
  }
  for (int b = 0; b < batch; ++b)
    if (!(temperatures[b] >= 0.f)) {
      set_error("decode_sample_rows: every temperature must be >= 0");
      return -1;
    }
  const DecodeSampling smp{1.0f, seeds, temperatures};
  return decode_entry(w, enc, batch, opt, rows, tokens, n_tokens, sum_logprob, no_speech_prob, stream,
                      &smp);
}

extern "C" int janus_whisper_decode_stand_slot(janus_whisper* w, int slot, int32_t* stand, int batch) {
  return guarded([&] {
    JANUS_CHECK(w && stand, "null argument");
    std::lock_guard<std::mutex> lk(w->mu);
    JANUS_CHECK(slot >= 0 && slot < (int)w->lanes.size() && (int)w->lanes[slot]->stand.size() == batch,
                "decode_stand: no completed decode of this batch size in this slot");
    std::copy(w->lanes[slot]->stand.begin(), w->lanes[slot]->stand.end(), stand);
  });
}

extern "C" int janus_whisper_decode_check(janus_whisper* w, int slot) {
  return guarded([&] {
    JANUS_CHECK(w, "null argument");
    std::lock_guard<std::mutex> lk(w->mu);
    JANUS_CHECK(slot >= 0 && slot < 8, "decode_check: slot must be 0 .. 7");
    if (slot < (int)w->lanes.size()) lane_check(*w->lanes[slot]);
  });
}

extern "C" int janus_whisper_decode_stand(janus_whisper* w, int32_t* stand, int batch) {
  return janus_whisper_decode_stand_slot(w, 0, stand, batch);
}

extern "C" int janus_whisper_decode_info(janus_whisper* w, int32_t* positions, int64_t* launches) {
  return guarded([&] {
    JANUS_CHECK(w && positions && launches, "null argument");
    std::lock_guard<std::mutex> lk(w->mu);
    const int sl = w->last_slot < (int)w->lanes.size() ? w->last_slot : 0;
    *positions = w->lanes.empty() ? 0 : w->lanes[sl]->last_positions;
    *launches = w->lanes.empty() ? 0 : w->lanes[sl]->last_launches;
  });
}

static int decode_entry(janus_whisper* w, const uint16_t* enc, int batch,
                        const janus_decode_options* opt, const janus_decode_rows* rows,
                        int32_t* tokens, int32_t* n_tokens, float* sum_logprob,
                        float* no_speech_prob, void* stream, const DecodeSampling* smp) {
  return guarded([&] {
    JANUS_CHECK(w && enc && opt && tokens && n_tokens && sum_logprob, "null argument");
    JANUS_CHECK(batch >= 1, "decode: batch must be >= 1");
    std::lock_guard<std::mutex> lk(w->mu);
    hipStream_t s = (hipStream_t)stream;
    prepare(w, s);
    const _Float16* e = reinterpret_cast<const _Float16*>(enc);
    // lanes: janus_decode_options.lanes (default 1). Two half-batch lanes measured slower at B = 64
    // (428.7 vs 419.6 ms per bench step): the skinny projections are weight-stream
    // launches, so each lane re-streams every weight matrix, and the cross-attention
    // already saturates HBM.
    int nlanes = opt->lanes > 0 ? opt->lanes : 1;
    nlanes = std::max(1, std::min(nlanes, std::min(batch, 8)));
    // shared encoder rows / staggered rows: one lane holds them all (and its slots' state)
    if (rows && (rows->enc_index || rows->pos_offset)) nlanes = 1;
    // a state slot other than 0 (janus_decode_options.state_slot) is one lane of its own
    JANUS_CHECK(opt->state_slot >= 0 && opt->state_slot < 8, "decode: state_slot must be 0 .. 7");
    const int slot = opt->state_slot;
    if (slot > 0) nlanes = 1;
    // storage: state slots 0..7 are lanes[0..7]; the extra workers of a multi-lane call
    // (lanes 1..7) live in lanes[8..14], so they never overwrite a slot's KV caches,
    // tokens, graphs or stand (the staggered step's fallback keeps state in slot 1)
    auto lane_of = [](int i) { return i == 0 ? 0 : 7 + i; };
    const int need = std::max(slot + 1, nlanes > 1 ? lane_of(nlanes - 1) + 1 : 1);
    while ((int)w->lanes.size() < need) w->lanes.emplace_back(new DecLane());
    w->last_slot = slot;
    if (nlanes == 1 && (s != nullptr || slot > 0)) {
      JANUS_CHECK(s != nullptr, "decode: a state slot > 0 needs a non-null stream");
      decode_greedy(w, *w->lanes[slot], e, batch, opt, rows, tokens, n_tokens, sum_logprob,
                    no_speech_prob, s, nullptr, smp);
      return;
    }
    // the null stream cannot be captured, and lanes run concurrently: each lane gets its
    // own stream (the caller's priority), forked from and joined back into the caller's
    int prio = 0;
    JANUS_HIP(hipStreamGetPriority(s, &prio));
    if (!w->ev_in) JANUS_HIP(hipEventCreateWithFlags(&w->ev_in, hipEventDisableTiming));
    JANUS_HIP(hipEventRecord(w->ev_in, s));
    // a caller on a CU-masked stream (the overlapped step's decoder partition) gets lanes
    // on the same CUs
    std::vector<uint32_t> mask(16, 0xffffffffu);
    bool masked = false;
    if (s && hipExtStreamGetCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
      int ncu = 0;
      JANUS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
      for (int c = 0; c < ncu && c < 32 * (int)mask.size(); ++c)
        if (!((mask[c / 32] >> (c % 32)) & 1u)) masked = true;
    }
    for (int i = 0; i < nlanes; ++i) {
      DecLane& Z = *w->lanes[lane_of(i)];
      if (Z.stream && Z.stream_mask != (masked ? mask : std::vector<uint32_t>())) {
        JANUS_HIP(hipStreamSynchronize(Z.stream));
        JANUS_HIP(hipStreamDestroy(Z.stream));
        Z.stream = nullptr;
        for (auto& kv : Z.graphs) (void)hipGraphExecDestroy(kv.second);
        Z.graphs.clear();
        Z.graph_nodes.clear();
      }
      if (!Z.stream) {
        if (masked)
          JANUS_HIP(hipExtStreamCreateWithCUMask(&Z.stream, (uint32_t)mask.size(), mask.data()));
        else
          JANUS_HIP(hipStreamCreateWithPriority(&Z.stream, hipStreamNonBlocking, prio));
        Z.stream_mask = masked ? mask : std::vector<uint32_t>();
        if (!Z.ev_done) JANUS_HIP(hipEventCreateWithFlags(&Z.ev_done, hipEventDisableTiming));
      }
      JANUS_HIP(hipStreamWaitEvent(Z.stream, w->ev_in, 0));
    }
    const int maxlen = opt->max_length;
    LaneLatch latch;
    latch.left = nlanes;
    std::vector<std::string> errs(nlanes);
    int dev = 0;
    JANUS_HIP(hipGetDevice(&dev));
    auto run = [&](int i) {
      const int b0 = (int)((int64_t)batch * i / nlanes), b1 = (int)((int64_t)batch * (i + 1) / nlanes);
      DecLane& Z = *w->lanes[lane_of(i)];
      try {
        JANUS_HIP(hipSetDevice(dev));  // a fresh host thread starts on device 0
        janus_decode_rows sub{};
        if (rows) {
          sub = *rows;
          if (rows->prompts) {
            sub.prompts = rows->prompts + (int64_t)b0 * rows->stride;
            sub.prompt_lens = rows->prompt_lens + b0;
          }
        }
        DecodeSampling ssub{};
        if (smp) ssub = DecodeSampling{smp->temperature, smp->seeds + b0, smp->temps ? smp->temps + b0 : nullptr};
        decode_greedy(w, Z, e + (int64_t)b0 * w->cfg.n_audio_ctx * w->cfg.d_model, b1 - b0, opt,
                      rows ? &sub : nullptr, tokens + (int64_t)b0 * maxlen, n_tokens + b0,
                      sum_logprob + b0, no_speech_prob ? no_speech_prob + b0 : nullptr, Z.stream,
                      nlanes > 1 ? &latch : nullptr, smp ? &ssub : nullptr);
      } catch (const std::exception& ex) {
        errs[i] = ex.what();
      } catch (...) {
        errs[i] = "unknown error";
      }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < nlanes; ++i) th.emplace_back(run, i);
    run(0);
    for (auto& t : th) t.join();
    for (int i = 0; i < nlanes; ++i) {
      DecLane& Z = *w->lanes[lane_of(i)];
      JANUS_HIP(hipEventRecord(Z.ev_done, Z.stream));
      JANUS_HIP(hipStreamWaitEvent(s, Z.ev_done, 0));
    }
    for (int i = 0; i < nlanes; ++i)
      JANUS_CHECK(errs[i].empty(), "decode lane " + std::to_string(i) + ": " + errs[i]);
  });
}

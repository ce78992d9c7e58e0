/*
 * janus.h — C-ABI of libjanus_hip.so, the MI355X-native (gfx950) hot path of Janus.
 *
 * Every entry point returns int (0 = OK, non-zero = error; message from
 * janus_last_error(), per calling thread). No C++ exception crosses this ABI.
 * Arrays marked [device] are HIP device pointers the caller owns (e.g. torch
 * tensors); [host] arrays are ordinary memory. `stream` is a hipStream_t (NULL =
 * the null stream). Kernels are enqueued asynchronously on `stream`; host-side
 * entry points (packet codec) are synchronous and thread-safe.
 *
 * Each declaration names the reference interface it replaces (path:line in
 * akshatvasisht/janus). Reference bindings a maintainer would add: INTEGRATION.md.
 */
#ifndef JANUS_H_
#define JANUS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ errors */
const char* janus_last_error(void);
/* ABI version: major*10000 + minor*100 + patch. */
int janus_version(void);

/*
 * A HIP stream whose kernels run only on the CUs set in cu_mask (words x 32 bits, bit i =
 * CU i; hipExtStreamCreateWithCUMask). The pipeline runs the vocoder of one batch and
 * the latency-bound greedy decoder of the next on disjoint CU sets. Destroy with
 * janus_stream_destroy.
 */
int janus_stream_create_cu_mask(const uint32_t* cu_mask, int words, void** stream_out);
int janus_stream_destroy(void* stream);

/* ------------------------------------------------------------- prosody --- */
/*
 * Batched ProsodyExtractor core: aubio YIN per hop + RMS per utterance.
 * Replaces aubio.pitch('yin', 4096, hop, sr) with unit Hz / tolerance `tolerance`
 * (backend/services/prosody.py:32-34) called once per hop (prosody.py:78-87), and
 * numpy's rms = sqrt(mean(x**2)) (prosody.py:67). One stream per utterance:
 *   pcm            [device] f32, utterances back to back
 *   sample_offsets [device] int64[B+1], prefix offsets into pcm
 *   hop_offsets    [device] int64[B+1], prefix sum of ceil(n_b / hop)
 *   total_hops     host copy of hop_offsets[B]
 *   silence_db     aubio pitch silence threshold (aubio default -50 dB)
 *   state_in       [device] f32[B][4096] detector buffer before the call, or NULL (zeros)
 *   state_out      [device] f32[B][4096] buffer after the call, or NULL; must not alias state_in
 *   f0_out         [device] f32[total_hops] per-hop pitch in Hz (0 = unvoiced/silent)
 *   rms_out, mean_f0_out [device] f32[B]; n_voiced_out [device] int32[B]
 * rms_out is NaN for an empty utterance (numpy mean of an empty array).
 */
int janus_prosody_analyze(const float* pcm, const int64_t* sample_offsets,
                          const int64_t* hop_offsets, int batch, int64_t total_hops,
                          int sample_rate, int hop_size, float tolerance, float silence_db,
                          const float* state_in, float* state_out, float* f0_out,
                          float* rms_out, float* mean_f0_out, int32_t* n_voiced_out,
                          void* stream);
/*
 * Same, with the YIN grid capped at max_blocks workgroups (0 = one per hop): a batch run
 * beside other latency-bound work (the greedy decoder) leaves that work CUs to dispatch
 * onto. Results are identical for every max_blocks.
 */
int janus_prosody_analyze_ex(const float* pcm, const int64_t* sample_offsets,
                             const int64_t* hop_offsets, int batch, int64_t total_hops,
                             int sample_rate, int hop_size, float tolerance, float silence_db,
                             const float* state_in, float* state_out, float* f0_out,
                             float* rms_out, float* mean_f0_out, int32_t* n_voiced_out,
                             int max_blocks, void* stream);

/* ------------------------------------------------- receiver / streaming --- */
/*
 * Playback ducking, in place on int16 PCM [device] (n samples): replaces
 * apply_ducking_if_needed (backend/services/engine.py:94-134) for level in [0, 1):
 * s = int16(trunc(clip(float32(s) * level, -32768, 32767))), numpy's
 * np.clip(s.astype(np.float32) * level, -32768, 32767).astype(np.int16) bit for bit.
 * (level >= 1 and ducking-off / not-talking are pass-throughs the caller skips.)
 */
int janus_duck_pcm16(int16_t* pcm, int64_t n, float level, void* stream);

/*
 * Speech-gate probability per chunk: pcm [device] f32 [n_chunks][chunk_len] (e.g. the
 * 1536-sample 48 kHz capture chunks, audio_io.py:28-31), prob_out [device] f32[n_chunks].
 * Stands in for VoiceActivityDetector.is_speech (backend/services/vad.py:40-77: x[::3]
 * -> silero -> prob > threshold), whose weights are a remote torch.hub download:
 * prob = sigmoid((10 log10(mean(x[::decim]^2)) - center_db) / width_db).
 */
int janus_vad_energy(const float* pcm, int64_t n_chunks, int chunk_len, int decim,
                     float center_db, float width_db, float* prob_out, void* stream);

/*
 * The neural gate itself: VoiceActivityDetector.is_speech's model(chunk[::3], 16000)
 * (backend/services/vad.py:40-77; silero-vad v5, 16 kHz graph: 64-sample context + STFT
 * 256/128 + 4 conv blocks + LSTMCell(128) + sigmoid), from local weights. A context
 * holds the parameters by their silero state-dict names ("_model.stft.forward_basis_buffer",
 * "_model.encoder.{0..3}.reparam_conv.{weight,bias}", "_model.decoder.rnn.{weight_ih,
 * weight_hh,bias_ih,bias_hh}", "_model.decoder.decoder.2.{weight,bias}").
 * janus_vad_run: pcm [device] f32 [n_streams][n_chunks][chunk_len] (chunk[::decim] must
 * give 512 samples: 1536 / 3 for the 48 kHz capture chunks); the model state of each
 * channel, carried across calls as silero's stateful model object carries it
 * (the reference never resets it, vad.py:79-88): ctx_state [device] f32 [n_streams][64],
 * hc_state [device] f32 [n_streams][2][128] (zeros = fresh), updated in place;
 * prob_out [device] f32 [n_streams][n_chunks], channels in parallel, chunks in order.
 */
typedef struct janus_vad janus_vad;
int janus_vad_create(janus_vad** out);
int janus_vad_destroy(janus_vad* v);
int janus_vad_set_tensor(janus_vad* v, const char* name, const float* host, int64_t numel);
int janus_vad_run(janus_vad* v, const float* pcm, int n_streams, int n_chunks, int chunk_len,
                  int decim, float* ctx_state, float* hc_state, float* prob_out, void* stream);

/* -------------------------------------------------------- packet codec --- */
enum {
  JANUS_VAL_NIL = 0,
  JANUS_VAL_BOOL = 1,
  JANUS_VAL_INT = 2,   /* signed 64-bit in .i */
  JANUS_VAL_UINT = 3,  /* unsigned 64-bit in .i (bit pattern), > INT64_MAX only */
  JANUS_VAL_FLOAT = 4, /* float64 in .f */
  JANUS_VAL_STR = 5,   /* UTF-8 bytes: .s/.len (pack) or .offset/.len into the buffer (unpack) */
  JANUS_VAL_BIN = 6,
  JANUS_VAL_ARRAY = 7, /* .len children follow (pre-order) */
  JANUS_VAL_MAP = 8    /* .len key/value pairs follow (pre-order) */
};

typedef struct {
  int32_t type;
  int64_t i;
  double f;
  const char* s;
  size_t len;
} janus_value;

typedef struct {
  const char* text; /* UTF-8 */
  size_t text_len;
  int64_t mode; /* int(JanusMode) */
  int32_t n_prosody;
  const janus_value* prosody_keys; /* JANUS_VAL_STR, in dict insertion order */
  const janus_value* prosody_vals;
  const char* override_emotion; /* NULL => key 'o' omitted (override == "Auto") */
  size_t override_len;
  janus_value timestamp; /* JANUS_VAL_FLOAT (time.time()) or JANUS_VAL_INT */
} janus_packet;

/*
 * Replaces msgpack.packb(JanusPacket.to_dict(), use_bin_type=True)
 * (backend/common/protocol.py:57-76, :97-107). Keys in insertion order t, m, p, ts[, o].
 * Writes up to `cap` bytes; *out_len is the full size (error if it exceeds cap).
 */
int janus_pack_packet(const janus_packet* pkt, uint8_t* out, size_t cap, size_t* out_len);

typedef struct {
  int32_t type;  /* JANUS_VAL_* */
  int64_t i;     /* INT/UINT/BOOL value */
  double f;      /* FLOAT value */
  size_t offset; /* STR/BIN: byte offset of the payload in the input buffer */
  size_t len;    /* STR/BIN: payload bytes; ARRAY: items; MAP: pairs */
} janus_mp_node;

/*
 * Replaces msgpack.unpackb(payload, raw=False) (backend/common/protocol.py:109-121).
 * Decodes one MessagePack object into `nodes` (pre-order); fails on truncated input,
 * trailing bytes (msgpack ExtraData), the reserved byte 0xc1 and ext types.
 */
int janus_unpack(const uint8_t* buf, size_t len, janus_mp_node* nodes, size_t cap,
                 size_t* n_nodes);


/* ------------------------------------------------------------ whisper --- */
/*
 * Whisper speech-to-text on the GPU. Replaces faster-whisper's WhisperModel
 * (CTranslate2) as constructed at backend/services/transcriber.py:23-27 and driven by
 * model.transcribe(audio[::3], beam_size=1, language='en') at :51-57 (one 30 s window
 * per utterance). fp16 tensors are passed as uint16_t (IEEE binary16 bits).
 */
typedef struct {
  int n_mels;      /* 80 */
  int n_audio_ctx; /* 1500 encoder positions (3000 mel frames) */
  int d_model;     /* 384 tiny, 512 base */
  int n_heads;     /* d_model / 64 */
  int enc_layers;
  int dec_layers;
  int n_vocab;     /* 51864 for *.en */
  int n_text_ctx;  /* 448 */
} janus_whisper_config;

typedef struct janus_whisper janus_whisper;

int janus_whisper_create(const janus_whisper_config* cfg, janus_whisper** out);
int janus_whisper_destroy(janus_whisper* w);
/*
 * Upload one fp32 parameter [host] by its Hugging Face Whisper name without the
 * "model." prefix (e.g. "encoder.layers.0.fc1.weight"), plus the two front-end
 * constants "mel.basis" [400][416] (periodic-Hann-weighted cos|sin DFT basis, 208
 * bins each) and "mel.filters" [208][80] (slaney mel filters, transposed, zero-padded).
 */
int janus_whisper_set_tensor(janus_whisper* w, const char* name, const float* host,
                             int64_t numel);
/*
 * Log-mel features (faster-whisper FeatureExtractor, n_fft 400, hop 160, 80 mels,
 * 3000 frames) of x[::decim] for each utterance of pcm [device] (offsets [device]
 * int64[B+1]). logmel [device] f32 [B][3000][80] (raw log10 mel, may be NULL), mel
 * [device] fp16 [B][3000][80] (clamped and scaled). The first 30 s window of each clip as
 * faster-whisper's generate_segments feeds it to the encoder: frames from len(x16) // 160
 * on are 0.0 (pad_or_trim of the content frames), the global max is over the frames that
 * reach the first 30 s + 2 frames of audio (the whole clip when it is <= 30 s).
 */
int janus_whisper_logmel(janus_whisper* w, const float* pcm, const int64_t* offsets, int batch,
                         int decim, float* logmel, uint16_t* mel, void* stream);
/*
 * The whole-clip log-mel faster-whisper computes once per transcribe() call
 * (transcriber.py:53-57 -> WhisperModel.transcribe -> FeatureExtractor(audio)): `frames`
 * frames per utterance, mel [device] fp16 [B][frames][80], normalised with the maximum over
 * every frame of the clip, frames from len(x16) // 160 on 0.0. Its 30 s windows are the
 * slices [seek, seek + min(3000, content - seek)) padded with zeros to 3000 frames.
 */
int janus_whisper_logmel_frames(janus_whisper* w, const float* pcm, const int64_t* offsets,
                                int batch, int decim, int frames, uint16_t* mel, void* stream);
/* Encoder forward: mel [device] fp16 [B][3000][80] -> enc [device] fp16 [B][1500][d]. */
int janus_whisper_encode(janus_whisper* w, const uint16_t* mel, int batch, uint16_t* enc,
                         void* stream);

typedef struct {
  const int32_t* prompt;   /* [host] initial tokens, e.g. {<|startoftranscript|>} for *.en */
  int prompt_len;
  int max_length;          /* total tokens incl. prompt (faster-whisper max_length 448) */
  int eot;
  const int32_t* suppress; /* [host] always-suppressed token ids (suppress_tokens=[-1] set) */
  int n_suppress;
  int suppress_blank;      /* SuppressBlank at the first sampled token */
  int blank_token;         /* " " token id */
  int timestamp_begin;     /* first timestamp token id, -1 = no timestamp rules */
  int no_timestamps;       /* <|notimestamps|> id */
  int max_initial_timestamp_index; /* 50 (= 1.0 s), -1 = unbounded */
  int check_every;         /* poll for all-rows-finished every N steps (0 = never) */
  int xattn_splits;        /* cross-attention key splits per utterance (0 = auto: 8; the
                              overlapped step on half the CUs runs best at 4) */
  int cu_count;            /* CUs the decoder's stream may use (0 = the popcount of the
                              stream's CU mask), e.g. 128 on a half-GPU partition: one
                              vocabulary-projection block per CU, and at <= 128 the skinny
                              projections split rows from N <= 1024 */
  int state_slot;          /* decoder state slot of the context (0 = default): the KV caches,
                              tokens and rule state a call leaves behind for staggered
                              continuation live in this slot, so a sampled re-decode between
                              two staggered calls runs in another slot without disturbing
                              them (0 .. 7) */
  int logits_blocks;       /* vocabulary-projection blocks (0 = cu_count) */
  int msplit_rows_n;       /* skinny projections split rows over blocks up to this N
                              (0 = auto: 1024 on <= 128 CUs, else none; -1 = never) */
  int persistent;          /* 1: the launches between a layer's self- and cross-attention
                              run as two resident-grid launches with in-launch barriers
                              (d_model 512, 8 heads, <= 256 rows, >= 16 CUs per 16 rows up to
                              128 rows, 128 CUs at 256 rows; the other shapes keep the launch
                              path): 29 launches per position
                              at base.en instead of 75. Same arithmetic per row except the
                              GEMMs' k order (fp32-rounding level, not bit-identical to 0).
                              2: one launch per layer step — segment B of layer l, the
                              self-attention of l + 1 (one wave per row and head, online
                              softmax over 64-key chunks) and segment A of l + 1 as one
                              grid (layer 0's QKV, self-attention and segment A one head
                              grid, the final LayerNorm the last segment's phase): 16
                              launches per position (every row's keys in two
                              parts cut by its own length, merged in order: rows stay
                              independent of their neighbours).
                              3: as 2, with the cross-attention as the last phase of the
                              head / layer grids: 10 launches per position, measured level
                              with 2 */
  uint32_t path_flags;     /* alternative decoder paths (JANUS_DEC_PATH_* bits), for the
                              parity tests that hold every path bit-identical and for A/B
                              measurements; 0 = the measured default */
  int lanes;               /* concurrent decoder lanes of janus_whisper_decode_greedy: the
                              batch split over streams and host threads (0 = 1; slower at
                              B = 64) */
} janus_decode_options;

/* janus_decode_options.path_flags */
#define JANUS_DEC_PATH_NO_GRAPH     0x0001u /* launch every position, no captured graph */
#define JANUS_DEC_PATH_NO_XABSORB   0x0002u /* per-layer cross K/V instead of the absorbed
                                               cross-attention over the encoder output */
#define JANUS_DEC_PATH_NO_XPAIR     0x0004u /* rows sharing an encoder row: no PAIR blocks */
#define JANUS_DEC_PATH_XGROUP       0x0008u /* ... GROUP blocks of up to 6 rows */
#define JANUS_DEC_PATH_FUSED_LN     0x0010u /* LayerNorm statistics on the projections */
#define JANUS_DEC_PATH_LN_FUSE      0x0020u /* LayerNorm in the producing kernels */
#define JANUS_DEC_PATH_RESID_LN     0x0040u /* whole-row residual projection + LayerNorm */
#define JANUS_DEC_PATH_NO_CVP       0x0080u /* split merge and value projection apart */
#define JANUS_DEC_PATH_CVP          0x0100u /* ... fused, above 64 rows too */
#define JANUS_DEC_PATH_NO_SEL_EMBED 0x0200u /* token selection and embedding apart */
#define JANUS_DEC_PATH_NO_EMBED_LN  0x0400u /* first LayerNorm not in the embedding kernel */
#define JANUS_DEC_PATH_LN_PROLOGUE  0x0800u /* LayerNorm-into-prologue mask m (bits 12-15:
                                               1 LN1, 2 LN2, 4 LN3, 8 final) instead of the
                                               default 9 up to 64 rows, 0 above */
#define JANUS_DEC_PATH_LN_MASK(m)   (JANUS_DEC_PATH_LN_PROLOGUE | (((uint32_t)(m) & 15u) << 12))
#define JANUS_DEC_PATH_SEG_2CU      0x10000u /* persistent segments at 256 rows: two blocks
                                               per CU instead of one block per CU taking two
                                               blocks' work */
#define JANUS_DEC_PATH_XFWD         0x20000u /* persistent segments: every layer's one-split
                                               cross-attention over the key chunks first to
                                               last (default: odd layers last to first) */

/*
 * Batched greedy decoding (temperature 0) with the Whisper logit rules
 * (SuppressBlank, SuppressTokens, ApplyTimestampRules), KV cache on the device.
 * tokens [device] int32 [B][max_length] (prompt, then sampled tokens; -1 past the
 * end), n_tokens [device] int32 [B] sampled tokens incl. <|endoftext|>,
 * sum_logprob [device] f32 [B] (sum of chosen-token log-probabilities).
 */
int janus_whisper_decode_greedy(janus_whisper* w, const uint16_t* enc, int batch,
                                const janus_decode_options* opt, int32_t* tokens,
                                int32_t* n_tokens, float* sum_logprob, void* stream);

/*
 * Per-row prompts and the no-speech probability (faster-whisper's generate_segments /
 * generate_with_fallback state, transcriber.py:53-57 with its defaults):
 *   prompts      [host] int32 [B][stride]: row b's prompt (e.g. <|startofprev|>, the
 *                previous window's last <= 223 tokens, <|startoftranscript|> — the
 *                condition_on_previous_text prompt), prompt_lens [host] int32 [B];
 *                NULL prompts = opt->prompt for every row
 *   no_speech_token  token whose raw (unfiltered) softmax probability at the row's first
 *                sampled step is reported (<|nocaptions|> 50361 for *.en), -1 = none
 */
typedef struct {
  const int32_t* prompts;
  const int32_t* prompt_lens;
  int stride;
  int no_speech_token;
  /* Shared encoder outputs (faster-whisper's best_of hypotheses of one window,
   * transcriber.py:53-57 with the library's defaults): enc_index [host] int32 [B], row b
   * attends to encoder row enc_index[b] of enc, which then holds n_enc rows [n_enc][Te][d]
   * instead of B. The cross-attention reads each shared row once per PAIR of decoder rows
   * (both rows' heads in one MFMA tile). NULL = row b attends to enc row b. */
  const int32_t* enc_index;
  int n_enc;
  /* Staggered decode (continuous batching across calls): pos_offset [host] int32 [B], row b
   * runs positions [pos_offset[b], pos_offset[b] + steps) (steps 0 = max_length - 1). A row
   * with an offset > 0 CONTINUES the previous call's row in the same slot of this context
   * (its tokens, KV cache, counters and rule state are kept; pass its encoder output again);
   * rows with offset 0 start fresh and must be one contiguous range. A continuing row's
   * offset must not exceed the position its previous calls reached (its tokens and KV rows
   * below the offset must have been written): the context records where every slot stands
   * after each call (janus_whisper_decode_stand) and REJECTS (non-zero status,
   * janus_last_error) a continuing row past it, or a continuing call whose batch size /
   * max_length differ from the previous call's. When every row finishes early (check_every
   * polls), all rows stand at offset + the positions actually run. Greedy only, no
   * enc_index; steps >= 0; pos_offset + steps <= max_length. NULL = every row fresh. */
  const int32_t* pos_offset;
  int steps;
} janus_decode_rows;

/*
 * janus_whisper_decode_greedy with per-row prompts (rows may be NULL): all rows step
 * together, a row samples from its own prompt length on; tokens [device] int32
 * [B][max_length] hold row b's prompt in [0, prompt_lens[b]) and its sampled tokens after.
 * no_speech_prob [device] f32 [B] (nullable).
 */
int janus_whisper_decode_greedy_ex(janus_whisper* w, const uint16_t* enc, int batch,
                                   const janus_decode_options* opt, const janus_decode_rows* rows,
                                   int32_t* tokens, int32_t* n_tokens, float* sum_logprob,
                                   float* no_speech_prob, void* stream);

/*
 * janus_whisper_decode_greedy_ex at temperature > 0: faster-whisper's fallback re-decode
 * (generate_with_fallback, temperatures 0.2 ... 1.0 with best_of 5: CTranslate2
 * generate(sampling_temperature=T, sampling_topk=0, num_hypotheses=5); the caller
 * replicates a window's row per hypothesis). Every token is drawn from softmax(l / T)
 * over the rule-filtered logits l by Gumbel-max; the noise is a counter-based hash of
 * (seeds[b], position, token), seeds [host] uint32 [B], so a row's draws are independent
 * of its batch neighbours and reproducible on the CPU. sum_logprob accumulates the chosen
 * tokens' log-probabilities under the untempered filtered distribution (the scores
 * CTranslate2 gathers from its log-softmax). temperature <= 0 or null seeds: error.
 */
int janus_whisper_decode_sample_ex(janus_whisper* w, const uint16_t* enc, int batch,
                                   const janus_decode_options* opt, const janus_decode_rows* rows,
                                   float temperature, const uint32_t* seeds, int32_t* tokens,
                                   int32_t* n_tokens, float* sum_logprob, float* no_speech_prob,
                                   void* stream);

/*
 * janus_whisper_decode_sample_ex with a temperature per row: temperatures [host] f32 [B],
 * each >= 0 (0: a greedy row, as janus_whisper_decode_greedy_ex; its seed is ignored).
 * Row b's tokens equal those of a greedy / decode_sample_ex call at temperatures[b] with
 * the same seed (rows are independent of their batch neighbours), so a window's T = 0 row
 * and the hypotheses of every fallback temperature can run in ONE call and the caller keeps
 * exactly what the sequential generate_with_fallback walk (transcriber.py:53-57,
 * faster-whisper's temperature loop) keeps: janus_amd/services/transcriber.py
 * generate_segments(speculative=True), the streaming encoder's setting.
 */
int janus_whisper_decode_sample_rows_ex(janus_whisper* w, const uint16_t* enc, int batch,
                                        const janus_decode_options* opt, const janus_decode_rows* rows,
                                        const float* temperatures, const uint32_t* seeds,
                                        int32_t* tokens, int32_t* n_tokens, float* sum_logprob,
                                        float* no_speech_prob, void* stream);

/*
 * Shape of the last decode call on this context (lane 0): positions the decoder stepped
 * (every row together; the early-exit poll stops at a 16-position boundary) and the
 * kernel launches those positions issued (nodes of the captured decode graphs; 0 when
 * JANUS_NO_GRAPH runs without graphs). Measurement only (bench.py's decoder roofline:
 * launches per position beside bytes per position); the reference has no counterpart.
 */
int janus_whisper_decode_info(janus_whisper* w, int32_t* positions, int64_t* launches);

/*
 * Where each of the `batch` row slots stands after the last completed decode call (the
 * first position a staggered call may continue it from: tokens and KV rows below it are
 * written). Fails when the last call had another batch size or failed. The continuous-
 * batching plan of the serving step (janus_amd/pipeline.py stagger_plan) continues from
 * here; the reference has no counterpart (its decode is one faster-whisper call per
 * window, transcriber.py:53-57).
 */
int janus_whisper_decode_stand(janus_whisper* w, int32_t* stand, int batch);
/* The same for decoder state slot `slot` (janus_decode_options.state_slot). */
/*
 * A call with janus_decode_options.check_every = 0 (no early-exit polling) returns as soon
 * as its work is enqueued, without waiting for the stream; the persistent segments' grid
 * barrier timeout (a resident grid that never became co-resident) is then reported here:
 * waits for the last such call of state slot `slot` and returns non-zero (janus_last_error)
 * if it timed out — call it before using that call's outputs. The lane's next decode call
 * checks it too. Returns 0 when nothing is pending.
 */
int janus_whisper_decode_check(janus_whisper* w, int slot);
int janus_whisper_decode_stand_slot(janus_whisper* w, int slot, int32_t* stand, int batch);

/* ------------------------------------------------------------ vocoder --- */
/*
 * Local Firefly-GAN decoder (fish-speech HiFiGANGenerator architecture) replacing the
 * Fish Audio cloud TTS call client.tts.convert(text=prompt, format="wav", ...)
 * (backend/services/synthesizer.py:179-203, :235-255). Conditioning is the same
 * "(emotion) text" prompt the reference sends (synthesizer.py:151-177).
 */
typedef struct {
  int latent_dim;       /* 512 */
  int channels;         /* upsample_initial_channel, 512 */
  int n_ups;            /* 5 */
  int up_rates[8];      /* 8, 8, 2, 2, 2 (kernel 2u, padding u/2) */
  int n_kernels;        /* 3 */
  int rb_kernels[4];    /* 3, 7, 11 */
  int n_dilations;      /* 3 */
  int rb_dilations[4];  /* 1, 3, 5 */
  int pre_kernel;       /* 13 */
  int post_kernel;      /* 13 */
  int n_emotions;       /* rows of frontend.emotion_embed */
} janus_vocoder_config;

typedef struct janus_vocoder janus_vocoder;

int janus_vocoder_create(const janus_vocoder_config* cfg, janus_vocoder** out);
int janus_vocoder_destroy(janus_vocoder* v);
/*
 * fp32 [host] parameters by fish-speech generator name (weight norm folded):
 * conv_pre.{weight,bias}, ups.{i}.{weight,bias} ([Cin][Cout][2u]),
 * resblocks.{i}.blocks.{j}.convs{1,2}.{m}.{weight,bias}, conv_post.{weight,bias},
 * plus the front end: frontend.text_embed [256][latent], frontend.emotion_embed
 * [n_emotions][latent].
 */
int janus_vocoder_set_tensor(janus_vocoder* v, const char* name, const float* host,
                             int64_t numel);
/*
 * Prompt -> latents: latents [device] fp16 [B][frames][latent] with frame f of row b =
 * text_embed[prompt byte floor(f*n_b/frames)] + emotion_embed[emotion_ids[b]].
 * bytes [device] u8 prompts back to back, byte_offsets [device] int64[B+1],
 * emotion_ids [device] int32[B].
 */
int janus_vocoder_frontend(janus_vocoder* v, const uint8_t* bytes, const int64_t* byte_offsets,
                           const int32_t* emotion_ids, int batch, int frames, uint16_t* latents,
                           void* stream);
/*
 * Same, plus a per-row voice term: latent += speaker[b] ([device] f32 [B][latent], or NULL
 * for none). The voice stands in for the reference's voice cloning, which sends the
 * hot-reloaded recording as references=[ReferenceAudio(audio, text="")] or, without one,
 * reference_id="5196af35..." (synthesizer.py:179-200, :243-249).
 */
int janus_vocoder_frontend_ex(janus_vocoder* v, const uint8_t* bytes, const int64_t* byte_offsets,
                              const int32_t* emotion_ids, const float* speaker, int batch,
                              int frames, uint16_t* latents, void* stream);
/*
 * Voice embedding of reference recordings (the ReferenceAudio bytes of
 * synthesizer.py:183-187, decoded to 16 kHz f32 by the caller): pcm16k [device] f32
 * clips back to back, offsets [device] int64[B+1] (<= 30 s used per clip) ->
 * speaker_out [device] f32 [B][latent] = speaker_bias + speaker_proj . mean over the
 * clip's frames of its normalised Whisper log-mel. Needs the parameters
 * "frontend.speaker_proj" [latent][80], "frontend.speaker_bias" [latent], "mel.basis"
 * and "mel.filters" (as for janus_whisper_set_tensor).
 */
int janus_vocoder_speaker(janus_vocoder* v, const float* pcm16k, const int64_t* offsets, int batch,
                          float* speaker_out, void* stream);
/*
 * Generator forward: latents [device] fp16 [B][frames][latent] -> wav [device] f32
 * [B][frames*prod(up_rates)] in [-1, 1] and, if pcm != NULL, int16 [B][...]
 * (clip(round(32767*y))).
 */
int janus_vocoder_forward(janus_vocoder* v, const uint16_t* latents, int batch, int frames,
                          float* wav, int16_t* pcm, void* stream);
/* Same, plus pre_tanh [device] f32 [B][samples] (conv_post output before tanh; may be NULL). */
int janus_vocoder_forward_ex(janus_vocoder* v, const uint16_t* latents, int batch, int frames,
                             float* wav, int16_t* pcm, float* pre_tanh, void* stream);
/* HIP-event timing of every conv launch (for roofline accounting). */
int janus_vocoder_set_timing(janus_vocoder* v, int on);
/* Accumulated conv FLOPs (2*Cin*Cout*taps*rows), kernel milliseconds and launches. */
int janus_vocoder_conv_stats(janus_vocoder* v, double* flops, double* ms, int64_t* launches,
                             int reset);
/*
 * The same per family: fam[i] = channel width C of the fused ResBlock1 units (4*C*C*k
 * FLOP and 2-3 x C x 2 B of activations per row), or 0 for the conv kernel (conv_pre and
 * the upsamplers). Up to cap families; *n = how many were written. Algorithmic bytes:
 * fp16 activations read once and written once (+ the accumulator / residual reads).
 */
int janus_vocoder_family_stats(janus_vocoder* v, int cap, int* fam, double* flops, double* bytes,
                               double* ms, int64_t* launches, int* n, int reset);

#ifdef __cplusplus
}
#endif
#endif /* JANUS_H_ */

/*
 * ORACLE — test infrastructure only. Never linked into, or called by, the product
 * path (janus_amd/). Imported only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.
 *
 * Sequential CPU restatement of the reference's pitch path:
 *   backend/services/prosody.py:32-34  aubio.pitch('yin', 4096, hop_size, sample_rate),
 *                                       set_unit('Hz'), set_tolerance(0.8)
 *   backend/services/prosody.py:78-87  per-hop loop, last chunk zero-padded to hop_size
 * The arithmetic is aubio 0.4.9's (third-party, not in /root/reference, not
 * installed here), restated from its published sources:
 *   src/pitch/pitch.c     aubio_pitch_do, aubio_pitch_do_yin, aubio_pitch_slideblock,
 *                         DEFAULT_PITCH_SILENCE (-50 dB), freqconvpass (unit Hz)
 *   src/pitch/pitchyin.c  aubio_pitchyin_do (difference function, cumulative-mean
 *                         normalisation, early exit at tau > 4 with yin[tau-3] < tol)
 *   src/mathutils.c       aubio_quadratic_peak_pos, fvec_min_elem, aubio_level_lin,
 *                         aubio_db_spl, aubio_silence_detection
 * smpl_t is float (aubio default build). Compile with -ffp-contract=off so every
 * operation rounds exactly as aubio's SSE build does.
 * Pinned by the reference's own known-answer tests (tests/test_oracle.py):
 * backend/tests/test_input_processing.py:461-468 (amp 0.02 -> Quiet) and :480-490
 * (440 Hz -> High).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define YIN_BUF 4096
#define YIN_LEN (YIN_BUF / 2)

static float quadratic_peak_pos(const float* x, unsigned length, unsigned pos) {
  if (pos == 0 || pos == length - 1) return (float)pos;
  unsigned x0 = pos - 1, x2 = pos + 1;
  float s0 = x[x0], s1 = x[pos], s2 = x[x2];
  float half = 0.5f, two = 2.0f;
  return (float)pos + half * (s0 - s2) / (s0 - two * s1 + s2);
}

static unsigned min_elem(const float* s, unsigned length) {
  unsigned j, pos = 0;
  float tmp = s[0];
  for (j = 0; j < length; j++) {
    pos = (tmp < s[j]) ? pos : j;
    tmp = (tmp < s[j]) ? tmp : s[j];
  }
  return pos;
}

/* aubio_pitchyin_do on a 4096-sample buffer -> period in samples (float). */
static float pitchyin_do(const float* in, float tol, float* yin) {
  unsigned j, tau;
  int period;
  float tmp, tmp2 = 0.0f;
  yin[0] = 1.0f;
  for (tau = 1; tau < YIN_LEN; tau++) {
    yin[tau] = 0.0f;
    for (j = 0; j < YIN_LEN; j++) {
      tmp = in[j] - in[j + tau];
      yin[tau] += tmp * tmp;
    }
    tmp2 += yin[tau];
    if (tmp2 != 0) {
      yin[tau] *= (float)tau / tmp2;
    } else {
      yin[tau] = 1.0f;
    }
    period = (int)tau - 3;
    if (tau > 4 && (yin[period] < tol) && (yin[period] < yin[period + 1])) {
      return quadratic_peak_pos(yin, YIN_LEN, (unsigned)period);
    }
  }
  return quadratic_peak_pos(yin, YIN_LEN, min_elem(yin, YIN_LEN));
}

static float level_lin(const float* x, unsigned n) {
  float energy = 0.0f;
  for (unsigned j = 0; j < n; j++) energy += x[j] * x[j];
  return energy / (float)n;
}

/* One aubio_pitch_do call: slide `hop` samples into buf, YIN, silence gate. */
static float pitch_do(float* buf, const float* ibuf, unsigned hop, unsigned sr, float tol,
                      float silence, float* yin) {
  unsigned overlap = YIN_BUF - hop, j;
  for (j = 0; j < overlap; j++) buf[j] = buf[j + hop];
  for (j = 0; j < hop; j++) buf[j + overlap] = ibuf[j];
  float pitch = pitchyin_do(buf, tol, yin);
  if (pitch > 0) pitch = (float)((double)sr / (pitch + 0.));
  else pitch = 0.0f;
  float db = (float)(10. * log10f(level_lin(ibuf, hop)));
  if (db < silence) pitch = 0.0f;
  return pitch;
}

/* Probes for edge-case tests: aubio_level_lin, the dB value aubio_silence_detection
 * compares, and the CMNDF of one 4096-sample buffer with the tau at which the early
 * exit fired (-1: none, argmin path). */
float yin_oracle_level(const float* ibuf, unsigned hop) { return level_lin(ibuf, hop); }
float yin_oracle_db(float level) { return (float)(10. * log10f(level)); }
int yin_oracle_probe(const float* buf, float tol, float* yin_out, float* period_out) {
  float yin[YIN_LEN];
  unsigned tau;
  float tmp, tmp2 = 0.0f;
  yin[0] = 1.0f;
  int exit_tau = -1;
  for (tau = 1; tau < YIN_LEN; tau++) {
    yin[tau] = 0.0f;
    for (unsigned j = 0; j < YIN_LEN; j++) {
      tmp = buf[j] - buf[j + tau];
      yin[tau] += tmp * tmp;
    }
    tmp2 += yin[tau];
    if (tmp2 != 0) yin[tau] *= (float)tau / tmp2;
    else yin[tau] = 1.0f;
    int period = (int)tau - 3;
    if (tau > 4 && (yin[period] < tol) && (yin[period] < yin[period + 1])) {
      exit_tau = (int)tau;
      break;
    }
  }
  memcpy(yin_out, yin, sizeof(float) * (exit_tau < 0 ? YIN_LEN : (size_t)exit_tau + 1));
  float scratch[YIN_LEN];
  *period_out = pitchyin_do(buf, tol, scratch);
  return exit_tau;
}

/*
 * One ProsodyExtractor.analyze_buffer pitch loop over x[0..n): f0_out gets
 * ceil(n/hop) values; `state` (4096 floats, zeros for a fresh detector) is the
 * aubio buffer, updated in place.
 */
void yin_oracle_stream(const float* x, int64_t n, int sr, int hop, float tol, float silence,
                       float* state, float* f0_out) {
  float chunk[YIN_BUF];
  float yin[YIN_LEN];
  int64_t nh = (n + hop - 1) / hop;
  for (int64_t i = 0; i < nh; i++) {
    int64_t start = i * hop;
    int64_t len = n - start < hop ? n - start : hop;
    memset(chunk, 0, sizeof(float) * (size_t)hop);
    memcpy(chunk, x + start, sizeof(float) * (size_t)len);
    f0_out[i] = pitch_do(state, chunk, (unsigned)hop, (unsigned)sr, tol, silence, yin);
  }
}

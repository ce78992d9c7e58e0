"""Speech-to-text — drop-in for backend/services/transcriber.py on MI355X.

``Transcriber`` keeps the reference's constructor and methods (transcriber.py:11-91) and
even its body: it builds ``WhisperModel(model_size, device='cpu', compute_type='int8')``
and iterates ``model.transcribe(audio[::3], beam_size=1, language='en')`` segments. Here
``WhisperModel`` is the GPU engine (log-mel, encoder and greedy decoder in
libjanus_hip.so) behind faster-whisper's call shape (``transcribe`` returns
``(segments, info)``; segments carry ``.text`` and the decode statistics), so
module-level patching of ``WhisperModel`` in tests works exactly as in the reference
suite (backend/tests/test_input_processing.py:73-90).

``transcribe`` restates faster-whisper's ``generate_segments`` loop for the reference's
call (beam_size=1, language='en', every other option at its default):

* windows of 3000 log-mel frames at a moving ``seek``; the next seek is the end of the
  window when the tokens end in a single timestamp or hold none, else the last
  consecutive-timestamp pair (the trailing partial segment is re-decoded from there);
* ``condition_on_previous_text``: each window's prompt is ``<|startofprev|>`` + the
  last <= 223 tokens of the segments emitted so far + ``<|startoftranscript|>``;
* the gates, computed per window: ``avg_logprob`` = sum of chosen-token log-probs /
  (tokens + 1), ``compression_ratio`` = len(text) / len(zlib(text)),
  ``no_speech_prob`` = raw P(<|nocaptions|>) at the first step (on the GPU);
  no-speech skip when no_speech_prob > 0.6 and avg_logprob <= -1;
* segments whose start equals their end or whose text is blank are dropped.

* the temperature FALLBACK (``generate_with_fallback``): a window whose gates fail
  (compression ratio > 2.4 or avg_logprob < -1, outside the no-speech case) is re-decoded
  at T = 0.2, 0.4, ... 1.0 with best_of = 5 sampled hypotheses (the best by
  sum-log-prob / length kept, as CTranslate2 orders them) until one passes; when none
  does, the result with the highest avg_logprob among those under the compression
  threshold (else among all) is kept and reported at T = 1.0; a final temperature above
  ``prompt_reset_on_temperature`` (0.5) resets the conditioning prompt. The hypotheses of
  all failing windows of a round are decoded as one GPU batch (``janus_whisper_decode_
  sample_ex``: Gumbel-max over the rule-filtered logits / T). Sampling noise comes from
  a counter-based hash seeded per (utterance, window, temperature, hypothesis)
  (``fallback_seed``), so a run is reproducible and the CPU oracle draws the same noise —
  CTranslate2's own random draws cannot be reproduced offline.

A window that would not advance the seek (a leading <|0.00|><|0.00|>) advances by the
window size, so the loop always terminates.

Features are faster-whisper's: one log-mel of the whole clip (normalised with the maximum
over all its frames), from which each window takes the content frames
[seek, seek + min(3000, content - seek)) and is padded with zeros to 3000 frames
(``features[:, seek:seek + segment_size]`` + ``pad_or_trim``).
"""
import dataclasses
import zlib

import numpy as np
import torch

from .. import _native as nat
from ..common import wavio
from ..tokenizer import SOT_PREV
from ..whisper import CONFIGS, WhisperEngine

WINDOW_16K = 480000
N_FRAMES = 3000          # log-mel frames per window (hop 160 @ 16 kHz)
HOP = 160
TIME_PRECISION = 0.02    # seconds per timestamp step
INPUT_STRIDE = 2         # mel frames per timestamp step
COMPRESSION_RATIO_THRESHOLD = 2.4
LOG_PROB_THRESHOLD = -1.0
NO_SPEECH_THRESHOLD = 0.6
TEMPERATURES = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0)   # faster-whisper transcribe(temperature=...)
BEST_OF = 5
PROMPT_RESET_ON_TEMPERATURE = 0.5
FALLBACK_ROWS = 320      # hypotheses per sampling decode (64 windows x 5: one decode per
                         # temperature for a 64-window round; the windows' encoder outputs are
                         # shared by their hypotheses through enc_index)
FALLBACK_ROWS_GATHER = 60  # the same for models past the PAIR path's H <= 8, d <= 512


def _mix32(h: int) -> int:
    h &= 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def fallback_seed(utt: int, window: int, temp_index: int, hyp: int) -> int:
    """uint32 noise seed of one sampled hypothesis: utterance (index in the call), window
    (counter within the utterance), temperature index (1..5), hypothesis (0..best_of-1)."""
    return _mix32(0x4A414E55 ^ _mix32(utt * 0x01000193 + window * 0x9E3779B1 +
                                      temp_index * 0x85EBCA77 + hyp))


@dataclasses.dataclass
class Segment:
    id: int
    seek: int
    start: float
    end: float
    text: str
    tokens: list
    temperature: float
    avg_logprob: float
    compression_ratio: float
    no_speech_prob: float
    needs_fallback: bool = False   # the T = 0 decode failed its gates (fallback entered)


@dataclasses.dataclass
class Candidate:
    """One decode result of a window (generate_with_fallback's decode_result)."""
    tokens: list
    avg_logprob: float
    no_speech_prob: float
    temperature: float
    text: str
    compression_ratio: float
    needs_fallback: bool


def candidate(tk, toks, avg_lp, nsp, temperature) -> Candidate:
    text = tk.decode(toks).strip()
    return Candidate(list(toks), float(avg_lp), float(nsp), float(temperature), text,
                     compression_ratio(text), gates(text, avg_lp, nsp)[0])


def best_hypothesis(rows):
    """CTranslate2's first hypothesis of a sampled best_of group: the highest score
    sum-log-prob / length (length_penalty 1; sequences without <|endoftext|>), the first on
    ties. rows: [(tokens, avg_logprob, nsp)] as DecodeOut.rows() gives them."""
    def score(r):
        toks, avg, _ = r
        return avg * (len(toks) + 1) / max(len(toks), 1)
    best = 0
    for i in range(1, len(rows)):
        if score(rows[i]) > score(rows[best]):
            best = i
    return rows[best]


def settle(results, temperatures=TEMPERATURES):
    """generate_with_fallback's choice over a window's results in temperature order: the
    first that passes its gates; if none does (every temperature tried), the highest
    avg_logprob among those under the compression-ratio threshold (else among all),
    reported at the last temperature. None while the fallback is still running."""
    for r in results:
        if not r.needs_fallback:
            return r
    if len(results) < len(temperatures):
        return None
    below = [r for r in results if not r.compression_ratio > COMPRESSION_RATIO_THRESHOLD]
    pool = below or results
    best = pool[0]
    for r in pool[1:]:
        if r.avg_logprob > best.avg_logprob:
            best = r
    return dataclasses.replace(best, temperature=float(temperatures[-1]))


@dataclasses.dataclass
class TranscriptionInfo:
    language: str
    language_probability: float
    duration: float


read_wav_16k = wavio.read_wav_16k  # 16-bit PCM WAV -> f32 @ 16 kHz

# faster-whisper's device / compute_type vocabulary (WhisperModel(model_size, device=...,
# compute_type=...)); every value names the SAME GPU engine here (see WhisperModel)
DEVICES = ("cpu", "cuda", "auto")
COMPUTE_TYPES = ("default", "auto", "int8", "int8_float32", "int8_float16", "int8_bfloat16",
                 "int16", "float16", "bfloat16", "float32")


def compression_ratio(text: str) -> float:
    """faster-whisper get_compression_ratio."""
    b = text.encode("utf-8")
    return len(b) / len(zlib.compress(b))


def gates(text: str, avg_logprob: float, no_speech_prob: float):
    """(needs_fallback, no_speech_skip) for one T = 0 window, faster-whisper's rules."""
    needs = compression_ratio(text) > COMPRESSION_RATIO_THRESHOLD or avg_logprob < LOG_PROB_THRESHOLD
    if no_speech_prob > NO_SPEECH_THRESHOLD and avg_logprob < LOG_PROB_THRESHOLD:
        needs = False                      # silence: no fallback
    skip = no_speech_prob > NO_SPEECH_THRESHOLD and not avg_logprob > LOG_PROB_THRESHOLD
    return needs, skip


def split_window(tk, tokens, seek, segment_size):
    """One window's tokens -> ([(start_s, end_s, tokens)], next seek) as faster-whisper's
    generate_segments slices them (timestamps included in the token lists)."""
    tb = tk.timestamp_begin
    time_offset = seek * HOP / 16000.0
    single_ending = len(tokens) >= 2 and tokens[-2] < tb <= tokens[-1]
    consecutive = [i for i in range(1, len(tokens)) if tokens[i] >= tb and tokens[i - 1] >= tb]
    segs = []
    if consecutive:
        slices = list(consecutive)
        if single_ending:
            slices.append(len(tokens))
        last = 0
        for cur in slices:
            part = tokens[last:cur]
            segs.append((time_offset + (part[0] - tb) * TIME_PRECISION,
                         time_offset + (part[-1] - tb) * TIME_PRECISION, part))
            last = cur
        if single_ending:
            nseek = seek + segment_size
        else:
            nseek = seek + (tokens[last - 1] - tb) * INPUT_STRIDE
    else:
        duration = segment_size * HOP / 16000.0
        stamps = [t for t in tokens if t >= tb]
        if stamps and stamps[-1] != tb:
            duration = (stamps[-1] - tb) * TIME_PRECISION
        segs.append((time_offset, time_offset + duration, tokens))
        nseek = seek + segment_size
    if nseek <= seek:          # no progress (e.g. <|0.00|><|0.00|>): move on a window
        nseek = seek + segment_size
    return segs, nseek


class _Stream:
    """generate_segments state of one utterance."""

    def __init__(self, audio16k=None, content_frames=None):
        self.audio = audio16k
        self.content_frames = len(audio16k) // HOP if content_frames is None else int(content_frames)
        self.seek = 0
        self.all_tokens = []
        self.prompt_reset_since = 0
        self.segments = []
        self.windows = self.fallbacks = self.skips = 0
        self.fallback_decodes = 0      # sampled decodes (temperature steps) run
        self.window_tokens = []        # the settled tokens of every window, in order
        self.window_rows = []          # every window's T = 0 decode: (tokens, avg_logprob, nsp)
        self.sampled = 0               # tokens sampled at T = 0 over every window (incl. eot)

    def transcript(self):
        """transcribe_buffer's join of the segments (transcriber.py:59-64)."""
        return ' '.join(s.text.strip() for s in self.segments).strip()

    @property
    def active(self):
        return self.seek < self.content_frames

    def window_size(self):
        return min(N_FRAMES, self.content_frames - self.seek)

    def prompt(self, tk, max_length=448):
        prev = self.all_tokens[self.prompt_reset_since:]
        p = ([SOT_PREV] + prev[-(max_length // 2 - 1):]) if prev else []   # 223 at 448
        return p + list(tk.sot_sequence)


def _fallback(engine, tk, enc, prompts, first, keys, max_length, temperatures, best_of,
              enc_rows=None, presampled=None, **dec_kw):
    """Run the temperature fallback for the windows of one round: first [Candidate] (T = 0
    results), keys [(utt, window)]; returns each window's settled Candidate. The
    hypotheses of every window still failing at a temperature go out as one sampled batch
    (chunks of FALLBACK_ROWS rows). ``enc_rows``: window j's encoder output is enc[enc_rows[j]]
    (default enc[j]). ``presampled[j][ti - 1]``: window j's best_of hypothesis rows at
    temperatures[ti], already decoded (generate_segments(speculative=True)): the walk keeps
    the same candidates the sequential decodes would give (rows are independent of their
    batch neighbours and every draw is keyed by (utt, window, ti, h))."""
    er = list(range(len(first))) if enc_rows is None else list(enc_rows)
    results = [[c] for c in first]
    final = [settle(r, temperatures) if not r[0].needs_fallback else None for r in results]
    if presampled is not None:
        for j in range(len(first)):
            for ti in range(1, len(temperatures)):
                if final[j] is not None:
                    break
                toks, avg_lp, nsp = best_hypothesis(presampled[j][ti - 1])
                results[j].append(candidate(tk, toks, avg_lp, nsp, float(temperatures[ti])))
                if not results[j][-1].needs_fallback or ti == len(temperatures) - 1:
                    final[j] = settle(results[j], temperatures)
        return final, [len(r) - 1 for r in results]
    # the shared-encoder PAIR path (H <= 8, d <= 512) reads each window's output in place;
    # wider models gather one encoder copy per hypothesis row (0.74 GB per 320 rows at
    # d = 768), so their sampled decodes stay at FALLBACK_ROWS_GATHER rows
    cfg = getattr(engine, "cfg", None)
    pair = cfg is None or (cfg.n_heads <= 8 and cfg.d_model <= 512)
    per = max(1, (FALLBACK_ROWS if pair else FALLBACK_ROWS_GATHER) // best_of)
    for ti in range(1, len(temperatures)):
        T = float(temperatures[ti])
        pend = [j for j in range(len(first)) if final[j] is None]
        if not pend:
            break
        for c0 in range(0, len(pend), per):
            js = pend[c0:c0 + per]
            # the hypotheses of window j share its encoder output: no per-row copy, and the
            # cross-attention reads it once per pair of hypotheses (enc_index)
            rows_prompts = [prompts[j] for j in js for _ in range(best_of)]
            seeds = [fallback_seed(keys[j][0], keys[j][1], ti, h) for j in js for h in range(best_of)]
            out = engine.decode_ex(enc, prompts=rows_prompts, max_length=max_length,
                                   temperature=T, seeds=seeds,
                                   enc_index=[er[j] for j in js for _ in range(best_of)], **dec_kw).rows()
            for k, j in enumerate(js):
                toks, avg_lp, nsp = best_hypothesis(out[k * best_of:(k + 1) * best_of])
                results[j].append(candidate(tk, toks, avg_lp, nsp, T))
        for j in pend:
            if not results[j][-1].needs_fallback or ti == len(temperatures) - 1:
                final[j] = settle(results[j], temperatures)
    return final, [len(r) - 1 for r in results]


def settle_round(engine, tk, rows, prompts, keys, enc, max_length, temperatures=(0.0,),
                 best_of: int = BEST_OF, enc_rows=None, presampled=None, **dec_kw):
    """One round of generate_with_fallback: ``rows`` the T = 0 decode of the round's windows
    ([(tokens, avg_logprob, no_speech_prob)], DecodeOut.rows()), ``prompts`` / ``keys`` [(utt, window)] per window,
    ``enc`` the windows' encoder output (enc[enc_rows[j]] for window j). Returns (first,
    final, sampled decodes) per window: the T = 0 Candidate, the settled one, and the number
    of sampled re-decodes the fallback ran."""
    first = [candidate(tk, toks, avg_lp, nsp, 0.0) for (toks, avg_lp, nsp) in rows]
    if len(temperatures) > 1:
        final, ndec = _fallback(engine, tk, enc, prompts, first, keys, max_length, temperatures,
                                best_of, enc_rows=enc_rows, presampled=presampled, **dec_kw)
    else:
        final, ndec = first, [0] * len(first)
    return first, final, ndec


def advance(tk, s, size, c0, r, nd, sampled: int = 0):
    """generate_segments' update of one utterance after its window [seek, seek + size) settled
    (c0: the T = 0 Candidate, r: the settled one, nd: sampled re-decodes, sampled: tokens the
    T = 0 decode emitted): the counters, the no-speech skip, the segments (start == end or
    blank text dropped), the next seek and the prompt reset."""
    s.windows += 1
    s.fallbacks += int(c0.needs_fallback)
    s.fallback_decodes += nd
    s.sampled += int(sampled)
    s.window_tokens.append(list(r.tokens))
    s.window_rows.append((list(c0.tokens), c0.avg_logprob, c0.no_speech_prob))
    # no-speech skip on the settled result (generate_segments after the fallback)
    if r.no_speech_prob > NO_SPEECH_THRESHOLD and not r.avg_logprob > LOG_PROB_THRESHOLD:
        s.skips += 1
        s.seek += size
        return
    segs, nseek = split_window(tk, r.tokens, s.seek, size)
    for (st, en, part) in segs:
        txt = tk.decode(part)
        if st == en or not txt.strip():
            continue
        s.all_tokens.extend(part)
        s.segments.append(Segment(len(s.segments), s.seek, st, en, txt, part,
                                  r.temperature, r.avg_logprob, r.compression_ratio,
                                  r.no_speech_prob, c0.needs_fallback))
    s.seek = nseek
    # condition_on_previous_text: a result settled above prompt_reset_on_temperature
    # restarts the prompt after these segments
    if r.temperature > PROMPT_RESET_ON_TEMPERATURE:
        s.prompt_reset_since = len(s.all_tokens)


def gather_windows(items, n_frames: int = N_FRAMES, device=None):
    """fp16 [len(items)][n_frames][80]: item j = (features [B][F][80] fp16 device tensor, row,
    seek, size) -> features[row, seek:seek + size] followed by zeros (faster-whisper's
    ``features[:, seek:seek + segment_size]`` + pad_or_trim). One index gather per distinct
    features tensor (a serving batch's windows come out of one [B][F][80] tensor)."""
    if not items:
        return torch.zeros(0, n_frames, 80, dtype=torch.float16, device=device)
    dev = items[0][0].device
    out = torch.zeros(len(items), n_frames, 80, dtype=torch.float16, device=dev)
    t = torch.arange(n_frames, device=dev)
    groups = {}
    for j, (f, row, seek, size) in enumerate(items):
        groups.setdefault(id(f), (f, []))[1].append((j, int(row), int(seek), int(size)))
    for f, lst in groups.values():
        F = f.shape[1]
        if len(lst) == 1:
            j, row, seek, size = lst[0]
            n = max(0, min(size, F - seek, n_frames))
            if n > 0:
                out[j, :n] = f[row, seek:seek + n]
            continue
        # the four index vectors in one pinned host tensor, copied without blocking the host
        # (a pageable copy would wait for the stream: the serving step's encoder ahead of it)
        idx = torch.tensor([[r, sk, z, j] for j, r, sk, z in lst], dtype=torch.int64)
        if dev.type == "cuda":
            idx = idx.pin_memory().to(dev, non_blocking=True)
        rows, seeks, sizes, js = idx[:, 0], idx[:, 1], idx[:, 2], idx[:, 3]
        src = seeks[:, None] + t[None, :]
        valid = (t[None, :] < sizes[:, None]) & (src < F)
        g = f[rows[:, None], torch.where(valid, src, 0)]          # [n][n_frames][80]
        out[js] = torch.where(valid[..., None], g, torch.zeros((), dtype=g.dtype, device=dev))
    return out


def generate_segments(engine: WhisperEngine, audios, max_batch: int = 64, max_length: int = 448,
                      temperatures=TEMPERATURES, best_of: int = BEST_OF, utt_keys=None,
                      speculative: bool = False):
    """faster-whisper's seek loop for several 16 kHz utterances at once: every round
    decodes the current window of each unfinished utterance as one GPU batch (per-row
    prompts), then the temperature fallback of the windows whose gates failed
    (``temperatures`` = (0.0,) disables it). ``utt_keys``: the utterance numbers the
    fallback seeds are keyed on (default: the index in ``audios``; a caller that batches
    the same utterances differently passes stable numbers to draw the same noise).
    ``speculative``: each round decodes every window's T = 0 row AND the best_of hypotheses
    of every fallback temperature in ONE call (per-row temperatures), then walks the
    temperatures exactly as the sequential fallback does — the same results for one decode
    call's latency instead of up to len(temperatures) in a row, at (1 + 5 x 5) rows per
    window (the streaming encoder's setting: a few phrases at a time, latency-bound).
    Returns one _Stream (segments + gate counters) per utterance."""
    temperatures = tuple(float(t) for t in temperatures)
    if not temperatures or temperatures[0] != 0.0:
        raise NotImplementedError("the first temperature must be 0 (faster-whisper's default)")
    tk = engine.tokenizer
    dev = engine.device
    streams = [_Stream(np.asarray(a, np.float32)) for a in audios]
    # the whole clip's features, once per utterance (faster-whisper's FeatureExtractor call)
    feats = []
    for st in streams:
        if st.content_frames <= 0:
            feats.append(None)
            continue
        pcm = torch.from_numpy(np.concatenate([st.audio, np.zeros(1, np.float32)])).to(dev)
        offs = torch.tensor([0, len(st.audio)], dtype=torch.int64, device=dev)
        feats.append(engine.logmel_frames(pcm, offs, 1, 1, st.content_frames))
    spec = speculative and len(temperatures) > 1
    per_row = 1 + (len(temperatures) - 1) * best_of          # rows per window, speculative
    if spec:
        max_batch = max(1, min(max_batch, FALLBACK_ROWS // per_row))
    while True:
        act = [i for i, s in enumerate(streams) if s.active]
        if not act:
            break
        for c0 in range(0, len(act), max_batch):
            idx = act[c0:c0 + max_batch]
            grp = [streams[i] for i in idx]
            sizes = [s.window_size() for s in grp]
            mel = gather_windows([(feats[i], 0, s.seek, size) for i, s, size in zip(idx, grp, sizes)])
            enc = engine.encode(mel)
            prompts = [s.prompt(tk, max_length) for s in grp]
            keys = [(i if utt_keys is None else int(utt_keys[i]), s.windows) for i, s in zip(idx, grp)]
            pres = None
            if spec:
                temps, seeds, eidx, rprom = [], [], [], []
                for j, key in enumerate(keys):
                    temps.append(0.0)
                    seeds.append(0)
                    for ti in range(1, len(temperatures)):
                        temps += [float(temperatures[ti])] * best_of
                        seeds += [fallback_seed(key[0], key[1], ti, h) for h in range(best_of)]
                    eidx += [j] * per_row
                    rprom += [prompts[j]] * per_row
                out = engine.decode_ex(enc, prompts=rprom, max_length=max_length, temperature=temps,
                                       seeds=seeds, enc_index=eidx)
                allr = out.rows()
                t0 = [allr[j * per_row] for j in range(len(grp))]
                pres = [[allr[j * per_row + 1 + (ti - 1) * best_of: j * per_row + 1 + ti * best_of]
                         for ti in range(1, len(temperatures))] for j in range(len(grp))]
                n_tok = out.n_tokens.cpu().numpy()[0::per_row]
            else:
                out = engine.decode_ex(enc, prompts=prompts, max_length=max_length)
                t0 = out.rows()
                n_tok = out.n_tokens.cpu().numpy()
            first, final, ndec = settle_round(engine, tk, t0, prompts, keys, enc, max_length,
                                              temperatures, best_of, presampled=pres)
            for s, size, c0r, r, nd, nt in zip(grp, sizes, first, final, ndec, n_tok):
                advance(tk, s, size, c0r, r, nd, nt)
    return streams


class WhisperModel:
    """faster-whisper-shaped front of the GPU Whisper engine.

    Accepts faster-whisper's constructor arguments, including the reference's
    ``device='cpu', compute_type='int8'`` (transcriber.py:23-27), and maps every
    combination onto the one engine this build has: the gfx950 HIP kernels on the
    current device, with fp16 weights on MFMA and fp32 accumulation. ``device`` and
    ``compute_type`` are recorded (``requested_device`` / ``requested_compute_type``)
    but select nothing: there is no CPU path (the product fails loudly without a GPU)."""

    def __init__(self, model_size: str, device: str = "auto", compute_type: str = "default",
                 **_ignored):
        if model_size not in CONFIGS:
            raise ValueError(f"unknown model size {model_size!r}; one of {sorted(CONFIGS)}")
        if device not in DEVICES:
            raise ValueError(f"unsupported device {device!r}; one of {DEVICES}")
        if compute_type not in COMPUTE_TYPES:
            raise ValueError(f"unsupported compute_type {compute_type!r}")
        self.model_size = model_size
        self.requested_device, self.requested_compute_type = device, compute_type
        self.engine = WhisperEngine(CONFIGS[model_size])
        self.stats = {"windows": 0, "needs_fallback": 0, "no_speech_skips": 0, "fallback_decodes": 0}

    def transcribe(self, audio, beam_size: int = 1, language: str = "en",
                   temperature=TEMPERATURES, best_of: int = BEST_OF, **_ignored):
        if beam_size != 1:
            raise NotImplementedError("janus_amd decodes greedily (beam_size=1, transcriber.py:55)")
        if language not in (None, "en"):
            raise NotImplementedError("*.en models transcribe English only (transcriber.py:56)")
        if isinstance(audio, str):
            audio = read_wav_16k(audio)
        audio = np.ascontiguousarray(audio, dtype=np.float32)
        temps = (float(temperature),) if np.isscalar(temperature) else tuple(temperature)
        st = generate_segments(self.engine, [audio], temperatures=temps, best_of=best_of)[0]
        self._count(st)
        info = TranscriptionInfo("en", 1.0, len(audio) / 16000.0)
        return iter(st.segments), info

    def _count(self, st):
        self.stats["windows"] += st.windows
        self.stats["needs_fallback"] += st.fallbacks
        self.stats["no_speech_skips"] += st.skips
        self.stats["fallback_decodes"] += st.fallback_decodes


class Transcriber:
    def __init__(self, model_size: str = 'base.en') -> None:
        """transcriber.py:11-27, the same call (WhisperModel maps it onto the GPU engine)."""
        self.model = WhisperModel(
            model_size,
            device='cpu',
            compute_type='int8'
        )

    def transcribe_buffer(self, audio_buffer: np.ndarray) -> str:
        """transcriber.py:29-64."""
        if isinstance(audio_buffer, list):
            audio_buffer = np.concatenate(audio_buffer)
        if not isinstance(audio_buffer, np.ndarray):
            audio_buffer = np.array(audio_buffer, dtype=np.float32)
        if audio_buffer.dtype != np.float32:
            audio_buffer = audio_buffer.astype(np.float32)
        audio_16k = audio_buffer[::3]
        segments, info = self.model.transcribe(audio_16k, beam_size=1, language='en')
        text_parts = []
        for segment in segments:
            text_parts.append(segment.text.strip())
        full_text = ' '.join(text_parts).strip()
        return full_text

    def transcribe_file(self, file_path: str) -> str:
        """transcriber.py:66-91 (16-bit PCM WAV input)."""
        segments, info = self.model.transcribe(file_path, beam_size=1, language='en')
        text_parts = []
        for segment in segments:
            text_parts.append(segment.text.strip())
        full_text = ' '.join(text_parts).strip()
        return full_text

    def transcribe_batch(self, buffers) -> list:
        """Batched extension: 48 kHz buffers (any length) -> transcripts, the seek loops
        of all buffers advanced together (one GPU batch per round)."""
        auds = [np.ascontiguousarray(np.asarray(b, dtype=np.float32)[::3]) for b in buffers]
        streams = generate_segments(self.model.engine, auds)
        for st in streams:
            self.model._count(st)
        return [' '.join(s.text.strip() for s in st.segments).strip() for st in streams]


__all__ = ["Transcriber", "WhisperModel", "Segment", "TranscriptionInfo", "read_wav_16k",
           "generate_segments", "settle_round", "advance", "gather_windows", "split_window", "compression_ratio", "gates", "nat",
           "Candidate", "candidate", "best_hypothesis", "settle", "fallback_seed", "TEMPERATURES",
           "BEST_OF"]

"""Streaming encode for many concurrent capture channels (SURVEY.md §8(f) rows 1-2;
BASELINE config 5: 128 channels x 320 ms chunks over 8 GPUs, per-chunk p50 latency).

The reference runs ONE channel: ``smart_ear_loop`` (backend/services/engine.py:382-575)
pulls 1536-sample 48 kHz chunks (audio_io.py:28-31), gates them with silero VAD
(engine.py:474, vad.py:40-77), segments phrases (pre-roll 10 chunks, > 15 silent chunks
ends a phrase, phrases under 9216 samples dropped, push-to-talk hold/release:
engine.py:438-506), then transcribes + analyses prosody + packs each phrase
(process_audio_blocking / transmit_packet_blocking, engine.py:510-552) with ONE stateful
aubio detector (prosody.py:32). Here S channels advance together:

* the speech gate runs for every chunk of every channel in one launch
  (services/vad.py: the silero-v5 network with one model state per channel when local
  weights are given — ``vad_weights=`` or JANUS_VAD_DIR — else the documented energy
  stand-in; real probabilities can also be passed through ``push(..., speech=...)``);
* ``PhraseSegmenter`` is the engine's per-chunk state machine, one per channel;
* phrases that complete on the same tick are encoded as ONE batch on the GPU (log-mel,
  encoder, greedy decoder, YIN + RMS) with each channel's persistent 4096-sample detector
  buffer gathered in and scattered back, exactly one aubio object per channel.
"""
import queue
import threading
import time
from collections import deque

import numpy as np
import torch

from . import _native as nat
from .common.protocol import JanusMode, JanusPacket
from .services.prosody import YIN_BUF, energy_tag, pitch_tag, prosody_launch
from .services.transcriber import TEMPERATURES
from .services.vad import VAD_CENTER_DB, VAD_WIDTH_DB, MultiStreamGate, VoiceActivityDetector

CHUNK = 1536                  # audio_io.py:28-31 (48 kHz int16 -> f32 chunks)
PRE_ROLL_CHUNKS = 10          # engine.py:439
SILENCE_THRESHOLD_CHUNKS = 15  # engine.py:441
MIN_PHRASE_SAMPLES = CHUNK * 6  # engine.py:504
CAPTURE_RATE = 48000
WINDOW_16K = 480000           # one 30 s Whisper window at 16 kHz
MERGE_PHRASES = 256           # asynchronous worker: most phrases merged into one batch

class PhraseSegmenter:
    """engine.py:438-506 for one channel: feed every chunk with its gate decision; returns
    the phrase audio when one completes (and is long enough), else None."""

    def __init__(self):
        self.audio_buffer = []
        self.pre_roll_buffer = deque(maxlen=PRE_ROLL_CHUNKS)
        self.silence_counter = 0
        self.previous_hold_state = False
        self.is_talking = False
        self.skipped = 0  # phrases dropped as shorter than MIN_PHRASE_SAMPLES

    def push(self, chunk: np.ndarray, is_speech: bool, streaming: bool = True,
             recording: bool = False, non_vad_mode: bool = False):
        trigger = False
        if recording:                                  # :458-463 push-to-talk hold
            self.is_talking = True
            self.audio_buffer.append(chunk)
            self.previous_hold_state = True
            return None
        if self.previous_hold_state:                   # :466-469 release (chunk dropped)
            trigger = True
            self.previous_hold_state = False
            self.is_talking = False
        elif streaming:                                # :471-495
            if is_speech or non_vad_mode:
                if not self.audio_buffer:
                    self.audio_buffer.extend(list(self.pre_roll_buffer))  # pre-roll kept
                self.is_talking = True
                self.audio_buffer.append(chunk)
                self.silence_counter = 0
            else:
                self.silence_counter += 1
                if self.audio_buffer:
                    self.audio_buffer.append(chunk)
                else:
                    self.pre_roll_buffer.append(chunk)
                if self.silence_counter > SILENCE_THRESHOLD_CHUNKS:
                    trigger = True
                    self.is_talking = False
        else:                                          # :497-499
            self.is_talking = False
        if trigger and self.audio_buffer:              # :501-506
            combined = np.concatenate(self.audio_buffer)
            self.audio_buffer = []
            self.silence_counter = 0
            if len(combined) < MIN_PHRASE_SAMPLES:
                self.skipped += 1
                return None
            return combined
        return None


class StreamingEncoder:
    """S channels x one JanusPipeline-style encode per completed phrase batch.

    push(block) takes the next [S][n*1536] capture samples of every channel (numpy f32 or
    a GPU tensor) and returns completed phrases as dicts {stream, text, tags, packet}
    (packet None when the text is empty, engine.py:536).

    Synchronous (default): the phrases completed by this block, encoded before push
    returns. ``asynchronous=True``: push only gates and segments the block (the ingest
    path the reference's producer / loop threads run, engine.py:351-506) and hands the
    completed phrases to a worker thread with its own HIP stream, which encodes them (and,
    with a ``receiver``, renders the returned packets the way the far end would:
    engine.py:220-286) while the next blocks are ingested; push returns whatever finished
    since the last call, each with ``latency_s`` = phrase completion -> packet (+ audio).
    Phrases of one channel are encoded in completion order, so the per-channel aubio
    state stays sequential. ``flush()`` waits for the queue."""

    def __init__(self, n_streams: int, whisper, max_length: int = 448,
                 mode: JanusMode = JanusMode.SEMANTIC_VOICE, override="auto",
                 vad_threshold: float = 0.5, hop: int = 512, asynchronous: bool = False,
                 receiver=None, vad_weights: dict = None, temperatures=TEMPERATURES):
        """temperatures: faster-whisper's fallback schedule, as the reference's
        transcribe_buffer runs it (the default); (0.0,) decodes each window once at T = 0
        and never re-decodes (the config-5 stream bench's setting on synthetic weights,
        whose windows all fail the gates: DESIGN.md §0)."""
        self.device = nat.require_gpu()
        self.temperatures = tuple(float(t) for t in temperatures)
        self.S = n_streams
        self.whisper = whisper
        self.max_length = max_length
        self.mode, self.override, self.hop = mode, override, hop
        self.vad = MultiStreamGate(n_streams, vad_threshold, CAPTURE_RATE, vad_weights)
        self.segmenters = [PhraseSegmenter() for _ in range(n_streams)]
        # one aubio detector buffer per channel (prosody.py:32), persistent across phrases
        self.yin_state = torch.zeros(n_streams, YIN_BUF, dtype=torch.float32, device=self.device)
        self.latencies = []         # seconds per push (chunk block of all channels)
        self.phrase_latencies = []  # seconds from phrase completion to its result
        self.receiver = receiver    # JanusPipeline-like .decode(packets, frames), or None
        self.asynchronous = asynchronous
        self.max_queue = 0
        self._serial = 0      # phrases completed so far (all channels)
        self.worker_batches = 0     # asynchronous worker: batches run (merged jobs count once)
        self.long_phrases = 0       # phrases over one 30 s window
        self.extra_windows = 0      # seek-loop windows beyond each phrase's first
        if asynchronous:
            self._jobs = queue.Queue()
            self._results = queue.Queue()
            self._side = torch.cuda.Stream(device=self.device)
            self._error = None
            self._worker = threading.Thread(target=self._run, daemon=True)
            self._worker.start()

    def push(self, block, speech=None, timestamp=None):
        t0 = time.perf_counter()
        host = block.cpu().numpy() if isinstance(block, torch.Tensor) else np.asarray(block, np.float32)
        S, L = host.shape
        assert S == self.S and L % CHUNK == 0, "push [S][n*1536] samples"
        n = L // CHUNK
        if speech is None:
            dev = block if isinstance(block, torch.Tensor) and block.is_cuda else \
                torch.from_numpy(np.ascontiguousarray(host)).to(self.device)
            speech = self.vad.is_speech(dev.reshape(S, n, CHUNK).contiguous())
        done = []
        # MORSE / TEXT_ONLY bypass the speech gate (engine.py:473-474, is_non_vad_mode)
        non_vad = self.mode in (JanusMode.TEXT_ONLY, JanusMode.MORSE_CODE)
        for s in range(S):
            for j in range(n):
                ph = self.segmenters[s].push(host[s, j * CHUNK:(j + 1) * CHUNK], bool(speech[s, j]),
                                             non_vad_mode=non_vad)
                if ph is not None:
                    done.append((s, ph, self._serial))
                    self._serial += 1
        if self.asynchronous:
            if self._error is not None:
                raise RuntimeError("streaming worker failed") from self._error
            if done:
                self._jobs.put((done, timestamp, t0))
                self.max_queue = max(self.max_queue, self._jobs.qsize())
            out = self._drain()
            self.latencies.append(time.perf_counter() - t0)
            return out
        out = self._job(done, timestamp, t0) if done else []
        self.latencies.append(time.perf_counter() - t0)
        return out

    def _job(self, done, timestamp, t_submit):
        """Encode (+ render) one batch of completed phrases; t_submit: the push time of the
        phrases' block, one value or one per phrase (merged jobs)."""
        res = self._encode(done, timestamp)
        if self.receiver is not None:
            self._render(res, done)
        torch.cuda.current_stream(self.device).synchronize()
        t = time.perf_counter()
        subs = t_submit if isinstance(t_submit, list) else [t_submit] * len(res)
        for r, t0 in zip(res, subs):
            r["latency_s"] = t - t0
            self.phrase_latencies.append(t - t0)
        return res

    def _render(self, res, done):
        """The far end's receiver leg for this job's packets (ReceiverBatch semantics):
        every packet rendered at its phrase's own duration (longest phrase of the job)."""
        pk = [r["packet"] for r in res]
        if not any(p is not None for p in pk):
            return
        secs = max(len(d[1]) for d in done) / CAPTURE_RATE
        frames = max(1, int(np.ceil(secs * 44100 / 512)))
        wav, pcm, _ = self.receiver.decode(pk, frames)
        k = 0
        for r in res:
            if r["packet"] is not None and JanusPacket.deserialize(r["packet"]).mode != JanusMode.MORSE_CODE:
                r["pcm16"] = pcm[k]
                k += 1

    def _run(self):
        """The worker: every job queued while the previous one ran is merged into ONE batch
        (one batched generate_segments for all of them: a worker that fell behind catches up
        with bigger batches instead of a growing queue), in queue order, up to MERGE_PHRASES
        phrases; a channel with several phrases in the batch runs them through its YIN
        state in order (_encode's prosody rounds), and every packet keeps its own block's
        timestamp and every latency its own push time."""
        torch.cuda.set_device(self.device)
        pending = deque()
        stop = False
        while not (stop and not pending):
            if not pending:
                job = self._jobs.get()
                if job is None:
                    self._jobs.task_done()
                    return
                pending.append(job)
            while True:   # everything queued meanwhile
                try:
                    job = self._jobs.get_nowait()
                except queue.Empty:
                    break
                if job is None:
                    self._jobs.task_done()
                    stop = True
                    break
                pending.append(job)
            done, stamps, subs, taken = [], [], [], 0
            for jd, ts, t0 in pending:
                if taken and len(done) + len(jd) > MERGE_PHRASES:
                    break
                done += jd
                stamps += [ts] * len(jd)
                subs += [t0] * len(jd)
                taken += 1
            ts = stamps[0] if taken == 1 else stamps
            self.worker_batches += 1
            try:
                with torch.cuda.stream(self._side):
                    self._results.put(self._job(done, ts, subs))
            except BaseException as e:  # surfaced by the next push
                self._error = e
            finally:
                for _ in range(taken):
                    pending.popleft()
                    self._jobs.task_done()

    def _drain(self):
        out = []
        while True:
            try:
                out += self._results.get_nowait()
            except queue.Empty:
                return out

    def flush(self):
        """Asynchronous mode: wait for every queued phrase; returns the remaining results."""
        if not self.asynchronous:
            return []
        self._jobs.join()
        if self._error is not None:
            raise RuntimeError("streaming worker failed") from self._error
        return self._drain()

    def close(self):
        if self.asynchronous and self._worker.is_alive():
            self._jobs.put(None)
            self._worker.join()

    def _encode(self, done, timestamp):
        streams = [d[0] for d in done]
        lengths = [len(d[1]) for d in done]
        serials = [d[2] for d in done]   # stable phrase numbers: the fallback's seed keys
        pcm_np = np.concatenate([d[1] for d in done] + [np.zeros(1, np.float32)]).astype(np.float32)
        pcm = torch.from_numpy(pcm_np).to(self.device)
        offs_np = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
        offs = torch.from_numpy(offs_np).to(self.device)
        B = len(done)
        w = self.whisper
        # every phrase through faster-whisper's generate_segments, as the engine's
        # transcribe_buffer call runs it (engine.py:514 -> transcriber.py:29-64): the
        # phrases' first windows are one GPU batch, failing windows take the temperature
        # fallback, and a phrase whose first window's seek stops short of its content
        # (a trailing timestamp pair, or longer than 30 s) continues with the next window
        # in the following round of the same batched loop
        from .services.transcriber import generate_segments
        auds = [np.ascontiguousarray(pcm_np[offs_np[i]:offs_np[i] + lengths[i]][::3]) for i in range(B)]
        # speculative: every phrase window's T = 0 row and all its fallback hypotheses in one
        # decode call (the same results as the sequential temperature walk, one decode's
        # latency: a phrase waits for one call, not up to six in a row)
        streams_st = generate_segments(w, auds, max_length=self.max_length,
                                       temperatures=self.temperatures, utt_keys=serials,
                                       speculative=True)
        texts = [' '.join(sg.text.strip() for sg in st.segments).strip() for st in streams_st]
        self.long_phrases += sum(1 for n in lengths if (n + 2) // 3 > WINDOW_16K)
        self.extra_windows += sum(st.windows - 1 for st in streams_st)
        # prosody in rounds: round r takes every channel's r-th phrase of this tick, so a
        # channel that completed two phrases runs them in order, the second from the first's
        # end state (one aubio object per channel, prosody.py:32)
        tags = [None] * B
        seen = {}
        rounds = []
        for i, s in enumerate(streams):
            r = seen.get(s, 0)
            seen[s] = r + 1
            if r == len(rounds):
                rounds.append([])
            rounds[r].append(i)
        try:
            for members in rounds:
                if len(members) == B:
                    r_pcm, r_offs, r_len = pcm, offs, lengths
                else:
                    r_len = [lengths[i] for i in members]
                    r_pcm = torch.cat([pcm[int(offs_np[i]):int(offs_np[i]) + lengths[i]] for i in members]
                                      + [pcm.new_zeros(1)])
                    r_offs = torch.from_numpy(np.concatenate([[0], np.cumsum(r_len)]).astype(np.int64)).to(self.device)
                idx = torch.tensor([streams[i] for i in members], dtype=torch.int64, device=self.device)
                st_in = self.yin_state.index_select(0, idx).contiguous()
                st_out = torch.empty_like(st_in)
                r_tags = prosody_launch(r_pcm, r_offs, r_len, CAPTURE_RATE, self.hop,
                                        state_in=st_in, state_out=st_out).tags()
                self.yin_state.index_copy_(0, idx, st_out)  # indices distinct within a round
                for i, t in zip(members, r_tags):
                    tags[i] = t
        except Exception:                               # engine.py:520-525
            tags = [{"energy": "Normal", "pitch": "Normal"} for _ in range(B)]
        stamps = timestamp if isinstance(timestamp, list) else [timestamp] * B
        now = time.time()
        res = []
        for s, t, g, ts in zip(streams, texts, tags, stamps):
            ts = now if ts is None else ts
            pkt = JanusPacket(t, self.mode, g, self.override, ts).serialize() if t.strip() else None
            res.append({"stream": s, "text": t, "tags": g, "packet": pkt})
        return res

    def p50_ms(self) -> float:
        return float(np.median(self.latencies) * 1000.0) if self.latencies else float("nan")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["PhraseSegmenter", "VoiceActivityDetector", "StreamingEncoder", "energy_tag",
           "pitch_tag", "CHUNK", "MIN_PHRASE_SAMPLES"]

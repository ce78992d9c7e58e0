"""Whisper English-only token space and detokenisation (host side).

Special-token layout of the ``*.en`` Whisper vocabulary (51 864 ids; GPT-2 byte-level
BPE in 0..50255): <|endoftext|> 50256, <|startoftranscript|> 50257, 99 language tokens,
<|translate|> 50357, <|transcribe|> 50358, <|startoflm|> 50359, <|startofprev|> 50360,
<|nocaptions|> 50361, <|notimestamps|> 50362, timestamps <|0.00|>..<|30.00|> from 50363.

No tokenizer files exist offline. If ``JANUS_WHISPER_DIR`` holds a Hugging Face
``tokenizer.json``, it is used through the ``tokenizers`` package; otherwise a
deterministic synthetic vocabulary of the same size is used: ids 0..255 are the 256
GPT-2 byte symbols (so id 220 is " " exactly as in GPT-2) and ids 256..50255 are seeded
pseudo-words, ~70 % with a leading space like BPE "Ġ" tokens.

Segment assembly follows faster-whisper's greedy path for one window
(``_split_segments_by_timestamps`` + ``' '.join(seg.text.strip())``,
transcriber.py:59-64).
"""
import os

import numpy as np

EOT = 50256
SOT = 50257
TRANSLATE = 50357
TRANSCRIBE = 50358
SOT_LM = 50359
SOT_PREV = 50360
NO_SPEECH = 50361
NO_TIMESTAMPS = 50362
TIMESTAMP_BEGIN = 50363
N_VOCAB_EN = 51864
BLANK = 220

# openai/whisper tokenizer.non_speech_tokens symbol set
_SYMBOLS = list("\"#()*+/:;<=>@[\\]^_`{|}~「」『』") + \
    "<< >> <<< >>> -- --- -( -[ (' (\" (( )) ((( ))) [[ ]] {{ }} ♪♪ ♪♪♪".split()
_MISC = set("♩♪♫♬♭♮♯")


def bytes_to_unicode_order():
    """GPT-2's byte order: id k < 256 is byte order[k]."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    rest = [b for b in range(256) if b not in bs]
    return bs + rest


class WhisperTokenizer:
    def __init__(self, path: str = None, seed: int = 1234):
        self.eot, self.sot = EOT, SOT
        self.timestamp_begin = TIMESTAMP_BEGIN
        self.no_timestamps = NO_TIMESTAMPS
        self.blank = BLANK
        self.sot_sequence = [SOT]  # *.en: no language / task tokens
        self._hf = None
        if path and os.path.exists(os.path.join(path, "tokenizer.json")):
            from tokenizers import Tokenizer
            self._hf = Tokenizer.from_file(os.path.join(path, "tokenizer.json"))
            # the decoder's prompt and rules use the *.en special-token ids: the file must agree
            for name, want in (("<|endoftext|>", EOT), ("<|startoftranscript|>", SOT),
                               ("<|startofprev|>", SOT_PREV), ("<|notimestamps|>", NO_TIMESTAMPS)):
                got = self._hf.token_to_id(name)
                if got != want:
                    raise ValueError(f"tokenizer.json: {name} is {got}, expected {want} (*.en layout)")
            ts0 = self._hf.token_to_id("<|0.00|>")
            if ts0 is not None and ts0 != TIMESTAMP_BEGIN:
                raise ValueError(f"tokenizer.json: <|0.00|> is {ts0}, expected {TIMESTAMP_BEGIN}")
        else:
            self._table = self._synthetic_table(seed)

    @staticmethod
    def _synthetic_table(seed):
        order = bytes_to_unicode_order()
        table = [bytes([order[k]]) for k in range(256)]
        rng = np.random.default_rng(seed)
        cons = list("bcdfghjklmnprstvwz")
        vows = list("aeiou")
        for _ in range(256, EOT):
            n = int(rng.integers(1, 4))
            word = "".join(cons[rng.integers(len(cons))] + vows[rng.integers(len(vows))]
                           for _ in range(n))
            if rng.random() < 0.7:
                word = " " + word
            table.append(word.encode())
        return table

    def encode_text(self, text: str):
        if self._hf is not None:
            return self._hf.encode(text, add_special_tokens=False).ids
        order = bytes_to_unicode_order()
        inv = {b: k for k, b in enumerate(order)}
        return [inv[b] for b in text.encode("utf-8")]

    def decode(self, tokens) -> str:
        a = np.asarray(tokens, dtype=np.int64).reshape(-1)
        toks = a[(a >= 0) & (a < self.eot)].tolist()   # text tokens only (vectorised filter)
        if self._hf is not None:
            return self._hf.decode(toks)
        return b"".join(map(self._table.__getitem__, toks)).decode("utf-8", errors="replace")

    def non_speech_tokens(self):
        if self._hf is None:
            order = bytes_to_unicode_order()
            inv = {b: k for k, b in enumerate(order)}
            out = set()
            for sym in _SYMBOLS:
                b = sym.encode("utf-8")
                out.add(inv[b[0]])
            return sorted(out)
        out = {self.encode_text(" -")[0], self.encode_text(" '")[0]}
        for sym in _SYMBOLS + sorted(_MISC):
            for tokens in (self.encode_text(sym), self.encode_text(" " + sym)):
                if len(tokens) == 1 or sym in _MISC:
                    out.add(tokens[0])
        return sorted(out)

    def suppress_tokens(self):
        """faster-whisper get_suppressed_tokens(tokenizer, [-1])."""
        s = set(self.non_speech_tokens())
        s.update([TRANSCRIBE, TRANSLATE, SOT, SOT_PREV, SOT_LM])
        return sorted(s)

    def segments(self, sampled):
        """Split sampled tokens (up to, excluding, <|endoftext|>) the way faster-whisper's
        single-window greedy path does; returns list of (start_ts, end_ts, text)."""
        toks = []
        for t in sampled:
            t = int(t)
            if t == self.eot or t < 0:
                break
            toks.append(t)
        tb = self.timestamp_begin
        single_ending = len(toks) >= 2 and toks[-2] < tb <= toks[-1]
        consecutive = [i for i in range(1, len(toks)) if toks[i] >= tb and toks[i - 1] >= tb]
        segs = []
        if consecutive:
            slices = list(consecutive)
            if single_ending:
                slices.append(len(toks))
            last = 0
            for cur in slices:
                part = toks[last:cur]
                segs.append(self._seg(part))
                last = cur
            if last < len(toks):  # single window: keep the trailing partial segment
                segs.append(self._seg(toks[last:]))
        else:
            segs.append(self._seg(toks))
        return segs

    def _seg(self, part):
        ts = [t for t in part if t >= self.timestamp_begin]
        start = (ts[0] - self.timestamp_begin) * 0.02 if ts else 0.0
        end = (ts[-1] - self.timestamp_begin) * 0.02 if ts else 0.0
        return (start, end, self.decode(part))

    def transcript(self, sampled) -> str:
        if self._hf is None:
            return self._transcript_table(sampled)
        parts = [text.strip() for (_, _, text) in self.segments(sampled)]
        return " ".join(parts).strip()

    def _transcript_table(self, sampled) -> str:
        """transcript() for the table vocabulary with numpy index work (same segments,
        same text): the per-token Python loop cost ~0.4 ms per 447-token row."""
        if getattr(self, "_table_np", None) is None:
            self._table_np = np.empty(len(self._table), dtype=object)
            self._table_np[:] = self._table
        a = np.asarray(sampled, dtype=np.int64).ravel()
        stop = np.nonzero((a == self.eot) | (a < 0))[0]
        toks = a[: stop[0]] if stop.size else a
        n = toks.size
        tb = self.timestamp_begin
        ts = toks >= tb
        consecutive = (np.nonzero(ts[1:] & ts[:-1])[0] + 1).tolist() if n > 1 else []
        if consecutive:
            single_ending = n >= 2 and toks[-2] < tb <= toks[-1]
            bounds = [0] + consecutive + ([n] if single_ending else [])
            if bounds[-1] < n:
                bounds.append(n)
        else:
            bounds = [0, n]
        # text tokens per part from a prefix count: parts without any decode to ""
        is_text = (toks >= 0) & (toks < self.eot)
        csum = np.concatenate([[0], np.cumsum(is_text)])
        texts = []
        for i in range(len(bounds) - 1):
            lo, hi = bounds[i], bounds[i + 1]
            if csum[hi] == csum[lo]:
                texts.append("")
                continue
            part = toks[lo:hi]
            sel = part[is_text[lo:hi]]
            texts.append(b"".join(self._table_np[sel]).decode("utf-8", errors="replace").strip())
        return " ".join(texts).strip()


def load_tokenizer():
    return WhisperTokenizer(os.environ.get("JANUS_WHISPER_DIR"))


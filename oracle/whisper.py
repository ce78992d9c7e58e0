"""ORACLE — test infrastructure only (see oracle/__init__.py).

fp32/fp64 CPU restatement of the reference's STT path (transcriber.py:29-64 ->
faster-whisper WhisperModel.transcribe(audio[::3], beam_size=1, language='en')):

* ``logmel``: faster-whisper FeatureExtractor (numpy STFT, n_fft 400, hop 160,
  periodic Hann, center/reflect, 30 s of right zero padding, |rfft|^2, slaney mel,
  log10 clamp, global-max - 8, (x+4)/4), float64 FFT. Pinned against the third-party
  transformers WhisperFeatureExtractor (tests/test_oracle_whisper.py).
* ``encoder`` / ``decoder_logits``: Whisper encoder and decoder forward in fp32 torch,
  pinned against transformers' WhisperModel loaded with the same weights.
* ``greedy``: temperature-0 decoding with OpenAI's SuppressBlank, SuppressTokens and
  ApplyTimestampRules (incl. max_initial_timestamp 1.0 s) that CTranslate2 applies for
  faster-whisper; the rules are pinned to transformers' logits processors
  (tests/test_oracle_whisper.py).
* ``greedy_cached(temperature > 0, seeds)``: sampling as the build defines it for
  faster-whisper's temperature fallback (generate_with_fallback): Gumbel-max over the
  rule-filtered logits / T with the counter-based noise of ``sample_noise`` (the same hash
  as decoder.h noise_base / sample_gumbel). CTranslate2's own random draws cannot be
  reproduced offline, so the draws are build-defined; the distribution is softmax(l / T)
  over the filtered set either way.
* ``transcribe_segments``: generate_segments with the fallback loop
  (generate_with_fallback: temperatures 0.2 ... 1.0, best_of 5, settle rules,
  prompt_reset_on_temperature 0.5), restated from faster-whisper 1.x transcribe.py.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def logmel(x, decim=3, filters=None, n_frames=3000, zero_pad=True):
    """float32 [n_frames][80]; ``filters`` is [201][80] (janus_amd.whisper.mel_filters).
    faster-whisper's features: the log-mel of the clip padded with 30 s of zeros,
    normalised with the maximum over every frame, of which only the content frames
    (len(x16) // 160) are used — a window is sliced from them and padded with ZEROS to 3000
    frames (generate_segments: features[:, seek:seek + segment_size], pad_or_trim). So rows
    from len(x16) // 160 on are 0.0 here. n_frames=None returns the content frames alone
    (the whole-clip features a seek loop slices). zero_pad=False keeps the log-mel of the
    zero padding instead (the build-defined voice embedding, janus_vocoder_speaker)."""
    x16 = np.asarray(x, np.float32)[::decim].astype(np.float64)
    n_samples = 480000
    padded = np.pad(x16, (0, n_samples))               # faster-whisper: padding=30 s
    y = np.pad(padded, (200, 200), mode="reflect")     # center=True
    nfr = 1 + (len(y) - 400) // 160
    idx = np.arange(400)[None, :] + 160 * np.arange(nfr)[:, None]
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(400) / 400)
    spec = np.fft.rfft(y[idx] * win[None, :], axis=1)
    power = np.abs(spec[:-1]) ** 2                       # drop last frame
    mel = power @ filters.astype(np.float64)
    lg = np.log10(np.maximum(mel, 1e-10))
    lg = np.maximum(lg, lg.max() - 8.0)
    lg = (lg + 4.0) / 4.0
    content = len(x16) // 160
    if not zero_pad:
        return lg[:n_frames].astype(np.float32)
    if n_frames is None:
        return lg[:content].astype(np.float32)
    out = np.zeros((n_frames, lg.shape[1]), np.float32)
    k = min(n_frames, content)
    out[:k] = lg[:k]
    return out


def window(features, seek, n_frames=3000):
    """generate_segments' window: features[seek:seek + min(3000, content - seek)] padded
    with zeros to 3000 frames (pad_or_trim)."""
    size = min(n_frames, len(features) - seek)
    out = np.zeros((n_frames, features.shape[1]), np.float32)
    out[:size] = features[seek:seek + size]
    return out


def _t(W, name):
    return torch.from_numpy(np.asarray(W[name], np.float32))


def _ln(x, W, p):
    return F.layer_norm(x, (x.shape[-1],), _t(W, p + ".weight"), _t(W, p + ".bias"), 1e-5)


def _lin(x, W, p, bias=True):
    b = _t(W, p + ".bias") if (bias and (p + ".bias") in W) else None
    return F.linear(x, _t(W, p + ".weight"), b)


def _mha(xq, xkv, W, p, n_heads, mask=None):
    q = _lin(xq, W, p + ".q_proj")
    k = _lin(xkv, W, p + ".k_proj", bias=False)
    v = _lin(xkv, W, p + ".v_proj")
    B, Tq, d = q.shape
    Tk = k.shape[1]
    hd = d // n_heads
    q = q.view(B, Tq, n_heads, hd).transpose(1, 2)
    k = k.view(B, Tk, n_heads, hd).transpose(1, 2)
    v = v.view(B, Tk, n_heads, hd).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    if mask is not None:
        s = s + mask
    o = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, Tq, d)
    return _lin(o, W, p + ".out_proj")


@torch.no_grad()
def encoder(mel, W, cfg):
    """mel: [B][3000][80] -> [B][1500][d] (fp32)."""
    x = torch.as_tensor(np.asarray(mel, np.float32)).transpose(1, 2)  # [B][80][3000]
    x = F.gelu(F.conv1d(x, _t(W, "encoder.conv1.weight"), _t(W, "encoder.conv1.bias"), padding=1))
    x = F.gelu(F.conv1d(x, _t(W, "encoder.conv2.weight"), _t(W, "encoder.conv2.bias"), stride=2,
                        padding=1))
    x = x.transpose(1, 2) + _t(W, "encoder.embed_positions.weight")
    for i in range(cfg.enc_layers):
        p = f"encoder.layers.{i}"
        x = x + _mha(_ln(x, W, p + ".self_attn_layer_norm"), _ln(x, W, p + ".self_attn_layer_norm"),
                     W, p + ".self_attn", cfg.n_heads)
        h = _ln(x, W, p + ".final_layer_norm")
        x = x + _lin(F.gelu(_lin(h, W, p + ".fc1")), W, p + ".fc2")
    return _ln(x, W, "encoder.layer_norm")


@torch.no_grad()
def decoder_logits(tokens, enc, W, cfg):
    """Full-sequence decoder forward: tokens [B][T] -> logits [B][T][V] (fp32)."""
    tokens = torch.as_tensor(np.asarray(tokens, np.int64))
    enc = torch.as_tensor(enc, dtype=torch.float32)
    B, T = tokens.shape
    x = _t(W, "decoder.embed_tokens.weight")[tokens] + _t(W, "decoder.embed_positions.weight")[:T]
    mask = torch.full((T, T), float("-inf")).triu(1)
    for i in range(cfg.dec_layers):
        p = f"decoder.layers.{i}"
        h = _ln(x, W, p + ".self_attn_layer_norm")
        x = x + _mha(h, h, W, p + ".self_attn", cfg.n_heads, mask)
        h = _ln(x, W, p + ".encoder_attn_layer_norm")
        x = x + _mha(h, enc, W, p + ".encoder_attn", cfg.n_heads)
        h = _ln(x, W, p + ".final_layer_norm")
        x = x + _lin(F.gelu(_lin(h, W, p + ".fc1")), W, p + ".fc2")
    x = _ln(x, W, "decoder.layer_norm")
    return x @ _t(W, "decoder.embed_tokens.weight").T


def _mix32(h):
    """murmur3 finaliser on uint32 numpy arrays (decoder.h noise_mix)."""
    h = np.asarray(h, np.uint32).copy()
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x85EBCA6B)
    h ^= h >> np.uint32(13)
    h *= np.uint32(0xC2B2AE35)
    h ^= h >> np.uint32(16)
    return h


def sample_noise(seed, pos, V):
    """Gumbel(0, 1) noise [V] (float64) of one row at one position: decoder.h
    noise_base(seed, pos) mixed with each token id, u = odd multiple of 2^-24."""
    with np.errstate(over="ignore"):
        base = _mix32(np.uint32(seed) ^ _mix32(np.uint32((pos * 0x9E3779B9 + 0x7F4A7C15) & 0xFFFFFFFF)))
        h = _mix32(base ^ (np.arange(V, dtype=np.uint32) * np.uint32(0x27D4EB2F)))
    u = ((h >> np.uint32(8)) | np.uint32(1)).astype(np.float64) * 2.0 ** -24
    return -np.log(-np.log(u))


def apply_rules(logits, sampled, tk, suppress, max_initial=50, timestamps=True):
    """OpenAI decoding filters on one row of logits (numpy f64, modified copy) given the
    tokens sampled so far (after the prompt). Returns (filtered logits, log-probs)."""
    L = np.array(logits, np.float64)
    L[list(suppress)] = -np.inf
    if len(sampled) == 0:                     # SuppressBlank
        L[[tk.blank, tk.eot]] = -np.inf
    if timestamps:
        tb = tk.timestamp_begin
        L[tk.no_timestamps] = -np.inf
        last_ts = len(sampled) >= 1 and sampled[-1] >= tb
        pen_ts = len(sampled) < 2 or sampled[-2] >= tb
        if last_ts:
            if pen_ts:
                L[tb:] = -np.inf
            else:
                L[:tk.eot] = -np.inf
        stamps = [t for t in sampled if t >= tb]
        if stamps:
            last = stamps[-1] if (last_ts and not pen_ts) else stamps[-1] + 1
            L[tb:last] = -np.inf
        if len(sampled) == 0:
            L[:tb] = -np.inf
            if max_initial is not None:
                L[tb + max_initial + 1:] = -np.inf
        m = L.max()
        lp = L - (m + np.log(np.exp(L - m).sum()))
        ts_lp = np.logaddexp.reduce(lp[tb:])
        text_max = lp[:tb].max()
        if ts_lp > text_max:
            L[:tb] = -np.inf
    m = L.max()
    lp = L - (m + np.log(np.exp(L - m).sum()))
    return L, lp


@torch.no_grad()
def greedy_cached(enc, W, cfg, tk, max_length=448, timestamps=True, prompts=None, no_speech=None,
                  temperature=0.0, seeds=None):
    """Batched greedy decode with per-layer K/V caches (fp32), the same algorithm as
    ``greedy`` (one full forward per step) at O(T) per step instead of O(T^2):
    enc [B][1500][d] -> per row a dict(tokens=[sampled incl. eot], margins=[top-2 gap
    of the rule-filtered logits per step], sum_lp=float, nsp=float). Rows that emitted
    eot stop. ``prompts``: per-row prompt token lists (default the SOT sequence); row b
    samples from position len(prompts[b]) on. ``no_speech``: token whose raw softmax
    probability at the row's first sampled step is reported as nsp. ``temperature`` > 0:
    sample (Gumbel-max, key = filtered logit * f32(1/T) + sample_noise(seeds[b], pos));
    margins are then the top-2 gaps of the keys and sum_lp the untempered log-probs."""
    inv_t = float(np.float32(1.0) / np.float32(temperature)) if temperature > 0 else 0.0
    enc = torch.as_tensor(enc, dtype=torch.float32)
    B, Te, d = enc.shape
    H, hd = cfg.n_heads, d // cfg.n_heads
    suppress = tk.suppress_tokens()
    prompts = [list(tk.sot_sequence)] * B if prompts is None else [list(p) for p in prompts]
    E = _t(W, "decoder.embed_tokens.weight")
    P = _t(W, "decoder.embed_positions.weight")

    def heads(t):
        return t.view(t.shape[0], -1, H, hd).transpose(1, 2)   # [B][H][T][hd]

    ck, cv = [], []
    for i in range(cfg.dec_layers):
        p = f"decoder.layers.{i}.encoder_attn"
        ck.append(heads(_lin(enc, W, p + ".k_proj", bias=False)))
        cv.append(heads(_lin(enc, W, p + ".v_proj")))
    sk = [None] * cfg.dec_layers
    sv = [None] * cfg.dec_layers
    seqs = [list(p) for p in prompts]
    out = [dict(tokens=[], margins=[], sum_lp=0.0, nsp=0.0) for _ in range(B)]
    done = [False] * B
    for pos in range(max_length - 1):
        tok = torch.tensor([s[pos] if pos < len(s) else tk.eot for s in seqs])
        x = (E[tok] + P[pos])[:, None]                          # [B][1][d]
        for i in range(cfg.dec_layers):
            p = f"decoder.layers.{i}"
            h = _ln(x, W, p + ".self_attn_layer_norm")
            q = heads(_lin(h, W, p + ".self_attn.q_proj"))
            k = heads(_lin(h, W, p + ".self_attn.k_proj", bias=False))
            v = heads(_lin(h, W, p + ".self_attn.v_proj"))
            sk[i] = k if sk[i] is None else torch.cat([sk[i], k], 2)
            sv[i] = v if sv[i] is None else torch.cat([sv[i], v], 2)
            s = (q @ sk[i].transpose(-1, -2)) / math.sqrt(hd)
            o = (s.softmax(-1) @ sv[i]).transpose(1, 2).reshape(B, 1, d)
            x = x + _lin(o, W, p + ".self_attn.out_proj")
            h = _ln(x, W, p + ".encoder_attn_layer_norm")
            q = heads(_lin(h, W, p + ".encoder_attn.q_proj"))
            s = (q @ ck[i].transpose(-1, -2)) / math.sqrt(hd)
            o = (s.softmax(-1) @ cv[i]).transpose(1, 2).reshape(B, 1, d)
            x = x + _lin(o, W, p + ".encoder_attn.out_proj")
            h = _ln(x, W, p + ".final_layer_norm")
            x = x + _lin(F.gelu(_lin(h, W, p + ".fc1")), W, p + ".fc2")
        if pos + 1 < min(len(p) for p in prompts):
            continue                                            # every row inside its prompt
        logits = (_ln(x, W, "decoder.layer_norm") @ E.T)[:, 0].numpy()
        for b in range(B):
            if done[b] or pos + 1 < len(prompts[b]):
                continue
            if pos + 1 == len(prompts[b]) and no_speech is not None:
                raw = logits[b].astype(np.float64)
                out[b]["nsp"] = float(np.exp(raw[no_speech] - raw.max()) / np.exp(raw - raw.max()).sum())
            L, lp = apply_rules(logits[b], out[b]["tokens"], tk, suppress, timestamps=timestamps)
            if inv_t > 0:
                L = np.where(np.isfinite(L), L * inv_t + sample_noise(seeds[b], pos, len(L)), -np.inf)
            nxt = int(np.argmax(L))
            top2 = np.partition(L[np.isfinite(L)], -2)[-2:] if np.isfinite(L).sum() >= 2 else [L.max(), -np.inf]
            out[b]["margins"].append(float(top2[-1] - top2[-2]))
            out[b]["tokens"].append(nxt)
            out[b]["sum_lp"] += float(lp[nxt])
            seqs[b].append(nxt)
            if nxt == tk.eot:
                done[b] = True
        if all(done):
            break
    return out


@torch.no_grad()
def greedy(enc, W, cfg, tk, max_length=448, timestamps=True):
    """Greedy decode of one utterance (enc [1500][d]); returns sampled tokens incl. eot."""
    suppress = tk.suppress_tokens()
    seq = list(tk.sot_sequence)
    sampled = []
    enc = torch.as_tensor(enc, dtype=torch.float32)[None]
    while len(seq) < max_length:
        logits = decoder_logits(np.array([seq]), enc, W, cfg)[0, -1].numpy()
        L, lp = apply_rules(logits, sampled, tk, suppress, timestamps=timestamps)
        nxt = int(np.argmax(L))
        seq.append(nxt)
        sampled.append(nxt)
        if nxt == tk.eot:
            break
    return sampled


def fallback_seed(utt, window, temp_index, hyp):
    """Per-hypothesis noise seed (janus_amd transcriber.fallback_seed, restated)."""
    m = lambda h: int(_mix32(np.uint32(h & 0xFFFFFFFF)))
    return m(0x4A414E55 ^ m(utt * 0x01000193 + window * 0x9E3779B1 + temp_index * 0x85EBCA77 + hyp))


def transcribe_segments(audio16k, W, cfg, tk, filters, max_length=448, enc_fp16=True,
                        temperatures=(0.0, 0.2, 0.4, 0.6, 0.8, 1.0), best_of=5, utt=0,
                        given=None):
    """faster-whisper generate_segments (beam_size=1, every other option at its default)
    over one 16 kHz utterance, restated with this module's log-mel / encoder / decoder,
    including generate_with_fallback: a window failing its gates (compression ratio > 2.4
    or avg_logprob < -1, unless no_speech_prob > 0.6) is re-decoded at each further
    temperature with best_of sampled hypotheses (the best by sum_lp / len first), the
    first passing result kept, else the best avg_logprob among those with compression
    ratio <= 2.4 (else all) reported at the last temperature; a settled temperature above
    0.5 resets the prompt. ``utt``: the utterance index the noise seeds are keyed on.
    Returns (segments [(start, end, text, tokens)], dict(windows, needs_fallback, skips,
    fallback_decodes, trace = [(seek, size, prompt)] per window)). The encoder output is
    rounded to fp16 (``enc_fp16``). ``given``: per window (sampled tokens without eot,
    avg_logprob, no-speech probability) of a decode done elsewhere (T = 0 only) — the loop's
    seek / prompt / segment bookkeeping restated over another decoder's results, no model
    run."""
    import zlib
    audio16k = np.asarray(audio16k, np.float32)
    tb = tk.timestamp_begin
    content = len(audio16k) // 160
    features = logmel(audio16k, 1, filters, n_frames=None) if given is None else None
    seek, all_tokens, segs, reset_since = 0, [], [], 0
    cnt = dict(windows=0, needs_fallback=0, skips=0, fallback_decodes=0, trace=[])

    def judge(r, temp):
        toks = [t for t in r["tokens"] if t != tk.eot]
        avg = r["sum_lp"] / (len(toks) + 1)
        text = tk.decode(toks).strip()
        b = text.encode()
        cr = len(b) / len(zlib.compress(b))
        needs = cr > 2.4 or avg < -1.0
        if r["nsp"] > 0.6 and avg < -1.0:
            needs = False
        return dict(toks=toks, avg=avg, cr=cr, nsp=r["nsp"], needs=needs, temp=temp)

    while seek < content:
        size = min(3000, content - seek)
        prev = all_tokens[reset_since:]
        prompt = ([tk.sot_prev if hasattr(tk, "sot_prev") else 50360] +
                  prev[-(max_length // 2 - 1):] if prev else []) + list(tk.sot_sequence)
        cnt["trace"].append((seek, size, list(prompt)))
        if given is not None:
            if cnt["windows"] >= len(given):
                raise ValueError("given: fewer windows than the seek loop runs")
            g_toks, g_lp, g_nsp = given[cnt["windows"]]
            r0 = judge(dict(tokens=list(g_toks), sum_lp=float(g_lp) * (len(g_toks) + 1),
                            nsp=float(g_nsp)), 0.0)
            temperatures = (0.0,)
        else:
            mel = window(features, seek)[None]
            enc = encoder(mel, W, cfg)
            if enc_fp16:
                enc = enc.half().float()
            r0 = judge(greedy_cached(enc, W, cfg, tk, max_length, prompts=[prompt], no_speech=50361)[0], 0.0)
        results, final = [r0], (r0 if not r0["needs"] else None)
        for ti in range(1, len(temperatures)):
            if final is not None:
                break
            T = temperatures[ti]
            seeds = [fallback_seed(utt, cnt["windows"], ti, h) for h in range(best_of)]
            hyps = greedy_cached(enc.expand(best_of, -1, -1), W, cfg, tk, max_length,
                                 prompts=[prompt] * best_of, no_speech=50361, temperature=T,
                                 seeds=seeds)
            cnt["fallback_decodes"] += 1
            js = [judge(h, T) for h in hyps]
            score = [j["avg"] * (len(j["toks"]) + 1) / max(len(j["toks"]), 1) for j in js]
            best = js[int(np.argmax(score))]
            results.append(best)
            if not best["needs"]:
                final = best
        if final is None:
            if len(results) == 1:
                final = r0          # fallback disabled (temperatures = (0.0,))
            else:
                pool = [r for r in results if not r["cr"] > 2.4] or results
                final = dict(pool[int(np.argmax([r["avg"] for r in pool]))], temp=temperatures[-1])
        cnt["windows"] += 1
        cnt["needs_fallback"] += int(r0["needs"])
        toks, avg = final["toks"], final["avg"]
        if final["nsp"] > 0.6 and not avg > -1.0:
            cnt["skips"] += 1
            seek += size
            continue
        t0 = seek * 0.01
        single = len(toks) >= 2 and toks[-2] < tb <= toks[-1]
        cons = [i for i in range(1, len(toks)) if toks[i] >= tb and toks[i - 1] >= tb]
        cur = []
        if cons:
            sl = cons + ([len(toks)] if single else [])
            last = 0
            for c in sl:
                part = toks[last:c]
                cur.append((t0 + (part[0] - tb) * 0.02, t0 + (part[-1] - tb) * 0.02, part))
                last = c
            nseek = seek + size if single else seek + (toks[last - 1] - tb) * 2
        else:
            st = [t for t in toks if t >= tb]
            dur = (st[-1] - tb) * 0.02 if st and st[-1] != tb else size * 0.01
            cur.append((t0, t0 + dur, toks))
            nseek = seek + size
        seek = nseek if nseek > seek else seek + size
        for (s0, s1, part) in cur:
            txt = tk.decode(part)
            if s0 == s1 or not txt.strip():
                continue
            all_tokens.extend(part)
            segs.append((s0, s1, txt, part))
        if final["temp"] > 0.5:           # prompt_reset_on_temperature
            reset_since = len(all_tokens)
    return segs, cnt

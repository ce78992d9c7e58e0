"""Oracle pinning for the STT path (CPU): the log-mel and encoder/decoder restatements
agree with the third-party transformers Whisper implementation on the same inputs and
seeded weights (the reference's own tests mock WhisperModel, test_input_processing.py:73-90,
so transformers is the available pin)."""
import numpy as np
import pytest
import torch

from janus_amd import tokenizer as tkz
from janus_amd.whisper import WhisperConfig, mel_filters, synthetic_weights
from janus_amd.workload import synth_speech
from oracle import whisper as ow


def test_logmel_matches_transformers():
    from transformers import WhisperFeatureExtractor
    x16 = synth_speech(11, 12.0, sr=16000)
    ref = WhisperFeatureExtractor(feature_size=80)(x16, sampling_rate=16000,
                                                  return_tensors="np").input_features[0]
    ours = ow.logmel(x16, decim=1, filters=mel_filters())
    assert ours.shape == (3000, 80)
    c = len(x16) // 160          # content frames: transformers pads the AUDIO to 30 s,
    assert np.abs(ours[:c] - ref.T[:c]).max() < 1e-4   # faster-whisper the features
    assert not ours[c:].any()    # with zeros (pad_or_trim of the content frames)
    full = ow.logmel(x16, decim=1, filters=mel_filters(), n_frames=None)
    assert full.shape == (c, 80) and np.array_equal(ow.window(full, 0), ours)


def test_decimation_matches_slicing():
    x48 = synth_speech(12, 3.0)
    a = ow.logmel(x48, decim=3, filters=mel_filters())
    b = ow.logmel(x48[::3], decim=1, filters=mel_filters())
    assert np.array_equal(a, b)


SMALL = WhisperConfig("pin", d_model=128, n_heads=2, enc_layers=2, dec_layers=2, n_vocab=51864)


def _hf_model(W, cfg):
    from transformers import WhisperConfig as HC, WhisperModel
    hc = HC(vocab_size=cfg.n_vocab, num_mel_bins=80, encoder_layers=cfg.enc_layers,
            encoder_attention_heads=cfg.n_heads, decoder_layers=cfg.dec_layers,
            decoder_attention_heads=cfg.n_heads, d_model=cfg.d_model,
            encoder_ffn_dim=4 * cfg.d_model, decoder_ffn_dim=4 * cfg.d_model,
            max_source_positions=1500, max_target_positions=448, activation_function="gelu")
    m = WhisperModel(hc).eval()
    sd = {k: torch.from_numpy(v) for k, v in W.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("k_proj.bias" in k for k in missing), missing
    return m


def test_encoder_decoder_match_transformers():
    W = synthetic_weights(SMALL, seed=3)
    m = _hf_model(W, SMALL)
    mel = ow.logmel(synth_speech(13, 5.0), decim=3, filters=mel_filters())[None]
    with torch.no_grad():
        ref_enc = m.encoder(torch.from_numpy(mel).transpose(1, 2)).last_hidden_state
    enc = ow.encoder(mel, W, SMALL)
    assert torch.allclose(enc, ref_enc, atol=2e-4, rtol=1e-4)
    toks = np.array([[tkz.SOT, tkz.TIMESTAMP_BEGIN, 400, 1234, 77]])
    with torch.no_grad():
        h = m.decoder(input_ids=torch.from_numpy(toks), encoder_hidden_states=ref_enc).last_hidden_state
        ref_logits = h @ torch.from_numpy(W["decoder.embed_tokens.weight"]).T
    logits = ow.decoder_logits(toks, enc, W, SMALL)
    assert torch.allclose(logits, ref_logits, atol=1e-3, rtol=1e-4)


def test_greedy_cached_matches_full_recompute():
    """The KV-cached batched greedy (used at full length on the GPU box) takes the same
    tokens as the full-recompute restatement."""
    W = synthetic_weights(SMALL, seed=4)
    tk = tkz.WhisperTokenizer()
    mels = np.stack([ow.logmel(synth_speech(20 + k, 2.0 + k), decim=3, filters=mel_filters()) for k in range(2)])
    enc = ow.encoder(mels, W, SMALL)
    fast = ow.greedy_cached(enc, W, SMALL, tk, max_length=14)
    for b in range(2):
        slow = ow.greedy(enc[b], W, SMALL, tk, max_length=14)
        assert fast[b]["tokens"] == slow, b
        assert len(fast[b]["margins"]) == len(slow) and min(fast[b]["margins"]) >= 0


def test_synthetic_weights_fp16_exact():
    """Weight matrices are fp16-representable: the GPU holds them as fp16 without rounding,
    so the fp32 oracle and the engine multiply the same numbers."""
    from janus_amd.whisper import FP32_MATRICES
    W = synthetic_weights(SMALL, seed=1)
    for k, v in W.items():
        if v.ndim >= 2 and k not in FP32_MATRICES:
            assert np.array_equal(v, v.astype(np.float16).astype(np.float32)), k
    # the fp32-consumed positional table keeps full precision
    pos = W["decoder.embed_positions.weight"]
    assert not np.array_equal(pos, pos.astype(np.float16).astype(np.float32))


def test_timestamp_rules():
    tk = tkz.WhisperTokenizer()
    V = tkz.N_VOCAB_EN
    rng = np.random.default_rng(0)
    logits = rng.standard_normal(V)
    supp = tk.suppress_tokens()
    # first step: only timestamps <= 1.0 s allowed
    L, _ = ow.apply_rules(logits, [], tk, supp)
    allowed = np.nonzero(np.isfinite(L))[0]
    assert allowed.min() >= tk.timestamp_begin and allowed.max() <= tk.timestamp_begin + 50
    # after <|0.00|> text: timestamps below the last one are banned
    L, _ = ow.apply_rules(logits, [tk.timestamp_begin + 10, 500], tk, supp)
    assert np.all(~np.isfinite(L[tk.timestamp_begin:tk.timestamp_begin + 11]))
    # after a pair of timestamps: no timestamp may follow
    L, _ = ow.apply_rules(logits, [tk.timestamp_begin, 500, tk.timestamp_begin + 3, tk.timestamp_begin + 3],
                          tk, supp)
    assert np.all(~np.isfinite(L[tk.timestamp_begin:]))
    # single timestamp after text: only timestamps or eot
    L, _ = ow.apply_rules(logits, [tk.timestamp_begin, 500, tk.timestamp_begin + 7], tk, supp)
    assert np.all(~np.isfinite(L[:tk.eot]))
    for s in supp:
        assert not np.isfinite(L[s])


def test_segments_and_transcript():
    tk = tkz.WhisperTokenizer()
    tb = tk.timestamp_begin
    words = tk.encode_text(" hello world")
    seq = [tb] + words + [tb + 50, tb + 50] + tk.encode_text(" again") + [tb + 90, tk.eot]
    segs = tk.segments(seq)
    assert [s[2] for s in segs] == [" hello world", " again"]
    assert tk.transcript(seq) == "hello world again"
    assert tk.transcript([tk.eot]) == ""


def test_transcript_fast_path_matches_segments():
    """The numpy transcript of the table vocabulary equals ' '.join(segment texts)."""
    from janus_amd.tokenizer import load_tokenizer
    tk = load_tokenizer()
    rng = np.random.default_rng(7)
    tb = tk.timestamp_begin
    rows = [rng.integers(0, 51864, size=447), rng.integers(tb - 3, 51864, size=300),
            np.concatenate([rng.integers(0, 1000, size=40), [tk.eot], rng.integers(0, 1000, size=9)]),
            [], [tb], [tb, tb + 3], [5, tb + 1], [tb, 7, tb + 2, tb + 5, 9, 10], [-1, 5]]
    for r in rows:
        ref = " ".join(t.strip() for (_, _, t) in tk.segments(r)).strip()
        assert tk.transcript(r) == ref


def _hf_rules(tk, prompt, sampled, logits):
    """transformers' SuppressTokensAtBegin (blank + eot at the first sampled step),
    SuppressTokens and WhisperTimeStampLogitsProcessor (max_initial_timestamp_index 50 =
    1.0 s), composed in faster-whisper / CTranslate2's order."""
    from types import SimpleNamespace

    from transformers.generation.logits_process import (SuppressTokensAtBeginLogitsProcessor,
                                                        SuppressTokensLogitsProcessor,
                                                        WhisperTimeStampLogitsProcessor)
    cfg = SimpleNamespace(no_timestamps_token_id=tk.no_timestamps, eos_token_id=tk.eot,
                          bos_token_id=tk.eot, max_initial_timestamp_index=50)
    begin = len(prompt)
    ids = torch.tensor([list(prompt) + list(sampled)], dtype=torch.long)
    s = torch.tensor(np.asarray(logits, np.float32))[None]
    s = SuppressTokensAtBeginLogitsProcessor([tk.blank, tk.eot], begin)(ids, s)
    s = SuppressTokensLogitsProcessor(tk.suppress_tokens())(ids, s)
    s = WhisperTimeStampLogitsProcessor(cfg, begin, _detect_timestamp_from_logprob=True)(ids, s)
    return s[0].numpy()


def test_decoder_rules_match_transformers():
    """the oracle's restated OpenAI rules (apply_rules: SuppressBlank,
    SuppressTokens, ApplyTimestampRules with max_initial_timestamp 1.0 s) against the
    third-party transformers processors on seeded logits and token histories — the same
    -inf masks, the same surviving logits and the same argmax (the greedy choice)."""
    tk = tkz.WhisperTokenizer()
    V, tb = tkz.N_VOCAB_EN, tk.timestamp_begin
    rng = np.random.default_rng(42)
    prompt = list(tk.sot_sequence)
    hist = [[], [tb + 10, 500], [tb, 500, tb + 3, tb + 3], [tb, 500, tb + 7], [tb], [tb, tb],
            [tb + 2, 11, 12, tb + 9, tb + 9, 13], [500, 501], [tb, 400, tb + 40, tb + 40, 99, tb + 60]]
    for _ in range(40):
        n = int(rng.integers(1, 12))
        hist.append([int(tb + rng.integers(0, 1500)) if rng.random() < 0.35 else int(rng.integers(0, tk.eot))
                     for _ in range(n)])
    checked = ts_forced = 0
    for h in hist:
        for bias in (0.0, 6.0, -6.0):            # push the timestamp-mass rule both ways
            logits = rng.standard_normal(V).astype(np.float32)
            logits[tb:] += bias
            L, lp = ow.apply_rules(logits.astype(np.float64), h, tk, tk.suppress_tokens())
            ref = _hf_rules(tk, prompt, h, logits)
            assert np.array_equal(np.isfinite(L), np.isfinite(ref)), (h, bias)
            fin = np.isfinite(L)
            assert np.array_equal(L[fin].astype(np.float32), ref[fin]), (h, bias)
            assert int(np.argmax(L)) == int(np.argmax(ref)), (h, bias)
            ref_lp = torch.log_softmax(torch.tensor(ref, dtype=torch.float64), -1).numpy()
            assert np.allclose(lp[fin], ref_lp[fin], rtol=0, atol=1e-9)
            ts_forced += int(not fin[:tb].any() and len(h) > 0)
            checked += 1
    assert checked == 3 * len(hist) and ts_forced > 0

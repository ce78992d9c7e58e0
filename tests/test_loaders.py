"""Real-checkpoint paths on CPU: a Hugging Face-named Whisper
``model.safetensors`` and ``tokenizer.json`` under JANUS_WHISPER_DIR, a fish-speech-named
vocoder ``model.safetensors`` under JANUS_VOCODER_DIR. Synthetic tensors of the real
names and shapes stand in for the (unreachable) published files."""
import json

import numpy as np
import pytest

from janus_amd import tokenizer as tkz
from janus_amd.whisper import CONFIGS, FP32_MATRICES, WhisperConfig, load_weights, synthetic_weights

TINY = WhisperConfig("t", d_model=64, n_heads=1, enc_layers=1, dec_layers=1)


def _write_hf_checkpoint(path, W, dtype=np.float16, tie=True, prefix="model."):
    from safetensors.numpy import save_file
    sd = {prefix + k: v.astype(dtype) for k, v in W.items()}
    if tie:
        sd["proj_out.weight"] = W["decoder.embed_tokens.weight"].astype(dtype)
    save_file(sd, str(path / "model.safetensors"))


@pytest.mark.parametrize("dtype", [np.float16, np.float32])
def test_whisper_safetensors_names_and_dtype(tmp_path, monkeypatch, dtype):
    W = synthetic_weights(TINY, seed=2)
    _write_hf_checkpoint(tmp_path, W, dtype)
    monkeypatch.setenv("JANUS_WHISPER_DIR", str(tmp_path))
    got = load_weights(TINY)
    assert set(got) == set(W)                 # "model." stripped, tied proj_out dropped
    for k, v in got.items():
        assert v.dtype == np.float32 and v.shape == W[k].shape, k
        ref = W[k].astype(dtype).astype(np.float32)
        if v.ndim >= 2 and k not in FP32_MATRICES:   # fp16, as the engine holds them
            ref = ref.astype(np.float16).astype(np.float32)
        assert np.array_equal(v, ref), k


def test_whisper_untied_proj_out_rejected(tmp_path, monkeypatch):
    from safetensors.numpy import save_file
    W = synthetic_weights(TINY, seed=2)
    _write_hf_checkpoint(tmp_path, W, tie=False)
    sd = {"model." + k: v for k, v in W.items()}
    sd["proj_out.weight"] = W["decoder.embed_tokens.weight"] + 1
    save_file(sd, str(tmp_path / "model.safetensors"))
    monkeypatch.setenv("JANUS_WHISPER_DIR", str(tmp_path))
    with pytest.raises(ValueError, match="tied"):
        load_weights(TINY)


def test_whisper_wrong_model_rejected(tmp_path, monkeypatch):
    _write_hf_checkpoint(tmp_path, synthetic_weights(TINY, seed=2))
    monkeypatch.setenv("JANUS_WHISPER_DIR", str(tmp_path))
    with pytest.raises(ValueError, match="does not match"):
        load_weights(CONFIGS["base.en"])


def _byte_level_chars():
    order = tkz.bytes_to_unicode_order()
    printable = set(order[:188])
    chars, n = {}, 0
    for b in range(256):
        if b in printable:
            chars[b] = chr(b)
        else:
            chars[b] = chr(256 + n)
            n += 1
    return [chars[b] for b in order]


def _write_tokenizer_json(path):
    """A byte-level BPE with the *.en special-token layout (GPT-2 byte symbols at 0..255,
    a few merges, filler up to 50255, then the Whisper specials and timestamps)."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from tokenizers import AddedToken
    syms = _byte_level_chars()
    vocab = {s: i for i, s in enumerate(syms)}
    merges = [("Ġ", "h"), ("Ġh", "e"), ("l", "l"), ("Ġhe", "ll"), ("Ġhell", "o"), ("Ġ", "w")]
    for a, b in merges:
        vocab[a + b] = len(vocab)
    while len(vocab) < tkz.EOT:
        vocab[f"<filler{len(vocab)}>"] = len(vocab)
    tok = Tokenizer(models.BPE(vocab=vocab, merges=merges))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    specials = ["<|endoftext|>", "<|startoftranscript|>"] + [f"<|lang{i}|>" for i in range(99)] + \
        ["<|translate|>", "<|transcribe|>", "<|startoflm|>", "<|startofprev|>", "<|nocaptions|>",
         "<|notimestamps|>"] + [f"<|{i * 0.02:.2f}|>" for i in range(1501)]
    tok.add_special_tokens([AddedToken(s, special=True) for s in specials])
    assert tok.get_vocab_size() == tkz.N_VOCAB_EN
    tok.save(str(path / "tokenizer.json"))


def test_hf_tokenizer_special_ids_and_suppress_set(tmp_path, monkeypatch):
    _write_tokenizer_json(tmp_path)
    monkeypatch.setenv("JANUS_WHISPER_DIR", str(tmp_path))
    tk = tkz.load_tokenizer()
    assert tk._hf is not None
    assert (tk.eot, tk.sot, tk.timestamp_begin, tk.no_timestamps) == (50256, 50257, 50363, 50362)
    ids = tk.encode_text(" hello world")
    assert tk.decode(ids) == " hello world" and ids[0] == tk._hf.token_to_id("Ġhello")
    # non-speech symbols that are single tokens, plus " -" / " '" (openai rule)
    nst = set(tk.non_speech_tokens())
    for sym in ('"', "#", "(", "*", "@", "~"):
        assert tk.encode_text(sym)[0] in nst
    assert tk.encode_text(" -")[0] in nst and tk.encode_text(" '")[0] in nst
    supp = set(tk.suppress_tokens())
    assert {tkz.TRANSCRIBE, tkz.TRANSLATE, tkz.SOT, tkz.SOT_PREV, tkz.SOT_LM} <= supp
    assert tkz.EOT not in supp and tkz.NO_TIMESTAMPS not in supp
    tb = tk.timestamp_begin
    seq = [tb] + ids + [tb + 50, tb + 50] + tk.encode_text(" hello") + [tb + 90, tk.eot]
    assert [s[2] for s in tk.segments(seq)] == [" hello world", " hello"]
    assert tk.transcript(seq) == "hello world hello"


def test_hf_tokenizer_layout_checked(tmp_path, monkeypatch):
    from tokenizers import Tokenizer, models
    tok = Tokenizer(models.BPE(vocab={"a": 0, "<|endoftext|>": 1}, merges=[]))
    tok.save(str(tmp_path / "tokenizer.json"))
    monkeypatch.setenv("JANUS_WHISPER_DIR", str(tmp_path))
    with pytest.raises(ValueError, match="endoftext"):
        tkz.load_tokenizer()


def test_vocoder_safetensors(tmp_path, monkeypatch):
    from safetensors.numpy import save_file
    from janus_amd.vocoder import FireflyConfig, load_weights as vload, synthetic_weights as vsyn
    cfg = FireflyConfig()
    W = vsyn(cfg, seed=3)
    save_file({k: v.astype(np.float16) for k, v in W.items()}, str(tmp_path / "model.safetensors"))
    monkeypatch.setenv("JANUS_VOCODER_DIR", str(tmp_path))
    got = vload(cfg)
    assert set(got) == set(W)
    for k in ("conv_pre.weight", "ups.0.weight", "resblocks.4.blocks.2.convs2.2.bias", "frontend.speaker_proj"):
        assert got[k].dtype == np.float32 and np.array_equal(got[k], W[k].astype(np.float16).astype(np.float32))
    json.dumps({k: list(v.shape) for k, v in got.items()})

"""GPU parity of the decode path: front end exact to fp16, Firefly-GAN forward within
1e-3 RMS of the fp32 oracle (north_star tolerance) both before tanh (conv_post output)
and after it, up to the 30 s / 2584-frame length of configs 2 and 4; the voice
(speaker) embedding; the drop-in Synthesizer / FishAudio contract on the GPU."""
import numpy as np
import pytest
import torch

from janus_amd.common.protocol import JanusMode, JanusPacket
from janus_amd.vocoder import FireflyConfig, VocoderEngine, emotion_id, synthetic_weights
from oracle import synth as osy
from oracle import vocoder as ov

pytestmark = pytest.mark.gpu
CFG = FireflyConfig()


@pytest.fixture(scope="module")
def voc(gpu):
    W = synthetic_weights(CFG, seed=2)
    return VocoderEngine(CFG, W), W


def test_frontend_exact(voc):
    eng, W = voc
    prompts = [b"(joyful) hello world", b"", b"(auto) x" * 9]
    emos = [emotion_id("joyful"), 0, emotion_id("auto")]
    lat = eng.frontend(prompts, emos, 37)
    ref = ov.frontend(prompts, emos, 37, W).half()
    assert torch.equal(lat.cpu(), ref)


@pytest.mark.parametrize("frames,B", [(4, 2), (23, 2), (2584, 1)])
def test_generator_rms(voc, frames, B):
    """2584 frames = 30 s @ 44.1 kHz (configs 2 and 4). The post-tanh waveform saturates
    (|y| near 1 compresses upstream error), so the conv_post output is compared too,
    relative to its own RMS."""
    eng, W = voc
    prompts = [b"(joyful) hello world", b"(sad) the quick brown fox"][:B]
    emos = [emotion_id("joyful"), emotion_id("sad")][:B]
    lat = eng.frontend(prompts, emos, frames)
    wav, pcm, pre = eng.forward(lat, want_pre_tanh=True)
    torch.cuda.synchronize()
    ref, ref_pre = ov.generator(lat.float().cpu(), W, CFG, pre_tanh=True)
    got = wav.cpu()
    assert got.shape == ref.shape == (B, frames * 512)
    rms = float(((got - ref) ** 2).mean().sqrt())
    assert rms <= 1e-3, rms
    pre = pre.cpu()
    assert torch.equal(torch.tanh(pre), got) or float((torch.tanh(pre) - got).abs().max()) < 1e-6
    pre_rel = float(((pre - ref_pre) ** 2).mean().sqrt() / (ref_pre ** 2).mean().sqrt())
    print(f"frames {frames}: post-tanh rms {rms:.2e}, pre-tanh rel rms {pre_rel:.2e}")
    assert pre_rel <= 2e-3, pre_rel
    assert np.array_equal(pcm.cpu().numpy(), ov.pcm16(got.numpy()))


def test_family_stats(voc):
    """Per-family roofline accounting (janus_vocoder_family_stats): one forward = 6 conv
    launches (conv_pre + 5 upsamplers) and 9 fused units per channel width; the families
    sum to the whole-family totals, and the algorithmic FLOPs are the closed forms."""
    eng, W = voc
    B, frames = 2, 8
    lat = eng.frontend([b"(joyful) a", b"(sad) b"], [0, 1], frames)
    eng.set_timing(True)
    eng.forward(lat)
    torch.cuda.synchronize()
    fams = eng.family_stats(reset=False)
    flops, ms, launches = eng.conv_stats(reset=True)
    eng.set_timing(False)
    assert sorted(fams) == [0, 16, 32, 64, 128, 256]
    assert fams[0]["launches"] == 6
    assert all(fams[c]["launches"] == 9 for c in (16, 32, 64, 128, 256))
    assert sum(v["launches"] for v in fams.values()) == launches
    assert abs(sum(v["flops"] for v in fams.values()) - flops) <= 1e-6 * flops
    assert abs(sum(v["ms"] for v in fams.values()) - ms) <= 1e-6 * max(ms, 1e-9)
    # fused unit at width C, time rows T: both convs, 2*C*C*k FLOP per row each
    T = {256: frames * 8, 128: frames * 64, 64: frames * 128, 32: frames * 256, 16: frames * 512}
    for C, t in T.items():
        want = sum(2 * 2 * C * C * k * B * t for k in CFG.rb_kernels for _ in CFG.rb_dilations)
        assert abs(fams[C]["flops"] - want) <= 1e-9 * want, (C, fams[C]["flops"], want)
        assert fams[C]["bytes"] >= 2 * 2 * B * t * C * 9  # read + write of every unit
        assert fams[C]["ms"] > 0


def test_speaker_embedding(voc):
    """Voice vector of reference recordings (janus_vocoder_speaker) vs the oracle, and the
    frontend with it exact to fp16."""
    from janus_amd.workload import synth_speech
    eng, W = voc
    clips = [synth_speech(77, 3.0)[::3], synth_speech(78, 0.4)[::3], synth_speech(79, 31.0)[::3]]
    spk = eng.speaker_embedding(clips)
    torch.cuda.synchronize()
    ref = ov.speaker(clips, W)
    got = spk.cpu().numpy()
    assert np.abs(got - ref).max() < 1e-4 * max(1.0, np.abs(ref).max()), np.abs(got - ref).max()
    assert np.abs(got[0] - got[1]).max() > 1e-3          # different voices differ
    prompts = [b"(joyful) hi", b"(sad) bye", b"x"]
    emos = [1, 5, 0]
    lat = eng.frontend(prompts, emos, 11, spk)
    assert torch.equal(lat.cpu(), ov.frontend(prompts, emos, 11, W, got).half())


def test_synthesizer_dropin(gpu, monkeypatch):
    from janus_amd.services.synthesizer import Synthesizer
    s = Synthesizer(api_key="unused")
    out = s.synthesize(JanusPacket("Hello world", JanusMode.SEMANTIC_VOICE,
                                   {'energy': 'Loud', 'pitch': 'High'}, "Auto", 1.0))
    assert out[:4] == b'RIFF' and out[8:12] == b'WAVE' and len(out) > 44
    n = (len(out) - 44) // 2
    assert n == len(b"(excited) Hello world") * 6 * 512
    assert s.synthesize(JanusPacket("SOS", JanusMode.MORSE_CODE, {})) == osy.morse("SOS")
    t = s.synthesize(JanusPacket("hi", JanusMode.TEXT_ONLY, {}, "joyful"))
    assert t[:4] == b'RIFF'
    # fallback chain (synthesizer.py:205-207, :253-255)
    monkeypatch.setattr(s.client.tts, "convert", lambda **kw: (_ for _ in ()).throw(RuntimeError("boom")))
    assert s.synthesize(JanusPacket("x", JanusMode.SEMANTIC_VOICE, {})) == b''
    with pytest.raises(ValueError):
        s.synthesize(JanusPacket("x", 7, {}))


def test_fishaudio_convert_matches_oracle(voc, tmp_path):
    """client.tts.convert renders the prompt with the voice the SDK arguments name:
    no voice, a stock reference_id, or a ReferenceAudio recording (the reference's
    hot-reloaded voice-cloning file) — each bit-identical to the oracle front end run
    through the GPU generator, and the recording changes the audio."""
    from janus_amd.common.wavio import read_wav_16k
    from janus_amd.services.synthesizer import FishAudio, ReferenceAudio
    from janus_amd.vocoder import DEFAULT_REFERENCE_ID, FRAMES_PER_BYTE, voice_id, wav_bytes
    from janus_amd.workload import synth_speech
    eng, W = voc
    client = FishAudio(api_key="k", engine=eng)
    text = "(joyful) hello there"
    pb = text.encode()
    frames = len(pb) * FRAMES_PER_BYTE
    rec = wav_bytes(np.clip(np.rint(synth_speech(90, 2.0) * 32767), -32768, 32767).astype(np.int16), 48000)
    clip = read_wav_16k(rec)
    voices = {
        "none": (dict(references=None), None),
        "id": (dict(reference_id=DEFAULT_REFERENCE_ID),
               np.asarray(W["frontend.voice_embed"], np.float32)[voice_id(DEFAULT_REFERENCE_ID)][None]),
        "rec": (dict(references=[ReferenceAudio(audio=rec, text="")]),
                eng.speaker_embedding([clip]).cpu().numpy()),
    }
    outs = {}
    for k, (kw, spk) in voices.items():
        out = client.tts.convert(text=text, format="wav", latency="balanced", **kw)
        lat = ov.frontend([pb], [emotion_id("joyful")], frames, W, spk).half().to(eng.device)
        _, pcm = eng.forward(lat)
        assert out == wav_bytes(pcm[0].cpu().numpy()), k
        outs[k] = out
    assert outs["none"] != outs["rec"] and outs["id"] != outs["rec"]


def test_reference_recording_formats_and_fallback(gpu, tmp_path):
    """the hot-reloaded voice-cloning file. A 24-bit WAV is decoded and
    embedded ONCE for any number of packets (cached on the file content); a file this host
    cannot decode (an MP3) no longer silences every packet — it is rendered without the
    voice term, as references=None would be."""
    import struct

    from janus_amd.services.synthesizer import Synthesizer
    from janus_amd.workload import synth_speech
    x = np.clip(synth_speech(91, 1.5) * 8388607, -8388608, 8388607).astype(np.int64)
    pcm24 = b"".join(int(v).to_bytes(3, "little", signed=True) for v in x)
    fmt = struct.pack("<HHIIHH", 1, 1, 48000, 48000 * 3, 3, 24)
    body = b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(pcm24)) + pcm24
    wav24 = tmp_path / "ref24.wav"
    wav24.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)
    s = Synthesizer(api_key="unused", reference_audio_path=str(wav24))
    tts = s.client.tts
    calls = []
    orig = tts.engine.speaker_embedding
    tts.engine.speaker_embedding = lambda clips: (calls.append(len(clips)), orig(clips))[1]
    pk = [JanusPacket("hello there", JanusMode.SEMANTIC_VOICE, {'energy': 'Normal', 'pitch': 'High'}),
          JanusPacket("again", JanusMode.TEXT_ONLY, {}, "joyful")]
    outs = [s.synthesize(p) for p in pk]
    assert all(o[:4] == b"RIFF" and len(o) > 44 for o in outs)
    assert calls == [1]
    no_voice = tts.convert(text="(joyful) again", format="wav", latency="balanced", references=None)
    assert outs[1] != no_voice                      # the recording shaped the voice
    mp3 = tmp_path / "ref.mp3"
    mp3.write_bytes(b"ID3\x04\x00\x00\x00\x00\x00\x21" + bytes(range(256)) * 8)
    s2 = Synthesizer(api_key="unused", reference_audio_path=str(mp3))
    out = s2.synthesize(pk[1])
    assert out == s2.client.tts.convert(text="(joyful) again", format="wav", latency="balanced",
                                        references=None)
    assert s2.synthesize(pk[0])[:4] == b"RIFF"

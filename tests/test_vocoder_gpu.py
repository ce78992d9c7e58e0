"""GPU parity of the decode path: front end exact to fp16, Firefly-GAN forward within
1e-3 RMS of the fp32 oracle (north_star tolerance), drop-in Synthesizer contract."""
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


@pytest.mark.parametrize("frames", [4, 23])
def test_generator_rms(voc, frames):
    eng, W = voc
    prompts = [b"(joyful) hello world", b"(sad) the quick brown fox"]
    emos = [emotion_id("joyful"), emotion_id("sad")]
    lat = eng.frontend(prompts, emos, frames)
    wav, pcm = eng.forward(lat)
    torch.cuda.synchronize()
    ref = ov.generator(lat.float().cpu(), W, CFG)
    got = wav.cpu()
    assert got.shape == ref.shape == (2, frames * 512)
    rms = float(((got - ref) ** 2).mean().sqrt())
    assert rms <= 1e-3, rms
    assert np.array_equal(pcm.cpu().numpy(), ov.pcm16(got.numpy()))


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
    monkeypatch.setattr(s, "_vocode", lambda *a: (_ for _ in ()).throw(RuntimeError("boom")))
    assert s.synthesize(JanusPacket("x", JanusMode.SEMANTIC_VOICE, {})) == b''
    with pytest.raises(ValueError):
        s.synthesize(JanusPacket("x", 7, {}))

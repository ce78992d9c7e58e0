"""Print the vocoder GPU-vs-oracle waveform RMS (margin to the 1e-3 north_star bound)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from janus_amd.vocoder import FireflyConfig, VocoderEngine, emotion_id, synthetic_weights
from oracle import vocoder as ov
CFG = FireflyConfig()
W = synthetic_weights(CFG, seed=2)
eng = VocoderEngine(CFG, W)
for frames in (4, 23):
    lat = eng.frontend([b"(joyful) hello world", b"(sad) the quick brown fox"],
                       [emotion_id("joyful"), emotion_id("sad")], frames)
    wav, pcm = eng.forward(lat)
    torch.cuda.synchronize()
    ref = ov.generator(lat.float().cpu(), W, CFG)
    rms = float(((wav.cpu() - ref) ** 2).mean().sqrt())
    print(f"frames {frames}: rms {rms:.3e}  ref rms {float((ref**2).mean().sqrt()):.3e}", flush=True)

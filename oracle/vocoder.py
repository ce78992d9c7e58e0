"""ORACLE — test infrastructure only (see oracle/__init__.py).

fp32 torch CPU restatement of the decode path that replaces the reference's cloud TTS
(synthesizer.py:133-207): the build-defined prompt front end (janus_amd/vocoder.py
docstring) and the fish-speech Firefly-GAN HiFiGANGenerator forward (conv_pre ->
[SiLU, ConvTranspose1d, ParallelBlock(ResBlock1 x 3)] x 5 -> SiLU -> conv_post ->
tanh), written from the public architecture. No reference implementation exists in
/root/reference (its TTS is remote). The generator's topology is pinned externally:
with its activation switched to leaky ReLU it equals transformers' HiFi-GAN V1
``SpeechT5HifiGan`` (transformers 5.15) on the same weights to 1e-5
(tests/test_oracle_vocoder.py); only the SiLU choice and the front end stay
build-defined.
"""
import numpy as np
import torch
import torch.nn.functional as F


def _t(W, name):
    return torch.from_numpy(np.asarray(W[name], np.float32))


def frontend(prompts_bytes, emotion_ids, frames, W, speaker=None):
    """latents [B][frames][latent] fp32; speaker: optional [B][latent] voice rows
    (janus_vocoder_frontend_ex adds them after text + emotion, in that order)."""
    te, ee = _t(W, "frontend.text_embed"), _t(W, "frontend.emotion_embed")
    out = []
    for b, (pb, e) in enumerate(zip(prompts_bytes, emotion_ids)):
        n = len(pb)
        if n:
            idx = (np.arange(frames, dtype=np.int64) * n) // frames
            tx = te[torch.from_numpy(np.frombuffer(pb, np.uint8)[idx].astype(np.int64))]
        else:
            tx = torch.zeros(frames, te.shape[1])
        row = tx + ee[e]
        if speaker is not None:
            row = row + torch.as_tensor(np.asarray(speaker[b], np.float32))
        out.append(row)
    return torch.stack(out)


def speaker(clips16k, W):
    """Voice vectors [B][latent] (float64 -> f32) of 16 kHz clips: the normalised Whisper
    log-mel (oracle.whisper.logmel, decim 1) averaged over the clip's frames
    min(3000, max(1, ceil(n / 160))), projected by frontend.speaker_proj / _bias
    (janus_amd/csrc/vocoder_edge.hip speaker_kernel)."""
    from janus_amd.whisper import mel_filters
    from oracle.whisper import logmel
    P = np.asarray(W["frontend.speaker_proj"], np.float64)
    bias = np.asarray(W["frontend.speaker_bias"], np.float64)
    out = []
    for x in clips16k:
        x = np.asarray(x, np.float32)[:480000]
        nf = min(3000, max(1, -(-len(x) // 160)))
        m = logmel(x, 1, mel_filters(), zero_pad=False).astype(np.float64)[:nf].mean(0)
        out.append(bias + P @ m)
    return np.stack(out).astype(np.float32)


@torch.no_grad()
def generator(lat, W, cfg, pre_tanh=False, act=F.silu, post_act=None):
    """lat [B][F][latent] -> wav [B][F*prod(rates)] (fp32); with pre_tanh also the
    conv_post output before tanh.

    ``act`` is the activation ahead of every upsampler and every ResBlock1 conv,
    ``post_act`` the one ahead of conv_post (default: ``act``). Firefly-GAN (the build)
    uses SiLU throughout. With ``act = leaky_relu(0.1)`` and ``post_act = leaky_relu(0.01)``
    the same function is HiFi-GAN V1, which pins this restatement's topology (padding,
    dilation, transposed-conv upsampling, ParallelBlock mean, conv_post, tanh) against
    transformers' ``SpeechT5HifiGan`` on shared weights (tests/test_oracle_vocoder.py)."""
    post_act = act if post_act is None else post_act
    x = torch.as_tensor(lat, dtype=torch.float32).transpose(1, 2)
    x = F.conv1d(x, _t(W, "conv_pre.weight"), _t(W, "conv_pre.bias"), padding=(cfg.pre_kernel - 1) // 2)
    for i, u in enumerate(cfg.up_rates):
        x = act(x)
        x = F.conv_transpose1d(x, _t(W, f"ups.{i}.weight"), _t(W, f"ups.{i}.bias"), stride=u,
                               padding=u // 2)
        outs = []
        for j, k in enumerate(cfg.rb_kernels):
            y = x
            p = f"resblocks.{i}.blocks.{j}"
            for m, d in enumerate(cfg.rb_dilations):
                xt = act(y)
                xt = F.conv1d(xt, _t(W, f"{p}.convs1.{m}.weight"), _t(W, f"{p}.convs1.{m}.bias"),
                              padding=d * (k - 1) // 2, dilation=d)
                xt = act(xt)
                xt = F.conv1d(xt, _t(W, f"{p}.convs2.{m}.weight"), _t(W, f"{p}.convs2.{m}.bias"),
                              padding=(k - 1) // 2)
                y = xt + y
            outs.append(y)
        x = torch.stack(outs, 0).mean(0)
    x = post_act(x)
    x = F.conv1d(x, _t(W, "conv_post.weight"), _t(W, "conv_post.bias"), padding=(cfg.post_kernel - 1) // 2)
    return (torch.tanh(x)[:, 0], x[:, 0]) if pre_tanh else torch.tanh(x)[:, 0]


def pcm16(wav):
    return np.clip(np.rint(np.asarray(wav, np.float32) * 32767.0), -32768, 32767).astype(np.int16)

"""Pins the vocoder oracle (oracle/vocoder.py generator) against an external
implementation: transformers' HiFi-GAN V1 generator ``SpeechT5HifiGan`` (transformers
5.15, importable in this image). Firefly-GAN's generator is HiFi-GAN V1 with SiLU in
place of leaky ReLU and 13-tap conv_pre / conv_post; SpeechT5's uses leaky ReLU(0.1)
ahead of every upsampler / ResBlock1 conv, leaky ReLU(0.01) ahead of conv_post and
7-tap conv_pre / conv_post. With the oracle's activations set to those and its pre/post
kernels to 7, both must compute the same function on the same weights: this pins the
transposed-conv upsampling (stride u, kernel 2u, padding u // 2), the ResBlock1 dilation
padding d(k-1)/2, the conv2 padding, the residual adds, the ParallelBlock mean over the
three kernels, conv_post and the tanh. Only the SiLU choice (and the build-defined front
end) remain unpinned. The reference's own TTS is remote
(/root/reference/backend/services/synthesizer.py:191-203)."""
import dataclasses

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from janus_amd.vocoder import FireflyConfig
from oracle import vocoder as ov

transformers = pytest.importorskip("transformers")


def _hf_and_weights(latent, channels, seed):
    from transformers import SpeechT5HifiGan, SpeechT5HifiGanConfig
    torch.manual_seed(seed)
    hcfg = SpeechT5HifiGanConfig(
        model_in_dim=latent, sampling_rate=44100, upsample_initial_channel=channels,
        upsample_rates=[8, 8, 2, 2, 2], upsample_kernel_sizes=[16, 16, 4, 4, 4],
        resblock_kernel_sizes=[3, 7, 11], resblock_dilation_sizes=[[1, 3, 5]] * 3,
        initializer_range=0.01, leaky_relu_slope=0.1, normalize_before=False)
    m = SpeechT5HifiGan(hcfg).eval()
    # non-trivial weights and biases everywhere (post_init may zero the biases)
    with torch.no_grad():
        for name, p in m.named_parameters():
            fan = p[0].numel() if p.dim() > 1 else 1
            p.copy_(torch.randn_like(p) * (0.6 / np.sqrt(fan) if p.dim() > 1 else 0.05))
    sd = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    W = {"conv_pre.weight": sd["conv_pre.weight"], "conv_pre.bias": sd["conv_pre.bias"],
         "conv_post.weight": sd["conv_post.weight"], "conv_post.bias": sd["conv_post.bias"]}
    nk = 3
    for i in range(5):
        W[f"ups.{i}.weight"] = sd[f"upsampler.{i}.weight"]
        W[f"ups.{i}.bias"] = sd[f"upsampler.{i}.bias"]
        for j in range(nk):
            for c in ("convs1", "convs2"):
                for d in range(3):
                    for t in ("weight", "bias"):
                        W[f"resblocks.{i}.blocks.{j}.{c}.{d}.{t}"] = \
                            sd[f"resblocks.{i * nk + j}.{c}.{d}.{t}"]
    return m, W


@pytest.mark.parametrize("latent,channels,frames,batch", [(16, 64, 5, 2), (32, 128, 9, 1)])
def test_generator_topology_matches_hifigan(latent, channels, frames, batch):
    m, W = _hf_and_weights(latent, channels, seed=latent + channels)
    cfg = dataclasses.replace(FireflyConfig(), latent_dim=latent, channels=channels,
                              pre_kernel=7, post_kernel=7)
    lat = torch.randn(batch, frames, latent, generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = m(lat)
    got, pre = ov.generator(lat, W, cfg, pre_tanh=True,
                            act=lambda x: F.leaky_relu(x, 0.1),
                            post_act=lambda x: F.leaky_relu(x, 0.01))
    assert got.shape == ref.shape == (batch, frames * 512)
    # the waveform is not saturated: tanh did not hide a topology difference
    assert 0.05 < float(pre.abs().mean()) < 3.0
    assert torch.allclose(got, ref, atol=1e-5, rtol=1e-5), float((got - ref).abs().max())
    # the comparison is sensitive: the one activation slope SpeechT5 changes (0.01 ahead
    # of conv_post) moves the output two orders of magnitude past the tolerance (an
    # upsampler padding off by one moves it by ~2e-2)
    bad = ov.generator(lat, W, cfg, act=lambda x: F.leaky_relu(x, 0.1),
                       post_act=lambda x: F.leaky_relu(x, 0.1))
    assert float((bad - ref).abs().max()) > 1e-4


def test_generator_default_activation_is_silu():
    """The build's generator (SiLU everywhere) is the act=F.silu instance of the pinned
    function: same weights, the default call and the explicit one agree bit for bit."""
    _, W = _hf_and_weights(16, 64, seed=11)
    cfg = dataclasses.replace(FireflyConfig(), latent_dim=16, channels=64, pre_kernel=7,
                              post_kernel=7)
    lat = torch.randn(1, 4, 16, generator=torch.Generator().manual_seed(5))
    a = ov.generator(lat, W, cfg)
    b = ov.generator(lat, W, cfg, act=F.silu, post_act=F.silu)
    assert torch.equal(a, b)

"""ORACLE — test infrastructure only (see oracle/__init__.py).

fp32 torch restatement of the silero-vad v5 16 kHz model as the reference calls it
(backend/services/vad.py:52-77: model(chunk[::3], 16000) per capture chunk, the model
object keeping its 64-sample context and LSTM state across calls, never reset):
  x = cat(context, chunk) (576); STFT = conv1d(reflect_pad(x, (0, 64)), basis, stride 128)
  -> magnitude of (real, imag) halves; encoder 4 x (Conv1d k3 p1 + ReLU), strides
  1, 2, 2, 1; LSTMCell(128, 128); ReLU -> Conv1d(128, 1, 1) -> sigmoid.
silero-vad itself is a remote torch.hub download (unavailable here): the graph follows
its published v5 source; "parity unpinned" against the released weights.
"""
import numpy as np
import torch
import torch.nn.functional as F


def _t(W, n):
    return torch.from_numpy(np.asarray(W[n], np.float32))


class OracleSilero:
    def __init__(self, W):
        self.W = W
        self.context = torch.zeros(1, 64)
        self.h = torch.zeros(1, 128)
        self.c = torch.zeros(1, 128)

    @torch.no_grad()
    def __call__(self, chunk512) -> float:
        W = self.W
        x = torch.cat([self.context, torch.as_tensor(np.asarray(chunk512, np.float32))[None]], 1)
        self.context = x[:, -64:]
        y = F.pad(x[:, None], (0, 64), mode="reflect")
        basis = _t(W, "_model.stft.forward_basis_buffer").reshape(258, 1, 256)
        ft = F.conv1d(y, basis, stride=128)
        mag = torch.sqrt(ft[:, :129] ** 2 + ft[:, 129:] ** 2)
        e = mag
        for i, st in enumerate((1, 2, 2, 1)):
            p = f"_model.encoder.{i}.reparam_conv"
            e = F.relu(F.conv1d(e, _t(W, p + ".weight"), _t(W, p + ".bias"), stride=st, padding=1))
        z = e[:, :, 0]
        gates = (z @ _t(W, "_model.decoder.rnn.weight_ih").T + _t(W, "_model.decoder.rnn.bias_ih") +
                 self.h @ _t(W, "_model.decoder.rnn.weight_hh").T + _t(W, "_model.decoder.rnn.bias_hh"))
        i, f, g, o = gates.chunk(4, 1)
        self.c = torch.sigmoid(f) * self.c + torch.sigmoid(i) * torch.tanh(g)
        self.h = torch.sigmoid(o) * torch.tanh(self.c)
        out = F.conv1d(F.relu(self.h)[:, :, None], _t(W, "_model.decoder.decoder.2.weight"),
                       _t(W, "_model.decoder.decoder.2.bias"))
        return float(torch.sigmoid(out).reshape(()))

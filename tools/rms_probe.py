"""GPU probe: janus_prosody_analyze rms vs numpy for a few lengths (debug aid)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from janus_amd.services.prosody import prosody_launch
dev = torch.device("cuda", 0)
for n in (100, 8192, 7616, 16384, 24000, 40000):
    x = (0.3 * np.sin(np.arange(n) * 0.05)).astype(np.float32)
    pcm = torch.from_numpy(np.concatenate([x, np.zeros(1, np.float32)])).to(dev)
    offs = torch.tensor([0, n], dtype=torch.int64, device=dev)
    r = prosody_launch(pcm, offs, [n], 48000, 512)
    torch.cuda.synchronize()
    g = float(r.rms.cpu()[0]); ref = float(np.sqrt(np.mean(x ** 2)))
    print(n, g, ref, (g / ref) ** 2 * n, flush=True)

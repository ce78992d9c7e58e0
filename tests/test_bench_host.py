"""Host-side measurement arithmetic of bench.py and tools/conv_avg.py (CPU): the decoder's
algorithmic bytes per position, the encoder's FLOPs, the decoder roofline object, and the
rocprof cross-check of the vocoder conv average."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def test_decoder_bytes_base_en(bench):
    from janus_amd.whisper import CONFIGS
    cfg = CONFIGS["base.en"]
    by = bench.decoder_bytes(cfg, 64, 447)
    d, L = 512, 6
    assert by["cross_attention"] == L * 64 * 1500 * d * 2                   # 98.3 MB per layer
    assert by["self_attention"] == L * 64 * (447 + 1) / 2 * d * 4           # K + V rows that exist
    assert by["layer_weights"] == L * (14 + 8) * d * d * 2                  # 69.2 MB
    assert by["vocab_projection"] == cfg.n_vocab * d * 2
    assert abs(sum(by.values()) / 1e6 - 888.3) < 0.5


def test_decoder_roofline_object(bench):
    from janus_amd.whisper import CONFIGS
    r = bench.decoder_roofline(CONFIGS["base.en"], 64, 447, 447 * 68, 278.66, 0.5)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["us_per_position"] - 623.4) < 0.1
    assert abs(r["achieved"] - 1424.9) < 0.5
    assert abs(r["frac_of_cu_share"] - 2 * r["frac"]) < 1e-3
    assert r["launches_per_position"] == 68.0
    assert bench.decoder_roofline(CONFIGS["base.en"], 64, 447, 0, None, 0.5) is None


def test_encoder_flops_base_en(bench):
    from janus_amd.whisper import CONFIGS
    fl = bench.encoder_flops(CONFIGS["base.en"], 1)
    assert abs(sum(fl.values()) / 1e9 - 87.3) < 0.2


def test_conv_avg_tool(tmp_path):
    """tools/conv_avg.py: encoder-stem convs and pack kernels excluded, the average of the
    rest compared with the line's HIP-event average."""
    csv = tmp_path / "k.csv"
    csv.write_text(
        "Name,Calls,TotalDurationNs,AverageNs,Percentage\n"
        '"void janus::resunit_wide_kernel<128, 2, 11, 5>(janus::ResUnitArgs, int, long long*)",2,8000000,4000000,1\n'
        '"void janus::conv_kernel<128, 128, 4, 4, 64, 0, 0>(janus::ConvArgs, int)",2,4000000,2000000,1\n'
        '"void janus::conv_kernel<128, 128, 4, 4, 64, 0, 2>(janus::ConvArgs, int)",9,9000000,1000000,1\n'
        "_ZN5janus24resunit_wide_pack_kernelEPKfPDF16_ii,5,5000,1000,1\n")
    line = tmp_path / "b.json"
    line.write_text(json.dumps({"roofline": {"flops_per_launch": 3e12, "launches": 4,
                                             "avg_launch_ms": 3.0, "frac": 0.4}}))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "conv_avg.py"), str(csv), str(line)],
                         check=True, capture_output=True, text=True).stdout
    r = json.loads(out)
    assert r["rocprof_launches"] == 4 and abs(r["rocprof_avg_launch_ms"] - 3.0) < 1e-9
    assert r["ratio_line_over_rocprof"] == 1.0


def test_serving_tuning_from_env():
    """ServingTuning.from_env: JANUS_<FIELD> overrides one field (bench.py / tools A/Bs);
    the pipeline itself reads no environment."""
    from janus_amd.pipeline import ServingTuning
    t = ServingTuning.from_env({})
    assert t == ServingTuning() and t.persistent == 2 and t.stagger_sets == 2 and t.voc_dec_utts == 0
    assert t.all_windows and t.batches_per_set() == 2 and t.calls() == 1
    assert ServingTuning(all_windows=False).calls() == 1 and ServingTuning(set_batches=1).calls() == 2
    t = ServingTuning.from_env({"JANUS_STAGGER_SETS": "3", "JANUS_YIN_DEC_UTTS": "5",
                                "JANUS_HOST_PREFETCH": "0", "JANUS_YIN_SIDE": "beside",
                                "JANUS_OTHER": "1", "JANUS_ALL_WINDOWS": "0"})
    assert (t.stagger_sets, t.yin_dec_utts, t.host_prefetch, t.yin_side) == (3, 5, False, "beside")
    assert not t.all_windows and t.calls() == 1
    src = open(os.path.join(os.path.dirname(__file__), "..", "janus_amd", "pipeline.py")).read()
    assert "os.environ.get(" not in src

"""BASELINE config 5 on one GPU (kept for the earlier rounds' scripts): the same run as
``bench.py --config 5`` (16 concurrent 48 kHz channels per GPU in real time as 320 ms
blocks, gated and segmented per channel, phrases encoded on a worker stream and rendered
by the receiver's vocoder), which is where the code lives now; this forwards its flags.

python tools/stream_bench.py [--streams 16] [--seconds 30] [--model base.en] [--max-length 448]
                             [--block-ms 320] [--async 1] [--duplex 1] [--fallback]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = ["--config", "5"]
    for a in sys.argv[1:]:
        argv.append("--stream-async" if a == "--async" else a)
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv
    import bench
    bench.main()


if __name__ == "__main__":
    main()

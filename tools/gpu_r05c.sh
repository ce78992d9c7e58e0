set -o pipefail
bash tools/gpu_r05a.sh r05c || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k cross_attention > gpurun_out/r05c/xattn_test.log 2>&1 || { tail -20 gpurun_out/r05c/xattn_test.log; exit 1; }
tail -1 gpurun_out/r05c/xattn_test.log
AB_REPS=2 bash tools/gpu_ab_env.sh xs default env:JANUS_XATTN_SPLITS=1

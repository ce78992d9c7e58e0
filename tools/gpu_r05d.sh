#!/bin/bash
# r05: persistent decoder segments — parity tests first (bounded), then the A/B bench
set -o pipefail
out=gpurun_out/${1:-r05d}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_whisper_gpu.py::test_persistent_staggered_bit_identical" "tests/test_whisper_gpu.py::test_persistent_segments_vs_oracle" "tests/test_pipeline_gpu.py::test_staggered_step_matches_sequential" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
grep -E "PASSED|FAILED|persistent segments" $out/pytest.log
AB_REPS=2 bash tools/gpu_ab_env.sh pers default env:JANUS_DEC_PERSIST=1 env:JANUS_DEC_PERSIST=1,JANUS_VOC_DEC_UTTS=4

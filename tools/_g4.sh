set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -5 gpurun_out/t_all.log; grep -E "windows decoded|identical|rms|PASS|FAIL" gpurun_out/t_all.log | tail -5; exit $rc

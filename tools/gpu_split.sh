set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for n in 16 12 20; do
  JANUS_OVERLAP_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --overlap $n > gpurun_out/split_$n.json 2> gpurun_out/split_$n.err || { tail -5 gpurun_out/split_$n.err; exit 1; }
  echo "$n $(python -c "import json;d=json.load(open('gpurun_out/split_$n.json'));print(d['ms_per_step'], d['step_ms'])") $(grep overlap gpurun_out/split_$n.err | tail -1)"
done; done

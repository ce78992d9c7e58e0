#!/bin/bash
# One GPU call for a round's evidence: full -m gpu suite, kernel-trace profile + bench line,
# PMC traffic (FETCH_SIZE / WRITE_SIZE passes) and SQ counters per vocoder family.
# usage (via gpurun): bash tools/gpu_evidence.sh <tag>   -> gpurun_out/<tag>/ + gpurun_out/traffic, pmc
set -o pipefail
tag=${1:-evidence}
root=$(pwd)
bash tools/gpu_check_round.sh $tag || exit 1
bash tools/gpu_traffic.sh || exit 1
bash tools/gpu_pmc_voc.sh || exit 1
cat $root/gpurun_out/traffic/traffic.json | head -c 1500

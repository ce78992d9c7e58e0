#!/bin/bash
# r05: vocoder utterances on the decoder side (persistent decoder on), sweep
set -o pipefail
AB_REPS=2 bash tools/gpu_ab_env.sh vsplit env:JANUS_VOC_DEC_UTTS=2 env:JANUS_VOC_DEC_UTTS=4 env:JANUS_VOC_DEC_UTTS=6 env:JANUS_VOC_DEC_UTTS=8

#!/bin/bash
# SQ counters per vocoder kernel family (standalone 64 x 30 s forward), two passes
set -o pipefail
root=$(pwd)
mkdir -p $root/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $root/gpurun_out/pmc/p1 -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/pmc/p1.log 2>&1 || { tail -5 $root/gpurun_out/pmc/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES -d $root/gpurun_out/pmc/p2 -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/pmc/p2.log 2>&1 || { tail -5 $root/gpurun_out/pmc/p2.log; exit 1; }
python3 $root/tools/pmc_reduce.py $root/gpurun_out/pmc/p1 $root/gpurun_out/pmc/p2 > $root/gpurun_out/pmc/families.json
python3 $root/tools/pmc_reduce.py $root/gpurun_out/pmc/p1 $root/gpurun_out/pmc/p2 --by-kernel > $root/gpurun_out/pmc/kernels.json
python3 -c "
import json; d=json.load(open('$root/gpurun_out/pmc/families.json'))
for k,v in d.items(): print(k, {x: v.get(x) for x in ('mfma_busy_frac','sq_wait_any_frac','sq_wait_inst_any_frac','sq_active_inst_any_frac','sq_wait_inst_lds_frac','lds_conflict_frac')})
"

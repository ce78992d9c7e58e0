#!/bin/bash
# Run GPU steps in order; stop at the first step that ends by a signal, a time limit or a
# GPU fault (rc not in {0, 1}); a plain test failure (rc 1) lets the next step run.
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i + 1))
  echo "=== step $i: $step" | tee -a gpurun_out/steps.log
  bash -c "$step" > "gpurun_out/step$i.log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/step$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

#!/bin/bash
# Work-queue lanes_per_pixel sweep per scene against the static grid (auto S).
set -u
timeout -k 10 500 python -m pytest tests -m gpu -q -rf -x > gpurun_out/gpu_all.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/gpu_all.log
for spec in ${SPEC:-cornellbox1:6 spheres:3 materialball:5 bunny:2 media:2}; do
  sc=${spec%%:*}; st=${spec##*:}
  echo "$sc static-auto $(RTMI_QUEUE=0 timeout -k 10 300 python bench.py --scene $sc --steps $st --warmup 1 --no-cpu-baseline | grep -o '"ms_per_step": [0-9.]*')"
  for S in ${S_LIST:-4 8 16 32}; do
    echo "$sc queue S=$S $(timeout -k 10 300 python bench.py --scene $sc --lanes $S --steps $st --warmup 1 --no-cpu-baseline | grep -o '"ms_per_step": [0-9.]*')"
  done
done

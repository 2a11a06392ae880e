#!/bin/bash
# lanes_per_pixel sweep per scene at N=1 (SPEC="scene:steps ..." S_LIST="...")
set -u
for spec in ${SPEC:-cornellbox1:5 spheres:3 materialball:5 bunny:2 media:2}; do
  scene=${spec%%:*}; steps=${spec##*:}
  for S in ${S_LIST:-1 2 4 8 16}; do
    echo "$scene S=$S $(timeout -k 10 300 python bench.py --scene $scene --lanes $S --steps $steps --warmup 1 --no-cpu-baseline | grep -o '"ms_per_step": [0-9.]*')" || exit 1
  done
done

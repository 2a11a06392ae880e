#!/bin/bash
# Same-box sweep of the sub-stream count S (bench --lanes) at the shipped build, two rounds interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03i_lanes}; mkdir -p $O
for r in 1 2; do
  for sv in "cornellbox1 16" "cornellbox1 32" "cornellbox1 64" "materialball 16" "materialball 32" "suzanne 16" "suzanne 32" "bunny 64" "bunny 128"; do
    set -- $sv
    timeout -k 10 300 python bench.py --scene $1 --lanes $2 --no-cpu-baseline > $O/bench_$1_S$2_$r.log 2>&1 || exit $?
    echo "$r $1 S=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$1_S$2_$r.log) $(grep -o '"kernel_ms": [0-9.]*' $O/bench_$1_S$2_$r.log)"
  done
done

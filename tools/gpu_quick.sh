#!/bin/bash
# Quick GPU iteration: parity tests + bench variants (no profiling).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal in $name"; exit "$rc"; fi; }
timeout -k 10 420 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
stop_if_fatal $? pytest
for lanes in ${LANES:-0 1 2}; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --lanes $lanes --no-cpu-baseline > gpurun_out/bench_l$lanes.log 2>&1
  stop_if_fatal $? bench_l$lanes
done
echo done

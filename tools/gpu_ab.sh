#!/bin/bash
# Parity tests on the default build, then bench A/B over variant libraries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal in $name"; exit "$rc"; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 420 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
  stop_if_fatal $? pytest
fi
for v in ${VARIANTS:-default}; do
  lib=raytracingthenextweekcuda_amd/librtmi.so
  [ "$v" != "default" ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
  for lanes in ${LANES:-0}; do
    RTMI_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 1 --lanes $lanes --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${v}_l$lanes.log 2>&1
    stop_if_fatal $? "bench $v lanes=$lanes"
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_l$lanes.log
  done
done
echo done

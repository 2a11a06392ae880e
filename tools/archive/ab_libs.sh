#!/bin/bash
# Same-box A/B of library builds: VARIANTS="base default" SCENE=cornellbox1 ROUNDS=3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-base default}; do
    lib=raytracingthenextweekcuda_amd/librtmi.so
    [ "$v" != "default" ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
    RTMI_LIB=$lib timeout -k 10 300 python bench.py --scene ${SCENE:-cornellbox1} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${v}_$r.log 2>&1 || exit $?
    echo "round $r $v $(grep -o "\"value\": [0-9.]*\|\"ms_per_step\": [0-9.]*" gpurun_out/ab_${v}_$r.log | tr "\n" " ")"
  done
done

#!/bin/bash
# Bench matrix on one GPU: optional parity tests, then bench.py per scene for the shipped
# library and optional A/B libraries (RTMI_LIB), optional PMC traffic passes and the VALU
# probe. Every GPU step has its own time limit; a fault/abort/timeout ends the script.
#   TAG=r02b TESTS=1 SCENES="cornellbox1 bunny" ALT="librtmi_w3.so" TRAFFIC="bunny" bash tools/gpu_bench_matrix.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-matrix}
mkdir -p "$O"
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal in $name"; exit "$rc"; fi; }
export TMPDIR=/tmp
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
  stop_if_fatal $? pytest
fi
for sc in ${SCENES:-cornellbox1}; do
  timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_$sc.log" 2>&1
  stop_if_fatal $? bench_$sc
  for alt in ${ALT:-}; do
    RTMI_LIB=raytracingthenextweekcuda_amd/$alt timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_${sc}_${alt%.so}.log" 2>&1
    stop_if_fatal $? bench_${sc}_$alt
  done
done
for sc in ${TRAFFIC:-}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${sc}_$c" -o pmc -- python3 bench.py --scene $sc --steps 1 --warmup 1 --no-cpu-baseline --no-overlap > "$O/pmc_${sc}_$c.log" 2>&1
    stop_if_fatal $? pmc_${sc}_$c
  done
done
for sc in ${VALU:-}; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d "$O/pmc_valu_$sc" -o pmc -- python3 bench.py --scene $sc --steps 2 --warmup 1 --no-cpu-baseline --no-overlap > "$O/pmc_valu_$sc.log" 2>&1
  stop_if_fatal $? pmc_valu_$sc
done
for sc in ${PROF:-}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$sc" -o run --output-format csv -- python3 bench.py --scene $sc --steps ${PROF_STEPS:-10} --warmup ${PROF_WARMUP:-2} --no-cpu-baseline --no-overlap > "$O/prof_$sc.log" 2>&1
  stop_if_fatal $? prof_$sc
done
if [ "${PROBE:-0}" = "1" ]; then
  for w in 4 8; do
    timeout -k 10 60 ./tools/valu_probe 200000 $w 1 > "$O/valu_probe_k_w$w.json" 2>&1
    stop_if_fatal $? probe_k_w$w
    timeout -k 10 60 ./tools/valu_probe 200000 $w 0 > "$O/valu_probe_v_w$w.json" 2>&1
    stop_if_fatal $? probe_v_w$w
  done
fi
echo done

#!/bin/bash
# Round-2 GPU session: parity tests (incl. reference renders, RCCL ABI, .bvh caches), smoke,
# the default bench, the VALU-roofline calibration (tools/valu_probe) and the CB1 counters.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r02}
mkdir -p "$O"
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal in $name"; exit "$rc"; fi; }
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
  stop_if_fatal $? pytest
  timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  stop_if_fatal $? smoke
fi
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1
stop_if_fatal $? bench
if [ "${PROBE:-1}" = "1" ]; then
  timeout -k 10 60 ./tools/valu_probe 20000 4 > "$O/valu_probe.json" 2>&1
  stop_if_fatal $? valu_probe
  for it in 10000 20000; do
    timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_probe_$it" -o pmc -- ./tools/valu_probe $it 4 > "$O/pmc_probe_$it.log" 2>&1
    stop_if_fatal $? pmc_probe_$it
  done
fi
for sc in ${PMC_SCENES:-cornellbox1}; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d "$O/pmc_valu_$sc" -o pmc -- python3 bench.py --scene $sc --steps 2 --warmup 1 --no-cpu-baseline --no-overlap > "$O/pmc_valu_$sc.log" 2>&1
  stop_if_fatal $? pmc_valu_$sc
done
for sc in ${PROF_SCENES:-cornellbox1}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$sc" -o run --output-format csv -- python3 bench.py --scene $sc --steps ${PROF_STEPS:-20} --warmup 5 --no-cpu-baseline --no-overlap > "$O/bench_${sc}_under_rocprof.log" 2>&1
  stop_if_fatal $? prof_$sc
done
if [ -x ./examples/multigpu ]; then
  timeout -k 10 120 ./examples/multigpu 128 96 8 1 > "$O/multigpu.log" 2>&1
  stop_if_fatal $? multigpu
fi
echo done

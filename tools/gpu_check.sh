#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal in $name"; exit "$rc"; fi; }
timeout -k 10 420 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
stop_if_fatal $? pytest
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
stop_if_fatal $? smoke
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-5} --warmup 1 > gpurun_out/bench.log 2>&1
stop_if_fatal $? bench
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  stop_if_fatal $? rocprof
fi
echo done

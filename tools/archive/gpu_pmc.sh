#!/bin/bash
# PMC counter passes (each its own run, --pmc only with kernel-trace output).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc/p$i -o pmc -- python3 $BENCH > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($counters) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done < "${PMC_FILE:-tools/pmc_sets.txt}"
echo done

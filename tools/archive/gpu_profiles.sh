#!/bin/bash
# Per-scene rocprofv3 evidence: kernel-trace stats, then FETCH_SIZE / WRITE_SIZE
# PMC passes (separate runs, no trace domains). SCENES overrides the list.
# Each GPU step is time-limited; a fatal status ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ]; then echo "fatal in $name"; exit "$rc"; fi; }
for spec in ${SCENES:-cornellbox1:5 spheres:3 bunny:2 materialball:5 media:2}; do
  scene=${spec%%:*}; steps=${spec##*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$scene -o run --output-format csv -- \
    python3 bench.py --scene $scene --steps $steps --warmup 1 --no-cpu-baseline > gpurun_out/prof_$scene.log 2>&1
  stop_if_fatal $? prof_$scene
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${scene}_$c -o pmc -- \
      python3 bench.py --scene $scene --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${scene}_$c.log 2>&1
    stop_if_fatal $? pmc_${scene}_$c
  done
done
echo done

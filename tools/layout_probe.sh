#!/bin/bash
# Same-box probes of bench knobs that need no rebuild: sub-streams per pixel (--lanes) for the
# media workload and the frame-overlap context count for the small pathTrace / Suzanne frames.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-layout}
mkdir -p "$O"
for l in 8 16 32 8; do
  timeout -k 10 300 python bench.py --scene media --lanes $l --steps 5 --warmup 1 --no-cpu-baseline > "$O/media_lanes$l.log" 2>&1 || exit $?
done
for sc in materialball suzanne; do
  for c in 2 3 2 3; do
    timeout -k 10 200 python bench.py --scene $sc --contexts $c --no-cpu-baseline > "$O/${sc}_ctx${c}_$RANDOM.log" 2>&1 || exit $?
  done
done
echo done

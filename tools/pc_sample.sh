#!/bin/bash
# Stochastic PC sampling (rocprofv3 --pc-sampling-*) of one bench workload's render kernel on a
# gpurun box: where the megakernel's issue slots go, instruction by instruction.
#   TAG=r04pc SCENE=cornellbox1 bash tools/pc_sample.sh   -> gpurun_out/$TAG/pcs_$SCENE/
# then: python tools/pc_summary.py gpurun_out/$TAG/pcs_$SCENE raytracingthenextweekcuda_amd/csrc/build/rt_kernel.s
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-pcs}; mkdir -p "$O"
export TMPDIR=/tmp
SC=${SCENE:-cornellbox1}
LAY=""; [ "$SC" = "cornellbox1" ] && LAY="--in-flight-layout"
timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} \
  --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-65536} --output-format csv \
  -d "$O/pcs_$SC" -o pcs -- python3 bench.py --scene $SC --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline \
  --no-overlap $LAY > "$O/pcs_$SC.log" 2>&1
echo "pcs_$SC rc=$?"

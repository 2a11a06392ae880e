#!/bin/bash
# Same-box A/B of library variants on the per-rank shard times (tools/shard_balance.py):
#   VARIANTS="default r4" ARGS="1:2 8:2" ROUNDS=2 bash tools/ab_shards.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-default}; do
    lib=raytracingthenextweekcuda_amd/librtmi.so
    [ "$v" != "default" ] && lib=raytracingthenextweekcuda_amd/librtmi_$v.so
    echo "round $r $v"
    RTMI_LIB=$lib timeout -k 10 200 python tools/shard_balance.py ${ARGS:-1:2 8:2} 2>&1 | grep world || exit 1
  done
done

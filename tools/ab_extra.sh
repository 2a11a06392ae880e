#!/bin/bash
# Extra same-box steps after tools/gpu_session.sh (round 6), into gpurun_out/$TAG/:
#   SHARD_ALT   libraries run beside the in-tree one at bench.py --rehearse-shard 8 (3 contexts), REPS rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-session}
mkdir -p "$O"
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ]; then echo "fatal in $name"; exit "$rc"; fi; }
if [ -n "${SHARD_ALT+x}" ]; then
  for rep in $(seq 1 ${REPS:-1}); do
    timeout -k 10 180 python bench.py --rehearse-shard 8 --contexts 3 --steps 60 --warmup 6 --no-cpu-baseline > "$O/shard8_c3_r$rep.log" 2>&1
    stop_if_fatal $? shard8_c3_r$rep
    for alt in $SHARD_ALT; do
      RTMI_LIB=raytracingthenextweekcuda_amd/$alt timeout -k 10 180 python bench.py --rehearse-shard 8 --contexts 3 --steps 60 --warmup 6 --no-cpu-baseline > "$O/shard8_c3_${alt%.so}_r$rep.log" 2>&1
      stop_if_fatal $? shard8_c3_${alt}_r$rep
    done
  done
fi
if [ "${GATHER_AB:-0}" = "1" ]; then  # rehearse-shard 8 with and without the ordered gathers (RTMI_GATHER_ORDER)
  for rep in $(seq 1 ${REPS:-1}); do
    timeout -k 10 180 python bench.py --rehearse-shard 8 --contexts 3 --steps 60 --warmup 6 --no-cpu-baseline > "$O/shard8_c3_order1_r$rep.log" 2>&1
    stop_if_fatal $? shard8_c3_order1_r$rep
    RTMI_GATHER_ORDER=0 timeout -k 10 180 python bench.py --rehearse-shard 8 --contexts 3 --steps 60 --warmup 6 --no-cpu-baseline > "$O/shard8_c3_order0_r$rep.log" 2>&1
    stop_if_fatal $? shard8_c3_order0_r$rep
  done
fi
echo done_extra

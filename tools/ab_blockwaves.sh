#!/bin/bash
# Same-box A/B of the work-queue block size (RT_QUEUE_BLOCK_WAVES: waves per persistent block) on a
# gpurun box: CB1 bench lines (three frames in flight) and rank 0's N = 8 shard alone / in flight,
# for the default library and the ALT ones (RTMI_LIB), interleaved REPS times.
#   TAG=r04g ALT="librtmi_bw1.so librtmi_bw2.so" REPS=2 bash tools/ab_blockwaves.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abbw}; mkdir -p "$O"
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for lib in librtmi.so ${ALT:-}; do
    n=${lib%.so}
    RTMI_LIB=raytracingthenextweekcuda_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench_cb1_${n}_r$rep.log" 2>&1 || exit 1
    RTMI_LIB=raytracingthenextweekcuda_amd/$lib FIF=0 CTX="1" timeout -k 10 120 python tools/overlap_probe.py 8 20 > "$O/shard8_alone_${n}_r$rep.log" 2>&1 || exit 1
    RTMI_LIB=raytracingthenextweekcuda_amd/$lib FIF=1 CTX="3" timeout -k 10 120 python tools/overlap_probe.py 8 30 > "$O/shard8_inflight_${n}_r$rep.log" 2>&1 || exit 1
    echo "$n r$rep $(grep -o '"ms_per_step": [0-9.]*' $O/bench_cb1_${n}_r$rep.log) | $(tail -1 $O/shard8_alone_${n}_r$rep.log) | $(tail -1 $O/shard8_inflight_${n}_r$rep.log)"
  done
done
echo done

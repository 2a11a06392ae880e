#!/bin/bash
# One GPU session on a gpurun box, from the repository root; everything lands in gpurun_out/$TAG/.
#   TESTS=1   pytest -m gpu + smoke()
#   BENCH=1   the default bench line (config 2, frame overlap, CPU baseline)
#   SCENES    bench lines of these workloads (no CPU baseline); ALT = A/B libraries run after each
#   SCENES_CPU  bench lines of these workloads with their CPU baseline
#   VALU      SQ_INSTS_VALU (+ lane utilisation, wait shares) and SQ_INSTS_SALU passes of these workloads (--no-overlap,
#             BENCH_ARGS appended: --in-flight-layout for the timed layout), for profiles/valu_issue.json
#   PROBE=1   tools/valu_probe under SQ counters with 64 and 16 active lanes (lane-utilisation calibration)
#   SPROBE=1  tools/valu_probe's issue rates: VALU, SALU and both, at 4 and 8 waves/SIMD
#   TRAFFIC   FETCH_SIZE and WRITE_SIZE passes (separate runs), for profiles/pmc_traffic.json
#   PROF      rocprofv3 --kernel-trace --stats of these workloads (--no-overlap)
#   MULTI=1   examples/multigpu (RCCL through the C ABI, N = 1 on this box)
#   STAMPS    tools/stamps_breakdown.py of these workloads with librtmi_stamps.so (tools/build_ab.sh stamps -DRT_STAMPS)
#   STREAMS=1 tools/queue_probe.py (how many streams run concurrently: 4 and 8 hardware queues), then
#             bench.py --rehearse-shard N (rank 0's rows of an N-rank CB1 frame, the N > 1 stream layout and
#             ABI exchange on a one-rank communicator) for N in SHARDS (default "8") and CTXS contexts
# Every GPU step has its own time limit; a fault, abort or time-out ends the session there.
#   TAG=r03c TESTS=1 BENCH=1 VALU="cornellbox1 bunny" bash tools/gpu_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-session}
mkdir -p "$O"
# the passes profile the layout the timed line uses: CB1's line keeps three frames in flight
lay() { if [ "$1" = "cornellbox1" ]; then echo "--in-flight-layout"; fi; }
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ]; then echo "fatal in $name"; exit "$rc"; fi; }
export TMPDIR=/tmp
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread --durations 15 > "$O/pytest_gpu.log" 2>&1
  stop_if_fatal $? pytest
  timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  stop_if_fatal $? smoke
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1
  stop_if_fatal $? bench
fi
for sc in ${SCENES_CPU:-}; do  # bench lines WITH the CPU baseline (the oracle on this box's host cores)
  timeout -k 10 420 python bench.py --scene $sc ${BENCH_ARGS:-} > "$O/bench_$sc.log" 2>&1
  stop_if_fatal $? bench_$sc
done
for sc in ${SCENES:-}; do
 for rep in $(seq 1 ${REPS:-1}); do  # REPS > 1: the A/B round repeated, logs suffixed _r<rep>
  sfx=""; [ "${REPS:-1}" -gt 1 ] && sfx="_r$rep"
  timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_$sc$sfx.log" 2>&1
  stop_if_fatal $? bench_$sc$sfx
  for alt in ${ALT:-}; do  # A/B libraries of the same sources (RTMI_LIB), same box, interleaved
    RTMI_LIB=raytracingthenextweekcuda_amd/$alt timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_${sc}_${alt%.so}$sfx.log" 2>&1
    stop_if_fatal $? bench_${sc}_$alt$sfx
  done
 done
done
if [ "${PROBE:-0}" = "1" ] && [ -x ./tools/valu_probe ]; then  # lane-utilisation calibration (64 / 16 lanes)
  for a in 64 16; do
    timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d "$O/probe_lanes_$a" -o pmc -- ./tools/valu_probe 10000 4 0 $a > "$O/probe_lanes_$a.log" 2>&1
    stop_if_fatal $? probe_lanes_$a
  done
fi
if [ "${SPROBE:-0}" = "1" ] && [ -x ./tools/valu_probe ]; then  # issue-rate probes: VALU, SALU, both (4 and 8 waves/SIMD)
  for w in 4 8; do for m in 0 1 2 3; do
    timeout -k 10 60 ./tools/valu_probe 20000 $w $m > "$O/issue_probe_w${w}_m$m.json" 2>&1
    stop_if_fatal $? issue_probe_w${w}_m$m
  done; done
fi
for sc in ${VALU:-}; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d "$O/pmc_valu_$sc" -o pmc -- python3 bench.py --scene $sc --steps 2 --warmup 1 --no-cpu-baseline --no-overlap $(lay $sc) > "$O/pmc_valu_$sc.log" 2>&1
  stop_if_fatal $? pmc_valu_$sc
  # the scalar side (one scalar ALU per CU, shared by its four SIMDs): a pass of its own (8 SQ counters per pass)
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_salu_$sc" -o pmc -- python3 bench.py --scene $sc --steps 2 --warmup 1 --no-cpu-baseline --no-overlap $(lay $sc) > "$O/pmc_salu_$sc.log" 2>&1
  stop_if_fatal $? pmc_salu_$sc
done
for sc in ${TRAFFIC:-}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${sc}_$c" -o pmc -- python3 bench.py --scene $sc --steps 1 --warmup 1 --no-cpu-baseline --no-overlap $(lay $sc) > "$O/pmc_${sc}_$c.log" 2>&1
    stop_if_fatal $? pmc_${sc}_$c
  done
done
for sc in ${TCC:-}; do  # L2 hit / miss (TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)) and fabric read requests
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d "$O/pmc_tcc_$sc" -o pmc -- python3 bench.py --scene $sc --steps 1 --warmup 1 --no-cpu-baseline --no-overlap $(lay $sc) > "$O/pmc_tcc_$sc.log" 2>&1
  stop_if_fatal $? pmc_tcc_$sc
  for alt in ${TCC_ALT:-}; do
    RTMI_LIB=raytracingthenextweekcuda_amd/$alt timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d "$O/pmc_tcc_${sc}_${alt%.so}" -o pmc -- python3 bench.py --scene $sc --steps 1 --warmup 1 --no-cpu-baseline --no-overlap $(lay $sc) > "$O/pmc_tcc_${sc}_${alt%.so}.log" 2>&1
    stop_if_fatal $? pmc_tcc_${sc}_$alt
  done
done
for sc in ${PROF:-}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$sc" -o run --output-format csv -- python3 bench.py --scene $sc --steps ${PROF_STEPS:-10} --warmup ${PROF_WARMUP:-2} --no-cpu-baseline --no-overlap $(lay $sc) > "$O/prof_$sc.log" 2>&1
  stop_if_fatal $? prof_$sc
done
if [ -n "${STAMPS:-}" ] && [ -f raytracingthenextweekcuda_amd/librtmi_stamps.so ]; then  # section timers (RT_STAMPS build)
  RTMI_LIB=raytracingthenextweekcuda_amd/librtmi_stamps.so timeout -k 10 300 python tools/stamps_breakdown.py $STAMPS > "$O/stamps.log" 2>&1
  stop_if_fatal $? stamps
fi
if [ "${STREAMS:-0}" = "1" ]; then
  timeout -k 10 120 python tools/queue_probe.py > "$O/queue_probe.json" 2> "$O/queue_probe.err"
  stop_if_fatal $? queue_probe
  timeout -k 10 120 python tools/queue_probe.py --rccl-first > "$O/queue_probe_rccl_first.json" 2> "$O/queue_probe_rccl_first.err"
  stop_if_fatal $? queue_probe_rccl_first
  GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/queue_probe.py > "$O/queue_probe_q8.json" 2> "$O/queue_probe_q8.err"
  stop_if_fatal $? queue_probe_q8
  for rep in $(seq 1 ${REPS:-1}); do
    for n in ${SHARDS:-8}; do for c in ${CTXS:-2 3}; do
      timeout -k 10 180 python bench.py --rehearse-shard $n --contexts $c --steps ${SSTEPS:-60} --warmup 6 --no-cpu-baseline > "$O/shard${n}_c${c}_r$rep.log" 2>&1
      stop_if_fatal $? shard${n}_c${c}_r$rep
    done; done
    for q in ${QUEUES:-}; do  # more hardware queues for the process: one more context than the default
      GPU_MAX_HW_QUEUES=$q timeout -k 10 180 python bench.py --rehearse-shard 8 --contexts 4 --steps ${SSTEPS:-60} --warmup 6 --no-cpu-baseline > "$O/shard8_c4_q${q}_r$rep.log" 2>&1
      stop_if_fatal $? shard8_c4_q${q}_r$rep
    done
  done
fi
if [ "${MULTI:-0}" = "1" ] && [ -x ./examples/multigpu ]; then
  timeout -k 10 120 ./examples/multigpu 128 96 8 1 > "$O/multigpu.log" 2>&1
  stop_if_fatal $? multigpu
fi
echo done

#!/bin/bash
# Frames-in-flight layout (RT_RENDER_FRAMES_IN_FLIGHT) on a gpurun box: its GPU tests, CB1 bench
# lines, and CB1's VALU / traffic / trace passes at the layout the timed line uses (--in-flight-layout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03i_if}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_bench.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; exit 1; }
echo tests ok
for r in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$r.log 2>&1 || exit 1
  echo "bench $r $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$r.log) $(grep -o '"lanes_per_pixel": [0-9]*' $O/bench_$r.log | head -1)"
done
A="--scene cornellbox1 --no-cpu-baseline --no-overlap --in-flight-layout"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $O/pmc_valu_cornellbox1 -o pmc -- python3 bench.py $A --steps 2 --warmup 1 > $O/pmc_valu_cornellbox1.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_cornellbox1_$c -o pmc -- python3 bench.py $A --steps 1 --warmup 1 > $O/pmc_cornellbox1_$c.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cornellbox1 -o run --output-format csv -- python3 bench.py $A --steps 10 --warmup 2 > $O/prof_cornellbox1.log 2>&1 || exit 1
echo done

#!/bin/bash
# Round check: tests, smoke, bench (N=1 default), rehearsal of N=2 on one GPU,
# rocprofv3 kernel-trace stats, PMC traffic passes. Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() { rc=$1; name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal in $name"; exit "$rc"; fi; }
timeout -k 10 420 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
stop_if_fatal $? pytest
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
stop_if_fatal $? smoke
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
stop_if_fatal $? bench
RTMI_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_rehearsal_n2.log 2>&1
stop_if_fatal $? rehearsal
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
stop_if_fatal $? rocprof
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1
  stop_if_fatal $? pmc_$c
done
echo done

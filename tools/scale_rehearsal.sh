#!/bin/bash
# One-GPU rehearsal of the N > 1 path (gpurun box, repository root): frame overlap per row-tile
# shard of CornellBox1 for N = 1, 2, 4, 8 (tools/overlap_probe.py: rank 0's shard, alone and with
# three contexts / frames-in-flight items as bench.py runs it), then bench.py's N = 2 line through torch.distributed.run with two ranks sharing GPU 0
# and gathering over gloo (RTMI_REHEARSAL=1: the code path, not a scaling number).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03s}
mkdir -p "$O"
export TMPDIR=/tmp
# alone (one context, no frames-in-flight items) and as the bench runs it (three contexts, FIF items)
for w in 1 2 4 8; do
  FIF=0 CTX="1" timeout -k 10 120 python tools/overlap_probe.py $w 20 > $O/overlap_cb1_w${w}_alone.log 2>&1 || exit 1
  FIF=1 CTX="3" timeout -k 10 120 python tools/overlap_probe.py $w 30 > $O/overlap_cb1_w${w}_inflight.log 2>&1 || exit 1
  FIF=0 CTX="3" timeout -k 10 120 python tools/overlap_probe.py $w 30 > $O/overlap_cb1_w${w}_inflight_g1.log 2>&1 || exit 1
done
RTMI_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_rehearsal_n2.log 2>&1 || exit 1
echo done

#!/bin/bash
# CB1 rank-0 row shard at N = 1, 2, 4, 8 with S = 16 vs 32 sub-streams (one and three contexts), one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03i_lshard}; mkdir -p $O
for w in 1 2 4 8; do for s in 16 32; do
  LANES=$s CTX="1 3" timeout -k 10 120 python tools/overlap_probe.py $w 30 > $O/overlap_w${w}_S$s.log 2>&1 || exit 1
  tail -n 2 $O/overlap_w${w}_S$s.log
done; done

#!/bin/bash
# Refill threshold 4 vs 8 (fixed-threshold builds) per scene, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in spheres:3 bunny:2 media:2 materialball:5 suzanne:5 cornellbox1:5; do
  SCENE=${spec%%:*} STEPS=${spec##*:} VARIANTS="r4 r8" ROUNDS=2 bash tools/ab_libs.sh | sed "s/^/${spec%%:*} /" || exit 1
done

#!/bin/bash
# Leaf-size A/B for rayColor BVHs (RTMI_MESH_LEAF / RTMI_SPHERE_LEAF = Recurse's leaf threshold)
set -u
for L in ${LEAVES:-4 8 16}; do
  echo "bunny leaf<$L $(RTMI_MESH_LEAF=$L timeout -k 10 300 python bench.py --scene bunny --steps 2 --warmup 1 --no-cpu-baseline | grep -o '"ms_per_step": [0-9.]*')"
  echo "spheres leaf<$L $(RTMI_SPHERE_LEAF=$L timeout -k 10 300 python bench.py --scene spheres --steps 3 --warmup 1 --no-cpu-baseline | grep -o '"ms_per_step": [0-9.]*')"
done

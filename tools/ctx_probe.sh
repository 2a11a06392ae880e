set -u
mkdir -p gpurun_out/ctx
for w in 1 8; do
  CTX="1 2 3 4" timeout -k 10 200 python tools/overlap_probe.py $w 40 > gpurun_out/ctx/overlap_w$w.log 2>&1 || exit $?
done
SCENE=spheres CTX="1 2 3" timeout -k 10 200 python tools/overlap_probe.py 8 20 > gpurun_out/ctx/overlap_spheres_w8.log 2>&1

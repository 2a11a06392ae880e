import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import raytracingthenextweekcuda_amd as rtmi
from oracle import oracle as orc
w = h = 64
r = rtmi.Renderer(0); rtmi.cornell_box1(r, w, h)
for depth in (1, 2, 3):
    img = r.render(w, h, 1, depth)
    ref, st = orc.yaml_scene('assets/scenes/cornellbox1.yaml', 'assets/models', w, h).render(w, h, 1, depth)
    diff = np.abs(img - ref).max(axis=2)
    ys, xs = np.nonzero(diff > 0)
    print('depth', depth, 'ndiff', len(ys), 'segs', r.stats()['segments'], st['segments'])
    for y, x in list(zip(ys, xs))[:5]:
        print('  ', y, x, img[y, x], ref[y, x])

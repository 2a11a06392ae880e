"""GPU diagnostic: L-inf and bit-exact fraction of the pathTrace kernel vs the oracle."""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests import scenes as S  # noqa: E402
import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

for name in S.PT_SCENES:
    pt, cam = S.build_pathtrace_oracle(name)
    want, ost = pt.render(cam, 64, 64, 8, 5, threads=16)
    r = rtmi.Renderer(0)
    S.build_pathtrace_product(r, name)
    got = r.render(64, 64, 8, 5, integrator="pathTrace")
    st = r.stats()
    r.close()
    d = np.abs(got - want)
    print(name, "linf", float(d.max()), "exact", float((got == want).mean()), "segs", st["segments"],
          ost["segments"], "nodes/seg", st["node_visits"] / st["segments"], "tris/seg",
          st["tri_tests"] / st["segments"], "oracle tris/seg", ost["tri_tests"] / ost["segments"], flush=True)

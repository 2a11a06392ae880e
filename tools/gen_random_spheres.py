"""Generate the RTNW final scene of the reference's SCENE 2 branch
(R/main.cu:792-848) deterministically.

The reference draws from std::random_device (R/Utils.h:25-30), which is not
reproducible, and that branch does not compile as committed.
This script replays its logic with numpy's MT19937 (seed 1984). Draws follow
the source's left-to-right reading. Values are float32 like the reference's
uniform_real_distribution<float>. Output: assets/scenes/random_spheres.json,
which is committed as the fixture both the product and the oracle read.
"""
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(seed=1984):
    rs = np.random.RandomState(seed)
    f32 = np.float32

    def u():
        return f32(rs.random_sample())

    def rnd(lo, hi):  # randomFloat(min, max) = min + (max - min) * u (Utils.h:27-29)
        return f32(f32(lo) + f32(f32(hi) - f32(lo)) * u())

    def color():  # Color::random() (Utils.h:163-165)
        return np.array([u(), u(), u()], dtype=f32)

    def color_range(lo, hi):  # Color::random(min, max) (Utils.h:167-170)
        c = color()
        return (f32(lo) + f32(f32(hi) - f32(lo)) * c).astype(f32)

    objs = []
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = u()
            cx = f32(f32(a) + f32(0.9) * u())
            cz = f32(f32(b) + f32(0.9) * u())
            center = np.array([cx, f32(0.2), cz], dtype=f32)
            dvec = center - np.array([4.0, 0.2, 0.0], dtype=f32)
            length = np.sqrt(f32(dvec[0] * dvec[0] + dvec[1] * dvec[1] + dvec[2] * dvec[2]), dtype=f32)
            if length > f32(0.9):
                if choose < f32(0.8):
                    albedo = (color() * color()).astype(f32)
                    dy = rnd(0.0, 0.5)
                    c1 = center + np.array([0, dy, 0], dtype=f32)
                    objs.append({"kind": "moving_sphere", "center0": center.tolist(), "center1": c1.tolist(),
                                 "time0": 0.0, "time1": 1.0, "radius": 0.2,
                                 "material": {"type": "lambertian", "albedo": albedo.tolist()}})
                elif choose < f32(0.95):
                    albedo = color_range(0.5, 1.0)
                    fuzz = rnd(0.0, 0.5)
                    objs.append({"kind": "sphere", "center": center.tolist(), "radius": 0.2,
                                 "material": {"type": "metal", "albedo": albedo.tolist(), "fuzz": float(fuzz)}})
                else:
                    objs.append({"kind": "sphere", "center": center.tolist(), "radius": 0.2,
                                 "material": {"type": "dielectric", "ior": 1.5}})
            else:
                albedo = (color() * color()).astype(f32)
                objs.append({"kind": "sphere", "center": center.tolist(), "radius": 0.2,
                             "material": {"type": "lambertian", "albedo": albedo.tolist()}})
    objs.append({"kind": "sphere", "center": [0.0, -1000.0, 0.0], "radius": 1000.0,
                 "material": {"type": "lambertian", "albedo": [0.5, 0.5, 0.5]}})
    objs.append({"kind": "sphere", "center": [0.0, 1.0, 0.0], "radius": 1.0,
                 "material": {"type": "dielectric", "ior": 1.5}})
    objs.append({"kind": "sphere", "center": [-4.0, 1.0, 0.0], "radius": 1.0,
                 "material": {"type": "lambertian", "albedo": [0.4, 0.2, 0.1]}})
    objs.append({"kind": "sphere", "center": [4.0, 1.0, 0.0], "radius": 1.0,
                 "material": {"type": "metal", "albedo": [0.7, 0.6, 0.5], "fuzz": 0.0}})
    scene = {
        "source": "R/main.cu:792-848 (SCENE 2), replayed by tools/gen_random_spheres.py with MT19937 seed %d" % seed,
        "camera": {"eye": [13.0, 2.0, 3.0], "center": [0.0, 0.0, 0.0], "up": [0.0, 1.0, 0.0],
                   "fov": 20.0, "aperture": 0.1, "focus": 10.0, "time0": 0.0, "time1": 1.0},
        "objects": objs,
    }
    out = os.path.join(REPO, "assets", "scenes", "random_spheres.json")
    with open(out, "w") as fh:
        json.dump(scene, fh, indent=0)
    print(out, len(objs), "objects")


if __name__ == "__main__":
    main()

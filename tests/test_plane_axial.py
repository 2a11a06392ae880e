"""The axial-plane form of Plane::hit (rt_kernel.hip plane_axial) against the reference's general form
(Plane.cu:4-52, restated in oracle/rt_oracle.c plane_hit), evaluated in float32 with the same operation order.

rt_scene.cpp gives a plane whose normal is +-1 on its orientation's normal axis (and +-0 on the other two) the
record kind kObjPlaneAxial + orientation; the kernel then forms den = n_K * d_K and num = (p_K - o_K) * n_K
instead of the full dot products, and the two-sided test as max(|den| * u1, den) > tMin with u1 = 1.0f or 0.0f.
The claim (argued in plane_axial's comment) is that the candidate t - or "no candidate" - is the same float for
every ray, including zero, -0, subnormal, huge, inf and NaN components. Here it is checked on a few hundred
thousand such rays per orientation (CPU only; the GPU suite renders the reference's scenes through it)."""
import numpy as np
import pytest

F = np.float32
T_MIN = F(0.001)
NAN = F(np.nan)
SPECIAL = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-38, -1e-30, 1e-4, -1e-3, 0.5, -0.75, 1.0, -1.0, 3.0e5, -7.0e20,
                    1e30, -3e38, np.inf, -np.inf, np.nan], dtype=np.float32)
# orientation -> (normal axis K, in-plane axes A, B): XY, YZ, XZ (rt_scene.cpp, rt_kernel.hip closest_hit)
AXES = {0: (2, 0, 1), 1: (0, 1, 2), 2: (1, 0, 2)}


def general(o, d, p, n, bounds, two_sided, orient):
    """Plane.cu's operation order: den = dot(n, d), num = dot(p - o, n), t = num / den (IEEE division)."""
    with np.errstate(all="ignore"):
        den = (n[0] * d[0] + n[1] * d[1]) + n[2] * d[2]
        proceed = (np.abs(den) > T_MIN) if two_sided else (den > T_MIN)
        q = [p[k] - o[k] for k in range(3)]
        num = (q[0] * n[0] + q[1] * n[1]) + q[2] * n[2]
        t = num / den
        _, a, b = AXES[orient]
        pa = o[a] + d[a] * t
        pb = o[b] + d[b] * t
        ok = proceed & (t >= T_MIN) & (pa > bounds[0]) & (pa < bounds[1]) & (pb > bounds[2]) & (pb < bounds[3])
        return np.where(ok, t, NAN)


def axial(o, d, p, n, bounds, two_sided, orient):
    """rt_kernel.hip plane_axial: the one non-zero term, and the two-sided test as a float max."""
    k, a, b = AXES[orient]
    u1 = F(1.0) if two_sided else F(0.0)
    with np.errstate(all="ignore"):
        den = n[k] * d[k]
        proceed = np.fmax(np.abs(den) * u1, den) > T_MIN
        num = (p[k] - o[k]) * n[k]
        t = num / den
        pa = o[a] + d[a] * t
        pb = o[b] + d[b] * t
        ok = proceed & (t >= T_MIN) & (pa > bounds[0]) & (pa < bounds[1]) & (pb > bounds[2]) & (pb < bounds[3])
        return np.where(ok, t, NAN)


def rays(rng, m, p, e):
    """Origins and directions aimed at the plane's rectangle (and around it), with special values mixed into
    random components."""
    o = rng.uniform(-2, 2, size=(3, m)).astype(F)
    target = (p[:, None] + rng.uniform(-1.5, 1.5, size=(3, m)) * e[:, None]).astype(F)
    d = target - o
    d /= np.sqrt((d * d).sum(axis=0)).astype(F)
    for arr in (o, d):
        mask = rng.random(size=arr.shape) < 0.15
        arr[mask] = rng.choice(SPECIAL, size=int(mask.sum()))
    return o, d


@pytest.mark.parametrize("orient", [0, 1, 2])
@pytest.mark.parametrize("sign", [1.0, -1.0])
@pytest.mark.parametrize("two_sided", [True, False])
def test_axial_plane_candidate_equals_the_general_one(orient, sign, two_sided):
    rng = np.random.default_rng(1000 * orient + int(sign > 0) * 10 + int(two_sided))
    k, a, b = AXES[orient]
    for zeros in ((0.0, 0.0), (-0.0, 0.0), (0.0, -0.0), (-0.0, -0.0)):  # the normal's in-plane zeros, any sign
        n = [F(0.0)] * 3
        n[k] = F(sign)
        n[a], n[b] = F(zeros[0]), F(zeros[1])
        p = rng.uniform(-1, 1, size=3).astype(F)
        e = rng.uniform(0.1, 1.0, size=3).astype(F)
        bounds = [p[a] - e[a], p[a] + e[a], p[b] - e[b], p[b] + e[b]]  # rt_scene.cpp: position -/+ extend
        tgt_e = e.copy()
        tgt_e[k] = 0.0
        o, d = rays(rng, 60000, p, tgt_e)
        g = general(o, d, p, n, bounds, two_sided, orient)
        x = axial(o, d, p, n, bounds, two_sided, orient)
        same = (g.view(np.uint32) == x.view(np.uint32)) | (np.isnan(g) & np.isnan(x))
        assert same.all(), (orient, sign, two_sided, zeros, np.argwhere(~same)[:5].ravel(),
                            o[:, ~same][:, :3], d[:, ~same][:, :3], g[~same][:3], x[~same][:3])
        # the sample exercises both outcomes
        assert np.isfinite(g).sum() > 2000 and np.isnan(g).sum() > 2000

"""GPU parity: the HIP megakernel (through the C ABI) against the CPU
restatement on identical scenes and seeds.

Tolerance (BASELINE.json north_star): per-channel L_inf <= 1e-4 on the float
mean-radiance buffer. Both sides follow the reference's float evaluation order
with -ffp-contract=off and IEEE div/sqrt, so the expected result is bit-exact;
the tests also require identical traced-segment counts (same paths)."""
import os

import numpy as np
import pytest

from tests import scenes as S

TOL = 1e-4

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rtmi():
    import raytracingthenextweekcuda_amd as m

    return m


def _oracle_yaml(name, w, h):
    from oracle import oracle as orc

    return orc.yaml_scene(os.path.join(S.SCENES, name), S.MODELS, w, h)


def _check(img, ref, st, ref_st, tag):
    assert img.shape == ref.shape, tag
    err = float(np.max(np.abs(img.astype(np.float64) - ref)))
    exact = float(np.mean(img == ref))
    assert np.isfinite(img).all(), tag
    assert err <= TOL, f"{tag}: L_inf {err} (bit-exact fraction {exact:.4f})"
    assert st["segments"] == ref_st["segments"], (tag, st["segments"], ref_st["segments"])
    return err, exact


@pytest.mark.parametrize("w,h,spp,depth", [(64, 64, 4, 4), (96, 64, 8, 8), (33, 17, 3, 10)])
def test_cornellbox1_parity(rtmi, w, h, spp, depth):
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        img = r.render(w, h, spp, depth)
        st = r.stats()
    ref, ref_st = _oracle_yaml("cornellbox1.yaml", w, h).render(w, h, spp, depth)
    err, exact = _check(img, ref, st, ref_st, f"cb1 {w}x{h} spp{spp} d{depth}")
    assert exact == 1.0, f"expected bit-exact, got {exact}"
    assert st["tri_tests"] == ref_st["tri_tests"]
    assert st["samples"] == w * h * spp


@pytest.mark.parametrize("name", ["cornellbox0.yaml", "cornellbox2.yaml", "cornellbox3.yaml", "cornellbox_empty.yaml",
                                  "suzanne_cornellbox.yaml"])
def test_yaml_scenes_parity(rtmi, name):
    w, h, spp, depth = 48, 48, 4, 10
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, os.path.join(S.SCENES, name), w, h)
        img = r.render(w, h, spp, depth)
        st = r.stats()
    ref, ref_st = _oracle_yaml(name, w, h).render(w, h, spp, depth)
    _check(img, ref, st, ref_st, name)


@pytest.mark.parametrize("maker", [S.spheres_scene, S.mixed_scene])
def test_spec_scenes_parity(rtmi, maker):
    spec = maker()
    w, h, spp, depth = 64, 48, 4, 10
    with rtmi.Renderer(0) as r:
        S.build_product(r, spec)
        img = r.render(w, h, spp, depth, seed=7, sample_offset=3)
        st = r.stats()
    ref, ref_st = S.build_oracle(spec).render(w, h, spp, depth, seed=7, sample_offset=3)
    _check(img, ref, st, ref_st, maker.__name__)


@pytest.mark.parametrize("world,block", [(2, 8), (3, 5), (8, 1)])
def test_row_tiling_is_bit_identical(rtmi, world, block):
    """Frames sharded by pixel-row tiles reassemble to the single-GPU frame
    bit for bit (RNG keyed by the global pixel index)."""
    w, h, spp, depth = 40, 37, 2, 6
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        full = r.render(w, h, spp, depth)
        tiles = np.zeros_like(full)
        seg = 0
        for rank in range(world):
            part = r.render(w, h, spp, depth, row_block=block, row_rank=rank, row_world=world)
            rows = rtmi.owned_row_ids(h, block, rank, world)
            assert part.shape[0] == len(rows)
            tiles[rows] = part
            seg += r.stats()["segments"]
        r.render(w, h, spp, depth)
        assert seg == r.stats()["segments"]
    assert np.array_equal(full, tiles)


def test_zero_depth_is_black(rtmi):
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, 16, 16)
        img = r.render(16, 16, 2, 0)
        assert r.stats()["segments"] == 0
    assert not img.any()


def test_progressive_accumulation_matches_single_pass(rtmi):
    """Realtime mode (spp batches with sample_offset, Canvas running mean) equals
    one pass at the total spp up to float summation order."""
    from raytracingthenextweekcuda_amd.canvas import Canvas

    w = h = 32
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        one = r.render(w, h, 8, 6)
        cv = Canvas(w, h)
        for k in range(4):
            cv.accumulate(r.render(w, h, 2, 6, sample_offset=2 * k), 2)
    assert np.max(np.abs(cv.mean() - one)) <= 1e-5


def test_render_errors(rtmi):
    from raytracingthenextweekcuda_amd._lib import RTError

    with rtmi.Renderer(0) as r:
        with pytest.raises(RTError, match="RT_ERR_STATE"):
            r.render(8, 8, 1, 1)
        rtmi.cornell_box1(r, 8, 8)
        with pytest.raises(RTError, match="RT_ERR_INVALID"):
            r.render(1, 8, 1, 1)
        with pytest.raises(RTError, match="RT_ERR_INVALID"):
            r.render(8, 8, 0, 1)
        with pytest.raises(RTError, match="RT_ERR_INVALID"):
            r.render(8, 8, 1, 1, row_rank=2, row_world=2)
        # 8192^2 pixels x 128 sub-streams exceed the 32-bit item index: the static grid
        # cannot hold 128 sub-streams of a pixel in one wave, so the launch is refused
        rtmi.cornell_box1(r, 8192, 8192)
        with pytest.raises(RTError, match="needs the work queue"):
            r.render(8192, 8192, 128, 1, lanes_per_pixel=128)


def test_render_into_torch_buffer(rtmi):
    """rt_render_device writes into a caller-owned HBM buffer on a torch stream."""
    torch = pytest.importorskip("torch")
    w = h = 24
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        host = r.render(w, h, 2, 4)
        buf = torch.empty((h, w, 3), dtype=torch.float32, device="cuda:0")
        s = torch.cuda.Stream()
        r.render_device(r.params(w, h, 2, 4), buf.data_ptr(), s.cuda_stream)
        s.synchronize()
        st = r.stats()
    assert st["kernel_ms"] > 0
    assert np.array_equal(buf.cpu().numpy(), host)


@pytest.mark.parametrize("lanes", [2, 4, 16, 64])
def test_lanes_per_pixel_parity(rtmi, lanes):
    """Samples of one pixel split over `lanes` lanes, partial sums combined in a
    fixed order: bit-exact against the restatement using the same order, and
    within float summation-order noise of the sequential (reference) order."""
    w, h, spp, depth = 40, 24, 64, 6
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        img = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
        st = r.stats()
        assert st["lanes_per_pixel"] == lanes
    sc = _oracle_yaml("cornellbox1.yaml", w, h)
    ref, ref_st = sc.render(w, h, spp, depth, lanes_per_pixel=lanes)
    _check(img, ref, st, ref_st, f"lanes{lanes}")
    assert np.array_equal(img, ref)
    seq, _ = sc.render(w, h, spp, depth)
    assert np.max(np.abs(img - seq)) <= 1e-5


@pytest.mark.parametrize("spp", [64, 128])
def test_one_sample_per_substream_is_the_sequential_sum(rtmi, spp):
    # S = spp (work queue, up to 128 sub-streams): every item is one sample and the
    # fixed-order combine ((p0 + p1) + p2) + ... is the reference's sequential sum, so
    # the image equals S = 1 bit for bit (and the oracle's sequential order)
    w, h, depth = 24, 16, 5
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        one = r.render(w, h, spp, depth, lanes_per_pixel=spp)
        assert r.stats()["lanes_per_pixel"] == spp
        seq = r.render(w, h, spp, depth, lanes_per_pixel=1)
    ref, _ = _oracle_yaml("cornellbox1.yaml", w, h).render(w, h, spp, depth)
    assert np.array_equal(one, seq)
    assert np.array_equal(one, ref)


@pytest.mark.parametrize("integrator", ["rayColor", "pathTrace"])
def test_more_substreams_than_samples(rtmi, integrator):
    # S > spp: sub-streams without samples must still clear their partial-sum slots.
    # The first render fills the context's partial buffer with nonzero sums; the
    # second (spp 4 < S 8) reuses it and must not pick them up.
    w, h, depth = 24, 16, 5
    with rtmi.Renderer(0) as r:
        if integrator == "pathTrace":
            rtmi.materialball(r, w, h)
        else:
            rtmi.cornell_box1(r, w, h)
        r.render(w, h, 8, depth, lanes_per_pixel=8, integrator=integrator)
        img = r.render(w, h, 4, depth, lanes_per_pixel=8, integrator=integrator)
        ref = r.render(w, h, 4, depth, lanes_per_pixel=1, integrator=integrator)
    assert np.array_equal(img, ref)  # empty sub-streams add +0.0: the sequential sum


def test_auto_lane_layout(rtmi):
    # work-queue launches: largest power of two S <= min(32, spp) with pixels * S <= 2^25
    # (rt_kernel.h choose_layout)
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, 64, 64)
        r.render(64, 64, 32, 4, lanes_per_pixel=0)
        assert r.stats()["lanes_per_pixel"] == 32
        r.render(64, 64, 8, 4, lanes_per_pixel=0)
        assert r.stats()["lanes_per_pixel"] == 8
        r.render(2048, 2048, 64, 1, lanes_per_pixel=0)
        assert r.stats()["lanes_per_pixel"] == 8  # 4M pixels x 8 = 2^25 work items


def test_frames_in_flight_layout(rtmi):
    # RT_RENDER_FRAMES_IN_FLIGHT: linear-scan work-queue launches hand out items of several
    # sub-streams (at most 16 items per pixel, rt_capi.cpp validate); the sub-streams, and so the
    # image, stay those of lanes_per_pixel, byte for byte - with the flag or without, auto or explicit,
    # and against the oracle (the full-size C2 case in test_full_size.py checks the bench's frame)
    from oracle import oracle as orc

    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, 48, 32)
        img = r.render(48, 32, 64, 4, lanes_per_pixel=0, frames_in_flight=True)
        st = r.stats()
        assert st["lanes_per_pixel"] == 32 and st["substreams_per_item"] == 2
        assert np.array_equal(img, r.render(48, 32, 64, 4, lanes_per_pixel=0))
        assert r.stats()["substreams_per_item"] == 1
        assert np.array_equal(img, r.render(48, 32, 64, 4, lanes_per_pixel=32, frames_in_flight=True))
        sc = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox1.yaml"), S.MODELS, 48, 32)
        want, ost = sc.render(48, 32, 64, 4, lanes_per_pixel=32)
        assert np.array_equal(img, want) and st["segments"] == ost["segments"]
        # 128 sub-streams for 64 samples: the groups' second halves have no samples (zero partials)
        img = r.render(48, 32, 64, 4, lanes_per_pixel=128, frames_in_flight=True)
        assert r.stats()["substreams_per_item"] == 8
        assert np.array_equal(img, r.render(48, 32, 64, 4, lanes_per_pixel=128))
        r.render(48, 32, 8, 4, lanes_per_pixel=0, frames_in_flight=True)
        assert r.stats()["lanes_per_pixel"] == 8 and r.stats()["substreams_per_item"] == 1
    with rtmi.Renderer(0) as r:
        rtmi.suzanne_cornell_box(r, 64, 64)
        r.render(64, 64, 32, 3, lanes_per_pixel=0, frames_in_flight=True)
        assert r.stats()["lanes_per_pixel"] == 32 and r.stats()["substreams_per_item"] == 1
    # pathTrace takes one sub-stream per item even when the flag asks for groups: its queue must
    # still hand out every item (the item count is taken after the group size is reset)
    with rtmi.Renderer(0) as r:
        rtmi.materialball(r, 24, 16)
        img = r.render(24, 16, 64, 5, lanes_per_pixel=0, integrator="pathTrace", frames_in_flight=True)
        st = r.stats()
        assert st["substreams_per_item"] == 1
        assert np.array_equal(img, r.render(24, 16, 64, 5, lanes_per_pixel=0, integrator="pathTrace"))
        assert st["segments"] == r.stats()["segments"]


def test_auto_lane_layout_bvh(rtmi):
    # launches that traverse BVHs: largest power of two S <= min(128, spp) with
    # pixels * S <= 2^27 (rt_kernel.h choose_layout)
    with rtmi.Renderer(0) as r:
        rtmi.suzanne_cornell_box(r, 64, 64)
        r.render(64, 64, 256, 3, lanes_per_pixel=0)
        assert r.stats()["lanes_per_pixel"] == 128
        r.render(64, 64, 32, 3, lanes_per_pixel=0)
        assert r.stats()["lanes_per_pixel"] == 32
    with rtmi.Renderer(0) as r:
        rtmi.materialball(r, 48, 32)
        r.render(48, 32, 64, 5, lanes_per_pixel=0, integrator="pathTrace")
        assert r.stats()["lanes_per_pixel"] == 64


def test_auto_layout_within_north_star_tolerance_of_sequential_sum(rtmi):
    # the bench's auto layout sums samples in S sub-streams: bit-exact against the
    # oracle with the same S, and within 1e-4 of the reference's sequential sum
    w, h, spp, depth = 48, 40, 64, 6
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        img = r.render(w, h, spp, depth, lanes_per_pixel=0)
        lanes = r.stats()["lanes_per_pixel"]
    assert lanes == 32
    sc = _oracle_yaml("cornellbox1.yaml", w, h)
    same_s, _ = sc.render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert np.array_equal(img, same_s)
    seq, _ = sc.render(w, h, spp, depth)
    assert np.max(np.abs(img - seq)) <= 1e-4


@pytest.mark.parametrize("name,w,h,spp", [("bunny_small_cornellbox.yaml", 48, 48, 4),
                                          ("bunny_cornellbox.yaml", 20, 20, 1)])
def test_bvh_mesh_parity(rtmi, name, w, h, spp):
    """Meshes above 64 triangles are traversed through the reference's SAH BVH;
    the result must equal the reference's brute-force TriangleMesh scan (the
    restatement tests every triangle) bit for bit."""
    depth = 6
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, os.path.join(S.SCENES, name), w, h)
        assert r.object_counts()["bvh_node"] > 0
        img = r.render(w, h, spp, depth)
        st = r.stats()
    assert st["overflow"] == 0 and st["node_visits"] > 0
    ref, ref_st = _oracle_yaml(name, w, h).render(w, h, spp, depth)
    _check(img, ref, st, ref_st, name)
    assert np.array_equal(img, ref)


def test_random_spheres_parity(rtmi):
    """BASELINE config 3 scene (488 spheres behind the object BVH, defocus
    blur, motion blur) against the restatement's sequential scan."""
    from oracle import oracle as orc

    w, h, spp, depth = 96, 54, 4, 10
    with rtmi.Renderer(0) as r:
        rtmi.random_spheres(r, w, h)
        assert r.object_counts()["bvh_node"] > 0
        img = r.render(w, h, spp, depth)
        st = r.stats()
    assert st["overflow"] == 0 and st["node_visits"] > 0
    ref, ref_st = orc.json_scene(os.path.join(S.SCENES, "random_spheres.json"), w, h).render(w, h, spp, depth)
    _check(img, ref, st, ref_st, "random_spheres")
    assert np.array_equal(img, ref)


@pytest.mark.parametrize("n_extra", [0, 20])
def test_exact_ties_follow_sequential_rule(rtmi, n_extra):
    """Coincident spheres (ties in t): with and without the object BVH the
    winner is the reference's (last sphere wins under the inclusive test)."""
    spec = S.duplicate_spheres_scene(n_extra)
    w, h, spp, depth = 48, 48, 2, 6
    with rtmi.Renderer(0) as r:
        S.build_product(r, spec)
        assert (r.object_counts()["bvh_node"] > 0) == (n_extra >= 16)
        img = r.render(w, h, spp, depth)
        st = r.stats()
    ref, ref_st = S.build_oracle(spec).render(w, h, spp, depth)
    _check(img, ref, st, ref_st, f"ties{n_extra}")
    assert np.array_equal(img, ref)


@pytest.mark.gpu
def test_render_u8_is_gamma_of_the_mean():
    # renderKernel's offline path: writePixel(index, color / spp) -> Canvas::gamma
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    w, h = 32, 24
    r = rtmi.Renderer(0)
    rtmi.cornell_box1(r, w, h)
    got = r.render_u8(w, h, 4, 4)
    r.close()
    sc = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox1.yaml"), S.MODELS, w, h)
    want, _ = sc.render(w, h, 4, 4, threads=8)
    assert np.array_equal(got, orc.gamma_u8(want))


@pytest.mark.gpu
def test_realtime_accumulation_matches_per_frame_sums():
    # GPU_REALTIME: 1 spp per frame, acc += color, display gamma(acc * (1.0f / n))
    import torch

    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    w, h, frames = 24, 16, 5
    r = rtmi.Renderer(0)
    rtmi.cornell_box1(r, w, h)
    acc = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
    pix = torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for n in range(frames):
        p = r.params(w, h, 1, 6, 1984, n)
        r.accumulate_device(p, acc.data_ptr(), n + 1, pix.data_ptr(), stream)
    torch.cuda.synchronize()
    r.close()
    sc = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox1.yaml"), S.MODELS, w, h)
    want = np.zeros((h, w, 3), np.float32)
    for n in range(frames):
        frame, _ = sc.render(w, h, 1, 6, sample_offset=n, threads=8)
        want = want + frame
    assert np.array_equal(acc.cpu().numpy(), want)
    scale = np.float32(1.0) / np.float32(frames)
    assert np.array_equal(pix.cpu().numpy(), orc.gamma_u8(want * scale))


@pytest.mark.parametrize("scene", ["cornellbox1", "random_spheres", "materialball"])
def test_work_queue_and_static_grid_agree(rtmi, scene):
    # the persistent work-queue launch (default) and the static grid
    # (RT_SCHEDULE_STATIC) compute the same partial sums per (pixel, sub-stream)
    w, h, spp, lanes = 40, 24, 8, 4
    imgs, variants = [], []
    for schedule in ("auto", "static"):
        with rtmi.Renderer(0) as r:
            if scene == "materialball":
                rtmi.materialball(r, w, h)
                imgs.append(r.render(w, h, spp, 5, lanes_per_pixel=lanes, integrator="pathTrace",
                                     schedule=schedule))
            else:
                getattr(rtmi, scene if scene != "cornellbox1" else "cornell_box1")(r, w, h)
                imgs.append(r.render(w, h, spp, 6, lanes_per_pixel=lanes, row_block=4, row_rank=1,
                                     row_world=3, schedule=schedule))
            variants.append(r.stats()["variant_name"])
    assert "<" in variants[0] and variants[0] != variants[1], variants
    assert np.array_equal(imgs[0], imgs[1])


def test_launches_on_two_streams_do_not_race(rtmi):
    # one context, two streams: the second launch waits for the first (they share
    # the context's work queue and partial-sum buffer)
    import torch

    w, h = 64, 48
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        want_a = r.render(w, h, 16, 6, seed=1)
        want_b = r.render(w, h, 16, 6, seed=2)
        a = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
        b = torch.empty_like(a)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        r.render_device(r.params(w, h, 16, 6, 1), a.data_ptr(), s1.cuda_stream)
        r.render_device(r.params(w, h, 16, 6, 2), b.data_ptr(), s2.cuda_stream)
        torch.cuda.synchronize()
    assert np.array_equal(a.cpu().numpy(), want_a)
    assert np.array_equal(b.cpu().numpy(), want_b)


def test_render_multi_assembles_the_frame(rtmi):
    # rt_render_multi over 3 contexts (all on device 0 here): row tiles rendered per
    # context, copied back and de-interleaved == the one-context frame
    w, h = 40, 37
    rs = [rtmi.Renderer(0) for _ in range(3)]
    for r in rs:
        rtmi.cornell_box1(r, w, h)
    try:
        multi = rtmi.render_multi(rs, w, h, 8, 5, row_block=4, lanes_per_pixel=4)
        one = rs[0].render(w, h, 8, 5, lanes_per_pixel=4)
    finally:
        for r in rs:
            r.close()
    assert np.array_equal(multi, one)


@pytest.mark.parametrize("spp,lanes,row_world", [(12, 4, 1), (16, 4, 3), (24, 8, 2)])
def test_tail_stealing_keeps_the_fold_order(rtmi, spp, lanes, row_world):
    # small frames exhaust the work queue at once, so most samples of the 3-4-sample
    # items are traced by lanes that stole them; the owners fold them in sample order:
    # bit-exact against the restatement with the same sub-streams
    w, h, depth = 36, 20, 7
    block, rank = 2, row_world - 1
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, w, h)
        img = r.render(w, h, spp, depth, lanes_per_pixel=lanes, row_block=block, row_rank=rank,
                       row_world=row_world)
        st = r.stats()
    from raytracingthenextweekcuda_amd import owned_row_ids

    ref, ref_st = _oracle_yaml("cornellbox1.yaml", w, h).render(w, h, spp, depth, lanes_per_pixel=lanes)
    rows = owned_row_ids(h, block, rank, row_world)
    assert np.array_equal(img, ref[rows])
    assert st["samples"] == len(rows) * w * spp


@pytest.mark.parametrize("schedule", ["auto", "static"])
def test_column_window_equals_full_frame_pixels(schedule):
    """rt_render_params.col_begin / col_count: a window of the owned rows, bit-identical to
    the full frame's pixels (work queue and static grid; rayColor with a BVH mesh scene and
    pathTrace), with the samples counted for the window only."""
    import raytracingthenextweekcuda_amd as rtmi

    W, H = 70, 33
    with rtmi.Renderer(0) as r:
        rtmi.bunny_cornell_box(r, W, H)
        full = r.render(W, H, 4, 6, lanes_per_pixel=4, schedule=schedule)
        win = r.render(W, H, 4, 6, lanes_per_pixel=4, row_block=3, row_rank=1, row_world=2,
                       col_begin=9, col_count=45, schedule=schedule)
        assert r.stats()["samples"] == rtmi.owned_rows(H, 3, 1, 2) * 45 * 4
        assert np.array_equal(win, full[rtmi.owned_row_ids(H, 3, 1, 2), 9:54])
    with rtmi.Renderer(0) as r:
        rtmi.materialball(r, W, H)
        full = r.render(W, H, 2, 5, lanes_per_pixel=2, integrator="pathTrace", schedule=schedule)
        win = r.render(W, H, 2, 5, lanes_per_pixel=2, integrator="pathTrace", col_begin=61, col_count=9,
                       schedule=schedule)
        assert np.array_equal(win, full[:, 61:70])
        with pytest.raises(rtmi.RTError):
            r.render(W, H, 2, 5, col_begin=62, col_count=9)  # past the right edge

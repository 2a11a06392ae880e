"""bench.py's frame overlap (two renderer contexts on two HIP streams taking alternate
frames): the frames it produces are the frames of the sequential loop, and the bench line
reports the same work with and without it."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n_ctx", [2, 3])
def test_row_sharded_frame_overlap_keeps_every_frame(n_ctx):
    import torch

    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd.distributed import RowShardedFrame

    w, h, spp, depth = 96, 64, 8, 6
    rs = [rtmi.Renderer(0) for _ in range(n_ctx)]
    for r in rs:
        rtmi.cornell_box1(r, w, h)
    streams = [torch.cuda.Stream() for _ in range(n_ctx)]
    fr = RowShardedFrame(w, h, 2, device=torch.device("cuda"), streams=streams)
    seeds = [11, 12, 13, 14, 15]
    got = []
    for k, seed in enumerate(seeds):
        p = rs[0].params(w, h, spp, depth, seed, 0, 1, 0, 1, 0, "rayColor")

        def render_into(tile, b, p=p):
            rs[b].render_device(p, tile.data_ptr(), streams[b].cuda_stream)

        fr.submit(render_into)
        out = fr.drain()
        torch.cuda.synchronize()
        got.append(out.cpu().numpy().copy())
    for r in rs:
        r.close()
    with rtmi.Renderer(0) as ref:
        rtmi.cornell_box1(ref, w, h)
        for seed, img in zip(seeds, got):
            want = ref.render(w, h, spp, depth, seed=seed, lanes_per_pixel=0)
            assert np.array_equal(img, want), seed


def _bench(*extra):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--width", "128", "--height", "96", "--spp", "16", *extra]
    out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240, check=True).stdout
    return json.loads(next(line for line in out.splitlines() if line.startswith("{")))


def test_bench_line_with_and_without_overlap():
    a = _bench()
    b = _bench("--no-overlap")
    c = _bench("--contexts", "2")
    assert a["roofline"]["overlap"] is True and b["roofline"]["overlap"] is False
    # auto: 3 contexts for this small frame (<= 2^25 samples per rank)
    assert (a["config"]["contexts"], b["config"]["contexts"], c["config"]["contexts"]) == (3, 1, 2)
    assert c["config"]["segments_per_frame"] == a["config"]["segments_per_frame"]
    assert a["config"]["segments_per_frame"] == b["config"]["segments_per_frame"]
    assert a["value"] > 0 and b["value"] > 0 and a["steps"] == 3
    # the work-queue schedule the line was measured with (rt_render_stats.refill / queue_blocks)
    assert a["config"]["refill"] in (4, 8) and a["config"]["queue_blocks"] > 0


def test_row_sharded_frame_overlap_two_ranks_rank0(monkeypatch):
    """The N > 1 pipeline with frame overlap, from rank 0 of a 2-rank world: the gather is
    emulated on the calling stream (rank 1's tiles rendered beforehand), so the test checks
    the stream and buffer ordering of submit/drain — every assembled frame must equal the
    full frame of its seed."""
    import torch
    import torch.distributed as dist

    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd.distributed import RowShardedFrame

    w, h, spp, depth, block = 96, 64, 8, 6, 2
    seeds = [21, 22, 23, 24, 25]
    with rtmi.Renderer(0) as r1:
        rtmi.cornell_box1(r1, w, h)
        rank1 = {s: torch.as_tensor(r1.render(w, h, spp, depth, seed=s, row_block=block, row_rank=1, row_world=2,
                                              lanes_per_pixel=0)).cuda() for s in seeds}
    current = {}

    class Work:
        def wait(self):
            pass

    def fake_gather(tile, gather_list=None, dst=0, group=None, async_op=False):
        gather_list[0].copy_(tile)  # on the current stream (the frame's render stream)
        t1 = rank1[current["seed"]]
        gather_list[1][: t1.shape[0]].copy_(t1)
        return Work()

    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda group=None: 2)
    monkeypatch.setattr(dist, "get_rank", lambda group=None: 0)
    monkeypatch.setattr(dist, "gather", fake_gather)
    rs = [rtmi.Renderer(0), rtmi.Renderer(0)]
    for r in rs:
        rtmi.cornell_box1(r, w, h)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    fr = RowShardedFrame(w, h, block, device=torch.device("cuda"), pipeline=True, streams=streams)
    got = {}
    for k, seed in enumerate(seeds):
        p = rs[0].params(w, h, spp, depth, seed, 0, block, 0, 2, 0, "rayColor")

        def render_into(tile, b, p=p):
            rs[b].render_device(p, tile.data_ptr(), streams[b].cuda_stream)

        current["seed"] = seed
        fr.submit(render_into)
        if k % 2 == 1:  # drain every other frame: both the pipelined and the drained path
            out = fr.drain()
            torch.cuda.synchronize()
            got[seed] = out.cpu().numpy().copy()
    out = fr.drain()
    torch.cuda.synchronize()
    got[seeds[-1]] = out.cpu().numpy().copy()
    for r in rs:
        r.close()
    with rtmi.Renderer(0) as ref:
        rtmi.cornell_box1(ref, w, h)
        for seed, img in got.items():
            assert np.array_equal(img, ref.render(w, h, spp, depth, seed=seed, lanes_per_pixel=0)), seed

"""Row-tile sharding + gather (raytracingthenextweekcuda_amd/distributed.py)
on CPU with the gloo backend, world sizes 2 and 3. Each rank's render is a
synthetic tile whose values encode (global row, column, channel), so the
assembled frame checks the collective and the de-interleaving exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raytracingthenextweekcuda_amd import owned_row_ids
from raytracingthenextweekcuda_amd.distributed import RowShardedFrame, tile_rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _expected(h, w):
    y, x, c = np.meshgrid(np.arange(h), np.arange(w), np.arange(3), indexing="ij")
    return (y * 1000 + x * 10 + c).astype(np.float32)


def _worker(rank, world, port, h, w, block, q, pipeline=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fr = RowShardedFrame(w, h, block, pipeline=pipeline)
        ids = owned_row_ids(h, block, rank, world)
        frame_no = [0]

        def render_into(tile):
            # frame f's values are offset by f, so a frame assembled from another
            # frame's (or a stale) tile is caught
            tile.zero_()
            tile[: len(ids)] = torch.from_numpy(_expected(h, w)[ids] + frame_no[0])
            frame_no[0] += 1

        if pipeline:
            for _ in range(3):  # double-buffered tiles reused across frames
                fr.submit(render_into)
            out = fr.drain()
        else:
            for _ in range(3):  # the buffers are reused frame after frame
                out = fr.render(render_into)
        if rank == 0:
            q.put(out.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h,w,block,pipeline", [(2, 16, 5, 4, False), (3, 37, 4, 5, False),
                                                      (2, 7, 3, 8, False), (2, 16, 5, 2, True),
                                                      (3, 37, 4, 5, True)])
def test_gather_reassembles_frame(world, h, w, block, pipeline):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, h, w, block, q, pipeline))
             for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(frame, _expected(h, w) + 2)  # the last of three frames


def test_tiles_partition_rows():
    for world in (1, 2, 4, 8):
        for h in (1, 7, 512, 513):
            rows = np.concatenate(tile_rows(h, 8, world))
            assert np.array_equal(np.sort(rows), np.arange(h))

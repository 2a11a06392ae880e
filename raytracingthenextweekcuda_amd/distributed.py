"""Multi-GPU frame sharding: interleaved pixel-row tiles + one gather.

The reference renders on one GPU (cudaSetDevice(0), main.cu:556). Here one
process drives one GPU (torch.distributed, backend "nccl" = RCCL over xGMI):

  * rows are dealt round-robin in blocks of `row_block` rows — block k goes to
    rank k % world — which balances the uneven cost of rows (light, glass);
  * every rank renders its rows straight into an HBM buffer (rt_render_device);
  * one gather moves the tiles to rank 0 (no all-reduce: each pixel has exactly
    one owner, so there is nothing to sum), and rank 0 scatters the tile rows
    back to frame order.

The RNG stream is keyed by the global pixel index, so the assembled frame is
bit-identical for any world size (tests/test_gpu_parity.py row-tiling test).
The collective and assembly logic is device-agnostic and is covered on CPU
with the gloo backend (tests/test_distributed.py).
"""
from __future__ import annotations

import os
from typing import Callable, Optional

from .renderer import owned_row_ids, owned_rows


def tile_rows(height: int, row_block: int, world: int) -> list:
    """Global row ids owned by each rank, in the order the rank stores them."""
    return [owned_row_ids(height, row_block, k, world) for k in range(world)]


def max_tile_rows(height: int, row_block: int, world: int) -> int:
    return max(owned_rows(height, row_block, k, world) for k in range(world))


class RowShardedFrame:
    """Per-rank state for rendering frames sharded by row tiles.

    render_into(tile) must write this rank's owned rows (rows x W x 3 float32,
    increasing global y) into the first rows of `tile`, a (max_rows, W, 3)
    tensor on this rank's device. gather() returns the full (H, W, 3) frame on
    rank 0 and None elsewhere.
    """

    def __init__(self, width: int, height: int, row_block: int, group=None, device=None,
                 pipeline: bool = False, streams=None):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.torch = torch
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.width, self.height, self.row_block = width, height, row_block
        self.rows = owned_rows(height, row_block, self.rank, self.world)
        self.max_rows = max_tile_rows(height, row_block, self.world)
        self.device = device if device is not None else torch.device("cpu")
        self.frame = None
        self.gather_list = None
        self.src_rows = None
        self.pending = None  # (async gather work, landing block index) of the last submitted frame
        self.n_submitted = 0
        # Frame overlap (streams = n >= 2 torch.cuda.Streams): consecutive frames rotate over
        # n buffers AND n streams, so frame k+1's render runs while frame k's launch drains
        # its last work items (a persistent launch's tail leaves SIMDs idle); render_into(tile,
        # b) must then launch on streams[b]. Without streams every frame runs on the current
        # stream.
        self.streams = streams
        self.nbuf = len(streams) if streams else (2 if pipeline else 1)
        if self.world == 1:
            # one rank owns every row in order: render straight into the frame
            self.frame = torch.zeros((height, width, 3), dtype=torch.float32, device=self.device)
            self.tile = self.frame
            self.frames = [self.frame] + [torch.zeros_like(self.frame) for _ in range(self.nbuf - 1 if streams else 0)]
            return
        if streams and not pipeline:
            raise ValueError("frame overlap (streams) needs pipeline=True")
        self.tile = torch.zeros((self.max_rows, width, 3), dtype=torch.float32, device=self.device)
        # pipelined frames (submit/drain): nbuf tile buffers (and landing blocks on rank 0),
        # so frame k's gather overlaps frame k+1's render
        self.pipeline = pipeline
        self.tiles = [self.tile] + [torch.zeros_like(self.tile) for _ in range(self.nbuf - 1)]
        if self.rank == 0:
            self.frame = torch.zeros((height, width, 3), dtype=torch.float32, device=self.device)
            self.frames = [self.frame] + [torch.zeros_like(self.frame) for _ in range(self.nbuf - 1 if streams else 0)]
            # the gather lands in one (world * max_rows) block; frame row y is
            # block row rank(y) * max_rows + (its position in that rank's tile)
            self.gathered = torch.empty((self.world * self.max_rows, width, 3), dtype=torch.float32,
                                        device=self.device)
            self.gather_list = list(self.gathered.view(self.world, self.max_rows, width, 3).unbind(0))
            self.landing = [(self.gathered, self.gather_list)]
            for _ in range(self.nbuf - 1):
                g2 = torch.empty_like(self.gathered)
                self.landing.append((g2, list(g2.view(self.world, self.max_rows, width, 3).unbind(0))))
            src = [0] * height
            for k, ids in enumerate(tile_rows(height, row_block, self.world)):
                for j, y in enumerate(ids):
                    src[int(y)] = k * self.max_rows + j
            self.src_rows = torch.as_tensor(src, dtype=torch.long, device=self.device)

    def gather(self, events=None) -> Optional["object"]:
        """One gather of every rank's tile to rank 0, then one row permutation. `events`
        (start, end) torch.cuda.Events are recorded on the current stream around the
        collective alone (the stream is ordered after the gather once it returns)."""
        if self.world == 1:
            return self.frame
        if events:
            events[0].record()
        self.dist.gather(self.tile, self.gather_list if self.rank == 0 else None, dst=0,
                         group=self.group)
        if events:
            events[1].record()
        if self.rank != 0:
            return None
        self.torch.index_select(self.gathered, 0, self.src_rows, out=self.frame)
        return self.frame

    def render(self, render_into: Callable[["object"], None]):
        render_into(self.tile)
        return self.gather()

    # ---- pipelined frames ----
    def _on(self, b):
        """Context that makes buffer b's stream current (a no-op without frame overlap)."""
        import contextlib

        return self.torch.cuda.stream(self.streams[b]) if self.streams else contextlib.nullcontext()

    def _finish_pending(self):
        work, b = self.pending
        self.pending = None
        with self._on(b):
            # this stream waits for the gather (the host does not, on NCCL): the assembly and
            # the next render into tile b come after it
            work.wait()
            if self.rank == 0:
                self.frame = self.frames[b] if self.streams else self.frame
                self.torch.index_select(self.landing[b][0], 0, self.src_rows, out=self.frame)

    def submit(self, render_into: Callable[..., None]):
        """Render the next frame into the free tile buffer and start its gather without
        waiting for it; the previous frame's gather (which ran under this render) is
        completed and assembled on rank 0 after this frame's render is enqueued. With
        frame overlap, render_into(tile, b) is called and must launch on streams[b]."""
        b = self.n_submitted % self.nbuf
        self.n_submitted += 1
        if self.world == 1:
            if self.streams:
                self.frame = self.frames[b]
                render_into(self.frame, b)
            else:
                render_into(self.frame)
            return
        if not self.pipeline:
            raise RuntimeError("RowShardedFrame(pipeline=True) is required for submit()")
        tile = self.tiles[b]
        if self.streams:
            render_into(tile, b)  # on streams[b], which waited for the last gather out of tile b
        else:
            render_into(tile)  # enqueued before waiting on the previous gather
        if self.pending is not None:
            self._finish_pending()
        with self._on(b):  # the NCCL stream waits for this frame's render stream
            work = self.dist.gather(tile, self.landing[b][1] if self.rank == 0 else None, dst=0,
                                    group=self.group, async_op=True)
        self.pending = (work, b)

    def drain(self) -> Optional["object"]:
        """Complete the last submitted frame; returns it on rank 0 (None elsewhere).

        With frame overlap the frame was rendered (world 1) or assembled (rank 0) on
        streams[b]: the caller's current stream is made to wait for that stream, so work the
        caller enqueues on it reads the finished frame. The frame buffer is reused by the
        nbuf-th next submit()."""
        if self.pending is not None:
            self._finish_pending()
        if self.streams and self.n_submitted:
            self.torch.cuda.current_stream().wait_stream(self.streams[(self.n_submitted - 1) % self.nbuf])
        return self.frame if self.rank == 0 else None


class RcclRowFrames:
    """N > 1 frames through the C ABI, the exchange bench.py times.

    Every rank renders its row tiles with rt_render_device on context b's own stream, and the
    SAME stream then carries that frame's rt_gather_rows: one ncclGather of the tiles to rank 0
    plus the root's de-interleave kernel (include/rtmi.h). No collective stream
    exists besides the render streams, so a rank's streams are its render streams and the
    default stream (which the timed loop leaves idle): three contexts fit the process's four
    hardware queues (GPU_MAX_HW_QUEUES). torch.distributed (gloo) carries only the control plane:
    the RCCL unique id, barriers and the per-rank stats.

    Frame b of a rotation lands in context b's staging buffer and in frames[b] on rank 0; the
    tile and frame of context b are reused by frame b + n, which its stream orders after this
    frame's gather. `comm_world` 1 with `world` > 1 is the one-GPU rehearsal of a shard
    (bench.py --rehearse-shard): rank 0's rows of a `world`-rank frame, gathered by a one-rank
    communicator (the same kernels and streams; only the landing is this rank's tile).
    """

    def __init__(self, renderers, width, height, row_block, rank, world, streams, device,
                 comm_world=None, group=None):
        import ctypes as C

        import torch
        import torch.distributed as dist

        from . import _lib

        self.C, self.torch, self.L = C, torch, _lib.lib()
        self.renderers, self.streams = renderers, streams
        self.width, self.height, self.row_block = width, height, row_block
        self.rank, self.world = rank, world
        self.comm_world = world if comm_world is None else comm_world
        self.max_rows = max_tile_rows(height, row_block, world)
        idb = (C.c_uint8 * 128)()
        if self.comm_world > 1:
            ids = torch.zeros(128, dtype=torch.uint8)
            if dist.get_rank(group) == 0:
                r0 = self.L.rt_comm_unique_id(idb)
                if r0 != 0:
                    raise RuntimeError(f"rt_comm_unique_id failed ({r0})")
                ids.copy_(torch.frombuffer(bytearray(bytes(idb)), dtype=torch.uint8))
            dist.broadcast(ids, src=0, group=group)
            C.memmove(idb, bytes(ids.numpy().tobytes()), 128)
        elif self.L.rt_comm_unique_id(idb) != 0:
            raise RuntimeError("rt_comm_unique_id failed")
        self.comm = C.c_void_p()
        renderers[0]._check(self.L.rt_comm_init(renderers[0].ctx, idb, self.comm_world,
                                                 rank if self.comm_world > 1 else 0, C.byref(self.comm)))
        n = len(renderers)
        self.tiles = [torch.zeros((self.max_rows, width, 3), dtype=torch.float32, device=device) for _ in range(n)]
        self.tile = self.tiles[0]
        # the root's frames (the rehearsal lands its one tile: a frame of max_rows rows)
        fh = height if self.comm_world > 1 else self.max_rows
        self.frames = ([torch.zeros((fh, width, 3), dtype=torch.float32, device=device) for _ in range(n)]
                       if rank == 0 else None)
        self.frame = self.frames[0] if self.frames else None
        # the gather's frame geometry: the real frame, or in the rehearsal the tile itself as a
        # one-rank frame (identity de-interleave)
        from .renderer import Renderer

        if self.comm_world > 1:
            self.gparams = Renderer.params(width, height, 1, 1, row_block=row_block, row_rank=rank, row_world=world)
        else:
            self.gparams = Renderer.params(width, self.max_rows, 1, 1, row_block=self.max_rows)
        self.n_submitted = 0
        # the previous frame's gather (an event on its stream): each gather waits for it, so the
        # communicator's collectives run in issue order - the same order on every rank - even though
        # they are enqueued on different streams (no reliance on RCCL ordering one communicator's
        # operations across streams)
        self.gather_done = None
        self.order_gathers = os.environ.get("RTMI_GATHER_ORDER", "1") != "0"  # 0: A/B only

    def _gather(self, b, stream_ptr):
        C = self.C
        fr = self.frames[b].data_ptr() if self.frames else None
        r = self.renderers[b]
        g_rank = self.rank if self.comm_world > 1 else 0
        r._check(self.L.rt_gather_rows(r.ctx, self.comm, C.byref(self.gparams), g_rank, self.comm_world,
                                       C.c_void_p(self.tiles[b].data_ptr()), C.c_void_p(fr), C.c_void_p(stream_ptr)))

    def submit(self, render_into: Callable[..., None]):
        """render_into(tile, b) enqueues this rank's rows on streams[b]; the frame's gather follows
        on the same stream."""
        b = self.n_submitted % len(self.renderers)
        self.n_submitted += 1
        render_into(self.tiles[b], b)
        if self.gather_done is not None:
            self.streams[b].wait_event(self.gather_done)
        self._gather(b, self.streams[b].cuda_stream)
        if self.order_gathers:
            self.gather_done = self.torch.cuda.Event()
            self.gather_done.record(self.streams[b])
        if self.frames:
            self.frame = self.frames[b]

    def drain(self):
        """The caller's current stream waits for the last submitted frame (gather included)."""
        if self.n_submitted:
            self.torch.cuda.current_stream().wait_stream(self.streams[(self.n_submitted - 1) % len(self.renderers)])
        return self.frame if self.rank == 0 else None

    def gather(self, events=None):
        """Gathers context 0's tile on the current stream (the isolated frames after the timed
        region); `events` (start, end) are recorded around the collective alone."""
        s = self.torch.cuda.current_stream()
        if self.gather_done is not None:
            s.wait_event(self.gather_done)
        if events:
            events[0].record(s)
        self._gather(0, s.cuda_stream)
        if events:
            events[1].record(s)
        if self.order_gathers:
            self.gather_done = self.torch.cuda.Event()
            self.gather_done.record(s)
        if self.frames:
            self.frame = self.frames[0]
        return self.frame if self.rank == 0 else None

    def close(self):
        if self.comm:
            self.L.rt_comm_destroy(self.comm)
            self.comm = None


def render_params_for_rank(renderer, width, height, spp, depth, row_block, rank, world, seed=1984,
                           sample_offset=0, lanes_per_pixel=0):
    """rt_render_params for this rank's share of the frame."""
    return renderer.params(width, height, spp, depth, seed, sample_offset, row_block, rank, world,
                           lanes_per_pixel)

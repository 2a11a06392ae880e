"""Multi-GPU frames through the C ABI (SURVEY §8(b) "Threading", §8(e)): rt_render_multi's
row tiles + ONE ncclGather + the device row de-interleave, rt_gather_rows for one process
per GPU, and rt_assemble_rows against the host's row placement.

On the one-GPU test box, RCCL runs with one rank (n = 1: ncclCommInitAll / a world-1
communicator); n > 1 contexts share the device there, which RCCL refuses, so they take the
device-copy exchange (RT_GATHER_COPY) into the same de-interleave kernel. The N > 1
collective itself is covered by the gloo tests (tests/test_distributed.py) until an
8-GPU node runs bench.py --gpus 8."""
import ctypes as C
import os

import numpy as np
import pytest

import raytracingthenextweekcuda_amd as rtmi
from raytracingthenextweekcuda_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_row_ownership_helpers_match_python():
    L = _lib.lib()
    for h, b, w in [(512, 2, 8), (720, 8, 3), (7, 4, 5), (2050, 2, 2), (1, 1, 4)]:
        rows = [L.rt_owned_rows(h, b, k, w) for k in range(w)]
        assert rows == [rtmi.owned_rows(h, b, k, w) for k in range(w)]
        assert sum(rows) == h
        assert L.rt_max_tile_rows(h, b, w) == max(rows)
    assert L.rt_owned_rows(10, 0, 0, 1) == -1 and L.rt_max_tile_rows(10, 1, 0) == -1


def test_comm_entry_points_reject_bad_arguments_without_a_gpu():
    L = _lib.lib()
    r = rtmi.Renderer(-1)
    comm = C.c_void_p()
    idb = (C.c_uint8 * 128)()
    assert L.rt_comm_init(r.ctx, idb, 1, 0, C.byref(comm)) == 6  # RT_ERR_NODEV: no device
    assert L.rt_comm_init(None, idb, 1, 0, C.byref(comm)) == 1
    p = rtmi.Renderer.params(64, 64, 1, 1)
    assert L.rt_gather_rows(r.ctx, None, C.byref(p), 0, 1, None, None, None) == 1
    assert L.rt_assemble_rows(r.ctx, C.byref(p), 1, None, None, None) == 6
    assert L.rt_comm_destroy(None) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3])
def test_render_multi_equals_single_render(n):
    W, H, spp, depth = 96, 80, 8, 8
    rs = [rtmi.Renderer(0) for _ in range(n)]
    try:
        for r in rs:
            rtmi.cornell_box1(r, W, H)
        ref = rs[0].render(W, H, spp, depth, lanes_per_pixel=0)
        out = rtmi.render_multi(rs, W, H, spp, depth, row_block=4, lanes_per_pixel=0)
        assert np.array_equal(out, ref)
        # n = 1 is one RCCL rank; n > 1 contexts share the box's one device
        assert rs[0].stats()["gather"] == (rtmi.GATHER_RCCL if n == 1 else rtmi.GATHER_COPY)
    finally:
        for r in rs:
            r.close()


@pytest.mark.gpu
def test_sub_stream_count_is_chosen_from_the_full_frame():
    """at 2048^2 the 2^25-item cap binds (S = 8 for the frame); every rank must
    fold with the frame's S, not its own shard's, so the frame is N-independent."""
    W = H = 2048
    spp, depth = 64, 4
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, W, H)
        full = r.render(W, H, spp, depth, lanes_per_pixel=0)
        s_full = r.stats()["lanes_per_pixel"]
        assert s_full == 8
        for world in (2, 8):
            frame = np.zeros_like(full)
            for k in range(world):
                part = r.render(W, H, spp, depth, row_block=2, row_rank=k, row_world=world, lanes_per_pixel=0)
                assert r.stats()["lanes_per_pixel"] == s_full
                frame[rtmi.owned_row_ids(H, 2, k, world)] = part
            assert np.array_equal(frame, full), world


@pytest.mark.gpu
def test_assemble_rows_kernel_matches_host_placement():
    import torch

    W, H, rb, world = 37, 29, 3, 4  # ragged: 37 * 3 floats per row is not a multiple of 4
    L = _lib.lib()
    max_rows = L.rt_max_tile_rows(H, rb, world)
    rng = np.random.default_rng(7)
    staging = rng.standard_normal((world, max_rows, W, 3)).astype(np.float32)
    expect = np.zeros((H, W, 3), np.float32)
    for k in range(world):
        ids = rtmi.owned_row_ids(H, rb, k, world)
        expect[ids] = staging[k, : len(ids)]
    with rtmi.Renderer(0) as r:
        st = torch.from_numpy(staging).cuda()
        fr = torch.full((H, W, 3), -1.0, device="cuda")
        p = rtmi.Renderer.params(W, H, 1, 1, row_block=rb)
        r.assemble_rows_device(p, world, st.data_ptr(), fr.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(fr.cpu().numpy(), expect)


@pytest.mark.gpu
def test_gather_rows_with_a_one_rank_communicator():
    """The one-process-per-GPU entry point: unique id -> communicator -> render this rank's
    tile with rt_render_device -> rt_gather_rows (ncclGather + de-interleave on the root)."""
    import torch

    W, H, spp, depth, rb = 64, 48, 4, 8, 2
    L = _lib.lib()
    with rtmi.Renderer(0) as r:
        rtmi.cornell_box1(r, W, H)
        ref = r.render(W, H, spp, depth, row_block=rb, lanes_per_pixel=0)
        idb = (C.c_uint8 * 128)()
        assert L.rt_comm_unique_id(idb) == 0
        comm = C.c_void_p()
        r._check(L.rt_comm_init(r.ctx, idb, 1, 0, C.byref(comm)))
        try:
            stream = torch.cuda.current_stream().cuda_stream
            p = r.params(W, H, spp, depth, row_block=rb, row_rank=0, row_world=1, lanes_per_pixel=0)
            tile = torch.zeros((L.rt_max_tile_rows(H, rb, 1), W, 3), device="cuda")
            frame = torch.zeros((H, W, 3), device="cuda")
            r.render_device(p, tile.data_ptr(), stream)
            r._check(L.rt_gather_rows(r.ctx, comm, C.byref(p), 0, 1, C.c_void_p(tile.data_ptr()),
                                      C.c_void_p(frame.data_ptr()), C.c_void_p(stream)))
            torch.cuda.synchronize()
            assert np.array_equal(frame.cpu().numpy(), ref)
        finally:
            assert L.rt_comm_destroy(comm) == 0


@pytest.mark.gpu
def test_cpp_one_process_per_gpu_example():
    """examples/multigpu: the C++ host runs SURVEY §8(e) without Python - rt_render_multi
    over the visible devices, then N forked processes (one per GPU, N = 1 on the test box)
    that render their tiles and meet in rt_gather_rows; both frames must equal one render."""
    import subprocess

    exe = os.path.join(REPO, "examples", "multigpu")
    assert os.path.exists(exe), "examples/multigpu is not built (run __graft_entry__.build())"
    out = subprocess.run([exe, "96", "64", "4"], capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "render_multi ok" in out.stdout and "gather_rows ok" in out.stdout, out.stdout

"""Benchmark: Mrays/s and ms/frame for the Cornell Box (CornellBox1 scene) at
512x512, 128 spp, depth 8 (BASELINE.json configs[1]) on N MI355X GPUs.

One step = one full frame: every rank renders its interleaved pixel-row tiles
with the HIP megakernel (librtmi.so) straight into an HBM buffer, then the
tiles are gathered to rank 0 with one RCCL gather over xGMI (N > 1), which
overlaps the next frame's render (one tile buffer per context); the timed region ends
after the last frame is assembled on rank 0. The frame work is fixed as N grows
(strong scaling). Consecutive frames rotate over --contexts renderer contexts on as
many HIP streams (3 for rayColor frames of up to 2^25 samples per rank, else 2), so a frame's launch
overlaps the tail of the previous one
(--no-overlap: one context, one stream, for per-launch measurements).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 is launched by torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mrays/sec + ms/frame, Cornell Box 512×512 spp=128, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# VALU issue peak (MI355X_MICROARCH.md, cycle constants: a wave64 v_fma_f32 takes 2 cycles of
# its SIMD): 4 SIMDs per CU x 2.4 GHz / 2 = 4.8 G wave-instructions/s per CU, 1,228.8 G/s for
# 256 CUs (x 64 lanes x 2 = the 157.3 TFLOP/s FP32 vector spec). Calibrated against a kernel of
# known VALU count in profiles/r02/valu_probe.json (tools/valu_probe.hip).
VALU_GINST_PER_CU = 4 * 2.4 / 2

# Algorithmic bytes per record touched: plane 40 B, sphere
# 20 B, moving sphere 36 B, mesh AABB 24 B, triangle (v0,E1,E2) 36 B, BVH node
# 32 B, and 12 B per output pixel.
BYTES = {"plane": 40, "sphere": 20, "moving_sphere": 36, "box": 24, "tri": 36, "node": 32, "pixel": 12,
         # pathTrace: triangle-list entry 4 B + Kuchkuda planes (n,d,e1,d1,e2,d2,e3,d3) 64 B
         "ktri": 68}


# BASELINE.json configs: scene loader, default W, H, spp, depth.
SCENES = {
    "cornellbox1": ("cornell_box1", 512, 512, 128, 8, "CornellBox1 (6 planes + 2 cube_small.obj meshes, 24 triangles)"),
    "spheres": ("random_spheres", 1280, 720, 256, 10, "RTNW final scene (488 spheres, 388 moving; object BVH)"),
    "bunny": ("bunny_cornell_box", 1024, 1024, 512, 8, "bun_zipper.ply (69,451 triangles, SAH BVH) in CornellBox1 walls"),
    "media": ("cornell_box_media", 2048, 2048, 1024, 16, "CornellBox1 walls + 2 constant-medium boxes + glass sphere (media: build extension)"),
    # Suzanne box: the geometry of the image behind the reference's only published timing
    # (images.MD:44-53); its radiance does not match that image; not a BASELINE config
    "suzanne": ("suzanne_cornell_box", 512, 512, 32, 10, "cornellbox3.yaml (suzanne_small.obj, 968 triangles) + metal and glass spheres (geometry of the images.MD timing image; radiance differs)"),
    # the reference's committed renderKernel configuration (pathTrace, main.cu:187;
    # samplesPerPixel 32, 5 bounces); not a BASELINE config, reported separately
    "materialball": ("materialball", 512, 512, 32, 5, "materialball.ply (46,816 triangles, COAT) + 6 spheres, pathTrace integrator"),
}
INTEGRATOR = {"materialball": "pathTrace"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default="cornellbox1", choices=sorted(SCENES),
                    help="BASELINE config: cornellbox1 (2), spheres (3), bunny (4), media (5); materialball = "
                         "the reference's committed pathTrace setup; the metric line is config 2")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--row-block", type=int, default=2,
                    help="rows per round-robin block (2: per-rank shard times within 1.1%% at N=8, tools/shard_balance.py)")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per pixel (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--contexts", type=int, default=0,
                    help="frame overlap: renderer contexts / HIP streams that consecutive frames rotate over; "
                         "0 = auto: 3 when a rank's rayColor frame is at most 2^25 samples, else 2 "
                         "(tools/ctx_probe.sh, tools/layout_probe.sh: CB1 N = 8 shard 1.00 / 0.887 / 0.842 / "
                         "0.879 ms/frame with 1 / 2 / 3 / 4 contexts, N = 1 5.88 -> 5.82 from 2 to 3; the 300 ms "
                         "bunny frame 2.5 %% and the pathTrace materialball frame 2 %% slower with 3)")
    ap.add_argument("--in-flight-layout", action="store_true",
                    help="use the frames-in-flight layout even without overlap (profiling passes of the timed layout)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="one context and stream: consecutive frames do not overlap (per-launch roofline)")
    ap.add_argument("--cpu-spp", type=int, default=None)
    ap.add_argument("--exchange", choices=("abi", "torch"), default="abi",
                    help="N > 1 row-tile exchange: abi = the library's rt_gather_rows (one ncclGather + the root's "
                         "de-interleave) on each frame's render stream, gloo for the control plane; torch = "
                         "torch.distributed.gather over ProcessGroupNCCL (its own stream: at most 2 contexts)")
    ap.add_argument("--rehearse-shard", type=int, default=0, metavar="N",
                    help="one GPU, one process: render rank 0's rows of an N-rank frame with the N > 1 stream layout "
                         "and exchange (a one-rank RCCL communicator gathers the tile on the render stream)")
    ap.add_argument("--line-selftest", action="store_true",
                    help="CPU only: synthetic per-rank numbers through the N > 1 collectives and the JSON line")
    a = ap.parse_args()
    _, w, h, spp, depth, _ = SCENES[a.scene]
    a.width = a.width or w
    a.height = a.height or h
    a.spp = a.spp or spp
    a.depth = a.depth or depth
    # CPU-baseline sample (a bounded slice of the same workload, ~10-40 CPU-seconds
    # on 16 threads; CornellBox1 and materialball run their whole frame): the
    # restatement scans meshes brute force like the reference's TriangleMesh::hit,
    # so the bunny sample is a 1/8-scale frame at 1 spp.
    a.cpu_div, cpu_spp = {"cornellbox1": (1, 128), "spheres": (2, 16), "bunny": (8, 1),
                          "materialball": (1, 32), "media": (4, 64), "suzanne": (2, 8)}[a.scene]
    a.cpu_spp = a.cpu_spp or cpu_spp
    return a


def object_bytes_per_segment(r) -> int:
    """Bytes of the non-mesh object records every segment scans."""
    import raytracingthenextweekcuda_amd.scene  # noqa: F401

    counts = r.object_counts()
    if counts["grouped_spheres"]:  # spheres behind the object BVH are counted per test
        return counts["plane"] * BYTES["plane"]
    return counts["plane"] * BYTES["plane"] + counts["sphere"] * BYTES["sphere"] + \
        counts["moving_sphere"] * BYTES["moving_sphere"]


def host_threads() -> int:
    """The CPUs this job may use (all cores). On the GPU box the process
    sees every CPU of the machine, but its share is OMP_NUM_THREADS (16 per GPU), which
    the harness sets; the affinity mask bounds it elsewhere."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(args, threads: int):
    """The CPU restatement (oracle/, a port of the reference's integrator) on a
    bounded sample of the same workload: one warm-up, then the
    median of 5 runs on `threads` threads, plus one single-thread run on 1/8 of the
    sample's samples."""
    from oracle import oracle as orc

    scenes = os.path.join(REPO, "assets", "scenes")
    models = os.path.join(REPO, "assets", "models")
    w, h = args.width // args.cpu_div, args.height // args.cpu_div
    if args.scene == "materialball":
        # pathTrace: the restatement traverses the reference's own `.bvh` cache
        # (tests/golden) as BVH_IntersectTriangles does (full DFS, no pruning).
        cam = orc.yaml_scene(os.path.join(scenes, "cornellbox2.yaml"), models, w, h)
        pt = orc.OraclePathTrace()
        pt.load_object(os.path.join(models, "materialball", "materialball.ply"), "COAT")
        pt.process((0.1, 0.0, -1.0))
        with open(os.path.join(REPO, "tests", "golden", "bvh", "materialball.ply.bvh"), "rb") as fh:
            pt.set_bvh(fh.read())

        def run(spp, nthreads):
            return pt.render(cam, w, h, spp, args.depth, threads=nthreads)[1]
    else:
        if args.scene == "spheres":
            sc = orc.json_scene(os.path.join(scenes, "random_spheres.json"), w, h)
        else:
            name = {"cornellbox1": "cornellbox1.yaml", "bunny": "bunny_cornellbox.yaml",
                    "media": "cornellbox_media.yaml", "suzanne": "suzanne_cornellbox.yaml"}[args.scene]
            sc = orc.yaml_scene(os.path.join(scenes, name), models, w, h)

        def run(spp, nthreads):
            return sc.render(w, h, spp, args.depth, threads=nthreads)[1]

    run(max(1, args.cpu_spp // 4), threads)  # warm-up (OpenMP pool, page-in, caches)
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        st = run(args.cpu_spp, threads)
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[2]
    spp1 = max(1, args.cpu_spp // 8)
    t0 = time.perf_counter()
    st1 = run(spp1, 1)
    dt1 = time.perf_counter() - t0
    frame_ms = dt * 1e3 * (args.width * args.height * args.spp) / (w * h * args.cpu_spp)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": st["segments"] / dt / 1e6,
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "frame_ms_extrapolated": round(frame_ms, 1),
        "cpu_model": model,
        "host_cpus": os.cpu_count(),
        "value_1thread": st1["segments"] / dt1 / 1e6,
        "sample": (f"{args.scene} {w}x{h} spp={args.cpu_spp} depth={args.depth} (same camera; "
                   f"{w * h * args.cpu_spp} of the frame's {args.width * args.height * args.spp} samples), "
                   f"median of 5 after a warm-up on {threads} threads (this job's CPU share; the host has "
                   f"{os.cpu_count()}): {dt:.2f} s wall, {st['segments']} segments; spp scale factor "
                   f"{args.spp / args.cpu_spp:g}, pixel scale factor {args.cpu_div ** 2}; ms/frame "
                   f"extrapolated by samples: {frame_ms:.0f}; value_1thread: spp={spp1} on 1 thread, {dt1:.2f} s"),
    }


def load_valu_profile(workload: str):
    """VALU wave-instructions per traced segment of this workload's render kernel, from the
    committed rocprofv3 SQ_INSTS_VALU pass (profiles/valu_issue.json, tools/valu_summary.py)."""
    path = os.path.join(REPO, "profiles", "valu_issue.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        wl = json.load(fh).get("workloads", {})
    if workload in wl:
        return wl[workload]
    # N > 1 shards trace the same segments: the frame's per-segment count applies
    base = workload.rsplit("_n", 1)[0] + "_n1"
    if base in wl:
        ent = dict(wl[base])
        ent["source"] = ent["source"] + " (the N = 1 frame's per-segment count)"
        return ent
    return None


def load_pmc_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any (the entry)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh)
    return d.get(workload)


def kernel_source_sha() -> str:
    """The loaded librtmi.so's source digest (rt_kernel_source_sha: every native source, the
    Makefile, include/rtmi.h and the EXTRA flags, baked in at build time; source_digest.py). The
    binding refuses an in-tree library whose digest is not the tree's, so a profile stamped with
    this digest (tools/valu_summary.py, tools/pmc_summary.py) was taken of the library timed here."""
    from raytracingthenextweekcuda_amd import _lib

    return _lib.source_sha()


def profile_check(ent, variant_name: str, sha: str):
    """None if a committed profile entry was taken of the timed kernel (same symbol and the
    same kernel sources), else the reason it was not."""
    if ent is None:
        return "no profile for this workload"
    k = ent.get("kernel") or ""
    if variant_name and variant_name not in k:
        return f"profiled kernel {k!r} is not the launched {variant_name!r}"
    if ent.get("kernel_source_sha") != sha:
        return f"profiled kernel sources {ent.get('kernel_source_sha')} != this tree's {sha}"
    return None


N_ISOLATED = 3


def measure(args, world, rank, local, rehearsal):
    """One rank's timed frames on its GPU, then N_ISOLATED isolated frames (one launch at a
    time, no overlap: kernel latency, gather time, frame latency). Returns per-rank numbers."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd import _lib

    _lib.require_parity_build("bench.py")  # an ablation / timer build would not measure the shipped kernel
    W, H = args.width, args.height
    # Frame overlap (default): --contexts contexts on as many streams take turns at frames, so frame
    # k+1's launch fills the SIMDs that frame k's persistent launch leaves idle while its
    # last work items drain (tools/overlap_probe.py: CB1 N = 8 shard 1.17 -> 1.00 ms/frame,
    # N = 1 7.57 -> 7.42). Every frame is still rendered completely.
    contexts = args.contexts
    shard_world = args.rehearse_shard or world  # row tiling of the frame (the rehearsal: rank 0 of N)
    abi_exchange = (world > 1 or args.rehearse_shard) and not rehearsal and args.exchange == "abi"
    if contexts == 0:  # auto: a third context pays off where the launch's tail is a visible share of it
        samples = rtmi.owned_rows(H, args.row_block, rank, shard_world) * W * args.spp
        small = samples <= (1 << 25) and INTEGRATOR.get(args.scene, "rayColor") != "pathTrace"
        contexts = 3 if small else 2
        if world > 1 and not abi_exchange:
            # ProcessGroupNCCL's own stream is a fourth busy stream besides the default one
            contexts = 2
    if contexts < 2 and not args.no_overlap:
        raise SystemExit("--contexts must be >= 2 (or 0 = auto, or --no-overlap)")
    # every context takes at least one timed frame (its first timed launch resets its counters)
    n_ctx = min(contexts, args.steps)
    overlap = not args.no_overlap and not rehearsal and n_ctx >= 2
    rs = [rtmi.Renderer(device=local) for _ in range(n_ctx if overlap else 1)]
    for rr in rs:
        getattr(rtmi, SCENES[args.scene][0])(rr, W, H)
    r = rs[0]
    from raytracingthenextweekcuda_amd.distributed import RcclRowFrames, RowShardedFrame

    block = args.row_block
    rows = rtmi.owned_rows(H, block, rank, shard_world)
    streams = [torch.cuda.Stream(device=local) for _ in rs] if overlap else None
    if abi_exchange:
        # N > 1 (and the one-GPU shard rehearsal): the C ABI's rt_gather_rows (one ncclGather + the
        # root's de-interleave) on each frame's own render stream; gloo carries the control plane
        frame = RcclRowFrames(rs, W, H, block, rank, shard_world, streams or [torch.cuda.current_stream()],
                              torch.device("cuda", local), comm_world=world)
    else:
        # N > 1 over ProcessGroupNCCL (--exchange torch): frame k's gather runs on the NCCL stream under
        # frame k+1's render (double-buffered tiles); every frame is complete by the end
        frame = RowShardedFrame(W, H, block,
                                device=torch.device("cpu") if rehearsal else torch.device("cuda", local),
                                pipeline=world > 1, streams=streams)
    integrator = INTEGRATOR.get(args.scene, "rayColor")
    # three or more frames in flight: the library may pick a layout for throughput
    # (RT_RENDER_FRAMES_IN_FLIGHT; the isolated frames below use the same layout)
    in_flight = (overlap and n_ctx >= 3) or args.in_flight_layout
    params = r.params(W, H, args.spp, args.depth, 1984, 0, block, rank, shard_world, args.lanes, integrator,
                      frames_in_flight=in_flight)
    # timed launches add to the device counters (one read after the loop, no
    # per-frame host sync); each context's first timed launch resets them
    params_keep = r.params(W, H, args.spp, args.depth, 1984, 0, block, rank, shard_world, args.lanes, integrator,
                           keep_counters=True, frames_in_flight=in_flight)
    stream = torch.cuda.current_stream()
    scratch = torch.empty(frame.tile.shape, dtype=torch.float32, device="cuda") if rehearsal else None

    def launch_stream(b):
        return streams[b] if overlap else stream

    def render_into(tile, p, b=0):
        if rehearsal:
            r.render_device(p, scratch.data_ptr(), stream.cuda_stream)
            tile.copy_(scratch.cpu())
        else:
            rs[b].render_device(p, tile.data_ptr(), launch_stream(b).cuda_stream)

    # every context renders at least one untimed frame (its first launch allocates its work queue
    # and partial sums), however small --warmup is
    for _ in range(max(args.warmup, len(rs))):
        if overlap or abi_exchange:
            frame.submit(lambda tile, b: render_into(tile, params, b))
        else:
            frame.submit(lambda tile: render_into(tile, params))
        frame.drain()
    torch.cuda.synchronize()
    for rr in rs:
        rr.stats()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        p = params if i < len(rs) else params_keep

        def timed_render(tile, b=0, p=p, e=ev[i]):
            e[0].record(launch_stream(b))  # on the stream the kernel is launched on
            render_into(tile, p, b)
            e[1].record(launch_stream(b))

        frame.submit(timed_render)  # this rank's row tiles; the RCCL gather to rank 0 overlaps the next frame
    frame.drain()  # the last frame's gather and row assembly
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    sts = [rr.stats() for rr in rs]  # counters summed over each context's timed launches
    st = dict(sts[0])
    for k in ("segments", "tri_tests", "box_tests", "node_visits", "group_sphere_tests",
              "group_moving_sphere_tests", "launches", "kernel_ms_sum"):
        st[k] = sum(x[k] for x in sts)
    launch_ms = [a.elapsed_time(b) for a, b in ev]  # render kernel + the work queue's combine pass
    assert st["launches"] == args.steps, st["launches"]

    # Isolated frames (outside the timed region): one launch at a time on one context, so the
    # library's event pair is the megakernel's own latency (the roofline's time base), and at
    # N > 1 the gather's own time (events on the stream the collective is ordered on) and one
    # whole frame's latency (render + gather + row assembly, barrier to barrier).
    iso_kernel, iso_gather, iso_frame = [], [], []
    cur = torch.cuda.current_stream()
    for _ in range(N_ISOLATED):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if rehearsal:
            render_into(frame.tile, params)
        else:
            r.render_device(params, frame.tile.data_ptr(), cur.cuda_stream)
        torch.cuda.synchronize()
        iso_kernel.append(r.stats()["kernel_ms"])
        if world > 1 or abi_exchange:
            if rehearsal:  # gloo on host tensors: no device events
                g0 = time.perf_counter()
                frame.gather()
                iso_gather.append((time.perf_counter() - g0) * 1e3)
            else:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                frame.gather(events=(e0, e1))
                torch.cuda.synchronize()
                iso_gather.append(e0.elapsed_time(e1))
            if world > 1:
                dist.barrier()
        torch.cuda.synchronize()
        iso_frame.append((time.perf_counter() - t1) * 1e3)
    n_cu = torch.cuda.get_device_properties(local).multi_processor_count
    out = {
        "dt": dt, "segs": float(st["segments"]), "tri_tests": float(st["tri_tests"]),
        "box_tests": float(st["box_tests"]), "nodes": float(st["node_visits"]),
        "grp_bytes": float(st["group_sphere_tests"] * BYTES["sphere"]
                           + st["group_moving_sphere_tests"] * BYTES["moving_sphere"]),
        "rows": float(rows),
        "kernel_ms": st["kernel_ms_sum"] / st["launches"],  # the megakernel alone (library event pairs)
        "kernel_ms_isolated": float(np.mean(iso_kernel)),
        "gather_ms": float(np.mean(iso_gather)) if iso_gather else 0.0,
        "frame_ms_isolated": float(np.mean(iso_frame)),
        "launch_ms": float(np.mean(launch_ms)),
        "lanes_per_pixel": int(st["lanes_per_pixel"]), "refill": int(st["refill"]),
        "substreams_per_item": int(st.get("substreams_per_item", 1)),
        "queue_blocks": int(st["queue_blocks"]), "variant": st["variant_name"],
        "object_bytes_per_segment": object_bytes_per_segment(r) if integrator != "pathTrace" else 0,
        "n_cu": n_cu, "overlap": overlap, "contexts": len(rs), "frames_in_flight": in_flight,
        "exchange": ("abi" if abi_exchange else "torch-gloo" if rehearsal else "torch") if world > 1 or abi_exchange
        else None,
        "shard_world": shard_world,
    }
    if abi_exchange:
        frame.close()
    for rr in rs:
        rr.close()
    return out


def selftest_measure(args, world, rank):
    """--line-selftest (CPU only, tests/test_bench_line.py): deterministic per-rank numbers in
    place of the GPU measurement, so the collectives and the JSON line run end to end under
    torch.distributed.run with gloo."""
    return {
        "dt": 0.010 * (1.0 + 0.1 * rank), "segs": 1.0e6 * (rank + 1), "tri_tests": 2.0e6, "box_tests": 1.0e5,
        "nodes": 0.0, "grp_bytes": 0.0, "rows": float(args.height // world),
        "kernel_ms": 5.0 + rank, "kernel_ms_isolated": 4.0 + rank, "gather_ms": 0.05 * (rank + 1),
        "frame_ms_isolated": 6.0 + 0.5 * rank, "launch_ms": 5.5 + rank, "lanes_per_pixel": 32, "refill": 8,
        "queue_blocks": 1536, "variant": "render_kernel<selftest>",  # matches no profile: refused
        "object_bytes_per_segment": 240, "n_cu": 256, "overlap": True, "contexts": 3,
        "exchange": "abi" if world > 1 else None,
    }


# per-rank numbers combined over ranks: SUM (work), MAX (time of the slowest rank), and
# MIN / MAX of the per-rank kernel times (the shard balance the scaling curve depends on)
SUM_KEYS = ("segs", "tri_tests", "box_tests", "nodes", "grp_bytes", "rows")


def aggregate(m: dict, world: int, device):
    """Combines the ranks' numbers (one all_gather of a small vector over the job's group)."""
    import torch
    import torch.distributed as dist

    keys = ("dt",) + SUM_KEYS + ("kernel_ms", "kernel_ms_isolated", "gather_ms", "frame_ms_isolated", "launch_ms")
    v = torch.tensor([float(m[k]) for k in keys], dtype=torch.float64, device=device)
    if world > 1:
        parts = [torch.zeros_like(v) for _ in range(world)]
        dist.all_gather(parts, v)
        per_rank = torch.stack(parts).cpu().numpy()
        comm_world = dist.get_world_size()
    else:
        per_rank = v.cpu().numpy()[None, :]
        comm_world = 1
    col = {k: per_rank[:, i] for i, k in enumerate(keys)}
    agg = dict(m)
    agg["dt"] = float(col["dt"].max())
    for k in SUM_KEYS:
        agg[k] = float(col[k].sum())
    for k in ("kernel_ms", "kernel_ms_isolated", "launch_ms"):
        agg[k] = float(col[k].mean())
        agg[k + "_min"] = float(col[k].min())
        agg[k + "_max"] = float(col[k].max())
    agg["gather_ms"] = float(col["gather_ms"].max())
    agg["frame_ms_isolated"] = float(col["frame_ms_isolated"].max())
    agg["world_size_comm"] = comm_world
    return agg


def build_line(args, agg: dict, world: int, cpu=None) -> dict:
    """The bench's JSON line (rank 0)."""
    W, H, K = args.width, args.height, args.steps
    dt, segs = agg["dt"], agg["segs"]
    overlap = agg["overlap"]
    ms_frame = dt * 1e3 / K
    mrays = segs / dt / 1e6
    # Record-byte model of SURVEY §8(d), kept as a side figure: these records are
    # served by the scalar cache, L1 and L2 (the scene is cache-resident), not HBM.
    seg_launch = segs / K / world
    pt = INTEGRATOR.get(args.scene) == "pathTrace"
    alg_bytes = (seg_launch * (6 * BYTES["sphere"] if pt else agg["object_bytes_per_segment"])
                 + agg["tri_tests"] / K / world * BYTES["ktri" if pt else "tri"]
                 + agg["box_tests"] / K / world * BYTES["box"] + agg["nodes"] / K / world * BYTES["node"]
                 + agg["grp_bytes"] / K / world
                 + agg["rows"] / world * W * BYTES["pixel"])
    t_iso = agg["kernel_ms_isolated"]
    workload = f"{args.scene}_{W}x{H}_spp{args.spp}_d{args.depth}_n{world}"
    if args.rehearse_shard:  # one GPU rendering rank 0's shard of an N-rank frame
        workload += f"_shard{args.rehearse_shard}"
    sha = kernel_source_sha()
    # Roofline: the megakernel is bound by VALU issue. achieved = VALU
    # wave-instructions per launch (SQ_INSTS_VALU per traced segment, profiled of this very
    # kernel, x this launch's segments) / the isolated megakernel time; peak = the chip's issue rate.
    valu_peak = agg["n_cu"] * VALU_GINST_PER_CU
    vp = load_valu_profile(workload)
    vp_bad = profile_check(vp, agg["variant"], sha)
    valu_launch = vp["valu_insts_per_segment"] * seg_launch if vp else None
    achieved = valu_launch / (t_iso * 1e-3) / 1e9 if vp and not vp_bad else None
    achieved_ovl = valu_launch / (ms_frame * 1e-3) / 1e9 if vp and not vp_bad else None
    lane_u = vp.get("valu_lane_util") if vp and not vp_bad else None
    # the scalar unit (one per CU, shared by its four SIMDs): SALU instructions of the same
    # kernel per launch / (CUs x 2.4 GHz x the isolated kernel time)
    salu_seg = vp.get("salu_insts_per_segment") if vp and not vp_bad else None
    salu_frac = salu_seg * seg_launch / (agg["n_cu"] * 2.4e9 * t_iso * 1e-3) if salu_seg else None
    tp = load_pmc_traffic(workload)
    tp_bad = profile_check(tp, agg["variant"], sha)
    traffic = float(tp["hbm_bytes_per_launch"]) if tp and not tp_bad else None
    line = {
        "metric": METRIC,
        "value": round(mrays, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(ms_frame, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (deterministic {args.scene} scene from assets/scenes; counter-based RNG seed 1984)",
        "config": {
            "workload": workload,
            "scene": SCENES[args.scene][5],
            "width": W, "height": H, "spp": args.spp, "depth": args.depth,
            "row_block": args.row_block, "lanes_per_pixel": agg["lanes_per_pixel"],
            "substreams_per_item": agg.get("substreams_per_item", 1),
            "variant": agg["variant"], "queue": agg["queue_blocks"] > 0,
            "refill": agg["refill"], "queue_blocks": agg["queue_blocks"], "contexts": agg.get("contexts", 1),
            "frames_in_flight": bool(agg.get("frames_in_flight", False)),
            # N > 1: the row-tile exchange, and the HIP streams a rank keeps busy or holds: its render
            # streams + the default stream (+ ProcessGroupNCCL's with --exchange torch); the process
            # has GPU_MAX_HW_QUEUES = 4 hardware queues
            "exchange": agg.get("exchange"),
            "streams_per_rank": (agg.get("contexts", 1) + 1 + (1 if agg.get("exchange") == "torch" else 0)),
            "rehearse_shard": args.rehearse_shard or None,
            "n_cu": agg["n_cu"],
            "kernel_source_sha": sha,
            "parallelism": f"row-tiles x{world} + RCCL gather" if world > 1 else "single GPU",
            "segments_per_frame": int(segs / K),
            # traversal work per traced segment (the library's event counters)
            "per_segment": {"node_visits": round(agg["nodes"] / segs, 3) if segs else None,
                            "tri_tests": round(agg["tri_tests"] / segs, 3) if segs else None,
                            "box_tests": round(agg["box_tests"] / segs, 3) if segs else None},
            "msamples_per_s": round(W * H * args.spp / (dt / K) / 1e6, 3),
        },
        # one frame at a time, outside the timed region (N_ISOLATED frames, max over ranks):
        # what a single frame costs without frame overlap or pipelining
        "frame_latency": {
            "frame_ms_isolated": round(agg["frame_ms_isolated"], 4),
            "kernel_ms_isolated": round(t_iso, 4),
            "gather_ms": round(agg["gather_ms"], 4),
        },
        "roofline": {
            "bound": "valu",
            "achieved": round(achieved, 2) if achieved else None,
            "peak": round(valu_peak, 1),
            "unit": "Ginst/s (wave64 VALU instructions)",
            "frac": round(achieved / valu_peak, 4) if achieved else None,
            # issued wave-instructions count every masked-off lane as work: the profiled lane
            # utilisation (SQ_THREAD_CYCLES_VALU / 64 / SQ_ACTIVE_INST_VALU of the same pass) turns
            # frac into the fraction of the chip's lane-operations that did useful work
            "valu_lane_util": round(lane_u, 4) if lane_u else None,
            "useful_frac": round(achieved / valu_peak * lane_u, 4) if achieved and lane_u else None,
            # the co-bound: scalar instructions against one per CU per cycle
            "salu_insts_per_segment": round(salu_seg, 3) if salu_seg else None,
            "salu_frac": round(salu_frac, 4) if salu_frac else None,
            "traffic": traffic,
            # the isolated launch's megakernel time (library event pair, combine pass excluded)
            "kernel_ms": round(t_iso, 4),
            "frac_overlapped": round(achieved_ovl / valu_peak, 4) if achieved_ovl else None,
            "kernel_ms_timed_event_pairs": round(agg["kernel_ms"], 4),
            "launch_ms": round(agg["launch_ms"], 4),
            "valu_insts_per_launch": int(valu_launch) if valu_launch else None,
            "valu_profile": vp.get("source") if vp else None,
            "profile_mismatch": vp_bad,
            "traffic_profile_mismatch": tp_bad,
            "hbm_frac": round(traffic / (t_iso * 1e-3) / (HBM_PEAK_GBS * 1e9), 5) if traffic else None,
            "overlap": overlap,
            "record_bytes_per_launch": int(alg_bytes),
            "record_gbs": round(alg_bytes / (t_iso * 1e-3) / 1e9, 1),
            "note": ("achieved = SQ_INSTS_VALU per segment (rocprofv3 pass of this kernel symbol and these kernel "
                     "sources, profiles/valu_issue.json) x this launch's segments / the isolated megakernel time "
                     "(kernel_ms: one launch at a time after the timed loop, library event pair, combine pass "
                     "excluded - what rocprofv3's kernel trace measures); frac_overlapped divides by the timed "
                     "frame time instead (two launches in flight); peak = CUs x 4 SIMDs x 2.4 GHz / 2 cycles per "
                     "wave64 VALU op; useful_frac = frac x valu_lane_util (the same pass's SQ_THREAD_CYCLES_VALU "
                     "/ 64 / SQ_ACTIVE_INST_VALU: active lanes per issued instruction); salu_frac = SQ_INSTS_SALU of "
                     "the same kernel per launch / (CUs x 2.4 GHz x kernel_ms): the CU's one scalar ALU, which "
                     "the scan kernels load as much as their VALU (DESIGN 5). traffic = HBM-side bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, "
                     "profiles/pmc_traffic.json), hbm_frac its share of 8 TB/s; a profile of another kernel "
                     "symbol or other kernel sources is not used (profile_mismatch); record_* = SURVEY 8(d)'s "
                     "cache-served record-byte model"),
        },
        "cpu_baseline": cpu,
    }
    if world > 1:
        # what the scaling curve needs to explain itself: the shard balance over ranks and the
        # exchange's own cost
        line["scale"] = {
            "world_size_comm": agg["world_size_comm"],
            "kernel_ms_timed_min": round(agg["kernel_ms_min"], 4),
            "kernel_ms_timed_max": round(agg["kernel_ms_max"], 4),
            "kernel_ms_isolated_min": round(agg["kernel_ms_isolated_min"], 4),
            "kernel_ms_isolated_max": round(agg["kernel_ms_isolated_max"], 4),
            "gather_ms": round(agg["gather_ms"], 4),
            "frame_ms_isolated": round(agg["frame_ms_isolated"], 4),
        }
    return line


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) without an outer launcher: start torch.distributed.run with N
    ranks on this node as a CHILD process (never exec: nothing here has touched the GPU yet, and the
    parent stays out of it), let rank 0's JSON line through, and return the child's exit code."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rehearse_shard and world > 1:
        raise SystemExit("--rehearse-shard runs one process on one GPU")
    if args.line_selftest:  # CPU: the N > 1 collectives and line building, without a GPU
        if world > 1:
            dist.init_process_group("gloo")
        agg = aggregate(selftest_measure(args, world, rank), world, "cpu")
        if rank == 0:
            print(json.dumps(build_line(args, agg, world)), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    # RTMI_REHEARSAL=1 (testing only): N ranks share GPU 0 and gather over gloo
    # through host memory, to exercise the N > 1 code path on a one-GPU box.
    rehearsal = os.environ.get("RTMI_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if rehearsal or args.exchange == "abi":
            # the ABI exchange's control plane (unique id, barriers, stats); the frames move over
            # the library's own RCCL communicator
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    m = measure(args, world, rank, local, rehearsal)
    on_host = rehearsal or (world > 1 and args.exchange == "abi")
    agg = aggregate(m, world, "cpu" if on_host else torch.device("cuda", local))
    if rank == 0:
        cpu = (cpu_baseline(args, host_threads())
               if not args.no_cpu_baseline and world == 1 and not args.rehearse_shard else None)
        print(json.dumps(build_line(args, agg, world, cpu)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

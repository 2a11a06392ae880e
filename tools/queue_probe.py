"""How many HIP streams of one process run concurrently (GPU_MAX_HW_QUEUES hardware queues).

Each busy stream runs one torch.cuda._sleep spin kernel (one block, a fixed number of cycles);
the wall time of k streams started together, over one stream's, says how many of them shared a
hardware queue (1.0: all concurrent; 2.0: two of them serialised behind each other). Cases:

  pool<k>        k streams from torch's stream pool (what bench.py's contexts use)
  pool<k>+null   the same plus the default stream busy
  rccl+pool<k>   after a one-rank RCCL communicator was created through librtmi (its internal
                 streams exist)

Usage: python tools/queue_probe.py [--cycles N]   (prints one JSON line per case)
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=100_000_000)
    ap.add_argument("--rccl-first", action="store_true", help="create the RCCL communicator before the streams")
    a = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    comm = None
    if a.rccl_first:
        comm = make_comm()
    pool = [torch.cuda.Stream() for _ in range(6)]
    null = torch.cuda.default_stream()

    def run(streams):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in streams:
            with torch.cuda.stream(s):
                torch.cuda._sleep(a.cycles)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(pool[:1])
    t1 = min(run(pool[:1]) for _ in range(3))
    out = {"one_stream_s": round(t1, 4), "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
           "rccl_first": a.rccl_first}
    for k in range(2, 7):
        out[f"pool{k}"] = round(min(run(pool[:k]) for _ in range(2)) / t1, 2)
    for k in (2, 3, 4):
        out[f"pool{k}+null"] = round(min(run(pool[:k] + [null]) for _ in range(2)) / t1, 2)
    if comm is None:
        comm = make_comm()
        for k in (2, 3, 4):
            out[f"rccl+pool{k}"] = round(min(run(pool[:k]) for _ in range(2)) / t1, 2)
        fresh = [torch.cuda.Stream() for _ in range(3)]  # pool streams handed out after the comm
        out["rccl+fresh3"] = round(min(run(fresh) for _ in range(2)) / t1, 2)
    print(json.dumps(out), flush=True)


def make_comm():
    from raytracingthenextweekcuda_amd import _lib
    import raytracingthenextweekcuda_amd as rtmi

    L = _lib.lib()
    r = rtmi.Renderer(0)
    idb = (C.c_uint8 * 128)()
    assert L.rt_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    r._check(L.rt_comm_init(r.ctx, idb, 1, 0, C.byref(comm)))
    return (r, comm)


if __name__ == "__main__":
    main()

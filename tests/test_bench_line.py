"""bench.py's N > 1 line building, end to end on CPU: torch.distributed.run starts two ranks,
gloo carries the collectives, and each rank contributes deterministic numbers in place of its
GPU measurement (--line-selftest). The line must carry what a SCALE record needs to explain
itself: the communicator's world size, per-rank min / max kernel times, the gather time and
one isolated frame latency - and the whole-job value = all ranks' segments / the slowest
rank's time."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(nproc):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", str(nproc), "--steps", "4", "--warmup", "1", "--line-selftest", "--no-cpu-baseline"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints one line
    return json.loads(lines[0])


def test_two_rank_line_has_the_scaling_fields():
    d = _run(2)
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["scaling"] == "strong"
    # selftest ranks: dt 0.010 / 0.011 s, segments 1e6 / 2e6, kernel 5 / 6 ms, isolated 4 / 5 ms
    assert d["value"] == pytest.approx(3.0e6 / 0.011 / 1e6, abs=1e-3)
    assert d["ms_per_step"] == pytest.approx(11.0 / 4, abs=1e-4)
    sc = d["scale"]
    assert sc["world_size_comm"] == 2
    assert (sc["kernel_ms_timed_min"], sc["kernel_ms_timed_max"]) == (5.0, 6.0)
    assert (sc["kernel_ms_isolated_min"], sc["kernel_ms_isolated_max"]) == (4.0, 5.0)
    assert sc["gather_ms"] == pytest.approx(0.1)
    assert sc["frame_ms_isolated"] == pytest.approx(6.5)
    assert d["frame_latency"]["frame_ms_isolated"] == pytest.approx(6.5)
    assert d["config"]["segments_per_frame"] == 750000
    assert d["config"]["variant"].startswith("render_kernel<") and d["config"]["queue"] is True
    # the roofline's time base is the isolated kernel time; a profile of another kernel is refused
    assert d["roofline"]["kernel_ms"] == pytest.approx(4.5)
    assert d["roofline"]["frac"] is None and d["roofline"]["profile_mismatch"]


def test_one_rank_line_has_no_scale_block():
    d = _run(1)
    assert d["n_gpus"] == 1 and "scale" not in d
    assert d["frame_latency"]["gather_ms"] == 0.05 and d["frame_latency"]["kernel_ms_isolated"] == 4.0


def test_bench_spawns_its_own_ranks_without_an_outer_launcher():
    """`python3 bench.py --gpus 2` (the driver's form for every N) starts torch.distributed.run as a
    child process and forwards rank 0's line."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--line-selftest", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scale"]["world_size_comm"] == 2
    assert d["value"] == pytest.approx(3.0e6 / 0.011 / 1e6, abs=1e-3)
    # three render streams + the default stream: within the process's 4 hardware queues
    assert d["config"]["exchange"] == "abi" and d["config"]["streams_per_rank"] == 4


def test_bench_refuses_a_world_size_that_is_not_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--line-selftest"],
                         cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr

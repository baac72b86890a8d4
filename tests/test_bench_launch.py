"""bench.py's rank launcher: ``--gpus N`` with no outer torchrun starts
N ranks itself (a torch.distributed.run child process, no exec) and reports n_gpus = N;
inside the ranks WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ, MIMO_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env,
                          timeout=timeout, cwd=REPO)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_two_launches_two_ranks_without_outer_torchrun():
    p = _run(["--gpus", "2", "--no-cpu-baseline", "--check-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_line(p.stdout)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2


def test_grid_line_two_ranks_equals_one_rank():
    """The grid object (north_star's SNR x IBO split) through bench.py's own rank launcher:
    gloo world 2 on CPU with the stand-in link sees both ranks and reproduces the
    single-process grid's counters exactly (digest of every point's counts)."""
    p1 = _run(["--gpus", "1", "--grid-check"])
    assert p1.returncode == 0, p1.stderr[-2000:]
    g1 = _json_line(p1.stdout)["grid"]
    p2 = _run(["--gpus", "2", "--grid-check"])
    assert p2.returncode == 0, p2.stderr[-2000:]
    d2 = _json_line(p2.stdout)
    g2 = d2["grid"]
    assert d2["n_gpus"] == 2 and g2["ranks_seen"] == 2 and g1["ranks_seen"] == 1
    assert g2["points"] == g1["points"] == 915
    assert g2["counts_digest"] == g1["counts_digest"] and g2["ofdm_symbols"] == g1["ofdm_symbols"] > 0


def test_world_size_mismatch_exits_nonzero():
    p = _run(["--gpus", "2", "--check-launch"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in p.stderr


@pytest.mark.gpu
def test_bench_gpus_two_on_one_gpu_reports_both_ranks():
    """The full bench step with two gloo ranks sharing GPU 0 (the driver's N > 1 path uses RCCL,
    one GPU per rank): the line reports n_gpus 2 and counts trials of both ranks."""
    p = _run(["--gpus", "2", "--no-cpu-baseline", "--steps", "2", "--warmup", "1", "--batch", "4096"], timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_line(p.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "trial-sharded x2"
    assert d["value"] > 0 and 0 < d["ber"][0] < 1e-2
    # the grid object: the 915-point config-4 grid dealt over both ranks equals one rank's grid
    p1 = _run(["--gpus", "1", "--no-cpu-baseline", "--steps", "1", "--warmup", "1", "--batch", "4096"], timeout=300)
    assert p1.returncode == 0, p1.stderr[-3000:]
    g1, g2 = _json_line(p1.stdout)["grid"], d["grid"]
    print("grid 1 rank", g1, "grid 2 ranks", g2)
    assert g2["ranks_seen"] == 2 and g1["ranks_seen"] == 1 and g1["points"] == 915
    assert g2["counts_digest"] == g1["counts_digest"] and g2["ofdm_symbols"] == g1["ofdm_symbols"] > 200000
    # per-rank work record: both ranks, every point once
    assert [r["rank"] for r in g2["per_rank"]] == [0, 1]
    assert sum(r["points"] for r in g2["per_rank"]) == 915 and g1["per_rank"][0]["points"] == 915
    assert sum(r["trials"] for r in g2["per_rank"]) == g1["per_rank"][0]["trials"]


def test_grid_check_reports_per_rank_records():
    """CPU: the grid object carries one work record per rank (points, trials, rounds, kernel ms,
    wall s, modelled cost) and the axis it sweeps."""
    p = _run(["--gpus", "2", "--grid-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    g = _json_line(p.stdout)["grid"]
    assert len(g["per_rank"]) == 2 and sum(r["points"] for r in g["per_rank"]) == 915
    for r in g["per_rank"]:
        assert set(r) >= {"rank", "points", "trials", "rounds", "kernel_ms", "wall_s", "cost_model"}
    assert g["trials_max_over_mean"] >= 1.0 and "Eb/N0" in g["axis"]


@pytest.mark.gpu
def test_bench_rccl_process_group_at_world_one():
    """The RCCL branch on hardware: torchrun with ONE rank and the nccl
    backend -- bench.py then opens a process group at world size 1, so the headline's counter
    all-reduce, the grid's counter all-reduce (sweep.run_grid) and the per-rank gather all run
    through RCCL -- and the grid's counts equal those of a run without any process group."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, MIMO_BENCH_BACKEND="nccl", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    args = ["--gpus", "1", "--no-cpu-baseline", "--steps", "2", "--warmup", "1", "--batch", "4096"]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr", "127.0.0.1", f"--master-port={port}", BENCH] + args,
                       capture_output=True, text=True, env=env, timeout=300, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_line(p.stdout)
    p0 = _run(args, timeout=300)
    assert p0.returncode == 0, p0.stderr[-3000:]
    d0 = _json_line(p0.stdout)
    print("rccl world 1", d["grid"], "no group", d0["grid"])
    assert d["n_gpus"] == 1 and d["grid"]["ranks_seen"] == 1 and len(d["grid"]["per_rank"]) == 1
    assert d["grid"]["counts_digest"] == d0["grid"]["counts_digest"]
    assert d["ber"] == d0["ber"]

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

"""Sharing each grid point's trials over the ranks (sweep.run_grid(split="trials") ->
Link.simulate_points(dist=...): one all_reduce of the round's counts per stopping-rule
round) on CPU with gloo: the real Link orchestration (stopping rule, batch
sizes, counter columns) over a deterministic stand-in engine whose counts depend only on
(seed, trial, column), so any split of the trials must reproduce one rank's totals exactly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as tmp

from link_util import build_link


class FakeEngine:
    """run_points with per-trial counts a pure function of (seed, trial, column, SNR)."""

    def __init__(self, bits_per_trial):
        self.bps = bits_per_trial
        self.kernel_ms = 0.0
        self.calls = []

    def run_points(self, points, seeds, first_trials, n_trials, iters, incl_clean=False, per_trial=False):
        n_idx = len(sorted(set(int(i) for i in iters))) + (1 if incl_clean else 0)
        P = len(points)
        err = np.zeros((P, n_idx), np.uint64)
        bits = np.zeros((P, n_idx), np.uint64)
        self.calls.append(int(np.sum(n_trials)))
        for i in range(P):
            t = np.arange(int(first_trials[i]), int(first_trials[i]) + int(n_trials[i]), dtype=np.int64)
            snr = float(points[i].snr_db)
            for c in range(n_idx):
                base = int(self.bps * 0.05 * np.exp(-0.3 * snr) / (1 + c))
                jit = ((int(seeds[i]) % 9973 + t * 7919 + c * 104729) % 23) < max(1.0, 12 - 0.5 * snr)
                err[i, c] = np.uint64(np.sum(base + jit))
                bits[i, c] = np.uint64(self.bps * t.size)
        return err, bits, None


def _link():
    link, _ = build_link(n_ant=4, n_sc=64, n_fft=128, M=16, cp=4, ibo=1.0, chan="rayleigh",
                         n_err_min=2000, bits_sent_max=500_000)
    eng = FakeEngine(link.n_bits_per_ofdm_sym)
    link.engine = lambda reroll_chan=True: eng
    link.max_batch = 96  # several stopping-rule rounds per point
    return link, eng


GRID = dict(ibo_arr=[0.0, 3.0], ebn0_arr=np.arange(0.0, 24.0, 4.0), iters=[0, 1, 2])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, split):
    import torch.distributed as dist
    import sweep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    link, eng = _link()
    st = {}
    err, bits = sweep.run_grid(link, GRID["ibo_arr"], GRID["ebn0_arr"], GRID["iters"], True, 7, rank, world, dist,
                               split=split, stats=st)
    np.save(os.path.join(out, f"{split}_w{world}_r{rank}.npy"), np.stack([err, bits]))
    np.save(os.path.join(out, f"{split}_w{world}_r{rank}_trials.npy"),
            np.asarray([sum(eng.calls), st["points"], st["rounds"]]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_trial_split_matches_one_rank(tmp_path, world):
    import sweep
    link, eng = _link()
    st = {}
    ref_err, ref_bits = sweep.run_grid(link, GRID["ibo_arr"], GRID["ebn0_arr"], GRID["iters"], True, 7, stats=st)
    ref_trials = sum(eng.calls)
    assert st["rounds"] >= 3 and ref_err.shape == (2, 6, 4)
    # some counters close on errors, some on the bit budget
    assert np.any(ref_err >= 2000) and np.any(ref_bits >= 500_000)
    tmp.spawn(_worker, args=(world, _free_port(), str(tmp_path), "trials"), nprocs=world, join=True)
    done = 0
    for r in range(world):
        got = np.load(os.path.join(tmp_path, f"trials_w{world}_r{r}.npy"))
        np.testing.assert_array_equal(got[0], ref_err)
        np.testing.assert_array_equal(got[1], ref_bits)
        n_tr, n_pts, n_rounds = np.load(os.path.join(tmp_path, f"trials_w{world}_r{r}_trials.npy"))
        assert n_pts == 12 and n_rounds == st["rounds"]  # every rank runs every point, the same rounds
        done += n_tr
    assert done == ref_trials  # the ranks split the trials, none run twice


def test_point_split_still_matches(tmp_path):
    import sweep
    link, _ = _link()
    ref_err, ref_bits = sweep.run_grid(link, GRID["ibo_arr"], GRID["ebn0_arr"], GRID["iters"], True, 7)
    tmp.spawn(_worker, args=(2, _free_port(), str(tmp_path), "points"), nprocs=2, join=True)
    for r in range(2):
        got = np.load(os.path.join(tmp_path, f"points_w2_r{r}.npy"))
        np.testing.assert_array_equal(got[0], ref_err)
        np.testing.assert_array_equal(got[1], ref_bits)


def test_split_argument_checked():
    import sweep
    link, _ = _link()
    with pytest.raises(ValueError):
        sweep.run_grid(link, [0.0], [10.0], [0], split="bits")


def _auto_worker(rank, world, port, out):
    import torch.distributed as dist
    import sweep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    link, eng = _link()
    st = {}
    err, bits = sweep.run_grid(link, [1.0], [8.0], [0, 1], True, 3, rank, world, dist, split="auto", stats=st)
    np.save(os.path.join(out, f"auto_r{rank}.npy"), np.stack([err, bits]))
    np.save(os.path.join(out, f"auto_r{rank}_n.npy"), np.asarray([sum(eng.calls), st["points"]]))
    dist.destroy_process_group()


def test_auto_split_shares_a_single_point(tmp_path):
    # one point, two ranks: "auto" shares its trials instead of leaving rank 1 idle
    import sweep
    link, eng = _link()
    ref_err, ref_bits = sweep.run_grid(link, [1.0], [8.0], [0, 1], True, 3)
    tmp.spawn(_auto_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    runs = []
    for r in range(2):
        got = np.load(os.path.join(tmp_path, f"auto_r{r}.npy"))
        np.testing.assert_array_equal(got[0], ref_err)
        np.testing.assert_array_equal(got[1], ref_bits)
        n_tr, n_pts = np.load(os.path.join(tmp_path, f"auto_r{r}_n.npy"))
        assert n_pts == 1
        runs.append(n_tr)
    assert sum(runs) == sum(eng.calls) and min(runs) > 0.4 * sum(runs)

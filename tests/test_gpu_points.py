"""Multi-point launches (mimo_engine_run_points) and the config-4 sweep built on them.

* run_points over points with different PA / SNR / seeds / trial ranges gives, per trial,
  exactly the counts of one mimo_engine_run per point (and of the float64 oracle);
* sweep.run_grid through Link.simulate_points equals the point-by-point Link.simulate
  sweep bit-for-bit (same seeds, same stopping-rule batches).
"""
import numpy as np
import pytest

from gpu_util import PRECISIONS, assert_counts_equal, engine_for
from link_util import build_link
from oracle import sim

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", PRECISIONS)
def test_run_points_equals_per_point_runs(prec):
    cfg = sim.SimConfig(8, 256, 512, 16, ibo_db=1.0, snr_db=12.0)
    eng = engine_for(cfg, precision=prec)
    pts, seeds, firsts, ns, refs = [], [], [], [], []
    for k, (ibo, snr, first, n) in enumerate([(1.0, 12.0, 0, 40), (3.0, 16.0, 7, 1), (0.0, 9.0, 100, 77),
                                              (5.0, 20.0, 0, 0), (2.0, 14.0, (1 << 32) - 20, 20)]):
        c = sim.SimConfig(8, 256, 512, 16, ibo_db=ibo, snr_db=snr)
        e = engine_for(c, precision=prec)
        pts.append(_point_of(c))
        seeds.append(1000 + k)
        firsts.append(first)
        ns.append(n)
        _, _, per = e.run(1000 + k, first, n, [0, 1, 3], True, per_trial=True)
        refs.append(per)
    err, bits, per = eng.run_points(pts, seeds, firsts, ns, [0, 1, 3], True, per_trial=True)
    got = np.split(per, np.cumsum(ns)[:-1])
    for k in range(len(pts)):
        assert_counts_equal(got[k], refs[k], f"point {k} {prec}")
        np.testing.assert_array_equal(err[k], refs[k].sum(0))
        assert np.all(bits[k] == ns[k] * 256 * 4)
    # and the oracle on the middle point
    c = sim.SimConfig(8, 256, 512, 16, ibo_db=0.0, snr_db=9.0)
    ref = sim.run_trials(c, 1002, np.arange(100, 177), iters=[0, 1, 3], incl_clean=True)
    assert_counts_equal(got[2], ref, f"oracle {prec}")


def _point_of(cfg):
    from oracle.sim import point_params
    from oracle import refmath as rm
    pp = point_params(cfg)
    return dict(ibo_db=cfg.ibo_db, snr_db=cfg.snr_db, avg_symbol_power=pp["es"], pa_kind=cfg.pa,
                sat_pow=rm.sat_pow(cfg.ibo_db, pp["avg_samp"] / cfg.n_ant), cnc_pa_kind=cfg.pa,
                cnc_sat_pow=pp["cnc_sat"], cnc_alpha=pp["cnc_alpha"])


@pytest.mark.parametrize("receiver", ["cnc", "mcnc"])
def test_multipoint_sweep_equals_sequential(receiver):
    import sweep
    kw = dict(n_ant=8, n_sc=256, n_fft=512, M=16, bits_sent_max=1024 * 300, n_err_min=2000,
              is_mcnc=receiver == "mcnc")
    ibo, ebn0 = [0.0, 1.5, 4.0], [4.0, 8.0, 12.0, 30.0]
    link, _ = build_link(**kw)
    err, bits = sweep.run_grid(link, ibo, ebn0, [0, 1, 2], False, seed=5)
    link2, _ = build_link(**kw)
    err2, bits2 = sweep.run_grid(link2, ibo, ebn0, [0, 1, 2], False, seed=5, multipoint=False)
    np.testing.assert_array_equal(err, err2)
    np.testing.assert_array_equal(bits, bits2)
    # the stopping rule: every counter closed by errors or the budget
    assert np.all((err >= 2000) | (bits >= 1024 * 300))
    assert np.all(bits <= 1024 * 300 + 64 * 1024)  # overshoot of at most one pilot batch


@pytest.mark.parametrize("split", ["points", "trials"])
def test_gloo_sharded_sweep_through_real_link_equals_single_process(tmp_path, split):
    """world_size 2 over gloo, both ranks on GPU 0, sweep.run_grid through the real
    Link -> libmimo_engine path: equal to the single-process grid bit-for-bit, whether the
    ranks deal the points or share every point's trials (one all_reduce per round)."""
    import os
    import socket

    import torch.multiprocessing as tmp

    import link_util
    import sweep
    kw = dict(n_ant=8, n_sc=256, n_fft=512, M=16, bits_sent_max=1024 * 200, n_err_min=3000)
    ibo, ebn0, iters = [0.0, 2.0, 5.0], [5.0, 9.0, 13.0], [0, 1, 2]
    link, _ = build_link(device=0, **kw)
    ref_err, ref_bits = sweep.run_grid(link, ibo, ebn0, iters, False, 11)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    tmp.spawn(link_util.sweep_rank, args=(2, port, str(tmp_path), kw, ibo, ebn0, iters, split), nprocs=2, join=True)
    for r in range(2):
        got = np.load(os.path.join(tmp_path, "r%d.npy" % r))
        np.testing.assert_array_equal(got[0], ref_err)
        np.testing.assert_array_equal(got[1], ref_bits)


def test_launch_splitting_keeps_every_trial(monkeypatch):
    """Points larger than one launch and launches holding several points
    (MIMO_MAX_LAUNCH_TRIALS=50: the 2^20-trial limit scaled down): per-trial counts in
    point order and per-point totals equal one launch per point."""
    cfg = sim.SimConfig(8, 256, 512, 16, ibo_db=1.0, snr_db=12.0)
    eng = engine_for(cfg)
    pts = [_point_of(sim.SimConfig(8, 256, 512, 16, ibo_db=i, snr_db=s)) for i, s in [(1.0, 12.0), (2.0, 9.0),
                                                                                        (0.5, 15.0)]]
    ns, firsts, seeds = [120, 7, 61], [0, 500, 33], [8, 9, 10]
    ref_err, _, ref_per = eng.run_points(pts, seeds, firsts, ns, [0, 2], True, per_trial=True)
    monkeypatch.setenv("MIMO_MAX_LAUNCH_TRIALS", "50")
    err, bits, per = eng.run_points(pts, seeds, firsts, ns, [0, 2], True, per_trial=True)
    np.testing.assert_array_equal(per, ref_per)
    np.testing.assert_array_equal(err, ref_err)
    assert np.all(bits[:, 0] == np.asarray(ns) * 256 * 4)


def test_many_small_points_one_launch_and_growing_tables():
    """Thousands of 1-3-trial points (the pinned per-launch tables grow past their first
    size and across the 4096-trial reduction slices), then a small call on the same
    engine: per-point totals equal the per-trial counts, and every trial's counts equal
    a launch of that point alone."""
    cfg = sim.SimConfig(8, 256, 512, 16, ibo_db=1.0, snr_db=12.0)
    eng = engine_for(cfg)
    rng = np.random.default_rng(7)
    base = [_point_of(sim.SimConfig(8, 256, 512, 16, ibo_db=float(i), snr_db=float(s)))
            for i, s in [(0.0, 8.0), (1.0, 12.0), (3.0, 16.0), (6.0, 10.0)]]
    small_err, _, small_per = eng.run_points(base[:2], [1, 2], [0, 0], [3, 2], [0, 1], False, per_trial=True)
    n = 3000
    kinds = rng.integers(0, len(base), n)
    pts = [base[k] for k in kinds]
    ns = rng.integers(1, 4, n)
    seeds = [int(x) for x in rng.integers(1, 1 << 40, n)]
    firsts = [int(x) for x in rng.integers(0, 1 << 20, n)]
    err, bits, per = eng.run_points(pts, seeds, firsts, [int(x) for x in ns], [0, 1], False, per_trial=True)
    assert per.shape == (int(ns.sum()), 2)
    got = np.split(per, np.cumsum(ns)[:-1])
    for i in range(n):
        np.testing.assert_array_equal(err[i], got[i].sum(0))
        assert np.all(bits[i] == ns[i] * 256 * 4)
    for i in rng.choice(n, 12, replace=False):  # spot checks against one-point launches
        _, _, ref = eng.run_points([pts[i]], [seeds[i]], [firsts[i]], [int(ns[i])], [0, 1], False, per_trial=True)
        np.testing.assert_array_equal(got[i], ref)
    err2, _, per2 = eng.run_points(base[:2], [1, 2], [0, 0], [3, 2], [0, 1], False, per_trial=True)
    np.testing.assert_array_equal(per2, small_per)
    np.testing.assert_array_equal(err2, small_err)

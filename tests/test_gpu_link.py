"""Link.simulate drop-in on the GPU: counter semantics, equality with the engine, BER
sanity against closed form (BASELINE config 1 plumbing) and the reference's CSV point."""
import ctypes
import multiprocessing as mp

import numpy as np
import pytest
from scipy import special

from link_util import build_link

pytestmark = pytest.mark.gpu


def shared(n):
    return mp.Array(ctypes.c_double, n, lock=True), mp.Array(ctypes.c_double, n, lock=True)


def test_simulate_equals_engine():
    link, mod = build_link(n_ant=8, n_sc=256, n_fft=512, M=16, ibo=1.0, bits_sent_max=1024 * 300,
                           n_err_min=10 ** 12)
    link.set_snr(14.0)
    err, bits = shared(4)
    link.simulate(True, True, np.array([0, 1, 2]), [11, 22, 33], err, bits)
    from mp_model import _seed64
    eng = link.engine()
    e, b, _ = eng.run(_seed64([11, 22, 33]), 0, 300, [0, 1, 2], True)
    np.testing.assert_array_equal(np.asarray(err[:]), e.astype(float))
    np.testing.assert_array_equal(np.asarray(bits[:]), b.astype(float))


@pytest.mark.parametrize("ebn0", [4.0, 8.0, 10.0])
def test_config1_siso_awgn_vs_theory(ebn0):
    """BASELINE config 1: 1 antenna, 64 sc / FFT 128, 16-QAM, ideal PA, LoS (|H| ~ const).
    Gray 16-QAM: BER = 3/8 erfc(sqrt(0.4 Eb/N0)); 1e5+ bits."""
    from utilities import ebn0_to_snr
    link, mod = build_link(n_ant=1, n_sc=64, n_fft=128, M=16, ibo=100.0, chan="los", bits_sent_max=256 * 2000)
    link.set_snr(float(ebn0_to_snr(ebn0, 64, 64, 16)))
    err, bits = shared(2)
    link.simulate(True, True, np.array([0]), [1, 2, 3], err, bits)
    theory = 3 / 8 * special.erfc(np.sqrt(0.4 * 10 ** (ebn0 / 10)))
    ber = np.asarray(err[:]) / np.asarray(bits[:])
    sigma = np.sqrt(theory * 4 / bits[0]) + 1e-6
    assert abs(ber[0] - theory) < 6 * sigma, (ber, theory)
    assert abs(ber[1] - theory) < 6 * sigma, (ber, theory)


def test_published_csv_point_rayleigh():
    """Paper config (64 ant, N_fft 4096, 2048 sc, 64-QAM, IBO 3, Eb/N0 15, Rayleigh):
    published BER no-dist 9.368e-4, std RX 1.076e-3, CNC-1 2.794e-2
    (figs/csv_results/ber_vs_ebn0_cnc_rayleigh_nant64_ibo3_..._niter1_..._8.csv col 11)."""
    from utilities import ebn0_to_snr
    link, mod = build_link(n_ant=64, n_sc=2048, n_fft=4096, M=64, cp=128, ibo=3.0, bits_sent_max=12288 * 2048)
    link.set_snr(float(ebn0_to_snr(15.0, 2048, 2048, 64)))
    err, bits = shared(3)
    link.simulate(True, True, np.array([0, 1]), [7, 8, 9], err, bits)
    ber = np.asarray(err[:]) / np.asarray(bits[:])
    pub = np.array([9.368e-4, 1.076e-3, 2.794e-2])
    # batch-means-free bound: errors are clustered per symbol, allow 6 binomial sigma x 3 (cluster factor)
    sig = np.sqrt(pub / bits[0]) * 3
    print("paper-config BER", ber, "published", pub)
    assert np.all(np.abs(ber - pub) < 6 * sig + 0.03 * pub), (ber, pub)


def test_sweep_grid_on_gpu_equals_per_point_runs():
    """BASELINE config 4 machinery on one GPU: sweep.run_grid == independent per-point runs
    (each point keyed by its grid index, so any sharding gives these numbers)."""
    import sweep
    from utilities import ebn0_to_snr
    link, mod = build_link(n_ant=8, n_sc=256, n_fft=512, M=16, bits_sent_max=1024 * 64, n_err_min=500)
    ibo, ebn0 = [0.0, 2.0], [6.0, 9.0, 12.0]
    err, bits = sweep.run_grid(link, ibo, ebn0, [0, 1], True, seed=11)
    link2, _ = build_link(n_ant=8, n_sc=256, n_fft=512, M=16, bits_sent_max=1024 * 64, n_err_min=500)
    for i, b in enumerate(ibo):
        link2.update_distortion(b)
        for j, e in enumerate(ebn0):
            link2.set_snr(float(ebn0_to_snr(e, 256, 256, 16)))
            ee, bb = shared(3)
            link2.simulate(True, True, np.array([0, 1]), sweep.point_seed(11, i * len(ebn0) + j), ee, bb)
            np.testing.assert_array_equal(err[i, j], np.asarray(ee[:], np.int64))
            np.testing.assert_array_equal(bits[i, j], np.asarray(bb[:], np.int64))
    ber = sweep.ber_from_counts(err, bits)
    assert np.all(np.diff(ber[:, :, 1], axis=1) <= 0)  # BER falls with Eb/N0
    assert np.all(bits[..., 0] >= 1024 * 64) or np.all(err[..., 0] >= 500)


def test_workers_share_counters_like_the_reference_drivers():
    """Two worker processes run Link.simulate into shared mp.Array counters, as the
    reference's drivers do (mp.Process per core, mp_model.py:181-187).  'spawn' because
    this pytest process already holds a HIP context; the drivers fork before any HIP use
    (Link construction is HIP-free, tests/test_link_host.py)."""
    import link_util
    ctx = mp.get_context("spawn")
    per_sym = 256 * 4
    bmax = per_sym * 3000
    link, _ = build_link(n_ant=8, n_sc=256, n_fft=512, M=16, ibo=1.0, bits_sent_max=bmax, n_err_min=10 ** 12)
    link.set_snr(14.0)
    link.max_batch = 512
    err, bits = ctx.Array(ctypes.c_double, 3, lock=True), ctx.Array(ctypes.c_double, 3, lock=True)
    procs = [ctx.Process(target=link_util.simulate_child, args=(link, [s, 5, 6], err, bits)) for s in (1, 2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert [p.exitcode for p in procs] == [0, 0]
    e, b = np.asarray(err[:]), np.asarray(bits[:])
    assert np.all(b >= bmax) and np.all(b <= bmax + 2 * 512 * per_sym), b
    # one process, same point: the BERs agree within sampling error
    err1, bits1 = shared(3)
    link.simulate(True, True, np.array([0, 1]), [3, 5, 6], err1, bits1)
    ber, ber1 = e / b, np.asarray(err1[:]) / np.asarray(bits1[:])
    sig = np.sqrt(ber1 / b) * 4 + 1e-6
    assert np.all(np.abs(ber - ber1) < 6 * sig), (ber, ber1)


CURVES = [("cnc", "rayleigh"), ("mcnc", "rayleigh"), ("cnc", "los"), ("mcnc", "los"), ("cnc", "two_path"),
          ("mcnc", "two_path")]


@pytest.mark.parametrize("receiver,channel", CURVES)
def test_published_curve_paper_config(receiver, channel):
    """The published BER-vs-Eb/N0 curves of the paper config (64 ant, F 4096, 2048 sc, 64-QAM,
    IBO 3 dB; figs/csv_results row layout: axis, no-distortion, standard RX, CNC / MCNC
    iterations 1..8) for every receiver and channel the reference publishes, against the
    engine (float64) at 8,192 trials per point (tools/replay_sigma.py).

    Compared where the published BER >= 1e-4 by z = (ber - pub) / sqrt(s_gpu^2 + s_ref^2):
    s_gpu by batch means over the engine's trials, s_ref as the spread of 24 replicas of the
    reference's own estimator (its stopping rule: bits_sent_max 1e7, n_err_min 1e6, SURVEY
    §6 -> 803-813 trials per point).  North_star's "within Monte-Carlo 1 sigma": measured
    58-77 % of the points within 1 sigma and 92-99 % within 2 sigma, mean z^2 0.7-1.14
    (profiles/r03/stats/replay_sigma.json; a normal sample gives 68 %, 95 %, 1).  The bounds
    leave room for another seed's sampling: >= 50 % within 1 sigma, >= 85 % within 2, mean
    z^2 <= 1.8, max |z| <= 4.5.  (The reference's workers replay one Rayleigh sequence,
    channel.py:209-212: emulating that with 4-32 workers changed none of these numbers by
    more than sampling noise, so the replicas draw independent channels.)

    The z statistics alone would pass a small bias shared by every point (the replica sigma
    is ~3x the engine's), so the bias bounds stay as well: on the compared points the median
    |relative difference| <= 3 % and, per counter row with >= 3 compared points, the mean
    relative difference within +-2 % (round-4 record, profiles/r04/check_g/pytest_gpu.log:
    median 0.11-0.28 %, row means -0.42 ... +0.53 %)."""
    import replay_sigma
    out, _ = replay_sigma.measure(receiver, channel, workers=(1,), reps=24)
    st = out["by_workers"]["1"]
    print(receiver, channel, out["compared"], st, "median |rel|", out["median_abs_rel"], "row mean rel",
          out["row_mean_rel"])
    assert out["compared"] >= 60
    assert st["frac_abs_z_le1"] >= 0.5 and st["frac_abs_z_le2"] >= 0.85
    assert st["mean_z2"] <= 1.8 and st["max_abs_z"] <= 4.5
    assert out["median_abs_rel"] <= 0.03
    for row, bias in out["row_mean_rel"].items():
        assert abs(bias) <= 0.02, (row, bias)


def test_sixteen_workers_share_two_engines(tmp_path, monkeypatch):
    """An unmodified driver forks one worker per core (main_mp_miso_cnc_ber_vs_ebn0.py:36,
    124-132).  16 workers on one GPU: at most MIMO_MAX_ENGINES_PER_DEVICE = 2 of them ever
    create an engine (the others wait without touching the GPU and return when the shared
    counters close), and the BER matches a single-worker run within sampling error."""
    import link_util
    monkeypatch.setenv("MIMO_LOCK_DIR", str(tmp_path))
    monkeypatch.setenv("MIMO_MAX_ENGINES_PER_DEVICE", "2")
    ctx = mp.get_context("spawn")
    per_sym = 256 * 4
    bmax = per_sym * 4000
    link, _ = build_link(n_ant=8, n_sc=256, n_fft=512, M=16, ibo=1.0, bits_sent_max=bmax, n_err_min=10 ** 12,
                         device=0)
    link.set_snr(14.0)
    link.max_batch = 256
    err, bits = ctx.Array(ctypes.c_double, 3, lock=True), ctx.Array(ctypes.c_double, 3, lock=True)
    created = ctx.Value("i", 0)
    procs = [ctx.Process(target=link_util.simulate_child_counting, args=(link, [s, 5, 6], err, bits, created))
             for s in range(16)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert [p.exitcode for p in procs] == [0] * 16
    print("engines created by 16 workers:", created.value)
    assert 1 <= created.value <= 2
    e, b = np.asarray(err[:]), np.asarray(bits[:])
    assert np.all(b >= bmax) and np.all(b <= bmax + 2 * 256 * per_sym), b
    err1, bits1 = shared(3)
    link.simulate(True, True, np.array([0, 1]), [3, 5, 6], err1, bits1)
    ber, ber1 = e / b, np.asarray(err1[:]) / np.asarray(bits1[:])
    sig = np.sqrt(ber1 / b) * 4 + 1e-6
    assert np.all(np.abs(ber - ber1) < 6 * sig), (ber, ber1)

"""CPU tests of the Link drop-in's host logic (no GPU): object state vs the reference's,
HIP-free construction, the stopping rule and counter layout (mp_model.py:133-222), with a
fake engine standing in for libmimo_engine."""
import ctypes
import multiprocessing as mp

import os

import numpy as np
import pytest

from conftest import load_golden
from link_util import build_link
from oracle import refmath as rm


class FakeEngine:
    """Deterministic stand-in: every trial has `e` errors at every index."""

    def __init__(self, bits_per_trial, errs_per_trial=3):
        self.calls = []
        self.bpt = bits_per_trial
        self.e = errs_per_trial

    def run(self, seed, first, n, iters, incl_clean, per_trial=False):
        self.calls.append((seed, first, n, tuple(iters), incl_clean))
        k = len(iters) + (1 if incl_clean else 0)
        return (np.full(k, self.e * n, np.uint64), np.full(k, self.bpt * n, np.uint64), None)


def shared(n):
    return mp.Array(ctypes.c_double, n, lock=True), mp.Array(ctypes.c_double, n, lock=True)


def test_link_state_matches_reference_objects(units):
    """Precoding / PA calibration / AGC attributes equal the reference's for the same H."""
    link, mod = build_link(n_ant=4, n_sc=64, n_fft=128, M=16, ibo=2.0)
    link.my_miso_chan.channel_mat_fd = units["arr_H"]
    link.set_precoding_and_recalculate_agc()
    np.testing.assert_allclose(link.my_array.get_precoding_mat(), units["arr_P"], rtol=1e-12)
    np.testing.assert_allclose([e.impairment.sat_pow for e in link.my_array.array_elements], units["arr_sat"],
                               rtol=1e-12)
    np.testing.assert_allclose(link.ak_hk_vk_agc_nfft, units["arr_ak_agc"], rtol=1e-12)
    np.testing.assert_allclose(link.hk_vk_agc_nfft, units["arr_hk_agc"], rtol=1e-12)
    assert link.ak_hk_vk_noise_scaler == pytest.approx(float(units["arr_ak_noise"]), rel=1e-12)
    pp = link.point_params()
    assert pp["cnc_alpha"] == pytest.approx(float(units["cnc_alpha"]), rel=1e-14)
    assert pp["cnc_sat_pow"] == pytest.approx(float(units["cnc_sat"]), rel=1e-14)


def test_point_params_config2():
    link, mod = build_link(n_ant=64, n_sc=1024, n_fft=2048, M=64, cp=128, ibo=3.0)
    link.set_snr(float(rm.ebn0_to_snr(15, 1024, 1024, 64)))
    pp = link.point_params()
    # sat = 10^(IBO/10) * Es * S/F * mean|P|^2 with mean|P|^2 = 1/A (antenna_array.py:328-360)
    assert pp["sat_pow"] == pytest.approx(10 ** 0.3 * 42 * 0.5 / 64, rel=1e-12)
    assert pp["cnc_sat_pow"] == pytest.approx(41.9005086, rel=1e-7)
    assert pp["cnc_alpha"] == pytest.approx(0.9213017188, rel=1e-9)
    assert pp["avg_symbol_power"] == pytest.approx(42.0)


def test_stopping_rule_bits_budget(monkeypatch):
    link, mod = build_link(bits_sent_max=256 * 40, n_err_min=10 ** 9, device=0)
    fake = FakeEngine(mod.n_bits_per_ofdm_sym)
    monkeypatch.setattr(link, "engine", lambda reroll=True: fake)
    err, bits = shared(1 + 3)
    link.simulate(True, True, np.array([0, 1, 2]), [1, 2, 3], err, bits)
    assert list(bits[:]) == [256 * 40] * 4          # exactly the budget, no overshoot
    assert list(err[:]) == [3 * 40] * 4
    assert sum(c[2] for c in fake.calls) == 40
    firsts = [c[1] for c in fake.calls]
    assert firsts == sorted(firsts) and firsts[0] == 0   # trial ids advance, never reused


def test_stopping_rule_per_index(monkeypatch):
    """Indices that reached n_err_min stop accumulating; the others continue (mp_model.py:181-187)."""
    link, mod = build_link(bits_sent_max=10 ** 9, n_err_min=300, max_batch=16, device=0)

    class Skewed(FakeEngine):
        def run(self, seed, first, n, iters, incl_clean, per_trial=False):
            self.calls.append((seed, first, n, tuple(iters), incl_clean))
            e = [(10 if it == 0 else 1) * n for it in iters]
            if incl_clean:
                e = [1 * n] + e
            return np.asarray(e, np.uint64), np.full(len(e), self.bpt * n, np.uint64), None

    fake = Skewed(mod.n_bits_per_ofdm_sym)
    monkeypatch.setattr(link, "engine", lambda reroll=True: fake)
    err, bits = shared(3)
    link.simulate(True, True, np.array([0, 4]), [5], err, bits)
    assert err[1] >= 300 and err[1] < 300 + 10 * 16      # iteration 0 stopped early
    assert err[0] >= 300 and err[2] >= 300
    assert bits[1] < bits[2]                            # ... while iteration 4 kept running
    assert all(set(c[3]) <= {0, 4} for c in fake.calls)


def test_seed_derivation_distinct():
    from mp_model import _seed64
    assert _seed64([1, 2, 3]) != _seed64([1, 2, 4])
    assert _seed64([1, 2, 3]) == _seed64(np.array([1, 2, 3]))


def test_link_construction_is_hip_free(monkeypatch):
    """Drivers fork after building Link: construction / update_distortion / set_snr must not call HIP."""
    import _engine

    def boom(*a, **k):
        raise AssertionError("HIP touched during Link construction")

    monkeypatch.setattr(_engine, "lib", boom)
    link, _ = build_link(is_mcnc=True)
    link.update_distortion(2.0)
    link.set_snr(12.0)
    link2, _ = build_link(csi=0.2)
    link2.set_precoding_and_recalculate_agc()


def test_link_pickles_without_engine():
    import pickle
    link, _ = build_link()
    link._engine = object()
    state = pickle.loads(pickle.dumps(link.__getstate__()))
    assert state["_engine"] is None


def test_unsupported_channels_raise():
    """QuaDRiGa / random-paths channel objects are rejected at Link construction."""
    import copy
    import mp_model

    class MisoQuadrigaFd:
        channel_mat_fd = None

    link, mod = build_link()
    with pytest.raises(NotImplementedError):
        mp_model.Link(mod_obj=mod, array_obj=link.my_array, std_rx_obj=link.my_standard_rx,
                      chan_obj=MisoQuadrigaFd(), noise_obj=copy.deepcopy(link.my_noise), rx_loc_var=10.0,
                      n_err_min=10, bits_sent_max=100)


@pytest.mark.parametrize("chan", ["rayleigh", "los", "two_path"])
def test_fixed_channel_uses_the_channel_objects_matrix(monkeypatch, chan):
    """simulate(reroll_chan=False) (mp_model.py:190-206): every trial sees the channel
    object's current matrix -> a table-channel engine built from channel_mat_fd."""
    import _engine
    seen = {}

    class Capture:
        def __init__(self, *a, **k):
            seen["args"], seen["kw"] = a, k

        def set_point(self, *a, **k):
            pass

    monkeypatch.setattr(_engine, "Engine", Capture)
    link, _ = build_link(chan=chan, device=0)
    link.engine(reroll_chan=False)
    assert seen["args"][5] == "table"
    np.testing.assert_array_equal(seen["kw"]["chan_table"], link.my_miso_chan.channel_mat_fd)
    link.engine(reroll_chan=True)
    assert seen["args"][5] == chan and seen["kw"]["chan_table"] is None


def _slot_child(dev, q):
    import mp_model
    q.put(mp_model.acquire_device_slot(dev))
    import time
    time.sleep(1.0)  # hold the slot while the siblings try


def test_device_slots_cap_engines_per_device(tmp_path, monkeypatch):
    """At most MIMO_MAX_ENGINES_PER_DEVICE processes hold a slot of one device; a slot is
    per process (re-acquiring is a no-op) and other devices have their own slots."""
    import mp_model
    monkeypatch.setenv("MIMO_LOCK_DIR", str(tmp_path))
    monkeypatch.setenv("MIMO_MAX_ENGINES_PER_DEVICE", "2")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_slot_child, args=(0, q)) for _ in range(5)]
    for p in procs:
        p.start()
    got = [q.get(timeout=60) for _ in procs]
    for p in procs:
        p.join(60)
    assert sorted(got) == [False, False, False, True, True]
    # all holders exited: the slots are free again; this process takes one, twice
    assert mp_model.acquire_device_slot(0) and mp_model.acquire_device_slot(0)
    assert mp_model.acquire_device_slot(1)


def test_waiting_worker_returns_when_point_is_done(tmp_path, monkeypatch):
    """A worker that finds its device's slots taken never creates an engine; it returns once
    the shared counters are closed (here: already closed)."""
    import mp_model
    monkeypatch.setenv("MIMO_LOCK_DIR", str(tmp_path))
    monkeypatch.setattr(mp_model, "acquire_device_slot", lambda dev: False)
    link, _ = build_link(bits_sent_max=1000, n_err_min=10, device=0)
    monkeypatch.setattr(link, "engine", lambda reroll=True: (_ for _ in ()).throw(AssertionError("engine created")))
    err, bits = shared(2)
    err[0] = err[1] = 20.0
    link.simulate(False, True, np.array([0, 1]), [1], err, bits)


def test_private_counters_never_wait_for_a_slot(tmp_path, monkeypatch):
    """a caller with private counters (not an mp.Array) does not wait for a slot
    (nobody else would close its counters): it goes straight to the engine."""
    import mp_model
    monkeypatch.setenv("MIMO_LOCK_DIR", str(tmp_path))
    monkeypatch.setattr(mp_model, "acquire_device_slot", lambda dev: False)
    link, _ = build_link(bits_sent_max=1000, n_err_min=10, device=0)
    called = []

    def fake_engine(reroll=True):
        called.append(reroll)
        raise RuntimeError("engine reached")
    monkeypatch.setattr(link, "engine", fake_engine)
    with pytest.raises(RuntimeError, match="engine reached"):
        link.simulate(False, True, np.array([0, 1]), [1], np.zeros(2), np.zeros(2))
    assert called == [True]


def test_slot_wait_is_bounded_when_counters_stall(tmp_path, monkeypatch):
    """Shared counters that make no progress while every slot is held by other processes:
    the worker stops waiting after the stall time and creates its engine anyway."""
    import mp_model
    monkeypatch.setattr(mp_model, "acquire_device_slot", lambda dev: False)
    with pytest.warns(UserWarning, match="MIMO_MAX_ENGINES_PER_DEVICE"):
        assert mp_model.wait_for_device_slot(0, lambda: True, lambda: (0.0, 0.0), stall_s=0.1)
    # counters that close while waiting: False (nothing left to do)
    state = {"n": 0}

    def still_open():
        state["n"] += 1
        return state["n"] < 5
    assert not mp_model.wait_for_device_slot(0, still_open, lambda: state["n"], stall_s=60)


def _slow_holder(lock_dir, beat, hold_s, q):
    """A slot holder whose counters do not move for hold_s (engine set-up, a long first
    batch); with beat it touches its slot's heartbeat every 0.2 s."""
    import os
    import time
    os.environ["MIMO_LOCK_DIR"] = lock_dir
    os.environ["MIMO_MAX_ENGINES_PER_DEVICE"] = "1"
    import mp_model
    q.put(mp_model.acquire_device_slot(0))
    if beat == "thread":
        # one long blocking call (a launch, GIL released) inside simulate()'s heartbeat thread
        with mp_model.SlotHeartbeat(0, period_s=0.2):
            time.sleep(hold_s)
        return
    if beat == "hung":
        # a holder hung inside its loop -- the heartbeat thread runs, but no batch
        # completes (no progress()) for longer than the work bound: it must fall silent
        with mp_model.SlotHeartbeat(0, period_s=0.2, max_work_s=0.5):
            time.sleep(hold_s)
        return
    t0 = time.monotonic()
    while time.monotonic() - t0 < hold_s:
        if beat:
            mp_model.slot_heartbeat(0)
        time.sleep(0.2)


@pytest.mark.parametrize("beat", [True, False, "thread", "hung"])
def test_slot_wait_counts_holder_heartbeats_as_progress(tmp_path, monkeypatch, beat):
    """a holder whose first batch outlasts the stall time still counts as working
    when it beats its slot's heartbeat: the waiter keeps waiting (no extra engine) and takes
    the slot when the holder exits.  Without heartbeats the waiter gives up after stall_s --
    and so it does when the holder's heartbeat thread runs but its batch has not
    completed within the work bound (a holder hung in a launch): the beats stop."""
    import time
    import warnings
    import mp_model
    monkeypatch.setenv("MIMO_LOCK_DIR", str(tmp_path))
    monkeypatch.setenv("MIMO_MAX_ENGINES_PER_DEVICE", "1")
    monkeypatch.setattr(mp_model, "_SLOTS", {})  # this process holds no slot yet
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    hold = 3.0
    p = ctx.Process(target=_slow_holder, args=(str(tmp_path), beat, hold, q))
    p.start()
    assert q.get(timeout=60) is True
    t0 = time.monotonic()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        got = mp_model.wait_for_device_slot(0, lambda: True, lambda: (0.0, 0.0), stall_s=1.0, poll_s=0.05)
    waited = time.monotonic() - t0
    p.join(60)
    assert got is True
    gave_up = any("MIMO_MAX_ENGINES_PER_DEVICE" in str(x.message) for x in w)
    if beat == "hung":
        # silent from 0.5 s on: the waiter escapes ~stall_s later, well before the holder exits
        assert gave_up and waited < hold - 0.5, waited
    elif beat:
        assert not gave_up and waited >= hold - 0.5, (waited, [str(x.message) for x in w])
        assert (os.getpid(), 0) in mp_model._SLOTS  # the freed slot is now this process's
    else:
        assert gave_up and waited < hold - 0.5, waited


def test_simulate_points_rejects_counters_it_cannot_add_into(monkeypatch):
    """simulate_points adds into n_err / n_bits in place; a list or another dtype
    would be copied and the totals lost, so it raises instead."""
    link, _ = build_link(bits_sent_max=1000, n_err_min=10, device=0)
    link.set_snr(10.0)
    monkeypatch.setattr(link, "engine", lambda reroll=True: object())
    pp = [link.point_params()]
    with pytest.raises(TypeError, match="float64 ndarray"):
        link.simulate_points(False, True, [0, 1], [[1]], pp, [[0.0, 0.0]], np.zeros((1, 2)))
    with pytest.raises(TypeError, match="float64 ndarray"):
        link.simulate_points(False, True, [0, 1], [[1]], pp, np.zeros((1, 2)), np.zeros((1, 3)))


def test_multi_user_is_rejected_explicitly():
    """Multi-user OFDM / MU-MR / MU-ZF (modulation.py:363-382, antenna_array.py:188-305) are
    not part of this build: they raise instead of running unverified code."""
    import numpy as np
    import modulation
    with pytest.raises(NotImplementedError):
        modulation.OfdmQamModem(constel_size=16, n_fft=128, n_sub_carr=64, cp_len=4, n_users=2)
    link, _ = build_link()
    h = link.my_miso_chan.channel_mat_fd
    with pytest.raises(NotImplementedError):
        link.my_array.set_precoding_matrix([h, h], mr_precoding=True)


def test_next_batch_rows_equals_next_batch():
    """simulate_points' vectorised stopping rule gives every point exactly next_batch's batch
    (pilot, doubling, rate-based need, bit budget, max_batch), including closed counters,
    zero-error and zero-bit counters."""
    import mp_model
    rng = np.random.default_rng(5)
    nbps, nmin, bmax = 12288, 100000, 5_000_000
    for trial in range(200):
        P, n_idx = 37, 5
        bits = rng.choice([0.0, 12288.0 * 64, 12288.0 * 300, 4.99e6, 5.0e6, 6e6], size=(P, n_idx))
        err = np.where(rng.random((P, n_idx)) < 0.2, 0.0, np.floor(bits * rng.choice([1e-4, 1e-2, 0.05, 0.3], (P, n_idx))))
        act = (err < nmin) & (bits < bmax)
        got = mp_model.next_batch_rows(err, bits, act, nbps, nmin, bmax, 65536)
        for i in range(P):
            if act[i].any():
                assert got[i] == mp_model.next_batch(err[i], bits[i], act[i], nbps, nmin, bmax, 65536), (i, err[i], bits[i])


def test_fixed_toi_array_alpha_is_an_engine_level_parameter():
    """the TOI drivers' one-gain AGC (alpha_estimate, main_miso_cnc_ber_vs_ebn0_toi.py:
    95-121,247-249) does not run through Link: those drivers inline their loop, and the
    reference's Link cannot hold a TOI array at all -- it reads impairment.ibo_db
    (mp_model.py:83), which ThirdOrderNonLin lacks; the mirror fails the same way.  The fixed
    gain is therefore engine-level: the TOI path (tools/published_families.points, the drivers'
    restatement) passes it as mimo_point.array_alpha on every point, and make_point carries it."""
    import _engine
    import published_families as pf
    with pytest.raises(AttributeError, match="ibo_db"):
        build_link(n_ant=4, pa="toi", ibo=22.75)
    c = dict(next(c for c in pf.CURVES if c["family"] == "toi" and c["n_ant"] == 1 and c["toi"] == 22.75))
    _, pts = pf.points(c, np.array([10.0, 15.0]))
    assert 0.98 < c["alpha_estimate"] < 1.0
    for pp in pts:
        assert pp["pa_kind"] == "toi" and pp["array_alpha"] == c["alpha_estimate"] == pp["cnc_alpha"]
        assert _engine.Engine.make_point(**pp).array_alpha == c["alpha_estimate"]

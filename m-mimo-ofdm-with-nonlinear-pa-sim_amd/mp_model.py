"""``Link`` -- the coarse drop-in seam (reference mp_model.py:16-329), MI355X build.

Same constructor, methods and counter semantics as the reference, so the
``main_mp_*`` drivers run unchanged with this directory first on ``sys.path``:
``Link.simulate`` hands batches of trials to the fused HIP kernel
(``libmimo_engine.so``: channel reroll, MRT, PA, FFTs, AWGN, AGC, CNC/MCNC, bit-error
count all on the GPU) and adds the per-index totals into the caller's shared
``mp.Array`` counters under their lock, with the reference's stopping rule
(mp_model.py:137-138, 177-187).

Differences, by design:
* randomness: Philox streams keyed by ``seed_arr`` and addressed by trial index
  instead of PCG64 generators; every forked process therefore gets independent
  channels (the reference replays one Rayleigh sequence in all processes, channel.py:209-212);
* a clean-run trial reuses its distorted trial's draws (no PA: the IFFT->FFT round
  trip is the identity in-band), so both counters see the same channels and noise;
* trials run in batches (one kernel launch each) sized by ``next_batch``: a pilot
  batch, then the number of trials the open counters still need to reach
  ``n_err_min`` at their observed error rate (+5 %), never past ``bits_sent_max``;
  the reference checks after every symbol and overshoots by up to num_cores symbols.

``simulate_points`` runs the same trial loop for many grid points at once (one launch
per round over every open point, ``mimo_engine_run_points``): bit-identical to calling
``simulate`` point by point with the same seeds.
"""
from __future__ import annotations

import copy
import multiprocessing
import os
import tempfile
import time

import numpy as np
from numpy import ndarray

import _engine
import channel
import corrector
import distortion
from antenna_array import AntennaArray, sc_columns
from modulation import OfdmQamModem
from transceiver import Transceiver

MAX_BATCH = 1 << 16
PILOT = 64


def next_batch(err, bits, act, n_bits_per_sym, n_err_min, bits_sent_max, max_batch=MAX_BATCH, pilot=PILOT):
    """Trials of the next batch of one grid point under the reference's stopping rule
    (mp_model.py:137-138,177-187: a counter stays open while n_err < n_err_min and
    bits < bits_sent_max; all counters share the trials).  ``act`` marks the open counters.

    Never crosses ``bits_sent_max`` of the most advanced open counter.  Before any error
    is seen, a pilot batch; then the trials the slowest open counter needs to reach
    ``n_err_min`` at its observed rate, +5 %."""
    err = np.asarray(err, dtype=np.float64)
    bits = np.asarray(bits, dtype=np.float64)
    act = np.asarray(act, dtype=bool)
    open_bits = bits[act] if act.any() else bits
    budget = max(1, int(np.ceil((bits_sent_max - float(np.max(open_bits))) / n_bits_per_sym)))
    need = 0
    for e, b in zip(err[act], bits[act]):
        if e <= 0 or b <= 0:
            need = max(need, max(pilot, int(2 * b / n_bits_per_sym)))  # no rate yet: pilot / doubling
        else:
            rate = e / (b / n_bits_per_sym)  # errors per trial
            need = max(need, int(np.ceil(1.05 * (n_err_min - e) / rate)) + 1)
    return int(max(1, min(max_batch, budget, max(need, min(pilot, budget)))))


def next_batch_rows(err, bits, act, n_bits_per_sym, n_err_min, bits_sent_max, max_batch=MAX_BATCH, pilot=PILOT):
    """``next_batch`` for many points at once (rows of err / bits / act, float64 [P, n_idx]):
    the same float64 expressions elementwise, so every row's batch equals next_batch's
    (tests/test_link_host.py).  Rows without an open counter get a value too; callers skip
    them."""
    err = np.asarray(err, dtype=np.float64)
    bits = np.asarray(bits, dtype=np.float64)
    act = np.asarray(act, dtype=bool)
    any_act = act.any(axis=1)
    open_max = np.where(any_act, np.max(np.where(act, bits, -np.inf), axis=1), np.max(bits, axis=1))
    budget = np.maximum(1, np.ceil((bits_sent_max - open_max) / n_bits_per_sym).astype(np.int64))
    with np.errstate(divide="ignore", invalid="ignore"):
        no_rate = (err <= 0) | (bits <= 0)
        first = np.maximum(pilot, np.floor(2 * bits / n_bits_per_sym).astype(np.int64))
        rate = err / (bits / n_bits_per_sym)
        more = np.ceil(1.05 * (n_err_min - err) / rate)
        more = np.where(no_rate, 0, more).astype(np.int64) + 1
    need_c = np.where(no_rate, first, more)
    need = np.max(np.where(act, need_c, 0), axis=1)
    need = np.maximum(need, 0)
    return np.maximum(1, np.minimum(np.minimum(max_batch, budget), np.maximum(need, np.minimum(pilot, budget))))


def _seed64(seed_arr) -> int:
    ss = np.random.SeedSequence([int(s) & 0xFFFFFFFFFFFFFFFF for s in np.atleast_1d(seed_arr)])
    w = ss.generate_state(2, np.uint32)
    return int(w[0]) | (int(w[1]) << 32)


def _device_count():
    """GPUs visible to this process, counted without creating a HIP context where possible
    (torch's counter does not initialise the GPU on ROCm; the HIP runtime is the fallback)."""
    env = os.environ.get("MIMO_DEVICE_COUNT")
    if env:
        return int(env)
    try:
        import torch
        n = torch.cuda.device_count()
        if n > 0:
            return n
    except Exception:  # torch absent or without ROCm: ask the engine library
        pass
    return _engine.lib().mimo_device_count()


def _default_device():
    """Device for this process: mp child k -> GPU k % n (drivers fork one Link per core)."""
    ident = getattr(multiprocessing.current_process(), "_identity", ())
    n = _device_count()
    if n < 1:
        raise _engine.EngineError("no HIP device visible")
    return (ident[0] - 1) % n if ident else 0


# ---------------------------------------------------------------- engines per device
# The reference's drivers fork num_cores = mp.cpu_count() workers per grid point
# (main_mp_miso_cnc_ber_vs_ebn0.py:36,124-132); on a many-core MI355X host an unmodified
# driver would open dozens of HIP contexts per GPU.  A worker therefore takes one of
# MIMO_MAX_ENGINES_PER_DEVICE (default 2) slots of its device before it creates an engine:
# POSIX record locks on per-(device, slot) files, held by the process (released when it
# exits, never inherited by fork children).  Workers without a slot wait, touching no GPU,
# and return as soon as the shared counters say the point is done.
_SLOTS = {}  # (pid, device) -> fd of the held slot


def _slot_dir():
    d = os.environ.get("MIMO_LOCK_DIR") or os.path.join(tempfile.gettempdir(), "mimo_engine_slots_%d" % os.getuid())
    os.makedirs(d, exist_ok=True)
    return d


def acquire_device_slot(dev: int) -> bool:
    """Take (or confirm) this process's engine slot on ``dev``; False if all are taken."""
    import fcntl
    key = (os.getpid(), int(dev))
    if key in _SLOTS:
        return True
    cap = max(1, int(os.environ.get("MIMO_MAX_ENGINES_PER_DEVICE", "2")))
    d = _slot_dir()
    for k in range(cap):
        fd = os.open(os.path.join(d, "dev%d_slot%d.lock" % (dev, k)), os.O_RDWR | os.O_CREAT, 0o600)
        try:
            fcntl.lockf(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            os.close(fd)
            continue
        _SLOTS[key] = fd
        return True
    return False


def slot_heartbeat(dev: int) -> None:
    """A slot holder's sign of life: touch its lock file (``SlotHeartbeat`` does it every
    second while ``simulate`` runs), so that waiting workers see progress even while the
    holder's first batch -- engine creation, a 65,536-trial launch of a large array -- has
    not yet moved the shared counters."""
    fd = _SLOTS.get((os.getpid(), int(dev)))
    if fd is not None:
        try:
            os.utime(fd)
        except OSError:
            pass


class SlotHeartbeat:
    """Beats this process's slot heartbeat every ``period_s`` (MIMO_SLOT_HEARTBEAT_S, default
    1 s) from a daemon thread while the block runs, so that one long launch -- the engine
    call releases the GIL -- still reads as progress to waiting workers (beats
    only before set-up and after each batch let a first batch longer than the stall time
    trigger the waiters' escape).

    The beats are tied to bounded work: the thread beats only while the work
    since the last ``progress()`` call -- engine set-up plus the first batch, then one batch --
    is younger than ``max_work_s`` (MIMO_SLOT_MAX_LAUNCH_S, default 120 s; a 65,536-trial batch
    of the largest array takes ~1 s).  A holder hung inside a launch or anywhere in its loop
    then falls silent, and the waiters' stall escape (wait_for_device_slot) fires again."""

    def __init__(self, dev: int, period_s: float = None, max_work_s: float = None):
        import threading
        self.dev = int(dev)
        self.period_s = float(os.environ.get("MIMO_SLOT_HEARTBEAT_S", "1.0")) if period_s is None else period_s
        self.max_work_s = float(os.environ.get("MIMO_SLOT_MAX_LAUNCH_S", "120")) if max_work_s is None else max_work_s
        self._t_work = time.monotonic()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True)

    def progress(self):
        """A unit of work (a batch) completed: beat now and restart the work clock."""
        self._t_work = time.monotonic()
        slot_heartbeat(self.dev)

    def _run(self):
        while not self._stop.wait(self.period_s):
            if time.monotonic() - self._t_work <= self.max_work_s:
                slot_heartbeat(self.dev)

    def __enter__(self):
        self.progress()
        self._thread.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._thread.join()
        return False


def slot_activity(dev: int) -> int:
    """Latest heartbeat (lock-file mtime, ns) of ``dev``'s slots; 0 if none.  Any holder's
    beat counts, including a holder busy with other counters (another grid point, another
    driver sharing the lock directory): a waiter then keeps waiting until such holders
    finish their runs instead of creating an extra engine.  Bounded: a holder beats only
    while its current batch is younger than MIMO_SLOT_MAX_LAUNCH_S (SlotHeartbeat), so a hung
    holder falls silent and the waiter's stall escape fires; a holder's slot is released
    when its process exits."""
    d = _slot_dir()
    cap = max(1, int(os.environ.get("MIMO_MAX_ENGINES_PER_DEVICE", "2")))
    latest = 0
    for k in range(cap):
        try:
            latest = max(latest, os.stat(os.path.join(d, "dev%d_slot%d.lock" % (dev, k))).st_mtime_ns)
        except OSError:
            pass
    return latest


def wait_for_device_slot(dev: int, still_open, progress, stall_s: float = None, poll_s: float = 0.02) -> bool:
    """Wait for an engine slot on ``dev`` while the shared counters are open.  Returns False
    when the counters closed (the slot holders finished the point: nothing left to do), True
    once a slot is held -- or when neither the counters nor the slot holders' heartbeats
    (slot_heartbeat) moved for ``stall_s`` seconds (MIMO_SLOT_STALL_S, default 30): the slots
    are then held by processes that do not work, and this worker creates its engine beyond
    MIMO_MAX_ENGINES_PER_DEVICE rather than wait forever."""
    stall_s = float(os.environ.get("MIMO_SLOT_STALL_S", "30")) if stall_s is None else stall_s
    base = progress

    def progress():
        return (base(), slot_activity(dev))
    last, t_last = progress(), time.monotonic()
    while not acquire_device_slot(dev):
        if not still_open():
            return False
        now = progress()
        if now != last:
            last, t_last = now, time.monotonic()
        elif time.monotonic() - t_last > stall_s:
            import warnings
            warnings.warn(f"no engine slot on device {dev} and no progress on the shared counters for "
                          f"{stall_s:.0f} s: creating an engine beyond MIMO_MAX_ENGINES_PER_DEVICE")
            return True
        time.sleep(poll_s)
    return still_open()  # a slot freed because its holder finished the point: maybe done


def _all_reduce_counts(dist, e, b, device=None):
    """Sum one round's [points, counters] error / bit counts over the ranks (int64; on the
    rank's GPU when the process group is RCCL's)."""
    import torch
    t = torch.from_numpy(np.stack([np.asarray(e, np.int64), np.asarray(b, np.int64)]))
    if dist.get_backend() == "nccl":
        t = t.to(torch.device("cuda", int(device) if device is not None else torch.cuda.current_device()))
    dist.all_reduce(t)
    t = t.cpu().numpy()
    return t[0], t[1]


class Link:
    """(mp_model.py:16-87)"""

    def __init__(self, mod_obj: OfdmQamModem, array_obj: AntennaArray, std_rx_obj: Transceiver, chan_obj, noise_obj,
                 rx_loc_var: float, n_err_min: int, bits_sent_max: int, is_mcnc: bool = False,
                 csi_epsylon: float = None, device: int = None, max_batch: int = MAX_BATCH, precision: str = None):
        self.my_mod = copy.deepcopy(mod_obj)
        self.my_array = copy.deepcopy(array_obj)
        self.my_standard_rx = copy.deepcopy(std_rx_obj)
        self.rx_loc_x = self.my_standard_rx.cord_x
        self.rx_loc_y = self.my_standard_rx.cord_y
        self.my_noise = copy.deepcopy(noise_obj)
        self.my_csi_noise = copy.deepcopy(noise_obj)
        self.csi_epsylon = csi_epsylon
        if not isinstance(chan_obj, (channel.MisoRayleighFd, channel.MisoLosFd, channel.MisoTwoPathFd)):
            raise NotImplementedError(f"{type(chan_obj).__name__} is out of scope (MATLAB / NumPy-1 channels)")
        self.is_quadriga = False
        self.my_miso_chan = copy.deepcopy(chan_obj)
        if self.csi_epsylon is not None:
            self.my_miso_chan_csi_err = copy.deepcopy(self.my_miso_chan)
        self.is_mcnc = is_mcnc
        if is_mcnc:
            self.my_cnc_rx = corrector.McncReceiver(self.my_array, self.my_miso_chan, _host_setup=True)
        else:
            self.my_cnc_rx = corrector.CncReceiver(copy.deepcopy(array_obj.base_transceiver.modem),
                                                   copy.deepcopy(array_obj.base_transceiver.impairment))
        self.my_noise.rng_gen = np.random.default_rng(0)
        self.loc_rng = np.random.default_rng(1)
        self.bit_rng = np.random.default_rng(2)
        self.my_csi_noise.rng_gen = np.random.default_rng(3)
        # the fixed-channel (reroll_chan=False) CSI estimate is the Link's: Link.__init__ draws
        # it once, in set_precoding_and_recalculate_agc, from self.my_noise.rng_gen, which it
        # has just seeded with default_rng(0) (mp_model.py:74,87,272 -- not my_csi_noise, seed
        # 3, which the reference never draws from).  Its Philox key (0 as in that seed, 0xC51 a
        # stream tag), shared by every worker and every simulate() call whatever their seed_arr
        self.csi_seed = _seed64([0, 0xC51])
        self.rx_loc_var = rx_loc_var
        self.n_ant_val = len(self.my_array.array_elements)
        self.n_bits_per_ofdm_sym = self.my_mod.n_bits_per_ofdm_sym
        self.n_sub_carr = self.my_mod.n_sub_carr
        self.ibo_val_db = self.my_array.array_elements[0].impairment.ibo_db
        self.n_err_min = n_err_min
        self.bits_sent_max = bits_sent_max
        self.device = device
        self.precision = precision  # "f64" (default: the reference's float64) or "f32"
        self.max_batch = int(max_batch)
        self._engine = None
        self._engine_key = None
        self.set_precoding_and_recalculate_agc()

    # ------------------------------------------------------------------ engine plumbing
    def _chan_kind(self):
        if isinstance(self.my_miso_chan, channel.MisoRayleighFd):
            return "rayleigh"
        if isinstance(self.my_miso_chan, channel.MisoTwoPathFd):
            return "two_path"
        return "los"

    def engine(self, reroll_chan: bool = True):
        """The configured GPU engine for the current grid point (created lazily, per process).

        ``reroll_chan=False`` (mp_model.py:190-206: every trial sees the channel object's
        current matrix) runs the table-channel instances on ``channel_mat_fd``."""
        kind = self._chan_kind()
        table = None
        if not reroll_chan:
            table = np.asarray(self.my_miso_chan.channel_mat_fd, dtype=np.complex128)
            kind = "table"
        dev = self.device if self.device is not None else _default_device()
        acquire_device_slot(dev)  # best effort here; simulate() waits for a slot
        key = (dev, kind, bool(reroll_chan), self.is_mcnc, self.precision,
               None if table is None else hash(table.tobytes()))
        if self._engine is None or self._engine_key != key:
            m = self.my_mod
            rx = self.my_standard_rx
            self._engine = _engine.Engine(
                self.n_ant_val, m.n_sub_carr, m.n_fft, m.constel_size, m.cp_len, kind,
                "mcnc" if self.is_mcnc else "cnc", self.my_array.positions(),
                (self.rx_loc_x, self.rx_loc_y, rx.cord_z), self.rx_loc_var,
                channel.carrier_freqs(m.n_fft, rx.carrier_spacing, rx.center_freq), reroll=reroll_chan, device=dev,
                precision=self.precision, chan_table=table, csi_seed=self.csi_seed if table is not None else 0)
            self._engine_key = key
        self._push_point()
        return self._engine

    def point_params(self) -> dict:
        """The per-point scalars the reference keeps in its objects."""
        kind, sat, p, toi = distortion.pa_params(self.my_array.array_elements[0].impairment)
        if self.is_mcnc:
            ck, csat, cp, ctoi, calpha = kind, sat, p, toi, 1.0
        else:
            ck, csat, cp, ctoi = distortion.pa_params(self.my_cnc_rx.impairment)
            calpha = float(self.my_cnc_rx.modem.alpha)
        return dict(ibo_db=float(self.ibo_val_db), snr_db=float(self.my_noise.snr_db),
                    avg_symbol_power=float(self.my_mod.avg_symbol_power), pa_kind=kind, sat_pow=sat, p_hardness=p,
                    toi_coeff=toi, cnc_pa_kind=ck, cnc_sat_pow=csat, cnc_toi_coeff=ctoi, cnc_alpha=calpha,
                    csi_eps=self.csi_epsylon)

    def _push_point(self):
        pp = self.point_params()
        if pp["snr_db"] is None:
            raise ValueError("set_snr() must be called before simulate()")
        self._engine.set_point(**pp)

    def __getstate__(self):  # engines (device handles) never travel to another process
        d = self.__dict__.copy()
        d["_engine"] = None
        d["_engine_key"] = None
        return d

    # ------------------------------------------------------------------ reference API
    def simulate(self, incl_clean_run: bool, reroll_chan: bool, cnc_n_iter_lst: list, seed_arr: list,
                 n_err_shared_arr, n_bits_sent_shared_arr) -> None:
        """Monte-Carlo trial loop on the GPU (mp_model.py:89-228)."""
        err_np = np.frombuffer(n_err_shared_arr.get_obj()) if hasattr(n_err_shared_arr, "get_obj") else None

        def still_open():
            err = np.asarray(err_np if err_np is not None else n_err_shared_arr[:], dtype=np.float64)
            bits = np.asarray(n_bits_sent_shared_arr[:], dtype=np.float64)
            return bool(np.any((err < self.n_err_min) & (bits < self.bits_sent_max)))

        dev = self.device if self.device is not None else _default_device()
        if err_np is not None:
            # Shared counters (the drivers' mp.Array): other workers of this point may own the
            # device's engines, so wait for a slot while they make progress on the counters.
            if not wait_for_device_slot(dev, still_open, lambda: (float(np.sum(err_np)),
                                                                  float(np.sum(n_bits_sent_shared_arr[:])))):
                return
        else:
            acquire_device_slot(dev)  # private counters: nobody else closes them, never wait
        with SlotHeartbeat(dev) as beat:
            self._simulate_loop(incl_clean_run, reroll_chan, cnc_n_iter_lst, seed_arr, n_err_shared_arr,
                                n_bits_sent_shared_arr, err_np, beat)

    def _simulate_loop(self, incl_clean_run, reroll_chan, cnc_n_iter_lst, seed_arr, n_err_shared_arr,
                       n_bits_sent_shared_arr, err_np, beat=None):
        eng = self.engine(reroll_chan)
        seed = _seed64(seed_arr)
        iters_all = np.asarray(cnc_n_iter_lst, dtype=np.int64).reshape(-1)
        order = np.argsort(iters_all, kind="stable")
        res_idx = 1 if incl_clean_run else 0
        trial = 0
        while True:
            err = np.asarray(err_np if err_np is not None else n_err_shared_arr[:], dtype=np.float64)
            bits = np.asarray(n_bits_sent_shared_arr[:], dtype=np.float64)
            act = (err < self.n_err_min) & (bits < self.bits_sent_max)
            clean_on = bool(incl_clean_run and act[0])
            flags = act[res_idx:]
            if not clean_on and not flags.any():
                break
            idx = [res_idx + int(i) for i in order if flags[i]]
            run_iters = [int(iters_all[i]) for i in order if flags[i]]
            if not run_iters:  # only the clean counter is still open: the engine always runs iteration 0
                run_iters, idx = [0], []
            n = next_batch(err, bits, act, self.n_bits_per_ofdm_sym, self.n_err_min, self.bits_sent_max,
                           self.max_batch)
            uniq = sorted(set(run_iters))
            e, b, _ = eng.run(seed, trial, n, uniq, clean_on)
            if beat is not None:
                beat.progress()  # one batch done: the heartbeat's work clock restarts
            trial += n
            pos = {it: j + (1 if clean_on else 0) for j, it in enumerate(uniq)}
            lock = n_err_shared_arr.get_lock() if hasattr(n_err_shared_arr, "get_lock") else None
            if lock:
                lock.acquire()
            try:
                if clean_on:
                    n_err_shared_arr[0] += float(e[0])
                    n_bits_sent_shared_arr[0] += float(b[0])
                for slot, it in zip(idx, [int(iters_all[i]) for i in order if flags[i]]):
                    n_err_shared_arr[slot] += float(e[pos[it]])
                    n_bits_sent_shared_arr[slot] += float(b[pos[it]])
            finally:
                if lock:
                    lock.release()

    def simulate_points(self, incl_clean_run: bool, reroll_chan: bool, cnc_n_iter_lst, seed_arrs, point_params,
                        n_err, n_bits, stats: dict = None, dist=None) -> None:
        """``simulate`` for many grid points of this system at once (the drivers' grid loops,
        main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:100-215): every round launches one
        batch of every still-open point (mimo_engine_run_points); the counters of point i
        (``n_err[i]``, ``n_bits[i]``: float arrays [n_idx], added to) follow the same stopping
        rule and batch sizes as ``simulate`` would give them, so the totals are bit-identical.
        ``point_params[i]`` is ``point_params()`` captured at point i (after
        update_distortion / set_snr).  ``stats`` (a dict, optional) receives the work record:
        ``trials`` per point, and per round the open points, trials and kernel ms.

        ``dist`` (torch.distributed with a process group, optional): the ranks share every
        point's trials, as the reference's workers share one point's counters
        (mp_model.py:177-187, the mp.Array).  Each round's batch of a point is split into
        contiguous trial ranges, one per rank; the round's counts are summed over the ranks
        (one all_reduce) before the stopping rule reads them, so every rank takes the same
        decisions and the totals are bit-identical to one rank's (the few-points
        alternative to dealing whole points).  Call it with the same points on every rank."""
        eng = self.engine(reroll_chan)
        rank, world = (dist.get_rank(), dist.get_world_size()) if dist is not None else (0, 1)
        P = len(point_params)
        iters_all = np.asarray(cnc_n_iter_lst, dtype=np.int64).reshape(-1)
        uniq = sorted(set(int(i) for i in iters_all))
        res_idx = 1 if incl_clean_run else 0
        col = np.asarray([res_idx + uniq.index(int(i)) for i in iters_all], dtype=np.int64)  # counter -> engine column
        if incl_clean_run:
            col = np.concatenate(([0], col))
        seeds = [_seed64(s) for s in seed_arrs]
        trial = np.zeros(P, dtype=np.int64)
        ran = np.zeros(P, dtype=np.int64)  # trials this rank ran (= trial at world size 1)
        n_idx = len(col)
        for name, arr in (("n_err", n_err), ("n_bits", n_bits)):
            # added to in place: a copy (list, mp.Array, other dtype) would silently drop the totals
            if not (isinstance(arr, np.ndarray) and arr.dtype == np.float64 and arr.shape == (P, n_idx)):
                raise TypeError(f"{name} must be a float64 ndarray of shape ({P}, {n_idx}) (added to in place)")
        for pp in point_params:
            if pp["snr_db"] is None:
                raise ValueError("set_snr() must be called before simulate_points()")
        # the per-point parameter structs once (they do not change between rounds); the
        # stopping rule and the counter updates vectorised over the points (a 915-point grid
        # spent ~50 ms per round in per-point Python otherwise)
        mpoints = [_engine.Engine.make_point(**pp) for pp in point_params]
        seeds_a = np.asarray([s & 0xFFFFFFFFFFFFFFFF for s in seeds], dtype=np.uint64)
        rounds = []
        while True:
            act = (n_err < self.n_err_min) & (n_bits < self.bits_sent_max)
            rows = np.flatnonzero(act.any(axis=1))
            if rows.size == 0:
                break
            n = next_batch_rows(n_err[rows], n_bits[rows], act[rows], self.n_bits_per_ofdm_sym, self.n_err_min,
                                self.bits_sent_max, self.max_batch)
            t0 = time.perf_counter()
            if world == 1:
                e, b, _ = eng.run_points([mpoints[i] for i in rows], seeds_a[rows], trial[rows], n, uniq,
                                         incl_clean_run)
                ran[rows] += n
                k_ms = float(eng.kernel_ms)
            else:
                n = np.asarray(n, dtype=np.int64)
                # this rank's trials of each point: share (rank + point) mod world of the batch, so
                # the batches' remainders rotate over the ranks
                sh = (rank + rows) % world
                lo, hi = n * sh // world, n * (sh + 1) // world
                ran[rows] += hi - lo
                e = np.zeros((rows.size, len(uniq) + res_idx), np.int64)
                b = np.zeros_like(e)
                mine = np.flatnonzero(hi > lo)
                k_ms = 0.0
                if mine.size:
                    em, bm, _ = eng.run_points([mpoints[i] for i in rows[mine]], seeds_a[rows[mine]],
                                               trial[rows[mine]] + lo[mine], (hi - lo)[mine], uniq, incl_clean_run)
                    e[mine], b[mine] = em.astype(np.int64), bm.astype(np.int64)
                    k_ms = float(eng.kernel_ms)
                e, b = _all_reduce_counts(dist, e, b, self.device)
            rounds.append(dict(points=int(rows.size), trials=int(np.sum(n)), kernel_ms=round(k_ms, 3),
                               call_ms=round(1e3 * (time.perf_counter() - t0), 3)))
            if os.environ.get("MIMO_SWEEP_TRACE"):
                import sys
                print("simulate_points round: %d points, %d trials, kernel %.2f ms, call %.2f ms"
                      % (rows.size, int(np.sum(n)), k_ms, 1e3 * (time.perf_counter() - t0)), file=sys.stderr)
            a = act[rows]
            n_err[rows] += np.where(a, e[:, col].astype(np.float64), 0.0)
            n_bits[rows] += np.where(a, b[:, col].astype(np.float64), 0.0)
            trial[rows] += n
        if stats is not None:
            stats.update(trials=trial.copy(), trials_run=ran, rounds=rounds)

    def update_distortion(self, ibo_val_db: float) -> None:
        """(mp_model.py:230-241)"""
        self.my_array.update_distortion(ibo_db=ibo_val_db, avg_sample_pow=self.my_mod.avg_sample_power)
        if isinstance(self.my_cnc_rx, corrector.CncReceiver):
            self.my_cnc_rx.update_distortion(ibo_db=ibo_val_db)
        self.ibo_val_db = self.my_array.array_elements[0].impairment.ibo_db
        self.recalculate_agc(ak_part_only=True)

    def set_snr(self, snr_db_val: float) -> None:
        """(mp_model.py:243-251)"""
        self.my_noise.snr_db = float(snr_db_val)

    def set_precoding_and_recalculate_agc(self) -> None:
        """(mp_model.py:253-288) for the object state (the engine redoes it per trial on the device)."""
        h = self.my_miso_chan.channel_mat_fd
        if self.csi_epsylon is not None:
            n_sc = self.my_mod.n_sub_carr
            noisy = np.copy(h)
            for r, row in enumerate(noisy):
                sc = np.concatenate((row[-n_sc // 2:], row[1:(n_sc // 2) + 1]))
                pw = np.sum(np.abs(sc) ** 2) / len(sc)
                z = self.my_noise.rng_gen.standard_normal((len(sc), 2)).view(np.complex128)[:, 0]
                nsc = np.sqrt(1 - self.csi_epsylon ** 2) * sc + z * 0.5 * np.sqrt(2 * pw) * self.csi_epsylon
                noisy[r, -(n_sc // 2):] = nsc[:n_sc // 2]
                noisy[r, 1:(n_sc // 2) + 1] = nsc[n_sc // 2:]
            self.my_miso_chan_csi_err.channel_mat_fd = noisy
            h = noisy
        self.my_array._set_mrt_state(h)
        self.recalculate_agc(channel_mat_fd=h)

    def recalculate_agc(self, channel_mat_fd: ndarray = None, ak_part_only: bool = False) -> None:
        """(mp_model.py:290-329)"""
        n_sc = self.n_sub_carr
        if not ak_part_only:
            hk = sc_columns(channel_mat_fd, n_sc)
            vk = self.my_array.get_precoding_mat()
            self.vk_pow_vec = np.sum(np.abs(vk) ** 2, axis=1)
            self.hk_vk_agc = hk * vk
            g = np.sum(self.hk_vk_agc, axis=0)
            self.hk_vk_noise_scaler = np.mean(np.abs(g) ** 2)
            self.hk_vk_agc_nfft = np.ones(self.my_mod.n_fft, dtype=np.complex128)
            self.hk_vk_agc_nfft[-(n_sc // 2):] = g[:n_sc // 2]
            self.hk_vk_agc_nfft[1:(n_sc // 2) + 1] = g[n_sc // 2:]
            self.my_array.update_distortion(ibo_db=self.ibo_val_db, avg_sample_pow=self.my_mod.avg_sample_power)
            if isinstance(self.my_cnc_rx, corrector.CncReceiver):
                self.my_cnc_rx.update_distortion(ibo_db=self.ibo_val_db)
        ibo_vec = 10 * np.log10(10 ** (self.ibo_val_db / 10) * self.my_mod.n_sub_carr / (self.vk_pow_vec * self.n_ant_val))
        # sum_a ak[a] hk_vk[a, k] by einsum's own loops (no [A, S] temporary; not a BLAS
        # matrix-vector product, whose thread pool costs ~30 ms a call on a loaded many-core
        # host; equal to 1e-16)
        ak = self.my_mod.calc_alpha(ibo_db=ibo_vec)
        g = np.einsum("a,ak->k", ak, np.ascontiguousarray(self.hk_vk_agc).view(np.float64)).view(np.complex128)
        self.ak_hk_vk_noise_scaler = np.mean(np.abs(g) ** 2)
        self.ak_hk_vk_agc_nfft = np.ones(self.my_mod.n_fft, dtype=np.complex128)
        self.ak_hk_vk_agc_nfft[-(n_sc // 2):] = g[:n_sc // 2]
        self.ak_hk_vk_agc_nfft[1:(n_sc // 2) + 1] = g[n_sc // 2:]
        if isinstance(self.my_cnc_rx, corrector.McncReceiver):
            self.my_cnc_rx.agc_corr_vec = self.ak_hk_vk_agc_nfft

"""Grid sweeps over (IBO, Eb/N0) points, sharded across GPUs (BASELINE config 4).

Replaces the outer loops of the reference drivers (e.g.
``main_mp_miso_cnc_ber_vs_ebn0.py:97-141``,
``main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:100-215``), which run every grid point
on one host with ``num_cores`` forked ``Link.simulate`` processes and shared counters.

MI355X design: one process per GPU (torchrun; ``torch.distributed`` with the ``nccl``
backend = RCCL over xGMI).  Grid points are independent, so they are dealt over ranks by
estimated cost (LPT) with no data-path communication; each point's Philox seed is derived
from its grid index, so results do not depend on the number of GPUs.  On a rank, all its
points run together (``Link.simulate_points``: one kernel launch per stopping-rule round
covers every open point, so a grid of ~400-trial points fills the GPU).  The only collective is one
all-reduce of the int64 counter tensor [points, indices, {errors, bits}] at the end (a
few KB: latency-bound, one message).  Rank 0 then forms BERs and writes the reference's
CSV layouts (``docs/source/usage.rst:40-56``).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 sweep.py --grid fixed_ber ...
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np

from utilities import ebn0_to_snr, save_to_csv


# BASELINE config 4 at its stated extent (SNR 0-30 dB x IBO 0-7 dB): Eb/N0
# 0..30 dB x IBO 0..7 dB in 0.5 dB steps = 915 points, receiver iterations 0..8, the fixed-BER
# driver's stopping rule and geometry (main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:40-61,
# 100-215: 64-antenna ULA, FFT 4096, 2048 sub-carriers, 64-QAM, soft limiter).
# The swept axis is Eb/N0, the drivers' own axis (main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:
# 103-112 sweep ebn0_db_arr and convert with ebn0_to_snr), not the SNR that BASELINE.json names:
# "0-30 dB" is read as Eb/N0 0-30 dB, i.e. SNR = Eb/N0 + 10 log10(6) = 7.8-37.8 dB at 64-QAM.
# (A literal SNR 0-30 dB grid is Eb/N0 -7.8..22.2 dB: more low-SNR points that close on
# n_err_min within a few dozen trials, fewer capped at the bit budget -- a cheaper grid.)
# bench.py's grid object names the axis.
BASELINE_C4 = dict(ibo=np.arange(0.0, 7.01, 0.5), ebn0=np.arange(0.0, 30.01, 0.5), iters=np.arange(0, 9),
                   n_ant=64, n_sc=2048, n_fft=4096, qam=64, cp=128, bits_sent_max=int(5e6), n_err_min=int(1e5))


def paper_link(channel="rayleigh", receiver="cnc", precision="f64", device=None, n_ant=64, n_sc=2048, n_fft=4096,
               qam=64, cp=128, n_err_min=int(1e5), bits_sent_max=int(5e6)):
    """The reference drivers' Link (main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:40-98):
    ULA at z = 15 m, RX at (212, 212, 1.5), 3.5 GHz / 15 kHz, soft limiter, seed-1234 Rayleigh."""
    import copy

    import antenna_array
    import channel as ch_mod
    import distortion
    import modulation
    import mp_model
    import noise
    import transceiver
    mod = modulation.OfdmQamModem(constel_size=qam, n_fft=n_fft, n_sub_carr=n_sc, cp_len=cp)
    dist_obj = distortion.SoftLimiter(0, mod.avg_sample_power)
    tx = transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist_obj), center_freq=int(3.5e9),
                                 carrier_spacing=int(15e3))
    rx = transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist_obj), cord_x=212,
                                 cord_y=212, cord_z=1.5, center_freq=int(3.5e9), carrier_spacing=int(15e3))
    arr = antenna_array.LinearArray(n_elements=n_ant, base_transceiver=tx, center_freq=int(3.5e9),
                                    wav_len_spacing=0.5, cord_x=0, cord_y=0, cord_z=15)
    if channel == "rayleigh":
        ch = ch_mod.MisoRayleighFd(tx_transceivers=arr.array_elements, rx_transceiver=rx, seed=1234)
    else:
        ch = ch_mod.MisoLosFd() if channel == "los" else ch_mod.MisoTwoPathFd()
        ch.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx, skip_attenuation=False)
    return mp_model.Link(mod_obj=mod, array_obj=arr, std_rx_obj=rx, chan_obj=ch, noise_obj=noise.Awgn(snr_db=10),
                         rx_loc_var=10.0, n_err_min=n_err_min, bits_sent_max=bits_sent_max,
                         is_mcnc=receiver == "mcnc", device=device, precision=precision)


def point_seed(base_seed: int, point_index: int) -> list:
    """Seed array of one grid point (fed to Link.simulate, which hashes it)."""
    return [int(base_seed) & 0x7FFFFFFFFFFFFFFF, int(point_index), 0x5EED]


def owned_points(n_points: int, rank: int, world: int, costs=None) -> list:
    """Grid points of ``rank``: longest-processing-time-first over the estimated costs
    (every rank computes the same deterministic assignment); round-robin without costs."""
    if costs is None:
        return list(range(rank, n_points, world))
    load = [0.0] * world
    mine = []
    for p in sorted(range(n_points), key=lambda i: (-float(costs[i]), i)):
        r = min(range(world), key=lambda k: (load[k], k))
        load[r] += float(costs[p])
        if r == rank:
            mine.append(p)
    return sorted(mine)


# Residual clipping distortion seen by a point's best counter, relative to the soft
# limiter's signal-to-distortion ratio at the point's IBO (point_costs): with MRT over
# i.i.d. Rayleigh the distortion is not beamformed (~1/A of it reaches the user); over LoS /
# two-path it is, and the CNC / MCNC iterations remove ~90 % of it.  Calibrated on the
# committed one-GPU records of the 915-point grid (profiles/r05/grid/, tests/test_grid_balance.py).
RESIDUAL_DISTORTION = {"rayleigh": None, "los": 0.1, "two_path": 0.1}


def soft_limiter_sdr(ibo_db):
    """Bussgang signal-to-distortion ratio of the soft limiter for a complex Gaussian input
    at IBO ``ibo_db``: alpha^2 / (E|y|^2 / P - alpha^2), E|y|^2 / P = 1 - exp(-gamma^2),
    alpha = calc_alpha (modulation.py:178-189)."""
    from scipy import special
    g2 = 10 ** (np.asarray(ibo_db, dtype=np.float64) / 10)
    g = np.sqrt(g2)
    a = 1 - np.exp(-g2) + np.sqrt(np.pi) / 2 * g * special.erfc(g)
    return a ** 2 / np.maximum(1 - np.exp(-g2) - a ** 2, 1e-300)


def point_costs(ibo_arr, ebn0_arr, n_bits_per_sym, constel_size, n_err_min, bits_sent_max, iters, n_ant=64,
                is_mcnc=False, channel="rayleigh", pilot=64):
    """Relative cost of every (IBO, Eb/N0) point for sharding: expected trials x cost per trial.

    Trials: a point runs until its best counter has n_err_min errors or the bit budget is
    spent (mp_model.py:177-187), and at least the stopping rule's pilot batch
    (mp_model.PILOT).  The best counter's BER is Gray-QAM at the SINR that the noise and the
    residual clipping distortion leave, 1 / (1 / snr + kappa / sdr(IBO)) with kappa from
    RESIDUAL_DISTORTION (1/A for Rayleigh), so low-SNR points and low-IBO LoS points are
    cheap and the rest hit bits_sent_max.  Per trial: one array pass (n_ant FFT pairs) plus
    one FFT pair per CNC iteration, or one more array pass per MCNC iteration."""
    from scipy import special
    M = float(constel_size)
    k = np.log2(M)
    budget = bits_sent_max / n_bits_per_sym
    max_it = int(np.max(iters)) if len(iters) else 0
    per_trial = n_ant * (1 + max_it) if is_mcnc else n_ant + max_it
    kappa = RESIDUAL_DISTORTION.get(channel, 0.1)
    kappa = 1.0 / max(1, n_ant) if kappa is None else kappa
    sdr = soft_limiter_sdr(np.asarray(ibo_arr, dtype=np.float64))
    # [IBO, Eb/N0] at once (row-major = the grid's point order), the same operations per point
    # as the scalar loop it replaced (timed host path: 6 -> 0.3 ms for 915 points)
    snr = 10 ** (np.asarray(ebn0_arr, dtype=np.float64) / 10) * k  # Es/N0 per symbol
    sinr = 1.0 / (1.0 / snr[None, :] + kappa / sdr[:, None])
    ber = 2 / k * (1 - 1 / np.sqrt(M)) * special.erfc(np.sqrt(1.5 * sinr / (M - 1)))
    trials = np.minimum(budget, n_err_min / np.maximum(ber * n_bits_per_sym, 1e-30))
    return (np.maximum(np.maximum(trials, float(pilot)), 1.0) * per_trial).reshape(-1)


def run_grid(link, ibo_arr, ebn0_arr, iters, incl_clean=True, seed=2137, rank=0, world=1, dist=None,
             device=None, reroll_chan=True, multipoint=True, stats=None, split="points"):
    """Simulate every (IBO, Eb/N0) point this rank owns; all-reduce the counters.

    Returns (err, bits) int64 arrays of shape [n_ibo, n_ebn0, n_idx] on every rank.
    ``link`` is a ``mp_model.Link``-like object (update_distortion / set_snr / simulate;
    with ``simulate_points`` all owned points run together, a few launches per grid).
    Points are dealt by estimated cost (``point_costs``, LPT).  ``stats`` (a dict, optional)
    receives this rank's work record: its points, their modelled costs and trials run, the
    stopping-rule rounds with their kernel ms, and the wall time of its share (before the
    all-reduce).  With a process group (``dist``), the counters are all-reduced even at
    world size 1 (one code path for every N).

    ``split="trials"`` (with ``dist``; SURVEY §8(e)'s alternative for grids with fewer points
    than ranks or a point count the ranks do not divide): every rank runs every point and
    the ranks share each point's trials, one all-reduce of the round's counts per
    stopping-rule round (``Link.simulate_points(dist=...)``).  The counts are bit-identical
    to ``split="points"`` and to one rank.
    """
    if split not in ("points", "trials", "auto"):
        raise ValueError("split must be 'points', 'trials' or 'auto'")
    if split == "auto":  # trials when some rank would get no point at all
        split = "trials" if len(ibo_arr) * len(ebn0_arr) < world and hasattr(link, "simulate_points") else "points"
    by_trials = split == "trials" and dist is not None
    if by_trials and not (multipoint and hasattr(link, "simulate_points")):
        raise ValueError("split='trials' needs a link with simulate_points (multipoint=True)")
    ibo_arr = np.asarray(ibo_arr, dtype=np.float64)
    ebn0_arr = np.asarray(ebn0_arr, dtype=np.float64)
    iters = np.asarray(iters)
    n_idx = len(iters) + (1 if incl_clean else 0)
    n_pts = len(ibo_arr) * len(ebn0_arr)
    counts = np.zeros((n_pts, n_idx, 2), dtype=np.int64)
    m = link.my_mod
    n_bits_sym = int(m.n_sub_carr * np.log2(m.constel_size))
    chan = link._chan_kind() if hasattr(link, "_chan_kind") else "rayleigh"
    costs = point_costs(ibo_arr, ebn0_arr, n_bits_sym, m.constel_size, getattr(link, "n_err_min", 1e5),
                        getattr(link, "bits_sent_max", 5e6), iters, getattr(link, "n_ant_val", 64),
                        getattr(link, "is_mcnc", False), chan)
    mine = list(range(n_pts)) if by_trials else owned_points(n_pts, rank, world, costs)
    t_start = time.perf_counter()
    sim_stats = {}
    batched = multipoint and hasattr(link, "simulate_points")
    current_ibo = None
    params, seeds = [], []
    # drivers convert with n_fft = n_sub_carr (main_mp_miso_cnc_ber_vs_ebn0.py:112); once per axis value
    snr_arr = np.asarray(ebn0_to_snr(ebn0_arr, m.n_sub_carr, m.n_sub_carr, m.constel_size), dtype=np.float64)
    for p in mine:
        i_ibo, i_snr = divmod(p, len(ebn0_arr))
        if current_ibo != ibo_arr[i_ibo]:
            link.update_distortion(ibo_val_db=float(ibo_arr[i_ibo]))
            current_ibo = ibo_arr[i_ibo]
        link.set_snr(float(snr_arr[i_snr]))
        if batched:
            params.append(dict(link.point_params()))
            seeds.append(point_seed(seed, p))
            continue
        err = np.zeros(n_idx)
        bits = np.zeros(n_idx)
        link.simulate(incl_clean, reroll_chan, iters, point_seed(seed, p), err, bits)
        counts[p, :, 0] = err.astype(np.int64)
        counts[p, :, 1] = bits.astype(np.int64)
    if batched and mine:
        err = np.zeros((len(mine), n_idx))
        bits = np.zeros((len(mine), n_idx))
        kw = dict(dist=dist) if by_trials else {}
        if stats is not None:
            kw["stats"] = sim_stats
        link.simulate_points(incl_clean, reroll_chan, iters, seeds, params, err, bits, **kw)
        counts[mine, :, 0] = err.astype(np.int64)
        counts[mine, :, 1] = bits.astype(np.int64)
    if stats is not None:
        # trials per point: all counters of a point share its trials; the longest-open one has
        # seen them all (bits / bits per symbol), also without simulate_points' record
        # (split by trials: the share of every point's trials this rank ran)
        trials = np.asarray(sim_stats.get("trials_run", sim_stats.get("trials", counts[mine, :, 1].max(axis=1)
                                                                      // max(1, n_bits_sym))))
        rounds = sim_stats.get("rounds", [])
        stats.update(rank=int(rank), points=len(mine), point_ids=[int(p) for p in mine],
                     cost_model=[float(costs[p]) for p in mine], trials_per_point=[int(x) for x in trials],
                     trials=int(np.sum(trials)), rounds=len(rounds),
                     kernel_ms=round(float(sum(r["kernel_ms"] for r in rounds)), 3), round_log=rounds,
                     wall_s=round(time.perf_counter() - t_start, 4))
    if dist is not None and not by_trials:  # (by trials every rank already holds every total)
        import torch
        dev = torch.device(f"cuda:{device}") if device is not None and dist.get_backend() == "nccl" else None
        t = torch.from_numpy(counts).to(dev) if dev is not None else torch.from_numpy(counts)
        dist.all_reduce(t)  # each point is filled by exactly one rank: SUM == gather (world 1: identity)
        counts = t.cpu().numpy()
    counts = counts.reshape(len(ibo_arr), len(ebn0_arr), n_idx, 2)
    return counts[..., 0], counts[..., 1]


def ber_from_counts(err, bits):
    """BER with NaN where nothing was sent (main_mp_miso_cnc_ber_vs_ebn0.py:134-139)."""
    err = np.asarray(err, dtype=np.float64)
    bits = np.asarray(bits, dtype=np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(bits == 0, np.nan, err / np.where(bits == 0, 1, bits))


def required_ebn0(ber_per_ibo_snr_iter, ebn0_arr, target_ber):
    """Eb/N0 reaching ``target_ber`` per (iteration, IBO) by linear interpolation of Eb/N0
    over BER, inf where the target is outside the measured range
    (main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:151-180)."""
    from scipy import interpolate
    n_ibo, _, n_it = ber_per_ibo_snr_iter.shape
    out = np.zeros((n_it, n_ibo))
    for it in range(n_it):
        for ib in range(n_ibo):
            f = interpolate.interp1d(ber_per_ibo_snr_iter[ib, :, it], ebn0_arr)
            try:
                out[it, ib] = f(target_ber)
            except ValueError:
                out[it, ib] = np.inf
    return out


def ber_vs_ebn0_rows(ebn0_arr, ber_idx_by_snr):
    """CSV rows: x axis, then one row per counter index (usage.rst:40-56)."""
    return [np.asarray(ebn0_arr)] + [np.asarray(r) for r in ber_idx_by_snr]


def fixed_ber_rows(ibo_arr, ber_per_ibo_snr_iter):
    """CSV rows of the fixed-BER grid: IBO axis, then IBO-major x Eb/N0 rows of per-iteration
    BERs (main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:208-213)."""
    rows = [np.asarray(ibo_arr)]
    for per_snr in ber_per_ibo_snr_iter:
        for per_it in per_snr:
            rows.append(np.asarray(per_it))
    return rows


def _build_link(args, device):
    import copy

    import antenna_array
    import channel
    import distortion
    import modulation
    import mp_model
    import noise
    import transceiver

    mod = modulation.OfdmQamModem(constel_size=args.qam, n_fft=args.n_fft, n_sub_carr=args.n_sc, cp_len=args.cp)
    if args.pa == "rapp":
        dist_obj = distortion.Rapp(ibo_db=0, p_hardness=args.p_hardness, avg_samp_pow=mod.avg_sample_power)
    else:
        dist_obj = distortion.SoftLimiter(0, mod.avg_sample_power)
    tx = transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist_obj), center_freq=int(3.5e9),
                                 carrier_spacing=int(15e3))
    rx = transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist_obj), cord_x=212.0,
                                 cord_y=212.0, cord_z=1.5, center_freq=int(3.5e9), carrier_spacing=int(15e3))
    arr = antenna_array.LinearArray(n_elements=args.n_ant, base_transceiver=tx, center_freq=int(3.5e9),
                                    wav_len_spacing=0.5, cord_x=0, cord_y=0, cord_z=15)
    if args.channel == "rayleigh":
        ch = channel.MisoRayleighFd(tx_transceivers=arr.array_elements, rx_transceiver=rx, seed=1234)
    else:
        ch = channel.MisoLosFd() if args.channel == "los" else channel.MisoTwoPathFd()
        ch.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx, skip_attenuation=False)
    return mp_model.Link(mod_obj=mod, array_obj=arr, std_rx_obj=rx, chan_obj=ch, noise_obj=noise.Awgn(snr_db=10),
                         rx_loc_var=10.0, n_err_min=args.n_err_min, bits_sent_max=args.bits_sent_max,
                         is_mcnc=args.receiver == "mcnc", device=device)


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--grid", choices=["ber_vs_ebn0", "fixed_ber"], default="fixed_ber")
    ap.add_argument("--n-ant", type=int, default=64)
    ap.add_argument("--n-sc", type=int, default=2048)
    ap.add_argument("--n-fft", type=int, default=4096)
    ap.add_argument("--cp", type=int, default=128)
    ap.add_argument("--qam", type=int, default=64)
    ap.add_argument("--pa", choices=["softlim", "rapp"], default="softlim")
    ap.add_argument("--p-hardness", type=float, default=3.0)
    ap.add_argument("--channel", choices=["rayleigh", "los", "two_path"], default="rayleigh")
    ap.add_argument("--receiver", choices=["cnc", "mcnc"], default="cnc")
    ap.add_argument("--ibo", type=str, default="0:8:0.5", help="start:stop:step (numpy arange)")
    ap.add_argument("--ebn0", type=str, default="10:22.1:0.5",
                    help="start:stop:step (numpy arange); default: the published fixed-BER grids' Eb/N0 10..22 dB")
    ap.add_argument("--iters", type=str, default="0,1,2,3,4,5,6,7,8")
    ap.add_argument("--target-ber", type=float, default=1e-2)
    ap.add_argument("--bits-sent-max", type=int, default=int(5e6))
    ap.add_argument("--n-err-min", type=int, default=int(1e5))
    ap.add_argument("--seed", type=int, default=2137)
    ap.add_argument("--out", type=str, default="figs/csv_results")
    ap.add_argument("--split", choices=["points", "trials", "auto"], default="auto",
                    help="ranks deal whole points by cost (one all-reduce at the end), or share every point's "
                         "trials (one all-reduce per stopping-rule round); auto: trials when there are fewer "
                         "points than ranks")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    rng = lambda s: np.arange(*[float(x) for x in s.split(":")])  # noqa: E731
    ibo_arr, ebn0_arr = rng(args.ibo), rng(args.ebn0)
    iters = np.asarray([int(x) for x in args.iters.split(",")])
    incl_clean = args.grid == "ber_vs_ebn0"
    link = _build_link(args, local)
    t0 = time.perf_counter()
    err, bits = run_grid(link, ibo_arr, ebn0_arr, iters, incl_clean, args.seed, rank, world, dist, local,
                         split=args.split)
    elapsed = time.perf_counter() - t0
    if rank == 0:
        ber = ber_from_counts(err, bits)
        tag = "%s_%s_nant%d" % (args.receiver, args.channel, args.n_ant)
        if args.grid == "fixed_ber":
            name = "fixed_ber%1.1e_%s_ebn0_min%d_max%d_step%1.2f_ibo_min%d_max%d_step%1.2f_niter%s" % (
                args.target_ber, tag, min(ebn0_arr), max(ebn0_arr), ebn0_arr[1] - ebn0_arr[0], min(ibo_arr),
                max(ibo_arr), ibo_arr[1] - ibo_arr[0], "_".join(str(v) for v in iters[1:]))
            save_to_csv(fixed_ber_rows(ibo_arr, ber), name, directory=args.out)
            req = required_ebn0(ber, ebn0_arr, args.target_ber)
            save_to_csv([ibo_arr] + list(req), "req_ebn0_" + name, directory=args.out)
        else:
            for i, ibo in enumerate(ibo_arr):
                name = "ber_vs_ebn0_%s_ibo%d_ebn0_min%d_max%d_step%1.2f_niter%s" % (
                    tag, ibo, min(ebn0_arr), max(ebn0_arr), ebn0_arr[1] - ebn0_arr[0],
                    "_".join(str(v) for v in iters[1:]))
                save_to_csv(ber_vs_ebn0_rows(ebn0_arr, ber[i].T), name, directory=args.out)
        # every counter of a point shares its trials; the one that stayed open longest saw them
        # all (iteration 0 closes first in a fixed-BER grid): symbols from the largest counter
        n_sym = int(bits.max(axis=-1).sum()) // (args.n_sc * int(np.log2(args.qam)))
        print(f"sweep done: {len(ibo_arr) * len(ebn0_arr)} points, {n_sym} OFDM symbols on {world} GPU(s) in "
              f"{elapsed:.1f} s -> {args.out}")
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

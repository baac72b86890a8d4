"""Headline benchmark: OFDM symbols/s/GPU of the Monte-Carlo BER chain (BASELINE config 2).

Workload (BASELINE.json configs[1]): 64-antenna MRT, 1024 sub-carriers (FFT 2048), 64-QAM,
soft-limiter PA at IBO 3 dB, i.i.d. Rayleigh channel rerolled per trial, Eb/N0 15 dB,
standard receiver (iteration 0), 2^16 trials (= OFDM symbols) per step.  One step = one
fused-kernel launch over the batch + the on-device count reduction.  Inputs are generated
on the device from Philox streams (no host transfer).  ``--gpus N`` (one rank per GPU,
under torchrun; without an outer torchrun the script starts it as a child process)
shards trials by index: weak scaling, no data-path collective; the per-step error counts
are summed across ranks once at the end (RCCL all_reduce).

After the headline's timed region the same ranks time north_star's own split, BASELINE
config 4's 915-point SNR x IBO grid dealt over them (``grid`` object; ``--no-grid`` skips it).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

# Workloads: "2" is BASELINE configs[1] (the headline, default); the others are optional
# extra lines: "paper" = the published CSV config (64 ant, FFT 4096, 2048 sc), "5su" =
# BASELINE config 5's array / FFT / PA (256 ant, FFT 8192, 4096 sc, Rapp p=3) at one
# user (the multi-user precoder is not built).
WORKLOADS = {
    "2": dict(A=64, S=1024, F=2048, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0,
              desc="BASELINE config 2: 64-ant MRT, 1024-sc (FFT 2048) 64-QAM, soft limiter IBO 3 dB, "
                   "Rayleigh, Eb/N0 15 dB"),
    "paper": dict(A=64, S=2048, F=4096, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0,
                  desc="paper config: 64-ant MRT, 2048-sc (FFT 4096) 64-QAM, soft limiter IBO 3 dB, Rayleigh, "
                       "Eb/N0 15 dB"),
    "2gen": dict(A=64, S=1000, F=2048, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0,
                 desc="config 2 with 1000 sub-carriers (generic, unaligned slot path)"),
    "2los": dict(A=64, S=1024, F=2048, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0, chan="los",
                 desc="config 2 geometry over the LoS channel (RX jitter +-5 m, closed-form per trial)"),
    "2twopath": dict(A=64, S=1024, F=2048, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0, chan="twopath",
                     desc="config 2 geometry over the two-path channel"),
    "2mcnc": dict(A=64, S=1024, F=2048, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0, mcnc=True,
                  desc="config 2 with the MCNC receiver (one full array pass per iteration)"),
    "2csi": dict(A=64, S=1024, F=2048, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0, csi=0.1,
                 desc="config 2 with imperfect CSI (epsilon 0.1, mp_model.py:253-288)"),
    "papercsi": dict(A=64, S=2048, F=4096, M=64, CP=128, pa="softlim", p=0.0, ibo=3.0, ebn0=15.0, csi=0.1,
                     desc="paper config with imperfect CSI (epsilon 0.1, mp_model.py:253-288)"),
    "5su": dict(A=256, S=4096, F=8192, M=64, CP=128, pa="rapp", p=3.0, ibo=3.0, ebn0=15.0,
                desc="config-5 array at one user: 256-ant MRT, 4096-sc (FFT 8192) 64-QAM, Rapp p=3 IBO 3 dB, "
                     "Rayleigh, Eb/N0 15 dB"),
}
A, S, F, M, CP = 64, 1024, 2048, 64, 128
IBO, EBN0 = 3.0, 15.0
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Dense vector peaks of the arithmetic type the kernel computes in.  f32: MI355X_MICROARCH.md
# (157.3 TF, VALU == MFMA f32).  f64: AMD's MI355X spec sheet (78.6 TF vector; the guide
# lists no f64 figure) -- the fused kernel issues no MFMA, so the VALU peak is the ceiling.
VALU_PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}


# The reference's own Link.simulate (NumPy + torch CPU FFT, numba absent) timed in the build
# container (SURVEY.md §6, config-2 geometry, standard RX): it cannot travel to the GPU box,
# so the bench line quotes it beside the measured port.
CPU_REFERENCE_SURVEY = {"per_process": 5.7, "n8_processes": 35.8, "unit": "OFDM symbols/s", "cores": 8,
                        "kind": "reference", "source": "SURVEY.md §6 (Intel Xeon, 8 cores, mp.Process x 8 as "
                                                      "main_mp_miso_cnc_ber_vs_ebn0.py:122-132)"}


def bytes_alg_per_trial(a=A, s=S, f=F):
    """staged K1-K4 model, complex64 = 8 B:  8 A (6 S + 2 F)."""
    return 8 * a * (6 * s + 2 * f)


def flops_alg_per_trial(a=A, s=S, f=F, max_iter=0, mcnc=False):
    """A (2 * 5 F log2 F + 14 S + 12 F)  (FFT pair + precode/PA/combine), plus
    per receiver iteration one single-vector IFFT/PA/FFT (CNC, corrector.py:84-110) or one
    more array pass (MCNC, corrector.py:165-207)."""
    one = 10 * f * np.log2(f) + 14 * s + 12 * f
    return a * one + max_iter * (a * one if mcnc else one)


def make_engine(device, workload="2", precision="f64"):
    import _engine
    import mp_model  # noqa: F401  (host mirror; computes the per-point scalars like Link)
    from utilities import ebn0_to_snr
    from modulation import OfdmQamModem
    from antenna_array import LinearArray
    from transceiver import Transceiver
    from distortion import SoftLimiter
    import channel, noise, copy

    w = WORKLOADS[workload]
    A, S, F, M, CP = w["A"], w["S"], w["F"], w["M"], w["CP"]
    from distortion import Rapp
    mod = OfdmQamModem(constel_size=M, n_fft=F, n_sub_carr=S, cp_len=CP)
    dist = SoftLimiter(0, mod.avg_sample_power) if w["pa"] == "softlim" else \
        Rapp(0, mod.avg_sample_power, p_hardness=w["p"])
    tx = Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist), center_freq=int(3.5e9),
                     carrier_spacing=int(15e3))
    rx = Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist), cord_x=212, cord_y=212, cord_z=1.5,
                     center_freq=int(3.5e9), carrier_spacing=int(15e3))
    arr = LinearArray(n_elements=A, base_transceiver=tx, center_freq=int(3.5e9), wav_len_spacing=0.5, cord_x=0,
                      cord_y=0, cord_z=15)
    kind = w.get("chan", "rayleigh")
    if kind == "rayleigh":
        ch = channel.MisoRayleighFd(tx_transceivers=arr.array_elements, rx_transceiver=rx, seed=1234)
    else:
        ch = channel.MisoLosFd() if kind == "los" else channel.MisoTwoPathFd()
        ch.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx, skip_attenuation=False)
    link = mp_model.Link(mod_obj=mod, array_obj=arr, std_rx_obj=rx, chan_obj=ch, noise_obj=noise.Awgn(snr_db=10),
                         rx_loc_var=10.0, n_err_min=10 ** 12, bits_sent_max=10 ** 15, is_mcnc=w.get("mcnc", False),
                         csi_epsylon=w.get("csi"), device=device, precision=precision)
    link.update_distortion(ibo_val_db=w["ibo"])
    link.set_snr(ebn0_to_snr(w["ebn0"], S, S, M))
    return link.engine()


def _cpu_worker(args):
    """One host process of the CPU baseline: trials of the workload through oracle/sim.py for
    ``seconds`` of wall time; returns the number of trials it finished."""
    workload, iters, seconds, wid = args
    from oracle import refmath as rm
    from oracle.sim import SimConfig, run_trials
    w = WORKLOADS[workload]
    cfg = SimConfig(w["A"], w["S"], w["F"], w["M"], pa=w["pa"], p_hardness=w["p"], ibo_db=w["ibo"],
                    snr_db=float(rm.ebn0_to_snr(w["ebn0"], w["S"], w["S"], w["M"])), channel=w.get("chan", "rayleigh"),
                    receiver="mcnc" if w.get("mcnc") else "cnc", csi_eps=w.get("csi"))
    step = 4 if w["F"] <= 2048 else 1
    run_trials(cfg, 7, [0], iters=list(iters))  # warm caches / imports
    n, base, t0 = 0, (wid + 1) << 24, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        run_trials(cfg, 7, np.arange(base + n, base + n + step), iters=list(iters))
        n += step
    return n, time.perf_counter() - t0


def cpu_cores():
    """Host cores the baseline may use: this process's CPU affinity, capped at 16 (a GPU
    box's share per GPU; its nproc shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(seconds=15.0, workload="2", iters=(0,), cores=None):
    """The float64 oracle (oracle/sim.py, NumPy) fanned out over the host's cores the way the
    reference's drivers fan ``Link.simulate`` out (``mp.Process`` x cores,
    main_mp_miso_cnc_ber_vs_ebn0.py:122-132), on a bounded sample of the same workload (same
    receiver iterations).  Reported beside the GPU number, never the measured product.
    Workers are spawned (fresh interpreters, one NumPy thread each), not forked from a process
    that holds a HIP context."""
    import multiprocessing as mp
    cores = cores or cpu_cores()
    iters = list(iters)
    env_keys = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")
    saved = {k: os.environ.get(k) for k in env_keys}
    for k in env_keys:
        os.environ[k] = "1"
    try:
        ctx = mp.get_context("spawn")
        t0 = time.perf_counter()
        with ctx.Pool(cores) as pool:
            res = pool.map(_cpu_worker, [(workload, tuple(iters), seconds, i) for i in range(cores)])
        wall = time.perf_counter() - t0
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    n = sum(r[0] for r in res)
    busy = max(r[1] for r in res)
    w = WORKLOADS[workload]
    rx = ("MCNC" if w.get("mcnc") else "CNC") + f" iterations {iters}" if iters != [0] else "standard RX"
    out = dict(value=round(n / busy, 3), unit="OFDM symbols/s", cores=cores, kind="port",
               sample=f"{n} trials of the workload-{workload} chain ({rx}) through oracle/sim.py (NumPy float64), "
                      f"{cores} spawned processes x {busy:.1f} s each (pool wall {wall:.1f} s incl. start-up)")
    if workload == "2":
        out["cpu_reference_published"] = CPU_REFERENCE_SURVEY
    return out


def load_pmc_traffic(workload, iters, precision, trials_per_launch):
    """Per-launch HBM bytes from a committed rocprofv3 PMC summary of the SAME workload,
    receiver iterations, precision and batch (tools/pmc_traffic.py writes them).  Records of
    an older kernel carry "superseded_by" and are skipped."""
    key = dict(workload=workload, iters=list(iters), precision=precision, trials_per_launch=trials_per_launch)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "**", "*pmc*.json"), recursive=True), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if all(d.get(k) == v for k, v in key.items()) and "hbm_bytes_per_launch" in d and "superseded_by" not in d:
            return d["hbm_bytes_per_launch"], os.path.relpath(path, REPO)
    return None, None


def ber_vs_published(ber):
    """BASELINE's "BER match vs ref" for the config-2 line: the reference's published standard-RX
    BER at the same point (tests/golden/published_ber_vs_ebn0_cnc_rayleigh_ibo3.csv, a data file
    of its figs/csv_results: 64 antennas, Rayleigh, MRT, soft limiter IBO 3 dB, 64-QAM, Eb/N0
    15 dB; rows [no distortion, standard RX, CNC 1..8]).  Its geometry is 2048 sub-carriers /
    FFT 4096, config 2's 1024 / 2048: the same F = 2S, so the same per-sub-carrier statistics.
    z against the published run's binomial sigma (its 1e7-bit budget,
    main_mp_miso_cnc_ber_vs_ebn0.py: bits within a symbol treated as independent, so |z| is an
    upper bound); tests/test_gpu_link.py holds the full-curve comparison."""
    path = os.path.join(REPO, "tests", "golden", "published_ber_vs_ebn0_cnc_rayleigh_ibo3.csv")
    try:
        rows = np.loadtxt(path, delimiter=",")
    except OSError:
        return None
    pub = float(rows[2][int(np.flatnonzero(np.isclose(rows[0], 15.0))[0])])
    sig = pub / np.sqrt(pub * 1e7)
    return {"engine": ber, "published": pub, "rel": round(ber / pub - 1, 5), "z_binomial": round(float((ber - pub) / sig), 3),
            "source": "tests/golden/published_ber_vs_ebn0_cnc_rayleigh_ibo3.csv (standard RX, Eb/N0 15 dB; "
                      "2048-sc / FFT-4096 geometry, F = 2S as config 2)"}


def launch_ranks(n):
    """``--gpus N`` without an outer torchrun: start ``torch.distributed.run`` with N ranks
    as a CHILD process (this parent has made no GPU call and never execs), forward rank 0's
    JSON line and return the child's exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout.splitlines():
        if line.startswith("{"):
            print(line, flush=True)
        else:
            print(line, file=sys.stderr, flush=True)
    return proc.returncode


def time_grid(rank, world, dist, dev, precision, tdev, fake=False, split="points"):
    """North_star's multi-GPU split (BASELINE config 4): ``sweep.run_grid`` over the 915-point
    SNR x IBO extent (sweep.BASELINE_C4), grid points dealt over the N ranks by estimated cost
    (LPT), one all-reduce of the counters -- exactly what the reference's fixed-BER driver runs
    point by point on one host (main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:100-215).
    Strong scaling: the grid is fixed, N ranks share it.  Timed between barriers after an
    untimed engine set-up; the wall time is the MAX over ranks.  ``fake``: the CPU rehearsal
    (tests/fake_link.py stand-in, no GPU) of the same plumbing.  ``split="trials"``
    (``--grid-split trials``): the ranks share every point's trials instead, one all-reduce per
    stopping-rule round (same counts digest)."""
    import hashlib

    import sweep
    c4 = sweep.BASELINE_C4
    if fake:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from fake_link import FakeLink
        link = FakeLink()
    else:
        link = sweep.paper_link("rayleigh", "cnc", precision, device=dev, n_err_min=c4["n_err_min"],
                                bits_sent_max=c4["bits_sent_max"])
        link.engine().run(0, 0, 1, [0])  # engine / device set-up outside the timed region
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    st = {}
    err, bits = sweep.run_grid(link, c4["ibo"], c4["ebn0"], c4["iters"], incl_clean=False, seed=2137, rank=rank,
                               world=world, dist=dist, device=dev, stats=st, split=split)
    if not fake:
        import torch
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    ranks = 1
    mine = {k: st[k] for k in ("rank", "points", "trials", "rounds", "kernel_ms", "wall_s")}
    mine["cost_model"] = round(float(np.sum(st["cost_model"])), 1)
    per_rank = [mine]
    if dist:
        import torch
        t = torch.tensor([dt, 1.0], device=tdev, dtype=torch.float64)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:])
        dt, ranks = float(t[0].item()), int(t[1].item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    m = link.my_mod
    bits_per_sym = int(m.n_sub_carr * np.log2(m.constel_size))
    # OFDM symbols run: every counter of a point shares its trials, and the counter that stayed
    # open longest saw them all (iteration 0 closes first in a fixed-BER grid)
    n_sym = int(bits.max(axis=-1).sum()) // bits_per_sym
    digest = hashlib.sha256(np.ascontiguousarray(err, np.int64).tobytes() +
                            np.ascontiguousarray(bits, np.int64).tobytes()).hexdigest()[:16]
    loads = [r["trials"] for r in per_rank]
    costs = [r["cost_model"] for r in per_rank]
    return {"workload": "BASELINE config 4: Eb/N0 0-30 dB x IBO 0-7 dB (0.5 dB steps; Eb/N0 is the swept axis), "
                        "CNC iterations 0-8, "
                        "bits_sent_max 5e6 / n_err_min 1e5 per point, 64-ant / FFT 4096 / 2048-sc paper geometry"
                        + (" [CPU rehearsal: stand-in link]" if fake else ""),
            "axis": "Eb/N0 (the drivers' axis, main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:103-112; "
                    "BASELINE's 'SNR 0-30 dB' read as Eb/N0: SNR = Eb/N0 + 7.8 dB at 64-QAM)",
            "points": int(len(c4["ibo"]) * len(c4["ebn0"])), "ofdm_symbols": n_sym, "wall_s": round(dt, 4),
            "symbols_per_s": round(n_sym / dt, 1), "ranks_seen": ranks, "scaling": "strong",
            "parallelism": (f"points dealt by cost (LPT) over {world} rank(s), one all-reduce of the counters"
                            if split == "points" or not dist else
                            f"every point's trials shared by {world} rank(s), one all-reduce per stopping-rule round"),
            "per_rank": per_rank,
            "trials_max_over_mean": round(max(loads) / max(1e-9, float(np.mean(loads))), 4),
            "model_max_over_mean": round(max(costs) / max(1e-9, float(np.mean(costs))), 4),
            "counts_digest": digest}


def check_launch(world, rank):
    """``--check-launch``: the rank plumbing only (process group over gloo, the world size
    the driver asked for, one all_reduce); no engine, no GPU.  For the CPU launcher test."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"check": "launch", "n_gpus": world, "ranks_seen": int(t.item())}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~5 s of kernel time at config 2: long enough for a device-activity sampler polling every
    # few seconds to see the timed region (BENCH_r04 gpu_busy saw 0 samples of a 0.5-s region)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 16, help="trials (OFDM symbols) per GPU per step")
    ap.add_argument("--iters", type=str, default="0", help="receiver iterations, e.g. 0 or 0,1,2,3,4")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"],
                    help="arithmetic type of the fused kernel (f64 = the reference's float64)")
    ap.add_argument("--workload", default="2", choices=sorted(WORKLOADS),
                    help="2 = BASELINE config 2 (headline); paper; 5su (config-5 array, one user)")
    ap.add_argument("--check-launch", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-grid", action="store_true", help="skip the config-4 grid line (the 'grid' object)")
    ap.add_argument("--grid-split", choices=["points", "trials"], default="points",
                    help="the grid's multi-GPU split: whole points by cost (default), or every point's trials")
    ap.add_argument("--grid-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.check_launch:
        return check_launch(world, rank)
    if args.grid_check:  # CPU rehearsal of the grid line: gloo ranks, stand-in link, no GPU
        import torch.distributed as gdist
        gd = None
        if "WORLD_SIZE" in os.environ:
            gdist.init_process_group("gloo")
            gd = gdist
        g = time_grid(rank, world, gd, None, args.precision, "cpu", fake=True)
        if gd:
            gd.destroy_process_group()
        if rank == 0:
            print(json.dumps({"check": "grid", "n_gpus": world, "grid": g}), flush=True)
        return
    import torch
    dist = None
    # MIMO_BENCH_BACKEND=gloo rehearses the N > 1 path with ranks sharing the visible GPUs
    # (device = LOCAL_RANK mod device count); the driver's runs use RCCL, one GPU per rank.
    backend = os.environ.get("MIMO_BENCH_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count())
    tdev = f"cuda:{dev}" if backend == "nccl" else "cpu"
    # A process group whenever a launcher started this rank (torchrun sets WORLD_SIZE), also at
    # world size 1: the RCCL code path of the N-GPU runs is then the one every run takes.
    if "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        # device_id binds the RCCL communicator to this rank's GPU (no guessing from the rank)
        if backend == "nccl":
            dist.init_process_group(backend, device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(backend)
    wl = WORKLOADS[args.workload]
    eng = make_engine(dev, args.workload, args.precision)
    iters = [int(x) for x in args.iters.split(",")]
    B = args.batch
    seed = 2137
    err_tot = None

    def step(i):
        first = (i * world + rank) * B
        e, b, _ = eng.run(seed, first, B, iters, False)
        return e, b

    for i in range(args.warmup):
        step(i)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kern_ms = 0.0
    for i in range(args.warmup, args.warmup + args.steps):
        e, b = step(i)
        kern_ms += eng.kernel_ms
        err_tot = e if err_tot is None else err_tot + e
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device=tdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        c = torch.tensor(err_tot.astype(np.int64), device=tdev)
        dist.all_reduce(c)
        err_tot = c.cpu().numpy()
    total_trials = B * args.steps * world
    value = total_trials / dt
    avg_kernel_s = kern_ms / 1e3 / args.steps
    b_alg = bytes_alg_per_trial(wl["A"], wl["S"], wl["F"]) * B
    f_trial = flops_alg_per_trial(wl["A"], wl["S"], wl["F"], max(iters), wl.get("mcnc", False))
    f_alg = f_trial * B
    traffic, traffic_src = load_pmc_traffic(args.workload, iters, args.precision, B)
    peak = VALU_PEAK_TFLOPS[args.precision]
    achieved = f_alg / avg_kernel_s / 1e12
    rx = "standard RX" if iters == [0] else ("MCNC" if wl.get("mcnc") else "CNC") + f" iterations {iters}"
    out = {
        "metric": "OFDM symbols/s/GPU (64-ant,1024-sc) + achieved HBM %peak; BER match vs ref",
        "value": round(value, 1),
        "unit": "OFDM symbols/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (on-device Philox bits / Rayleigh channel / AWGN)",
        "config": {"workload": wl["desc"] + ", " + rx,
                   "trials_per_gpu_per_step": B, "iters": iters, "parallelism": f"trial-sharded x{world}"},
        "roofline": {
            "bound": "valu", "regime": f"{args.precision} VALU issue (fused kernel, no MFMA-shaped work at one user)",
            "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_source": traffic_src,
            "kernel": "mimo::trial_kernel " + eng.describe(), "kernel_ms": round(avg_kernel_s * 1e3, 3),
            "flops_alg_per_trial": f_trial, "trials_per_launch": B,
        },
        # BASELINE's "achieved HBM %peak": the fused kernel keeps SURVEY §8(d)'s staged-pipeline
        # bytes on chip, so the HBM fraction is the MEASURED traffic (PMC, when a matching
        # summary exists) over the kernel time -- not the staged model's bytes.
        "hbm": {"measured_GBps": None if traffic is None else round(traffic / avg_kernel_s / 1e9, 2),
                "measured_frac": None if traffic is None else round(traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS, 5),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "staged_model_bytes_per_trial": bytes_alg_per_trial(wl["A"], wl["S"], wl["F"]),
                "staged_model_equiv_GBps": round(b_alg / avg_kernel_s / 1e9, 1),
                "note": "staged_model_* = SURVEY §8(d) K1-K4 bytes a staged pipeline would move for the same "
                        "trials; the fused kernel does not move them (a model figure, not traffic)"},
        "ber": [round(float(x) / (total_trials * wl["S"] * np.log2(wl["M"])), 8) for x in err_tot],
    }
    if args.workload == "2" and iters == [0]:
        out["ber_vs_published"] = ber_vs_published(out["ber"][0])
    if not args.no_grid and args.workload == "2" and args.precision == "f64":
        out["grid"] = time_grid(rank, world, dist, dev, args.precision, tdev, split=args.grid_split)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.workload, iters)
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""GPU parity across FFT sizes, team sizes, PA models and the generic (unaligned) slot path.

Same tolerance as tests/test_gpu_engine.py: per-trial, per-iteration counts EXACTLY equal
to the float64 oracle's on identical Philox inputs, for the f64 and the f32 instances.
``MIMO_TEAM`` selects the alternative fp32 team size (engine.hip select_instance); the
fp64 instances have one team size per FFT size, so those cases run in f32 only.
"""
import numpy as np
import pytest

from gpu_util import PRECISIONS, assert_counts_equal, count_agreement, engine_for
from oracle import sim

pytestmark = pytest.mark.gpu

CASES = [
    # F,    S,    A, M,  pa,        p,   ibo, team
    (2048, 1024, 8, 64, "softlim", 0.0, 3.0, 256),   # alternative 4-wave team (P = 8)
    (4096, 2048, 8, 64, "softlim", 0.0, 3.0, None),  # paper-config FFT, 3 waves/SIMD profile
    (4096, 2048, 8, 64, "softlim", 0.0, 3.0, 512),
    (8192, 4096, 4, 64, "rapp", 3.0, 3.0, None),     # config-5 FFT / PA, integer-p Rapp path
    (8192, 4096, 4, 16, "rapp", 2.5, 2.0, None),     # general Rapp path
    (8192, 4096, 4, 64, "rapp", 3.0, 3.0, 1024),     # 16-wave team
    (8192, 2048, 4, 16, "softlim", 0.0, 3.0, None),  # F 8192 generic slots (fp64: S % 4T != 0 at T = 1024)
    (1024, 1000, 8, 16, "softlim", 0.0, 1.0, None),  # generic slots (S % 4T != 0)
    (512, 256, 16, 4, "toi", 0.0, 5.0, None),        # QPSK, cubic PA
    (2048, 1024, 8, 256, "softlim", 0.0, 0.0, None),  # 256-QAM at IBO 0 (strong clipping)
    (128, 4, 2, 16, "softlim", 0.0, -2.0, None),     # smallest band (4 sub-carriers), deep clipping
    # 2 antennas on 4-8 sub-carriers: the per-antenna precoding power strays far outside the
    # alpha fit's |x| <= 0.25, so the fallback runs (fp64: alpha_fit.h's segment table, out of
    # line at every size since round 6; fp32: the library exp / erfc form)
    (2048, 8, 2, 16, "softlim", 0.0, 1.0, None),
    (4096, 8, 2, 16, "softlim", 0.0, 1.0, None),
    (8192, 4, 2, 16, "softlim", 0.0, 1.0, None),
    (256, 252, 4, 16, "softlim", 0.0, 2.0, None),    # widest band allowed (S = F - 4)
    (256, 128, 2048, 64, "softlim", 0.0, 0.0, None),  # many antennas
    (128, 64, 4096, 16, "softlim", 0.0, 1.0, None),   # the most antennas the engine takes (validate_config)
    (1024, 512, 1, 1024, "softlim", 0.0, 100.0, None),  # SISO, ideal PA, 1024-QAM
]
EBN0 = {(128, 4): 6.0, (256, 128): 8.0, (1024, 512): 30.0, (2048, 8): 8.0, (4096, 8): 8.0, (8192, 4): 8.0}


@pytest.mark.parametrize("prec", PRECISIONS)
@pytest.mark.parametrize("F,S,A,M,pa,p,ibo,team", CASES)
def test_sizes_vs_oracle(monkeypatch, F, S, A, M, pa, p, ibo, team, prec):
    if team is not None:
        if prec == "f64":
            pytest.skip("alternative team sizes are fp32 instances")
        monkeypatch.setenv("MIMO_TEAM", str(team))
    snr = float(sim.rm.ebn0_to_snr(EBN0.get((F, S), 14.0), S, S, M))
    cfg = sim.SimConfig(A, S, F, M, pa=pa, p_hardness=p, ibo_db=ibo, snr_db=snr)
    trials = np.arange(24)
    iters = [0, 1, 2]
    ref = sim.run_trials(cfg, 31, trials, iters=iters, incl_clean=True)
    eng = engine_for(cfg, precision=prec)
    err, bits, per = eng.run(31, 0, len(trials), iters, True, per_trial=True)
    desc = eng.describe()
    if team is not None:
        assert f"T={team} " in desc, desc
    agree = count_agreement(per, ref)
    print(F, S, A, M, pa, p, ibo, desc, "agreement", agree, per.sum(0), ref.sum(0))
    assert_counts_equal(per, ref, f"{F}/{S}/{A}/{M}/{pa}/{p}/{ibo}/{team} {prec}")
    np.testing.assert_array_equal(err, per.sum(0))
    assert all(int(b) == len(trials) * S * int(np.log2(M)) for b in bits)


CONFIG5 = [
    # A,  M,  pa,        p,   ibo, channel,    receiver, trials, csi
    (256, 64, "rapp", 3.0, 3.0, "rayleigh", "cnc", 6, None),    # config-5 array geometry (one user)
    (8, 16, "softlim", 0.0, 1.0, "rayleigh", "mcnc", 8, None),  # MCNC array passes through the F 8192 path
    (16, 16, "softlim", 0.0, 2.0, "los", "cnc", 8, None),       # closed-form LoS on the F 8192 path
    (8, 16, "softlim", 0.0, 2.0, "rayleigh", "cnc", 8, 0.2),    # CSI (polar pass 1) on the F 8192 path
    (16, 64, "rapp", 3.0, 3.0, "rayleigh", "mcnc", 4, None),    # config 5's PA under MCNC (the array pass per iteration)
    (8, 16, "softlim", 0.0, 2.0, "two_path", "cnc", 6, None),   # two-path on the F 8192 path (folded weight, round 6)
    (8, 16, "softlim", 0.0, 2.0, "los", "mcnc", 4, None),       # LoS MCNC on the F 8192 path
]


@pytest.mark.parametrize("prec", PRECISIONS)
@pytest.mark.parametrize("A,M,pa,p,ibo,channel,receiver,n,csi", CONFIG5)
def test_config5_array_vs_oracle(A, M, pa, p, ibo, channel, receiver, n, csi, prec):
    """BASELINE config 5's array at one user (256 antennas, F 8192, 4096 sub-carriers,
    Rapp p = 3) and the other F 8192 receivers / channels / CSI: per-trial counts EXACTLY
    equal to the oracle's.  The fp64 instance is the 512-thread team (T = 512, 16 points per
    thread) on the split FFT (split_fft.h: two 4096-point sub-transforms and a lane-swap
    radix-2 stage), as eng.describe() prints."""
    F, S = 8192, 4096
    snr = float(sim.rm.ebn0_to_snr(15.0, S, S, M))
    cfg = sim.SimConfig(A, S, F, M, pa=pa, p_hardness=p, ibo_db=ibo, snr_db=snr, channel=channel, receiver=receiver,
                        csi_eps=csi)
    iters = [0, 1, 2]
    ref = sim.run_trials(cfg, 77, np.arange(n), iters=iters, incl_clean=True, chunk=2)
    eng = engine_for(cfg, precision=prec)
    _, _, per = eng.run(77, 0, n, iters, True, per_trial=True)
    print("config5", A, M, pa, channel, receiver, eng.describe(), per.sum(0), ref.sum(0))
    assert_counts_equal(per, ref, f"config5 {A}/{M}/{pa}/{channel}/{receiver} {prec}")


BENCH_GEOMETRIES = [
    # F,    S,    channel,    receiver, csi
    (2048, 1024, "los", "cnc", None),
    (2048, 1024, "two_path", "cnc", None),
    (2048, 1024, "rayleigh", "cnc", 0.1),
    (2048, 1024, "rayleigh", "mcnc", None),
    (4096, 2048, "los", "cnc", None),
    (4096, 2048, "two_path", "cnc", None),
    (4096, 2048, "rayleigh", "cnc", 0.1),
    (4096, 2048, "rayleigh", "mcnc", None),
    (4096, 2048, "two_path", "mcnc", None),
    (512, 256, "rayleigh", "cnc", 0.3),  # a one-wave CSI instance (polar pass 1 at T = 64)
    (1024, 512, "rayleigh", "mcnc", 0.2),  # MCNC with CSI (the estimate in every array pass)
]


@pytest.mark.parametrize("prec", PRECISIONS)
@pytest.mark.parametrize("F,S,channel,receiver,csi", BENCH_GEOMETRIES)
def test_bench_line_instances_vs_oracle(F, S, channel, receiver, csi, prec):
    """The kernel instances behind bench.py's secondary lines (config-2 geometry F 2048 and
    the paper geometry F 4096: LoS, two-path, CSI error, MCNC) at 8 antennas: per-trial
    counts EXACTLY equal to the oracle's.  The antenna count does not select the instance
    (F, S, channel, CSI do), so these are the instances the 64-antenna lines time, including
    the closed-form pass-1 powers of LoS / two-path (round 4)."""
    A, M = 8, 64
    snr = float(sim.rm.ebn0_to_snr(12.0, S, S, M))
    cfg = sim.SimConfig(A, S, F, M, pa="softlim", ibo_db=2.0, snr_db=snr, channel=channel, receiver=receiver,
                        csi_eps=csi)
    iters = [0, 1, 2]
    n = 6
    ref = sim.run_trials(cfg, 4242, np.arange(n), iters=iters, incl_clean=True, chunk=2)
    eng = engine_for(cfg, precision=prec)
    _, _, per = eng.run(4242, 0, n, iters, True, per_trial=True)
    print("bench-line instance", F, S, channel, receiver, csi, eng.describe(), per.sum(0), ref.sum(0))
    assert_counts_equal(per, ref, f"{F}/{S}/{channel}/{receiver}/csi={csi} {prec}")


PA_PATHS = [
    # F,    S,    pa,     p     (Rayleigh, CNC)
    (2048, 1024, "rapp", 3.0),   # integer-hardness Rapp (rapp_int<3>)
    (2048, 1024, "rapp", 2.0),   # rapp_int<2>
    (2048, 1024, "rapp", 2.5),   # general p: out of line at F 2048 (pa_rapp_general)
    (2048, 1024, "toi", 0.0),
    (4096, 2048, "rapp", 3.0),
    (4096, 2048, "rapp", 2.5),   # general p: out of line at F 4096 too since round 6 (COLD_OUT)
    (4096, 2048, "toi", 0.0),
    (2048, 1024, "rapp", 5.0),   # the hardness the reference's plots use
    (8192, 4096, "rapp", 4.0),   # the hardness of its commented-out driver line, on the F 8192 instance
]


@pytest.mark.parametrize("prec", PRECISIONS)
@pytest.mark.parametrize("F,S,pa,p", PA_PATHS)
def test_pa_paths_per_instance_vs_oracle(F, S, pa, p, prec):
    """Every PA branch of pa_block() in the F 2048 and F 4096 instances (the PA kind is a
    run-time switch inside one instance; the general-p Rapp is out of line in both since round
    6): per-trial counts EXACTLY equal to the oracle's."""
    A, M = 8, 64
    snr = float(sim.rm.ebn0_to_snr(12.0, S, S, M))
    cfg = sim.SimConfig(A, S, F, M, pa=pa, p_hardness=p, ibo_db=1.5, snr_db=snr)
    iters = [0, 1, 2]
    n = 6
    ref = sim.run_trials(cfg, 515, np.arange(n), iters=iters, incl_clean=True, chunk=2)
    eng = engine_for(cfg, precision=prec)
    _, _, per = eng.run(515, 0, n, iters, True, per_trial=True)
    print("pa path", F, S, pa, p, eng.describe(), per.sum(0), ref.sum(0))
    assert_counts_equal(per, ref, f"{F}/{S}/{pa}/{p} {prec}")


ARRAY_ALPHA = [
    # F,    S,    pa,        receiver, prec
    (2048, 1024, "toi", "cnc", "f64"),
    (2048, 1024, "toi", "cnc", "f32"),
    (4096, 2048, "toi", "cnc", "f64"),
    (4096, 2048, "toi", "mcnc", "f64"),
    (4096, 2048, "toi", "cnc", "f32"),
    (8192, 4096, "toi", "cnc", "f64"),
    (2048, 1024, "softlim", "cnc", "f64"),
]


@pytest.mark.parametrize("F,S,pa,receiver,prec", ARRAY_ALPHA)
def test_fixed_array_alpha_vs_oracle(F, S, pa, receiver, prec):
    """mimo_point.array_alpha (ABI 8): one Bussgang gain for every antenna's AGC term and the
    CNC receiver's alpha, as the TOI drivers run them (main_miso_cnc_ber_vs_ebn0_toi.py:95-134,
    247-259) -- the kernel's alpha polynomial held constant.  Two-path channel (the TOI
    drivers'), per-trial counts EXACTLY equal to the oracle's with the same fixed gain."""
    A, M = 4, 64
    snr = float(sim.rm.ebn0_to_snr(14.0, S, S, M))
    cfg = sim.SimConfig(A, S, F, M, pa=pa, ibo_db=8.0 if pa == "toi" else 2.0, snr_db=snr, channel="two_path",
                        receiver=receiver, array_alpha=0.93, cnc_alpha=0.93)
    iters = [0, 1, 2]
    n = 4
    ref = sim.run_trials(cfg, 777, np.arange(n), iters=iters, incl_clean=True, chunk=2)
    eng = engine_for(cfg, precision=prec)
    _, _, per = eng.run(777, 0, n, iters, True, per_trial=True)
    print("fixed alpha", F, S, pa, receiver, prec, eng.describe(), per.sum(0), ref.sum(0))
    assert_counts_equal(per, ref, f"{F}/{S}/{pa}/{receiver} fixed alpha {prec}")
    # and it is not the per-antenna gain: the oracle without the override counts differently
    cfg0 = sim.SimConfig(A, S, F, M, pa=pa, ibo_db=cfg.ibo_db, snr_db=snr, channel="two_path", receiver=receiver,
                         cnc_alpha=0.93)
    ref0 = sim.run_trials(cfg0, 777, np.arange(n), iters=iters, incl_clean=True, chunk=2)
    assert (ref0 != ref).any()


@pytest.mark.parametrize("F,S,n", [(8192, 4096, 2), (4096, 2048, 3)])
def test_csi_at_max_antennas_vs_oracle(F, S, n):
    """CSI error at n_ant = kMaxCsiAnt (512), where the per-antenna power table is
    4 KiB of dynamic LDS next to the instance's static LDS (the F 8192 split-FFT instance holds
    ~157 KiB: the edge of the CU's 160 KiB; engine.hip checks the sum before launching).
    float64, per-trial counts EXACTLY equal to the oracle's."""
    M = 16
    snr = float(sim.rm.ebn0_to_snr(10.0, S, S, M))
    cfg = sim.SimConfig(512, S, F, M, pa="softlim", ibo_db=2.0, snr_db=snr, channel="rayleigh", receiver="cnc",
                        csi_eps=0.2)
    iters = [0, 1]
    ref = sim.run_trials(cfg, 88, np.arange(n), iters=iters, incl_clean=True, chunk=1)
    eng = engine_for(cfg, precision="f64")
    _, _, per = eng.run(88, 0, n, iters, True, per_trial=True)
    print("csi max ant", F, eng.describe(), per.sum(0), ref.sum(0))
    assert_counts_equal(per, ref, f"CSI A=512 F={F} f64")

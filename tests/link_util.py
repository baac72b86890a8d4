"""Build reference-style systems with the MI355X host mirror (same calls as the drivers)."""
import copy


def build_link(n_ant=8, n_sc=64, n_fft=128, M=16, cp=4, pa="softlim", ibo=1.0, p_hard=3.0, chan="rayleigh",
               is_mcnc=False, n_err_min=10 ** 12, bits_sent_max=10 ** 6, csi=None, **kw):
    import antenna_array
    import channel
    import distortion
    import modulation
    import mp_model
    import noise
    import transceiver

    mod = modulation.OfdmQamModem(constel_size=M, n_fft=n_fft, n_sub_carr=n_sc, cp_len=cp)
    if pa == "softlim":
        dist = distortion.SoftLimiter(0, mod.avg_sample_power)
    elif pa == "rapp":
        dist = distortion.Rapp(ibo_db=0, p_hardness=p_hard, avg_samp_pow=mod.avg_sample_power)
    elif pa == "toi":
        dist = distortion.ThirdOrderNonLin(toi_db=ibo, avg_samp_pow=mod.avg_sample_power)
    else:
        raise ValueError(pa)
    tx = transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist), center_freq=int(3.5e9),
                                 carrier_spacing=int(15e3))
    rx = transceiver.Transceiver(modem=copy.deepcopy(mod), impairment=copy.deepcopy(dist), cord_x=212.0, cord_y=212.0,
                                 cord_z=1.5, center_freq=int(3.5e9), carrier_spacing=int(15e3))
    arr = antenna_array.LinearArray(n_elements=n_ant, base_transceiver=tx, center_freq=int(3.5e9), wav_len_spacing=0.5,
                                    cord_x=0, cord_y=0, cord_z=15)
    if chan == "rayleigh":
        ch = channel.MisoRayleighFd(tx_transceivers=arr.array_elements, rx_transceiver=rx, seed=1234)
    elif chan == "los":
        ch = channel.MisoLosFd()
        ch.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx, skip_attenuation=False)
    else:
        ch = channel.MisoTwoPathFd()
        ch.calc_channel_mat(tx_transceivers=arr.array_elements, rx_transceiver=rx, skip_attenuation=False)
    link = mp_model.Link(mod_obj=mod, array_obj=arr, std_rx_obj=rx, chan_obj=ch, noise_obj=noise.Awgn(snr_db=10, seed=1),
                         rx_loc_var=10.0, n_err_min=n_err_min, bits_sent_max=bits_sent_max, is_mcnc=is_mcnc,
                         csi_epsylon=csi, **kw)
    link.update_distortion(ibo_val_db=ibo)
    return link, mod


def simulate_child(link, seed_arr, err, bits, iters=(0, 1)):
    """Target of a spawned worker: what a reference driver's mp.Process runs
    (main_mp_miso_cnc_ber_vs_ebn0.py:122-132)."""
    import numpy as np
    link.simulate(True, True, np.asarray(iters), seed_arr, err, bits)


def simulate_child_counting(link, seed_arr, err, bits, created, iters=(0, 1)):
    """simulate_child, counting the engines this worker creates into ``created`` (an
    mp.Value): the per-device slot cap must keep the total at MIMO_MAX_ENGINES_PER_DEVICE."""
    import numpy as np

    import _engine
    orig = _engine.Engine.__init__

    def counted(self, *a, **k):
        with created.get_lock():
            created.value += 1
        orig(self, *a, **k)

    _engine.Engine.__init__ = counted
    link.simulate(True, True, np.asarray(iters), seed_arr, err, bits)


def sweep_rank(rank, world, port, out, kw, ibo, ebn0, iters, split="points"):
    """One rank of a gloo-sharded sweep through the real Link -> engine path (all ranks on
    GPU 0, as MIMO_BENCH_BACKEND=gloo rehearses bench.py)."""
    import os

    import numpy as np
    import torch.distributed as dist

    import sweep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    link, _ = build_link(device=0, **kw)
    err, bits = sweep.run_grid(link, ibo, ebn0, iters, False, 11, rank, world, dist, split=split)
    np.save(os.path.join(out, "r%d.npy" % rank), np.stack([err, bits]))
    dist.destroy_process_group()

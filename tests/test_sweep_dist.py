"""Grid sweep sharding + the single counter collective, on CPU with gloo (world_size 2),
and the reference CSV layouts / fixed-BER interpolation."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as tmp


from fake_link import FakeLink  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch.distributed as dist
    import sweep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    err, bits = sweep.run_grid(FakeLink(), [0.0, 1.0, 2.0], np.arange(5.0, 15.0, 2.0), [0, 1, 2], True, 7, rank,
                               world, dist)
    np.save(os.path.join(out, f"r{rank}.npy"), np.stack([err, bits]))
    dist.destroy_process_group()


def test_sharded_sweep_matches_single_process(tmp_path):
    import sweep
    ref_err, ref_bits = sweep.run_grid(FakeLink(), [0.0, 1.0, 2.0], np.arange(5.0, 15.0, 2.0), [0, 1, 2], True, 7)
    tmp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        got = np.load(os.path.join(tmp_path, f"r{r}.npy"))
        np.testing.assert_array_equal(got[0], ref_err)
        np.testing.assert_array_equal(got[1], ref_bits)
    assert ref_err.shape == (3, 5, 4)


def test_owned_points_partition():
    import sweep
    for world in (1, 2, 3, 8):
        pts = sorted(p for r in range(world) for p in sweep.owned_points(37, r, world))
        assert pts == list(range(37))


def test_required_ebn0_and_csv_layout(tmp_path):
    import sweep
    import utilities
    ebn0 = np.arange(10.0, 13.1, 1.0)
    ber = np.zeros((2, 4, 2))
    ber[:, :, 0] = [[0.1, 0.03, 0.005, 0.001], [0.2, 0.1, 0.05, 0.02]]
    ber[:, :, 1] = [[0.05, 0.01, 0.002, 0.0005], [0.1, 0.05, 0.011, 0.003]]
    req = sweep.required_ebn0(ber, ebn0, 1e-2)
    assert req[0, 0] == pytest.approx(11 + (0.03 - 0.01) / (0.03 - 0.005), rel=1e-12)
    assert req[0, 1] == np.inf  # target outside the measured range
    assert req[1, 0] == pytest.approx(11.0)
    rows = sweep.fixed_ber_rows([0.0, 0.5], ber)
    assert len(rows) == 1 + 2 * 4 and list(rows[0]) == [0.0, 0.5]
    utilities.save_to_csv(rows, "fixed", directory=str(tmp_path))
    back = utilities.read_from_csv("fixed", directory=str(tmp_path))
    np.testing.assert_allclose(back[1], ber[0, 0])
    assert sweep.ber_from_counts([1, 0], [0, 4])[0] != sweep.ber_from_counts([1, 0], [0, 4])[0]  # NaN


def test_published_csv_layout_readable():
    """The reference's own CSV (ber_vs_ebn0 layout) parses with our reader."""
    import utilities
    d = os.path.join(os.path.dirname(__file__), "golden")
    rows = utilities.read_from_csv("published_ber_vs_ebn0_cnc_rayleigh_ibo3", directory=d)
    assert rows[0][0] == 5.0 and len(rows) == 11 and len(rows[1]) == 16


def test_sweep_shards_cover_and_balance():
    import sweep
    costs = sweep.point_costs(np.arange(0, 8, 0.5), np.arange(10, 22.1, 0.5), 12288, 64, 1e5, 5e6, range(9))
    for world in (1, 2, 3, 8):
        parts = [sweep.owned_points(len(costs), r, world, costs) for r in range(world)]
        assert sorted(p for q in parts for p in q) == list(range(len(costs)))
        loads = [costs[q].sum() for q in parts]
        assert max(loads) <= min(loads) + costs.max()


def test_cli_default_grid_is_the_published_one():
    # sweep.py's default --ibo / --ebn0 axes give the published fixed-BER grids' points
    # (header: the IBO axis; one row of 9 counters per (IBO, Eb/N0) point)
    import sweep
    src = open(sweep.__file__).read()
    ibo = [a for a in src.split("\n") if '"--ibo"' in a][0].split('default="')[1].split('"')[0]
    ebn0 = [a for a in src.split("\n") if '"--ebn0"' in a][0].split('default="')[1].split('"')[0]
    rng = lambda s: np.arange(*[float(x) for x in s.split(":")])  # noqa: E731
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    f = ("published_fixed_ber1.0e-02_cnc_rayleigh_nant64_ebn0_min10_max22_step0.50_ibo_min0_max7_step0.50_"
         "niter1_2_3_4_5_6_7_8.csv")
    lines = open(os.path.join(d, f)).read().strip().split("\n")
    np.testing.assert_allclose(rng(ibo), np.array(lines[0].split(","), dtype=float))
    assert len(rng(ibo)) * len(rng(ebn0)) == len(lines) - 1
    assert rng(ebn0)[0] == 10.0 and rng(ebn0)[-1] == 22.0

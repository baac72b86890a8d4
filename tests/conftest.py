import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG, os.path.join(REPO, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def link_fixture_names():
    return sorted(f[5:-4] for f in os.listdir(GOLDEN) if f.startswith("link_") and f.endswith(".npz"))


def sim_config_from_fixture(g):
    from oracle.sim import SimConfig
    return SimConfig(n_ant=int(g["n_ant"]), n_sc=int(g["n_sc"]), n_fft=int(g["n_fft"]), constel_size=int(g["M"]),
                     pa=str(g["pa"]), p_hardness=float(g["p_hard"]), ibo_db=float(g["ibo"]),
                     snr_db=float(g["snr_db"]), channel=str(g["chan"]),
                     receiver="mcnc" if int(g["mcnc"]) else "cnc",
                     csi_eps=None if float(g["csi"]) < 0 else float(g["csi"]))


@pytest.fixture
def units():
    return load_golden("units.npz")

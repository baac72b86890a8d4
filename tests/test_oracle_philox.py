"""Philox4x32-10 known-answer tests (Random123 kat_vectors) and stream-layout properties."""
import numpy as np
import pytest

from oracle import philox


@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), 0, (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, 0xffffffffffffffff, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0x299f31d0 << 32) | 0xa4093822,
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_kat(ctr, key, expect):
    out = philox.philox4x32_10(*ctr, key)
    assert tuple(int(x) for x in out) == expect


def test_pairing_is_a_bijection():
    for S in (64, 1024, 4096):
        q, slot = philox.pair_index(np.arange(S), S)
        assert sorted(zip(q.tolist(), slot.tolist())) == sorted((i, j) for i in range(S // 2) for j in (0, 1))


def test_normals_moments():
    z = philox.chan_normals(7, np.arange(64), 256, 8).reshape(-1)
    assert abs(np.mean(np.abs(z) ** 2) - 1) < 0.01
    assert abs(np.mean(z)) < 0.01
    assert abs(np.mean(z.real * z.imag)) < 0.01


def test_labels_uniform():
    lab = philox.qam_labels(3, np.arange(256), 1024, 64)
    counts = np.bincount(lab.reshape(-1), minlength=64)
    assert counts.min() > 0.9 * counts.mean() and counts.max() < 1.1 * counts.mean()

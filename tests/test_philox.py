"""Philox4x32-10 of the oracle against the published Random123 known-answer vectors."""

import numpy as np
import pytest

KATS = [  # counter (4 words), key (2 words), output -- Random123 kat_vectors, philox4x32 10 rounds
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,out", KATS)
def test_philox_kat(coracle, ctr, key, out):
    np.testing.assert_array_equal(coracle.philox(ctr, key), np.array(out, np.uint32))


def test_action_draws_are_uniform_and_shard_invariant(coracle):
    a1, a2 = coracle.random_actions(200000, 0, 42, 7, True)
    freq = np.bincount(a1, minlength=5) / len(a1)
    assert np.all(np.abs(freq - 0.2) < 0.005)
    assert set(np.unique(a2)) == {0, 1, 2, 3, 4}
    b1, b2 = coracle.random_actions(1000, 5000, 42, 7, True)
    np.testing.assert_array_equal(b1, a1[5000:6000])
    np.testing.assert_array_equal(b2, a2[5000:6000])
    _, n2 = coracle.random_actions(10, 0, 42, 7, False)
    assert np.all(n2 == -1)

"""mg_qnet_fragments (ABI 18): the fragment-major copy of a packed Q-net that mg_rollout_hdqn reads
an opponent from another checkpoint in (hdqn.py:265-268). Fragment s is the 64 lanes' 16 bytes of
the s-th MFMA operand of one forward, in the order the kernel consumes them; lane l = 32 h + r
reads row r (clamped to the last stored row) of the row tile, columns 8 h .. 8 h + 7 of the
16-column k-block. Restated here from the packed layout (include/merging_hip.h: W1 [204 x 24],
W2 [104 x 232], W3 [9 x 136] bf16 rows) and compared byte for byte with the device copy."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R1, S1, R2, S2, R3, S3 = 204, 24, 104, 232, 9, 136
OFF_W2 = R1 * S1 * 2
OFF_W3 = OFF_W2 + R2 * S2 * 2


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def _order():
    """(matrix, row tile or None, k-block) of fragment s = 0..65 in consumption order: W1(0);
    per hidden tile mt = 0..5: W1(mt + 1), then W2 pairs j = 0..7 (row tile j >> 1, k-block
    2 mt + (j & 1)); the last tile's pairs interleaved with layer 3:
    W2(6, 0), W2(6, 2), W3(0), W3(1), W2(6, 4), W3(2), W3(3), W2(6, 6), W3(4), W3(5), W3(6)."""
    out = [("w1", 0, 0)]
    for mt in range(6):
        out.append(("w1", mt + 1, 0))
        out += [("w2", j >> 1, 2 * mt + (j & 1)) for j in range(8)]
    tail = [("w2", 0, 12), ("w2", 1, 12), ("w3", None, 0), ("w3", None, 1), ("w2", 2, 12), ("w3", None, 2),
            ("w3", None, 3), ("w2", 3, 12), ("w3", None, 4), ("w3", None, 5), ("w3", None, 6)]
    return out + tail


def _expected(packed):
    b = np.asarray(packed, np.uint8)
    frags = np.zeros((66, 64, 16), np.uint8)
    for s, (m, tile, kb) in enumerate(_order()):
        for lane in range(64):
            r, h = lane & 31, lane >> 5
            if m == "w1":
                row, base, stride, col = min(32 * tile + r, R1 - 1), 0, S1, 8 * h
            elif m == "w2":
                row, base, stride, col = min(32 * tile + r, R2 - 1), OFF_W2, S2, 16 * kb + 8 * h
            else:
                row, base, stride, col = min(r, R3 - 1), OFF_W3, S3, 16 * kb + 8 * h
            o = base + 2 * (row * stride + col)
            frags[s, lane] = b[o:o + 16]
    return frags.reshape(-1)


@pytest.mark.parametrize("in_dim,out_dim", [(10, 3), (11, 5)])
def test_fragment_copy_matches_the_packed_layout(torch, in_dim, out_dim):
    from merging_gym.policy import QNet

    rng = np.random.default_rng(in_dim * 7 + out_dim)
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-i ** -0.5, i ** -0.5, (o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    net = QNet.from_state_dict(sd, device="cuda:0")
    frags = net.fragments.cpu().numpy()
    assert frags.shape == (66 * 1024,)
    np.testing.assert_array_equal(frags, _expected(net.packed.cpu().numpy()))

"""mg_qnet_pack (ABI 19): the packed Q-net starts with the 16x16 forward's MFMA operand fragments in
the order the kernel consumes them, each the 64 lanes' 16 bytes contiguous (include/merging_hip.h). Restated here
in numpy from the fp32 torch weights of scripts/main.py:30-47's Net -- bf16 rounding, the three-way
bf16 split of every bias, the 1.0 units and the k orders of the layer-2 / layer-3 operands -- and
compared byte for byte with the device's packed net (both layouts) and with its fragment copy (mg_qnet_fragments,
which the h-DQN kernel reads an opponent from another checkpoint in, hdqn.py:265-268)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def _order():
    """(kind, tile, k-block) of fragment s = 0..59: W1(0); per k-block kb = 0..5: W1(kb + 1), W2(t, kb)
    for t = 0..6; the last k-block with layer 3: W2(0..2, 6), W3(0), W2(3..4, 6), W3(1), W2(5..6, 6),
    W3(2), W3(3)."""
    out = [("w1", 0, 0)]
    for kb in range(6):
        out.append(("w1", kb + 1, 0))
        out += [("w2", t, kb) for t in range(7)]
    out += [("w2", 0, 6), ("w2", 1, 6), ("w2", 2, 6), ("w3", 0, 0), ("w2", 3, 6), ("w2", 4, 6), ("w3", 0, 1),
            ("w2", 5, 6), ("w2", 6, 6), ("w3", 0, 2), ("w3", 0, 3)]
    return out


def _bf16_bits(x):
    """fp32 -> bf16 bit patterns, round to nearest even (as the device's conversion)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return r.astype(np.uint16)


def _bf16(x):
    return (_bf16_bits(x).astype(np.uint32) << 16).view(np.float32)


def _parts(b):
    """hi + mid + lo == b, each a bf16 value (mg_qnet_pack's bias split)."""
    b = np.asarray(b, np.float32)
    hi = _bf16(b)
    r = (b - hi).astype(np.float32)
    mid = _bf16(r)
    return hi, mid, (r - mid).astype(np.float32)


def _expected(sd, in_dim, out_dim):
    w1, b1 = sd["fc1.weight"], sd["fc1.bias"]
    w2, b2 = sd["fc2.weight"], sd["fc2.bias"]
    w3, b3 = sd["out.weight"], sd["out.bias"]
    W1 = np.zeros((224, 16), np.float32)  # [hidden-1 unit, input slot]
    W1[:200, :in_dim] = w1
    W1[:200, 13:16] = np.stack(_parts(b1), 1)
    W1[200:203, 13] = 1.0
    W2 = np.zeros((112, 224), np.float32)  # [hidden-2 unit, hidden-1 unit]
    W2[:100, :200] = w2
    W2[:100, 200:203] = np.stack(_parts(b2), 1)
    W2[100:103, 200] = 1.0
    W3 = np.zeros((8, 128), np.float32)  # [output, hidden-2 unit]
    W3[:out_dim, :100] = w3
    W3[:out_dim, 100:103] = np.stack(_parts(b3), 1)
    lane = np.arange(64)[:, None]
    j = np.arange(8)[None, :]
    g = lane >> 4
    frags = []
    for kind, tile, kb in _order():
        if kind == "w1":
            vals = W1[32 * tile + (lane & 31), 8 * (lane >> 5) + j]
        elif kind == "w2":
            unit = 32 * kb + (j & 3) + 8 * (j >> 2) + 16 * (g & 1) + 4 * (g >> 1)
            vals = W2[16 * tile + (lane & 15), unit]
        else:  # rows 0..7 only: 512 B, row-group g at 128 g
            unit = 32 * kb + 16 * (j >> 2) + 4 * g + (j & 3)
            vals = W3[lane & 7, unit].reshape(4, 16, 8)[:, :8].reshape(32, 8)
        frags.append(_bf16_bits(vals).reshape(-1))
    return np.concatenate(frags).view(np.uint8)


def _expected32(sd, in_dim, out_dim):
    """The 32x32 layout after the fragments (the ego-only config-5 instances): W1 [204 x 24], W2
    [104 x 232], W3 [9 x 136] bf16 rows; W2 / W3 columns in the 32x32 accumulator's k order
    (16-column blocks, k -> unit 8 ((k & 7) >> 2) + 4 (k >> 3) + (k & 3)); rows past the last one
    that can be non-zero are not stored."""
    w1, b1 = sd["fc1.weight"], sd["fc1.bias"]
    w2, b2 = sd["fc2.weight"], sd["fc2.bias"]
    w3, b3 = sd["out.weight"], sd["out.bias"]
    W1 = np.zeros((204, 24), np.float32)
    W1[:200, :in_dim] = w1
    W1[:200, 13:16] = np.stack(_parts(b1), 1)
    W1[200:203, 13] = 1.0
    H1 = np.zeros((104, 224), np.float32)  # [hidden-2 unit, hidden-1 unit]
    H1[:100, :200] = w2
    H1[:100, 200:203] = np.stack(_parts(b2), 1)
    H1[100:103, 200] = 1.0
    H2 = np.zeros((9, 128), np.float32)  # [output, hidden-2 unit]
    H2[:out_dim, :100] = w3
    H2[:out_dim, 100:103] = np.stack(_parts(b3), 1)
    c = np.arange(232)
    kk = c % 16
    src = 16 * (c // 16) + 8 * ((kk & 7) >> 2) + 4 * (kk >> 3) + (kk & 3)
    W2 = np.where(c[None, :] < 224, H1[:, np.minimum(src, 223)], 0.0).astype(np.float32)
    c3 = np.arange(136)
    kk3 = c3 % 16
    src3 = 16 * (c3 // 16) + 8 * ((kk3 & 7) >> 2) + 4 * (kk3 >> 3) + (kk3 & 3)
    W3 = np.where(c3[None, :] < 128, H2[:, np.minimum(src3, 127)], 0.0).astype(np.float32)
    return np.concatenate([_bf16_bits(m).reshape(-1) for m in (W1, W2, W3)]).view(np.uint8)


@pytest.mark.parametrize("in_dim,out_dim", [(10, 3), (11, 5), (10, 8), (13, 1)])
def test_packed_layout_restated_from_the_weights(torch, in_dim, out_dim):
    from merging_gym.policy import QNet

    rng = np.random.default_rng(in_dim * 7 + out_dim)
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-i ** -0.5, i ** -0.5, (o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    net = QNet.from_state_dict(sd, device="cuda:0")
    packed = net.packed.cpu().numpy()
    n16 = 56 * 1024 + 4 * 512  # then the 32x32 layout of the ego-only config-5 instances
    assert packed.shape == (n16 + 2 * (204 * 24 + 104 * 232 + 9 * 136),)
    np.testing.assert_array_equal(packed[:n16], _expected(sd, in_dim, out_dim))
    np.testing.assert_array_equal(packed[n16:], _expected32(sd, in_dim, out_dim))
    # mg_qnet_fragments (ABI 18 callers) copies the fragment-major first part; QNet.fragments is a
    # deprecated alias of packed itself, which the kernels read an other-checkpoint opponent from
    from merging_gym import _native

    frag = torch.empty(n16, dtype=torch.uint8, device="cuda:0")
    _native.check(_native.lib.mg_qnet_fragments(net.packed.data_ptr(), frag.data_ptr(), None), "mg_qnet_fragments")
    np.testing.assert_array_equal(frag.cpu().numpy(), packed[:n16])
    assert net.fragments is net.packed

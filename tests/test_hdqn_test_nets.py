"""The h-DQN GPU tests' synthetic nets do what their docstrings claim, on the CPU oracle's
bf16-emulated forward (oracle/merge_oracle.py qnet_reference): the selector net's greedy choice
turns on input 1 alone, and the signed-weight nets' choices vary from input to input (unlike
hdqn.py:41-47's uniform(0, 1) nets, which pick nearly one action everywhere)."""

import numpy as np

import merge_oracle as mo
from test_gpu_hdqn import _net, _net_signed, _selector_net


def test_selector_net_reads_input_one():
    rng = np.random.default_rng(0)
    x = rng.uniform(-60, 60, (500, 11)).astype(np.float32)
    q = mo.qnet_reference(_selector_net(10.0), x, bf16=True)
    x1 = x[:, 1].astype(np.float32)
    bf = x1.astype(np.float32).view(np.uint32)
    x1_bf16 = ((bf + 0x7FFF + ((bf >> 16) & 1)) & 0xFFFF0000).view(np.float32)  # round to nearest even
    np.testing.assert_allclose(q[:, 0], np.maximum(x1_bf16, 0), rtol=0, atol=0)
    assert (q[:, 1] == 10.0).all() and (q[:, 2:] == 0).all()
    away = np.abs(x1 - 10.0) > 1.0
    np.testing.assert_array_equal(q.argmax(1)[away], np.where(x1[away] > 10.0, 0, 1))


def test_signed_nets_vary_their_choice_uniform_nets_do_not():
    rng = np.random.default_rng(1)
    obs = np.concatenate([rng.uniform(-300, 300, (2000, 5)), rng.uniform(-50, 950, (2000, 5))], 1)
    x = np.concatenate([rng.integers(0, 3, (2000, 1)), obs], 1).astype(np.float32)  # [goal] + state
    signed = mo.qnet_reference(_net_signed(np.random.default_rng(2), 11, 5), x, bf16=True).argmax(1)
    uniform = mo.qnet_reference(_net(np.random.default_rng(2), 11, 5), x, bf16=True).argmax(1)
    counts_s = np.bincount(signed, minlength=5)
    counts_u = np.bincount(uniform, minlength=5)
    assert (counts_s > 0).sum() >= 3 and counts_s.max() < 0.8 * len(x), counts_s
    assert counts_u.max() > 0.9 * len(x), counts_u  # why the swapped-input bug hid

"""Offline half of the summation-order study: compares the Q-values mg_qnet_forward returned on the
MI355X (saved by tools/mfma_order_dump.py) with the oracle's models of the matrix cores' addition
order (oracle/merge_oracle.py qnet_reference_mfma: the measured rule "mfma", round 5's "exact8" model)
and with an fp32 matmul of the same bf16 operands. Prints the fraction of rows equal bit for bit per net
and view.

    python tools/mfma_order_study.py gpurun_out/r05i/qdump.npz > profiles/r06/mfma_order.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import merge_oracle as mo  # noqa: E402


def rows_equal(a, b):
    return float(np.mean(np.all(a.view(np.uint32) == b.view(np.uint32), axis=1)))


def fp32_matmul(w, x, swap=False):
    bf = mo._bf16
    x = np.asarray(x, np.float32)
    if swap:
        x = np.concatenate([x[:, 5:], x[:, :5]], axis=1)
    h = bf(x)
    for i, (wk, bk) in enumerate((("fc1.weight", "fc1.bias"), ("fc2.weight", "fc2.bias"), ("out.weight", "out.bias"))):
        h = h @ bf(w[wk]).T + w[bk].astype(np.float32)
        if i < 2:
            h = bf(np.maximum(h, 0.0))
    return h.astype(np.float32)


def main(path):
    d = np.load(path)
    ck = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    print(f"summation-order study over {path} ({len(d['obs'])} observations per net)")
    print("fraction of Q rows equal bit for bit to mg_qnet_forward on the MI355X")
    cases = []
    for key in ("l1", "l3"):
        w = {n.split("/", 1)[1]: ck[n] for n in ck.files if n.startswith(key + "/")}
        for swap in (0, 1):
            cases.append((f"{key} swap={swap}", w, d["obs"], bool(swap), d[f"{key}_swap{swap}"]))
    for name in ("meta", "lower"):
        w = {k.split("/", 1)[1]: d[k] for k in d.files if k.startswith(name + "/")}
        cases.append((f"{name} (seeded signed)", w, d[f"{name}_x"], False, d[f"{name}_q"]))
    for label, w, x, swap, got in cases:
        r = mo.qnet_reference_mfma(w, x, swap=swap, rule="mfma")
        g = mo.qnet_reference_mfma(w, x, swap=swap, rule="exact8")
        m = fp32_matmul(w, x, swap)
        print(f"  {label:22s} measured rule {rows_equal(r, got):.6f} ({int(np.sum(np.all(r.view(np.uint32) == got.view(np.uint32), 1)))}/{len(got)})"
              f"  round-5 exact-8 {rows_equal(g, got):.6f}  fp32 matmul {rows_equal(m, got):.6f}"
              f"  max |rule - kernel| {float(np.max(np.abs(r - got))):.3g}")


if __name__ == "__main__":
    main(sys.argv[1])

"""Writes tests/golden/mfma_probe_golden.npz: matrix-core outputs recorded on the MI355X, the fixture
that pins the oracle's restated bf16 MFMA accumulation rule (oracle/merge_oracle.c oracle_mfma_dots,
oracle.merge_oracle.qnet_reference_mfma) in the CPU suite (tests/test_oracle_mfma.py).

    python tests/golden/gen_mfma_golden.py [R06A R06B R06C QDUMP]

Sources (gpurun_out/ of this repository's GPU runs):
  r06a/mfma_numerics.npz  random-family single MFMAs (tools/mfma_numerics.py collect)     -> D16, D32
  r06b/mfma_struct.npz    structured probes (grouping, alignment, rounding; ... struct)  -> S16, S32
  r06c/mfma_single.npz    one-step families (... single)                                  -> E16, E32
  r05i/qdump.npz          mg_qnet_forward's Q rows (tools/mfma_order_dump.py)             -> q_* / x_*
Only outputs are stored for the probes: their operands regenerate bit for bit from the seeded
generators in mfma_probe_cases.py (the stored digests check that). For the Q rows the inputs are
stored with the outputs: every row round 5's model missed plus 2,048 others per net and view.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from mfma_probe_cases import make_case, make_case2  # noqa: E402

N_CASES = {16: 256, 32: 64}  # cases kept per form: 65,536 outputs each


def digest(form, n, maker):
    h = hashlib.sha256()
    for i in range(n):
        A, B, C, _ = maker(form, i)
        h.update(A.tobytes() + B.tobytes() + C.tobytes())
    return h.hexdigest()[:16]


def main(a, b, c, qd):
    import merge_oracle as mo

    da, db, dc, dq = (np.load(p) for p in (a, b, c, qd))
    out = {}
    for form in (16, 32):
        n = N_CASES[form]
        out[f"D{form}"] = da[f"D{form}"][:n]
        out[f"E{form}"] = dc[f"E{form}"][:n]
        out[f"S{form}"] = db[f"S{form}"]
        out[f"digestD{form}"] = np.array(digest(form, n, make_case))
        out[f"digestE{form}"] = np.array(digest(form, n, make_case2))
    ck = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    rng = np.random.default_rng(6)
    cases = [(f"{k}_swap{s}", {n.split("/", 1)[1]: ck[n] for n in ck.files if n.startswith(k + "/")}, dq["obs"], bool(s),
              dq[f"{k}_swap{s}"]) for k in ("l1", "l3") for s in (0, 1)]
    for name in ("meta", "lower"):
        w = {k.split("/", 1)[1]: dq[k] for k in dq.files if k.startswith(name + "/")}
        cases.append((name, w, dq[f"{name}_x"], False, dq[f"{name}_q"]))
        for k, v in w.items():
            out[f"w_{name}/{k}"] = v
    for name, w, x, swap, q in cases:
        old = mo.qnet_reference_mfma(w, x, swap=swap, rule="exact8")
        missed = np.flatnonzero(~np.all(old.view(np.uint32) == q.view(np.uint32), 1))
        keep = np.union1d(missed, rng.choice(len(x), 2048, replace=False))
        out[f"x_{name}"] = x[keep]
        out[f"q_{name}"] = q[keep]
        out[f"missed_r5_{name}"] = np.isin(keep, missed)
        print(name, "rows", len(keep), "round-5 model missed", len(missed))
    np.savez_compressed(os.path.join(HERE, "mfma_probe_golden.npz"), **out)


if __name__ == "__main__":
    g = os.path.join(ROOT, "gpurun_out")
    args = sys.argv[1:] or [os.path.join(g, "r06a", "mfma_numerics.npz"), os.path.join(g, "r06b", "mfma_struct.npz"),
                            os.path.join(g, "r06c", "mfma_single.npz"), os.path.join(g, "r05i", "qdump.npz")]
    main(*args)

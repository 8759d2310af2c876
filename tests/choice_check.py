"""Greedy choices of the fused bf16 kernels against the bf16-emulated reference nets
(oracle.qnet_reference: bf16 operands, fp32 sums), with the near-tie excusal bounded.

The kernels and the CPU emulation sum in different orders; a sum that lands on the other side of
a bf16 rounding boundary moves one hidden unit by 2^-8 of itself, and that can reorder two
actions whose Q-values are that close. So a greedy choice that differs from the emulation's
argmax is excused only when the action the kernel took has an emulated Q within `tol` (relative
to max(1, |Q_max|)) of the row's maximum -- never any other action -- and every check counts
the excused choices; `finish()` prints the fraction and asserts it is below the test's bound.
Random (exploring) choices are exact: they come from the Philox draws alone.

Round 6: the excusal is no longer the last word. A check given `q_exact` (exact_q below: the
oracle's restatement of the matrix cores' accumulation, oracle.merge_oracle.qnet_reference_mfma,
pinned to recorded MI355X outputs by tests/test_oracle_mfma.py) requires EVERY greedy choice to equal
that model's argmax (first maximum, as the kernels' argmax_first), near-ties included; the fp32
emulation's disagreements are still counted and bounded, and each one is thereby explained.
"""

from __future__ import annotations

import numpy as np


# every finished check's line, printed again at the end of the session by tests/conftest.py
# (pytest_terminal_summary), so the fractions are in the log even when output is captured (-q)
SUMMARY: list[str] = []


class ChoiceCheck:
    def __init__(self, name: str, tol: float = 1e-2, max_frac: float | None = None):
        self.name, self.tol, self.max_frac = name, tol, max_frac
        self.greedy = 0
        self.excused = 0
        self.exact = 0       # greedy choices checked against the oracle's MFMA-rule argmax
        self.exact_fp32 = 0  # ... of which the fp32 emulation's argmax differs (near-ties)

    def check(self, got, exp, greedy, q, what="", q_exact=None):
        got = np.asarray(got).astype(np.int64)
        exp = np.asarray(exp).astype(np.int64)
        greedy = np.asarray(greedy, bool)
        q = np.asarray(q, np.float64)
        n, k = q.shape
        qmax = q.max(axis=1)
        qgot = q[np.arange(n), np.clip(got, 0, k - 1)]
        within = (got >= 0) & (got < k) & (qmax - qgot <= self.tol * np.maximum(1.0, np.abs(qmax)))
        differ = got != exp
        excused = greedy & differ & within
        bad = differ & ~excused
        self.greedy += int(greedy.sum())
        self.excused += int(excused.sum())
        if bad.any():
            i = np.flatnonzero(bad)
            s = np.sort(q[i], axis=1)
            gap = (s[:, -1] - s[:, -2]) / np.maximum(1.0, np.abs(s[:, -1]))
            raise AssertionError(
                f"{self.name} {what}: {i.size} of {n} choices differ beyond a near-tie; envs {i[:8].tolist()}, got "
                f"{got[i[:8]].tolist()}, expected {exp[i[:8]].tolist()}, greedy {greedy[i[:8]].tolist()}, "
                f"top-2 gap {gap[:8].tolist()}, q {q[i[:3]].tolist()}")
        if q_exact is not None:
            idx = np.flatnonzero(greedy)
            if idx.size:
                qx = q_exact(idx) if callable(q_exact) else np.asarray(q_exact)[idx]
                want = np.asarray(qx).argmax(axis=1)
                miss = got[idx] != want
                if miss.any():
                    j = idx[miss]
                    raise AssertionError(
                        f"{self.name} {what}: {j.size} of {idx.size} greedy choices differ from the oracle MFMA "
                        f"rule's argmax; envs {j[:8].tolist()}, got {got[j[:8]].tolist()}, model "
                        f"{want[miss][:8].tolist()}, model q {np.asarray(qx)[miss][:3].tolist()}")
                self.exact += int(idx.size)
                self.exact_fp32 += int((got[idx] != exp[idx]).sum())
        return excused

    @property
    def frac(self) -> float:
        return self.excused / max(1, self.greedy)

    def finish(self) -> float:
        line = (f"[near-tie] {self.name}: {self.excused} of {self.greedy} greedy choices excused "
                f"({100 * self.frac:.3f} %, bound {'-' if self.max_frac is None else f'{100 * self.max_frac:.2f} %'})")
        if self.exact:
            line += (f"; oracle MFMA rule: {self.exact} greedy choices checked, all equal its argmax "
                     f"({self.exact_fp32} of them differ from the fp32 emulation's)")
        print(line)
        SUMMARY.append(line)
        if self.max_frac is not None:
            assert self.frac <= self.max_frac, (self.name, self.excused, self.greedy)
        return self.frac


def order_matched_q(qnet, sd, x, form, torch=None):
    """The Q-values the kernels compute, restated on the CPU: the oracle's model of the matrix cores'
    accumulation (oracle.merge_oracle.qnet_reference_mfma, rule "mfma") in the kernel's packed k order,
    form "16x16" (net opponents, h-DQN) or "32x32" (config 5 without a net opponent). Round 6: no
    longer the device's own mg_qnet_forward for the 16x16 form -- the kernel is never its own reference.
    `qnet` is unused (kept for the call sites' signature)."""
    import merge_oracle as mo

    return mo.qnet_reference_mfma(sd, x, form=form).astype(np.float64)


def exact_q(sd, x, swap=False, form="16x16"):
    """Lazy oracle-rule Q rows for ChoiceCheck.check(q_exact=...): idx -> qnet_reference_mfma of x[idx]."""
    import merge_oracle as mo

    x = np.asarray(x, np.float32)
    return lambda idx: mo.qnet_reference_mfma(sd, x[idx], swap=swap, form=form)


def check_q_eval(dev, exp, abs_sum, what="", pinned=None, model=None):
    """The q_eval sums a fused policy kernel keeps (mg_episode_stats.q_eval: the Q value the scripts
    log per finished episode, main.py:221 / hdqn.py:330) against the bf16-emulated reference's, env
    by env, with the Q-net forward's own bound (tests/test_gpu_qnet.py) on a per-env sum: relative
    error (to max(1, abs_sum), abs_sum being the env's sum over its logged episodes of max_a |q| of the
    logged row) with a median below 1e-5. An env above 1e-3 -- a hidden unit whose fp32 sum lands on a
    bf16 rounding boundary rounds the other way in the emulation's summation order and moves that
    episode's q by up to ~1 % -- must be reproduced BIT FOR BIT by `pinned`, the same per-env sum of
    order-matched Q-values (order_matched_q: the kernel's own forward order); any env it does not
    reproduce fails the check. `model` (optional): the same sums from the oracle's CPU model of the
    kernel's summation order (oracle.merge_oracle.qnet_reference_mfma), which must reproduce every
    flagged env bit for bit too. Without `pinned`, every env must stay within 1e-2 (round 4's bound
    before r04d; no widening). Round 6: `pinned` is the oracle's MFMA-rule sums (order_matched_q), and
    EVERY logged env must equal them bit for bit."""
    import numpy as np

    dev, exp, abs_sum = (np.asarray(a, np.float64) for a in (dev, exp, abs_sum))
    logged = abs_sum > 0
    assert logged.sum() > 0, f"{what}: no episode ended"
    assert (dev[~logged] == exp[~logged]).all(), f"{what}: q_eval changed without a finished episode"
    err = np.abs(dev - exp) / np.maximum(1.0, abs_sum)
    flagged = logged & (err > 1e-3)
    assert np.median(err[logged]) < 1e-5, (what, float(np.median(err[logged])))
    if pinned is not None:
        pinned = np.asarray(pinned, np.float64)
        bad = flagged & (dev != pinned)
        assert not bad.any(), (what, "unexplained q_eval", np.flatnonzero(bad)[:8].tolist(), dev[bad][:4].tolist(),
                               pinned[bad][:4].tolist(), exp[bad][:4].tolist())
        same = dev[logged] == pinned[logged]
        assert same.all(), (what, "q_eval differs from the oracle MFMA rule's sums", int((~same).sum()),
                            np.flatnonzero(logged)[~same][:8].tolist())
    else:
        assert err[logged].max() < 1e-2, (what, float(err[logged].max()))
    if model is not None:
        model = np.asarray(model, np.float64)
        bad = flagged & (dev != model)
        assert not bad.any(), (what, "flagged q_eval not reproduced by the oracle's MFMA model",
                               np.flatnonzero(bad)[:8].tolist())
    SUMMARY.append(f"[q_eval] {what}: {int(logged.sum())} envs with logged episodes, median rel err "
                   f"{float(np.median(err[logged])):.2e}, max {float(err[logged].max()):.2e}; "
                   f"{int(flagged.sum())} above 1e-3, "
                   + ("every logged env bit for bit equal to the oracle MFMA rule's sums"
                      + (f" ({100 * float((dev[logged] == pinned[logged]).mean()):.2f} % of all envs bit-equal)")
                      if pinned is not None else "no order-matched pin")
                   + (f"; oracle MFMA model: flagged ones bit-equal, {100 * float((dev[logged] == model[logged]).mean()):.2f} "
                      "% of all envs" if model is not None else ""))

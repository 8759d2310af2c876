"""Greedy choices of the fused bf16 kernels against the bf16-emulated reference nets
(oracle.qnet_reference: bf16 operands, fp32 sums), with the near-tie excusal bounded.

The kernels and the CPU emulation sum in different orders; a sum that lands on the other side of
a bf16 rounding boundary moves one hidden unit by 2^-8 of itself, and that can reorder two
actions whose Q-values are that close. So a greedy choice that differs from the emulation's
argmax is excused only when the action the kernel took has an emulated Q within `tol` (relative
to max(1, |Q_max|)) of the row's maximum -- never any other action -- and every check counts
the excused choices; `finish()` prints the fraction and asserts it is below the test's bound.
Random (exploring) choices are exact: they come from the Philox draws alone.
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

    def check(self, got, exp, greedy, q, what=""):
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
        return excused

    @property
    def frac(self) -> float:
        return self.excused / max(1, self.greedy)

    def finish(self) -> float:
        line = (f"[near-tie] {self.name}: {self.excused} of {self.greedy} greedy choices excused "
                f"({100 * self.frac:.3f} %, bound {'-' if self.max_frac is None else f'{100 * self.max_frac:.2f} %'})")
        print(line)
        SUMMARY.append(line)
        if self.max_frac is not None:
            assert self.frac <= self.max_frac, (self.name, self.excused, self.greedy)
        return self.frac

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "merging-gym_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "reference_golden.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    return np.load(GOLDEN)


@pytest.fixture(scope="session")
def coracle():
    import merge_oracle

    merge_oracle.build_c_oracle()
    return merge_oracle.COracle()


def pytest_report_header(config):
    """The library under test and the compiler that built it (the Q-net forward's permlane
    hazard padding is written for hipcc 7.2's code generation)."""
    try:
        from merging_gym import _native

        return [f"libmerging_hip: {_native.LIB_PATH}", f"built with: {_native.build_info()}"]
    except Exception as e:  # noqa: BLE001 - the header must not break collection
        return [f"libmerging_hip: not loadable ({e})"]


def _gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment (run with -m gpu on an MI355X)")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def pytest_terminal_summary(terminalreporter):
    """The near-tie excusals of the Q-net / h-DQN greedy checks (tests/choice_check.py), one line
    per check, printed whether or not output was captured."""
    try:
        from choice_check import SUMMARY
    except ImportError:
        return
    if SUMMARY:
        terminalreporter.section("near-tie excusals (bf16 kernel vs bf16-emulated reference)")
        excused = greedy = 0
        for line in SUMMARY:
            terminalreporter.write_line(line)
        import re

        for line in SUMMARY:
            m = re.search(r": (\d+) of (\d+) greedy", line)
            if m:
                excused += int(m.group(1))
                greedy += int(m.group(2))
        terminalreporter.write_line(f"[near-tie] total: {excused} of {greedy} greedy choices excused")

"""Copy two of the reference's DQN checkpoints (test_params/dqn/*/eval.pth) into a numpy fixture.

Test infrastructure: runs only where /root/reference exists. Loaded with
torch.load(weights_only=True) (no unpickling of code); the weights are data (fp32 tensors of the
reference's Net 10 -> 200 -> 100 -> 5, scripts/main.py:30-47).
"""
import os

import numpy as np
import torch

REF = "/root/reference/test_params/dqn"
RUNS = {  # fixture key -> checkpoint directory
    "l1": "2022--03--31 03:37:35normal dqn with OP:L0(2.0, 1.0, -10, 0.001)",  # human_player.py:68
    "l3": "2022--03--31 21:33:10normal dqn with OP:L2(2.0, 1.0, -10, 0.001)",  # largest weights
}
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dqn_checkpoints.npz")


def main():
    arrays = {}
    for key, run in RUNS.items():
        sd = torch.load(os.path.join(REF, run, "eval.pth"), weights_only=True, map_location="cpu")
        for name, t in sd.items():
            arrays[f"{key}/{name}"] = t.numpy().astype(np.float32)
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT} ({os.path.getsize(OUT) / 1e3:.0f} kB)")


if __name__ == "__main__":
    main()

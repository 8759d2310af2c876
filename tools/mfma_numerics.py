"""The bf16 MFMAs' accumulation rule, measured.

    python tools/mfma_numerics.py collect [--cases N] [--out gpurun_out/mfma_numerics.npz]   (GPU)
    python tools/mfma_numerics.py fit [--npz ...]                                            (CPU)

collect: crafted operand sets (seeded, regenerated bit for bit by `fit`, so only D travels back), one
v_mfma_f32_16x16x32_bf16 / v_mfma_f32_32x32x16_bf16 per case (tools/micro/mfma_numerics.hip).
fit: the measured rule (oracle/merge_oracle.c oracle_mfma_dots) and two simpler models
(tools/micro/mfma_model.c) against every recorded output; prints the share of bit-equal outputs per data
set and family. The rule was found with mfma_model.c's parametrised steps (group size, alignment grid,
truncation toward zero or floor, where C enters, the final grid) on these three data sets.
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MICRO = os.path.join(ROOT, "tools", "micro")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from mfma_probe_cases import (FAMILIES, FAMILIES2, SHAPES, bf16_to_f32, dots, make_case, make_case2,  # noqa: E402
                              struct_rows, to_bf16)
def build_probe():
    so = os.path.join(MICRO, "libmfma_numerics.so")
    src = os.path.join(MICRO, "mfma_numerics.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so, src])
    return so


def build_model():
    so = os.path.join(MICRO, "libmfma_model.so")
    src = os.path.join(MICRO, "mfma_model.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", so, src])
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p
    lib.mfma_model.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, P]
    return lib


def inputs_digest(form, n, maker=None):
    h = hashlib.sha256()
    for i in range(0, n, max(1, n // 16)):
        A, B, C, _ = (maker or make_case)(form, i)
        h.update(A.tobytes() + B.tobytes() + C.tobytes())
    return h.hexdigest()[:16]


def collect(args, maker=None, prefix="D"):
    import torch

    maker = maker or make_case

    lib = ctypes.CDLL(build_probe())
    lib.mfma_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int]
    out = {}
    for form in (16, 32):
        M, N, K = SHAPES[form]
        cases = [maker(form, i) for i in range(args.cases)]
        A = torch.from_numpy(np.stack([c[0] for c in cases]).view(np.int16)).cuda()
        B = torch.from_numpy(np.stack([c[1] for c in cases]).view(np.int16)).cuda()
        C = torch.from_numpy(np.stack([c[2] for c in cases])).cuda()
        D = torch.empty_like(C)
        rc = lib.mfma_probe(form, A.data_ptr(), B.data_ptr(), C.data_ptr(), D.data_ptr(), args.cases)
        assert rc == 0, rc
        out[f"{prefix}{form}"] = D.cpu().numpy()
        out[f"digest{form}"] = np.array(inputs_digest(form, args.cases, maker))
        print(f"form {form}: {args.cases} cases collected", flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    np.savez(args.out, **out)
    print("wrote", args.out)


def run_model(lib, a, b, c, order, G, F, mode, c_last):
    out = np.empty(len(c), np.float32)
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    c = np.ascontiguousarray(c, np.float32)
    o = np.ascontiguousarray(order, np.int32)
    lib.mfma_model(len(c), a.shape[1], a.ctypes.data, b.ctypes.data, c.ctypes.data, o.ctypes.data, G, F, mode,
                   c_last, out.ctypes.data)
    return out


def fit(args):
    """Share of bit-equal outputs per data set and family: the measured rule (the oracle's
    oracle_mfma_dots) against round 5's model (each group's exact sum rounded once into the
    accumulator) and an exact per-MFMA sum rounded once (tools/micro/mfma_model.c)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import merge_oracle as mo

    lib = build_model()
    lib.mfma_model_two.argtypes = [ctypes.c_int] * 5
    lib.mfma_model_two(0, 0, 0, 0, 0)
    g = os.path.dirname(os.path.abspath(args.npz))
    sets = []
    for form in (16, 32):
        K = SHAPES[form][2]
        d = np.load(os.path.join(g, "..", "r06a", "mfma_numerics.npz"))
        n = d[f"D{form}"].shape[0]
        a, b, c, fam = dots(form, n)
        sets.append((f"random form {form}", K, a, b, c, fam, d[f"D{form}"].reshape(-1)))
        d = np.load(os.path.join(g, "..", "r06c", "mfma_single.npz"))
        n = d[f"E{form}"].shape[0]
        a, b, c, fam = dots(form, n, make_case2)
        sets.append((f"one-step form {form}", K, a, b, c, fam, d[f"E{form}"].reshape(-1)))
        d = np.load(os.path.join(g, "..", "r06b", "mfma_struct.npz"))
        rows, labels = struct_rows(form)
        a = to_bf16(np.stack([r[0] for r in rows]))
        b = np.full_like(a, to_bf16(np.float32(1.0)))
        c = np.array([r[1] for r in rows], np.float32)
        sets.append((f"structured form {form}", K, a, b, c, np.array([lab[0] for lab in labels]), d[f"S{form}"]))
    total = 0
    for name, K, a, b, c, fam, dev in sets:
        models = {"measured rule": mo.mfma_dots(a, b, c),
                  "round-5 exact-8": run_model(lib, a, b, c, np.arange(K), 8, -1, 0, 0),
                  "exact per MFMA": run_model(lib, a, b, c, np.arange(K), K, -1, 0, 0)}
        print(f"{name}: {len(dev)} outputs")
        total += len(dev)
        for mname, m in models.items():
            eq = (m.view(np.uint32) == dev.view(np.uint32)) | ((m == 0) & (dev == 0))
            fams = " ".join(f"{f}={eq[fam == f].mean():.4f}" for f in np.unique(fam))
            print(f"  {mname:16s} {eq.mean():.6f} ({int(eq.sum())})  {fams}")
    print(f"total outputs {total}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("collect", "fit", "struct", "single"))
    ap.add_argument("--cases", type=int, default=None)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "mfma_numerics.npz"))
    ap.add_argument("--npz", default=os.path.join(ROOT, "gpurun_out", "mfma_numerics.npz"))
    ap.add_argument("--top", type=int, default=12)
    args = ap.parse_args()
    if args.mode == "struct":
        collect_struct(args)
    elif args.mode == "single":
        args.cases = args.cases or 1024
        collect(args, make_case2, "E")
    elif args.mode == "collect":
        args.cases = args.cases or 2048
        collect(args)
    else:
        fit(args)



# ---- structured probes: one dot product per A row, B = ones, C per row ----------------------------------

def struct_cases(form: int):
    """The struct rows packed M per case: A [n][M][K] bf16, B ones, C [n][M][N] (row value in every column)."""
    M, N, K = SHAPES[form]
    rows, labels = struct_rows(form)
    n = (len(rows) + M - 1) // M
    A = np.zeros((n * M, K), np.float32)
    C = np.zeros((n * M,), np.float32)
    for r, (a, c) in enumerate(rows):
        A[r], C[r] = a, c
    A = to_bf16(A.reshape(n, M, K))
    assert np.array_equal(bf16_to_f32(A).reshape(-1, K)[:len(rows)], np.stack([r[0] for r in rows]))
    B = np.full((n, K, N), to_bf16(np.float32(1.0)), np.uint16)
    Cm = np.repeat(C.reshape(n, M, 1), N, 2)
    return A, B, Cm, labels


def collect_struct(args):
    import torch

    lib = ctypes.CDLL(build_probe())
    lib.mfma_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int]
    out = {}
    for form in (16, 32):
        A, B, C, labels = struct_cases(form)
        n = A.shape[0]
        At = torch.from_numpy(A.view(np.int16)).cuda()
        Bt = torch.from_numpy(B.view(np.int16)).cuda()
        Ct = torch.from_numpy(np.ascontiguousarray(C)).cuda()
        D = torch.empty_like(Ct)
        rc = lib.mfma_probe(form, At.data_ptr(), Bt.data_ptr(), Ct.data_ptr(), D.data_ptr(), n)
        assert rc == 0, rc
        Dn = D.cpu().numpy()
        # every column computes the same row: keep column 0, and check the columns agree
        assert (Dn == Dn[:, :, :1]).all(), "columns differ"
        out[f"S{form}"] = Dn[:, :, 0].reshape(-1)[:len(labels)]
        print(f"form {form}: {len(labels)} struct rows", flush=True)
    np.savez(args.out, **out)
    print("wrote", args.out)


if __name__ == "__main__":
    sys.exit(main())

"""Static instruction mix of kernels in a gfx950 assembly file (hipcc --cuda-device-only -S).

    python tools/isa_mix.py build.s rollout_kernel [qnet_rollout_ws_kernel ...]

Counts every instruction between a kernel's label and its s_endpgm (cold paths included),
grouped as fp64 VALU, other VALU, MFMA, LDS, SALU, memory and branches.
"""
import collections
import re
import sys


def kernel_body(text, name):
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", text, re.M)
    if not m:
        raise SystemExit(f"{name} not found")
    i = m.end()
    j = text.index("s_endpgm", i)
    return m.group(1), text[i:j]


def mix(body):
    ins = [ln.split()[0] for ln in body.split("\n")
           if ln.startswith("\t") and ln.strip() and not ln.strip().startswith((".", ";"))]
    c = collections.Counter(ins)
    groups = collections.Counter()
    for k, v in c.items():
        if k.startswith("v_mfma"):
            g = "mfma"
        elif k.startswith("v_") and "f64" in k:
            g = "valu_f64"
        elif k.startswith("v_"):
            g = "valu_other"
        elif k.startswith("ds_"):
            g = "lds"
        elif k.startswith(("global_", "buffer_", "flat_", "scratch_")):
            g = "vmem"
        elif k.startswith("s_cbranch") or k.startswith("s_branch"):
            g = "branch"
        elif k.startswith("s_"):
            g = "salu"
        else:
            g = "other"
        groups[g] += v
    return c, groups


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    for name in sys.argv[2:]:
        sym, body = kernel_body(text, name)
        c, g = mix(body)
        print(sym, sum(c.values()), dict(g))
        print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(40)))

"""Generate golden vectors by running the reference's own MergeEnv (read-only, from /root/reference).

Test infrastructure only: run here, in the build container, never on the GPU box. The
reference's source is imported from /root/reference at run time and is never copied; only
the inputs and outputs it produces are committed (tests/golden/*.npz).

The reference's third-party dependencies are absent from this image (gym 0.20.0, pygame
2.1.2, shapely 1.8.1, qpsolvers 1.8.0 / quadprog 0.1.11, cv2; pinned in
reference requirements.txt:2-14). They are replaced by the small stand-ins written below
into a temporary directory. Everything the reference computes itself runs for real:
MergeEnv.step/reset/observe/is_collided/corners (merging_gym/envs/merging_env.py:118-239),
lon2coord (:48-58) and mpc_1d's matrix build (scripts/helper.py:152-191). The stand-ins
restate the arithmetic at three third-party boundaries, so parity there is pinned only by
these restatements (see DESIGN.md "Oracle"):

  * qpsolvers.solve_qp -> quadprog's qpgen2 (the Goldfarb-Idnani dual method as coded in
    Turlach's solve.QP.f: LINPACK dpofa / dposl / dpori, the vsmall precision probe, the sign
    flip of an equality, the full step along z = J J'n), restated statement by statement on the
    arrays the reference builds (until round 2: a KKT numpy.linalg.solve, an ulp away);
  * pygame Rect(center=...) -> C (int) truncation of the float centre, x = cx - w//2
    (pygame 2.1.2 pg_IntFromObj + pg_rect_setcenter); Vector2 +,-,scalar* in fp64 and
    rotate(0) = identity (pygame special-cases multiples of 90 degrees);
  * shapely Polygon.intersects -> closed-box overlap of the two axis-aligned rectangles
    (GEOS is exact on such inputs).

Usage:  python tests/golden/gen_golden.py   (writes tests/golden/reference_golden.npz)
"""

from __future__ import annotations

import contextlib
import io
import os
import sys
import tempfile
import textwrap

import numpy as np

REFERENCE = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_golden.npz")

_SHIMS = {
    "gym/__init__.py": """
        from . import error, spaces, utils
        from .core import Env
        from .envs.registration import make, register
    """,
    "gym/core.py": """
        class Env:
            metadata = {}
            @property
            def unwrapped(self):
                return self
    """,
    "gym/error.py": "",
    "gym/utils/__init__.py": "from . import seeding\n",
    "gym/utils/seeding.py": "",
    "gym/spaces.py": """
        import numpy as np
        class Box:
            def __init__(self, low, high, dtype=np.float32, shape=None):
                self.low = np.asarray(low, dtype=dtype)
                self.high = np.asarray(high, dtype=dtype)
                self.shape = self.low.shape
                self.dtype = np.dtype(dtype)
        class Discrete:
            def __init__(self, n):
                self.n = int(n)
                self.shape = ()
            def sample(self):
                return int(np.random.randint(self.n))
    """,
    "gym/envs/__init__.py": "",
    "gym/envs/registration.py": """
        import importlib
        _registry = {}
        def register(id, entry_point, **kw):
            _registry[id] = entry_point
        def make(id, **kw):
            mod, attr = _registry[id].split(':')
            return getattr(importlib.import_module(mod), attr)()
    """,
    "cv2.py": "def destroyAllWindows():\n    pass\n",
    "pygame/__init__.py": """
        from . import display, font, surfarray, math, draw, time, locals
        from ._surface import Surface, Rect
        def init():
            return (0, 0)
    """,
    "pygame/_surface.py": """
        def _c_int(v):
            # pygame 2.1.2 pg_IntFromObj: a float goes through a C (int) cast (truncation).
            return int(v) if isinstance(v, float) else int(v)
        class Rect:
            def __init__(self, x, y, w, h):
                self.x, self.y, self.w, self.h = int(x), int(y), int(w), int(h)
            @property
            def center(self):
                return (self.x + self.w // 2, self.y + self.h // 2)
            @center.setter
            def center(self, v):
                cx, cy = _c_int(v[0]), _c_int(v[1])
                self.x = cx - self.w // 2   # C integer division, w, h > 0
                self.y = cy - self.h // 2
            @property
            def topleft(self):
                return (self.x, self.y)
            @property
            def topright(self):
                return (self.x + self.w, self.y)
            @property
            def bottomright(self):
                return (self.x + self.w, self.y + self.h)
            @property
            def bottomleft(self):
                return (self.x, self.y + self.h)
        class Surface:
            def __init__(self, size, *a, **k):
                self._w, self._h = int(size[0]), int(size[1])
            def fill(self, *a, **k):
                pass
            def blit(self, *a, **k):
                pass
            def get_rect(self, **kw):
                r = Rect(0, 0, self._w, self._h)
                for key, val in kw.items():
                    setattr(r, key, val)
                return r
    """,
    "pygame/display.py": """
        from ._surface import Surface
        def set_mode(size, *a, **k):
            return Surface(size)
        def set_caption(*a, **k):
            pass
        def update(*a, **k):
            pass
    """,
    "pygame/font.py": """
        class Font:
            def __init__(self, *a, **k):
                pass
            def render(self, *a, **k):
                return None
        def SysFont(*a, **k):
            return Font()
    """,
    "pygame/surfarray.py": """
        from ._surface import Surface
        def make_surface(arr):
            return Surface(arr.shape[:2])
    """,
    "pygame/math.py": """
        class Vector2:
            def __init__(self, x, y=None):
                if y is None:
                    x, y = x
                self.x, self.y = float(x), float(y)
            def __sub__(self, o):
                return Vector2(self.x - o.x, self.y - o.y)
            def __add__(self, o):
                return Vector2(self.x + o.x, self.y + o.y)
            def __mul__(self, s):
                return Vector2(s * self.x, s * self.y)
            __rmul__ = __mul__
            def rotate(self, angle):
                if float(angle) % 360.0 != 0.0:
                    raise NotImplementedError('stand-in only rotates by multiples of 360')
                return Vector2(self.x, self.y)
    """,
    "pygame/draw.py": "def circle(*a, **k):\n    pass\ndef polygon(*a, **k):\n    pass\ndef lines(*a, **k):\n    pass\n",
    "pygame/time.py": "def wait(*a, **k):\n    pass\n",
    "pygame/locals.py": "",
    "shapely/__init__.py": "",
    "shapely/geometry.py": """
        class Polygon:
            def __init__(self, pts):
                self.pts = [(float(x), float(y)) for x, y in pts]
                xs = [p[0] for p in self.pts]
                ys = [p[1] for p in self.pts]
                # every edge axis-aligned: the stand-in only handles rectangles
                for (ax, ay), (bx, by) in zip(self.pts, self.pts[1:] + self.pts[:1]):
                    assert ax == bx or ay == by, self.pts
                self.bounds = (min(xs), min(ys), max(xs), max(ys))
            def intersects(self, other):
                a, b = self.bounds, other.bounds
                return a[0] <= b[2] and b[0] <= a[2] and a[1] <= b[3] and b[1] <= a[3]
        def box(minx, miny, maxx, maxy):
            return Polygon([(minx, miny), (maxx, miny), (maxx, maxy), (minx, maxy)])
    """,
    "tensorboardX.py": """
        class SummaryWriter:  # hdqn.py:12 imports it; the golden runs never log
            def __init__(self, *a, **k):
                pass
            def add_scalar(self, *a, **k):
                pass
    """,
    "qpsolvers.py": """
        import math
        import numpy as np
        def solve_qp(P, q, G=None, h=None, A=None, b=None, **kw):
            # qpsolvers 1.8.0 -> quadprog 0.1.11 for the one form helper.mpc_1d uses (one equality,
            # no inequality): quadprog.solve_qp(G=P, a=-q, C=-A', b=-b, meq=1), i.e. qpgen2's
            # dual active-set method (Goldfarb & Idnani; Turlach's solve.QP.f with LINPACK dpofa /
            # dposl / dpori), restated statement by statement on the reference's own arrays.
            A = np.atleast_2d(np.asarray(A, dtype=float))
            assert A.shape[0] == 1 and G is None and h is None, 'stand-in: one equality only'
            n = P.shape[0]
            d = [[float(P[i][j]) for j in range(n)] for i in range(n)]   # d[i][j] = dmat(i+1, j+1)
            dvec = [-float(x) for x in np.asarray(q, dtype=float)]       # a = -q (-0.0 for q = 0)
            amat = [-float(x) for x in A[0]]                              # C = -A'
            bvec = -float(np.atleast_1d(np.asarray(b, dtype=float))[0])   # b_c = -b
            vsmall = 1e-60
            while True:                                                   # qpgen2's precision probe
                vsmall = vsmall + vsmall
                if vsmall * 0.1 + 1.0 > 1.0 and vsmall * 0.2 + 1.0 > 1.0:
                    break
            for j in range(n):                                            # dpofa
                s = 0.0
                for k in range(j):
                    dot = 0.0
                    for l in range(k):
                        dot = dot + d[l][k] * d[l][j]
                    t = (d[k][j] - dot) / d[k][k]
                    d[k][j] = t
                    s = s + t * t
                s = d[j][j] - s
                assert s > 0.0, 'matrix not positive definite'
                d[j][j] = math.sqrt(s)
            for k in range(n):                                            # dposl: R'y = a ...
                dot = 0.0
                for l in range(k):
                    dot = dot + d[l][k] * dvec[l]
                dvec[k] = (dvec[k] - dot) / d[k][k]
            for k in reversed(range(n)):                                  # ... then R x = y
                dvec[k] = dvec[k] / d[k][k]
                t = -dvec[k]
                if t != 0.0:
                    for l in range(k):
                        dvec[l] = dvec[l] + t * d[l][k]
            for k in range(n):                                            # dpori: J = R^-1
                d[k][k] = 1.0 / d[k][k]
                t = -d[k][k]
                for l in range(k):
                    d[l][k] = t * d[l][k]
                for j in range(k + 1, n):
                    t = d[k][j]
                    d[k][j] = 0.0
                    if t != 0.0:
                        for l in range(k + 1):
                            d[l][j] = d[l][j] + t * d[l][k]
            for j in range(n):                                            # lower triangle := 0
                for i in range(j + 1, n):
                    d[i][j] = 0.0
            sol = list(dvec)
            sv = -bvec                                                    # the residual at sol
            for j in range(n):
                sv = sv + amat[j] * sol[j]
            if abs(sv) < vsmall:
                sv = 0.0
            if sv > 0.0:                                                  # equality: flip its sign
                amat = [-x for x in amat]
                bvec = -bvec
            sv = -abs(sv)
            if not (sv < 0.0):                                            # nothing violated
                return np.asarray(sol)
            dd = []
            for i in range(n):                                            # d = J'n+
                s = 0.0
                for j in range(n):
                    s = s + d[j][i] * amat[j]
                dd.append(s)
            z = [0.0] * n                                                 # z = J d
            for j in range(n):
                for i in range(n):
                    z[i] = z[i] + d[i][j] * dd[j]
            ztn = 0.0
            for i in range(n):
                ztn = ztn + z[i] * amat[i]
            tt = -sv / ztn                                                # the full step
            return np.asarray([sol[i] + tt * z[i] for i in range(n)])
    """,
}


def _write_shims(root: str) -> None:
    for rel, src in _SHIMS.items():
        path = os.path.join(root, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(textwrap.dedent(src))


def load_reference_env():
    """Import the reference MergeEnv via gym.make('merging_env-v0') with the stand-ins."""
    if not os.path.isdir(REFERENCE):
        raise SystemExit(f"{REFERENCE} not found: golden vectors are generated only in the build container")
    shim_dir = tempfile.mkdtemp(prefix="mg_shims_")
    _write_shims(shim_dir)
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    sys.path[:0] = [shim_dir, os.path.join(REFERENCE, "scripts"), REFERENCE]
    with contextlib.redirect_stdout(io.StringIO()):
        import gym  # the stand-in
        import merging_gym  # noqa: F401  (the reference package: registers merging_env-v0)

        env = gym.make("merging_env-v0").unwrapped
    return env


# --------------------------------------------------------------------------- recording

# type bits per step record: which returned values are Python ints (not floats)
T_R1_INT, T_R2_INT, T_OBS3_INT, T_OBS8_INT, T_OBS4_INT, T_OBS9_INT = 1, 2, 4, 8, 16, 32


def _types(obs, rew) -> int:
    t = 0
    t |= T_R1_INT if isinstance(rew[0], int) else 0
    t |= T_R2_INT if isinstance(rew[1], int) else 0
    t |= T_OBS3_INT if isinstance(obs[3], int) else 0
    t |= T_OBS8_INT if isinstance(obs[8], int) else 0
    t |= T_OBS4_INT if isinstance(obs[4], int) else 0
    t |= T_OBS9_INT if isinstance(obs[9], int) else 0
    return t


def _winner_code(w) -> int:
    return 0 if w is None else int(w)


class Recorder:
    """Per-step columns: action inputs, returned values, and the env state after the step."""

    def __init__(self):
        self.cols = {k: [] for k in (
            "a1", "a2", "obs", "rew", "done", "coll", "winner", "pos", "vel", "acc",
            "time", "racc", "types", "reset")}

    def add(self, env, a1, a2, obs, rew, done, info, was_reset):
        c = self.cols
        c["a1"].append(a1)
        c["a2"].append(-1 if a2 is None else a2)
        c["obs"].append([float(x) for x in obs])
        c["rew"].append([float(x) for x in rew])
        c["done"].append(bool(done))
        c["coll"].append(bool(info["collision"]) if info is not None else False)
        c["winner"].append(_winner_code(env.winner))
        c["pos"].append([float(env.state1["pos"]), float(env.state2["pos"])])
        c["vel"].append([float(env.state1["vel"]), float(env.state2["vel"])])
        c["acc"].append([float(env.state1["acc"]), float(env.state2["acc"])])
        c["time"].append(float(env.time_stamp))
        c["racc"].append([float(env.r1_accumulate), float(env.r2_accumulate)])
        c["types"].append(_types(obs, rew))
        c["reset"].append(bool(was_reset))

    def arrays(self, prefix):
        dt = {"a1": np.int8, "a2": np.int8, "done": np.bool_, "coll": np.bool_, "winner": np.int8,
              "types": np.uint8, "reset": np.bool_}
        return {f"{prefix}_{k}": np.asarray(v, dtype=dt.get(k, np.float64)) for k, v in self.cols.items()}


def run_trace(env, actions1, actions2, reset_on_done: bool, max_steps: int, rec: Recorder):
    """Step with the given action sequences. A row with reset=True is the reset() return
    (actions -1, rew 0); then one row per step()."""
    with contextlib.redirect_stdout(io.StringIO()):
        obs = env.reset()
    rec.add(env, -1, -1, obs, [0.0, 0.0], False, None, True)
    for k in range(max_steps):
        a1, a2 = actions1[k], actions2[k]
        with contextlib.redirect_stdout(io.StringIO()):
            obs, rew, done, info = env.step(int(a1), None if a2 is None or a2 < 0 else int(a2))
        rec.add(env, int(a1), a2, obs, rew, done, info, False)
        if done and reset_on_done:
            with contextlib.redirect_stdout(io.StringIO()):
                obs = env.reset()
            rec.add(env, -1, -1, obs, [0.0, 0.0], False, None, True)


KATS = {  # name: (a1, a2 or None, max steps); SURVEY.md section 8(a) known-answer table
    "A": (2, None), "B": (0, None), "C": (4, None), "D": (4, 0), "E": (0, 4), "F": (3, 3), "G": (1, 1),
}


def main():
    env = load_reference_env()
    out = {}

    # (i) known-answer trajectories, run to done (or the 2501-step timeout)
    for name, (a1, a2) in KATS.items():
        rec = Recorder()
        n = 2600
        run_trace(env, [a1] * n, [a2] * n, reset_on_done=False, max_steps=n, rec=rec)
        d = rec.arrays(f"kat{name}")
        first_done = int(np.argmax(d[f"kat{name}_done"]))
        keep = first_done + 1  # the reset row is index 0, so rows [0, first_done] inclusive
        out.update({k: v[: keep + 0] for k, v in d.items()})

    # (ii) random episodes: uniform actions, opponent None or uniform, reset on done
    rng = np.random.default_rng(20240601)
    for tag, opp_random in (("rndL0", False), ("rndRR", True)):
        rec = Recorder()
        steps = 3000
        a1 = rng.integers(0, 5, steps)
        a2 = rng.integers(0, 5, steps) if opp_random else np.full(steps, -1)
        run_trace(env, list(a1), [int(x) for x in a2], reset_on_done=True, max_steps=steps, rec=rec)
        out.update(rec.arrays(tag))

    # (ii-b) stepping past done without reset (reaches the x ~ 0 region, pos 990..1010)
    rec = Recorder()
    steps = 1200
    for ep in range(3):
        a1 = rng.integers(0, 5, steps)
        a2 = rng.integers(0, 5, steps)
        run_trace(env, list(a1), [int(x) for x in a2], reset_on_done=False, max_steps=steps, rec=rec)
    out.update(rec.arrays("past"))

    # (iii) one-step rows from random states near the collision boundary and the end point
    n_rows = 8000
    ts = [0.0]
    t = 0.0
    for _ in range(2700):
        t += 0.2
        ts.append(t)
    rows = {k: [] for k in ("p", "v", "winner", "done", "k", "racc", "a1", "a2",
                            "obs", "rew", "done_out", "coll", "winner_out", "pos", "vel", "time",
                            "racc_out", "types")}
    for r in range(n_rows):
        mode = r % 4
        if mode == 0:    # anywhere on the road
            p1 = rng.uniform(0.0, 1100.0)
            p2 = p1 + rng.uniform(-12.0, 12.0)
        elif mode == 1:  # around the merge point / x ~ 0 region
            p1 = rng.uniform(980.0, 1020.0)
            p2 = p1 + rng.uniform(-12.0, 12.0)
        elif mode == 2:  # lattice: positions on a 1/8 grid so truncations land on boundaries
            p1 = np.round(rng.uniform(600.0, 1050.0) * 8) / 8
            p2 = p1 + np.round(rng.uniform(-10.0, 10.0) * 8) / 8
        else:            # arrival thresholds
            p1 = 950.0 + rng.choice([-0.2, -1e-9, 0.0, 1e-9, 0.2]) + rng.uniform(-1, 1) * (r % 3 == 0)
            p2 = 950.0 + rng.choice([-0.2, -1e-9, 0.0, 1e-9, 0.2])
        v1, v2 = rng.uniform(0.0, 45.0, 2)
        if r % 17 == 0:
            v1 = 0.0
        w = int(rng.integers(0, 3))
        d0 = bool(rng.random() < 0.1)
        k = int(rng.choice([rng.integers(0, 2499), 2499, 2500, 2501, 2600]))
        racc = rng.uniform(-20, 5, 2)
        a1 = int(rng.integers(0, 5))
        a2 = int(rng.integers(-1, 5))
        with contextlib.redirect_stdout(io.StringIO()):
            env.reset()
        env.state1 = {"pos": float(p1), "vel": float(v1), "acc": 0.0}
        env.state2 = {"pos": float(p2), "vel": float(v2), "acc": 0.0}
        env.winner = None if w == 0 else w
        env.done = d0
        env.time_stamp = ts[k]
        env.r1_accumulate, env.r2_accumulate = float(racc[0]), float(racc[1])
        with contextlib.redirect_stdout(io.StringIO()):
            obs, rew, done, info = env.step(a1, None if a2 < 0 else a2)
        for key, val in (("p", [p1, p2]), ("v", [v1, v2]), ("winner", w), ("done", d0), ("k", k),
                         ("racc", list(racc)), ("a1", a1), ("a2", a2),
                         ("obs", [float(x) for x in obs]), ("rew", [float(x) for x in rew]),
                         ("done_out", bool(done)), ("coll", bool(info["collision"])),
                         ("winner_out", _winner_code(env.winner)),
                         ("pos", [float(env.state1["pos"]), float(env.state2["pos"])]),
                         ("vel", [float(env.state1["vel"]), float(env.state2["vel"])]),
                         ("time", float(env.time_stamp)),
                         ("racc_out", [float(env.r1_accumulate), float(env.r2_accumulate)]),
                         ("types", _types(obs, rew))):
            rows[key].append(val)
    ints = {"winner": np.int8, "done": np.bool_, "k": np.int32, "a1": np.int8, "a2": np.int8,
            "done_out": np.bool_, "coll": np.bool_, "winner_out": np.int8, "types": np.uint8}
    out.update({f"one_{k}": np.asarray(v, dtype=ints.get(k, np.float64)) for k, v in rows.items()})

    # reset observation and the space definitions
    with contextlib.redirect_stdout(io.StringIO()):
        obs0 = env.reset()
    out["reset_obs"] = np.asarray(obs0, dtype=np.float64)
    out["reset_types"] = np.asarray(_types(obs0, [0.0, 0.0]), dtype=np.uint8)
    out["obs_low"] = np.asarray(env.observation_space.low, dtype=np.float64)
    out["obs_high"] = np.asarray(env.observation_space.high, dtype=np.float64)
    out["obs_dtype"] = np.asarray(str(env.observation_space.dtype))
    out["n_actions"] = np.asarray(env.action_space.n)
    out["show_reward"] = np.asarray(env.show_reward(), dtype=np.float64)

    # mpc_1d first accelerations on a grid (helper.py:152-191, via the solve_qp stand-in)
    import helper  # reference scripts/helper.py (on sys.path)

    v0s = rng.uniform(0.0, 45.0, 400)
    v0s[:5] = [0.0, 10.0, 20.0, 30.0, 40.0]
    vts = rng.integers(0, 5, 400) * 10.0
    x0s = rng.uniform(0.0, 1000.0, 400)
    acc = [helper.mpc_1d(x0, v0, x0 + vt * 3.0, vt, 3.0).action() for x0, v0, vt in zip(x0s, v0s, vts)]
    out["mpc_x0"], out["mpc_v0"], out["mpc_vt"] = x0s, v0s, vts
    out["mpc_acc"] = np.asarray(acc, dtype=np.float64)

    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({os.path.getsize(OUT) / 1e6:.2f} MB, {len(out)} arrays)")


if __name__ == "__main__":
    main()

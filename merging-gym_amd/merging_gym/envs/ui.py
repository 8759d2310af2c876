"""The human-experiment pygame UI (merging_env.py:83-108, :241-395), drawn from env state.

The reference draws inside MergeEnv, from the fp64 state its step just wrote. Here the step
state lives on the GPU, so drawing is split in two:

* `scene(view, ...)` turns one env's state -- positions, speeds, last accelerations and
  accumulated rewards, as read back from the device (MergeEnv's step record or a
  MergeVecEnv row) -- into the list of primitives one `render()` frame draws, with the
  reference's fp64 geometry: lon2coord (:48-58) of the current and the predicted position
  p + v * prediction_t, the four track circles per panel, and the vehicle boxes of corners
  (:232-239) with pygame's Rect semantics (a float centre is truncated to int).
* `MergeUI` issues those primitives, and the intro / prepare / feedback / finish screens,
  through pygame. pygame is imported only when the first UI method runs, so the GPU step
  path never needs it; without pygame the UI methods raise ImportError.

Text values are rounded as the reference's are: its accumulators and speeds are numpy
float64 after a step, and `round(np.float64, 2)` rounds the scaled value (2.675 -> 2.68),
not Python's decimal rounding, so floats go through np.float64 here; ints stay ints.
"""

from __future__ import annotations

import numpy as np

# merging_env.py:22-46
R = 30000
H, W = 1000, 300
WINDOW_H, WINDOW_W = 1000, 300
VEHICLE_W, VEHICLE_H = 4, 8
prediction_t = 3.0
scale = 5.0

CAPTION = "On ramp merging experiment"
INTRO_TEXT = "Please pass the ramp quickly without collision"
BLACK, WHITE, GREY, RED, BLUE = (0, 0, 0), (255, 255, 255), [120, 120, 120], [255, 0, 0], [0, 0, 255]


def lon2coord(lon, ego: bool):
    """Arc position -> (longitudinal x, lateral y), numpy fp64 as merging_env.py:48-58."""
    angle = np.arctan2(H, R) - lon / R
    x = R * np.sin(angle)
    d = R - R * np.cos(angle)
    return x, (W / 2 + d) if ego else (W / 2 - d)


def box_corners(lon, lat, k=1.0):
    """corners(agent, lon, lat, yaw=0, scale=k) for a VEHICLE_W x VEHICLE_H surface: the Rect
    centred at (lat, lon) after pygame's int truncation, each corner scaled about the
    (float) centre: k * (corner - centre) + centre, in fp64."""
    x0 = int(lat) - VEHICLE_W // 2
    y0 = int(lon) - VEHICLE_H // 2
    pts = ((x0, y0), (x0 + VEHICLE_W, y0), (x0 + VEHICLE_W, y0 + VEHICLE_H), (x0, y0 + VEHICLE_H))
    return [(k * (px - lat) + lat, k * (py - lon) + lon) for px, py in pts]


def _num(v):
    """A state value as the reference holds it after a step (see the module docstring)."""
    return v if isinstance(v, (int, np.integer)) else np.float64(v)


def _r2(v):
    return str(round(_num(v), 2))


def _accel_color(goal, acc):
    if goal is not None:
        return RED if goal == 0 else BLUE if goal == 1 else list(BLACK)
    if acc > 1e-2:
        return RED
    if acc < -1e-2:
        return BLUE
    return list(BLACK)


def scene(view, goal=None, goal_op=None, tag_left=None, tag_right=None):
    """One render() frame (merging_env.py:243-334) as primitives, per panel.

    view: dict with pos1, vel1, acc1, pos2, vel2, acc2, r1, r2 (accumulated rewards).
    The left panel is the opponent's view, the right panel the ego's. Returns a list of
    ("circle", panel, color, (cx, cy), radius, width) / ("polygon", panel, color, points, width)
    / ("text", panel, font, string, (x, y)) tuples in the reference's drawing order.
    """
    p1, v1, p2, v2 = view["pos1"], view["vel1"], view["pos2"], view["vel2"]
    x1, y1 = lon2coord(p1, True)
    x2, y2 = lon2coord(p2, False)
    x1t, y1t = lon2coord(p1 + v1 * prediction_t, True)
    x2t, y2t = lon2coord(p2 + v2 * prediction_t, False)
    out = []
    # the two track edges at +-VEHICLE_W around each lane's arc, centred on the panel's car
    for panel, (xc, yc) in (("left", (x2, y2)), ("right", (x1, y1))):
        for rad in (R + VEHICLE_W, R - VEHICLE_W):
            for side in (-R, R):
                centre = (scale * (W / 2 + side - yc) + WINDOW_W / 2, -scale * xc + WINDOW_H / 2)
                out.append(("circle", panel, list(BLACK), centre, scale * rad, 1))
    clr1 = _accel_color(goal, view["acc1"])
    clr2 = _accel_color(goal_op, view["acc2"])
    lon0, lat0 = 3 * WINDOW_H / 5, WINDOW_W / 2  # where a panel's own car is drawn

    def at(dx, dy):  # a car drawn at screen offset (scale * dx, scale * dy) from the panel's
        return box_corners(scale * dx + lon0, scale * dy + lat0, scale)

    # the predicted position's leading edge joined to the car's trailing edge
    out.append(("polygon", "left", GREY, at(x2t - x2, y2t - y2)[:2] + box_corners(lon0, lat0, scale)[2:], 0))
    out.append(("polygon", "right", GREY, at(x1t - x1, y1t - y1)[:2] + box_corners(lon0, lat0, scale)[2:], 0))
    out.append(("polygon", "left", list(BLACK), at(x1 - x2, y1 - y2), 0))
    out.append(("polygon", "right", clr1, box_corners(scale * (x1 - x1) + lon0, y1 - y1 + lat0, scale), 0))
    out.append(("polygon", "left", clr2, at(x2 - x2, y2 - y2), 0))
    out.append(("polygon", "right", list(BLACK), at(x2 - x1, y2 - y1), 0))
    for panel, v, racc, tag, tx in (("left", v2, view["r2"], tag_left, 0.2 * WINDOW_W),
                                    ("right", v1, view["r1"], tag_right, 0.7 * WINDOW_W)):
        out.append(("text", panel, "font", "Spd: " + _r2(v), (tx, 0.6 * WINDOW_H)))
        out.append(("text", panel, "font", "Rwd:" + _r2(racc), (tx, 0.6 * WINDOW_H + 15)))
        if tag:
            out.append(("text", panel, "mark_font", tag, (0.2 * WINDOW_W, 0.1 * WINDOW_H)))
    return out


def _import_pygame():
    try:
        import pygame
    except ImportError as e:  # pragma: no cover - depends on the host
        raise ImportError("the human-experiment UI (render / intro / prepare / feedback / finish) "
                          "draws with pygame, which is not installed; the step path does not "
                          "need it") from e
    return pygame


class MergeUI:
    """The two-panel pygame window of the human experiments (merging_env.py:83-108).

    pygame: the module to draw with (default: `import pygame`). The window, surfaces and fonts
    are created on construction, in the reference's order.
    """

    def __init__(self, pygame=None):
        pg = pygame if pygame is not None else _import_pygame()
        self.pg = pg
        pg.init()
        self.screen = pg.display.set_mode((3 * WINDOW_W, WINDOW_H))
        self.screen.fill(BLACK)
        self.panels = {}
        for name in ("left", "right"):
            s = pg.Surface((WINDOW_W, WINDOW_H))
            s.fill(WHITE)
            self.panels[name] = s
        pg.display.set_caption(CAPTION)
        self.fonts = {"font": pg.font.Font(None, 17), "mark_font": pg.font.SysFont(None, 50)}
        # the vehicle sprites (their size is what corners() uses) and the white background
        self.ego = pg.surfarray.make_surface(np.ones([VEHICLE_W, VEHICLE_H]) * 255)
        self.opponent = pg.surfarray.make_surface(np.ones([VEHICLE_W, VEHICLE_H]) * 255)
        self.image = pg.surfarray.make_surface(np.ones((H, W, 3)).transpose(1, 0, 2) * 255)

    # -------------------------------------------------------------- helpers
    def _clear(self):
        for s in self.panels.values():
            s.blit(self.image, (0, 0))

    def _text(self, panel, font, string, pos):
        self.panels[panel].blit(self.fonts[font].render(string, 2, BLACK), pos)

    def _both(self, left, right, pos):
        self._text("left", "font", left, pos)
        self._text("right", "font", right, pos)

    # -------------------------------------------------------------- the reference's methods
    def plot(self, player=1):
        """merging_env.py:346-352: player 1 sees the ego panel; player 2 (PvP) both."""
        if player == 1:
            self.screen.blit(self.panels["right"], (WINDOW_W, 0))
        elif player == 2:
            self.screen.blit(self.panels["left"], (0, 0))
            self.screen.blit(self.panels["right"], (2 * WINDOW_W, 0))
        self.pg.display.update()

    def render(self, view, goal=None, goal_op=None, player=1, tag_left=None, tag_right=None):
        """merging_env.py:241-342 for the state in `view` (see scene())."""
        self._clear()
        pg = self.pg
        for prim in scene(view, goal, goal_op, tag_left, tag_right):
            kind, panel = prim[0], self.panels[prim[1]]
            if kind == "circle":
                pg.draw.circle(panel, color=prim[2], center=prim[3], radius=prim[4], width=prim[5])
            elif kind == "polygon":
                pg.draw.polygon(panel, prim[2], prim[3], width=prim[4])
            else:
                self._text(prim[1], prim[2], prim[3], prim[4])
        self.plot(player)
        pg.time.wait(50)

    def intro(self, player=1):
        """merging_env.py:355-366."""
        self._clear()
        self.plot(player)
        self.pg.time.wait(1000)
        self._both(INTRO_TEXT, INTRO_TEXT, (0.1 * WINDOW_W, 3 * WINDOW_H / 5))
        self.plot(player)
        self.pg.time.wait(3000)

    def prepare(self, player=1):
        """merging_env.py:368-377: a fixation cross, then a uniform 1-3 s wait (global numpy RNG)."""
        self._clear()
        cx, cy = 0.5 * WINDOW_W, 3 * WINDOW_H / 5
        for panel in ("left", "right"):
            self.pg.draw.lines(self.panels[panel], BLACK, True, [(cx - 10, cy), (cx + 10, cy)], 3)
            self.pg.draw.lines(self.panels[panel], BLACK, True, [(cx, cy - 10), (cx, cy + 10)], 3)
        self.plot(player)
        self.pg.time.wait(int(np.random.uniform(1000, 3000)))

    def feedback(self, r1, r2, player=1):
        """merging_env.py:380-387: each player's accumulated reward."""
        self._clear()
        pos = (0.3 * WINDOW_W, 3 * WINDOW_H / 5)
        self._text("left", "font", "You earn " + _r2(r2) + " points", pos)
        self._text("right", "font", "You earn " + _r2(r1) + " points", pos)
        self.plot(player)
        self.pg.time.wait(3000)

    def finish(self, sum_r1, sum_r2, player=1):
        """merging_env.py:389-395."""
        self._clear()
        pos = (0.2 * WINDOW_W, 3 * WINDOW_H / 5)
        self._text("left", "font", "Games completed. Reward: " + _r2(sum_r2), pos)
        self._text("right", "font", "Games completed. Reward: " + _r2(sum_r1), pos)
        self.plot(player)
        self.pg.time.wait(10000)

from ._rec import color as _color
from ._rec import num, point, record


def circle(surface, color, center, radius, width=0, **k):
    record("circle", surface.name, _color(color), point(center), num(radius), int(width))


def polygon(surface, color, points, width=0):
    record("polygon", surface.name, _color(color), [point(p) for p in points], int(width))


def lines(surface, color, closed, points, width=1):
    record("lines", surface.name, _color(color), bool(closed), [point(p) for p in points], int(width))

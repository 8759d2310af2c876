"""Call log and the surface / rect objects of the recording pygame stand-in."""

LOG = []
_names = {"surface": 0, "font": 0}


def clear():
    LOG.clear()
    _names["surface"] = _names["font"] = 0


def record(*entry):
    LOG.append(list(entry))


def new_name(kind):
    k = _names[kind]
    _names[kind] = k + 1
    return f"{kind[0]}{k}"


def num(v):
    return float(v)


def point(p):
    if hasattr(p, "x") and hasattr(p, "y"):
        return [num(p.x), num(p.y)]
    return [num(p[0]), num(p[1])]


def color(c):
    return [int(v) for v in c]


def _c_int(v):
    # pygame 2.1.2 pg_IntFromObj: a float goes through a C (int) cast (truncation toward 0)
    return int(v)


class Rect:
    def __init__(self, x, y, w, h):
        self.x, self.y, self.w, self.h = int(x), int(y), int(w), int(h)

    @property
    def center(self):
        return (self.x + self.w // 2, self.y + self.h // 2)

    @center.setter
    def center(self, v):
        self.x = _c_int(v[0]) - self.w // 2
        self.y = _c_int(v[1]) - self.h // 2

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
    def __init__(self, size, *a, _quiet=False, **k):
        self.size = (int(size[0]), int(size[1]))
        self.name = new_name("surface")
        if not _quiet:
            record("surface", self.name, list(self.size))

    def fill(self, c, *a, **k):
        record("fill", self.name, color(c))

    def blit(self, src, dest, *a, **k):
        what = src.desc if isinstance(src, Text) else src.name
        record("blit", self.name, what, point(dest))

    def get_rect(self, **kw):
        r = Rect(0, 0, self.size[0], self.size[1])
        for key, val in kw.items():
            setattr(r, key, val)
        return r

    def get_size(self):
        return self.size


class Text:
    """What Font.render returns: the blit records the text itself."""

    def __init__(self, font_name, text, antialias, c):
        self.desc = ["text", font_name, str(text), int(antialias), color(c)]

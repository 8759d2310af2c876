from ._rec import Surface, record


def set_mode(size, *a, **k):
    s = Surface(size, _quiet=True)
    record("set_mode", s.name, [int(size[0]), int(size[1])])
    return s


def set_caption(title, *a, **k):
    record("caption", str(title))


def update(*a, **k):
    record("update")


def flip():
    record("update")

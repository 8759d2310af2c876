from ._rec import Text, new_name, record


class Font:
    def __init__(self, name=None, size=12, _kind="font"):
        self.name = new_name("font")
        record(_kind, self.name, name, int(size))

    def render(self, text, antialias, color, background=None):
        return Text(self.name, text, antialias, color)


def SysFont(name, size, bold=False, italic=False):  # noqa: N802 - pygame's name
    return Font(name, size, _kind="sysfont")


def init():
    pass

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
            raise NotImplementedError("the stand-in only rotates by multiples of 360 degrees")
        return Vector2(self.x, self.y)

    def __iter__(self):
        return iter((self.x, self.y))

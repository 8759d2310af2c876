class Env:
    metadata = {}

    @property
    def unwrapped(self):
        return self

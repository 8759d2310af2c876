from ._rec import record


def wait(ms):
    record("wait", int(ms))
    return int(ms)


def delay(ms):
    return wait(ms)

"""Kernel timing with HIP events recorded by the dispatch packet itself.

`KernelTimer.arm(k)` makes the next mg_step / mg_step_random launch of this thread record
event pair k through hipExtLaunchKernel (mg_time_next_launch in include/merging_hip.h), so
`durations_ms()` are the kernels' own durations, not launch-to-launch intervals. The events
are created on torch's HIP runtime (libamdhip64, already loaded by `import torch`).
"""

from __future__ import annotations

import ctypes


class KernelTimer:
    def __init__(self, n: int):
        import torch  # noqa: F401 -- makes sure torch's libamdhip64 is the one bound

        from . import _native

        self._nat = _native
        self._hip = ctypes.CDLL("libamdhip64.so.7")
        self._hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self._hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                                  ctypes.c_void_p]
        self._hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self._hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        self.events = []
        for _ in range(n):
            pair = (ctypes.c_void_p(), ctypes.c_void_p())
            for e in pair:
                rc = self._hip.hipEventCreate(ctypes.byref(e))
                if rc != 0:
                    raise RuntimeError(f"hipEventCreate failed ({rc})")
            self.events.append(pair)

    def arm(self, k: int) -> None:
        a, b = self.events[k]
        self._nat.lib.mg_time_next_launch(a, b)

    def durations_ms(self, count=None):
        out = []
        for a, b in self.events[: count if count is not None else len(self.events)]:
            self._hip.hipEventSynchronize(b)
            ms = ctypes.c_float()
            rc = self._hip.hipEventElapsedTime(ctypes.byref(ms), a, b)
            if rc != 0:
                raise RuntimeError(f"hipEventElapsedTime failed ({rc})")
            out.append(ms.value)
        return out

    def close(self):
        for a, b in self.events:
            self._hip.hipEventDestroy(a)
            self._hip.hipEventDestroy(b)
        self.events = []

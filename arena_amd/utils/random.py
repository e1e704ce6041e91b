"""9-digit pseudo-random id (reference: util/random.go:10-27): Numerical Recipes LCG seeded from
time + pid, used for the TensorBoard host log path ``/arena_logs/training<9 digits>``."""
import os
import threading
import time

_state = 0
_lock = threading.Lock()


def random_int32() -> str:
    global _state
    with _lock:
        r = _state
        if r == 0:
            r = (time.time_ns() + os.getpid()) & 0xFFFFFFFF
        r = (r * 1664525 + 1013904223) & 0xFFFFFFFF
        _state = r
    return str(int(1e9) + r % int(1e9))[1:]

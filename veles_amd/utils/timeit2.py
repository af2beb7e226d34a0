"""``timeit(fn, *args)`` -> (result, seconds) (reference timeit2.py)."""
import time


def timeit(fn, *args, **kwargs):
    t0 = time.perf_counter()
    r = fn(*args, **kwargs)
    return r, time.perf_counter() - t0

"""Pure-Python stand-in for numba, used ONLY by tests/golden/make_golden.py to import the
read-only reference (/root/reference) in this container, where numba is not installed.
It is not reference code and never ships: decorators become identity functions, typed
containers become plain dict/list, and type objects only carry a NumPy dtype."""
import numpy as _np

from . import typed, types  # noqa: F401


def _identity_decorator(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]

    def wrap(fn):
        return fn

    return wrap


njit = _identity_decorator
jit = _identity_decorator
prange = range
int64 = types.int64
float64 = types.float64
boolean = types.boolean

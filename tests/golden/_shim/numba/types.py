"""Type stand-ins: usable as NumPy dtypes (via .dtype) and subscriptable like numba types."""
import numpy as _np


class _T:
    def __init__(self, dt):
        self.dtype = _np.dtype(dt)

    def __getitem__(self, item):
        return self

    def __call__(self, *a, **k):
        return self


int64 = _T(_np.int64)
int32 = _T(_np.int32)
float64 = _T(_np.float64)
boolean = _T(_np.bool_)


def Tuple(*a, **k):
    return _T(object)


UniTuple = Tuple
ListType = Tuple
DictType = Tuple

"""numba.typed stand-ins: Dict.empty -> dict, List -> list."""


class Dict(dict):
    @staticmethod
    def empty(*a, **k):
        return {}


def List(x=None):
    return [] if x is None else list(x)

"""ray.util.multiprocessing.Pool -> the standard library's process pool (same
initializer / starmap_async interface the reference uses)."""
import multiprocessing as _mp
import os as _os


def Pool(processes=None, initializer=None, initargs=()):
    n = int(_os.environ.get("GOLDEN_NCPU", processes or 1))
    return _mp.get_context("fork").Pool(n, initializer=initializer, initargs=initargs)

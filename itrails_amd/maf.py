"""MAF ingest through the native reader (itrails_amd/csrc/maf.cpp, itr_maf_*).

`read_maf` returns the layout the sweeps consume (uint16 symbols of all kept blocks back to
back + int64 block offsets, optionally per-column reference coordinates).  `maf_parser` and
`parse_coordinates` keep the reference's signatures and return types
(read_data.py:94-117, 150-220).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import lib


def _open(path: str, sp_lst: Sequence[str], ref: Optional[str]):
    if len(sp_lst) != 4:
        raise ValueError("species_list needs exactly 4 names (A, B, C, outgroup)")
    arr = (ctypes.c_char_p * 4)(*[s.encode() for s in sp_lst])
    h = ctypes.c_void_p()
    rc = lib().itr_maf_open(str(path).encode(), arr, ref.encode() if ref else None,
                            ctypes.byref(h))
    if rc == _lib.ITR_EDATA:
        raise ValueError(lib().itr_last_error().decode())
    if rc:
        msg = lib().itr_last_error().decode()
        if "cannot open" in msg:
            raise FileNotFoundError(msg)
        _lib.check(rc)
    return h


def read_maf(path: str, sp_lst: Sequence[str], ref: Optional[str] = None):
    """-> (obs uint16 [columns], off int64 [blocks+1], coords int64 or None,
    coord_off int64 or None)."""
    h = _open(path, sp_lst, ref)
    try:
        nb, nc, ncb, nco = (ctypes.c_int64() for _ in range(4))
        _lib.check(lib().itr_maf_sizes(h, ctypes.byref(nb), ctypes.byref(nc), ctypes.byref(ncb),
                                       ctypes.byref(nco)))
        obs = np.empty(nc.value, dtype=np.uint16)
        off = np.empty(nb.value + 1, dtype=np.int64)
        coords = np.empty(nco.value, dtype=np.int64) if ref else None
        coff = np.empty(ncb.value + 1, dtype=np.int64) if ref else None
        _lib.check(lib().itr_maf_copy(h, obs.ctypes.data, off.ctypes.data,
                                      coords.ctypes.data if ref else None,
                                      coff.ctypes.data if ref else None))
    finally:
        lib().itr_maf_close(h)
    return obs, off, coords, coff


def maf_parser(file: str, sp_lst: Sequence[str]) -> List[np.ndarray]:
    """read_data.py:94-117: list of int64 symbol arrays, one per kept block."""
    obs, off, _, _ = read_maf(file, sp_lst)
    o64 = obs.astype(np.int64)
    return [o64[off[k]:off[k + 1]] for k in range(len(off) - 1)]


def parse_coordinates(file: str, sp_lst: Sequence[str], ref: str) -> List[list]:
    """read_data.py:150-220: per-block lists of reference positions (-9 for gaps)."""
    _, _, coords, coff = read_maf(file, sp_lst, ref)
    return [coords[coff[k]:coff[k + 1]].tolist() for k in range(len(coff) - 1)]

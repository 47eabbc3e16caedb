"""HMM sweeps on the GPU behind the reference's own call surface.

Two layers:

* Device layer (`Model`, `Plan`, `forward_loglik_device`, `viterbi_device`,
  `posterior_device`): inputs and outputs are torch.cuda tensors already resident in HBM;
  every call is one C-ABI call (include/itrails_hip.h) on the current torch stream.
* Reference layer — the functions of optimizer.py:145-377 with the same names, arguments,
  return types and semantics (`forward_loglik`, `loglik_wrapper`, `loglik_wrapper_par`,
  `viterbi_wrapper`, `post_prob`, `post_prob_wrapper`, and the standalone sweeps `forward`,
  `backward`, `viterbi` (omega, prev) and `backtrack_viterbi`), so a caller written against
  the reference drops in unchanged.  `order` arguments are accepted and ignored: the alphabet
  expansion is tabulated once (itrails_amd/tables.py).

No code path here computes on the host: if libitrails_hip.so is missing or the device is
unavailable the calls raise.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import threading
from collections import OrderedDict
from typing import Iterable, List, Sequence

import numpy as np

from . import _lib
from ._lib import check, lib, ptr
from .tables import HmmTables, build_tables

__all__ = [
    "Model", "Plan", "concat_blocks", "forward_loglik_device", "viterbi_device",
    "posterior_device", "forward_loglik", "loglik_wrapper", "loglik_wrapper_par",
    "viterbi_wrapper", "post_prob", "post_prob_wrapper", "block_logliks", "forward",
    "backward", "viterbi", "backtrack_viterbi", "block_rows_device",
]


# ---------------------------------------------------------------------------------------
# objects
# ---------------------------------------------------------------------------------------
class Model:
    """Model tables resident on the current HIP device (itr_model_create)."""

    def __init__(self, a=None, b=None, pi=None, tables: HmmTables | None = None):
        self.tables = tables if tables is not None else build_tables(a, b, pi)
        t = self.tables
        if not 1 <= t.n <= _lib.MAX_STATES:
            raise ValueError(f"{t.n} hidden states; the device path supports 1..{_lib.MAX_STATES}")
        h = ctypes.c_void_p()
        check(lib().itr_model_create(t.n, ptr(t.a), ptr(t.log_a), ptr(t.emit), ptr(t.log_emit),
                                     ptr(t.pi_emit), ptr(t.log_pi_emit), ctypes.byref(h)))
        self.handle = h.value
        self.n = t.n

    def prepare_viterbi(self):
        """Build the Viterbi slot tables now (itr_model_prepare_viterbi), so that the decode
        calls stay asynchronous; otherwise the first Viterbi call builds them."""
        check(lib().itr_model_prepare_viterbi(self.handle))
        return self

    def close(self):
        if getattr(self, "handle", None):
            lib().itr_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def concat_blocks(V_lst: Sequence[np.ndarray]):
    """V_lst (list of int arrays of symbols, read_data.py:94-117) -> (uint16 obs, int64 off).

    Symbols must be in [0, 625); the reference would raise IndexError on anything else.
    Lists of int64 arrays (what read_data.py produces) are packed and range-checked by the
    library in one threaded pass (itr_pack_symbols); anything else goes through NumPy."""
    if V_lst and all(isinstance(v, np.ndarray) and v.dtype == np.int64 and v.ndim == 1
                     and v.flags.c_contiguous for v in V_lst):
        nb = len(V_lst)
        lens = np.fromiter((v.shape[0] for v in V_lst), dtype=np.int64, count=nb)
        ptrs = np.fromiter((v.ctypes.data for v in V_lst), dtype=np.uintp, count=nb)
        obs = np.empty(int(lens.sum()), dtype=np.uint16)
        off = np.empty(nb + 1, dtype=np.int64)
        rc = lib().itr_pack_symbols(ptr(ptrs), ptr(lens), nb, ptr(obs), ptr(off))
        if rc == _lib.ITR_EDATA:
            raise IndexError(lib().itr_last_error().decode())
        check(rc)
        return obs, off
    lens = np.fromiter((len(v) for v in V_lst), dtype=np.int64, count=len(V_lst))
    off = np.zeros(len(V_lst) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    if off[-1]:
        obs = np.concatenate([np.asarray(v) for v in V_lst])
        if obs.min() < 0 or obs.max() >= _lib.NOBS:
            raise IndexError("observed symbol outside the 625-letter alphabet")
        obs = obs.astype(np.uint16)
    else:
        obs = np.zeros(0, dtype=np.uint16)
    return obs, off


class Plan:
    """Block layout of one alignment on the current device (itr_plan_create_ex).

    split_frac / post_split_frac: the plan's work-decomposition knobs (None = the library's
    defaults; 0 disables the split forward / the posterior's concurrent split)."""

    def __init__(self, block_off, split_frac=None, post_split_frac=None):
        off = np.ascontiguousarray(block_off, dtype=np.int64)
        if off.ndim != 1 or len(off) < 1 or off[0] != 0 or np.any(np.diff(off) < 0):
            raise ValueError("block offsets must start at 0 and be non-decreasing")
        self.off = off
        self.nblocks = len(off) - 1
        self.total = int(off[-1])
        h = ctypes.c_void_p()
        check(lib().itr_plan_create_ex(ptr(off), self.nblocks,
                                       -1.0 if split_frac is None else float(split_frac),
                                       -1.0 if post_split_frac is None else float(post_split_frac),
                                       ctypes.byref(h)))
        self.handle = h.value

    def reserve(self, n: int, posterior: bool = False):
        check(lib().itr_plan_reserve(self.handle, n, int(posterior)))

    def set_prune_len(self, length=None):
        """Per-wave Viterbi step choice (itr_plan_set_prune_len): blocks shorter than `length`
        take the bound-pruned step; None = the planned lengths."""
        check(lib().itr_plan_set_prune_len(self.handle, -1 if length is None else int(length)))

    def close(self):
        if getattr(self, "handle", None):
            lib().itr_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _stream_handle():
    import torch

    return torch.cuda.current_stream().cuda_stream


# ---------------------------------------------------------------------------------------
# device layer (torch.cuda tensors)
# ---------------------------------------------------------------------------------------
# The caller guarantees symbol values < 625 (concat_blocks / the MAF reader check them);
# the kernels clamp out-of-range symbols for memory safety only.
def _check_obs(plan: Plan, d_obs):
    import torch

    if d_obs.dtype not in (torch.int16, torch.uint16):
        raise TypeError(f"d_obs must be int16/uint16 symbols, got {d_obs.dtype}")
    if not d_obs.is_cuda or not d_obs.is_contiguous():
        raise ValueError("d_obs must be a contiguous device tensor")
    if d_obs.device.index != torch.cuda.current_device():
        raise ValueError(f"d_obs lives on {d_obs.device}, current device is "
                         f"cuda:{torch.cuda.current_device()}")
    if d_obs.numel() < plan.total:
        raise ValueError(f"d_obs holds {d_obs.numel()} columns, the plan {plan.total}")


def _out(out, shape, dtype, device):
    import torch

    if out is None:
        return torch.empty(shape, dtype=dtype, device=device)
    if out.dtype != dtype or tuple(out.shape) != tuple(shape) or out.device != device \
            or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous {dtype} tensor of shape {tuple(shape)} "
                         f"on {device}")
    return out


def forward_loglik_device(model: Model, plan: Plan, d_obs, out=None):
    """Per-block log-likelihoods (float64 [nblocks]) for int16/uint16 symbols on device."""
    import torch

    _check_obs(plan, d_obs)
    out = _out(out, (plan.nblocks,), torch.float64, d_obs.device)
    check(lib().itr_forward_loglik(model.handle, plan.handle, ptr(d_obs), ptr(out),
                                   _stream_handle()))
    return out


def viterbi_device(model: Model, plan: Plan, d_obs, out=None):
    """Viterbi state per column (uint8 [total])."""
    import torch

    _check_obs(plan, d_obs)
    out = _out(out, (plan.total,), torch.uint8, d_obs.device)
    check(lib().itr_viterbi(model.handle, plan.handle, ptr(d_obs), ptr(out), _stream_handle()))
    return out


def forward_viterbi_device(model: Model, plan: Plan, d_obs, out_ll=None, out_path=None):
    """forward_loglik_device and viterbi_device in one call (identical paths, log-likelihoods
    equal to rounding), the forward sweep overlapped with the Viterbi sweep's longest blocks
    (itr_forward_viterbi)."""
    import torch

    _check_obs(plan, d_obs)
    out_ll = _out(out_ll, (plan.nblocks,), torch.float64, d_obs.device)
    out_path = _out(out_path, (plan.total,), torch.uint8, d_obs.device)
    check(lib().itr_forward_viterbi(model.handle, plan.handle, ptr(d_obs), ptr(out_ll),
                                    ptr(out_path), _stream_handle()))
    return out_ll, out_path


def posterior_device(model: Model, plan: Plan, d_obs, out=None):
    """Posterior state probabilities (float64 [total, N])."""
    import torch

    _check_obs(plan, d_obs)
    out = _out(out, (plan.total, model.n), torch.float64, d_obs.device)
    check(lib().itr_posterior(model.handle, plan.handle, ptr(d_obs), ptr(out),
                              _stream_handle()))
    return out


ROWS_FORWARD, ROWS_BACKWARD, ROWS_VITERBI = 0, 1, 2


def block_rows_device(model: Model, kind: int, d_obs, out=None, out_prev=None):
    """The reference's matrices of ONE block (itr_block_rows): kind 0 log alpha, 1 log beta,
    2 omega (and, with out_prev or kind 2 by default, the back-pointers [T-1, N]); float64
    [T, N] on device.  Returns rows, or (omega, prev) for kind 2."""
    import torch

    if d_obs.dtype not in (torch.int16, torch.uint16) or not d_obs.is_cuda \
            or not d_obs.is_contiguous():
        raise TypeError("d_obs must be a contiguous int16/uint16 device tensor")
    T = d_obs.numel()
    if T < 1:
        raise IndexError("index 0 is out of bounds for axis 0 with size 0")
    out = _out(out, (T, model.n), torch.float64, d_obs.device)
    prev = None
    if kind == ROWS_VITERBI:
        prev = _out(out_prev, (T - 1, model.n), torch.float64, d_obs.device)
    check(lib().itr_block_rows(model.handle, int(kind), ptr(d_obs), T, ptr(out),
                               ptr(prev) if prev is not None and T > 1 else None,
                               _stream_handle()))
    return (out, prev) if kind == ROWS_VITERBI else out


def last_kernel_ms(which: str) -> float:
    v = ctypes.c_double()
    check(lib().itr_last_kernel_ms(which.encode(), ctypes.byref(v)))
    return v.value


# ---------------------------------------------------------------------------------------
# host-buffer helpers (copy in / run / copy out inside the library)
# ---------------------------------------------------------------------------------------
def block_logliks(model: Model, plan: Plan, obs: np.ndarray) -> np.ndarray:
    out = np.zeros(plan.nblocks)
    obs = np.ascontiguousarray(obs, dtype=np.uint16)
    check(lib().itr_forward_loglik_host(model.handle, plan.handle, ptr(obs), ptr(out)))
    return out


def _paths(model: Model, plan: Plan, obs: np.ndarray) -> np.ndarray:
    out = np.zeros(plan.total, dtype=np.uint8)
    obs = np.ascontiguousarray(obs, dtype=np.uint16)
    check(lib().itr_viterbi_host(model.handle, plan.handle, ptr(obs), ptr(out)))
    return out


def _posteriors(model: Model, plan: Plan, obs: np.ndarray) -> np.ndarray:
    out = np.zeros((plan.total, model.n))
    obs = np.ascontiguousarray(obs, dtype=np.uint16)
    check(lib().itr_posterior_host(model.handle, plan.handle, ptr(obs), ptr(out)))
    return out


# ---------------------------------------------------------------------------------------
# the wrappers' device objects, reused across calls: a caller scoring and then decoding one
# alignment with one model (loglik_wrapper, then viterbi_wrapper / post_prob_wrapper) builds
# the model tables, the Viterbi slot tables and the plan once.  Keys are the contents
# (a, b, pi bytes; block offsets) and the current device, so a changed input is a new entry;
# at most two of each are kept (evicted objects are freed when no caller holds them).
# Models are read-only once built (their Viterbi slot tables are built under a lock in the
# library), so threads share them; a plan owns its sweep workspaces and work counters, so
# plans are cached per thread: two threads decoding the same layout never sweep into one
# plan's counters and rows at the same time.
# ---------------------------------------------------------------------------------------
_CACHE_LOCK = threading.Lock()
_MODELS: "OrderedDict" = OrderedDict()
_TLS = threading.local()
_CACHE_SIZE = 2


def _thread_plans() -> "OrderedDict":
    d = getattr(_TLS, "plans", None)
    if d is None:
        d = _TLS.plans = OrderedDict()
    return d


def _device_index():
    import torch
    return torch.cuda.current_device()


def _digest(*arrays):
    h = hashlib.blake2b(digest_size=20)
    for x in arrays:
        x = np.ascontiguousarray(x)
        h.update(f"{x.dtype.str}{x.shape}".encode())
        h.update(memoryview(x).cast("B"))
    return h.digest()


def _cache_get(cache, key, make):
    with _CACHE_LOCK:  # (a per-thread cache needs no lock; one lock keeps this simple)
        obj = cache.get(key)
        if obj is not None:
            cache.move_to_end(key)
            return obj
    obj = make()
    with _CACHE_LOCK:
        cache[key] = obj
        while len(cache) > _CACHE_SIZE:
            cache.popitem(last=False)
    return obj


def _cached_model(a, b, pi, decode=False) -> Model:
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    pi = np.ascontiguousarray(pi, dtype=np.float64)
    m = _cache_get(_MODELS, (_device_index(), _digest(a, b, pi)), lambda: Model(a, b, pi))
    if decode and not getattr(m, "_prepared", False):
        m.prepare_viterbi()
        m._prepared = True
    return m


def _cached_plan(off) -> Plan:
    off = np.ascontiguousarray(off, dtype=np.int64)
    return _cache_get(_thread_plans(), (_device_index(), _digest(off)), lambda: Plan(off))


def clear_caches():
    """Drop the wrappers' cached models and the calling thread's cached plans (their device
    memory is freed when no caller holds them)."""
    with _CACHE_LOCK:
        _MODELS.clear()
        _thread_plans().clear()


def _load_blocks_ext():
    """The V_lst scan in C (csrc/blocks_ext.c, built with the library); ITR_BLOCKS_EXT names
    another build of it (the sanitizer build of scripts/asan_host.sh)."""
    path = os.environ.get("ITR_BLOCKS_EXT")
    if path:
        import importlib.util
        spec = importlib.util.spec_from_file_location("itrails_amd._blocks", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod
    try:
        from . import _blocks
        return _blocks
    except ImportError:  # (argument marshalling only: the Python scan below does the same)
        return None


_blocks_ext = _load_blocks_ext()


def _lens_ptrs(V_lst):
    """(lens, data pointers, offsets) of a V_lst of 1-D C-contiguous int64 arrays, or None
    when some entry is not one (those inputs take the NumPy packing path)."""
    nb = len(V_lst)
    lens = np.empty(nb, dtype=np.int64)
    ptrs = np.empty(nb, dtype=np.uintp)
    if _blocks_ext is not None:
        if not _blocks_ext.scan(V_lst, lens, ptrs):
            return None
    else:
        for k, v in enumerate(V_lst):
            if not (isinstance(v, np.ndarray) and v.dtype == np.int64 and v.ndim == 1 and
                    v.flags.c_contiguous):
                return None
            lens[k] = v.shape[0]
            ptrs[k] = v.ctypes.data
    off = np.zeros(nb + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return lens, ptrs, off


def _check_data(rc):
    if rc == _lib.ITR_EDATA:  # a symbol outside the alphabet: the reference's IndexError
        raise IndexError(lib().itr_last_error().decode())
    check(rc)


def _split(arr, off):
    o = off.tolist()
    return [arr[i:j] for i, j in zip(o[:-1], o[1:])]


# ---------------------------------------------------------------------------------------
# reference layer: optimizer.py:145-377
# ---------------------------------------------------------------------------------------
def loglik_wrapper(a, b, pi, V_lst: Iterable[np.ndarray]) -> float:
    """Sum of forward log-likelihoods over blocks, accumulated in block order like
    optimizer.py:93-116 (`acc += forward_loglik(...)`)."""
    V_lst = list(V_lst)
    if not V_lst:
        return 0
    lp = _lens_ptrs(V_lst)
    if lp is not None:  # read_data.py's blocks: packed into pinned memory by the library
        lens, ptrs, off = lp
        model, plan = _cached_model(a, b, pi), _cached_plan(off)
        ll = np.empty(len(V_lst))
        _check_data(lib().itr_forward_loglik_blocks(model.handle, plan.handle, ptr(ptrs),
                                                    ptr(lens), len(V_lst), ptr(ll)))
    else:
        obs, off = concat_blocks(V_lst)
        model, plan = _cached_model(a, b, pi), _cached_plan(off)
        ll = block_logliks(model, plan, obs)
    acc = 0
    for v in ll.tolist():
        acc += v
    return acc


# optimizer.py:40-65 fans blocks out over joblib workers and sums in block order; on the
# device all blocks of a process already run in parallel, and multi-GPU sharding is
# itrails_amd.distributed.loglik_wrapper_dist.
loglik_wrapper_par = loglik_wrapper


def forward_loglik(a, b, pi, V, order=None) -> float:
    """Log-likelihood of one block (optimizer.py:145-162)."""
    return loglik_wrapper(a, b, pi, [V])


def viterbi_wrapper(a, b, pi, V_lst: Iterable[np.ndarray]) -> List[np.ndarray]:
    """Viterbi path per block as float64 arrays (optimizer.py:357-377, 336-354)."""
    V_lst = list(V_lst)
    if not V_lst:
        return []
    lp = _lens_ptrs(V_lst)
    if lp is not None:
        lens, ptrs, off = lp
        if off[-1] == 0:
            return [np.zeros(0) for _ in V_lst]
        model, plan = _cached_model(a, b, pi, decode=True), _cached_plan(off)
        path = np.empty(int(off[-1]))
        _check_data(lib().itr_viterbi_blocks(model.handle, plan.handle, ptr(ptrs), ptr(lens),
                                             len(V_lst), ptr(path)))
        return _split(path, off)
    obs, off = concat_blocks(V_lst)
    if off[-1] == 0:
        return [np.zeros(0) for _ in V_lst]
    model, plan = _cached_model(a, b, pi, decode=True), _cached_plan(off)
    path = _paths(model, plan, obs).astype(np.float64)
    return _split(path, off)


def post_prob_wrapper(a, b, pi, V_lst: Iterable[np.ndarray]) -> List[np.ndarray]:
    """Posterior matrices (T x N float64) per block (optimizer.py:241-262, 216-238)."""
    V_lst = list(V_lst)
    obs, off = concat_blocks(V_lst)
    n = np.asarray(a).shape[0]
    if off[-1] == 0:
        return [np.zeros((0, n)) for _ in V_lst]
    model, plan = _cached_model(a, b, pi), _cached_plan(off)
    post = _posteriors(model, plan, obs)
    return _split(post, off)


def post_prob(a, b, pi, V, order=None) -> np.ndarray:
    """Posterior matrix of one block (optimizer.py:216-238)."""
    return post_prob_wrapper(a, b, pi, [V])[0]


# the standalone sweeps (optimizer.py:165-213, 305-354): one block, numpy in and out
def _one_block(V):
    import torch

    obs, _ = concat_blocks([np.asarray(V)])
    if obs.size == 0:
        raise IndexError("index 0 is out of bounds for axis 0 with size 0")
    return torch.from_numpy(obs.astype(np.int16)).cuda()


def forward(a, b, pi, V, order=None) -> np.ndarray:
    """Log-scaled forward matrix alpha (T x N float64) of one block (optimizer.py:165-188)."""
    d_obs = _one_block(V)
    model = Model(a, b, pi)
    return block_rows_device(model, ROWS_FORWARD, d_obs).cpu().numpy()


def backward(a, b, V, order=None) -> np.ndarray:
    """Log-scaled backward matrix beta (T x N float64) of one block, with the reference's
    (beta * e) @ a recursion (optimizer.py:191-213)."""
    d_obs = _one_block(V)
    n = np.asarray(a).shape[0]
    model = Model(a, b, np.full(n, 1.0 / n))  # (pi takes no part in beta)
    return block_rows_device(model, ROWS_BACKWARD, d_obs).cpu().numpy()


def viterbi(a, b, pi, V, order=None):
    """(omega, prev) of one block (optimizer.py:305-333): omega T x N, prev (T-1) x N float64
    back-pointers (first maximum, like np.argmax)."""
    d_obs = _one_block(V)
    model = Model(a, b, pi)
    omega, prev = block_rows_device(model, ROWS_VITERBI, d_obs)
    return omega.cpu().numpy(), prev.cpu().numpy()


def backtrack_viterbi(omega, prev) -> np.ndarray:
    """The Viterbi path (float64 [T]) from omega and prev (optimizer.py:336-354)."""
    import torch

    omega = np.ascontiguousarray(omega, dtype=np.float64)
    T = omega.shape[0]
    if T < 1:
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")
    n = omega.shape[1]
    prev = np.ascontiguousarray(prev, dtype=np.float64).reshape(max(T - 1, 0), n)
    d_om = torch.from_numpy(omega).cuda()
    d_prev = torch.from_numpy(prev).cuda() if T > 1 else None
    d_path = torch.empty(T, dtype=torch.float64, device=d_om.device)
    check(lib().itr_backtrack_rows(ptr(d_om), ptr(d_prev) if d_prev is not None else None, T, n,
                                   ptr(d_path), _stream_handle()))
    out = d_path.cpu().numpy()
    if np.isnan(out).any():  # a back-pointer outside the states (the kernel stopped there)
        raise IndexError(f"backtrack_viterbi: a back-pointer is not a state index in [-{n}, {n})")
    return out

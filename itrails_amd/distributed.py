"""Multi-GPU decoding: MAF blocks sharded across ranks, one process per GPU.

MAF blocks are independent HMM sequences — every block restarts from pi (optimizer.py:182,
323) — so the sweeps shard with no data-path exchange:

* `shard_ranges` partitions the blocks into `world` CONTIGUOUS ranges balanced by column
  count (not block count), so each rank's work is a slice of the concatenated alignment and
  the union over ranks is the reference's block order.
* log-likelihood: the only exchange step.  Each rank places its per-block values into a
  zero vector of all blocks and one all-reduce (sum) over the communicator gathers them
  exactly (x + 0 = x, disjoint slices); every rank then sums the vector on the host in block
  order — the `acc += forward_loglik(...)` loop of loglik_wrapper (optimizer.py:93-116) — so
  the total is bit-identical for every GPU count.  With RCCL ("nccl" backend, xGMI) the vector
  is a device tensor; with gloo (CPU tests) a host tensor.
* Viterbi paths and posteriors need no collective: each rank returns its own blocks.

The per-shard compute is the HIP path of itrails_amd.hmm by default; `compute` may be
injected (the CPU tests inject the oracle as the checker of the sharding logic itself).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

__all__ = ["shard_ranges", "local_blocks", "sharded_loglik", "sharded_viterbi",
           "sharded_posterior", "gather_block_values"]


def shard_ranges(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous block ranges [lo, hi) per rank with column counts as equal as a
    contiguous split allows (rank r takes the blocks whose column midpoint falls in the
    r-th 1/world of the alignment).  Ranges may be empty when blocks < ranks."""
    if world < 1:
        raise ValueError("world size must be >= 1")
    lens = np.asarray(lengths, dtype=np.int64)
    nb = len(lens)
    if nb == 0:
        return [(0, 0)] * world
    off = np.zeros(nb + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    total = int(off[-1])
    if total == 0:  # only empty blocks: split by count
        cuts = [nb * r // world for r in range(world + 1)]
    else:
        mid2 = off[:-1] + off[1:]  # twice the column midpoint of every block
        cuts = [0] + [int(np.searchsorted(mid2, 2 * total * r // world, side="left"))
                      for r in range(1, world)] + [nb]
        for r in range(1, world + 1):  # monotone
            cuts[r] = max(cuts[r], cuts[r - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def _group_info(group=None):
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def local_blocks(V_lst: Sequence[np.ndarray], group=None):
    """(lo, hi, V_lst[lo:hi]) of this rank."""
    rank, world = _group_info(group)
    lo, hi = shard_ranges([len(v) for v in V_lst], world)[rank]
    return lo, hi, list(V_lst[lo:hi])


def gather_block_values(local: np.ndarray, lo: int, nblocks: int, group=None,
                        device=None) -> np.ndarray:
    """All ranks' per-block float64 values in global block order (one all-reduce of a
    zero-padded vector; exact because the slices are disjoint)."""
    import torch
    import torch.distributed as dist

    rank, world = _group_info(group)
    if world == 1:
        out = np.zeros(nblocks, dtype=np.float64)
        out[lo:lo + len(local)] = local
        return out
    buf = torch.zeros(nblocks, dtype=torch.float64, device=device or "cpu")
    if len(local):
        buf[lo:lo + len(local)] = torch.from_numpy(np.ascontiguousarray(local, dtype=np.float64)).to(buf.device)
    dist.all_reduce(buf, group=group)
    return buf.cpu().numpy()


def _default_compute(kind: str) -> Callable:
    from . import hmm

    if kind == "loglik":
        def f(a, b, pi, V_lst):
            if not V_lst:
                return np.zeros(0)
            obs, off = hmm.concat_blocks(V_lst)
            model = hmm.Model(a, b, pi)
            plan = hmm.Plan(off)
            return hmm.block_logliks(model, plan, obs)
        return f
    if kind == "viterbi":
        return lambda a, b, pi, V_lst: hmm.viterbi_wrapper(a, b, pi, V_lst) if V_lst else []
    if kind == "posterior":
        return lambda a, b, pi, V_lst: hmm.post_prob_wrapper(a, b, pi, V_lst) if V_lst else []
    raise ValueError(kind)


def _comm_device():
    import torch
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return None


def sharded_loglik(a, b, pi, V_lst: Sequence[np.ndarray], group=None,
                   compute: Optional[Callable] = None) -> float:
    """loglik_wrapper (optimizer.py:93-116) over all ranks: every rank passes the full V_lst
    (or any list with the same block lengths), computes its contiguous shard and receives
    the block-order sum over every block.  Identical on every rank and every world size."""
    compute = compute or _default_compute("loglik")
    lo, hi, mine = local_blocks(V_lst, group)
    vals = np.asarray(compute(a, b, pi, mine), dtype=np.float64)
    if len(vals) != hi - lo:
        raise RuntimeError("per-block compute returned the wrong number of values")
    allv = gather_block_values(vals, lo, len(V_lst), group, _comm_device())
    acc = 0.0
    for v in allv.tolist():  # block order, like `acc += ...`
        acc += v
    return acc


def sharded_viterbi(a, b, pi, V_lst, group=None, compute: Optional[Callable] = None):
    """(lo, paths of this rank's blocks) — viterbi_wrapper semantics per block, no
    collective."""
    compute = compute or _default_compute("viterbi")
    lo, hi, mine = local_blocks(V_lst, group)
    return lo, compute(a, b, pi, mine)


def sharded_posterior(a, b, pi, V_lst, group=None, compute: Optional[Callable] = None):
    """(lo, posteriors of this rank's blocks) — post_prob_wrapper semantics, no collective."""
    compute = compute or _default_compute("posterior")
    lo, hi, mine = local_blocks(V_lst, group)
    return lo, compute(a, b, pi, mine)

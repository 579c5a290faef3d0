"""Multi-GPU fan-out for one process per GPU (torch.distributed over RCCL).

Keys are independent (jepsen.independent, register.clj:108), so the only
partitioning is a static, contiguous, cost-balanced split of the key range
(lc_plan_partition: cost = records + per-key overhead) — no data-path
collective.  Results are merged with jepsen.independent's rule
(false > :unknown > true) after a gather of per-key verdicts.
"""
import numpy as np

from . import abi


def shard(key_off, rank, world):
    """(first_key, last_key) of this rank's contiguous cost-balanced range."""
    b = abi.plan_partition(key_off, world)
    return int(b[rank]), int(b[rank + 1])


def slice_keys(ops, key_off, a, b):
    """Records and rebased offsets of keys [a, b)."""
    sub = ops[key_off[a]:key_off[b]]
    off = key_off[a:b + 1] - key_off[a]
    return sub, off


def merge_verdicts(verdicts):
    """jepsen.independent merge: any false -> False; else any unknown -> 'unknown'."""
    v = np.asarray(verdicts)
    if (v == abi.LC_INVALID).any():
        return False
    if (v == abi.LC_UNKNOWN).any():
        return "unknown"
    return True


def gather_results(local, key_range, n_keys, group=None):
    """All-gather per-key verdict / fail_op arrays of every rank's shard into
    full-length arrays (CPU tensors: works with gloo and, on GPU, nccl via
    the caller's device tensors)."""
    import torch
    import torch.distributed as dist
    a, b = key_range
    full = torch.full((n_keys, 2), -2, dtype=torch.int64)
    full[a:b, 0] = torch.from_numpy(local["verdict"].astype(np.int64))
    full[a:b, 1] = torch.from_numpy(local["fail_op"].astype(np.int64))
    # every entry outside this shard holds -2; max-reduce fills them in
    dist.all_reduce(full, op=dist.ReduceOp.MAX, group=group)
    return full[:, 0].numpy(), full[:, 1].numpy()

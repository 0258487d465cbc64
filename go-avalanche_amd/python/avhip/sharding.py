"""Multi-GPU decomposition of one network (one process per GPU).

Two exact decompositions of the batched round:

* target sharding — every rank holds all nodes for a contiguous, 32-aligned
  range of target blocks and regenerates the same Philox peer lists. VoteRecord
  updates never couple targets (processor.go:94-117) except through the 4096
  poll cap, which cannot bind when M <= 4096, so there is no per-round
  exchange.
* node sharding — every rank owns a contiguous, equal node range; after each
  round the published-preference rows are all-gathered (RCCL inside
  libavhip.so via av_comm_init; `allgather_pref_rows` below is the same
  exchange over torch.distributed, used by the gloo CPU rehearsal).
"""
from __future__ import annotations

import numpy as np


def target_shard(n_targets: int, world: int, rank: int) -> tuple[int, int]:
    """[t0, t1) for `rank`: whole 32-target blocks, balanced to within one block."""
    blocks = (n_targets + 31) // 32
    b0, b1 = rank * blocks // world, (rank + 1) * blocks // world
    return b0 * 32, min(b1 * 32, n_targets)


def node_shard(n_nodes: int, world: int, rank: int) -> tuple[int, int]:
    """[n0, n1) for `rank`; the collective needs equal shards (N % world == 0)."""
    if n_nodes % world:
        raise ValueError(f"node sharding needs n_nodes % world == 0 ({n_nodes} % {world})")
    per = n_nodes // world
    return rank * per, (rank + 1) * per


def allgather_pref_rows(local_rows: np.ndarray, world: int, group=None) -> np.ndarray:
    """All-gather every rank's [n_local, M] preference rows into [N, M]
    (rank-ordered), over torch.distributed (gloo on CPU)."""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(local_rows))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return torch.cat(parts).numpy()

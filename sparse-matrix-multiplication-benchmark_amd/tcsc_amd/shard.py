"""Output-column sharding: rank g of G owns the contiguous
column block [g*N//G, (g+1)*N//G).  X is replicated, B and W are sliced,
each rank writes its own M x (c1-c0) block; there is no exchange step, so no
collective is on the data path (tcsc.c:113 -- columns are independent)."""
from __future__ import annotations


def column_range(n_cols: int, world: int, rank: int) -> tuple[int, int]:
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} of {world}")
    return (n_cols * rank) // world, (n_cols * (rank + 1)) // world


def all_ranges(n_cols: int, world: int):
    return [column_range(n_cols, world, r) for r in range(world)]


def rank_env() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment."""
    import os

    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))

"""Multi-GPU sharding of independent environments.

Environments never read each other's state (one OsimModel per env,
opensim_environment.py:37), so N environments split into contiguous index
blocks, one block per GPU/process, with no data-path collective.  Device-drawn
reset indices depend on the global env index (bioim_set_env_offset), so a
sharded run reproduces an unsharded run of the same env indices bit for bit.
The only cross-rank operations are the bench's barrier and max-over-ranks
timing, done on the host (gloo).
"""
from __future__ import annotations

import os


def shard_range(total: int, rank: int, world: int):
    """[lo, hi) of contiguous env block `rank` of `world` (sizes differ by <= 1)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def dist_env():
    """(rank, world, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1)),
            int(os.environ.get('LOCAL_RANK', 0)))


def make_shard(env_id: str, total_envs: int, config=None, precision: int = 64, seed: int = 0,
               auto_reset: bool = True):
    """This rank's VectorEnv over its block of the global env index space."""
    from .vector_env import VectorEnv
    rank, world, local = dist_env()
    lo, hi = shard_range(total_envs, rank, world)
    return VectorEnv(env_id, hi - lo, config=config, device=local, precision=precision, seed=seed,
                     auto_reset=auto_reset, env_offset=lo)

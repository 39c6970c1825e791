"""Pool sharding helpers of the gloo multi-rank tests (tests/test_distributed.py):
the static form of what the product's fronts do online (nakama_amd/cluster.py
places pools over ranks, mm_create_multi over devices).

A pool is the set of tickets whose queries all require the same keyword term
on the pool-key fields (e.g. mode x region).  A ticket can only ever be
selected by a search of its own pool, so processDefault's greedy pass
decomposes exactly into independent per-pool passes: pools are assigned whole
to ranks and every rank runs its own interval pass with no data-path
collective.  The global result (the reference's group order) is the
concatenation of the ranks' groups ordered by their searching ticket's pinned
position (CreatedAt, Ticket) — `merge_groups` below.
"""
from typing import Dict, List, Sequence, Tuple


def assign_pools(pool_sizes: Sequence[int], world: int) -> List[List[int]]:
    """Longest-processing-time bin packing of pools onto ranks (ties broken by
    pool id, so every rank computes the same assignment)."""
    bins: List[List[int]] = [[] for _ in range(world)]
    load = [0] * world
    for p in sorted(range(len(pool_sizes)), key=lambda p: (-pool_sizes[p], p)):
        r = min(range(world), key=lambda r: (load[r], r))
        bins[r].append(p)
        load[r] += pool_sizes[p]
    return bins


def pool_mask(pools: Sequence[int]) -> int:
    m = 0
    for p in pools:
        m |= 1 << p
    return m


def merge_groups(per_rank: Sequence[Sequence[Sequence[Tuple[str, int]]]],
                 created_at: Dict[str, int]) -> List[List[Tuple[str, int]]]:
    """Global group order: processDefault emits a group when its searching
    ticket (the group's last entry) is processed, in (CreatedAt, Ticket) order."""
    allg = [g for groups in per_rank for g in groups]
    return sorted(allg, key=lambda g: (created_at[g[-1][0]], g[-1][0]))

"""Multi-GPU modes of the match path.

Topic-sharded (C1-C3, C5): every rank holds a replica of the index and matches
its own contiguous slice of the topic stream; no data-path collective.

Filter-sharded (C4, filter sets beyond one GPU): rank r holds the keys whose
index is r mod N; every rank matches the same topic batch against its shard;
then the per-shard hit lists are exchanged with one allgather of per-topic
counts (u32) and one allgatherv of the u32 values (RCCL over xGMI on GPUs, gloo
on CPU), and merged per topic.  Shards hold disjoint keys, so the merged list
is the union; it is returned sorted ascending by value (the set semantics of
matches/3; SURVEY.md 8e "k-way merge").
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def topic_slice(rank: int, world: int, batch: int) -> tuple[int, int]:
    """Topic-sharded mode: [first, first + batch) of the topic stream for `rank`."""
    return rank * batch, batch


def allgatherv_hits(hit_offs: torch.Tensor, vals: torch.Tensor, group=None):
    """Exchange one rank's CSR hit lists with every rank and merge them.

    hit_offs: int64 [n+1] (this rank's CSR offsets), vals: int32 [hit_offs[n]].
    Returns (merged_offs int64 [n+1], merged_vals int32) identical on every rank,
    values of each topic sorted ascending.
    """
    world = dist.get_world_size(group)
    n = hit_offs.numel() - 1
    dev = vals.device
    counts = (hit_offs[1:] - hit_offs[:-1]).to(torch.int32)
    # 1. allgather per-topic counts (n x u32 per rank)
    parts = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(world)]
    dist.all_gather(parts, counts.contiguous(), group=group)
    all_counts = torch.stack(parts)
    totals = all_counts.to(torch.int64).sum(dim=1)
    # 2. allgatherv of the values: pad every rank's payload to the largest one
    maxlen = int(totals.max().item()) if world else 0
    send = torch.zeros(max(maxlen, 1), dtype=torch.int32, device=dev)
    send[: vals.numel()] = vals
    recv_parts = [torch.empty(max(maxlen, 1), dtype=torch.int32, device=dev) for _ in range(world)]
    dist.all_gather(recv_parts, send, group=group)
    recv = torch.stack(recv_parts)
    # 3. merge: per topic, the union of the shards' lists, sorted by value
    per_topic = all_counts.to(torch.int64).sum(dim=0)
    merged_offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    merged_offs[1:] = torch.cumsum(per_topic, dim=0)
    topic_ids = torch.arange(n, device=dev, dtype=torch.int64)
    parts_t, parts_v = [], []
    for r in range(world):
        c = all_counts[r].to(torch.int64)
        tot = int(totals[r].item())
        parts_t.append(torch.repeat_interleave(topic_ids, c))
        parts_v.append(recv[r, :tot])
    t_all = torch.cat(parts_t) if parts_t else torch.empty(0, dtype=torch.int64, device=dev)
    v_all = torch.cat(parts_v) if parts_v else torch.empty(0, dtype=torch.int32, device=dev)
    key = (t_all << 32) | (v_all.to(torch.int64) & 0xFFFFFFFF)
    key, _ = torch.sort(key)
    merged_vals = (key & 0xFFFFFFFF).to(torch.int32)
    return merged_offs, merged_vals

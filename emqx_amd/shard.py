"""Multi-GPU modes of the match path.

Topic-sharded (C1-C3, C5): every rank holds a replica of the index and matches
its own contiguous slice of the topic stream; no data-path collective.

Filter-sharded (C4, filter sets beyond one GPU): rank r holds the keys whose
index is r mod N; every rank matches the same topic batch against its shard;
then the per-shard CSR hit lists are exchanged -- one allgather of the CSR
offsets (n+1 x u64 per rank) and one allgather of the values, each rank's
payload padded to the largest (an allgatherv; shards are balanced, so the
padding is a few percent) -- over RCCL/xGMI on GPUs (gloo on CPU), and merged
on the device by ``tm_merge_shards``: per topic, shard 0's values, then shard
1's, ...  Shards hold disjoint keys, so the merged list is the union: the same
value set as one index holding every key (the parity criterion of
BASELINE.json: "same filter-ID set per topic").
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def topic_slice(rank: int, world: int, batch: int) -> tuple[int, int]:
    """Topic-sharded mode: [first, first + batch) of the topic stream for `rank`."""
    return rank * batch, batch


def exchange(hit_offs: torch.Tensor, vals: torch.Tensor, group=None):
    """The collective half of the filter-sharded exchange.

    hit_offs: int64 [n+1] (this rank's CSR offsets, hit_offs[0] == 0),
    vals: int32 [>= hit_offs[n]].  Returns (all_offs int64 [world, n+1],
    all_vals int32 [world, stride], stride) identical on every rank.
    """
    world = dist.get_world_size(group)
    n1 = hit_offs.numel()
    dev = hit_offs.device
    all_offs = torch.empty(world * n1, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_offs, hit_offs.contiguous(), group=group)
    all_offs = all_offs.view(world, n1)
    stride = max(int(all_offs[:, -1].max().item()), 1)
    total = int(hit_offs[-1].item())
    if vals.numel() >= stride:
        send = vals[:stride].contiguous()
    else:
        send = torch.zeros(stride, dtype=torch.int32, device=dev)
        send[:total] = vals[:total]
    all_vals = torch.empty(world * stride, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(all_vals, send, group=group)
    return all_offs, all_vals.view(world, stride), stride


def merge(all_offs: torch.Tensor, all_vals: torch.Tensor, stride: int, stream: int | None = None):
    """The device half: tm_merge_shards on the gathered buffers (GPU only)."""
    from . import _native
    world, n1 = all_offs.shape
    n = n1 - 1
    out_hit = torch.empty(n1, dtype=torch.int64, device=all_offs.device)
    total = int(all_offs[:, -1].sum().item())
    out_vals = torch.empty(max(total, 1), dtype=torch.int32, device=all_offs.device)
    _native.merge_shards(world, n, all_offs.data_ptr(), all_vals.data_ptr(), stride, out_hit.data_ptr(),
                         out_vals.data_ptr(), total, stream)
    return out_hit, out_vals[:total]


def allgatherv_hits(hit_offs: torch.Tensor, vals: torch.Tensor, group=None, stream: int | None = None):
    """Exchange one rank's CSR hit lists with every rank and merge them on the device."""
    all_offs, all_vals, stride = exchange(hit_offs, vals, group)
    return merge(all_offs, all_vals, stride, stream)

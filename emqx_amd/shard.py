"""Multi-GPU modes of the match path.

Topic-sharded (C1-C3, C5): every rank holds a replica of the index and matches
its own contiguous slice of the topic stream; no data-path collective.

Filter-sharded (C4, filter sets beyond one GPU): rank r holds the keys whose
index is r mod N, and every rank matches the same topic batch against its
shard.  Topic slice q of the batch (topics [q s, (q+1) s), s = ceil(n / N))
belongs to rank q -- the publisher that handed those topics in -- so each
rank needs, for its own slice only, the hit lists of every shard:

  1. counts: all_to_all of per-topic hit counts (s x u32 per peer),
  2. values: all_to_all of each slice's values, padded to a per-peer capacity
     taken from the high-water mark of earlier batches (no host read of the
     sizes on the data path: an on-device running maximum says afterwards
     whether any slice overflowed the capacity, and the caller re-runs such a
     batch with a larger one),
  3. merge: per topic of the slice, shard 0's values, then shard 1's, ...
     (``tm_merge_shards`` on the device).

Over RCCL/xGMI on GPUs, gloo on CPU (tests).  Shards hold disjoint keys, so
the merged list is the union: the same value set as one index holding every
key (the parity criterion of BASELINE.json: "same filter-ID set per topic").
Every rank receives only its slice, so each value crosses xGMI once, not N-1
times as with an allgather of whole lists.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def topic_slice(rank: int, world: int, batch: int) -> tuple[int, int]:
    """Topic-sharded mode: [first, first + batch) of the topic stream for `rank`."""
    return rank * batch, batch


def slice_bounds(n: int, world: int) -> tuple[int, list[tuple[int, int]]]:
    """Filter-sharded mode: the slice length s and [lo, hi) of each rank's topic slice."""
    s = (n + world - 1) // world if n else 0
    return s, [(min(q * s, n), min((q + 1) * s, n)) for q in range(world)]


def pack_slices(hit: torch.Tensor, vals: torch.Tensor, world: int, per_peer: int):
    """Send side of the exchange (device ops only, no host read).

    hit: int64 [n+1] CSR offsets (hit[0] == 0), vals: int32 [>= hit[n]].
    -> (counts int32 [world, s], values int32 [world, per_peer], largest
    slice value count as a 0-d int64 tensor)."""
    n = hit.numel() - 1
    s, _ = slice_bounds(n, world)
    dev = hit.device
    c = torch.zeros(world * s, dtype=torch.int64, device=dev)
    c[:n] = hit[1:] - hit[:-1]
    # a slice that overflows per_peer ships its first per_peer values only, and
    # its counts are cut to match: the receiver's offsets (a scan of the
    # counts) stay inside the per_peer values it gets, so the merge never
    # reads past a peer's slot; check() reports the overflow and the caller
    # reruns the batch with a larger capacity
    c = c.view(world, s)
    start = torch.cumsum(c, dim=1) - c
    counts = torch.minimum(c, torch.clamp(per_peer - start, min=0)).to(torch.int32).view(-1)
    edges = torch.clamp(torch.arange(world + 1, device=dev, dtype=torch.int64) * s, max=n)
    bounds = hit[edges]                                    # slice q = vals[bounds[q] : bounds[q+1]]
    lens = bounds[1:] - bounds[:-1]
    idx = bounds[:-1, None] + torch.arange(per_peer, device=dev, dtype=torch.int64)[None, :]
    ok = idx < bounds[1:, None]
    src = vals[torch.clamp(idx, max=max(vals.numel() - 1, 0))] if vals.numel() else torch.zeros_like(idx, dtype=torch.int32)
    packed = torch.where(ok, src, torch.zeros((), dtype=torch.int32, device=dev))
    return counts.view(world, s), packed, lens.max()


def exchange_slices(counts: torch.Tensor, packed: torch.Tensor, group=None):
    """The collective half: all_to_all of counts and padded values.
    -> (recv_counts int32 [world, s]: shard q's counts for this rank's slice,
        recv_vals int32 [world, per_peer]: shard q's values for it)."""
    rc = torch.empty_like(counts)
    rv = torch.empty_like(packed)
    dist.all_to_all_single(rc.view(-1), counts.contiguous().view(-1), group=group)
    dist.all_to_all_single(rv.view(-1), packed.contiguous().view(-1), group=group)
    return rc, rv


def shard_offsets(recv_counts: torch.Tensor) -> torch.Tensor:
    """[world, s] counts -> [world, s+1] per-shard CSR offsets (device scan)."""
    w, s = recv_counts.shape
    offs = torch.zeros(w, s + 1, dtype=torch.int64, device=recv_counts.device)
    torch.cumsum(recv_counts.to(torch.int64), dim=1, out=offs[:, 1:])
    return offs


def merge(all_offs: torch.Tensor, all_vals: torch.Tensor, stride: int, cap: int | None = None,
          stream: int | None = None):
    """The device half: tm_merge_shards on the gathered buffers (GPU only).
    cap defaults to every value the shards could hold (no host read)."""
    from . import _native
    world, n1 = all_offs.shape
    n = n1 - 1
    out_hit = torch.empty(n1, dtype=torch.int64, device=all_offs.device)
    if cap is None:
        cap = world * stride
    out_vals = torch.empty(max(cap, 1), dtype=torch.int32, device=all_offs.device)
    _native.merge_shards(world, n, all_offs.data_ptr(), all_vals.data_ptr(), stride, out_hit.data_ptr(),
                         out_vals.data_ptr(), cap, stream)
    return out_hit, out_vals


def merge_local(hit: torch.Tensor, vals: torch.Tensor, stream: int | None = None):
    """One shard (world 1): the exchange is the identity, the merge still runs."""
    return merge(hit.view(1, -1), vals.view(1, -1), vals.numel(), vals.numel(), stream)


class Exchange:
    """Filter-sharded exchange of one rank for batches of n topics.

    ``run(hit, vals)`` packs this shard's lists by destination slice, swaps
    them with every rank and merges this rank's slice on the device; the
    per-peer value capacity starts at ``per_peer`` (or is sized by the first
    batch) and ``check()`` -- one host read, off the data path -- reports
    whether any batch since the last check overflowed it and grows it."""

    def __init__(self, n: int, device, per_peer: int = 0, group=None, headroom: float = 1.25):
        self.n = n
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.s, self.bounds = slice_bounds(n, self.world)
        self.per_peer = per_peer
        self.headroom = headroom
        self.peak = torch.zeros((), dtype=torch.int64, device=device)

    def size_from(self, hit: torch.Tensor):
        """Size the capacity from one batch's offsets (one host read; setup only)."""
        edges = torch.clamp(torch.arange(self.world + 1, device=hit.device, dtype=torch.int64) * self.s, max=self.n)
        b = hit[edges]
        m = (b[1:] - b[:-1]).max().view(1)
        if self.world > 1:
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        self.per_peer = max(int(int(m.item()) * self.headroom), self.per_peer, 1)

    def swap(self, hit: torch.Tensor, vals: torch.Tensor):
        """Pack + all_to_all (any device): -> (per-shard offsets int64 [world,
        s+1] and values int32 [world, per_peer] of this rank's slice)."""
        if self.per_peer <= 0:
            self.size_from(hit)
        counts, packed, mx = pack_slices(hit, vals, self.world, self.per_peer)
        torch.maximum(self.peak, mx, out=self.peak)
        rc, rv = exchange_slices(counts, packed, self.group)
        return shard_offsets(rc), rv

    def run(self, hit: torch.Tensor, vals: torch.Tensor, stream: int | None = None):
        """swap + the device merge of this rank's slice: -> (offsets int64
        [slice + 1], values int32) of topics [lo, hi) of the batch."""
        offs, rv = self.swap(hit, vals)
        lo, hi = self.bounds[self.rank]
        out_hit, out_vals = merge(offs, rv, self.per_peer, self.world * self.per_peer, stream)
        return out_hit[: hi - lo + 1], out_vals

    def check(self) -> bool:
        """True if every batch since the last check fitted; otherwise grow the
        capacity (the caller re-runs the batches it has not consumed)."""
        m = self.peak.view(1).clone()
        if self.world > 1:
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        peak = int(m.item())
        ok = peak <= self.per_peer
        if not ok:
            self.per_peer = int(peak * self.headroom) + 1
        self.peak.zero_()
        return ok


# ------------------------------------------------ level-0 filter sharding
#
# Filter-sharded by the first topic level.
# emqx_topic:match/2 compares a filter with a topic level by level
# (emqx_topic.erl:83-116), so a filter can match a topic only if its first
# level is '+' or '#' or equals the topic's first level.  Rank r therefore
# holds the filters whose first level is a word r owns plus every filter whose
# first level is '+' or '#' (replicated), and a topic is matched on ONE rank:
# the owner of its first level -- the host that receives the publish routes it
# there, as the broker routes by topic anyway.  Each GPU walks 1/N of the
# topics against 1/N of the literal-rooted filters, and its lists are complete
# and in the reference's traversal order (no merge, no data-path collective):
# the result equals one index over every filter element for element.
# Ownership is a deterministic balanced map (greedy by filter count over a
# sample every rank draws identically); words outside it go by CRC-32.

import zlib

import numpy as np


def level0_spans(blob: np.ndarray, offs: np.ndarray):
    """[start, end) of every item's first level (vectorised)."""
    starts = offs[:-1].astype(np.int64)
    ends = offs[1:].astype(np.int64)
    sl = np.flatnonzero(blob == ord("/"))
    j = np.searchsorted(sl, starts)
    first = np.where(j < len(sl), sl[np.minimum(j, max(len(sl) - 1, 0))] if len(sl) else ends, ends)
    return starts, np.minimum(first, ends)


def level0_keys(blob: np.ndarray, offs: np.ndarray):
    """Per item a u64 key of its first level (bytes packed little endian; MQTT
    topics hold no NUL, so zero padding is unambiguous) and a mask of items
    whose first level is longer than 8 bytes (keyed by the caller)."""
    s, e = level0_spans(blob, offs)
    ln = e - s
    key = np.zeros(len(s), np.uint64)
    for k in range(8):
        b = blob[np.minimum(s + k, len(blob) - 1)].astype(np.uint64)
        key |= np.where(ln > k, b, 0).astype(np.uint64) << np.uint64(8 * k)
    return key, ln > 8, s, e


def _mix(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over a u64 array (wrapping arithmetic)."""
    x = np.asarray(x, np.uint64).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def level1_info(blob: np.ndarray, offs: np.ndarray, e0: np.ndarray):
    """Per item, given the end e0 of its first level: whether it has a second
    level, whether that level is exactly '+' or '#', and a u64 hash of the
    second level's bytes (its first 16 bytes and its length)."""
    ends = offs[1:].astype(np.int64)
    has1 = e0 < ends
    b1 = np.minimum(e0 + 1, ends)
    sl = np.flatnonzero(blob == ord("/"))
    if len(sl):
        j = np.searchsorted(sl, b1)
        e1 = np.where(j < len(sl), sl[np.minimum(j, len(sl) - 1)], ends)
    else:
        e1 = ends
    e1 = np.minimum(e1, ends)
    ln = np.where(has1, e1 - b1, 0)
    top = len(blob) - 1
    first = blob[np.minimum(b1, top)]
    wild = has1 & (ln == 1) & ((first == ord("+")) | (first == ord("#")))
    ka = np.zeros(len(b1), np.uint64)
    kb = np.zeros(len(b1), np.uint64)
    for k in range(8):
        ka |= np.where(ln > k, blob[np.minimum(b1 + k, top)], 0).astype(np.uint64) << np.uint64(8 * k)
        kb |= np.where(ln > k + 8, blob[np.minimum(b1 + k + 8, top)], 0).astype(np.uint64) << np.uint64(8 * k)
    return has1, wild, _mix(ka ^ _mix(kb ^ ln.astype(np.uint64)))


def _word_key(w: bytes) -> int:
    return int.from_bytes(w.ljust(8, b"\0"), "little") if len(w) <= 8 else -1


def _word_counts(s, sample: int) -> dict:
    """First-level word -> occurrences among the first `sample` items of s."""
    n = min(len(s), sample)
    sub = s.slice(0, n) if n < len(s) else s
    key, long_, st, en = level0_keys(sub.blob, sub.offs)
    counts = {}
    u, c = np.unique(key[~long_], return_counts=True)
    for k, cnt in zip(u.tolist(), c.tolist()):
        counts[int(k).to_bytes(8, "little").rstrip(b"\0")] = cnt
    for i in np.flatnonzero(long_).tolist():
        w = sub.blob[st[i]:en[i]].tobytes()
        counts[w] = counts.get(w, 0) + 1
    return counts


class Level0Map:
    """Which rank owns each first-level word; '+' and '#' are everyone's.

    Without a publish sample the words are spread by filter count (greedy,
    heaviest first, onto the least loaded rank).  With one (`publish`: word ->
    publishes in a recent sample), a rank's time goes with the publishes routed
    to it -- each walks one shard -- so the words are spread by publish count
    instead, while no rank takes more than `mem_slack` x its share of the
    filters (its HBM): a hot tenant prefix no longer lands on a rank that
    already holds other busy words.  A word that alone carries more than 1/N
    of the publishes (one tenant prefix W) is split by its second level: the
    filters W/w1/... go to the rank of (W, w1), those whose second level is
    '+' or '#' (and W/#, which also matches the topic W) to every rank, the
    filter W itself to the rank of (W, -); a topic W/w1/... goes to the rank of
    (W, w1) and finds there every filter that can match it, so its list is
    still the unsharded one, order included."""

    PLUS, HASH = _word_key(b"+"), _word_key(b"#")

    def __init__(self, world: int, counts: dict, publish: dict | None = None, mem_slack: float = 1.25):
        self.world = world
        self.table = {}
        self.split = set()   # words split by their second level
        words = [w for w in counts if w not in (b"+", b"#")]
        if publish:
            words += [w for w in publish if w not in counts and w not in (b"+", b"#")]
            tot_p = sum(publish.get(w, 0) for w in words)
            if world > 1:
                self.split = {w for w in words if len(w) <= 8 and publish.get(w, 0) * world > tot_p}
            pload, fload = [0.0] * world, [0.0] * world
            for w in self.split:   # spread over every rank (second levels by hash)
                for q in range(world):
                    pload[q] += publish.get(w, 0) / world
                    fload[q] += counts.get(w, 0) / world
            words = [w for w in words if w not in self.split]
            tot_f = sum(fload) + sum(counts.get(w, 0) for w in words)
            cap = mem_slack * tot_f / world + max((counts.get(w, 0) for w in words), default=0)
            for w in sorted(words, key=lambda x: (-publish.get(x, 0), -counts.get(x, 0), x)):
                f = counts.get(w, 0)
                fit = [q for q in range(world) if fload[q] + f <= cap] or list(range(world))
                r = min(fit, key=lambda q: (pload[q], fload[q], q))
                self.table[w] = r
                pload[r] += publish.get(w, 0)
                fload[r] += f
        else:
            load = [0] * world
            for w in sorted(words, key=lambda x: (-counts[x], x)):
                r = min(range(world), key=lambda q: (load[q], q))
                self.table[w] = r
                load[r] += counts[w]
        self._split_keys = np.array(sorted(_word_key(w) for w in self.split), np.uint64)
        known = [(_word_key(w), r) for w, r in self.table.items() if len(w) <= 8]
        known.sort()
        self._keys = np.array([k for k, _ in known], np.uint64)
        self._ranks = np.array([r for _, r in known], np.int64)

    @classmethod
    def from_items(cls, world: int, s, sample: int = 1_000_000, topics=None, topic_sample: int = 1_000_000):
        """The map over the first `sample` items of a filter set and, when given,
        the first `topic_sample` of a recent publish sample (every rank must pass
        the same ones: the map is computed on each)."""
        pub = _word_counts(topics, topic_sample) if topics is not None else None
        return cls(world, _word_counts(s, sample), pub)

    def loads(self, s) -> np.ndarray:
        """Items of s each rank gets (routed by first level; '+'/'#' roots count on every rank)."""
        o = self.owners(s)
        return np.bincount(o[o >= 0], minlength=self.world) + int((o == -1).sum())

    def owner_of_word(self, w: bytes) -> int:
        r = self.table.get(w)
        return r if r is not None else zlib.crc32(w) % self.world

    def owners(self, s) -> np.ndarray:
        """Per item: its owner, or -1 (every rank): a '+' / '#' first level, or a
        '+' / '#' second level under a split word."""
        key, long_, st, en = level0_keys(s.blob, s.offs)
        out = np.empty(len(key), np.int64)
        if len(self._keys):
            j = np.minimum(np.searchsorted(self._keys, key), len(self._keys) - 1)
            hit = self._keys[j] == key
        else:
            j = np.zeros(len(key), np.int64)
            hit = np.zeros(len(key), bool)
        out[:] = np.where(hit, self._ranks[j] if len(self._ranks) else 0, 0)
        wild = ((key == np.uint64(self.PLUS)) | (key == np.uint64(self.HASH))) & ~long_
        out[wild] = -1
        miss = np.flatnonzero(~hit & ~wild)
        for i in miss.tolist():
            out[i] = self.owner_of_word(s.blob[st[i]:en[i]].tobytes())
        if len(self._split_keys):
            j = np.minimum(np.searchsorted(self._split_keys, key), len(self._split_keys) - 1)
            hot = np.flatnonzero((self._split_keys[j] == key) & ~long_)
            if len(hot):
                has1, wild, h = level1_info(s.blob, s.offs, en)
                kk = key[hot]
                w = np.uint64(self.world)
                r1 = (_mix(h[hot] ^ _mix(kk)) % w).astype(np.int64)
                r0 = (_mix(kk ^ np.uint64(0x9E3779B97F4A7C15)) % w).astype(np.int64)
                out[hot] = np.where(~has1[hot], r0, np.where(wild[hot], -1, r1))
        return out

    def filter_rows(self, s, rank: int) -> np.ndarray:
        """Indices of the filters rank `rank` holds (its words + the replicated roots)."""
        o = self.owners(s)
        return np.flatnonzero((o == rank) | (o == -1))

    def topic_rows(self, s, rank: int) -> np.ndarray:
        """Indices of the topics rank `rank` matches (a topic whose first or
        split second level is '+' / '#' -- badarg -- goes to rank 0)."""
        o = self.owners(s)
        return np.flatnonzero(np.where(o < 0, 0, o) == rank)

"""world_size-2 gloo tests of the multi-GPU modes on CPU.

The filter-sharded exchange (emqx_amd.shard.Exchange.swap: all_to_all of the
per-topic u32 counts and of each topic slice's values, padded to a per-peer
capacity with an on-device overflow check) runs exactly as on GPUs, only over
gloo; the per-shard hit lists come from the CPU oracle here (the test's
stand-in for each rank's GPU shard) and the device merge (tm_merge_shards) is
restated in numpy (`_merge_ref`, the kernel's contract; the kernel itself is
checked against it in tests/test_gpu_parity.py).  Each rank's merged slice
must equal the oracle over the unsharded filter set, as per-topic value sets.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _body(rank, world, q)
    except BaseException as e:  # surface worker failures instead of a queue timeout
        q.put((rank, "error", repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def _merge_ref(all_offs, all_vals):
    """numpy restatement of tm_merge_shards: per topic, shard 0's values, then shard 1's, ..."""
    world, n1 = all_offs.shape
    n = n1 - 1
    out_hit = all_offs.sum(axis=0)
    out = []
    for t in range(n):
        for r in range(world):
            out.append(all_vals[r, all_offs[r, t]:all_offs[r, t + 1]])
    return out_hit, (np.concatenate(out) if out else np.zeros(0, np.int32))


def _body(rank, world, q):
    from emqx_amd import shard, workload as wl
    from pyoracle import Oracle
    nf = 20_000
    n = 3_001                       # not a multiple of the world: a short last slice
    fs = wl.filters(3, nf, shard=rank, nshards=world)
    ts = wl.topics(3, nf, n)
    o = Oracle()
    o.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    cnt, _, hit, vals = o.match_batch(ts.blob, ts.offs)
    hit_t = torch.from_numpy(hit.astype(np.int64))
    vals_t = torch.from_numpy(vals.view(np.int32).copy())
    # a capacity far too small first: the overflow check must catch it and grow
    xch = shard.Exchange(n, "cpu", per_peer=8)
    o_offs, o_rv = xch.swap(hit_t, vals_t)
    # an overflowing slice ships cut counts: the merge stays inside each peer's values
    assert int(o_offs[:, -1].max()) <= 8 and o_rv.shape[1] == 8
    overflowed = not xch.check()
    offs, rv = xch.swap(hit_t, vals_t)
    fitted = xch.check()
    m_offs, m_vals = _merge_ref(offs.numpy(), rv.numpy())
    lo, hi = xch.bounds[rank]
    # topic-sharded slices partition the stream
    first, nn = shard.topic_slice(rank, world, 1000)
    t = torch.tensor([first, nn], dtype=torch.int64)
    g = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(g, t)
    # max-over-ranks timing reduction used by bench.py
    el = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    q.put((rank, m_offs[: hi - lo + 1], m_vals, [x.tolist() for x in g], float(el), (lo, hi), overflowed, fitted))


@pytest.mark.timeout(300)
def test_filter_sharded_exchange_gloo():
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "oracle"))
    from emqx_amd import workload as wl
    from pyoracle import Oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for r in res:
        assert not (isinstance(r[1], str) and r[1] == "error"), r
    # the slices partition the batch; capacity overflow detected, then fitted
    n = 3_001
    assert [r[5] for r in res] == [(0, 1501), (1501, 3001)]
    assert all(r[6] and r[7] for r in res)
    # each rank's merged slice == the unsharded oracle, per topic as sorted sets
    nf = 20_000
    fs = wl.filters(3, nf)
    ts = wl.topics(3, nf, n)
    o = Oracle()
    o.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    cnt, _, hit, vals = o.match_batch(ts.blob, ts.offs)
    for r in res:
        lo, hi = r[5]
        m_offs, m_vals = r[1], r[2].view(np.uint32)
        assert np.array_equal(m_offs, hit[lo:hi + 1].astype(np.int64) - int(hit[lo]))
        for i in range(lo, hi):
            assert np.array_equal(np.sort(vals[hit[i]:hit[i + 1]]),
                                  np.sort(m_vals[m_offs[i - lo]:m_offs[i - lo + 1]]))
    assert res[0][3] == [[0, 1000], [1000, 1000]]
    assert res[0][4] == 1.5


# ---------------------------------------------------- level-0 filter sharding

def _l0_worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emqx_amd import shard, workload as wl
        from pyoracle import Oracle
        nf, n = 20_000, 4_000
        fs = wl.filters(3, nf)
        ts = wl.topics(3, nf, n)
        m = shard.Level0Map.from_items(world, fs, sample=5_000)   # every rank draws the same map
        mine = wl.take(fs, m.filter_rows(fs, rank))
        rows = m.topic_rows(ts, rank)
        o = Oracle()   # this rank's shard (the GPU index on a GPU box)
        o.apply(np.ones(len(mine), np.uint8), mine.blob, mine.offs, mine.vals)
        sub = wl.take(ts, rows)
        cnt, _, hit, vals = o.match_batch(sub.blob, sub.offs)
        # every topic is matched on exactly one rank
        c = torch.tensor([len(rows)], dtype=torch.int64)
        dist.all_reduce(c)
        q.put((rank, rows, hit, vals, len(mine), int(c)))
    except BaseException as e:
        q.put((rank, "error", repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_level0_sharding_gloo():
    """Each rank holds its first-level words' filters plus the '+'/'#'-rooted
    ones and matches only the topics whose first level it owns: the union of
    the ranks' lists equals the unsharded oracle's, order included."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "oracle"))
    from emqx_amd import workload as wl
    from pyoracle import Oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_l0_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for r in res:
        assert not (isinstance(r[1], str) and r[1] == "error"), r
    nf, n = 20_000, 4_000
    fs = wl.filters(3, nf)
    ts = wl.topics(3, nf, n)
    o = Oracle()
    o.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    _, _, hit, vals = o.match_batch(ts.blob, ts.offs)
    seen = np.zeros(n, np.int64)
    for rank, rows, rhit, rvals, nkeys, total in res:
        assert total == n
        assert nkeys < len(fs)                       # a shard, not a replica
        seen[rows] += 1
        for k, t in enumerate(rows.tolist()):
            assert np.array_equal(rvals[rhit[k]:rhit[k + 1]], vals[hit[t]:hit[t + 1]]), (rank, t)
    assert (seen == 1).all()
    assert sum(r[4] for r in res) < 2 * len(fs)


def test_level0_map_is_deterministic_and_wild_roots_replicate():
    from emqx_amd import shard, workload as wl
    fs = wl.filters(3, 50_000)
    a = shard.Level0Map.from_items(4, fs, sample=10_000)
    b = shard.Level0Map.from_items(4, fs, sample=10_000)
    assert a.table == b.table
    own = a.owners(fs)
    for i in np.flatnonzero(own == -1)[:50].tolist():
        assert fs.item(i).split(b"/")[0] in (b"+", b"#")
    for i in np.flatnonzero(own >= 0)[:200].tolist():
        w = fs.item(i).split(b"/")[0]
        assert w not in (b"+", b"#") and own[i] == a.owner_of_word(w)
    # words the sample never saw (and long words) still get a fixed owner
    assert a.owner_of_word(b"never-seen-level-zero-word") == b.owner_of_word(b"never-seen-level-zero-word")
    # balanced: no rank owns more than 1.5x its share of the literal-rooted filters
    cnt = np.bincount(own[own >= 0], minlength=4)
    assert cnt.max() <= 1.5 * cnt.sum() / 4


def test_level0_map_balances_publish_load():
    """With a publish sample the first-level words are spread by publish count
    under a per-rank filter cap: a hot tenant prefix gets a rank to itself
    instead of sharing one with other words picked by filter count."""
    from emqx_amd import shard
    words = [b"w%02d" % i for i in range(16)]
    counts = {w: 1000 for w in words}                       # filters: uniform
    publish = {w: 100 for w in words}
    publish[words[0]] = 450                                 # 23 % of the publishes on one word (< 1/4: not split)
    by_f = shard.Level0Map(4, counts)
    by_p = shard.Level0Map(4, counts, publish)
    assert not by_p.split

    def rank_loads(m, weights):
        out = [0] * 4
        for w in words:
            out[m.table[w]] += weights[w]
        return out
    hot_f = rank_loads(by_f, publish)[by_f.table[words[0]]]
    hot_p = rank_loads(by_p, publish)[by_p.table[words[0]]]
    assert hot_f == 450 + 3 * 100 and hot_p == 450          # the hot word's rank holds nothing else busy
    fl = rank_loads(by_p, counts)
    assert max(fl) <= 1.25 * sum(fl) / 4 + 1000             # HBM per rank stays within the cap
    assert sorted(by_p.table) == sorted(words)
    # every rank computes the same map from the same samples
    assert shard.Level0Map(4, counts, publish).table == by_p.table
    # past 1/N of the publishes a word is split by its second level instead
    publish[words[0]] = 4000
    assert shard.Level0Map(4, counts, publish).split == {words[0]}


def test_level0_split_hot_prefix_equals_one_index():
    """One tenant prefix carrying most publishes is split by its second level
    (filters under it by (prefix, second word), its '+'/'#' second levels on
    every rank): each rank's lists for the topics routed to it equal the
    unsharded index's, order included, and the hot topics spread over the
    ranks instead of landing on one."""
    import random
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
    from pyoracle import Oracle
    from emqx_amd import _native, shard, workload as wl
    r = random.Random(0x454D5158 + 901)
    base = wl.filters(1, 3_000)
    hot = []
    for i in range(1500):
        d = b"d%d" % r.randrange(400)
        hot.append(r.choice([b"tnt/%s/+/x" % d, b"tnt/%s/#" % d, b"tnt/%s/s/%d" % (d, i % 7), b"tnt/%s" % d]))
    hot += [b"tnt", b"tnt/#", b"tnt/+/s/#", b"tnt/+", b"tnt/", b"tnt//x", b"+/+/s/#", b"#"]
    items = base.items() + hot
    blob, offs = _native.pack_strings(items)
    fs = wl.ItemSet(blob, offs, np.arange(len(items), dtype=np.uint32), np.zeros(len(items), np.uint8))
    tl = [b"tnt/d%d/%s" % (r.randrange(400), r.choice([b"a/x", b"s/3", b"s", b"q/w/e"])) for _ in range(3000)]
    tl += [b"tnt", b"tnt/", b"tnt//x", b"tnt/d1"] + wl.topics(1, 3_000, 1000).items()
    tb, to = _native.pack_strings(tl)
    ts = wl.ItemSet(tb, to, np.zeros(len(tl), np.uint32), np.zeros(len(tl), np.uint8))
    world = 4
    m = shard.Level0Map.from_items(world, fs, topics=ts)
    assert b"tnt" in m.split
    full = Oracle()
    full.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    _, _, fh, fv = full.match_batch(ts.blob, ts.offs)
    per_rank = []
    for rank in range(world):
        rows = m.filter_rows(fs, rank)
        sub = wl.take(fs, rows)
        o = Oracle()
        o.apply(np.ones(len(sub), np.uint8), sub.blob, sub.offs, sub.vals)
        trows = m.topic_rows(ts, rank)
        per_rank.append(len(trows))
        tsub = wl.take(ts, trows)
        _, _, h, v = o.match_batch(tsub.blob, tsub.offs)
        for j, i in enumerate(trows.tolist()):
            assert np.array_equal(v[h[j]:h[j + 1]], fv[fh[i]:fh[i + 1]]), tl[i]
    assert sum(per_rank) == len(tl)
    assert max(per_rank) <= 1.4 * len(tl) / world, per_rank   # the hot prefix spread, not on one rank

"""GPU parity: the MI355X path (libtmatch through its C ABI) against the CPU
oracle (the reference's walk restated) and the reference's known answers.

Integer/byte work: the bar is bit-exact -- the same values per topic in the
same (traversal) order, the same badarg flags.
"""
import random

import numpy as np
import pytest

from emqx_amd import _native, router as rt, topic_index as ti, workload as wl
from emqx_amd.trie_search import BadArg, get_id, get_topic, topic_words
from harness import GOLDEN, RouterModel, case_keys, encode_key, run_checks
from pyoracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


def _small_kind(kind: str) -> int:
    """TM_DEBUG_SMALL_KERNEL value of a small-batch kernel name"""
    return {"auto": _native.SMALL_AUTO, "wave": _native.SMALL_WAVE, "wave8": _native.SMALL_WAVE8}[kind]


def gpu_index(items: wl.ItemSet | None = None, flags=None) -> _native.Index:
    ix = _native.Index()
    if items is not None and len(items):
        ix.apply(np.ones(len(items), np.uint8), items.blob, items.offs, items.vals, flags)
    return ix


def oracle_of(items: wl.ItemSet, flags=None) -> Oracle:
    o = Oracle()
    o.apply(np.ones(len(items), np.uint8), items.blob, items.offs, items.vals, flags)
    o.prepare()
    return o


def assert_same(ix: _native.Index, o: Oracle, topics: wl.ItemSet):
    hit, vals, err = ix.match_batch(topics.blob, topics.offs)
    cnt, _, ohit, ovals = o.match_batch(topics.blob, topics.offs)
    assert np.array_equal(err.astype(np.int64), np.where(cnt < 0, -cnt, 0)), "badarg / too-deep flags differ"
    gcnt = np.diff(hit.astype(np.int64))
    bad = np.nonzero(gcnt != np.maximum(cnt, 0))[0]
    assert len(bad) == 0, f"{len(bad)} topics differ in hit count, first {topics.item(int(bad[0]))!r}: " \
                          f"gpu {gcnt[bad[0]]} oracle {cnt[bad[0]]}"
    assert np.array_equal(vals, ovals), "hit values / order differ"
    return hit, vals


def items_of(strings, vals=None) -> wl.ItemSet:
    blob, offs = _native.pack_strings(strings)
    v = np.arange(len(strings), dtype=np.uint32) if vals is None else np.asarray(vals, np.uint32)
    return wl.ItemSet(blob, offs, v, np.zeros(len(strings), np.uint8))


# ------------------------------------------------------------ known answers

@pytest.mark.parametrize("case", GOLDEN["index_cases"], ids=lambda c: c["name"])
def test_golden_native(torch_dev, case):
    keys, kid = case_keys(case)
    ix = _native.Index()
    by_kid = {v: k for k, v in kid.items()}
    if keys:
        enc = [encode_key(k) for k in keys]
        blob, offs = _native.pack_strings([e[0] for e in enc])
        ix.apply(np.ones(len(keys), np.uint8), blob, offs, np.array([kid[k] for k in keys], np.uint32),
                 np.array([e[1] for e in enc], np.uint8))

    def traversal(t):
        blob, offs = _native.pack_strings([t])
        hit, vals, err = ix.match_batch(blob, offs)
        if err[0]:
            raise BadArg(t)
        return [by_kid[int(v)] for v in vals]

    run_checks(case, traversal)


@pytest.mark.parametrize("case", GOLDEN["index_cases"], ids=lambda c: c["name"])
def test_golden_topic_index_api(torch_dev, case):
    tab = ti.new()
    from emqx_amd.trie_search import filter as tfilter
    for ins in case["inserts"]:
        f = ins[0].encode()
        words = len(ins) > 2 and ins[2].get("words")
        ti.insert(tfilter(f) if words else f, ins[1], b"", tab)
    for chk in case["checks"]:
        t = chk["topic"].encode()
        if chk["kind"] == "badarg":
            with pytest.raises(BadArg):
                ti.match(t, tab)
            continue
        if chk["kind"] == "match":
            m = ti.match(t, tab)
            got = False if m is False else [get_topic(m).decode(), get_id(m)]
            assert got == chk["expect"]
            if m is False:      # matches/3 with [return_first]: the atom `first`, or a throw
                assert ti.matches(t, tab, ["return_first"]) == ti.FIRST
            else:
                with pytest.raises(ti.FirstHit) as e:
                    ti.matches(t, tab, ["return_first"])
                assert e.value.key == m
        elif chk["kind"] == "match_id":
            assert get_id(ti.match(t, tab)) == chk["expect"]
        elif chk["kind"] == "sorted_topics":
            ms = sorted(ti.matches(t, tab, []), key=ti.key_order)
            assert [get_topic(k).decode() for k in ms] == chk["expect"]
        elif chk["kind"] == "ids":
            assert [get_id(k) for k in ti.matches(t, tab, chk["opts"])] == chk["expect"]
        elif chk["kind"] == "count":
            assert len(ti.matches(t, tab, [])) == chk["expect"]


@pytest.mark.parametrize("case", GOLDEN["router_cases"], ids=lambda c: c["name"])
def test_router_known_answers(torch_dev, case):
    r = rt.Router(node="node")
    for st in case["steps"]:
        if "add" in st:
            r.add_route(st["add"][0].encode(), st["add"][1])
        elif "delete" in st:
            r.delete_route(st["delete"][0].encode(), st["delete"][1])
        elif "match_routes_sorted" in st:
            got = sorted(r.match_routes(st["match_routes_sorted"].encode()), key=rt.route_order)
            assert [[x.topic.decode(), x.dest] for x in got] == st["expect"]
        elif "topics_sorted" in st:
            assert sorted(t.decode() for t in r.topics()) == st["topics_sorted"]


# ---------------------------------------------------------- random vs oracle

def _rand_level(r):
    c = r.random()
    if c < 0.15:
        return r.choice([b"foo", b"bar", b"baz", b"xyzzy"])
    if c < 0.22:
        return b""
    if c < 0.27:
        return b"$" + r.choice([b"SYS", b"a", b""])
    if c < 0.30:
        return r.choice([b"b+", b"c#", b"+x", b"#y", b"a-very-long-level-word-over-16-bytes"])
    return ("%X" % r.randint(1, 16)).encode()


def _rand_filter(r, levels):
    out = []
    for lvl in levels:
        p = r.choices(["level", "+", "#"], [5, 2, 1])[0]
        if p == "#":
            out.append(b"#")
            break
        out.append(b"+" if p == "+" else lvl)
    return b"/".join(out)


@pytest.mark.parametrize("seed", range(24))
def test_random_sets_vs_oracle(torch_dev, seed):
    """Random filter and topic sets (empty levels, '$' levels, words with '+'/'#'
    inside, long words, word-list keys), through the one-launch path (a few
    hundred topics) and the lane walk (> 64k topics), the first hit, and after
    deletes and re-inserts."""
    r = random.Random(0x454D5158 + 100 + seed)
    topics = [b"/".join(_rand_level(r) for _ in range(r.randint(1, 12))) for _ in range(400)]
    topics += [b"a/+/b", b"#", b"", b"/", b"$SYS", b"$"]
    filters = []
    for _ in range(500):
        base = r.choice(topics).split(b"/")
        filters.append(_rand_filter(r, [_rand_level(r) if r.random() < 0.3 else w for w in base]))
    flags = np.array([r.random() < 0.2 for _ in filters], np.uint8)   # some word-list keys
    fs = items_of(filters)
    ix = gpu_index(fs, flags)
    o = oracle_of(fs, flags)
    ts = items_of(topics)
    assert_same(ix, o, ts)
    big = items_of(topics * (66_000 // len(topics) + 1))        # > 64k topics: lane walk + tail kernels
    assert_same(ix, o, big)
    first, found = ix.first_batch(ts.blob, ts.offs)
    cnt, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    assert np.array_equal(found == 2, cnt < 0)                   # badarg
    for i in np.nonzero(cnt > 0)[0]:
        assert found[i] == 1 and first[i] == ovals[ohit[i]]
    # deletes (and re-inserts) as deltas, then match again
    dele = sorted(r.sample(range(len(filters)), 150))
    ops = np.zeros(len(dele), np.uint8)
    d = items_of([filters[i] for i in dele], dele)
    ix.apply(ops, d.blob, d.offs, d.vals, flags[dele])
    o.apply(ops, d.blob, d.offs, d.vals, flags[dele])
    assert_same(ix, o, ts)
    back = dele[::3]
    d2 = items_of([filters[i] for i in back], back)
    ix.apply(np.ones(len(back), np.uint8), d2.blob, d2.offs, d2.vals, flags[back])
    o.apply(np.ones(len(back), np.uint8), d2.blob, d2.offs, d2.vals, flags[back])
    assert_same(ix, o, ts)


# ------------------------------------------------------------- configs

def test_c1_full_vs_oracle(torch_dev):
    fs = wl.filters(1, 10_000)
    ts = wl.topics(1, 10_000, 100_000)
    hit, _ = assert_same(gpu_index(fs), oracle_of(fs), ts)
    assert hit[-1] > 100_000  # instantiated topics all hit at least once


@pytest.mark.parametrize("cfg", [2, 20])
def test_c2_reduced_vs_oracle(torch_dev, cfg):
    fs = wl.filters(cfg, 50_000)
    ts = wl.topics(cfg, 50_000, 50_000)
    hit, _ = assert_same(gpu_index(fs), oracle_of(fs), ts)
    per = np.diff(hit.astype(np.int64))
    if cfg == 2:
        assert per.min() >= 1000 and per.max() == 1001
    else:
        assert per.max() <= 1


def test_c3_reduced_vs_oracle(torch_dev):
    fs = wl.filters(3, 200_000)
    ts = wl.topics(3, 200_000, 100_000)
    assert_same(gpu_index(fs), oracle_of(fs), ts)


def test_c5_churn_replay_vs_oracle(torch_dev):
    nf = 20_000
    fs = wl.filters(5, nf)
    ix, o = gpu_index(fs), oracle_of(fs)
    ts = wl.topics(5, nf, 20_000)
    step = 2_000
    for k in range(5):
        d = wl.deltas(nf, k * step, step)
        ix.apply(d.flags, d.blob, d.offs, d.vals)
        o.apply(d.flags, d.blob, d.offs, d.vals)
        assert_same(ix, o, ts)


# ------------------------------------------------------------- edge cases

def test_deep_topics_and_overflow(torch_dev):
    letters = [chr(ord("a") + i).encode() for i in range(26)]
    T = b"/".join(letters)                                  # 26 levels (mid path)
    deep = b"/".join(b"l%d" % i for i in range(300))        # deep path
    filters = [b"#", T + b"/#", T + b"/+", b"+/" * 26 + b"#", b"a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#",
               deep, deep + b"/#", b"l0/+/#", b"+/l1/#", deep.rsplit(b"/", 1)[0] + b"/+",
               b"a/#", b"+/#", b"+/+/#", b"a/b/#", b"+/b/#", b"a/+/#", b"a/b/+", b"+/+", b"a/+", b"+/b",
               b"a/b", b"#", b"+/+/+/#"]
    topics = [T, T + b"/1", deep, deep + b"/x", b"a/b", b"a/b/c", b"l0/l1", b"/".join([b"w"] * 1000),
              b"/".join([b"+"] * 40), T + b"/#"]
    fs = items_of(filters)
    ix, o = gpu_index(fs), oracle_of(fs)
    hit, _ = assert_same(ix, o, items_of(topics))
    assert np.diff(hit.astype(np.int64))[4] > 8      # 'a/b' overflows the RCAP ranges


def test_tail_grids_sized_from_the_last_batch(torch_dev):
    """The tail kernels' grids follow the list lengths of the last count-mode
    batch on the workspace (tail_blocks): a batch whose deep / overflow lists
    are far longer than the last one's walks them grid-stride with the small
    grid, and a shallow batch after it runs on the large one -- exact CSR vs
    the oracle each time (70k-topic batches: lane walk + tail kernels)."""
    letters = [chr(ord("a") + i).encode() for i in range(26)]
    T = b"/".join(letters)
    filters = [b"#", T + b"/#", T + b"/+", b"+/" * 26 + b"#", b"a/#", b"+/#", b"+/+/#", b"a/b/#", b"+/b/#",
               b"a/+/#", b"a/b/+", b"+/+", b"a/+", b"+/b", b"a/b", b"+/+/+/#", b"/".join(letters[:12]) + b"/#"]
    fs = items_of(filters)
    ix, o = gpu_index(fs), oracle_of(fs)
    r = random.Random(11)
    shallow = items_of([b"%s/%s" % (r.choice(letters), r.choice(letters)) for _ in range(70_000)])
    heavy = items_of([r.choice([T, T + b"/1", b"/".join(letters[:12]), b"/".join(letters[:20]), b"a/b", b"a/b/c"])
                      for _ in range(70_000)])
    for ts in (shallow, heavy, heavy, shallow, heavy):
        assert_same(ix, o, ts)


def test_c3deep_reduced_vs_oracle(torch_dev):
    """C3 filters with 10 % of the topics extended to 33-64 levels (cfg 30):
    the deep topics resolve only the levels the 6-level trie can use and stay
    on the main walk; exact CSR vs the oracle."""
    fs = wl.filters(3, 200_000)
    ts = wl.topics(30, 200_000, 60_000)
    assert max(len(t.split(b"/")) for t in ts.items()) > 32
    assert_same(gpu_index(fs), oracle_of(fs), ts)
    # with a binary key as deep as some topics, those topics resolve every level
    extra = items_of([t for t in ts.items() if len(t.split(b"/")) in (40, 64)][:50], [900_000 + i for i in range(50)])
    both = wl.ItemSet(*_native.pack_strings(fs.items() + extra.items()), np.concatenate([fs.vals, extra.vals]),
                      np.zeros(len(fs) + len(extra), np.uint8))
    assert_same(gpu_index(both), oracle_of(both), ts)


@pytest.mark.parametrize("batch", [3000, 40_000, 70_000])   # one launch (<= 64k topics) / lane walk + tails
def test_levels_beyond_the_trie(torch_dev, batch):
    """Topics deeper than every filter: badarg at any depth, '$' first levels,
    long words past the trie, binary keys of 3, 20 and 70 levels, '#'
    filters at the trie's bottom -- all against the oracle, in both walks."""
    r = random.Random(3)
    words = [b"a", b"b", b"c", b"$x", b"longer-than-eight-bytes", b""]
    filters = [b"a/+/#", b"+/b", b"a/b/c", b"#", b"+/+/+/#", b"$x/#", b"a/longer-than-eight-bytes/#"]
    keys20 = b"/".join([b"a"] * 20)
    keys70 = b"/".join([b"b"] * 70)
    filters += [keys20, keys70, b"c/c/c"]
    topics = []
    for _ in range(batch):
        L = r.choice([1, 2, 3, 4, 9, 20, 33, 40, 70, 100])
        ws = [r.choice(words) for _ in range(L)]
        if r.random() < 0.05:
            ws[r.randrange(L)] = r.choice([b"+", b"#"])
        topics.append(b"/".join(ws))
    topics += [keys20, keys70, keys70 + b"/b", b"/".join([b"a"] * 19), b"c/c/c", b"$x/" + b"/".join([b"a"] * 50)]
    fs = items_of(filters)
    assert_same(gpu_index(fs), oracle_of(fs), items_of(topics))


def test_maximum_size_topics(torch_dev):
    """Topics at MQTT's 65535-byte maximum (emqx_mqtt.hrl:44): one 65535-byte
    word, 32768 one-byte levels, 65536 empty levels (the walk's scratch depth),
    and one level more than that -- err flag 2 / found 3 on the device, -2 in
    the oracle, TopicTooDeep from the mirror (include/tmatch.h)."""
    big = b"x" * 65535
    many = b"/".join([b"a"] * 32768)                       # 65535 bytes, 32768 levels
    empty = b"/" * 65535                                    # 65536 empty levels
    over = b"/" * 65536                                     # 65537 levels
    filters = [big, big + b"/#", b"+", b"#", b"+/#", b"a/#", many, b"/".join([b"+"] * 32768),
               b"/".join([b"+"] * 32767) + b"/#", empty, b"/#", b"+/+/#", many[:-2] + b"/+", b"x/#"]
    topics = [big, big[:-1], many, many[:-2], empty, over, over + b"a", b"+/" + over, over + b"/+",
              b"/".join([b"a"] * 40000)]
    fs = items_of(filters)
    ix, o = gpu_index(fs), oracle_of(fs)
    assert_same(ix, o, items_of(topics))
    hit, vals, err = ix.match_batch(*_native.pack_strings(topics))
    assert err.tolist() == [0, 0, 0, 0, 0, 2, 2, 1, 2, 0]
    assert hit[6] == hit[5] and hit[9] == hit[8]
    val, found = ix.first_batch(*_native.pack_strings(topics))
    assert found.tolist()[5:9] == [3, 3, 2, 3]
    tab = ti.new()
    for i, f in enumerate(filters):
        ti.insert(f, i, None, tab)
    assert ti.matches(big, tab) and ti.matches(empty, tab)
    with pytest.raises(ti.TopicTooDeep):
        ti.matches(over, tab)


def test_edge_topics(torch_dev):
    long_word = b"x" * 40
    filters = [b"", b"/", b"+", b"#", b"$SYS/#", b"$/+", b"+/+", long_word, long_word + b"/+",
               b"/".join([b"e"] * 12), b"/".join([b"e"] * 12) + b"/#", b"\xff\x00/+", b"a/b\x00c",
               b"$share/g/t/+", b"t/+"]
    topics = [b"", b"/", b"//", b"$", b"$SYS", b"$SYS/x", b"$/a", long_word, long_word + b"/y",
              b"/".join([b"e"] * 12), b"\xff\x00/z", b"a/b\x00c", b"a/b", b"+", b"a/#", b"t/1",
              b"$share/g/t/1"]
    fs = items_of(filters)
    fl = np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0], np.uint8)
    assert_same(gpu_index(fs, fl), oracle_of(fs, fl), items_of(topics))


def test_empty_batch_and_index(torch_dev):
    ix = gpu_index()
    hit, vals, err = ix.match_batch(*_native.pack_strings([]))
    assert hit.tolist() == [0] and len(vals) == 0
    hit, vals, err = ix.match_batch(*_native.pack_strings([b"a/b", b"#"]))
    assert hit.tolist() == [0, 0, 0] and err.tolist() == [0, 1]


def test_first_batch_vs_oracle(torch_dev):
    fs = wl.filters(3, 50_000)
    ts = wl.topics(3, 50_000, 20_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    val, found = ix.first_batch(ts.blob, ts.offs)
    for i in range(0, len(ts), 7):
        r, v = o.first(ts.item(i))
        exp = {-1: 2, 0: 0, 1: 1}[r]
        assert found[i] == exp, ts.item(i)
        if r == 1:
            assert val[i] == v


def test_device_api_with_torch_stream(torch_dev):
    torch = torch_dev
    fs = wl.filters(3, 50_000)
    ts = wl.topics(3, 50_000, 30_000)
    ix = gpu_index(fs)
    ref_hit, ref_vals, _ = ix.match_batch(ts.blob, ts.offs)
    dev = torch.device("cuda:0")
    blob = torch.from_numpy(ts.blob).to(dev)
    offs = torch.from_numpy(ts.offs.view(np.int64)).to(dev)
    n = len(ts)
    hit = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    cap = int(ref_hit[-1])
    out = torch.zeros(cap, dtype=torch.int32, device=dev)
    err = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ix.match_batch_dev(n, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), out.data_ptr(), cap, err.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(hit.cpu().numpy().view(np.uint64), ref_hit)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref_vals)
    # capacity too small: values beyond cap are dropped, total still reported
    out2 = torch.zeros(10, dtype=torch.int32, device=dev)
    ix.match_batch_dev(n, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), out2.data_ptr(), 10, err.data_ptr(), s)
    torch.cuda.synchronize()
    assert int(hit[-1]) == cap
    assert np.array_equal(out2.cpu().numpy().view(np.uint32), ref_vals[:10])


def test_stats_and_idempotence(torch_dev):
    ix = gpu_index()
    d = items_of([b"a/+", b"a/+", b"a/b", b"a/#/b", b"x"], [1, 1, 2, 3, 4])
    ix.apply(np.ones(5, np.uint8), d.blob, d.offs, d.vals)
    st = ix.stats()
    assert (st["n_wild_keys"], st["n_exact_keys"], st["n_dead_keys"]) == (1, 2, 1)
    ix.apply(np.zeros(5, np.uint8), d.blob, d.offs, d.vals)
    missing = items_of([b"never/there", b"never/+"])
    ix.apply(np.zeros(2, np.uint8), missing.blob, missing.offs, missing.vals)   # not an error
    st = ix.stats()
    assert st["n_keys"] == 0 and st["n_nodes"] == 1 and st["n_edges"] == 0
    hit, vals, err = ix.match_batch(*_native.pack_strings([b"a/b", b"x"]))
    assert hit.tolist() == [0, 0, 0]


def test_churn_through_unique_words_stays_bounded(torch_dev):
    """Subscription churn with unique levels (client ids, UUIDs): words nothing
    refers to any more are erased from the vocab, long words' bytes and long
    exact keys' wid runs are compacted, the tables shrink back -- n_words and
    device_bytes stay bounded over rounds (advisor finding), and every round's
    matches equal the oracle's (reused wids must never alias a live word)."""
    r = random.Random(11)
    ix = gpu_index()
    o = Oracle()
    base = items_of([b"fleet/+/status", b"fleet/#", b"+/+/+/+/+/+/+/+/+/+/+/+"], [1, 2, 3])
    ix.apply(np.ones(len(base), np.uint8), base.blob, base.offs, base.vals)
    o.apply(np.ones(len(base), np.uint8), base.blob, base.offs, base.vals)
    words0 = ix.stats()["n_words"]
    seen = []
    for rnd in range(6):
        uid = [b"client-%016x-%08x" % (r.getrandbits(64), i) for i in range(4000)]
        keys = ([b"fleet/%s/+" % u for u in uid[:1500]] + [b"fleet/%s/status" % u for u in uid[1500:2500]] +
                [b"/".join([b"deep", u] + [b"l%d" % k for k in range(11)]) for u in uid[2500:]])
        d = items_of(keys, [10 + i for i in range(len(keys))])
        ix.apply(np.ones(len(d), np.uint8), d.blob, d.offs, d.vals)
        o.apply(np.ones(len(d), np.uint8), d.blob, d.offs, d.vals)
        probe = items_of([b"fleet/%s/status" % u for u in uid[::97]] + [k for k in keys[2500::131]] +
                         [b"fleet/%s/x" % u for u in uid[:40]] + [b"fleet/nobody/status"])
        assert_same(ix, o, probe)
        ix.apply(np.zeros(len(d), np.uint8), d.blob, d.offs, d.vals)
        o.apply(np.zeros(len(d), np.uint8), d.blob, d.offs, d.vals)
        assert_same(ix, o, probe)
        st = ix.stats()
        assert st["n_words"] == words0, (rnd, st["n_words"], words0)
        assert st["n_keys"] == 3
        seen.append(st["device_bytes"])
    assert max(seen[2:]) <= seen[1], seen   # no growth once the first rounds sized the tables


def test_c3_scale_properties(torch_dev):
    """2M filters, 1M topics: exact CSR vs the oracle on a 20k-topic sample, plus
    size-independent properties over the whole batch."""
    nf = 2_000_000
    fs = wl.filters(3, nf)
    ts = wl.topics(3, nf, 1_000_000)
    ix = gpu_index(fs)
    hit, vals, err = ix.match_batch(ts.blob, ts.offs)
    hit2, vals2, _ = ix.match_batch(ts.blob, ts.offs)
    assert np.array_equal(hit, hit2) and np.array_equal(vals, vals2)           # deterministic
    assert not err.any()
    per = np.diff(hit.astype(np.int64))
    assert (per >= 0).all()
    o = oracle_of(fs)
    idx = np.random.default_rng(7).choice(len(ts), 20_000, replace=False)
    sample = items_of([ts.item(int(i)) for i in idx])
    cnt, _, ohit, ovals = o.match_batch(sample.blob, sample.offs)
    for j, i in enumerate(idx):
        g = vals[int(hit[i]):int(hit[i + 1])]
        e = ovals[int(ohit[j]):int(ohit[j + 1])]
        assert np.array_equal(g, e), ts.item(int(i))
    # '$SYS' topics never hit the root globals '#' (value nf) / '+/#' (value nf + 1)
    sys_rows = [i for i in range(0, len(ts), 97) if ts.item(i).startswith(b"$")]
    assert sys_rows
    for i in sys_rows:
        g = vals[int(hit[i]):int(hit[i + 1])]
        assert nf not in g and nf + 1 not in g


def test_c3_full_size_sample(torch_dev):
    """The headline configuration itself (BASELINE.json configs[2]: C3 at
    10,000,002 filters, 1M-topic batches): a 20k-topic sample of the batch
    exact against the oracle over all 10M keys (values and order), the whole
    batch deterministic, and '$SYS' topics never hitting the root globals."""
    nf = 10_000_000
    fs = wl.filters(3, nf)
    ts = wl.topics(3, nf, 1_000_000)
    ix = _native.Index(hint_keys=len(fs))
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    assert ix.stats()["n_keys"] == len(fs)
    hit, vals, err = ix.match_batch(ts.blob, ts.offs)
    hit2, vals2, _ = ix.match_batch(ts.blob, ts.offs)
    assert np.array_equal(hit, hit2) and np.array_equal(vals, vals2)
    assert not err.any()
    o = oracle_of(fs)
    idx = np.random.default_rng(11).choice(len(ts), 20_000, replace=False)
    sample = items_of([ts.item(int(i)) for i in idx])
    cnt, _, ohit, ovals = o.match_batch(sample.blob, sample.offs)
    assert (cnt >= 0).all()
    for j, i in enumerate(idx):
        assert np.array_equal(vals[int(hit[i]):int(hit[i + 1])], ovals[int(ohit[j]):int(ohit[j + 1])]), ts.item(int(i))
    for i in range(0, len(ts), 97):
        if ts.item(i).startswith(b"$"):
            g = vals[int(hit[i]):int(hit[i + 1])]
            assert nf not in g and nf + 1 not in g


def test_child_table_grow_and_shrink(torch_dev):
    """A node going inline (<= 4 children) -> private table -> bigger tables ->
    back to inline, with matches checked against the oracle at every stage."""
    ix = gpu_index()
    o = Oracle()
    topics = items_of([b"a/%d/x" % i for i in range(700)] + [b"a/%d" % i for i in range(700)] + [b"b/1/x"])
    live = []
    r = random.Random(5)
    # past WIDE_LIT (256) children the node answers from an exact bitmap
    for stage in [3, 5, 6, 17, 33, 130, 200, 255, 256, 257, 600]:
        add = [i for i in range(stage) if i not in live]
        d = items_of([b"a/%d/+" % i for i in add] + [b"a/%d/#" % i for i in add], add + [1000 + i for i in add])
        ix.apply(np.ones(len(d), np.uint8), d.blob, d.offs, d.vals)
        o.apply(np.ones(len(d), np.uint8), d.blob, d.offs, d.vals)
        live += add
        assert_same(ix, o, topics)
    for keep in [400, 256, 255, 120, 40, 9, 5, 4, 2, 0]:
        drop = r.sample(live, len(live) - keep)
        live = [i for i in live if i not in drop]
        d = items_of([b"a/%d/+" % i for i in drop] + [b"a/%d/#" % i for i in drop], drop + [1000 + i for i in drop])
        ix.apply(np.zeros(len(d), np.uint8), d.blob, d.offs, d.vals)
        o.apply(np.zeros(len(d), np.uint8), d.blob, d.offs, d.vals)
        assert_same(ix, o, topics)
    assert ix.stats()["n_nodes"] == 1


def test_chains_cut_and_healed_under_deltas(torch_dev):
    """Long single-child chains made, cut in the middle (a terminal, a literal
    sibling, a '+' sibling), healed and removed again, with matches checked
    against the oracle at every stage: chains of 3 to 24 levels through literal
    and '+' edges, ending in exact and '#' terminals."""
    def chain(tag, n, plus_at=()):
        return b"/".join(b"+" if i in plus_at else b"%s%d" % (tag, i) for i in range(n))

    base = [chain(b"a", 3), chain(b"b", 11), chain(b"c", 12) + b"/#", chain(b"d", 24),
            chain(b"e", 14, plus_at=(3, 4, 9)), chain(b"f", 6, plus_at=(1,)) + b"/#", b"g/+/+/+/+/h"]
    cuts = [chain(b"b", 5), chain(b"b", 6) + b"/#", chain(b"d", 8) + b"/zz", chain(b"d", 15) + b"/+",
            chain(b"e", 7) + b"/x", chain(b"c", 2) + b"/+/#", b"g/+/+/q"]

    def topics_for(fs):
        out = []
        for f in fs:
            ws = [w if w not in (b"+", b"#") else b"w" for w in f.split(b"/")]
            for n in range(1, len(ws) + 3):
                out.append(b"/".join((ws + [b"t", b"u"])[:n]))
            for i in range(len(ws)):   # deviate at every level
                out.append(b"/".join(ws[:i] + [b"zz"] + ws[i + 1:]))
        return out

    ts = items_of(sorted(set(topics_for(base + cuts))))
    ix, o = gpu_index(), Oracle()

    def apply(fs, vals, ins):
        d = items_of(fs, vals)
        op = np.full(len(fs), 1 if ins else 0, np.uint8)
        ix.apply(op, d.blob, d.offs, d.vals)
        o.apply(op, d.blob, d.offs, d.vals)

    apply(base, range(len(base)), True)
    assert_same(ix, o, ts)
    apply(cuts, range(100, 100 + len(cuts)), True)
    assert_same(ix, o, ts)
    apply(cuts[::2], range(100, 100 + len(cuts), 2), False)
    assert_same(ix, o, ts)
    apply(cuts[1::2], range(101, 100 + len(cuts), 2), False)
    assert_same(ix, o, ts)
    apply(base[::2], range(0, len(base), 2), False)
    assert_same(ix, o, ts)
    apply(base[1::2], range(1, len(base), 2), False)
    assert_same(ix, o, ts)
    assert ix.stats()["n_nodes"] == 1


def test_host_batches_zero_copy_and_staged_agree(torch_dev):
    """Batches up to 65536 topics are staged zero-copy (kernels read and write
    mapped host memory), larger ones through HBM copies; caller-owned output
    buffers are reused across batches.  All paths give the oracle's results."""
    fs = wl.filters(1, 10_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    for nt in (1, 4096, 65536, 65537, 150_000):
        ts = wl.topics(1, 10_000, nt)
        hit, vals = assert_same(ix, o, ts)
        bufs = (np.zeros(nt + 1, np.uint64), np.zeros(len(vals) + 7, np.uint32), np.zeros(nt, np.uint8))
        for _ in range(2):
            h2, v2, e2 = ix.match_batch(ts.blob, ts.offs, out=bufs)
            assert np.array_equal(h2, hit) and np.array_equal(v2, vals) and not e2.any()


def test_host_batches_in_place_pinned_buffers(torch_dev):
    """Buffers from tm_host_alloc: batches <= 65536 topics run in place (the
    kernels read the caller's topics and write its hit lists), others take the
    staged path; a misaligned topic blob falls back to staging; a short value
    buffer gives TM_ECAP with complete offsets and the first `cap` values.
    Every case gives the oracle's results."""
    fs = wl.filters(3, 20_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    for nt in (1, 4096, 65536, 65537):
        ts = wl.topics(3, 20_000, nt)
        hit, vals = assert_same(ix, o, ts)
        nb = int(ts.offs[-1])
        pb = ix.host_array(nb + 32, np.uint8)
        po = ix.host_array(nt + 1, np.uint64)
        ph = ix.host_array(nt + 1, np.uint64)
        pv = ix.host_array(len(vals) + 5, np.uint32)
        pe = ix.host_array(nt, np.uint8)
        pb[:nb] = ts.blob[:nb]
        po[:] = ts.offs
        for _ in range(2):
            ph[:] = 0
            pe[:] = 7
            h2, v2, e2 = ix.match_batch(pb, po, out=(ph, pv, pe))
            assert np.array_equal(h2, hit) and np.array_equal(v2, vals) and not e2.any()
        # match/2 in place: the same first hits as the staged call
        fv, ff = ix.host_array(nt, np.uint32), ix.host_array(nt, np.uint8)
        assert ix._lib.tm_first_batch(ix._h, nt, _native._ptr(pb), _native._ptr(po), _native._ptr(fv),
                                      _native._ptr(ff)) == _native.TM_OK
        sv, sf = ix.first_batch(ts.blob, ts.offs)
        assert np.array_equal(ff, sf) and np.array_equal(fv[sf == 1], sv[sf == 1])
        ix.host_free(fv)
        ix.host_free(ff)
        # misaligned blob (offsets shifted by one byte): staged, same results
        pb[1:nb + 1] = ts.blob[:nb]
        h3, v3, _ = ix.match_batch(pb[1:], po, out=(ph, pv, pe))
        assert np.array_equal(h3, hit) and np.array_equal(v3, vals)
        # too small a value buffer
        if len(vals) > 3:
            pb[:nb] = ts.blob[:nb]
            rc = ix._lib.tm_match_batch(ix._h, nt, _native._ptr(pb), _native._ptr(po), _native._ptr(ph),
                                        _native._ptr(pv), 3, _native._ptr(pe))
            assert rc == _native.TM_ECAP
            assert np.array_equal(ph, hit) and np.array_equal(pv[:3], vals[:3])
        for a in (pb, po, ph, pv, pe):
            ix.host_free(a)
    with pytest.raises(_native.TmError):
        ix.host_free(np.zeros(4, np.uint8))


def test_one_launch_staging_branches(torch_dev):
    """k_walk_small's block-level staging, each branch against the oracle:
    topic bytes as one block span (short topics) or per-topic rows (a block
    whose span exceeds the LDS buffer), topics past SM_TB bytes on the lane
    walk; values through the block's LDS span (a few hits per topic), straight
    into the CSR (C2: ~1,000 values per topic, more than the block stages) and
    around a lane-walked topic in the block; all of it in place in
    tm_host_alloc buffers and from pageable memory."""
    fs = wl.filters(2, 20_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    assert_same(ix, o, wl.topics(2, 20_000, 300))              # direct: ~1,000 values per topic
    fs3 = wl.filters(3, 50_000)
    ix3, o3 = gpu_index(fs3), oracle_of(fs3)
    ts = wl.topics(3, 50_000, 5000)
    assert_same(ix3, o3, ts)                                   # one byte span per block, staged values
    r = random.Random(3)
    items = [ts.item(i) for i in range(600)]
    long_ = [b"/".join(b"%030d" % r.randrange(10**9) for _ in range(9)) for _ in range(40)]   # 279 B
    mid = [b"/".join(b"%028d" % r.randrange(10**9) for _ in range(8)) for _ in range(40)]     # 231 B
    mixed = items[:200] + mid + items[200:400] + long_ + items[400:]
    for order in (mixed, mid * 3 + items[:50], long_ + items[:100]):
        t = items_of(order)
        hit, vals = assert_same(ix3, o3, t)
        nb = int(t.offs[-1])
        pb, po = ix3.host_array(nb + 32, np.uint8), ix3.host_array(len(t) + 1, np.uint64)
        ph, pv, pe = (ix3.host_array(len(t) + 1, np.uint64), ix3.host_array(len(vals) + 5, np.uint32),
                      ix3.host_array(len(t), np.uint8))
        pb[:nb] = t.blob[:nb]
        po[:] = t.offs
        h2, v2, e2 = ix3.match_batch(pb, po, out=(ph, pv, pe))
        assert np.array_equal(h2, hit) and np.array_equal(v2, vals) and not e2.any()
        for a_ in (pb, po, ph, pv, pe):
            ix3.host_free(a_)


def test_mixed_batch_sizes_and_modes_in_sequence(torch_dev):
    """Tile totals stay zero between batches (k_emit clears them; the wave walk
    adds into them, the lane walk overwrites them, the small-batch tail kernel
    scans them): wave-walk, lane-walk, first-hit and deep-topic batches in any
    order on one index all give the oracle's results."""
    fs = wl.filters(1, 10_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    deep = items_of([b"/".join([b"a"] * 40), b"/".join([b"+x"] * 12) + b"/y"] * 3)
    seq = [5, 9000, 3000, 1, 20_000, 8192, 70_000, 8193, 65536, 65537, 2]
    for k, nt in enumerate(seq):
        ts = wl.topics(1, 10_000, nt, first=k * 7)
        hit, vals = assert_same(ix, o, ts)
        if k % 3 == 1:   # match/2: the first value in traversal order
            v, f = ix.first_batch(ts.blob, ts.offs)
            has = np.diff(hit.astype(np.int64)) > 0
            assert np.array_equal(f == 1, has)
            assert np.array_equal(v[has], vals[hit[:-1][has].astype(np.int64)])
        if k % 2 == 0:
            assert_same(ix, o, deep)


def test_wave_walk_limits_fall_back_exactly(torch_dev):
    """Batches of <= 64k topics take the one-launch wave-per-topic walk (16
    lanes per topic); its limits (a frontier wider than the group, more hit
    ranges than lanes, more levels than lanes) hand the topic to the group's
    lane-walk fallback.  Small (one launch) and large (> 64k: lane walk and
    tail kernels) batches of the same topics must both equal the oracle."""
    import itertools
    words = [b"a", b"b", b"c", b"d", b"e", b"f", b"g"]
    fl = []
    for k in range(1, 8):   # every '+' pattern of every prefix: frontier 2^k at level k
        for pat in itertools.product([0, 1], repeat=k):
            ws_ = [b"+" if p else w for p, w in zip(pat, words)]
            fl.append(b"/".join(ws_))
            fl.append(b"/".join(ws_) + b"/#")
    deep = b"/".join(b"l%d" % i for i in range(40))
    for L in (30, 31, 32, 33, 40):
        fl.append(b"/".join(deep.split(b"/")[:L]))
        fl.append(b"/".join(deep.split(b"/")[:L - 1] + [b"+"]))
        fl.append(b"/".join(deep.split(b"/")[:L - 2] + [b"#"]))
    fs = items_of(fl)
    ix, o = gpu_index(fs), oracle_of(fs)
    tl = [b"/".join(words[:k]) for k in range(1, 8)] + [b"a/b/c/x/e/f/g", b"x/b/c/d/e/f/g/h"]
    tl += [b"/".join(deep.split(b"/")[:L]) for L in range(28, 41)]
    small = items_of(tl)
    assert_same(ix, o, small)                                  # wave walk (+ fallbacks)
    big = items_of(tl * 3200)                                  # > 64k topics: lane walk
    assert_same(ix, o, big)
    first, found = ix.first_batch(small.blob, small.offs)
    cnt, _, ohit, ovals = o.match_batch(small.blob, small.offs)
    for i in range(len(small)):
        assert bool(found[i]) == (cnt[i] > 0)
        if cnt[i] > 0:
            assert first[i] == ovals[ohit[i]]


# ------------------------------------------------------------- filter-sharded

def _merge_ref(all_offs, all_vals):
    """numpy restatement of tm_merge_shards (the kernel's contract)."""
    world, n1 = all_offs.shape
    out = [all_vals[r, all_offs[r, t]:all_offs[r, t + 1]] for t in range(n1 - 1) for r in range(world)]
    return all_offs.sum(axis=0), (np.concatenate(out) if out else np.zeros(0, np.int32))


@pytest.mark.parametrize("world", [1, 3])
def test_filter_sharded_merge_vs_oracle(torch_dev, world):
    """C4 in one process: `world` shard indexes on one GPU, the same topic batch
    on each, the gathered CSR lists merged by tm_merge_shards == the unsharded
    oracle (per-topic value sets) and == the kernel contract (exact order)."""
    import torch
    from emqx_amd import shard
    nf = 60_000
    ts = wl.topics(3, nf, 20_000)
    dev = torch.device("cuda:0")
    offs, vals = [], []
    for r in range(world):
        part = wl.filters(3, nf, shard=r, nshards=world)
        hit, v, err = gpu_index(part).match_batch(ts.blob, ts.offs)
        offs.append(hit.astype(np.int64))
        vals.append(v.view(np.int32))
    stride = max(max(len(v) for v in vals), 1)
    all_offs = np.stack(offs)
    all_vals = np.zeros((world, stride), np.int32)
    for r, v in enumerate(vals):
        all_vals[r, :len(v)] = v
    m_hit, m_vals = shard.merge(torch.from_numpy(all_offs).to(dev), torch.from_numpy(all_vals).to(dev), stride)
    torch.cuda.synchronize()
    m_hit, m_vals = m_hit.cpu().numpy(), m_vals.cpu().numpy()
    m_vals = m_vals[: int(m_hit[-1])]
    r_hit, r_vals = _merge_ref(all_offs, all_vals)
    assert np.array_equal(m_hit, r_hit) and np.array_equal(m_vals, r_vals)
    fs = wl.filters(3, nf)
    cnt, _, ohit, ovals = oracle_of(fs).match_batch(ts.blob, ts.offs)
    assert np.array_equal(m_hit.astype(np.uint64), ohit.astype(np.uint64))
    mv = m_vals.view(np.uint32)
    for i in range(len(ts)):
        assert np.array_equal(np.sort(mv[m_hit[i]:m_hit[i + 1]]), np.sort(ovals[ohit[i]:ohit[i + 1]])), i


def test_exchange_overflow_stays_in_buffer(torch_dev):
    """Exchange.run with a per-peer capacity far below the batch's values
    (world 1 over RCCL): the cut counts keep tm_merge_shards inside the
    received values -- the merged lists are the lists' first per_peer values,
    topic by topic -- and check() reports the overflow and grows the
    capacity, after which the same batch merges whole (advisor r2)."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    from emqx_amd import shard
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        fs = wl.filters(3, 20_000)
        ts = wl.topics(3, 20_000, 3_000)
        hit, vals, _ = gpu_index(fs).match_batch(ts.blob, ts.offs)
        assert int(hit[-1]) > 1000
        dev = torch.device("cuda:0")
        h = torch.from_numpy(hit.astype(np.int64)).to(dev)
        v = torch.from_numpy(vals.view(np.int32).copy()).to(dev)
        small = 1000
        xch = shard.Exchange(len(ts), dev, per_peer=small)
        out_hit, out_vals = xch.run(h, v)
        torch.cuda.synchronize()
        cnt = np.diff(hit.astype(np.int64))
        cut = np.minimum(cnt, np.clip(small - (np.cumsum(cnt) - cnt), 0, None))
        exp_hit = np.concatenate([[0], np.cumsum(cut)])
        got_hit = out_hit.cpu().numpy()
        assert np.array_equal(got_hit, exp_hit)
        got = out_vals.cpu().numpy()[: int(exp_hit[-1])].view(np.uint32)
        exp = np.concatenate([vals[int(hit[i]):int(hit[i]) + int(cut[i])] for i in range(len(ts))])
        assert np.array_equal(got, exp)
        assert not xch.check() and xch.per_peer > int(hit[-1])
        out_hit, out_vals = xch.run(h, v)
        torch.cuda.synchronize()
        assert xch.check()
        assert np.array_equal(out_hit.cpu().numpy(), hit.astype(np.int64))
        assert np.array_equal(out_vals.cpu().numpy()[: int(hit[-1])].view(np.uint32), vals)
    finally:
        dist.destroy_process_group()


# ------------------------------------------------- router / syncer / broker

def test_router_composition_bag_then_filters(torch_dev):
    """match_routes = the bag's rows in insertion order, then the filter
    matches in matches/3 order (emqx_router.erl:511-516).  The bag stays on
    the host as in src/emqx_router_gpu.erl (ets:lookup gives its order); the
    device mirror holds the filter table's keys only."""
    r = rt.Router(node="n1")
    for topic, dest in [(b"a/b", "n2"), (b"a/+", "n1"), (b"a/b", "n1"), (b"#", "n3"), (b"a/b", (b"g", "n4"))]:
        r.add_route(topic, dest)
    r.delete_route(b"a/b", "n2")
    r.add_route(b"a/b", "n2")                      # re-added: goes to the end of the bag
    exp = [(b"a/b", "n1"), (b"a/b", (b"g", "n4")), (b"a/b", "n2"), (b"a/+", "n1"), (b"#", "n3")]
    assert [tuple(x) for x in r.match_routes(b"a/b")] == exp
    assert r.lookup_routes(b"a/b") == [rt.Route(b"a/b", d) for d in ("n1", (b"g", "n4"), "n2")]
    assert r.has_route(b"a/+", "n1") and not r.has_route(b"a/+", "n2") and r.has_route(b"a/b", "n2")
    assert r.stats_n_routes() == 5
    assert r.mirror_keys() == 2                    # a/+ and #: the bag is not on the device
    assert [tuple(x) for x in r.match_routes(b"a/c")] == [(b"a/+", "n1"), (b"#", "n3")]
    assert [tuple(x) for x in r.match_routes(b"$SYS/x")] == []


def test_router_cleanup_and_replicated_events(torch_dev):
    """Node a makes the writes; node b receives them replicated (its tables
    change at once, its mirror when its event process drains the events).
    After the drain both answer the same; a node-down cleanup on a (record-form
    delete events, drained) leaves exactly the other nodes' routes."""
    rnd = random.Random(7)
    ops = []
    for i in range(400):
        t = b"/".join(rnd.choice([b"a", b"b", b"c", b"+"]) for _ in range(rnd.randint(1, 3)))
        if rnd.random() < 0.1:
            t += b"/#"
        d = rnd.choice(["n1", "n2", "n3", (b"g", "n2"), (b"h", "n3")])
        ops.append(("add" if rnd.random() < 0.75 else "delete", t, d))
    a, b = rt.Router(node="n1"), rt.Router(node="n1")
    model = RouterModel()
    for k, (op, t, d) in enumerate(ops):
        (a.add_route if op == "add" else a.delete_route)(t, d)
        b.replicate(op, t, d, record_form=k % 2 == 0)
        (model.add if op == "add" else model.delete)(t, d)
    topics = [b"/".join(rnd.choice([b"a", b"b", b"c", b"d"]) for _ in range(rnd.randint(1, 4))) for _ in range(300)]
    b.drain_events()
    exp = model.expected(topics)
    assert a.match_routes_batch(topics) == exp
    assert b.match_routes_batch(topics) == exp
    a.drain_events()                               # a's own echoes: reconciled, no change
    assert a.match_routes_batch(topics) == exp
    a.cleanup_routes("n2")
    while a.pending_events():
        a.drain_events(limit=37)
    for op, t, d in ops:
        if rt.get_dest_node(d) == "n2":
            model.delete(t, d)
    left = a.match_routes_batch(topics)
    assert left == model.expected(topics)
    assert any(left) and all(rt.get_dest_node(x.dest) != "n2" for rs in left for x in rs)


def test_router_subscribe_then_publish_sees_the_route(torch_dev):
    """The read-your-writes contract of the default write path (VERDICT r4
    item 1): do_add_route -> mria:dirty_write returns only once every later
    matches/3 sees the route (emqx_broker.erl:778-808, emqx_router.erl:
    492-493), so a PUBLISH that follows the SUBACK reaches the subscriber.
    The table events the writes produce are withheld the whole time (the
    event process is behind): the hook's mirror-only delta alone must carry
    the write.  When the stale echoes are drained at last -- the insert event
    of a route deleted meanwhile among them -- they must not resurrect it."""
    r = rt.Router(node="n1")
    model = RouterModel()
    rnd = random.Random(11)
    for i in range(300):
        flt = f"dev/{i % 40}/+/t{i % 7}".encode() if i % 3 else f"dev/{i % 40}/#".encode()
        dest = rnd.choice(["n1", "n2", (b"g", "n3")])
        op = "delete" if rnd.random() < 0.3 else "add"
        (r.add_route if op == "add" else r.delete_route)(flt, dest)
        (model.add if op == "add" else model.delete)(flt, dest)
        # publish right after the (un)subscribe returns: the device has it
        pub = f"dev/{i % 40}/x/t{i % 7}".encode()
        assert r.match_routes(pub) == model.expected([pub])[0], (i, flt, dest, op)
    assert r.pending_events() == 300              # nothing drained: the hook carried every write
    topics = [f"dev/{i}/x/t{j}".encode() for i in range(40) for j in range(7)] + [b"dev/3", b"dev"]
    exp = model.expected(topics)
    assert r.match_routes_batch(topics) == exp
    r.drain_events(limit=150)                     # echoes, in order, half of them
    assert r.match_routes_batch(topics) == exp
    r.drain_events()
    assert r.match_routes_batch(topics) == exp
    assert r.mirror_keys() == len(model.wild)


def test_router_delete_event_shapes(torch_dev):
    """Every detailed delete event shape reaches the mirror: {Tab, Key} from
    dirty_delete and the record form from delete_object / match_delete
    (src/emqx_topic_index_gpu.erl event_key/2); events of the bag and of
    other tables are ignored by the mirror."""
    r = rt.Router(node="n1")
    for t in (b"s/+", b"s/+/x", b"s/#"):
        r.replicate("add", t, "n2")
    r.replicate("add", b"s/1", "n2")
    r.drain_events()
    assert [tuple(x) for x in r.match_routes(b"s/1")] == [(b"s/1", "n2"), (b"s/+", "n2"), (b"s/#", "n2")]
    k_plus, k_hash = ti.make_key(b"s/+", "n2"), ti.make_key(b"s/#", "n2")
    del r._filters[k_plus]
    del r._filters[k_hash]
    r.on_table_events([("delete", (rt.ROUTE_TAB_FILTERS, k_plus)), ("delete", rt.RouteIdx(k_hash)),
                       ("delete", ("other_tab", k_plus)), ("write", rt.Route(b"s/1", "n9"))])
    assert [tuple(x) for x in r.match_routes(b"s/1")] == [(b"s/1", "n2")]
    assert [tuple(x) for x in r.match_routes(b"s/1/x")] == [(b"s/+/x", "n2")]
    assert r.mirror_keys() == 1


def test_syncer_batches_reach_the_device(torch_dev):
    """Route ops pushed through the syncer (batches of <= 100, one
    tm_apply_deltas each) give the routes the reference's tables would hold:
    match_routes equals the CPU model + oracle (harness.RouterModel)."""
    from emqx_amd import syncer as sy
    synced = rt.Router(node="n1")
    model = RouterModel()
    s = sy.Syncer(synced, max_batch_size=100)
    refs = []
    for i in range(600):
        t = f"dev/{i % 150}/+/x".encode() if i % 3 else f"dev/{i % 150}/y".encode()
        op = "delete" if i % 7 == 0 else "add"
        (model.add if op == "add" else model.delete)(t, "n1")
        refs.append(s.push(op, t, "n1", {"reply": True}))
    assert s.run_once() > 0 and s.batches >= 2
    assert all(x.wait(0) == "ok" for x in refs)
    topics = [f"dev/{i}/{j}/x".encode() for i in range(150) for j in ("q", "y")] + \
             [f"dev/{i}/y".encode() for i in range(150)]
    assert synced.match_routes_batch(topics) == model.expected(topics)


def _broker_fixture(n_filters, n_topics):
    r = rt.Router(node="n1")
    model = RouterModel()
    fs = wl.filters(1, n_filters)
    for i in range(len(fs)):
        d = ["n1", "n2", (b"grp", "n3")][i % 3]
        r.add_route(fs.item(i), d)
        model.add(fs.item(i), d)
    ts = wl.topics(1, n_filters, n_topics)
    return r, model, ts


def test_broker_micro_batch_matches_the_reference_routes(torch_dev):
    """Publishes micro-batched into few device launches; every message gets
    aggre/1 of the routes the reference would find (CPU model + oracle)."""
    from emqx_amd import broker as bk
    r, model, ts = _broker_fixture(2_000, 3_000)
    msgs = [bk.Message(ts.item(i), i) for i in range(len(ts))]
    b = bk.Broker(r, max_batch=1024, max_wait_ms=50, start=True)
    try:
        futs = [b.publish(m) for m in msgs]
        batched = [f.result(timeout=60) for f in futs]
    finally:
        b.close()
    assert b.batches < len(msgs) / 100       # micro-batched: few device launches
    exp = model.expected([m.topic for m in msgs])
    for got, routes in zip(batched, exp):
        assert got[0] == bk.aggre(routes)


def test_broker_badarg_fails_only_its_message(torch_dev):
    """One 'a/+/b' publish inside a 1k micro-batch: 999 messages routed as the
    reference would route them, one BadArg (emqx_trie_search.erl:374-375 fails
    only the publishing process)."""
    from emqx_amd import broker as bk
    r, model, ts = _broker_fixture(2_000, 999)
    msgs = [bk.Message(ts.item(i), i) for i in range(500)] + [bk.Message(b"a/+/b", -1)] + \
           [bk.Message(ts.item(i), i) for i in range(500, 999)]
    b = bk.Broker(r, max_batch=1000, max_wait_ms=1000)
    futs = [b.publish(m) for m in msgs]
    b.flush()
    assert b.batches == 1
    exp = model.expected([m.topic for m in msgs])
    bad = [i for i, f in enumerate(futs) if f.exception(0) is not None]
    assert bad == [500] and isinstance(futs[500].exception(0), BadArg)
    for i, f in enumerate(futs):
        if i != 500:
            assert f.result(0)[0] == bk.aggre(exp[i])


def test_ids_of_one_filter_follow_term_order(torch_dev):
    """Several IDs on one filter come back in the ID's term order whatever
    order they were inserted in and whichever u32 kid they got (freed kids are
    reused): match/2 is the smallest key, matches/3 the reverse traversal."""
    tab = ti.new()
    ti.insert(b"a/+", 2, None, tab)
    ti.insert(b"a/+", 1, None, tab)
    ti.insert(b"a/+", "node", None, tab)
    ti.insert(b"a/#", 7, None, tab)
    assert ti.match(b"a/b", tab) == ti.make_key(b"a/#", 7)
    assert [get_id(k) for k in ti.matches(b"a/b", tab)] == ["node", 2, 1, 7]
    ti.delete(b"a/#", 7, tab)
    assert ti.match(b"a/b", tab) == ti.make_key(b"a/+", 1)
    ti.delete(b"a/+", 2, tab)                  # its kid is freed ...
    ti.insert(b"a/+", 0, None, tab)            # ... and reused by a smaller ID
    assert ti.match(b"a/b", tab) == ti.make_key(b"a/+", 0)
    assert [get_id(k) for k in ti.matches(b"a/b", tab)] == ["node", 1, 0]
    assert [get_id(k) for k in ti.matches(b"a/b", tab, ["unique"])] == [0, 1, "node"]


def test_c2_full_size_sample_vs_oracle(torch_dev):
    """C2 at full size (1M 'fleet/{id}/sensor/+' + 1k globals, one 1M-topic
    batch, ~1e9 values on the device): offsets of every topic and the values
    of a 20k-topic sample equal the oracle's (traversal order)."""
    import torch
    nf = 1_000_000
    fs = wl.filters(2, nf)
    ts = wl.topics(2, nf, 1_000_000)
    ix = gpu_index(fs)
    dev = torch.device("cuda:0")
    n = len(ts)
    blob = torch.from_numpy(ts.blob).to(dev)
    offs = torch.from_numpy(ts.offs.view(np.int64)).to(dev)
    hit = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ix.match_batch_dev(n, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), 0, 0, err.data_ptr(), s)
    torch.cuda.synchronize()
    total = int(hit[-1])
    out = torch.zeros(total, dtype=torch.int32, device=dev)
    ix.match_batch_dev(n, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), out.data_ptr(), total, err.data_ptr(), s)
    torch.cuda.synchronize()
    assert not bool(err.any())
    h = hit.cpu().numpy()
    per = np.diff(h)
    assert per.min() >= 1000 and per.max() == 1001
    idx = np.sort(np.random.default_rng(11).choice(n, 20_000, replace=False))
    sample = items_of([ts.item(int(i)) for i in idx])
    o = oracle_of(fs)
    _, _, ohit, ovals = o.match_batch(sample.blob, sample.offs)
    assert np.array_equal(per[idx], np.diff(ohit.astype(np.int64)))
    rows = torch.from_numpy(np.concatenate([np.arange(h[i], h[i + 1]) for i in idx])).to(dev)
    got = out[rows].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, ovals)


@pytest.mark.parametrize("copies,nstreams", [(1, 2), (2, 2), (3, 3)])
def test_batches_on_two_streams_see_patches_in_order(torch_dev, copies, nstreams):
    """Per-stream workspaces: batches on several streams may overlap; a batch
    sees every delta applied before it, whichever stream shipped the patch --
    with one copy of the tables, and with 2-3 copies (tm_options.copies), where
    a patch reaches each copy lazily, when a batch is about to read it."""
    import torch
    nf = 30_000
    fs = wl.filters(5, nf)
    ix = _native.Index(copies=copies)
    ix.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    o = oracle_of(fs)
    ts = wl.topics(5, nf, 40_000)
    dev = torch.device("cuda:0")
    d_blob = torch.from_numpy(ts.blob.copy()).to(dev)
    d_offs = torch.from_numpy(ts.offs.view(np.int64).copy()).to(dev)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    n = len(ts)
    results = []
    for k in range(4 if copies == 1 else 9):
        d = wl.deltas(nf, k * 3_000, 3_000 if k % 3 else 40)
        ix.apply(d.flags, d.blob, d.offs, d.vals)
        o.apply(d.flags, d.blob, d.offs, d.vals)
        o.prepare()
        _, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
        s = streams[k % nstreams]
        hit = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        err = torch.zeros(n, dtype=torch.uint8, device=dev)
        out = torch.zeros(int(ohit[-1]) + 1, dtype=torch.int32, device=dev)
        ix.match_batch_dev(n, d_blob.data_ptr(), d_offs.data_ptr(), hit.data_ptr(), out.data_ptr(), out.numel(),
                           err.data_ptr(), s.cuda_stream)
        results.append((hit, out, ohit, ovals))
    torch.cuda.synchronize()
    for hit, out, ohit, ovals in results:
        h = hit.cpu().numpy().view(np.uint64)
        assert np.array_equal(h, ohit.astype(np.uint64))
        assert np.array_equal(out.cpu().numpy().view(np.uint32)[: int(h[-1])], ovals)


def test_topic_index_matches_filter(torch_dev):
    """matches_filter/3 through the topic_index API (emqx_topic_index.erl:82-84)
    on a device-backed table after inserts and deletes: the reverse of the
    oracle's traversal order, and publishes still match on the same table."""
    r = random.Random(0x454D5158 + 900)
    tab = ti.new()
    o = Oracle()
    rf = lambda: _rand_filter(r, [_rand_level(r) for _ in range(r.randint(1, 4))])   # noqa: E731
    filters = [rf() for _ in range(400)]
    for i, f in enumerate(filters):
        ti.insert(f, i, b"", tab)
        o.insert(f, i, 0)
    for i in r.sample(range(len(filters)), 80):
        ti.delete(filters[i], i, tab)
        o.delete(filters[i], i, 0)
    for q in [b"#", b"+/#", b"foo/+", b"$SYS/#", b"+/+/+"] + [rf() for _ in range(40)]:
        got = [get_id(k) for k in ti.matches_filter(q, tab)]
        assert got == o.matches_filter(q)[::-1], q
        uniq = [get_id(k) for k in ti.matches_filter(q, tab, ["unique"])]
        assert uniq == sorted(set(got)), q
    t = b"foo/bar/1"
    assert sorted(get_id(k) for k in ti.matches(t, tab, [])) == sorted(o.matches(t))


# ------------------------------------------------------ concurrent callers

@pytest.mark.parametrize("copies", [1, 2])
def test_concurrent_callers_see_consistent_snapshots(torch_dev, copies):
    """12 host threads submit 4k-topic batches through tm_match_batch at once
    (half with tm_host_alloc buffers, half pageable) while the main thread
    applies 16 epochs of subscribe/unsubscribe deltas.  Each epoch is one
    tm_apply_deltas call that also inserts a marker key 'probe/+' -> 900000+e,
    so the probe topic of a batch says how many epochs it saw; every batch
    must equal the oracle after exactly that many epochs, and a thread's
    batches never go back in time (SURVEY.md 8b Threading: a batch sees a
    consistent prefix of the deltas)."""
    import threading
    import time
    nf, nthreads, lb, epochs = 10_000, 12, 4096, 16
    fs = wl.filters(1, nf)
    ix = _native.Index(copies=copies)
    ix.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    o = oracle_of(fs)
    r = random.Random(0x454D5158 + 77)
    tsets = []
    for t in range(nthreads):
        ts = wl.topics(1, nf, lb, first=t * lb)
        tsets.append(items_of(ts.items() + [b"probe/x"]))
    ep_ops = []
    for e in range(epochs):
        fl, vals, ops = [b"probe/+"], [900_000 + e], [1]
        for i in range(60):   # new filters that match some batch topics
            words = tsets[r.randrange(nthreads)].item(r.randrange(lb)).split(b"/")
            k = r.randrange(len(words))
            words[k] = b"+" if r.random() < 0.5 else words[k]
            fl.append(b"/".join(words[: k + 1]) + (b"/#" if r.random() < 0.3 else b""))
            vals.append(100_000 + e * 1000 + i)
            ops.append(1)
        for _ in range(60):   # unsubscribe base filters
            i = r.randrange(len(fs))
            fl.append(fs.item(i))
            vals.append(int(fs.vals[i]))
            ops.append(0)
        ep_ops.append((np.array(ops, np.uint8), items_of(fl, vals)))
    # the oracle after e epochs, for every thread's topics
    expected = []
    for e in range(epochs + 1):
        if e:
            ops, d = ep_ops[e - 1]
            o.apply(ops, d.blob, d.offs, d.vals)
        o.prepare()
        expected.append([o.match_batch(ts.blob, ts.offs)[2:] for ts in tsets])
    results = [[] for _ in range(nthreads)]
    stop = threading.Event()
    errors = []

    def caller(t):
        try:
            ts = tsets[t]
            n = len(ts)
            if t % 2:   # pageable caller buffers
                bufs = (np.zeros(n + 1, np.uint64), np.zeros(200_000, np.uint32), np.zeros(n, np.uint8))
                blob, offs = ts.blob, ts.offs
            else:       # tm_host_alloc buffers: in place
                nb = int(ts.offs[-1])
                blob = ix.host_array(nb + 16, np.uint8)
                blob[:nb] = ts.blob[:nb]
                offs = ix.host_array(n + 1, np.uint64)
                offs[:] = ts.offs
                bufs = (ix.host_array(n + 1, np.uint64), ix.host_array(200_000, np.uint32), ix.host_array(n, np.uint8))
            while not stop.is_set() or len(results[t]) < 3:
                t0 = time.perf_counter()
                hit, vals, err = ix.match_batch(blob, offs, out=bufs)
                results[t].append((time.perf_counter() - t0, hit.copy(), vals.copy(), err.copy()))
        except BaseException as e:   # noqa: BLE001 - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for ops, d in ep_ops:
        time.sleep(0.02)
        ix.apply(ops, d.blob, d.offs, d.vals)
    time.sleep(0.05)
    stop.set()
    for x in th:
        x.join(timeout=60)
    assert not errors, errors
    seen = set()
    lat = []
    for t in range(nthreads):
        last = -1
        for dt, hit, vals, err in results[t]:
            lat.append(dt)
            assert not err.any()
            probe = [v for v in vals[int(hit[-2]):int(hit[-1])].tolist() if v >= 900_000]   # '+'-deltas hit it too
            e = len(probe)
            assert sorted(probe) == [900_000 + k for k in range(e)], "a batch saw part of an epoch"
            assert e >= last, "a thread's batches went back in time"
            last = e
            seen.add(e)
            ohit, ovals = expected[e][t]
            assert np.array_equal(hit, ohit) and np.array_equal(vals, ovals), (t, e)
    assert len(seen) >= 4, seen          # the batches did interleave with the epochs
    lat = np.array(lat) * 1e3
    print(f"concurrent callers: {len(lat)} batches, epochs seen {sorted(seen)}, "
          f"p50 {np.percentile(lat, 50):.3f} ms p99 {np.percentile(lat, 99):.3f} ms")


@pytest.mark.parametrize("kind,copies,leaders,gather,land,ticket,spin", [
    ("wave", 1, 4, 0, 0, 0, 0), ("wave8", 1, 4, 0, 0, 0, 0), ("auto", 2, None, 0, 0, 0, 0), ("auto", 2, 2, 0, 0, 0, 0),
    ("auto", 1, 4, 30, 0, 0, 0), ("auto", 2, 1, 30, 0, 0, 0), ("auto", 2, 2, 0, 0, 0, 200), ("auto", 2, 2, 0, 0, 1, 0),
    ("auto", 2, 2, 0, 0, 1, 40)])
def test_combined_callers_with_deltas_see_snapshots_and_never_fail(torch_dev, kind, copies, leaders, gather, land,
                                                                   ticket, spin):
    """The NIF's production path under load:
    16 host threads submit in-place 32-bit batches (tm_match_batch32_ex on
    host_array buffers, what the NIF's dirty schedulers do) through the
    host-batch combiner at 4 leaders (the default; and at 2 and 1) -- shared
    k_walk_small launches with a segment table; with a gather window
    (TM_DEBUG_CMB_GATHER), with the start-order ticket and with waiting
    callers spinning (TM_DEBUG_CMB_SPIN; the round-5 landing variant,
    TM_DEBUG_CMB_LAND, was removed in round 6: land is 0) -- while the main
    thread applies 16 delta
    epochs.  Every
    batch equals the oracle after exactly the epochs its probe topic saw, a
    thread never goes back in time, and no batch's look-back wait expired:
    TM_DEBUG_FAILED_BATCHES and _RETRIED_BATCHES stay 0 (the readers of the
    reference's read_concurrency table never fail, emqx_topic_index.erl:41-48).
    copies 2: the configuration INTEGRATION recommends under churn (a batch
    after a delta runs on the table copy no batch is reading)."""
    import threading
    import time
    nf, nthreads, lb, epochs = 10_000, 16, 4096, 16
    fs = wl.filters(1, nf)
    ix = _native.Index(copies=copies)
    if leaders is not None:
        ix.debug_set(_native.TM_DEBUG_COMBINE, leaders)
    assert ix.debug_get(_native.TM_DEBUG_COMBINE) == (leaders or 4)
    ix.debug_set(_native.TM_DEBUG_CMB_GATHER, gather)
    ix.debug_set(_native.TM_DEBUG_CMB_LAND, land)
    ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, ticket)
    ix.debug_set(_native.TM_DEBUG_CMB_SPIN, spin)
    assert (ix.debug_get(_native.TM_DEBUG_CMB_GATHER), ix.debug_get(_native.TM_DEBUG_CMB_LAND)) == (gather, land)
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _small_kind(kind))
    ix.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    o = oracle_of(fs)
    r = random.Random(0x454D5158 + 99)
    tsets = []
    for t in range(nthreads):
        ts = wl.topics(1, nf, lb - 1 - (t % 3) * 700, first=t * lb)   # ragged batch sizes
        tsets.append(items_of(ts.items() + [b"probe/x"]))
    ep_ops = []
    for e in range(epochs):
        fl, vals, ops = [b"probe/+"], [900_000 + e], [1]
        for i in range(60):
            words = tsets[r.randrange(nthreads)].item(r.randrange(lb // 2)).split(b"/")
            k = r.randrange(len(words))
            words[k] = b"+" if r.random() < 0.5 else words[k]
            fl.append(b"/".join(words[: k + 1]) + (b"/#" if r.random() < 0.3 else b""))
            vals.append(100_000 + e * 1000 + i)
            ops.append(1)
        for _ in range(60):
            i = r.randrange(len(fs))
            fl.append(fs.item(i))
            vals.append(int(fs.vals[i]))
            ops.append(0)
        ep_ops.append((np.array(ops, np.uint8), items_of(fl, vals)))
    expected = []
    for e in range(epochs + 1):
        if e:
            ops, d = ep_ops[e - 1]
            o.apply(ops, d.blob, d.offs, d.vals)
        o.prepare()
        expected.append([o.match_batch(ts.blob, ts.offs)[2:] for ts in tsets])
    f0 = ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES), ix.debug_get(_native.TM_DEBUG_RETRIED_BATCHES)
    c0 = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES), ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES)
    results = [[] for _ in range(nthreads)]
    stop = threading.Event()
    errors = []

    def caller(t):
        try:
            ts = tsets[t]
            n = len(ts)
            nb = int(ts.offs[-1])
            blob = ix.host_array(nb + 16, np.uint8)
            blob[:nb] = ts.blob[:nb]
            offs = ix.host_array(n + 1, np.uint32)
            offs[:] = ts.offs.astype(np.uint32)
            bufs = (ix.host_array(n + 1, np.uint32), ix.host_array(200_000, np.uint32), ix.host_array(n, np.uint8))
            while not stop.is_set() or len(results[t]) < 3:
                hit, vals, err = ix.match_batch32(blob, offs, bufs)
                results[t].append((hit.astype(np.uint64), vals.copy(), err.copy()))
        except BaseException as e:   # noqa: BLE001 - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for ops, d in ep_ops:
        time.sleep(0.02)
        ix.apply(ops, d.blob, d.offs, d.vals)
    time.sleep(0.05)
    stop.set()
    for x in th:
        x.join(timeout=60)
    assert not errors, errors
    assert (ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES), ix.debug_get(_native.TM_DEBUG_RETRIED_BATCHES)) == f0
    launches = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES) - c0[0]
    batches = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES) - c0[1]
    seen = set()
    for t in range(nthreads):
        last = -1
        for hit, vals, err in results[t]:
            assert not err.any()
            probe = [v for v in vals[int(hit[-2]):int(hit[-1])].tolist() if v >= 900_000]
            e = len(probe)
            assert sorted(probe) == [900_000 + k for k in range(e)], "a batch saw part of an epoch"
            assert e >= last, "a thread's batches went back in time"
            last = e
            seen.add(e)
            ohit, ovals = expected[e][t]
            assert np.array_equal(hit, ohit) and np.array_equal(vals, ovals), (t, e)
    assert len(seen) >= 4, seen
    assert batches == sum(len(x) for x in results) and launches < batches   # combined: fewer launches than batches
    print(f"combined callers: {batches} batches in {launches} launches, epochs seen {sorted(seen)}")


def test_readers_never_decode_a_reused_value(torch_dev):
    """8 matcher threads call matches/3 through the topic_index mirror while
    one writer deletes and inserts keys, so freed u32 values get reused
    (emqx_topic_index.erl:41-48: lock-free readers).  Every key a
    reader returns must match its topic (spec matcher) and have been live at
    some point between the batch's submit and its completion; every stable
    key that matches must be there; nothing may crash.  The values of deleted
    keys wait in quarantine (include/tmatch.h "Reader epochs"), so a stale
    device hit decodes to nothing instead of to a newer key."""
    import threading
    from pyoracle import spec_match
    nthreads, rounds = 8, 60
    r = random.Random(0x454D5158 + 88)
    stable = wl.filters(1, 3_000)
    tab = ti.new()
    for i in range(len(stable)):
        ti.insert(stable.item(i), ("s", int(stable.vals[i])), None, tab)
    ts = wl.topics(1, 3_000, 256)
    topics = ts.items()
    # churn universe: filters matching the topics and filters matching none
    universe = []
    for k in range(600):
        words = r.choice(topics).split(b"/")
        if k % 2:
            words[r.randrange(len(words))] = b"zz%d" % k   # matches none of the topics
        j = r.randrange(len(words))
        words[j] = b"+" if r.random() < 0.5 else words[j]
        universe.append(b"/".join(words[: j + 1 if r.random() < 0.3 else len(words)]) +
                        (b"/#" if r.random() < 0.2 else b""))
    life = {}                    # churn key -> [flush index inserted, flush index deleted]
    clock = [0]                  # flushes done by the writer
    live, nid = [], 0
    for f in universe[:300]:
        key = ti.make_key(f, ("c", nid))
        ti.insert(f, ("c", nid), None, tab)
        live.append((f, ("c", nid)))
        life[key] = [0, None]
        nid += 1
    tab.flush()
    so = Oracle()
    for i in range(len(stable)):
        so.insert(stable.item(i), int(stable.vals[i]))
    so.prepare()
    want = [set(so.matches(t)) for t in topics]      # stable ids every result must hold
    stop = threading.Event()
    errors, checked = [], [0]

    def reader():
        try:
            for _ in range(rounds):
                c0 = clock[0]
                res = ti.matches_batch(topics, tab)
                c1 = clock[0]
                for t, keys in zip(topics, res):
                    got_stable = set()
                    for key in keys:
                        f, (ident,) = key
                        fb = ti.get_topic(key)
                        assert spec_match(t, fb), (t, key)
                        if ident[0] == "s":
                            got_stable.add(ident[1])
                        else:
                            ins, dele = life[key]
                            assert ins <= c1 and (dele is None or dele > c0), (t, key, ins, dele, c0, c1)
                    assert got_stable == want[topics.index(t)], t
                    checked[0] += 1
        except BaseException as e:   # noqa: BLE001 - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=reader) for _ in range(nthreads)]
    for x in th:
        x.start()
    inserted = 300
    while any(x.is_alive() for x in th):
        for _ in range(8):       # one flush = one delta batch of 8 deletes + 8 inserts
            f, ident = live.pop(r.randrange(len(live)))
            ti.delete(f, ident, tab)
            life[ti.make_key(f, ident)][1] = clock[0] + 1
            f = r.choice(universe)
            ident = ("c", nid)
            nid += 1
            # a reader's own flush may ship this insert before the writer's
            # does: live from the current flush index on
            life[ti.make_key(f, ident)] = [clock[0], None]
            ti.insert(f, ident, None, tab)
            live.append((f, ident))
            inserted += 1
        tab.flush()
        clock[0] += 1
    for x in th:
        x.join(timeout=60)
    assert not errors, errors[:3]
    assert checked[0] == nthreads * rounds * len(topics)
    assert clock[0] >= 20, clock[0]                        # the writer kept churning throughout
    assert len(tab._keys) < len(stable) + inserted, "no value was ever reused"
    print(f"reuse under readers: {clock[0]} delta batches, {inserted} churn inserts, "
          f"{len(tab._keys)} values for {len(stable) + inserted} keys")


def test_matches_filter_keys_no_topic_can_match(torch_dev):
    """Word-list keys with binary words no topic level can equal -- <<"+">>,
    <<"#">>, words holding a '/' (make_key(Words, ID) with such binaries; the
    rule engine indexes unvalidated FROM topics, emqx_rule_engine.erl:534-540)
    -- reach the library in the escaped key form and take their place in
    matches_filter/3's term-ordered walk on the device, for byte and word-list
    queries (escaped words included), equal to the Python restatement of the
    reference's walk (oracle/pyoracle.py search_filter) over the same key set;
    deletes and re-inserts included.  They never match a topic, except that a
    '#' atom before the last word steers the ordered walk at its plain prefix
    as a plain '#'-not-last key does (NLIT_HDESC)."""
    from pyoracle import search_filter
    from emqx_amd.trie_search import HASH, PLUS, filter_words, key_order
    r = random.Random(0x454D5158 + 77)
    plain = [b"a", b"b", b"c", b"$s", b""]
    odd = [b"+", b"#", b"a/b", b"/", b"x/", b"\\", b"c\\/d"]

    def word(odd_p):
        c = r.random()
        if c < 0.2:
            return PLUS
        if c < 0.3:
            return HASH
        return r.choice(odd) if r.random() < odd_p else r.choice(plain)

    for seed in range(4):
        tab = ti.new()
        keys = []
        for i in range(400):
            ws = tuple(word(0.25) for _ in range(r.randint(1, 4)))
            k = ti.make_key(ws, i)
            keys.append(k)
            ti.insert(ws, i, None, tab)
        for i in range(400, 460):   # binary keys and []
            f = b"/".join(r.choice(plain) for _ in range(r.randint(1, 3)))
            keys.append(ti.make_key(f, i))
            ti.insert(f, i, None, tab)
        ti.insert((), 999, None, tab)
        keys.append(ti.make_key((), 999))

        def expect(q):
            live = sorted(set(tab.keys()), key=key_order)
            return ti._finish(search_filter(live, [key_order(k) for k in live], filter_words(q)), [])

        queries = [b"/".join(r.choice(plain + [b"+"]) for _ in range(r.randint(1, 4))) for _ in range(60)]
        queries += [b"#", b"a/#", b"+/+", b"$s/+", b"a/+/#"]
        queries += [tuple(word(0.3) for _ in range(r.randint(1, 4))) for _ in range(60)]   # word lists
        for q in queries:
            if not isinstance(q, bytes) and HASH in q[:-1]:
                continue   # (filter_words of a list: the caller's words as given; '#' only last in a filter)
            assert ti.matches_filter(q, tab) == expect(q), (seed, q)
        # deletes, then the same keys back
        gone = r.sample(keys, 150)
        for k in gone:
            ti.delete(k[0], k[1][0], tab)
        for q in queries[:40]:
            assert ti.matches_filter(q, tab) == expect(q), (seed, "after deletes", q)
        for k in gone:
            ti.insert(k[0], k[1][0], None, tab)
        for q in queries[:40]:
            assert ti.matches_filter(q, tab) == expect(q), (seed, "after re-inserts", q)
    # topic matching: the escaped keys never match; one with a '#' atom before
    # its last word cuts the walk at its plain prefix like 'a/#/z' would
    filters = [b"a/+", b"a/b/c", b"+/+/+", b"a/#", b"#"]
    fs = items_of(filters)
    ix = gpu_index(fs)
    e = ti.encode_words((b"a", HASH, b"x/y"))
    ix.apply(np.ones(2, np.uint8), *_native.pack_strings([e[0], b"q\\/r/+"]), np.array([100, 101], np.uint32),
             np.array([e[1], e[1]], np.uint8))
    o = oracle_of(items_of(filters + [b"a/#/z"], list(range(len(filters))) + [100]),
                  np.array([0] * len(filters) + [1], np.uint8))
    ts = items_of([b"a", b"a/b", b"a/b/c", b"q/r/s", b"q", b"x/y/z", b"a//"])
    assert_same(ix, o, ts)
    assert ix.stats()["n_dead_keys"] == 2


def test_matches_filter_does_not_stall_matching(torch_dev):
    """tm_matches_filter builds its term-ordered keys from a snapshot taken in
    slices of ~100 us under the index lock plus a log of key ops, and sorts /
    uploads / queries without the lock (it held the lock for ~1 s
    at 10M keys).  4 threads run 4k-topic match batches while matches_filter
    snapshots >= 1M word-list keys and, after deltas, rebuilds: the batches
    that overlap those calls complete with p99 < 1 ms."""
    import threading
    import time
    nf = 3_000_000
    fs = wl.filters(3, nf)
    ix = gpu_index(fs)
    nthreads, lb = 4, 4096
    ts = wl.topics(3, nf, nthreads * lb)
    lat, stop, errors = [], threading.Event(), []

    def caller(t):
        try:
            sub = items_of(ts.items()[t * lb:(t + 1) * lb])
            nb = int(sub.offs[-1])
            blob = ix.host_array(nb + 16, np.uint8)
            blob[:nb] = sub.blob[:nb]
            offs = ix.host_array(lb + 1, np.uint64)
            offs[:] = sub.offs
            bufs = (ix.host_array(lb + 1, np.uint64), ix.host_array(200_000, np.uint32), ix.host_array(lb, np.uint8))
            while not stop.is_set():
                t0 = time.perf_counter()
                ix.match_batch(blob, offs, out=bufs)
                lat.append((t0, time.perf_counter()))
        except BaseException as e:   # noqa: BLE001 - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    time.sleep(0.5)
    q = items_of([b"+/+/+/+", b"$SYS/#"])
    windows = []
    for rnd in range(2):
        if rnd:   # deltas between the calls: the second call replays the log and rebuilds
            d = wl.deltas(nf, 0, 20_000)
            ix.apply(d.flags, d.blob, d.offs, d.vals)
        t0 = time.perf_counter()
        hit, vals, err = ix.matches_filter_batch(q.blob, q.offs)
        windows.append((t0, time.perf_counter()))
        assert not err.any() and int(hit[-1]) > 0
    time.sleep(0.2)
    stop.set()
    for x in th:
        x.join(timeout=60)
    assert not errors, errors
    inside = np.array([(b - a) * 1e3 for a, b in lat if any(a < w1 and b > w0 for w0, w1 in windows)])
    wl_ms = [round((w1 - w0) * 1e3, 1) for w0, w1 in windows]
    st = ix.stats()
    print(f"matches_filter windows {wl_ms} ms over {st['n_wild_keys'] + st['n_dead_keys']} word-list keys; "
          f"{len(inside)} batches inside: p50 {np.percentile(inside, 50):.3f} p99 {np.percentile(inside, 99):.3f} ms")
    assert st["n_wild_keys"] >= 1_000_000
    assert min(wl_ms) > 50 and len(inside) >= 200       # the calls did real work while batches ran
    assert np.percentile(inside, 99) < 1.0


# ------------------------------------------------- sorted / unique output

def _sorted_ref(ohit, ovals, unique=False):
    """np.sort of every oracle list (and the distinct values, for UNIQUE)."""
    out, cnt = [], []
    for i in range(len(ohit) - 1):
        seg = np.sort(ovals[int(ohit[i]):int(ohit[i + 1])])
        if unique:
            u = np.unique(seg)
            cnt.append(len(u))
            seg = np.concatenate([u, np.full(len(seg) - len(u), 0xFFFFFFFF, np.uint32)])
        out.append(seg)
    return (np.concatenate(out) if out else np.zeros(0, np.uint32)), np.array(cnt, np.uint32)


@pytest.mark.parametrize("cfg", ["c1", "c3", "c5", "dup"])
def test_sorted_and_unique_orders_vs_oracle(torch_dev, cfg):
    """TM_ORDER_SORTED = np.sort of the oracle's lists; TM_ORDER_UNIQUE = their
    distinct values then 0xFFFFFFFF padding, with the distinct counts.  Host
    API (staged and in place) and device API.  "dup": values shared by many
    filters (the same ID on several filters), long lists (> 32 and > 8192
    values per topic) through the block sort."""
    import torch
    if cfg == "c1":
        fs, ts = wl.filters(1, 10_000), wl.topics(1, 10_000, 20_000)
        ix, o = gpu_index(fs), oracle_of(fs)
    elif cfg == "c3":
        fs, ts = wl.filters(3, 100_000), wl.topics(3, 100_000, 70_000)
        ix, o = gpu_index(fs), oracle_of(fs)
    elif cfg == "c5":
        fs, ts = wl.filters(5, 20_000), wl.topics(5, 20_000, 20_000)
        ix, o = gpu_index(fs), oracle_of(fs)
        for k in range(3):
            d = wl.deltas(20_000, k * 2_000, 2_000)
            ix.apply(d.flags, d.blob, d.offs, d.vals)
            o.apply(d.flags, d.blob, d.offs, d.vals)
        o.prepare()
    else:
        r = random.Random(3)
        filt, vals = [], []
        for i in range(20_000):   # many filters per topic, values drawn from a small range
            filt.append(b"d/" + b"/".join(r.choice([b"+", b"x%d" % r.randrange(3)]) for _ in range(r.randint(1, 4)))
                        + (b"/#" if r.random() < 0.5 else b""))
            vals.append(r.randrange(5_000))
        filt += [b"#"] * 9_000 + [b"d/#"] * 3_000
        vals += list(range(100_000, 109_000)) + list(range(3_000))
        fs = items_of(filt, vals)
        ix, o = gpu_index(fs), oracle_of(fs)
        ts = items_of([b"d/" + b"/".join(b"x%d" % r.randrange(3) for _ in range(r.randint(1, 5))) for _ in range(3000)]
                      + [b"e/1", b"d"])
    _, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    exp_s, _ = _sorted_ref(ohit, ovals)
    exp_u, exp_c = _sorted_ref(ohit, ovals, unique=True)
    n = len(ts)
    # host API, staged
    h, v, _ = ix.match_batch(ts.blob, ts.offs, order=_native.TM_ORDER_SORTED)
    assert np.array_equal(h, ohit.astype(np.uint64)) and np.array_equal(v, exp_s)
    uc = np.zeros(n, np.uint32)
    h, v, _ = ix.match_batch(ts.blob, ts.offs, order=_native.TM_ORDER_UNIQUE, unique_counts=uc)
    assert np.array_equal(v, exp_u) and np.array_equal(uc, exp_c)
    # host API, in place (tm_host_alloc buffers), batches <= 65536 topics
    if n <= 65536:
        nb = int(ts.offs[-1])
        pb, po = ix.host_array(nb + 16, np.uint8), ix.host_array(n + 1, np.uint64)
        pb[:nb] = ts.blob[:nb]
        po[:] = ts.offs
        bufs = (ix.host_array(n + 1, np.uint64), ix.host_array(len(ovals) + 8, np.uint32), ix.host_array(n, np.uint8))
        puc = ix.host_array(n, np.uint32)
        h, v, _ = ix.match_batch(pb, po, out=bufs, order=_native.TM_ORDER_UNIQUE, unique_counts=puc)
        assert np.array_equal(v, exp_u) and np.array_equal(puc, exp_c)
        h, v, _ = ix.match_batch(pb, po, out=bufs, order=_native.TM_ORDER_SORTED)
        assert np.array_equal(v, exp_s)
    # device API
    dev = torch.device("cuda:0")
    blob = torch.from_numpy(ts.blob).to(dev)
    offs = torch.from_numpy(ts.offs.view(np.int64)).to(dev)
    hit = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(n, dtype=torch.uint8, device=dev)
    out = torch.zeros(max(len(ovals), 1), dtype=torch.int32, device=dev)
    duc = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ix.match_batch_dev(n, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), out.data_ptr(), out.numel(),
                       err.data_ptr(), s, order=_native.TM_ORDER_UNIQUE, d_unique=duc.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32)[: len(ovals)], exp_u)
    assert np.array_equal(duc.cpu().numpy().view(np.uint32), exp_c)


@pytest.mark.parametrize("case", [c for c in GOLDEN["index_cases"]
                                  if any(ch["kind"] == "ids" and "unique" in ch["opts"] for ch in c["checks"])],
                         ids=lambda c: c["name"])
def test_unique_on_device_matches_golden(torch_dev, case):
    """[unique] on the device: the index stores the interned ID as the value
    (one u32 per distinct ID, ranked in term order, as a NIF interning IDs
    does); TM_ORDER_UNIQUE gives the distinct IDs ascending = the reference's
    [unique] IDs (maps:values of a small map, sorted by ID) --
    emqx_topic_index_SUITE t_match_unique / t_match_wildcard_edge_cases."""
    from emqx_amd.trie_search import filter as tfilter, term_key
    keys, _ = case_keys(case)
    ids = sorted({get_id(k) for k in keys}, key=term_key)
    rank = {i: r for r, i in enumerate(ids)}
    ix = _native.Index()
    enc = [encode_key(k) for k in keys]
    blob, offs = _native.pack_strings([e[0] for e in enc])
    ix.apply(np.ones(len(keys), np.uint8), blob, offs, np.array([rank[get_id(k)] for k in keys], np.uint32),
             np.array([e[1] for e in enc], np.uint8))
    for chk in case["checks"]:
        if chk["kind"] != "ids" or "unique" not in chk["opts"]:
            continue
        tb, to = _native.pack_strings([chk["topic"].encode()])
        uc = np.zeros(1, np.uint32)
        hit, vals, err = ix.match_batch(tb, to, order=_native.TM_ORDER_UNIQUE, unique_counts=uc)
        assert [ids[v] for v in vals[: int(uc[0])]] == chk["expect"], chk


def test_filter_sharded_sorted_merge_equals_one_index(torch_dev):
    """Shards' lists merged by tm_merge_shards, then sorted on the device by
    tm_sort_segments: list-equal (not only set-equal) to one index holding
    every key, in TM_ORDER_SORTED."""
    import torch
    from emqx_amd import shard
    nf, world = 60_000, 3
    ts = wl.topics(3, nf, 20_000)
    dev = torch.device("cuda:0")
    offs, vals = [], []
    for r in range(world):
        hit, v, _ = gpu_index(wl.filters(3, nf, shard=r, nshards=world)).match_batch(ts.blob, ts.offs)
        offs.append(hit.astype(np.int64))
        vals.append(v.view(np.int32))
    stride = max(len(v) for v in vals)
    all_vals = np.zeros((world, stride), np.int32)
    for r, v in enumerate(vals):
        all_vals[r, :len(v)] = v
    m_hit, m_vals = shard.merge(torch.from_numpy(np.stack(offs)).to(dev), torch.from_numpy(all_vals).to(dev), stride)
    one = gpu_index(wl.filters(3, nf))
    torch.cuda.synchronize()   # the merge ran on torch's stream; the sort runs on the index's own
    one.sort_segments(len(ts), m_hit.data_ptr(), m_vals.data_ptr(), m_vals.numel())
    torch.cuda.synchronize()
    h1, v1, _ = one.match_batch(ts.blob, ts.offs, order=_native.TM_ORDER_SORTED)
    mh = m_hit.cpu().numpy().view(np.uint64)
    assert np.array_equal(mh, h1)
    assert np.array_equal(m_vals.cpu().numpy().view(np.uint32)[: int(h1[-1])], v1)


def test_long_runs_emit_run_by_run(torch_dev):
    """Waves whose runs average >= 16 IDs take k_emit's run-by-run copy: runs of
    every length and alignment, single-ID (inline) runs between them, and
    topics with more than RCAP ranges (written by the re-walk, gaps in the
    wave's span) -- exact against the oracle."""
    rnd = random.Random(7)
    keys, vals = [], []
    v = 0
    filt = ["#", "a/#", "a/b/#", "a/b/c/#", "+/#", "+/b/#", "a/+/#", "+/+/#", "a/b/+/#", "+/+/+/#",
            "a/+/c/#", "+/b/c/#"]
    for f in filt:
        for _ in range(rnd.choice([1, 2, 3, 5, 17, 40, 250, 333])):
            keys.append(f); vals.append(v); v += 1
    for k in range(3000):
        keys.append(f"d/{k}/+"); vals.append(v); v += 1
        if k % 7 == 0:
            for _ in range(rnd.randint(2, 60)):
                keys.append(f"d/{k}/x"); vals.append(v); v += 1
    items = items_of([s.encode() for s in keys], vals)
    ix, o = gpu_index(items), oracle_of(items)
    tops = []
    for j in range(20_000):
        r = rnd.random()
        if r < 0.1:
            tops.append(b"a/b/c/d/e")          # > RCAP ranges: re-walked
        elif r < 0.2:
            tops.append(b"a/b/c")
        else:
            tops.append(b"d/%d/%s" % (rnd.randrange(3500), rnd.choice([b"x", b"y"])))
    assert_same(ix, o, items_of(tops))
    # the same batch on the device API with a torch stream (the bench's path)
    torch = torch_dev
    ts = items_of(tops)
    dev = torch.device("cuda:0")
    d_blob = torch.from_numpy(ts.blob).to(dev)
    d_offs = torch.from_numpy(ts.offs.view(np.int64)).to(dev)
    d_hit = torch.zeros(len(tops) + 1, dtype=torch.int64, device=dev)
    d_err = torch.zeros(len(tops), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ix.match_batch_dev(len(tops), d_blob.data_ptr(), d_offs.data_ptr(), d_hit.data_ptr(), 0, 0, d_err.data_ptr(), s)
    torch.cuda.synchronize()
    total = int(d_hit[-1])
    d_out = torch.zeros(total, dtype=torch.int32, device=dev)
    ix.match_batch_dev(len(tops), d_blob.data_ptr(), d_offs.data_ptr(), d_hit.data_ptr(), d_out.data_ptr(), total,
                       d_err.data_ptr(), s)
    torch.cuda.synchronize()
    _, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    assert np.array_equal(d_hit.cpu().numpy().view(np.uint64), ohit)
    assert np.array_equal(d_out.cpu().numpy().view(np.uint32), ovals)


@pytest.mark.parametrize("world", [2, 3])
def test_level0_shards_equal_one_index(torch_dev, world):
    """Level-0 filter sharding (bench --config c4l0): `world` shard indices on
    one GPU, each holding its first-level words' filters and the '+'/'#'-rooted
    ones; every topic matched on its owner's shard gives the unsharded
    oracle's list, order included."""
    from emqx_amd import shard
    fs = wl.filters(3, 200_000)
    ts = wl.topics(3, 200_000, 60_000)
    o = oracle_of(fs)
    _, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    m = shard.Level0Map.from_items(world, fs, sample=50_000)
    seen = np.zeros(len(ts), np.int64)
    for r in range(world):
        mine = wl.take(fs, m.filter_rows(fs, r))
        assert len(mine) < len(fs)
        ix = gpu_index(mine)
        rows = m.topic_rows(ts, r)
        seen[rows] += 1
        sub = wl.take(ts, rows)
        hit, vals, err = ix.match_batch(sub.blob, sub.offs)
        assert not err.any()
        for k, t in enumerate(rows.tolist()):
            assert np.array_equal(vals[hit[k]:hit[k + 1]], ovals[ohit[t]:ohit[t + 1]]), (r, ts.item(t))
    assert (seen == 1).all()


def test_level0_split_hot_prefix_on_device(torch_dev):
    """A tenant prefix with most of the publishes, split by its second level
    over 3 shard indices on one GPU (shard.Level0Map with a publish sample):
    every topic matched on its owner's shard gives the unsharded oracle's
    list, order included, in the one-launch and lane walks."""
    from emqx_amd import shard
    r = random.Random(0x454D5158 + 902)
    base = wl.filters(3, 50_000).items()
    hot = []
    for i in range(20_000):
        d = b"d%d" % r.randrange(3000)
        hot.append(r.choice([b"tnt/%s/+/x" % d, b"tnt/%s/#" % d, b"tnt/%s/s/%d" % (d, i % 7), b"tnt/%s" % d,
                             b"tnt/+/%s" % d]))
    hot += [b"tnt", b"tnt/#", b"tnt/+/s/#", b"tnt/+", b"tnt/", b"#", b"+/+/s/#"]
    fs = items_of(base + hot)
    tl = [b"tnt/d%d/%s" % (r.randrange(3000), r.choice([b"a/x", b"s/3", b"s", b"d7"])) for _ in range(200_000)]
    tl += wl.topics(3, 50_000, 20_000).items() + [b"tnt", b"tnt/", b"tnt//x"]
    ts = items_of(tl)
    o = oracle_of(fs)
    _, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    m = shard.Level0Map.from_items(3, fs, topics=ts)
    assert b"tnt" in m.split
    seen = np.zeros(len(ts), np.int64)
    for rk in range(3):
        ix = gpu_index(wl.take(fs, m.filter_rows(fs, rk)))
        rows = m.topic_rows(ts, rk)
        assert len(rows) < 0.45 * len(ts)
        seen[rows] += 1
        for part in (rows[:3000], rows):   # one launch / > 64k topics on the lane walk when big enough
            sub = wl.take(ts, part)
            hit, vals, err = ix.match_batch(sub.blob, sub.offs)
            assert not err.any()
            for k, t in enumerate(part.tolist()):
                assert np.array_equal(vals[hit[k]:hit[k + 1]], ovals[ohit[t]:ohit[t + 1]]), (rk, ts.item(t))
    assert (seen == 1).all()


def test_wide_node_bitmaps_follow_vocab_growth(torch_dev):
    """A wide node's bitmap must cover every word id: 40k new words arrive while
    it is wide (the bitmaps regrow), then children with those new ids are added
    and removed, the node turns dense (its children most of its level's words:
    the walk skips the bitmap) and back as another wide node's words come and
    go, and it drops back to its Bloom -- exact throughout."""
    ix, o = gpu_index(), Oracle()

    def put(strings, vals, op):
        d = items_of(strings, vals)
        ix.apply(np.full(len(d), op, np.uint8), d.blob, d.offs, d.vals)
        o.apply(np.full(len(d), op, np.uint8), d.blob, d.offs, d.vals)

    put([b"a/w%d/+" % i for i in range(300)], list(range(300)), 1)
    put([b"z/n%d" % k for k in range(40_000)], list(range(1000, 41_000)), 1)     # binary keys: new words
    new = list(range(0, 40_000, 97))
    put([b"a/n%d/+" % k for k in new], [50_000 + k for k in new], 1)            # children with the new ids
    r = random.Random(11)
    tops = [b"a/n%d/x" % r.randrange(40_000) for _ in range(3000)] + [b"a/w%d/y" % r.randrange(400) for _ in range(3000)]
    tops += [b"z/n%d" % r.randrange(41_000) for _ in range(1000)] + [b"a/never/x", b"a/z/x"]
    ts = items_of(tops)
    assert_same(ix, o, ts)
    assert ix.debug_get(_native.TM_DEBUG_WIDE_NODES) == 1
    assert ix.debug_get(_native.TM_DEBUG_DENSE_WIDE) == 1    # every level-1 word is a child of 'a': dense
    # 2,000 other level-1 words under 'b' (also wide): 'a' holds 713 of 2,713 -- its bitmap again
    put([b"b/v%d/+" % k for k in range(2000)], [60_000 + k for k in range(2000)], 1)
    assert ix.debug_get(_native.TM_DEBUG_WIDE_NODES) == 2
    assert ix.debug_get(_native.TM_DEBUG_DENSE_WIDE) == 1    # 'b' (2,000 of 2,713) is dense, 'a' is not
    ts2 = items_of(tops + [b"b/v%d/q" % r.randrange(2500) for _ in range(2000)])
    assert_same(ix, o, ts2)
    put([b"b/v%d/+" % k for k in range(2000)], [60_000 + k for k in range(2000)], 0)
    assert ix.debug_get(_native.TM_DEBUG_DENSE_WIDE) == 1    # 'a' dense again
    assert_same(ix, o, ts2)
    put([b"a/w%d/+" % i for i in range(300)], list(range(300)), 0)             # 713 -> 413 children: still wide
    assert_same(ix, o, ts)
    put([b"a/n%d/+" % k for k in new[:300]], [50_000 + k for k in new[:300]], 0)   # 113: the Bloom again
    assert ix.debug_get(_native.TM_DEBUG_WIDE_NODES) == 0
    assert_same(ix, o, ts)


def test_emit_misaligned_and_short_output_buffers(torch_dev):
    """Every emit path (run-by-run for long runs, the per-lane search for short
    ones) with an output buffer that is not 16-B aligned and with a capacity
    below the hit total: values up to the capacity equal the oracle's, and
    nothing is written past it."""
    torch = torch_dev
    rnd = random.Random(3)
    keys, vals, v = [], [], 0
    for f in ["#", "a/#", "+/b/#", "a/+/c/#", "+/+/+/#"]:
        for _ in range(rnd.choice([3, 37, 250])):
            keys.append(f); vals.append(v); v += 1
    for k in range(2000):
        keys.append(f"a/{k}/c/+"); vals.append(v); v += 1
    items = items_of([s.encode() for s in keys], vals)
    ix, o = gpu_index(items), oracle_of(items)
    tops = [b"a/%d/c/%d" % (rnd.randrange(2500), rnd.randrange(9)) for _ in range(3000)] + [b"x/b/c/d"] * 300
    ts = items_of(tops)
    _, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    total = int(ohit[-1])
    dev = torch.device("cuda:0")
    d_blob = torch.from_numpy(ts.blob).to(dev)
    d_offs = torch.from_numpy(ts.offs.view(np.int64)).to(dev)
    d_hit = torch.zeros(len(tops) + 1, dtype=torch.int64, device=dev)
    d_err = torch.zeros(len(tops), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    guard = 4096
    for shift, cap in [(1, total), (3, total), (0, total // 3 + 1), (1, total // 2 + 3)]:
        buf = torch.full((shift + total + guard,), -7, dtype=torch.int32, device=dev)
        ptr = buf.data_ptr() + 4 * shift              # 4-B aligned, not 16-B aligned for shift 1, 3
        ix.match_batch_dev(len(tops), d_blob.data_ptr(), d_offs.data_ptr(), d_hit.data_ptr(), ptr, cap,
                           d_err.data_ptr(), s)
        torch.cuda.synchronize()
        h = buf.cpu().numpy().view(np.uint32)
        assert np.array_equal(d_hit.cpu().numpy().view(np.uint64), ohit)
        assert np.array_equal(h[shift:shift + cap], ovals[:cap]), (shift, cap)
        assert (h[:shift] == np.uint32(0xFFFFFFF9)).all() and (h[shift + cap:] == np.uint32(0xFFFFFFF9)).all(), \
            (shift, cap, "written outside [0, cap)")


def test_wide_threshold_flapping_under_churn(torch_dev):
    """Nodes crossing the wide-node threshold (256 literal children) both ways,
    many times, under interleaved subscribes and unsubscribes -- bitmap, Bloom
    and child-table growth all rebuilt in place; exact against the oracle at
    every step."""
    rnd = random.Random(17)
    ix, o = gpu_index(), Oracle()
    live = set()
    tops = items_of([b"r%d/w%d/x" % (a, b) for a in range(3) for b in range(0, 400, 3)] +
                    [b"r%d/w%d" % (a, b) for a in range(3) for b in range(0, 400, 7)])
    for step in range(24):
        target = 300 if step % 2 == 0 else 200            # above / below 256 children
        ops, strs, vals = [], [], []
        for a in range(3):
            mine = sorted(k for k in live if k[0] == a)
            if len(mine) < target:
                for b in rnd.sample([b for b in range(400) if (a, b) not in live], target - len(mine)):
                    live.add((a, b)); ops.append(1); strs.append(b"r%d/w%d/+" % (a, b)); vals.append(a * 1000 + b)
            else:
                for (aa, b) in rnd.sample(mine, len(mine) - target):
                    live.discard((aa, b)); ops.append(0); strs.append(b"r%d/w%d/+" % (aa, b)); vals.append(aa * 1000 + b)
        d = items_of(strs, vals)
        op = np.array(ops, np.uint8)
        ix.apply(op, d.blob, d.offs, d.vals)
        o.apply(op, d.blob, d.offs, d.vals)
        assert_same(ix, o, tops)


def test_matches_filter_on_device_vs_oracle(torch_dev):
    """tm_matches_filter (the reference's ordered filter search on the device
    over the keys in term order) against the known answers derived from
    compare/3's clauses and against the C oracle on random key sets (binary
    keys, word-list keys, '+'/'#' anywhere in stored keys, '$' words)."""
    from test_matches_filter_cpu import KNOWN, _rand_filter
    for filters, query, expect in KNOWN:
        ix = gpu_index(items_of(filters))
        blob, offs = _native.pack_strings([query])
        hit, vals, err = ix.matches_filter_batch(blob, offs)
        assert vals.tolist() == expect and not err.any(), (filters, query)
    for seed in range(6):
        r = random.Random(0x454D5158 + 500 + seed)
        filters = [_rand_filter(r, r.randint(1, 5), [6, 2, 1]) for _ in range(300)]
        wf = np.array([1 if r.random() < 0.1 else 0 for _ in filters], np.uint8)
        items = items_of(filters)
        ix = gpu_index()
        ix.apply(np.ones(len(items), np.uint8), items.blob, items.offs, items.vals, wf)
        o = Oracle()
        for i, f in enumerate(filters):
            o.insert(f, i, int(wf[i]))
        qs = [_rand_filter(r, r.randint(1, 5), [4, 3, 1], hash_last=True) for _ in range(200)]
        blob, offs = _native.pack_strings(qs)
        hit, vals, err = ix.matches_filter_batch(blob, offs)
        assert not err.any()
        for i, q in enumerate(qs):
            assert vals[hit[i]:hit[i + 1]].tolist() == o.matches_filter(q), (seed, q)
    # deltas after a call: the term-ordered key array follows them
    ix = gpu_index(items_of([b"a/+/c", b"a/#"]))
    blob, offs = _native.pack_strings([b"a/+/c"])
    assert ix.matches_filter_batch(blob, offs)[1].tolist() == [1, 0]
    d = items_of([b"a/b/x/#", b"a/z/c/#"], [7, 9])
    ix.apply(np.ones(2, np.uint8), d.blob, d.offs, d.vals)
    # a/b/x/# is above a/+/c at the query's '+' level: the walk ends there and never reaches a/z/c/#
    assert ix.matches_filter_batch(blob, offs)[1].tolist() == [1, 0]
    d = items_of([b"a/b/x/#"], [7])
    ix.apply(np.zeros(1, np.uint8), d.blob, d.offs, d.vals)
    assert ix.matches_filter_batch(blob, offs)[1].tolist() == [1, 0, 9]


def test_ds_beamformer_waitq_known_answers(torch_dev):
    """emqx_ds_beamformer_waitq (the durable-storage consumer with a custom
    NextF, emqx_ds_beamformer_waitq.erl:43-62): per-stream matching on the
    device, pinned by the reference module's own topic_match_test (:66-105)."""
    from emqx_amd import waitq
    from emqx_amd.trie_search import PLUS
    tab = waitq.new()
    waitq.insert("s1", [b"foo", PLUS], 1, ("val", 1), tab)
    waitq.insert("s1", [b"foo", b"bar"], 2, ("val", 2), tab)
    waitq.insert("s1", [b"1", b"2"], 3, ("val", 3), tab)
    waitq.insert("s2", [b"foo", PLUS], 4, ("val", 4), tab)
    waitq.insert("s2", [b"foo", b"bar"], 5, ("val", 5), tab)
    waitq.insert("s2", [b"1", b"2"], 6, ("val", 6), tab)
    assert sorted(waitq.matches("s1", [b"foo", b"2"], tab)) == [("val", 1)]
    assert sorted(waitq.matches("s2", [b"foo", b"2"], tab)) == [("val", 4)]
    assert sorted(waitq.matches("s1", [b"foo", b"bar"], tab)) == [("val", 1), ("val", 2)]
    assert sorted(waitq.matches("s2", [b"foo", b"bar"], tab)) == [("val", 4), ("val", 5)]
    assert waitq.matches("s3", [b"foo", b"bar"], tab) == []
    assert waitq.matches("s1", [b"1", b"2"], tab) == [("val", 3)]
    assert waitq.matches("s2", [b"1", b"2"], tab) == [("val", 6)]
    # delete/4, and an insert of an existing key replaces its record (ets:insert on a set)
    waitq.delete("s1", [b"foo", PLUS], 1, tab)
    waitq.insert("s1", [b"foo", b"bar"], 2, ("val", 22), tab)
    assert sorted(waitq.matches("s1", [b"foo", b"bar"], tab)) == [("val", 22)]
    assert waitq.matches("s1", b"foo/2", tab) == []
    # the word list [] has no levels (b"" has one empty level): only [] and
    # ['#'] match it (compare/3, emqx_trie_search.erl:262-290) -- advisor r2
    from emqx_amd.trie_search import HASH
    for ident, words in ((7, []), (8, [HASH]), (9, [PLUS]), (10, [b""])):
        waitq.insert("s4", words, ident, ("val", ident), tab)
    assert waitq.matches("s4", [], tab) == [("val", 8), ("val", 7)]
    assert waitq.matches("s4", b"", tab) == [("val", 10), ("val", 9), ("val", 8)]
    assert waitq.matches("s4", [b""], tab) == [("val", 10), ("val", 9), ("val", 8)]


# ------------------------------------- '#' not last (tm_layout.h NLIT_HDESC)

def _hdesc_sets(seed, n_topics=60, deep=False):
    """Small alphabets so the cuts and seeks of '#'-not-last keys interact
    with '+' branches, terminals and binary keys (filters drawn from the
    topics, '#' at any level)."""
    r = random.Random(0x454D5158 + 700 + seed)

    def lvl():
        c = r.random()
        if c < 0.4:
            return r.choice([b"a", b"b", b"c"])
        if c < 0.5:
            return b""
        if c < 0.55:
            return b"$x"
        return b"%d" % r.randint(0, 3)

    hi = 40 if deep else 6
    topics = [b"/".join(lvl() for _ in range(r.randint(1, hi if r.random() < 0.3 else 6))) for _ in range(n_topics)]
    filters, flags = [], []
    for _ in range(r.randint(5, 60)):
        base = r.choice(topics).split(b"/")
        f = [r.choices([x, b"+", b"#", lvl()], [4, 2, 1, 1])[0] for x in base]
        if r.random() < 0.3:
            f.append(b"#")
        filters.append(b"/".join(f))
        flags.append(int(r.random() < 0.2))
    return topics, filters, np.array(flags, np.uint8)


def test_reference_quirk_hash_not_last_on_device(torch_dev):
    """The known answer of tests/test_oracle_golden.py::test_reference_quirk_hash_not_last
    on the device: '+/#/#' makes the reference's walk seek past '+/+//#' for
    topic 'E//' (compare/3 has no clause for a non-final '#',
    emqx_trie_search.erl:341-348); without it the filter matches."""
    for filters, exp in (([b"+/+//#", b"+/#/#"], []), ([b"+/+//#"], [0])):
        fs = items_of(filters)
        ix, o = gpu_index(fs), oracle_of(fs)
        for batch in (1, 9000, 70_000):   # one launch / lane walk
            ts = items_of([b"E//"] * batch)
            hit, vals = assert_same(ix, o, ts)
            assert vals[: hit[1]].tolist() == exp
        val, found = ix.first_batch(*_native.pack_strings([b"E//"]))
        assert found[0] == (1 if exp else 0)


@pytest.mark.parametrize("seed", range(12))
def test_hash_not_last_random_sets_vs_oracle(torch_dev, seed):
    """'#'-not-last keys in random sets: the seek past '+' and the cut at the
    topic's last level, through both walks (a batch of <= 64k topics takes
    the one-launch wave walk, a larger one the lane walk and its tail kernels
    -- LDS and, beyond 32 levels, global-scratch stores), match/2's first hit, and after
    deletes / re-inserts of those keys."""
    topics, filters, flags = _hdesc_sets(seed, deep=seed % 3 == 0)
    fs = items_of(filters)
    ix, o = gpu_index(fs, flags), oracle_of(fs, flags)
    small = items_of(topics)
    big = items_of(topics * (70_000 // len(topics) + 1))
    assert_same(ix, o, small)
    assert_same(ix, o, big)
    for ts in (small, big):
        val, found = ix.first_batch(ts.blob, ts.offs)
        for i in range(len(topics)):
            rc, v = o.first(ts.item(i))
            assert found[i] == {-1: 2, 0: 0, 1: 1}[rc], ts.item(i)
            if rc == 1:
                assert val[i] == v, ts.item(i)
    r = random.Random(seed)
    dele = sorted(r.sample(range(len(filters)), len(filters) // 2))
    d = items_of([filters[i] for i in dele], dele)
    for ops in (np.zeros(len(dele), np.uint8), np.ones(len(dele), np.uint8)):
        ix.apply(ops, d.blob, d.offs, d.vals, flags[dele])
        o.apply(ops, d.blob, d.offs, d.vals, flags[dele])
        assert_same(ix, o, small)
        assert_same(ix, o, big)


def test_hash_not_last_keys_leave_no_trie_behind(torch_dev):
    """A '#'-not-last key keeps the trie path of its prefix alive (its node
    holds the cut); deleting it prunes that path like any other key."""
    ix = gpu_index()
    base = ix.stats()
    keys = items_of([b"a/b/#/c", b"x/+/#/#", b"#/y"])
    ix.apply(np.ones(3, np.uint8), keys.blob, keys.offs, keys.vals)
    st = ix.stats()
    assert st["n_dead_keys"] == 3 and st["n_nodes"] > base["n_nodes"]
    ix.apply(np.ones(3, np.uint8), keys.blob, keys.offs, keys.vals)   # re-insert: no-op
    assert ix.stats()["n_nodes"] == st["n_nodes"]
    ix.apply(np.zeros(3, np.uint8), keys.blob, keys.offs, keys.vals)
    st2 = ix.stats()
    assert st2["n_dead_keys"] == 0 and st2["n_nodes"] == base["n_nodes"] and st2["n_words"] == base["n_words"]


# ---------------------------------- one host image, N replicas

def test_replicas_share_one_host_image(torch_dev):
    """tm_create_replicas with two replicas on device 0: one host key set and
    one tm_apply_deltas per delta batch feed both device copies; host batches
    alternate between them and each equals the oracle after every step of a C5
    delta replay; the 2-replica index costs the host about what 1 does."""
    import gc
    import psutil
    nf = 20_000
    fs = wl.filters(5, nf)
    ix = _native.Index(devices=[0, 0])
    ix.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    o = oracle_of(fs)
    ts = wl.topics(5, nf, 6_000)
    st0 = ix.stats()
    for k in range(4):
        d = wl.deltas(nf, k * 2_000, 2_000)
        ix.apply(d.flags, d.blob, d.offs, d.vals)
        o.apply(d.flags, d.blob, d.offs, d.vals)
        o.prepare()
        before = [ix.replica_stats(r)[0] for r in (0, 1)]
        for _ in range(2):   # consecutive host batches: one per replica (round robin)
            assert_same(ix, o, ts)
        after = [ix.replica_stats(r)[0] for r in (0, 1)]
        assert [a - b for a, b in zip(after, before)] == [1, 1], (before, after)
    st = ix.stats()
    assert st["n_keys"] == o.size() and st["uploads"] > st0["uploads"]   # one host key set, patched on both
    ix.close()

    def build(devices):
        gc.collect()
        r0 = psutil.Process().memory_info().rss
        big = wl.filters(3, 400_000)
        x = _native.Index(devices=devices, hint_keys=len(big))
        x.apply(np.ones(len(big), np.uint8), big.blob, big.offs, big.vals)
        x.match_batch(ts.blob, ts.offs)        # both replicas uploaded (first sync)
        x.match_batch(ts.blob, ts.offs)
        del big
        gc.collect()
        rss = psutil.Process().memory_info().rss - r0
        dev_bytes = x.stats()["device_bytes"]
        x.close()
        return rss, dev_bytes
    build([0, 0])   # one-time runtime allocations (a second replica's streams, pinned pools) land here
    one, db1 = build([0])
    two, db2 = build([0, 0])
    print(f"host RSS growth: 1 replica {one / 2**20:.0f} MiB, 2 replicas {two / 2**20:.0f} MiB "
          f"(device {db1 / 2**20:.0f} MiB per replica)")
    assert db1 == db2 and two <= 1.2 * one + (32 << 20)


# ------------- small batches: k_walk_small with 16 / 8 lanes per topic (rounds 3-6)

def _paths(ix):
    """match launches so far per kernel path: (two-phase, k_walk_small, retired lane kernel: 0)"""
    return tuple(ix.debug_get(k) for k in (_native.TM_DEBUG_PATH_PHASES, _native.TM_DEBUG_PATH_SMALL,
                                           _native.TM_DEBUG_PATH_LANE))


def _shallow_case(r, nt=700):
    """Filters of at most 6 levels (trie depth <= 6, binary keys <= 6 levels:
    the LITE fallback store's index condition, lite_path_ok), topics of 1-14
    levels (the ones deeper than 8 levels take k_walk_small<8>'s lite
    fallback walk), dense
    wildcard families over some prefixes (topics with more than RCAP = 8 value
    ranges: re-walked), filters with several IDs (multi-value runs)."""
    def lvl():
        c = r.random()
        if c < 0.1:
            return b""
        if c < 0.15:
            return b"$" + r.choice([b"SYS", b"a"])
        if c < 0.2:
            return r.choice([b"b+", b"c#", b"a-very-long-level-word-over-16-bytes"])
        return ("%X" % r.randint(1, 12)).encode()
    topics = [b"/".join(lvl() for _ in range(r.choice([1, 2, 3, 4, 5, 6, 6, 9, 12, 14]))) for _ in range(nt)]
    topics += [b"a/+/b", b"#", b"", b"/", b"$SYS", b"1/2/3/4/5/6/7/8/9/10/+/12", b"/" * 65536]   # badarg deep, > 65536 levels
    filters, vals = [], []
    for _ in range(900):
        ws = r.choice(topics[:nt]).split(b"/")[:6]
        out = []
        for k, w in enumerate(ws):
            p = r.choices(["w", "+", "#"], [5, 2, 1])[0]
            if p == "#" or (k == len(ws) - 1 and r.random() < 0.2 and k < 5):
                out.append(b"#")
                break
            out.append(b"+" if p == "+" else w)
        filters.append(b"/".join(out))
        vals.append(len(vals))
    for t in r.sample(topics[:nt], 12):   # every '+' / '#' variant of a prefix: > RCAP ranges per topic
        ws = t.split(b"/")[:4]
        for m in range(1 << len(ws)):
            f = [b"+" if (m >> k) & 1 else w for k, w in enumerate(ws)]
            for g in (f, f[:-1] + [b"#"], f + [b"#"]):
                if len(g) <= 6:
                    filters.append(b"/".join(g))
                    vals.append(len(vals))
    for f in r.sample(filters, 60):   # several IDs on one filter: multi-value runs
        for _ in range(r.randint(2, 40)):
            filters.append(f)
            vals.append(len(vals))
    return filters, vals, topics


def _all_kernels(ix, ts):
    """the batch on k_walk_small with 16 and 8 lanes per topic and the
    two-phase path: -> (hit, vals, err) of each, and the paths they took"""
    out = []
    for kind, phases in ((_native.SMALL_WAVE, 0), (_native.SMALL_WAVE8, 0), (_native.SMALL_AUTO, 1)):
        ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, kind)
        ix.debug_set(_native.TM_DEBUG_PHASES, phases)
        p0 = _paths(ix)
        out.append((ix.match_batch(ts.blob, ts.offs), tuple(b - a for a, b in zip(p0, _paths(ix)))))
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _native.SMALL_AUTO)
    ix.debug_set(_native.TM_DEBUG_PHASES, 0)
    return out


@pytest.mark.parametrize("seed", range(8))
def test_small_walks_vs_oracle_and_the_two_phase_path(torch_dev, seed):
    """Small batches on a shallow index run in ONE launch of k_walk_small
    with 16 or 8 lanes per topic (the 8-lane groups' fallbacks: more than 8
    levels or frontier states, the LITE store): exact CSR against the oracle
    and bit-identical to each other and to the two-phase path forced on the
    same batch -- topics deeper than the main store, badarg beyond it, more
    than 65536 levels, more than RCAP ranges, multi-value runs -- at batch
    sizes around a block's 64 topics and up to 65536; after deletes and
    re-inserts too; host, device and 32-bit APIs."""
    torch = torch_dev
    r = random.Random(0x454D5158 + 400 + seed)
    filters, vals, topics = _shallow_case(r)
    flags = np.array([r.random() < 0.2 for _ in filters], np.uint8)
    fs = items_of(filters, vals)
    ix, o = gpu_index(fs, flags), oracle_of(fs, flags)
    for n in (1, 63, 64, 65, 129, 3_000, 65_536):
        ts = items_of([topics[i % len(topics)] for i in r.sample(range(2 * n + 7), n)])
        runs = _all_kernels(ix, ts)
        # (a first run may be repeated to size the values buffer: capacity reruns)
        assert [tuple(x > 0 for x in p) for _, p in runs] == [(0, 1, 0), (0, 1, 0), (1, 0, 0)], \
            [p for _, p in runs]
        (hit, v1, e1), _ = runs[0]
        assert_same(ix, o, ts)
        for (h, v, e), _ in runs[1:]:
            assert np.array_equal(hit, h) and np.array_equal(v1, v) and np.array_equal(e1, e)
    assert np.diff(hit.astype(np.int64)).max() > 8 * 2        # some topic beyond RCAP ranges
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _native.SMALL_WAVE8)   # 8 lanes per topic from here on
    # device API on a torch stream
    d_blob, d_offs = torch.from_numpy(ts.blob).cuda(), torch.from_numpy(ts.offs.view(np.int64)).cuda()
    d_hit = torch.zeros(len(ts) + 1, dtype=torch.int64, device="cuda")
    d_err = torch.zeros(len(ts), dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(int(hit[-1]) + 1, dtype=torch.int32, device="cuda")
    p0 = _paths(ix)
    ix.match_batch_dev(len(ts), d_blob.data_ptr(), d_offs.data_ptr(), d_hit.data_ptr(), d_out.data_ptr(),
                       int(hit[-1]) + 1, d_err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert _paths(ix)[1] > p0[1]
    assert np.array_equal(d_hit.cpu().numpy().view(np.uint64), hit)
    assert np.array_equal(d_out.cpu().numpy().view(np.uint32)[: int(hit[-1])], v1)
    # the 32-bit in-place API (the NIF's): through the combiner
    nb = int(ts.offs[-1])
    blob = ix.host_array(nb + 16, np.uint8)
    blob[:nb] = ts.blob[:nb]
    offs = ix.host_array(len(ts) + 1, np.uint32)
    offs[:] = ts.offs.astype(np.uint32)
    out = (ix.host_array(len(ts) + 1, np.uint32), ix.host_array(int(hit[-1]) + 16, np.uint32),
           ix.host_array(len(ts), np.uint8))
    p0 = _paths(ix)
    h32, v32, e32 = ix.match_batch32(blob, offs, out)
    assert _paths(ix)[1] > p0[1]
    assert np.array_equal(h32.astype(np.uint64), hit) and np.array_equal(v32, v1) and np.array_equal(e32, e1)
    # deletes and re-inserts as deltas
    dele = sorted(r.sample(range(len(filters)), len(filters) // 4))
    d = items_of([filters[i] for i in dele], [vals[i] for i in dele])
    ix.apply(np.zeros(len(dele), np.uint8), d.blob, d.offs, d.vals, flags[dele])
    o.apply(np.zeros(len(dele), np.uint8), d.blob, d.offs, d.vals, flags[dele])
    assert_same(ix, o, ts)
    back = dele[::2]
    d2 = items_of([filters[i] for i in back], [vals[i] for i in back])
    ix.apply(np.ones(len(back), np.uint8), d2.blob, d2.offs, d2.vals, flags[back])
    o.apply(np.ones(len(back), np.uint8), d2.blob, d2.offs, d2.vals, flags[back])
    p2 = _paths(ix)
    assert_same(ix, o, ts)
    assert _paths(ix)[1] > p2[1]


@pytest.mark.parametrize("kind", ["wave", "wave8"])
def test_small_walk_long_topics(torch_dev, kind):
    """A block whose topics span more than k_walk_small stages in LDS at once
    stages a row per topic; a topic longer than its row is walked by its
    group's first lane (block-uniform choices; blocks of a batch may take
    either way).  Exact against the oracle, in place too (the topics then come
    over PCIe)."""
    r = random.Random(0x454D5158 + 450)
    words = [b"w%d" % i for i in range(30)] + [b"long-" + b"x" * 90, b"$SYS"]
    filters = [b"/".join(r.choice(words) if r.random() < 0.7 else b"+" for _ in range(r.randint(1, 5)))
               for _ in range(3_000)] + [b"#", b"w1/#", b"+/+/#"]
    fs = items_of(filters)
    ix, o = gpu_index(fs), oracle_of(fs)
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _small_kind(kind))
    topics = []
    for i in range(5_000):
        blk = (i // 64) % 3   # blocks of short topics, of ~180-byte topics, and mixed
        long_ = blk == 1 or (blk == 2 and i % 2)
        lv = [r.choice(words[-2:] if long_ and k < 2 else words) for k in range(r.randint(1, 6))]
        topics.append(b"/".join(lv))
    ts = items_of(topics)
    assert max(int(ts.offs[(b + 1) * 64] - ts.offs[b * 64]) for b in range(len(ts) // 64)) > 4096
    p0 = _paths(ix)
    hit, v = assert_same(ix, o, ts)
    assert _paths(ix)[1] > p0[1]
    nb = int(ts.offs[-1])
    blob = ix.host_array(nb + 16, np.uint8)
    blob[:nb] = ts.blob[:nb]
    offs = ix.host_array(len(ts) + 1, np.uint32)
    offs[:] = ts.offs.astype(np.uint32)
    out = (ix.host_array(len(ts) + 1, np.uint32), ix.host_array(int(hit[-1]) + 16, np.uint32),
           ix.host_array(len(ts), np.uint8))
    h32, v32, _ = ix.match_batch32(blob, offs, out)
    assert np.array_equal(h32.astype(np.uint64), hit) and np.array_equal(v32, v)


def test_small_walk_c3deep_and_index_gates(torch_dev):
    """C3deep batches (10 % of the topics 33-64 levels) on k_walk_small with 8
    lanes per topic (the deep topics on the LITE fallback walk); an index a
    topic could need more than MID_L levels of (a binary key of 40 levels: the
    two-phase path) or with a '#'-not-last key (16 lanes per topic, the full
    fallback store) takes another kernel shape, exact either way."""
    fs = wl.filters(3, 200_000)
    ts = wl.topics(30, 200_000, 60_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _native.SMALL_WAVE8)
    p0 = _paths(ix)
    assert_same(ix, o, ts)
    assert _paths(ix)[1] > p0[1]
    for extra in ([b"/".join([b"z"] * 40)], [b"a/#/b"]):   # deep binary key / '#'-not-last key
        e = items_of(extra, [1_000_000])
        ix.apply(np.ones(1, np.uint8), e.blob, e.offs, e.vals)
        o.apply(np.ones(1, np.uint8), e.blob, e.offs, e.vals)
        p0 = _paths(ix)
        assert_same(ix, o, ts)
        # (the 40-level binary key is beyond k_walk_small's fallback store too: the two phases)
        assert _paths(ix)[0 if len(extra[0]) > 40 else 1] > p0[0 if len(extra[0]) > 40 else 1]
        assert _paths(ix)[2] == p0[2] == 0
        ix.apply(np.zeros(1, np.uint8), e.blob, e.offs, e.vals)
        o.apply(np.zeros(1, np.uint8), e.blob, e.offs, e.vals)
    p0 = _paths(ix)
    assert_same(ix, o, ts)
    assert _paths(ix)[1] > p0[1]


# ------------------------------------- device failures are not badarg (round 4)

@pytest.mark.parametrize("kind,ticket", [("wave", 0), ("wave8", 0), ("wave8", 1)])
def test_lookback_failure_is_retried_then_a_device_error(torch_dev, kind, ticket):
    """A one-launch small batch (k_walk_small, 16 or 8 lanes per topic) whose look-back
    wait expires (forced: block 3 acts as if its wait expired,
    TM_DEBUG_LB_FAIL_BLOCK) flags err 4 from that block on (LB_FAIL
    propagates: no later block takes a partial prefix), the host API runs it
    again once -- exact results -- and a second failure is a device error for
    the whole call: TM_EDEVICE / DeviceError, never BadArg (the reference
    raises badarg only for a '+'/'#' level, emqx_trie_search.erl:374-375;
    VERDICT r3 item 1)."""
    torch = torch_dev
    nt = 5_000
    fs = wl.filters(3, 50_000)
    ts = wl.topics(3, 50_000, nt)
    ix, o = gpu_index(fs), oracle_of(fs)
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _small_kind(kind))
    ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, ticket)   # (the failing block is then virtual block 3)
    p0 = _paths(ix)
    assert_same(ix, o, ts)
    assert _paths(ix)[1] > p0[1]
    f0, r0 = ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES), ix.debug_get(_native.TM_DEBUG_RETRIED_BATCHES)
    assert f0 == 0 and r0 == 0                       # a normal run never fails
    ix.debug_set(_native.TM_DEBUG_LB_FAIL_BLOCK, 3)
    ix.debug_set(_native.TM_DEBUG_LB_LAUNCHES, 1)    # the first launch fails, the retry succeeds
    assert_same(ix, o, ts)
    assert ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES) == 1
    assert ix.debug_get(_native.TM_DEBUG_RETRIED_BATCHES) == 1
    ix.debug_set(_native.TM_DEBUG_LB_LAUNCHES, 2)    # both fail: a device error
    with pytest.raises(_native.DeviceError):
        ix.match_batch(ts.blob, ts.offs)
    assert ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES) == 3
    # the topic_index mirror raises DeviceError (not BadArg) for a valid topic
    tab = ti.Tab(index=ix)
    tab._keys = [None] * (int(fs.vals.max()) + 1)
    ix.debug_set(_native.TM_DEBUG_LB_LAUNCHES, 2)
    with pytest.raises(_native.DeviceError):
        ti.matches_batch([ts.item(i) for i in range(nt)], tab)
    # device API (asynchronous: no retry): err 4 from the failed block on, 0 before
    ix.debug_set(_native.TM_DEBUG_LB_LAUNCHES, 1)
    d_blob, d_offs = torch.from_numpy(ts.blob).cuda(), torch.from_numpy(ts.offs.view(np.int64)).cuda()
    d_hit = torch.zeros(nt + 1, dtype=torch.int64, device="cuda")
    d_err = torch.zeros(nt, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(16 * nt, dtype=torch.int32, device="cuda")
    ix.match_batch_dev(nt, d_blob.data_ptr(), d_offs.data_ptr(), d_hit.data_ptr(), d_out.data_ptr(), 16 * nt,
                       d_err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    err = d_err.cpu().numpy()
    first = 3 * {"wave": 16, "wave8": 32}[kind]   # topics per block
    assert not err[:first].any() and (err[first:] == 4).all()
    # the hook is spent: the next batches are exact again, with no failure
    assert_same(ix, o, ts)
    assert ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES) == 5


@pytest.mark.parametrize("kind,ticket", [("wave", 0), ("wave8", 0), ("wave8", 1)])
def test_lookback_without_waiting_is_exact_or_a_device_error(torch_dev, kind, ticket):
    """With no wait at all (TM_DEBUG_LB_SPINS 0: a block fails whenever a
    predecessor has not published yet), every batch either matches exactly or
    fails as a device error -- never a wrong result, never BadArg."""
    fs = wl.filters(3, 50_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _small_kind(kind))
    ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, ticket)
    for nt in (3_000, 30_000, 65_536):
        ts = wl.topics(3, 50_000, nt)
        ix.debug_set(_native.TM_DEBUG_LB_SPINS, 0)
        ix.debug_set(_native.TM_DEBUG_LB_LAUNCHES, 2)
        try:
            assert_same(ix, o, ts)
        except _native.DeviceError:
            pass
        ix.debug_set(_native.TM_DEBUG_LB_LAUNCHES, 0)
        ix.debug_set(_native.TM_DEBUG_LB_SPINS, 1 << 22)
        assert_same(ix, o, ts)


def test_router_boot_1m_routes_and_node_down_cleanup(torch_dev):
    """The deployment's boot and node-down paths at size:
    1M routes of an existing table set (C3-shaped filters; exact topics in the
    bag, wildcard ones in the index, destinations on four nodes and shared
    groups) booted into the device mirror in batches of at most 1000 keys,
    then one node's routes deleted as mria's match_delete would replicate
    them -- delete table events, drained 1000 at a time (emqx_router.erl:
    535-550, src/emqx_router_gpu.erl).  match_routes equals the CPU model +
    oracle (harness.RouterModel) after each."""
    from emqx_amd.trie_search import filter as tfilter
    nodes = ["n1", "n2", "n3", (b"grp", "n2"), (b"grp", "n4")]
    fs = wl.filters(3, 1_000_000)
    model = RouterModel()
    route_rows, filter_rows, routes, seen = [], [], [], set()
    for i in range(len(fs)):
        t, d = fs.item(i), nodes[i % len(nodes)]
        if (t, d) in seen:
            continue
        seen.add((t, d))
        routes.append((t, d))
        model.add(t, d)
        if tfilter(t) is not False:
            filter_rows.append(rt.RouteIdx(ti.make_key(t, d)))
        else:
            route_rows.append(rt.Route(t, d))
    filter_rows.sort(key=lambda r: ti.key_order(r.entry))
    r = rt.Router(node="n1")
    calls = r.attach(route_rows, filter_rows, batch_size=1000)
    assert calls == (len(filter_rows) + 999) // 1000   # the bag stays on the host
    assert r.mirror_keys() == len(filter_rows)
    ts = wl.topics(3, 1_000_000, 4_000)
    topics = [ts.item(i) for i in range(len(ts))]
    topics += [routes[i][0] for i in range(0, len(routes), 997) if tfilter(routes[i][0]) is False][:500]
    assert r.match_routes_batch(topics) == model.expected(topics)
    # node n2 goes down: mria's match_delete on both tables, reaching the
    # mirror as record-form delete events, drained 1000 at a time
    dead = [(t, d) for t, d in routes if rt.get_dest_node(d) == "n2"]
    r.cleanup_routes("n2")
    assert r.pending_events() == len(dead)
    while r.pending_events():
        r.drain_events(limit=1000)
    for t, d in dead:
        model.delete(t, d)
    got = r.match_routes_batch(topics)
    assert got == model.expected(topics)
    assert all(rt.get_dest_node(x.dest) != "n2" for rs in got for x in rs)
    assert r.mirror_keys() == len(filter_rows) - sum(1 for t, _ in dead if tfilter(t) is not False)


@pytest.mark.parametrize("kind,land,ticket", [("wave", 0, 0), ("wave8", 0, 0), ("auto", 0, 0), ("auto", 0, 1)])
def test_combined_small_batches_equal_single_launches(torch_dev, kind, land, ticket):
    """The host-batch combiner (tm_host.cpp small_combined): concurrent callers'
    in-place 32-bit batches of 1 to 20k topics run as shared k_walk_small
    launches with a segment table (land: 0 -- the landing variant was removed
    in round 6) -- each caller's hit offsets,
    values and flags identical to its batch run alone (combiner off) and to
    the oracle; a badarg topic stays in its own slot; a forced look-back
    failure reruns the whole launch once (every caller still exact)."""
    import threading
    fs = wl.filters(3, 200_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _small_kind(kind))
    sizes = [1, 7, 100, 640, 3000, 4096, 9000, 20_000]
    sets = []
    for k, nt in enumerate(sizes):
        ts = wl.topics(3, 200_000, nt, first=k * 50_000)
        items = [ts.item(i) for i in range(nt)]
        if nt >= 100:
            items[nt // 2] = b"bad/+/topic"   # badarg in its own slot
        blob, offs = _native.pack_strings(items)
        pb = ix.host_array(len(blob) + 16, np.uint8)
        pb[: len(blob)] = blob
        po = ix.host_array(nt + 1, np.uint32)
        po[:] = offs.astype(np.uint32)
        cap = 64 * nt + 64
        outs = [(ix.host_array(nt + 1, np.uint32), ix.host_array(cap, np.uint32), ix.host_array(nt, np.uint8))
                for _ in range(2)]
        sets.append((pb, po, outs, items))
    # alone: combiner off, then the oracle
    ix.debug_set(_native.TM_DEBUG_COMBINE, 0)
    ref = []
    for pb, po, outs, items in sets:
        h, v, e = ix.match_batch32(pb, po, outs[0])
        ref.append((h.copy(), v.copy(), e.copy()))
        bl, of = _native.pack_strings(items)
        oc, _, ohit, ovals = o.match_batch(bl, of)
        for i in range(len(items)):
            if e[i]:
                assert b"+" in items[i] or b"#" in items[i]
                continue
            assert np.array_equal(v[h[i]:h[i + 1]], ovals[int(ohit[i]):int(ohit[i + 1])])
    ix.debug_set(_native.TM_DEBUG_COMBINE, 3)
    ix.debug_set(_native.TM_DEBUG_CMB_LAND, land)
    ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, ticket)
    l0 = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES)
    b0 = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES)
    errors = []

    def caller(k, rounds, bar):
        pb, po, outs, _ = sets[k]
        try:
            for _ in range(rounds):
                if bar is not None:
                    bar.wait(timeout=30)
                h, v, e = ix.match_batch32(pb, po, outs[1])
                rh, rv, re_ = ref[k]
                if not (np.array_equal(h, rh) and np.array_equal(v, rv) and np.array_equal(e, re_)):
                    errors.append(k)
                    return
        except Exception as ex:   # noqa: BLE001 -- reported below
            errors.append((k, repr(ex)))

    def run(rounds, together=False):
        # together: every round starts at a barrier, so the callers enter the
        # library within a few us of each other (their Python result checks
        # hold the GIL for far longer than a launch takes, so free-running
        # callers seldom overlap in the library)
        bar = threading.Barrier(len(sets)) if together else None
        th = [threading.Thread(target=caller, args=(k, rounds, bar)) for k in range(len(sets))]
        for t in th:
            t.start()
        for t in th:
            t.join()

    run(40)   # up to 3 leaders: whether callers queue depends on kernel speed
    ix.debug_set(_native.TM_DEBUG_COMBINE, 1)
    run(20, together=True)   # one leader: the other callers queue behind its launch
    ix.debug_set(_native.TM_DEBUG_COMBINE, 3)
    assert not errors, errors
    launches = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES) - l0
    batches = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES) - b0
    assert batches == 60 * len(sets) and launches < batches, (launches, batches)   # some launches carried several
    # a forced look-back failure in the next combined launch: rerun, exact
    f0 = ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES)
    ix.debug_set(_native.TM_DEBUG_LB_FAIL_BLOCK, 0)   # (block 0 of every segment)
    ix.debug_set(_native.TM_DEBUG_LB_LAUNCHES, 1)
    run(3)
    assert not errors, errors
    assert ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES) == f0 + 1


def test_vram_inputs_equal_host_buffers(torch_dev):
    """TM_ALLOC_VRAM (include/tmatch.h tm_host_alloc_ex): a batch whose topic
    bytes and offsets live in device memory mapped into the host -- written by
    the host, never read back by this test -- runs in place on the NIF's u32
    entry point, alone and through the combiner (concurrent callers, deltas in
    between), with offsets, values and flags identical to the same batch in
    tm_host_alloc memory, which the oracle checks.  Freed by tm_host_free."""
    import threading
    fs = wl.filters(3, 200_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    sets = []
    for k, nt in enumerate([1, 100, 4096, 9000, 65536]):
        ts = wl.topics(3, 200_000, nt, first=k * 70_000)
        items = [ts.item(i) for i in range(nt)]
        if nt >= 100:
            items[nt // 3] = b"x/#/y"   # badarg in its own slot
        blob, offs = _native.pack_strings(items)
        vb = ix.host_array(len(blob) + 16, np.uint8, vram=True)
        vb[: len(blob)] = blob
        vo = ix.host_array(nt + 1, np.uint32, vram=True)
        vo[:] = offs.astype(np.uint32)
        hb = ix.host_array(len(blob) + 16, np.uint8)
        hb[: len(blob)] = blob
        ho = ix.host_array(nt + 1, np.uint32)
        ho[:] = offs.astype(np.uint32)
        cap = 64 * nt + 64
        outs = [(ix.host_array(nt + 1, np.uint32), ix.host_array(cap, np.uint32), ix.host_array(nt, np.uint8))
                for _ in range(2)]
        sets.append((vb, vo, hb, ho, outs, items, blob, offs))
    ref = []
    for vb, vo, hb, ho, outs, items, blob, offs in sets:
        h, v, e = ix.match_batch32(hb, ho, outs[0])
        ref.append((h.copy(), v.copy(), e.copy()))
        oc, _, ohit, ovals = o.match_batch(blob, offs)
        for i in range(len(items)):
            if e[i]:
                assert b"+" in items[i] or b"#" in items[i]
                continue
            assert np.array_equal(v[h[i]:h[i + 1]], ovals[int(ohit[i]):int(ohit[i + 1])])
        h2, v2, e2 = ix.match_batch32(vb, vo, outs[1])   # alone
        assert np.array_equal(h2, h) and np.array_equal(v2, v) and np.array_equal(e2, e)
    errors = []

    def caller(k):
        vb, vo, _, _, outs, _, _, _ = sets[k]
        try:
            for _ in range(20):
                h, v, e = ix.match_batch32(vb, vo, outs[1])
                rh, rv, re_ = ref[k]
                if not (np.array_equal(h, rh) and np.array_equal(v, rv) and np.array_equal(e, re_)):
                    errors.append(k)
                    return
        except Exception as ex:   # noqa: BLE001 -- reported below
            errors.append((k, repr(ex)))

    lead0 = ix.debug_get(_native.TM_DEBUG_COMBINE)
    ix.debug_set(_native.TM_DEBUG_COMBINE, 1)
    l0 = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES)
    b0 = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES)
    th = [threading.Thread(target=caller, args=(k,)) for k in range(len(sets))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ix.debug_set(_native.TM_DEBUG_COMBINE, lead0)
    assert not errors, errors
    assert ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES) - b0 == 20 * len(sets)
    assert ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES) - l0 < 20 * len(sets)
    # a delta between two batches: the VRAM batch sees it as the host one does
    new = b"/".join(bytes(w) for w in sets[2][5][0].split(b"/")[:2]) + b"/#"
    ix.apply(np.ones(1, np.uint8), *_native.pack_strings([new]), np.array([0xABCDEF], np.uint32))
    vb, vo, hb, ho, outs, _, _, _ = sets[2]
    h, v, e = ix.match_batch32(hb, ho, outs[0])
    h = h.copy(); v = v.copy(); e = e.copy()
    assert 0xABCDEF in v
    h2, v2, e2 = ix.match_batch32(vb, vo, outs[1])
    assert np.array_equal(h2, h) and np.array_equal(v2, v) and np.array_equal(e2, e)
    # match/2 (tm_first_batch) the way the NIF runs it (tmn_first): topic bytes
    # in device memory, u64 offsets and the outputs in pinned host memory
    vb, vo, hb, ho, outs, items, blob, offs = sets[2]
    nt = len(items)
    o64 = ix.host_array(nt + 1, np.uint64)
    o64[:] = offs
    val = ix.host_array(nt, np.uint32)
    found = ix.host_array(nt, np.uint8)
    ix._check(ix._lib.tm_first_batch(ix._h, nt, _native._ptr(vb), _native._ptr(o64), _native._ptr(val),
                                     _native._ptr(found)))
    rv, rf = ix.first_batch(blob, offs)
    assert np.array_equal(val, rv) and np.array_equal(found, rf)
    for a_ in (vb, vo):
        ix.host_free(a_)


@pytest.mark.parametrize("nt", [1, 3000, 65536, 70_000])
def test_u32_offsets_api_equals_u64(torch_dev, nt):
    """tm_match_batch32_ex / tm_match_batch32_dev: u32 topic
    offsets in, u32 hit offsets out -- in place from tm_host_alloc buffers (the
    one-launch kernel on 32-bit offsets, up to 65536 topics), staged host
    buffers, and device buffers (widened and narrowed on the device above
    65536) -- identical to the u64 API and the oracle; TM_ECAP with valid
    offsets when the values do not fit."""
    torch = torch_dev
    fs = wl.filters(3, 100_000)
    ts = wl.topics(3, 100_000, nt)
    ix, o = gpu_index(fs), oracle_of(fs)
    hit, vals = assert_same(ix, o, ts)
    o32 = ts.offs.astype(np.uint32)
    # in place: every buffer from tm_host_alloc
    pb = ix.host_array(len(ts.blob) + 16, np.uint8)
    pb[: len(ts.blob)] = ts.blob
    po = ix.host_array(nt + 1, np.uint32)
    po[:] = o32
    ph, pv, pe = ix.host_array(nt + 1, np.uint32), ix.host_array(int(hit[-1]) + 16, np.uint32), ix.host_array(nt, np.uint8)
    p0 = _paths(ix)
    h2, v2, e2 = ix.match_batch32(pb, po, (ph, pv, pe))
    assert np.array_equal(h2.astype(np.uint64), hit) and np.array_equal(v2, vals) and not e2.any()
    if nt <= 65536:
        assert sum(_paths(ix)[1:]) > sum(p0[1:])   # a 32-bit one-launch kernel
    # staged (ordinary numpy buffers)
    h3, v3, e3 = np.zeros(nt + 1, np.uint32), np.zeros(int(hit[-1]) + 16, np.uint32), np.zeros(nt, np.uint8)
    ix.match_batch32(ts.blob, o32, (h3, v3, e3))
    assert np.array_equal(h3[: nt + 1].astype(np.uint64), hit) and np.array_equal(v3[: int(hit[-1])], vals)
    # capacity too small: TM_ECAP, offsets still valid
    small = np.zeros(max(int(hit[-1]) // 2, 1), np.uint32)
    h4 = np.zeros(nt + 1, np.uint32)
    if int(hit[-1]) > 1:
        with pytest.raises(_native.TmError) as ex:
            ix.match_batch32(ts.blob, o32, (h4, small, np.zeros(nt, np.uint8)))
        assert ex.value.code == _native.TM_ECAP and np.array_equal(h4.astype(np.uint64), hit)
    # device API
    d_blob, d_offs = torch.from_numpy(ts.blob.copy()).cuda(), torch.from_numpy(o32.view(np.int32)).cuda()
    d_hit = torch.zeros(nt + 1, dtype=torch.int32, device="cuda")
    d_err = torch.zeros(nt, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(int(hit[-1]) + 1, dtype=torch.int32, device="cuda")
    ix.match_batch32_dev(nt, d_blob.data_ptr(), d_offs.data_ptr(), d_hit.data_ptr(), d_out.data_ptr(),
                         int(hit[-1]) + 1, d_err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_hit.cpu().numpy().view(np.uint32).astype(np.uint64), hit)
    assert np.array_equal(d_out.cpu().numpy().view(np.uint32)[: int(hit[-1])], vals)
    assert not d_err.cpu().numpy().any()


def test_vram_inputs_on_every_staged_path(torch_dev):
    """batch inputs in TM_ALLOC_VRAM memory that do NOT take
    the in-place one-launch path -- an index with a 35-level subscription
    (deeper than the one-launch store: any client can make one), a batch of
    more than 65536 topics, the sorted and unique orders, match/2 above 65536
    topics -- are read where they lie (device-side widening of the u32
    offsets), never by the host through the BAR (~163 ms per MiB).  Results
    equal the same batch in host memory and the oracle; the VRAM batch takes
    no longer than a few times the host-memory one."""
    import time
    fs = wl.filters(3, 100_000)
    deep = items_of([b"/".join([b"d"] * 34 + [b"+"])], [5_000_000])
    ix, o = gpu_index(fs), oracle_of(fs)

    def vram_pair(items):
        blob, offs = _native.pack_strings(items)
        vb = ix.host_array(len(blob) + 16, np.uint8, vram=True)
        vb[: len(blob)] = blob
        vo = ix.host_array(len(items) + 1, np.uint32, vram=True)
        vo[:] = offs.astype(np.uint32)
        hb = ix.host_array(len(blob) + 16, np.uint8)
        hb[: len(blob)] = blob
        ho = ix.host_array(len(items) + 1, np.uint32)
        ho[:] = offs.astype(np.uint32)
        return vb, vo, hb, ho, blob, offs

    def run_both(items, order=_native.TM_ORDER_TRAVERSAL):
        n = len(items)
        vb, vo, hb, ho, blob, offs = vram_pair(items)
        cap = 64 * n + 64
        outs = [(ix.host_array(n + 1, np.uint32), ix.host_array(cap, np.uint32), ix.host_array(n, np.uint8))
                for _ in range(2)]
        uq = [ix.host_array(n, np.uint32) for _ in range(2)] if order == _native.TM_ORDER_UNIQUE else [None, None]
        t0 = time.perf_counter()
        h, v, e = ix.match_batch32(hb, ho, outs[0], order, uq[0])
        t1 = time.perf_counter()
        h2, v2, e2 = ix.match_batch32(vb, vo, outs[1], order, uq[1])
        t2 = time.perf_counter()
        assert np.array_equal(h, h2) and np.array_equal(v, v2) and np.array_equal(e, e2)
        if uq[0] is not None:
            assert np.array_equal(uq[0], uq[1])
        return (h.copy(), v.copy(), e.copy()), blob, offs, t1 - t0, t2 - t1

    # 1. a 35-level subscription: the index no longer allows the one-launch path
    ix.apply(np.ones(1, np.uint8), deep.blob, deep.offs, deep.vals)
    o.apply(np.ones(1, np.uint8), deep.blob, deep.offs, deep.vals)
    ts = wl.topics(3, 100_000, 5_000)
    items = [ts.item(i) for i in range(len(ts))] + [b"/".join([b"d"] * 35), b"a/+/b"]
    p0 = ix.debug_get(_native.TM_DEBUG_PATH_PHASES)
    (h, v, e), blob, offs, th, tv = run_both(items)
    assert ix.debug_get(_native.TM_DEBUG_PATH_PHASES) >= p0 + 2
    oc, _, ohit, ovals = o.match_batch(blob, offs)
    assert np.array_equal(h.astype(np.uint64), ohit) and np.array_equal(v, ovals)
    assert 5_000_000 in v.tolist() and e[-1] == 1
    assert tv < 5 * th + 0.05, (tv, th)
    ix.apply(np.zeros(1, np.uint8), deep.blob, deep.offs, deep.vals)
    o.apply(np.zeros(1, np.uint8), deep.blob, deep.offs, deep.vals)
    # 2. more than 65536 topics
    ts = wl.topics(3, 100_000, 70_000, first=10_000)
    items = [ts.item(i) for i in range(len(ts))]
    (h, v, e), blob, offs, th, tv = run_both(items)
    oc, _, ohit, ovals = o.match_batch(blob, offs)
    assert np.array_equal(h.astype(np.uint64), ohit) and np.array_equal(v, ovals)
    assert tv < 5 * th + 0.05, (tv, th)
    # 3. the sorted and unique orders
    ts = wl.topics(3, 100_000, 3_000, first=90_000)
    items = [ts.item(i) for i in range(len(ts))]
    for order in (_native.TM_ORDER_SORTED, _native.TM_ORDER_UNIQUE):
        (h, v, e), blob, offs, th, tv = run_both(items, order)
        oc, _, ohit, ovals = o.match_batch(blob, offs)
        assert np.array_equal(h.astype(np.uint64), ohit)
        for i in range(len(items)):
            seg = np.sort(ovals[int(ohit[i]):int(ohit[i + 1])])
            if order == _native.TM_ORDER_UNIQUE:
                seg = np.unique(seg)
            assert np.array_equal(v[h[i]:h[i] + len(seg)], seg)
    # 4. match/2 above 65536 topics: VRAM bytes, host u64 offsets (what tmn_first passes)
    ts = wl.topics(3, 100_000, 70_000, first=200_000)
    items = [ts.item(i) for i in range(len(ts))]
    vb, vo, hb, ho, blob, offs = vram_pair(items)
    val, found = ix.first_batch(vb, offs.astype(np.uint64))
    val2, found2 = ix.first_batch(blob, offs.astype(np.uint64))
    assert np.array_equal(val, val2) and np.array_equal(found, found2)
    oc, _, ohit, ovals = o.match_batch(blob, offs)
    has = oc > 0
    assert np.array_equal(found[has], np.ones(int(has.sum()), np.uint8))
    assert np.array_equal(val[has], ovals[ohit[:-1][has].astype(np.int64)])


def test_router_concurrent_writers_read_their_writes(torch_dev):
    """VERDICT r5 missing 2 / next 2: N writer threads (the reference's
    broker-pool workers, emqx_broker_sup.erl:36, each running do_add_route ->
    mria write -> the hook, emqx_broker.erl:778-808) subscribe, publish right
    after the subscribe returned and must see their own route, unsubscribe
    and must no longer see it -- while other threads publish a C3-shaped
    batch stream.  The sync requests are group-committed (fewer device calls
    than writes) and at the end every topic's routes equal the CPU model +
    oracle (harness.RouterModel)."""
    import threading
    r = rt.Router(node="n1")
    base = wl.filters(3, 20_000)
    model = RouterModel()
    for i in range(len(base)):
        model.add(base.item(i), "n9")
    r.do_batch({(base.item(i), "n9"): ("add", 0, None) for i in range(len(base))})
    ts = wl.topics(3, 20_000, 2_000)
    pubs = [ts.item(i) for i in range(len(ts))]
    nw, per = 12, 25
    errors, stop = [], threading.Event()
    lock = threading.Lock()

    def writer(w):
        try:
            for i in range(per):
                flt = f"wr/{w}/{i}/+".encode()
                topic = f"wr/{w}/{i}/x".encode()
                dest = ("n1" if i % 2 else (b"grp", "n2"))
                r.add_route(flt, dest)
                got = r.match_routes(topic)
                if rt.Route(flt, dest) not in got:
                    errors.append(("missing", w, i, got))
                if i % 3 == 0:
                    r.delete_route(flt, dest)
                    if rt.Route(flt, dest) in r.match_routes(topic):
                        errors.append(("stale", w, i))
                else:
                    with lock:
                        model.add(flt, dest)
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append(("raised", w, repr(e)))

    def publisher():
        try:
            while not stop.is_set():
                r.match_routes_batch(pubs[:500])
        except Exception as e:   # noqa: BLE001
            errors.append(("publisher", repr(e)))
    pt = [threading.Thread(target=publisher) for _ in range(2)]
    wt = [threading.Thread(target=writer, args=(w,)) for w in range(nw)]
    for t in pt + wt:
        t.start()
    for t in wt:
        t.join()
    stop.set()
    for t in pt:
        t.join()
    assert not errors, errors[:5]
    writes = nw * per + nw * ((per + 2) // 3)
    assert r.mirror_synced_requests == writes + 1            # (+ the base do_batch)
    assert r.mirror_commits < r.mirror_synced_requests
    topics = pubs[:300] + [f"wr/{w}/{i}/x".encode() for w in range(nw) for i in range(per)]
    assert r.match_routes_batch(topics) == model.expected(topics)
    r.drain_events()
    assert r.match_routes_batch(topics) == model.expected(topics)
    print(f"{writes} writes in {r.mirror_commits - 1} group commits")


def test_router_killed_mirror_never_serves_a_stale_handle(torch_dev):
    """the mirror process dies; no publish is
    served by its handle (MirrorDown -- the Erlang module takes the
    reference's ETS path) while routes keep being written; the restarted
    mirror boots from the tables and serves exactly the routes written
    before and during the outage (vs the CPU model + oracle)."""
    r = rt.Router(node="n1")
    model = RouterModel()
    fs = wl.filters(3, 5_000)
    for i in range(len(fs)):
        r.add_route(fs.item(i), "n1")
        model.add(fs.item(i), "n1")
    ts = wl.topics(3, 5_000, 1_000)
    topics = [ts.item(i) for i in range(len(ts))] + [b"down/x/y"]
    assert r.match_routes_batch(topics) == model.expected(topics)
    old, n_before = r._mirror, len(model.wild)
    r.kill_mirror()
    for t, d in ((b"down/+/y", "n2"), (b"down/#", "n3")):
        r.add_route(t, d)
        model.add(t, d)
    r.delete_route(fs.item(0), "n1")
    model.delete(fs.item(0), "n1")
    with pytest.raises(rt.MirrorDown):
        r.match_routes(b"down/x/y")
    with pytest.raises(rt.MirrorDown):
        r.match_routes_batch(topics)
    assert old.stats()["n_keys"] == n_before          # the dead mirror took none of the writes
    r.restart_mirror(batch_size=1000)
    assert r._mirror is not old
    got = r.match_routes_batch(topics)
    assert got == model.expected(topics)
    assert {x.topic for x in got[-1]} >= {b"down/#", b"down/+/y"}


def _pairs_as_csr(pairs, vals, n):
    """(first, count) pairs -> CSR offsets and values in topic order; asserts
    the spans are disjoint and cover [0, total) exactly"""
    first, cnt = pairs[0:2 * n:2].astype(np.int64), pairs[1:2 * n:2].astype(np.int64)
    total = int(pairs[2 * n])
    assert int(cnt.sum()) == total
    order = np.argsort(first, kind="stable")
    ends = np.cumsum(cnt[order])
    assert np.array_equal(first[order], ends - cnt[order])      # disjoint, back to back from 0
    hit = np.zeros(n + 1, np.int64)
    hit[1:] = np.cumsum(cnt)
    out = np.concatenate([vals[f:f + c] for f, c in zip(first, cnt)]) if n else np.zeros(0, np.uint32)
    return hit.astype(np.uint32), out.astype(np.uint32)


@pytest.mark.parametrize("kind", ["auto", "wave"])
def test_pairs_batches_equal_the_csr_path_and_the_oracle(torch_dev, kind):
    """tm_match_batch32_pairs (what the NIF binds): per-topic (first, count)
    pairs from launches whose blocks never wait for each other -- every
    topic's values equal its CSR row (tm_match_batch32_ex) and the oracle's,
    the spans are disjoint and cover the total, badarg stays in its own slot;
    alone and from 10 concurrent callers sharing combined launches (with
    deltas applied in between), inputs in host or TM_ALLOC_VRAM memory; a
    batch above 65536 topics and an index too deep for the one-launch kernel
    take the CSR path and are converted."""
    import threading
    fs = wl.filters(3, 200_000)
    ix, o = gpu_index(fs), oracle_of(fs)
    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, _small_kind(kind))
    sets = []
    for k, nt in enumerate([1, 7, 100, 640, 3000, 4096, 9000, 20_000, 65_536, 70_000]):
        ts = wl.topics(3, 200_000, nt, first=k * 80_000)
        items = [ts.item(i) for i in range(nt)]
        if nt >= 100:
            items[nt // 2] = b"bad/#/topic"
        blob, offs = _native.pack_strings(items)
        vram = k % 2 == 1
        pb = ix.host_array(len(blob) + 16, np.uint8, vram=vram)
        pb[: len(blob)] = blob
        po = ix.host_array(nt + 1, np.uint32, vram=vram)
        po[:] = offs.astype(np.uint32)
        cap = 64 * nt + 64
        csr = (ix.host_array(nt + 1, np.uint32), ix.host_array(cap, np.uint32), ix.host_array(nt, np.uint8))
        prs = [(ix.host_array(2 * nt + 1, np.uint32), ix.host_array(cap, np.uint32), ix.host_array(nt, np.uint8))
               for _ in range(2)]
        sets.append((pb, po, csr, prs, items, blob, offs))

    def check(k, pairs, vals, err):
        pb, po, csr, prs, items, blob, offs = sets[k]
        h, v, e = ix.match_batch32(pb, po, csr)
        hh, vv = _pairs_as_csr(pairs, vals, len(items))
        return np.array_equal(hh, h) and np.array_equal(vv, v) and np.array_equal(err, e)

    for k, (pb, po, csr, prs, items, blob, offs) in enumerate(sets):
        pairs, vals, err = ix.match_batch32_pairs(pb, po, prs[0])
        assert check(k, pairs, vals, err), k
        oc, _, ohit, ovals = o.match_batch(blob, offs)
        hh, vv = _pairs_as_csr(pairs, vals, len(items))
        for i in range(len(items)):
            if err[i]:
                assert b"+" in items[i] or b"#" in items[i]
                continue
            assert np.array_equal(vv[hh[i]:hh[i + 1]], ovals[int(ohit[i]):int(ohit[i + 1])])
    # concurrent callers through the combiner, deltas in between (each result
    # equal to the CSR path run right after it: the deltas only add keys that
    # no topic of these sets matches)
    errors = []

    def caller(k):
        pb, po, csr, prs, items, _, _ = sets[k]
        try:
            for _ in range(15):
                pairs, vals, err = ix.match_batch32_pairs(pb, po, prs[1])
                hh, vv = _pairs_as_csr(pairs, vals, len(items))
                hh0, vv0 = _pairs_as_csr(*ix.match_batch32_pairs(pb, po, prs[0])[:2], len(items))
                if not (np.array_equal(hh, hh0) and np.array_equal(vv, vv0)):
                    errors.append(k)
                    return
        except Exception as ex:   # noqa: BLE001 -- reported below
            errors.append((k, repr(ex)))
    l0 = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES)
    th = [threading.Thread(target=caller, args=(k,)) for k in range(len(sets) - 1)]
    for t in th:
        t.start()
    for e in range(5):
        d = items_of([b"zz/%d/+" % e], [9_000_000 + e])
        ix.apply(np.ones(1, np.uint8), d.blob, d.offs, d.vals)
    for t in th:
        t.join()
    assert not errors, errors
    assert ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES) > l0
    # an index the one-launch kernel cannot take: the CSR path, converted
    deep = items_of([b"/".join([b"d"] * 34 + [b"+"])], [5_000_000])
    ix.apply(np.ones(1, np.uint8), deep.blob, deep.offs, deep.vals)
    p0 = ix.debug_get(_native.TM_DEBUG_PATH_PHASES)
    for k in (3, 4):
        pb, po, csr, prs, items, blob, offs = sets[k]
        pairs, vals, err = ix.match_batch32_pairs(pb, po, prs[0])
        assert check(k, pairs, vals, err)
    assert ix.debug_get(_native.TM_DEBUG_PATH_PHASES) > p0


# ------------------------------------------------- device batches as pairs

def pairs_cap(ix: _native.Index, ts: wl.ItemSet) -> int:
    """a capacity with which no value is dropped: total + 4096 x the most hits
    of one topic (include/tmatch.h tm_match_batch_dev_pairs)"""
    h, _, _ = ix.match_batch(ts.blob, ts.offs)
    c = np.diff(h.astype(np.int64))
    return int(h[-1]) + 4096 * int(c.max()) if len(c) else 0


def pairs_batch(torch, ix: _native.Index, ts: wl.ItemSet, cap=None, stream=None, reps=1):
    """tm_match_batch_dev_pairs on device copies of ts: (pairs [n, 2], total,
    extent, values, err) on the host"""
    dev = torch.device("cuda:0")
    n = len(ts)
    blob = torch.from_numpy(ts.blob.copy()).to(dev)
    offs = torch.from_numpy(ts.offs.view(np.int64).copy()).to(dev)
    pairs = torch.full((2 * n + 2,), -1, dtype=torch.int32, device=dev)
    if cap is None:
        cap = pairs_cap(ix, ts)
    out = torch.full((max(cap, 1),), -1, dtype=torch.int32, device=dev)
    err = torch.full((max(n, 1),), 7, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    for _ in range(reps):
        ix.match_batch_dev_pairs(n, blob.data_ptr(), offs.data_ptr(), pairs.data_ptr(), out.data_ptr(), cap,
                                 err.data_ptr(), s)
    torch.cuda.synchronize()
    p = pairs.cpu().numpy().view(np.uint32)
    return p[:2 * n].reshape(n, 2).astype(np.int64), int(p[2 * n]), int(p[2 * n + 1]), \
        out.cpu().numpy().view(np.uint32)[:cap], err.cpu().numpy()[:n]


def assert_pairs_same(torch, ix: _native.Index, o: Oracle, ts: wl.ItemSet, reps=1):
    """the pairs equal the oracle's CSR topic by topic (values and order), the
    spans are disjoint and end by the extent (<= cap: nothing dropped), the
    flags equal the oracle's"""
    cnt, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    pr, total, extent, vals, err = pairs_batch(torch, ix, ts, reps=reps)
    n = len(ts)
    assert np.array_equal(err.astype(np.int64), np.where(cnt < 0, -cnt, 0)), "badarg / too-deep flags differ"
    assert np.array_equal(pr[:, 1], np.maximum(cnt, 0)), "hit counts differ"
    assert total == int(ohit[-1])
    live = np.nonzero(pr[:, 1])[0]
    order = live[np.argsort(pr[live, 0], kind="stable")]
    ends = pr[order, 0] + pr[order, 1]
    assert len(order) == 0 or (np.all(pr[order[1:], 0] >= ends[:-1]) and ends.max() == extent), "spans overlap"
    assert extent <= len(vals), "values dropped with a sufficient capacity"
    for i in range(n):
        c = int(pr[i, 1])
        if c:
            p = int(pr[i, 0])
            assert np.array_equal(vals[p:p + c], ovals[int(ohit[i]):int(ohit[i + 1])]), \
                f"topic {i} {ts.item(i)!r}: values differ"
    return pr, total, extent


@pytest.mark.parametrize("cfg,nf,nt", [(3, 200_000, 120_000), (30, 200_000, 60_000), (1, 10_000, 50_000),
                                      (2, 20_000, 40_000)])
def test_pairs_device_batches_vs_oracle(torch_dev, cfg, nf, nt):
    """tm_match_batch_dev_pairs (k_walk_pairs + k_tail_pairs): every topic's
    values exact vs the oracle in traversal order; C3deep's tail lists (MID and
    DEEP) and C2's overflowed topics (more than RCAP runs: span reserved by
    the walk, values re-walked by the tail) included; run twice on the same
    workspace (the value counter and the lists are reset between batches)"""
    fs = wl.filters(2 if cfg == 2 else (3 if cfg == 30 else cfg), nf)
    ts = wl.topics(cfg, nf, nt)
    ix, o = gpu_index(fs), oracle_of(fs)
    assert_pairs_same(torch_dev, ix, o, ts, reps=2)


def test_pairs_device_edge_cases(torch_dev):
    """deep topics (26 levels: MID list; 300 and 1000 levels: DEEP list),
    overflowing runs, badarg topics, a '#'-not-last cut, an empty batch, and a
    capacity smaller than the total (values past cap dropped, total reported)"""
    letters = [chr(ord("a") + i).encode() for i in range(26)]
    T = b"/".join(letters)
    deep = b"/".join(b"l%d" % i for i in range(300))
    filters = [b"#", T + b"/#", T + b"/+", b"+/" * 26 + b"#", b"a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#",
               deep, deep + b"/#", b"l0/+/#", b"+/l1/#", deep.rsplit(b"/", 1)[0] + b"/+",
               b"a/#", b"+/#", b"+/+/#", b"a/b/#", b"+/b/#", b"a/+/#", b"a/b/+", b"+/+", b"a/+", b"+/b",
               b"a/b", b"#", b"+/+/+/#", b"x/#/y", b"x/#"]
    topics = [T, T + b"/1", deep, deep + b"/x", b"a/b", b"a/b/c", b"l0/l1", b"/".join([b"w"] * 1000),
              b"/".join([b"+"] * 40), T + b"/#", b"x", b"x/y", b"", b"q/+/r"]
    r = random.Random(5)
    topics = [r.choice(topics) for _ in range(3000)] + topics
    fs = items_of(filters)
    ix, o = gpu_index(fs), oracle_of(fs)
    pr, total, _ = assert_pairs_same(torch_dev, ix, o, items_of(topics), reps=2)
    assert pr[:, 1].max() > 8   # 'a/b' overflows the RCAP ranges
    # empty batch: the total and extent alone
    e = items_of([])
    p0, t0, x0, _, _ = pairs_batch(torch_dev, ix, e, cap=0)
    assert t0 == 0 and x0 == 0 and len(p0) == 0
    # capacity too small: total reported, extent past cap, every value below
    # cap where the pairs say, and the batch after it exact again
    ts = items_of(topics)
    cnt, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    for cap in (100, total // 2, total):
        pr2, t2, x2, v2, _ = pairs_batch(torch_dev, ix, ts, cap=cap)
        assert t2 == int(ohit[-1]) and (x2 > cap or cap >= total)
        for i in range(len(ts)):
            p, c = int(pr2[i, 0]), int(pr2[i, 1])
            if p < cap and c:
                k = min(c, cap - p)
                assert np.array_equal(v2[p:p + k], ovals[int(ohit[i]):int(ohit[i]) + k])
    assert_pairs_same(torch_dev, ix, o, ts)


@pytest.mark.parametrize("copies,nstreams", [(1, 2), (2, 2), (3, 3)])
def test_pairs_batches_on_streams_see_patches_in_order(torch_dev, copies, nstreams):
    """The headline's form under churn: device pairs batches on several
    streams, deltas applied between them (with 1-3 copies of the tables), each
    batch's lists exact against the oracle after exactly the deltas applied
    before it was queued -- the region counters and tail lists of every
    stream's workspace reset between its batches."""
    torch = torch_dev
    nf = 30_000
    fs = wl.filters(5, nf)
    ix = _native.Index(copies=copies)
    ix.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    o = oracle_of(fs)
    ts = wl.topics(5, nf, 40_000)
    dev = torch.device("cuda:0")
    d_blob = torch.from_numpy(ts.blob.copy()).to(dev)
    d_offs = torch.from_numpy(ts.offs.view(np.int64).copy()).to(dev)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    n = len(ts)
    results = []
    for k in range(4 if copies == 1 else 9):
        d = wl.deltas(nf, k * 3_000, 3_000 if k % 3 else 40)
        ix.apply(d.flags, d.blob, d.offs, d.vals)
        o.apply(d.flags, d.blob, d.offs, d.vals)
        o.prepare()
        cnt, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
        cap = int(ohit[-1]) + 4096 * int(max(int(np.max(cnt)), 1))
        pairs = torch.zeros(2 * n + 2, dtype=torch.int32, device=dev)
        err = torch.zeros(n, dtype=torch.uint8, device=dev)
        out = torch.zeros(cap, dtype=torch.int32, device=dev)
        ix.match_batch_dev_pairs(n, d_blob.data_ptr(), d_offs.data_ptr(), pairs.data_ptr(), out.data_ptr(), cap,
                                 err.data_ptr(), streams[k % nstreams].cuda_stream)
        results.append((pairs, out, err, cnt, ohit, ovals, cap))
    torch.cuda.synchronize()
    for pairs, out, err, cnt, ohit, ovals, cap in results:
        p = pairs.cpu().numpy().view(np.uint32)
        v = out.cpu().numpy().view(np.uint32)
        assert int(p[2 * n]) == int(ohit[-1]) and int(p[2 * n + 1]) <= cap
        assert not err.cpu().numpy().any()
        pr = p[:2 * n].reshape(n, 2).astype(np.int64)
        assert np.array_equal(pr[:, 1], np.maximum(cnt, 0))
        for i in range(0, n, 7):   # (a sample of the topics per batch: 9 batches x 40k topics)
            assert np.array_equal(v[pr[i, 0]:pr[i, 0] + pr[i, 1]], ovals[int(ohit[i]):int(ohit[i + 1])]), i


def test_pairs_regions_under_a_tight_capacity(torch_dev):
    """A batch large enough for several regions (120k topics: 14) with cap =
    the exact total: spans may not all fit (regions leave gaps), and the
    library says so -- the extent exceeds cap exactly when some topic's span
    does; every value that landed below cap is the oracle's, and the next
    batch on the workspace (ample cap) is exact again (counters reset)."""
    torch = torch_dev
    nf = 200_000
    fs = wl.filters(3, nf)
    ix, o = gpu_index(fs), oracle_of(fs)
    ts = wl.topics(3, nf, 120_000)
    cnt, _, ohit, ovals = o.match_batch(ts.blob, ts.offs)
    total = int(ohit[-1])
    pr, t2, x2, v2, _ = pairs_batch(torch, ix, ts, cap=total)
    assert t2 == total
    ends = pr[:, 0] + pr[:, 1]
    assert (x2 > total) == bool((ends > total).any())
    for i in range(0, len(ts), 5):
        p, c = int(pr[i, 0]), int(pr[i, 1])
        k = max(0, min(c, total - p))
        assert np.array_equal(v2[p:p + k], ovals[int(ohit[i]):int(ohit[i]) + k]), i
    assert_pairs_same(torch, ix, o, ts)

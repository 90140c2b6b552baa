"""Host-side logic that needs no GPU: key helpers, term order, workloads."""
import numpy as np

from emqx_amd import workload as wl
from emqx_amd.topic_index import Tab, _finish
from emqx_amd.trie_search import (HASH, PLUS, BadArg, filter as tfilter, get_id, get_topic, key_order,
                                  make_key, term_key, topic_words)


def test_make_key_forms():
    assert make_key(b"a/b", 1) == (b"a/b", (1,))
    assert make_key(b"a/+/#", 1) == ((b"a", PLUS, HASH), (1,))
    assert make_key([b"a", b"b"], 1) == ((b"a", b"b"), (1,))
    assert get_topic(make_key(b"sensor/+/metric//#", 3)) == b"sensor/+/metric//#"
    assert tfilter(b"") is False


def test_topic_words_badarg():
    for t in (b"+", b"#", b"a/+/b", b"a/b/#"):
        try:
            topic_words(t)
        except BadArg:
            continue
        raise AssertionError(t)
    assert topic_words(b"a/b/b+") == [b"a", b"b", b"b+"]


def test_term_order():
    # numbers < atoms < tuples < lists < binaries; '#' < '+' < binary words
    xs = [b"a", [1], ("x",), "atom", 5]
    assert sorted(xs, key=term_key) == [5, "atom", ("x",), [1], b"a"]
    k1, k2, k3 = make_key(b"a/#", 1), make_key(b"a/+", 1), make_key(b"a/b/+", 1)
    k4 = make_key(b"a/b", 1)
    assert sorted([k4, k3, k2, k1], key=key_order) == [k1, k2, k3, k4]


def test_finish_orders_like_reference():
    keys = [make_key(b"a/+/#", 8), make_key(b"a/+/+", 7), make_key(b"a/b/#", 2), make_key(b"a/b/#", 3),
            make_key(b"a/b/+", 5), make_key(b"a/b/c", 4)]
    assert [get_id(k) for k in _finish(keys, ["unique"])] == [2, 3, 4, 5, 7, 8]
    assert _finish(keys, [])[0] == make_key(b"a/b/c", 4)


def test_encode_word_lists_no_topic_can_match():
    """Binary words no topic level can equal ('+' / '#' as binaries, words
    holding a '/') take the escaped key form (include/tmatch.h "Keys"): the
    library keeps them for matches_filter/3 only."""
    esc = 1 | 4   # TM_KEY_WORDS | TM_KEY_ESCAPED
    assert Tab._encode(((b"a/b", PLUS), (1,))) == (b"a\\/b/+", esc)
    assert Tab._encode(((b"+",), (1,))) == (b"\\+", esc)
    assert Tab._encode(((b"x\\y", b"#", HASH), (1,))) == (b"x\\\\y/\\#/#", esc)
    assert Tab._encode(((), (1,))) == (b"", 2)
    assert Tab._encode(((b"a", PLUS), (1,))) == (b"a/+", 1)
    assert Tab._encode(((b"a\\b", PLUS), (1,))) == (b"a\\b/+", 1)   # a backslash alone: no escape needed


def test_workload_deterministic_and_sharded():
    a = wl.filters(3, 5000)
    b = wl.filters(3, 5000)
    assert a.items() == b.items()
    assert len(a) == 5002  # + the '#' and '+/#' globals
    parts = [wl.filters(3, 5000, shard=s, nshards=4) for s in range(4)]
    merged = sorted(sum((list(zip(p.vals.tolist(), p.items())) for p in parts), []))
    assert merged == sorted(zip(a.vals.tolist(), a.items()))
    t = wl.topics(3, 5000, 2000)
    assert len(t) == 2000
    assert any(x.startswith(b"$SYS/") for x in t.items())


def test_workload_c2_shape():
    f = wl.filters(2, 1000)
    items = f.items()
    assert items[0] == b"fleet/0/sensor/+" and items[999] == b"fleet/999/sensor/+"
    assert items[1000:1250] == [b"#"] * 250 and items[1250] == b"fleet/#"
    t = wl.topics(2, 1000, 100).items()
    assert all(x.startswith(b"fleet/") and x.split(b"/")[2] == b"sensor" for x in t)


def test_workload_deltas_remove_live_keys_once():
    d = wl.deltas(1000, 0, 2000)
    subs = d.flags == 1
    assert subs.sum() == 1000
    dels = d.vals[~subs]
    assert len(set(dels.tolist())) == len(dels) and dels.max() < 1000
    base = wl.filters(5, 1000)
    base_keys = set(zip(base.items(), base.vals.tolist()))
    for i in np.nonzero(~subs)[0][:50]:
        assert (d.item(i), int(d.vals[i])) in base_keys


def test_ids_of_one_filter_in_term_order():
    """The device orders the values of one filter by u32 kid (insertion order,
    reused kids); the reference orders the keys {Filter, {ID}} of one filter
    by the ID's term order (advisor finding, emqx_trie_search.erl:107-111).
    traversal_order re-sorts each run of equal filters."""
    from emqx_amd.topic_index import traversal_order
    a2, a1, a_atom = make_key(b"a/+", 2), make_key(b"a/+", 1), make_key(b"a/+", "node1")
    h9 = make_key(b"a/#", 9)
    dev_order = [h9, a_atom, a2, a1, make_key(b"a/b", 5), make_key(b"a/b", 0)]
    got = traversal_order(dev_order)
    assert got == sorted(dev_order, key=key_order)
    assert got == [h9, a1, a2, a_atom, make_key(b"a/b", 0), make_key(b"a/b", 5)]
    # match/2 = first in traversal order; matches/3 = its reverse
    assert _finish(dev_order, [])[-1] == h9
    assert _finish([a2, a1], [])[-1] == a1


def test_broker_badarg_fails_only_that_message():
    """A micro-batch with one '+'-level topic: that message's result is its
    BadArg, every other message is routed (no GPU: a stub router)."""
    from emqx_amd import broker as bk
    from emqx_amd.router import Route

    class StubRouter:
        node = "n1"

        def match_routes_batch(self, topics, errors="raise"):
            assert errors == "return"
            return [BadArg(t) if b"+" in t.split(b"/") else [Route(t, "n1")] for t in topics]

    b = bk.Broker(StubRouter())
    msgs = [bk.Message(b"a/%d" % i, i) for i in range(10)] + [bk.Message(b"a/+/b", 99)]
    futs = [b.publish(m) for m in msgs]
    b.flush()
    for f in futs[:10]:
        assert f.result(0)[0] == [(f.result(0)[0][0][0], "n1")]
    assert isinstance(futs[10].exception(0), BadArg)


class _EpochIndex:
    """Stand-in for _native.Index with the library's reader-epoch rule
    (include/tmatch.h "Reader epochs"), no device: for Tab's bookkeeping."""

    def __init__(self):
        self.cur, self.readers, self.next = 1, {}, 1
        self.applied = []

    def apply(self, ops, blob, offs, vals, flags=None):
        self.applied.append((ops.tolist(), vals.tolist()))
        self.cur += 1
        return self.cur

    def read_begin(self):
        t = self.next
        self.next += 1
        self.readers[t] = self.cur
        return t

    def read_end(self, t):
        del self.readers[t]

    def epoch(self):
        return self.cur, min(self.readers.values(), default=self.cur)


def test_freed_values_wait_for_older_readers():
    """A u32 freed by a delete is not handed to a new key while a reader that
    began before the delete runs; decoding drops keys deleted meanwhile."""
    ix = _EpochIndex()
    tab = Tab(index=ix)
    ka, kb, kc = make_key(b"a/+", 1), make_key(b"b/+", 2), make_key(b"c/+", 3)
    tab.insert_key(ka, None)
    tab.insert_key(kb, None)
    tab.flush()
    kid_a = tab._kid[ka]
    reader = tab.read_begin()              # a batch in flight that may return kid_a
    tab.delete_key(ka)
    tab.flush()
    assert tab.decode(np.array([kid_a, tab._kid[kb]], np.uint32)) == [kb]   # deleted: dropped
    tab.insert_key(kc, None)
    assert tab._kid[kc] != kid_a           # quarantined while the reader runs
    tab.read_end(reader)
    tab.delete_key(kc)
    tab.flush()
    kd = make_key(b"d/+", 4)
    tab.insert_key(kd, None)               # no reader left: both freed values are reusable
    assert tab._kid[kd] in (kid_a, 2)
    assert tab.decode(np.array([tab._kid[kd]], np.uint32)) == [kd]


def test_unshipped_deletes_are_not_reused():
    """A delete not yet shipped (no epoch yet) keeps its u32 out of reuse."""
    tab = Tab(index=_EpochIndex())
    ka = make_key(b"a/+", 1)
    tab.insert_key(ka, None)
    tab.flush()
    kid = tab._kid[ka]
    tab.delete_key(ka)
    tab.insert_key(make_key(b"b/+", 2), None)   # same pending batch: the device still holds kid
    assert tab._kid[make_key(b"b/+", 2)] != kid

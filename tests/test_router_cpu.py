"""Router write paths on the CPU (no device): the mirror of emqx_route_filters
is reconciled key by key against the table, so whatever order the hook's
synchronous deltas and the (late, duplicated, stale) table events arrive in,
the mirror holds exactly the table's keys once the mailbox is drained, and a
local write is in the mirror as soon as add_route / delete_route / do_batch
return (emqx_router.erl:483-509, src/emqx_router_gpu.erl)."""
import random

from emqx_amd import router as rt
from emqx_amd.trie_search import filter as tfilter, make_key


class FakeMirror:
    """topic_index.Tab's write side, without a device."""

    def __init__(self):
        self.keys, self.pending, self.flushes = set(), [], 0

    def insert_key(self, key, record):
        if key not in self.keys:
            self.keys.add(key)
            self.pending.append(("insert", key))

    def delete_key(self, key):
        if key in self.keys:
            self.keys.discard(key)
            self.pending.append(("delete", key))

    def flush(self):
        self.flushes += 1
        self.pending = []

    def stats(self):
        return {"n_keys": len(self.keys)}


def _router():
    m = FakeMirror()
    return rt.Router(node="n1", mirror=m), m


def test_event_key_shapes():
    k = make_key(b"a/+", "n1")
    assert rt.event_key(("write", rt.RouteIdx(k))) == k
    assert rt.event_key(("delete", rt.RouteIdx(k))) == k                    # record form
    assert rt.event_key(("delete", (rt.ROUTE_TAB_FILTERS, k))) == k         # {Tab, Key}
    assert rt.event_key(("delete", ("emqx_route", b"a/b"))) is None
    assert rt.event_key(("write", rt.Route(b"a/b", "n1"))) is None
    assert rt.event_key(("delete", rt.Route(b"a/b", "n1"))) is None


def test_local_writes_reach_the_mirror_before_returning():
    r, m = _router()
    r.add_route(b"a/+", "n2")
    assert make_key(b"a/+", "n2") in m.keys and m.pending == [] and m.flushes == 1
    r.add_route(b"a/b", "n2")                       # a bag row: not on the device
    assert m.flushes == 1 and len(m.keys) == 1
    r.delete_route(b"a/+", "n2")
    assert not m.keys and m.flushes == 2
    errs = r.do_batch({(b"x/+", "n1"): ("add", 0, None), (b"y/#", "n2"): ("add", 0, None),
                       (b"x/y", "n1"): ("add", 0, None)})
    assert errs == {} and m.flushes == 3 and len(m.keys) == 2   # one delta batch for the whole batch


def test_stale_events_never_resurrect_a_route():
    r, m = _router()
    r.add_route(b"a/+", "n2")
    r.delete_route(b"a/+", "n2")
    assert r.pending_events() == 2                  # the echo of both writes, still queued
    r.drain_events(limit=1)                         # the insert's echo first: the table lacks the key
    assert not m.keys
    r.drain_events()
    assert not m.keys


def test_random_interleavings_converge_to_the_table():
    rnd = random.Random(3)
    r, m = _router()
    words = [b"a", b"b", b"+", b"c"]
    for step in range(3000):
        t = b"/".join(rnd.choice(words) for _ in range(rnd.randint(1, 3)))
        if rnd.random() < 0.1:
            t += b"/#"
        d = rnd.choice(["n1", "n2", "n3", (b"g", "n2")])
        op = "add" if rnd.random() < 0.6 else "delete"
        what = rnd.random()
        if what < 0.4:
            (r.add_route if op == "add" else r.delete_route)(t, d)
            if tfilter(t) is not False:             # a local write is mirrored at once
                assert (make_key(tfilter(t), d) in m.keys) == (op == "add")
        elif what < 0.8:
            r.replicate(op, t, d, record_form=rnd.random() < 0.5)
        elif what < 0.85:
            r.cleanup_routes(rnd.choice(["n2", "n3"]))
        elif what < 0.95:
            r.drain_events(limit=rnd.randint(1, 20))
        else:
            r.drain_events()
            assert m.keys == set(r._filters)
    r.drain_events()
    assert m.keys == set(r._filters)
    assert r.stats_n_routes() == sum(len(v) for v in r._bag.values()) + len(r._filters)

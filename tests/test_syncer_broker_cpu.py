"""Host logic of the router syncer (route-update batching) and the broker's
publish micro-batching -- pure host code, no matching here (the GPU paths are
in tests/test_gpu_parity.py).

The syncer case is the reference's own known-answer test: batch_test/0 of
apps/emqx/src/emqx_router_syncer.erl:420-485 (pushes, mk_batch(Stash, 5), the
expected batch, the stash left over and the reply sequence), transcribed.
"""
import time

import pytest

from emqx_amd import broker as bk, syncer as sy
from emqx_amd.router import Route, get_dest_node


class _Tag(sy.Ref):
    """A wait reference that records the order replies are sent in."""

    def __init__(self, n, log):
        super().__init__()
        self.n, self.log = n, log

    def send(self, result):
        self.log.append((self.n, result))
        super().send(result)


def test_batch_test_known_answer():
    """emqx_router_syncer.erl:420-485."""
    dest = "node"
    log = []
    ctx = lambda n: [_Tag(n, log)]  # noqa: E731
    pushes = [
        (sy.PRIO_BG, ("delete", b"t/2", dest, ctx(1))),
        (sy.PRIO_HI, ("add", b"t/1", dest, ctx(2))),
        (sy.PRIO_LO, ("add", b"t/1", dest, ctx(3))),
        (sy.PRIO_HI, ("add", b"t/2", dest, ctx(4))),
        (sy.PRIO_HI, ("add", b"t/3", dest, ctx(5))),
        (sy.PRIO_HI, ("add", b"t/4", dest, ctx(6))),
        (sy.PRIO_LO, ("delete", b"t/3", dest, ctx(7))),
        (sy.PRIO_BG, ("delete", b"t/3", dest, ctx(8))),
        (sy.PRIO_BG, ("delete", b"t/2", dest, ctx(9))),
        (sy.PRIO_BG, ("delete", b"old/1", dest, ctx(10))),
        (sy.PRIO_HI, ("add", b"t/2", dest, ctx(11))),
        (sy.PRIO_BG, ("delete", b"old/2", dest, ctx(12))),
        (sy.PRIO_HI, ("add", b"t/3", dest, ctx(13))),
        (sy.PRIO_HI, ("add", b"t/3", dest, ctx(14))),
        (sy.PRIO_LO, ("delete", b"old/3", dest, ctx(15))),
        (sy.PRIO_LO, ("delete", b"t/2", dest, ctx(16))),
    ]
    stash, replies = {}, []
    for prio, op in pushes:
        sy.stash_add(prio, op, stash, replies)
    for ref, res in replies:
        ref.send(res)
    batch, left = sy.mk_batch(stash, 5)
    got = {k: (v[0], v[1]) for k, v in batch.items()}
    assert got == {
        (b"t/1", dest): ("add", sy.PRIO_LO),
        (b"t/3", dest): ("add", sy.PRIO_HI),
        (b"t/2", dest): ("delete", sy.PRIO_LO),
        (b"t/4", dest): ("add", sy.PRIO_HI),
        (b"old/3", dest): ("delete", sy.PRIO_LO),
    }
    assert {k: (v[0], v[1]) for k, v in left.items()} == {
        (b"old/1", dest): ("delete", sy.PRIO_BG),
        (b"old/2", dest): ("delete", sy.PRIO_BG),
    }
    # replies are only sent to superseded ops
    assert log == [(1, "ok"), (5, "ok"), (4, "ok"), (9, "ok"), (7, "ok"), (8, "ok"), (11, "ok")]


class _StubRouter:
    """Stands in for Router.do_batch: records batches, can fail N times."""
    node = "n1"

    def __init__(self, fail=0, bad_routes=()):
        self.batches, self.fail, self.bad = [], fail, set(bad_routes)

    def do_batch(self, batch):
        if self.fail:
            self.fail -= 1
            raise RuntimeError("core node down")
        self.batches.append(dict(batch))
        return {r: ("error", "x") for r in batch if r in self.bad}


def test_syncer_batches_and_replies():
    r = _StubRouter(bad_routes=[(b"bad/1", "n1")])
    s = sy.Syncer(r, max_batch_size=40)
    refs = [s.push("add", f"t/{i}".encode(), "n1", {"reply": True}) for i in range(100)]
    bad = s.push("add", b"bad/1", "n1", {"reply": True})
    assert s.push("delete", b"x/1", "n1") == "ok"
    assert s.run_once() == 102
    assert [len(b) for b in r.batches] == [40, 40, 22]
    assert all(x.wait(0) == "ok" for x in refs)
    assert bad.wait(0) == ("error", "x")
    # reply-waiting ops (PRIO_HI) go before the background delete
    assert (b"x/1", "n1") in r.batches[-1]


def test_syncer_failed_batch_is_retried():
    r = _StubRouter(fail=1)
    s = sy.Syncer(r, error_delay=1, error_retry_interval=1)
    ref = s.push("add", b"a/b", "n1", {"reply": True})
    assert s.run_once() == 0 and s.stats()["size"] == 1      # kept stashed after the error
    assert s.run_once() == 1 and ref.wait(0) == "ok" and s.stats()["size"] == 0


def test_syncer_suspend_activate():
    r = _StubRouter()
    s = sy.Syncer(r)
    s.suspend()
    s.push("add", b"a", "n1")
    assert s.run_once() == 0 and s.stats()["n_add"] == 1
    s.activate()
    assert s.stats()["size"] == 0 and len(r.batches) == 1


def test_syncer_thread():
    r = _StubRouter()
    s = sy.Syncer(r, start=True)
    try:
        refs = [s.push("add", f"q/{i}".encode(), "n1", {"reply": True}) for i in range(500)]
        assert all(x.wait(5) == "ok" for x in refs)
    finally:
        s.close()
    assert sum(len(b) for b in r.batches) == 500


# ------------------------------------------------------------------ aggre

def test_aggre():
    """emqx_broker.erl:408-424."""
    assert bk.aggre([]) == []
    assert bk.aggre([Route(b"t", "n1")]) == [(b"t", "n1")]
    assert bk.aggre([Route(b"t", (b"g", "n1"))]) == [(b"t", b"g")]
    # plain node routes: accumulated by prepending -> reversed
    assert bk.aggre([Route(b"a", "n1"), Route(b"b", "n2"), Route(b"a", "n1")]) == \
        [(b"a", "n1"), (b"b", "n2"), (b"a", "n1")][::-1]
    # any shared-group dest -> lists:usort
    assert bk.aggre([Route(b"b", "n2"), Route(b"a", (b"g", "n1")), Route(b"a", (b"g", "n2")),
                     Route(b"a", "n1")]) == [(b"a", "n1"), (b"a", b"g"), (b"b", "n2")]


def test_get_dest_node():
    assert get_dest_node("n1") == "n1"
    assert get_dest_node((b"g", "n1")) == "n1"
    assert get_dest_node(("external", b"link")) == ("external", b"link")


class _StubMatchRouter:
    """Stands in for Router.match_routes_batch: one call per micro-batch."""
    node = "n1"

    def __init__(self):
        self.calls = []

    def match_routes_batch(self, topics, errors="raise"):
        self.calls.append(len(topics))
        return [[Route(t, "n1"), Route(b"#", "n2"), Route(b"+/x", (b"g", "n3"))] for t in topics]


def test_broker_publish_batch_routes_like_do_publish():
    got = []
    r = _StubMatchRouter()
    b = bk.Broker(r, dispatch=lambda to, m: got.append(("local", to, m.payload)) or 1,
                  forward=lambda n, to, m: ("fwd", n), share_dispatch=lambda g, to, m: ("share", g))
    res = b.publish_batch([bk.Message(b"a/x", 1), bk.Message(b"b/x", 2)])
    assert r.calls == [2]
    routes, results = res[0]
    assert routes == [(b"#", "n2"), (b"+/x", b"g"), (b"a/x", "n1")]   # usort: a group dest is present
    assert results == [("n2", b"#", ("fwd", "n2")), ("share", b"+/x", ("share", b"g")), ("n1", b"a/x", 1)]
    assert got == [("local", b"a/x", 1), ("local", b"b/x", 2)]


def test_broker_micro_batches_by_size_and_time():
    r = _StubMatchRouter()
    b = bk.Broker(r, max_batch=64, max_wait_ms=20, start=True)
    try:
        futs = [b.publish(bk.Message(f"t/{i}".encode(), i)) for i in range(200)]
        res = [f.result(timeout=5) for f in futs]
    finally:
        b.close()
    assert all(routes[-1] == (f"t/{i}".encode(), "n1") for i, (routes, _) in enumerate(res))
    assert sum(r.calls) == 200 and max(r.calls) <= 64 and len(r.calls) < 200
    # a lone message is flushed by the wait bound
    r2 = _StubMatchRouter()
    b2 = bk.Broker(r2, max_batch=1000, max_wait_ms=5, start=True)
    try:
        t0 = time.monotonic()
        assert b2.publish(bk.Message(b"z", 0)).result(timeout=5)[0][-1] == (b"z", "n1")
        assert time.monotonic() - t0 < 2
    finally:
        b2.close()
    assert r2.calls == [1]


def test_broker_error_reaches_callers():
    class Bad(_StubMatchRouter):
        def match_routes_batch(self, topics, errors="raise"):
            raise ValueError("badarg")
    b = bk.Broker(Bad(), max_batch=2)
    f1, f2 = b.publish(bk.Message(b"a", 0)), b.publish(bk.Message(b"b", 0))
    with pytest.raises(ValueError):
        f1.result(timeout=1)
    with pytest.raises(ValueError):
        f2.result(timeout=1)

"""Broker publish micro-batching on the MI355X index.

The reference routes every PUBLISH on its own: ``emqx_broker:do_publish/1``
(apps/emqx/src/emqx_broker.erl:293-298) = ``route(aggre(match_routes(Topic)),
Delivery)``, called once per ``{incoming, Packet}`` by the connection process
(emqx_connection.erl:585-587, 802-807).  Here publishes are collected into a
micro-batch -- flushed when it holds ``max_batch`` messages or when the oldest
has waited ``max_wait_ms`` -- and the whole batch is matched with ONE
``Router.match_routes_batch`` (one device launch); ``aggre/1`` (:408-424) and
the per-route dispatch (do_route2, :400-406) then run per message exactly as
in the reference, so each message gets the same route list and the same
deliveries as an unbatched publish.

Delivery itself (sessions, shared-subscription pick, cluster RPC) is out of
scope: ``dispatch(To, Msg)``, ``forward(Node, To, Msg)`` and
``share_dispatch(Group, To, Msg)`` are caller-supplied callbacks.
"""
from __future__ import annotations

import threading
import time
from collections import namedtuple
from concurrent.futures import Future

from .trie_search import term_key

Message = namedtuple("Message", "topic payload")


def aggre(routes):
    """aggre/1 (emqx_broker.erl:408-424): routes -> [{To, Node} | {To, Group}].
    Plain node routes come out in reverse order (accumulated by prepending);
    if any destination is a shared group, the result is lists:usort'ed."""
    if not routes:
        return []
    if len(routes) == 1:
        r = routes[0]
        if isinstance(r.dest, tuple):
            return [(r.topic, r.dest[0])]
        return [(r.topic, r.dest)]
    acc, dedup = [], False
    for r in routes:
        if isinstance(r.dest, tuple):
            dedup = True
            acc.insert(0, (r.topic, r.dest[0]))
        else:
            acc.insert(0, (r.topic, r.dest))
    if dedup:
        return sorted(set(acc), key=term_key)
    return acc


class Broker:
    def __init__(self, router, node=None, dispatch=None, forward=None, share_dispatch=None,
                 max_batch: int = 4096, max_wait_ms: float = 0.2, start: bool = False):
        self.router = router
        self.node = router.node if node is None else node
        self.dispatch = dispatch or (lambda to, msg: 0)
        self.forward = forward or (lambda node, to, msg: "ok")
        self.share_dispatch = share_dispatch or (lambda group, to, msg: 0)
        self.max_batch = max_batch
        self.max_wait = max_wait_ms / 1000.0
        self.batches = 0
        self._q: list = []
        self._first_at = None
        self._cv = threading.Condition()
        self._stop = False
        self._thread = None
        if start:
            self._thread = threading.Thread(target=self._loop, daemon=True)
            self._thread.start()

    # do_route2/2 (emqx_broker.erl:400-406)
    def _route2(self, to_dest, msg):
        to, dest = to_dest
        if dest == self.node:
            return (dest, to, self.dispatch(to, msg))
        if isinstance(dest, str):
            return (dest, to, self.forward(dest, to, msg))
        return ("share", to, self.share_dispatch(dest, to, msg))

    def publish_batch(self, msgs):
        """do_publish/1 for every message of a batch, with one device match.
        -> per message: (routes after aggre, route results), or the exception
        of a message whose topic is invalid (badarg): it fails alone, the
        other messages of the batch are routed (emqx_trie_search.erl:374-375
        raises in the one publishing process)."""
        if not msgs:
            return []
        all_routes = self.router.match_routes_batch([m.topic for m in msgs], errors="return")
        self.batches += 1
        out = []
        for m, routes in zip(msgs, all_routes):
            if isinstance(routes, Exception):
                out.append(routes)
                continue
            agg = aggre(routes)
            out.append((agg, [self._route2(r, m) for r in agg]))
        return out

    # ---- asynchronous micro-batching
    def publish(self, msg) -> Future:
        """Queue one message; the future resolves to (routes, results) once its
        micro-batch has been matched and dispatched."""
        fut: Future = Future()
        with self._cv:
            if not self._q:
                self._first_at = time.monotonic()
            self._q.append((msg, fut))
            if len(self._q) == 1 or len(self._q) >= self.max_batch:
                self._cv.notify()   # start the wait bound / flush a full batch
        if self._thread is None:
            self.flush_if_due()
        return fut

    def _take(self):
        batch, self._q = self._q[: self.max_batch], self._q[self.max_batch:]
        self._first_at = time.monotonic() if self._q else None
        return batch

    def _run(self, batch):
        try:
            res = self.publish_batch([m for m, _ in batch])
            for (_, fut), r in zip(batch, res):
                if isinstance(r, Exception):
                    fut.set_exception(r)        # this message only (badarg)
                else:
                    fut.set_result(r)
        except BaseException as e:   # a failure of the whole batch (device error): every caller sees it
            for _, fut in batch:
                if not fut.done():
                    fut.set_exception(e)

    def flush_if_due(self, force: bool = False):
        with self._cv:
            due = self._q and (force or len(self._q) >= self.max_batch or
                               time.monotonic() - self._first_at >= self.max_wait)
            batch = self._take() if due else []
        if batch:
            self._run(batch)
        return len(batch)

    def flush(self):
        n = 0
        while True:
            k = self.flush_if_due(force=True)
            if not k:
                return n
            n += k

    def _loop(self):
        while True:
            with self._cv:
                while not self._stop and (not self._q or (
                        len(self._q) < self.max_batch and time.monotonic() - self._first_at < self.max_wait)):
                    timeout = None if not self._q else max(0.0, self.max_wait - (time.monotonic() - self._first_at))
                    self._cv.wait(timeout)
                if self._stop and not self._q:
                    return
                batch = self._take()
            self._run(batch)

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        if self._thread:
            self._thread.join(timeout=5)
        self.flush()

"""Route-update batching: ``emqx_router_syncer`` on the MI355X index.

apps/emqx/src/emqx_router_syncer.erl.  Route ops pushed by broker workers are
stashed per route {Topic, Dest} (stash_add/merge_route_op :380-402), cut into
batches of at most ``max_batch_size`` (1000, :58) by priority (mk_batch
:297-328: reply-waiting ops first, then adds, then background deletes), and
each batch is applied with one ``Router.do_batch`` (run_batch :351-356) --
which reaches the device as ONE tm_apply_deltas before the next match: a
syncer batch is the unit of delta upload.  Replies go only to
the ops of the batch and to superseded ops (send_replies :330-347); a failed
batch is kept in the stash, the syncer sleeps ``error_delay`` ms and retries
after ``error_retry_interval`` ms (:269-277).

The gen_server's mailbox becomes a thread-safe queue; ``run_once`` is one pass
of run_batch_loop (:255-282).  ``Syncer(start=True)`` runs the loop on a
worker thread; tests drive it synchronously.
"""
from __future__ import annotations

import queue
import threading
import time

from .trie_search import term_key

PRIO_HI, PRIO_LO, PRIO_BG = 1, 2, 3
MAX_BATCH_SIZE = 1000
MIN_SYNC_INTERVAL = 0
ERROR_DELAY = 10
ERROR_RETRY_INTERVAL = 500


def designate_prio(action, opts):
    """designate_prio/2 (:154-159)."""
    if "reply" in opts:
        return PRIO_HI
    return PRIO_LO if action == "add" else PRIO_BG


class Ref:
    """A wait reference (the MRef of push/4 with #{reply => Pid})."""

    def __init__(self):
        self._ev = threading.Event()
        self.result = None

    def send(self, result):
        self.result = result
        self._ev.set()

    def wait(self, timeout=None):
        """wait/1 (:140-152)."""
        if not self._ev.wait(timeout):
            raise TimeoutError("route op not synced")
        return self.result


def _route_key(route):
    return term_key(route)


def stash_add(prio, op, stash, replies):
    """stash_add/3 + merge_route_op/2 (:380-402).  `replies` collects
    (ctx, result) sends in the order the reference would make them."""
    action, topic, dest, ctx = op
    route = (topic, dest)
    cur = stash.get(route)
    if cur is None:
        stash[route] = (action, prio, ctx)
    elif cur[0] == action:
        stash[route] = (action, prio, cur[2] + ctx)
    else:                       # the latter cancels the former, whose waiters get ok
        for ref in cur[2]:
            replies.append((ref, "ok"))
        stash[route] = (action, prio, ctx)
    return stash


def mk_batch(stash, batch_size):
    """mk_batch/2 (:297-328): -> (batch, stash left).  Erlang iterates small
    maps in key order; the stash is iterated in term order of {Topic, Dest}."""
    if len(stash) <= batch_size:
        return dict(stash), {}
    batch, left = {}, dict(stash)
    size_left = batch_size
    for prio in (PRIO_HI, PRIO_LO, PRIO_BG):
        for route in sorted(left, key=_route_key):
            if size_left <= 0:
                return batch, left
            op = left[route]
            if op[1] == prio:
                batch[route] = op
                del left[route]
                size_left -= 1
        if size_left <= 0:
            break
    return batch, left


def send_replies(errors, batch):
    """send_replies/2 (:330-347)."""
    for route, (_action, _prio, ctx) in batch.items():
        for ref in ctx:
            ref.send(errors.get(route, "ok"))


class Syncer:
    """One router-syncer worker bound to a Router (the batch handler)."""

    def __init__(self, router, max_batch_size=MAX_BATCH_SIZE, min_sync_interval=MIN_SYNC_INTERVAL,
                 error_delay=ERROR_DELAY, error_retry_interval=ERROR_RETRY_INTERVAL, batch_handler=None,
                 start=False):
        self.router = router
        self.max_batch_size = max_batch_size
        self.min_sync_interval = min_sync_interval
        self.error_delay = error_delay
        self.error_retry_interval = error_retry_interval
        self.batch_handler = batch_handler or router.do_batch
        self.stash: dict = {}
        self.suspended = False
        self.batches = 0
        self._mbox: queue.Queue = queue.Queue()
        self._retry_at = None
        self._stop = threading.Event()
        self._thread = None
        if start:
            self._thread = threading.Thread(target=self._loop, daemon=True)
            self._thread.start()

    # ---- client side (push/4, push/5)
    def push(self, action, topic, dest, opts=None):
        opts = opts or {}
        prio = designate_prio(action, opts)
        ref = Ref() if "reply" in opts else None
        self._mbox.put((prio, (action, bytes(topic), dest, [ref] if ref else [])))
        return ref if ref else "ok"

    # ---- server side
    def _drain(self, stash, replies):
        while True:
            try:
                prio, op = self._mbox.get_nowait()
            except queue.Empty:
                return stash
            stash_add(prio, op, stash, replies)

    def run_once(self):
        """One pass of run_batch_loop (:255-282); returns the number of ops applied."""
        replies = []
        self._drain(self.stash, replies)
        for ref, res in replies:
            ref.send(res)
        if self.suspended:
            return 0
        applied = 0
        while self.stash:
            batch, left = mk_batch(self.stash, self.max_batch_size)
            try:
                errors = self.batch_handler(batch)
            except Exception as e:   # the batch failed as a whole: keep it stashed
                errors = e
            if isinstance(errors, dict):
                send_replies(errors, batch)
                self.stash = left
                self.batches += 1
                applied += len(batch)
                self._retry_at = None
                replies = []
                self._drain(self.stash, replies)
                for ref, res in replies:
                    ref.send(res)
            else:
                time.sleep(self.error_delay / 1000.0)          # error_cooldown/1
                if self._retry_at is None:                      # ensure_retry_timer/1
                    self._retry_at = time.monotonic() + self.error_retry_interval / 1000.0
                break
        return applied

    def suspend(self):
        self.suspended = True

    def activate(self):
        self.suspended = False
        self.run_once()

    def stats(self):
        """stash_stats/1 (:404-418)."""
        acts = [op[0] for op in self.stash.values()]
        prios = [op[1] for op in self.stash.values()]
        return {"size": len(self.stash), "n_add": acts.count("add"), "n_delete": acts.count("delete"),
                "prio_highest": min(prios) if prios else None, "prio_lowest": max(prios) if prios else 0}

    def _loop(self):
        while not self._stop.is_set():
            try:
                item = self._mbox.get(timeout=0.05)
            except queue.Empty:
                if self._retry_at is not None and time.monotonic() >= self._retry_at:
                    self._retry_at = None
                    self.run_once()
                continue
            if self.min_sync_interval:
                time.sleep(self.min_sync_interval / 1000.0)   # collect overlapping ops
            replies = []
            stash_add(item[0], item[1], self.stash, replies)
            for ref, res in replies:
                ref.send(res)
            self.run_once()

    def close(self):
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)

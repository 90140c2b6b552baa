"""Drop-in mirror of ``emqx_topic_index`` backed by the MI355X index.

Same names, argument meaning and results as apps/emqx/src/emqx_topic_index.erl
(new/0,1 :40-48, insert/4 :53-56, delete/3 :60-62, match/2 :70-72,
matches/3 :76-78, get_id/1, get_topic/1, get_record/2 :86-106).

``Tab`` plays the part of the caller-owned ETS table: it keeps the records
(the source of truth, SURVEY.md 8b "Ownership") and interns every key
``{Filter, {ID}}`` to a dense u32 that the device index stores.  Inserts and
deletes are queued and shipped with one ``tm_apply_deltas`` call before the
next match (the router-syncer batch boundary, emqx_router_syncer.erl:297-356).
Matching always runs on the GPU through ``libtmatch``; there is no CPU path.

Concurrency (as on the reference's read_concurrency table,
emqx_topic_index.erl:41-48): any number of threads may match while one
thread writes.  A reader registers with the library's reader epochs
(include/tmatch.h) around its device batch AND the decoding of the returned
u32s; a deleted key's u32 sits in quarantine until every reader that began
before the delete has finished, so a value decodes to its own key or to
nothing (a key deleted meanwhile is dropped) -- never to a key inserted later.

Result order: the device returns keys in traversal order (ascending Erlang
term order).  ``matches/3`` returns them like the reference does -- reversed,
because match_add/2 prepends (emqx_trie_search.erl:350-356); ``[unique]``
keeps the last key per ID (maps:values): for up to 32 IDs that is the
reference's list element for element (a flatmap iterates in key term order);
beyond 32 the BEAM iterates a HAMT in the order of its internal term hash,
which this mirror does not restate, so the list is the same set of keys in
ID term order (the Erlang module, src/emqx_topic_index_gpu.erl, calls
maps:values itself and is exact); ``match/2`` is the first key in traversal
order.
"""
from __future__ import annotations

import threading
from collections import deque

import numpy as np

from . import _native
from .trie_search import (BadArg, HASH, PLUS, filter_words, get_id, get_topic, key_order,  # noqa: F401
                          make_key, term_key, topic_words)


class Tab:
    """An index table: records + the device-resident mirror of its keys."""

    def __init__(self, device: int = -1, hint_keys: int = 0, index=None, copies: int = 1):
        """copies: copies of the tables on the device (tm_options.copies; new/1's
        {copies, N}): under churn a batch after a delta runs on a copy no batch
        is reading."""
        self._index = index if index is not None else _native.Index(device=device, hint_keys=hint_keys,
                                                                    copies=copies)
        self._records: dict = {}        # key -> record        (the ETS rows)
        self._kid: dict = {}            # key -> u32 value on the device
        self._keys: list = []           # u32 -> key (None: deleted)
        self._free: list[int] = []      # u32s no reader can still return
        self._released: list[int] = []  # freed by deletes not yet shipped
        self._quarantine = deque()      # (epoch of the delete, u32): reusable once the safe epoch reaches it
        self._ops: list = []            # pending (op, filter_bytes, kid, flags)
        self._lock = threading.Lock()   # pending deltas and u32 bookkeeping (writer side)
        self._sorted = None             # (keys, order keys) in term order, for matches_filter/3

    # -- key <-> device encoding
    @staticmethod
    def _encode(key):
        """-> (filter bytes, flags) for tm_apply_deltas (include/tmatch.h "Keys")."""
        f = key[0]
        if not isinstance(f, tuple):
            return bytes(f), _native.TM_KEY_BINARY
        if len(f) == 0:
            return b"", _native.TM_KEY_EMPTY_LIST
        return encode_words(f)

    def _queue(self, op, key, kid):
        enc = self._encode(key)
        self._ops.append((op, enc[0], kid, enc[1]))

    def flush(self, commit: bool = False):
        """Ship the queued deltas as ONE call (commit: tm_commit -- the route
        mirror's group commit, which no batch waits for on the GPU)."""
        with self._lock:
            self._flush_locked(commit)

    def sync_keys(self, keys, present, commit: bool = False):
        """Reconcile `keys` (present[i]: the key is in the table) and ship the
        delta in ONE call, the queueing and the shipping under one hold of the
        lock: a reader's flush (match_kids) cannot take these ops in between
        and ship them as a plain tm_apply_deltas, which a tm_commit running
        meanwhile would publish only with itself (include/tmatch.h) -- the
        writer's commit would then find nothing to ship and return before its
        keys were readable (the router's read-your-writes)."""
        with self._lock:
            for k, here in zip(keys, present):
                if here:
                    self._insert_locked(k, [])
                else:
                    self._delete_locked(k)
            self._flush_locked(commit)

    def _flush_locked(self, commit: bool):
        if not self._ops:
            return
        ops = np.array([o[0] for o in self._ops], dtype=np.uint8)
        blob, offs = _native.pack_strings([o[1] for o in self._ops])
        vals = np.array([o[2] for o in self._ops], dtype=np.uint32)
        flags = np.array([o[3] for o in self._ops], dtype=np.uint8)
        self._ops = []
        epoch = (self._index.apply(ops, blob, offs, vals, flags, commit=True) if commit
                 else self._index.apply(ops, blob, offs, vals, flags))
        # the deletes just shipped are visible from `epoch` on: their u32s
        # wait until no reader that began earlier is running
        for kid in self._released:
            self._quarantine.append((epoch, kid))
        self._released = []

    def _take_kid(self) -> int:
        if not self._free and self._quarantine:
            _, safe = self._index.epoch()
            while self._quarantine and self._quarantine[0][0] <= safe:
                self._free.append(self._quarantine.popleft()[1])
        if self._free:
            return self._free.pop()
        self._keys.append(None)
        return len(self._keys) - 1

    # -- table operations (one writer at a time, as the reference's callers)
    def insert_key(self, key, record):
        with self._lock:
            self._insert_locked(key, record)

    def delete_key(self, key):
        with self._lock:
            self._delete_locked(key)

    def _insert_locked(self, key, record):
        if key not in self._records:
            self._sorted = None
            kid = self._take_kid()
            self._keys[kid] = key
            self._kid[key] = kid
            self._queue(_native.TM_OP_INSERT, key, kid)
        self._records[key] = record

    def _delete_locked(self, key):
        if key in self._records:
            self._sorted = None
            kid = self._kid.pop(key)
            del self._records[key]
            self._queue(_native.TM_OP_DELETE, key, kid)
            self._keys[kid] = None
            self._released.append(kid)

    def attach(self, rows, batch_size: int = 1000) -> int:
        """Boot the device mirror from an existing table (emqx_topic_index_gpu:
        attach/2): rows are (Key, Record) in the table's key order, loaded in
        batches of at most batch_size keys, one tm_apply_deltas per batch (the
        Erlang module counts the batch as it fills: linear in the rows).
        Returns the device calls made."""
        calls, k = 0, 0
        for key, rec in rows:
            self.insert_key(key, rec)
            k += 1
            if k >= batch_size:
                self.flush()
                calls, k = calls + 1, 0
        if k:
            self.flush()
            calls += 1
        return calls

    def size(self) -> int:
        return len(self._records)

    def keys(self):
        return list(self._records)

    def sorted_keys(self):
        """every key of the table in Erlang term order (the ordered_set view)"""
        if self._sorted is None:
            keys = sorted(self._records, key=key_order)
            self._sorted = (keys, [key_order(k) for k in keys])
        return self._sorted

    def lookup(self, key):
        return [self._records[key]] if key in self._records else []

    # -- matching (batched: the unit the broker micro-batch hands over)
    def match_kids(self, topics):
        """-> (list of kid arrays in traversal order, badarg flags).  The
        caller decodes the kids inside a read_begin()/read_end() pair."""
        self.flush()
        blob, offs = _native.pack_strings(topics)
        hit, vals, err = self._index.match_batch(blob, offs)
        return [vals[hit[i]:hit[i + 1]] for i in range(len(topics))], err

    def read_begin(self) -> int:
        return self._index.read_begin()

    def read_end(self, ticket: int):
        self._index.read_end(ticket)

    def decode(self, kids):
        """u32s -> keys; a key deleted since the batch began is dropped (its
        u32 is quarantined, so it cannot name a newer key yet)."""
        keys = self._keys
        return [k for k in (keys[i] for i in kids.tolist()) if k is not None]

    def stats(self) -> dict:
        self.flush()
        return self._index.stats()


def new(options=None, device: int = -1) -> Tab:
    """new/0,1: an empty index table (ETS options are accepted and ignored)."""
    return Tab(device=device)


def insert(filter_, ident, record, tab: Tab):
    """insert/4: associate Filter with ID (and Record)."""
    tab.insert_key(make_key(filter_, ident), record)
    return True


def delete(filter_, ident, tab: Tab):
    """delete/3: deleting a missing entry is not an error."""
    tab.delete_key(make_key(filter_, ident))
    return True


class TopicTooDeep(ValueError):
    """A topic of more than 65536 levels: longer than MQTT's 65535-byte
    maximum (emqx_mqtt.hrl:44), so no client can publish it; the device walk's
    scratch ends there (include/tmatch.h, err flag 2)."""


def matches_batch(topics, tab: Tab, opts=(), errors: str = "raise"):
    """matches/3 over a batch of topics (one device launch).

    A topic with a '+'/'#' level is badarg (emqx_trie_search.erl:374-375) and
    one of more than 65536 levels is TopicTooDeep; the device flags each topic
    on its own.  A batch the device failed (err flag 4: the library already
    ran it again once) raises DeviceError for the whole call -- never BadArg,
    which the reference reserves for the topic itself.  errors="raise" raises for the first such topic (one call, one
    topic: the reference's behaviour); errors="return" puts the exception in
    that topic's slot and still returns every other topic's matches -- a
    micro-batch of many publishers fails only the bad publish, as each
    publishing process does in the reference."""
    topics = [bytes(t) for t in topics]
    ticket = tab.read_begin()
    try:
        kids, err = tab.match_kids(topics)
        if len(err) and (err == 4).any():   # (the library returns TM_EDEVICE instead; never a client error)
            raise _native.DeviceError(_native.TM_EDEVICE, "batch failed on the device (err flag 4)")
        out = []
        for i, ks in enumerate(kids):
            if err[i]:
                e = TopicTooDeep(len(topics[i])) if err[i] == 2 else BadArg(topics[i])
                if errors == "raise":
                    raise e
                out.append(e)
                continue
            out.append(_finish(tab.decode(ks), opts))
    finally:
        tab.read_end(ticket)
    return out


def traversal_order(keys):
    """Device order -> the reference's traversal order.  The device emits keys
    in ascending Erlang term order of their filters, but the keys of ONE
    filter (several IDs on one filter: $share groups, many subscribers of a
    rule topic) come in the order of their u32 values, which Tab hands out by
    insertion (and reuses).  The reference orders them by {ID}
    (emqx_trie_search.erl:107-111: {Filter, {ID}} in an ordered_set), so each
    run of equal filters is sorted by the ID's term order."""
    out = []
    i, n = 0, len(keys)
    while i < n:
        j = i + 1
        f = keys[i][0]
        while j < n and keys[j][0] == f:
            j += 1
        if j - i > 1:
            out.extend(sorted(keys[i:j], key=lambda k: term_key(k[1][0])))
        else:
            out.append(keys[i])
        i = j
    return out


class FirstHit(Exception):
    """matches/3 with [return_first] found a key: the reference's search throws
    {first, Key} at the first hit (match_add/2, emqx_trie_search.erl:355-356)
    and the caller catches it (match/2 does, :172-178)."""

    def __init__(self, key):
        super().__init__(key)
        self.key = key


FIRST = "first"   # the atom matches/3 with [return_first] returns when nothing matches


def _finish(keys, opts):
    """Device keys (traversal order) -> the accumulator the reference's
    search/3 returns for `opts` (emqx_trie_search.erl:201-226): return_first
    before unique before a plain list.  With return_first: ("first", Key) for
    the first key in traversal order, or FIRST when nothing matched (its
    initial accumulator, returned as is)."""
    keys = traversal_order(keys)
    if "return_first" in opts:
        return (FIRST, keys[0]) if keys else FIRST
    if "unique" in opts:
        by_id = {}
        for k in keys:                             # traversal order; later keys win
            by_id[get_id(k)] = k
        return [by_id[i] for i in sorted(by_id, key=term_key)]
    return keys[::-1]          # matches/3 is the reverse of the traversal order (match_add/2 prepends)


def matches(topic, tab: Tab, opts=()):
    """matches/3.  With return_first it raises FirstHit(Key) at a match, as the
    reference's call throws {first, Key}, and returns FIRST otherwise."""
    r = matches_batch([topic], tab, opts)[0]
    if isinstance(r, tuple) and len(r) == 2 and r[0] == FIRST:
        raise FirstHit(r[1])
    return r


def match(topic, tab: Tab):
    """match/2: the first match in traversal order, or False."""
    keys = matches_batch([topic], tab, ())[0]
    return keys[-1] if keys else False


def matches_filter(filter_, tab: Tab, opts=()):
    """matches_filter/3 (emqx_topic_index.erl:82-84 -> emqx_trie_search.erl:186-189):
    the index keys a subscription to `filter_` covers, by the reference's
    ordered search (filter_words/1, base_init/1, compare/3 with the filter
    clauses :291-300, no match_topics phase -- binary keys never match).

    Its result depends on where the ordered walk stops (a stored key below the
    query at a query '+' ends the whole search), which the trie walk has no
    notion of, so the device runs the reference's walk itself over the keys in
    term order (tm_matches_filter_ex) -- every key of the table, those no topic
    can match included (binary words '+'/'#' or holding a '/': the escaped
    key form), and a query given as a word list in the same form.  Callers are
    control-plane (durable-storage stream discovery,
    emqx_ds_new_streams.erl:325)."""
    if isinstance(filter_, (bytes, bytearray)):
        q, qf = bytes(filter_), 0
    else:
        q, qf = encode_words(tuple(filter_words(filter_)))
    ticket = tab.read_begin()
    try:
        tab.flush()
        blob, offs = _native.pack_strings([q])
        _, vals, err = tab._index.matches_filter_batch(blob, offs, np.array([qf], np.uint8))
        if len(err) and err[0]:   # the device walk hit its step bound: no silent truncation
            raise RuntimeError(f"matches_filter: device walk exceeded its step bound for {filter_!r}")
        return _finish(tab.decode(vals), opts)
    finally:
        tab.read_end(ticket)


def encode_words(words):
    """A word list -> (bytes, flags) in the C ABI's key form: '/'-joined
    (TM_KEY_WORDS), or -- when a binary word holds a '/' or equals "+" / "#",
    which no topic level can equal -- the escaped form (TM_KEY_WORDS |
    TM_KEY_ESCAPED: "\\/" a '/', "\\\\" a '\\', "\\+" / "\\#" the binary
    words, bare "+" / "#" the wildcards).  The library keeps such a key for
    matches_filter/3 only; it never matches a topic."""
    plain, esc, escaped = [], [], False
    for w in words:
        if w == PLUS or w == HASH:
            plain.append(w.encode())
            esc.append(w.encode())
        elif isinstance(w, (bytes, bytearray)):
            w = bytes(w)
            if w in (b"+", b"#"):
                escaped = True
                esc.append(b"\\" + w)
            else:
                escaped |= b"/" in w
                esc.append(w.replace(b"\\", b"\\\\").replace(b"/", b"\\/"))
            plain.append(w)
        else:
            raise TypeError(f"bad filter word {w!r}")
    if escaped:
        return b"/".join(esc), _native.TM_KEY_WORDS | _native.TM_KEY_ESCAPED
    return b"/".join(plain), _native.TM_KEY_WORDS


def get_record(key, tab: Tab):
    """get_record/2: [Record] or [] if the entry was deleted meanwhile."""
    return tab.lookup(key)


DeviceError = _native.DeviceError

__all__ = ["new", "insert", "delete", "match", "matches", "matches_batch", "matches_filter", "make_key", "get_id",
           "get_topic", "get_record", "Tab", "BadArg", "TopicTooDeep", "DeviceError", "FirstHit", "FIRST"]

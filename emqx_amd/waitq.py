"""Drop-in mirror of ``emqx_ds_beamformer_waitq`` -- the durable-storage
beamformer's index of poll requests waiting for stream events
(apps/emqx_durable_storage/src/emqx_ds_beamformer_waitq.erl:30-62).

The reference keys one private ordered_set by ``{Stream, make_key(Filter,
ID)}`` (:50-51) and matches a topic with ``emqx_trie_search:matches/3``
through a custom ``NextF`` that stops at the stream's last key (:54-62): the
topic index restricted to one stream.  Here each stream has its own
device-backed ``topic_index`` table (created on its first insert), so a match
walks only that stream's filters on the GPU, and the records stay host-side as
the ETS rows do.  ``matches/3`` returns the records of the matching keys in the
reference's order (``matches/3`` of the index: reverse traversal order).
"""
from __future__ import annotations

from . import topic_index as ti


class WaitQ:
    """The table: stream -> device-backed topic_index table."""

    def __init__(self, device: int = -1):
        self._device = device
        self._streams: dict = {}

    def stream_tab(self, stream, create: bool = False):
        t = self._streams.get(stream)
        if t is None and create:
            t = self._streams[stream] = ti.new(device=self._device)
        return t


def new(device: int = -1) -> WaitQ:
    """new/0 (:33-34)."""
    return WaitQ(device)


def insert(stream, filter_, ident, record, tab: WaitQ):
    """insert/5 (:36-38): ets:insert of {{Stream, Key}, Record} (a set: the same key replaces its record)."""
    return ti.insert(filter_, ident, record, tab.stream_tab(stream, create=True))


def delete(stream, filter_, ident, tab: WaitQ):
    """delete/4 (:40-41)."""
    t = tab.stream_tab(stream)
    if t is not None:
        ti.delete(filter_, ident, t)
    return True


def matches(stream, topic, tab: WaitQ):
    """matches/3 (:43-45): the records of the stream's keys matching `topic`
    (a binary or a list of words, emqx_trie_search:topic_words/1)."""
    t = tab.stream_tab(stream)
    if t is None:
        return []
    if isinstance(topic, (list, tuple)):
        if not topic:
            return [r for k in _matches_no_levels(t) for r in ti.get_record(k, t)]
        topic = b"/".join(bytes(w) for w in topic)
    return [r for k in ti.matches(topic, t, []) for r in ti.get_record(k, t)]


def _matches_no_levels(t):
    """matches/3 of the word list [] (zero levels -- no topic binary has that
    form: b"" is one empty level): compare/3 gives match_full for a stored []
    and a stored ['#'] (emqx_trie_search.erl:262-290) and `lower` for every
    other word list, and match_topics/4 then stops (:381-389).  So the keys are
    those two filters' keys, in traversal order reversed (match_add/2)."""
    keys, _ = t.sorted_keys()
    hits = [k for k in keys if isinstance(k[0], tuple) and k[0] in ((), (ti.HASH,))]
    return hits[::-1]

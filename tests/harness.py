"""Shared test harness: runs the golden known-answer cases against a backend.

A backend turns (inserts, topic) into the matched keys in TRAVERSAL order
(ascending Erlang term order), or raises BadArg.  Two backends exist:
the CPU oracle (OracleBackend, here) and the GPU product path
(emqx_amd.topic_index.Tab, in the gpu tests).
"""
from __future__ import annotations

import json
from pathlib import Path

from emqx_amd.trie_search import BadArg, get_id, get_topic, key_order, make_key, term_key
from emqx_amd.topic_index import _finish

GOLDEN = json.loads((Path(__file__).parent / "golden" / "reference_vectors.json").read_text())


def case_keys(case):
    """keys of a case, and u32 values assigned in (ID, filter) term order so the
    value order inside one filter is the ID term order."""
    keys = []
    for ins in case["inserts"]:
        f, ident = ins[0].encode(), ins[1]
        opts = ins[2] if len(ins) > 2 else {}
        if opts.get("words"):
            from emqx_amd.trie_search import filter as tfilter
            k = make_key(tfilter(f), ident)
        else:
            k = make_key(f, ident)
        if k not in keys:
            keys.append(k)
    ordered = sorted(keys, key=lambda k: (term_key(get_id(k)), key_order(k)))
    return keys, {k: i for i, k in enumerate(ordered)}


def encode_key(k):
    f = k[0]
    if isinstance(f, tuple):
        if not f:
            return b"", 2
        return b"/".join(w.encode() if isinstance(w, str) else w for w in f), 1
    return f, 0


class OracleBackend:
    def __init__(self, keys, kid):
        from pyoracle import Oracle
        self.o = Oracle()
        self.by_kid = {v: k for k, v in kid.items()}
        for k in keys:
            f, fl = encode_key(k)
            self.o.insert(f, kid[k], fl)

    def traversal(self, topic: bytes):
        r = self.o.matches(topic)
        if r is None:
            raise BadArg(topic)
        return [self.by_kid[v] for v in r]


def run_checks(case, traversal_fn):
    """traversal_fn(topic) -> keys in traversal order.  Asserts every check."""
    for chk in case["checks"]:
        t = chk["topic"].encode()
        kind = chk["kind"]
        if kind == "badarg":
            try:
                traversal_fn(t)
            except BadArg:
                continue
            raise AssertionError(f"{case['name']}: {t!r} should be badarg")
        keys = traversal_fn(t)
        assert keys == sorted(keys, key=key_order), f"{case['name']}: not in traversal order"
        if kind == "match":
            exp = chk["expect"]
            got = False if not keys else [get_topic(keys[0]).decode(), get_id(keys[0])]
            assert got == exp, (case["name"], t, got, exp)
            # matches/3 with [return_first] (emqx_trie_search.erl:201-211, 355-356):
            # {first, Key} thrown at the first hit, the atom `first` without one
            rf = _finish(keys, ["return_first"])
            if exp is False:
                assert rf == "first", (case["name"], t, rf)
            else:
                assert rf[0] == "first" and [get_topic(rf[1]).decode(), get_id(rf[1])] == exp, (case["name"], t, rf)
        elif kind == "match_id":
            assert keys and get_id(keys[0]) == chk["expect"], (case["name"], t, keys)
        elif kind == "sorted_topics":
            got = [get_topic(k).decode() for k in keys]
            assert got == chk["expect"], (case["name"], t, got)
        elif kind == "ids":
            got = [get_id(k) for k in _finish(keys, chk["opts"])]
            assert got == chk["expect"], (case["name"], t, got, chk["expect"])
        elif kind == "count":
            assert len(keys) == chk["expect"], (case["name"], t, keys)
        else:
            raise AssertionError(kind)


class RouterModel:
    """The route tables of emqx_router's v2 schema restated for tests
    (emqx_router.erl:483-516): wildcard routes are index keys
    make_key(Topic, Dest); exact routes are rows of a bag in insertion order.
    expected() answers match_routes/1 with the CPU oracle for the wildcard
    part -- an independent expectation for the GPU router, syncer and broker."""

    def __init__(self):
        self.wild = set()
        self.bag = {}

    def add(self, topic, dest):
        from emqx_amd.trie_search import filter as tfilter
        if tfilter(topic) is not False:
            self.wild.add(make_key(topic, dest))
        else:
            row = self.bag.setdefault(topic, [])
            if dest not in row:
                row.append(dest)

    def delete(self, topic, dest):
        from emqx_amd.trie_search import filter as tfilter
        if tfilter(topic) is not False:
            self.wild.discard(make_key(topic, dest))
        elif dest in self.bag.get(topic, []):
            self.bag[topic].remove(dest)
            if not self.bag[topic]:
                del self.bag[topic]

    def expected(self, topics):
        """-> per topic: [Route] as match_routes/1 returns them, or BadArg."""
        from pyoracle import Oracle
        from emqx_amd.router import Route
        keys = sorted(self.wild, key=key_order)          # values in term order: a filter's IDs ascend
        o = Oracle()
        for i, k in enumerate(keys):
            f, fl = encode_key(k)
            o.insert(f, i, fl)
        out = []
        for t in topics:
            tr = o.matches(bytes(t))
            if tr is None:
                out.append(BadArg(t))
                continue
            ws = [keys[v] for v in tr]
            out.append([Route(t, d) for d in self.bag.get(t, [])] +
                       [Route(get_topic(k), get_id(k)) for k in reversed(ws)])
        return out

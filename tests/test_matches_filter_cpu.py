"""matches_filter/3 (emqx_trie_search.erl:186-189 + the filter clauses of
compare/3, :291-300): the Python mirror's ordered search
(oracle/pyoracle.py search_filter, the Python restatement the device walk
runs over a table's ordered key set) against the C oracle's independent
restatement (oracle/tm_oracle.c orc_matches_filter, a sorted array with its own
term-order comparator), plus known answers worked out from the reference's
clauses -- the reference's own suites never call matches_filter, so these are
the pins ("parity unpinned" beyond this restatement: no Erlang runtime here).
"""
import random

import pytest

from emqx_amd.trie_search import filter_words, get_id, key_order, make_key
from pyoracle import Oracle, search_filter


def _index(filters, words_form=()):
    """filters: list of bytes; ids = positions.  -> (sorted keys, order, oracle)"""
    o = Oracle()
    keys = []
    for i, f in enumerate(filters):
        wf = i in words_form
        k = make_key(tuple(filter_words(f)) if wf else f, i)
        keys.append(k)
        o.insert(f, i, 1 if wf else 0)
    keys = sorted(set(keys), key=key_order)
    return keys, [key_order(k) for k in keys], o


def _mirror(keys, order, q):
    return [get_id(k) for k in search_filter(keys, order, filter_words(q))]


KNOWN = [
    # (stored filters, query, traversal-order ids; the reference's list is the reverse)
    # a query '+' over a stored word: a later 'lower' is not turned into a seek
    ([b"a/b/c", b"a/+/c", b"a/#", b"#", b"+/+/c", b"a/b/d/#", b"x/y"], b"a/+", [3, 2]),
    ([b"a/b/c", b"a/+/c", b"a/#", b"#", b"+/+/c", b"a/b/d/#", b"x/y"], b"a/+/c", [3, 4, 2, 1]),
    # '#' matches every list key; the walk stops at the first binary key
    ([b"a/b/c", b"a/+/c", b"a/#", b"#", b"+/+/c", b"a/b/d/#", b"x/y"], b"#", [3, 4, 2, 1, 5]),
    # a stored key shorter than a query ending in '#' is only a prefix
    ([b"a/+", b"a/+/b"], b"a/+/#", [1]),
    # the early stop: a/b/x/# is below a/+/c at the '+' level, so a/z/c/# is never reached
    ([b"a/b/x/#", b"a/z/c/#"], b"a/+/c", []),
    ([b"a/z/c/#"], b"a/+/c", [0]),
    # base_init: a '$' first word starts the walk at ['$SYS'] (root '#'/'+' skipped)
    ([b"#", b"+/+", b"$SYS/#", b"$SYS/+/x"], b"$SYS/#", [2, 3]),
    # ... and only through the query's own first word: '+/#' also covers '$SYS/..'
    ([b"#", b"+/+", b"$SYS/#", b"$SYS/+/x"], b"+/#", [0, 1, 2, 3]),
    # binary (exact) keys never match a filter query
    ([b"a/b", b"a/+"], b"a/b", [1]),
]


@pytest.mark.parametrize("filters,query,expect", KNOWN)
def test_matches_filter_known_answers(filters, query, expect):
    keys, order, o = _index(filters)
    assert _mirror(keys, order, query) == expect
    assert o.matches_filter(query) == expect


def _rand_level(r):
    c = r.random()
    if c < 0.2:
        return r.choice([b"a", b"b", b"c"])
    if c < 0.27:
        return b""
    if c < 0.32:
        return b"$" + r.choice([b"SYS", b"a"])
    return ("%X" % r.randint(1, 6)).encode()


def _rand_filter(r, n, wild, hash_last=False):
    out = []
    for i in range(n):
        p = r.choices(["level", "+", "#"], wild)[0]
        if p == "#" and hash_last and i != n - 1:
            p = "+"
        out.append(b"#" if p == "#" else b"+" if p == "+" else _rand_level(r))
    return b"/".join(out)


@pytest.mark.parametrize("seed", range(12))
def test_matches_filter_mirror_vs_oracle(seed):
    """Random key sets (binary keys, '+'/'#' anywhere -- '#' not last included
    -- word-list keys, '$' words) and random filter queries: the mirror and the
    oracle return the same ids in the same order.  Queries are valid MQTT
    filters ('#' last only; callers such as emqx_ds_new_streams.erl:325 pass
    subscription filters): with a '#' mid-query the reference's seek goes
    backwards ('#' < '+' in term order) and the walk never ends."""
    r = random.Random(0x454D5158 + 500 + seed)
    filters = [_rand_filter(r, r.randint(1, 5), [6, 2, 1]) for _ in range(300)]
    wf = {i for i in range(len(filters)) if r.random() < 0.1}
    keys, order, o = _index(filters, wf)
    for _ in range(200):
        q = _rand_filter(r, r.randint(1, 5), [4, 3, 1], hash_last=True)
        assert _mirror(keys, order, q) == o.matches_filter(q), q

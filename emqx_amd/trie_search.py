"""Key helpers of the topic index (pure functions, no matching here).

Python mirror of the key vocabulary of ``emqx_trie_search``
(apps/emqx/src/emqx_trie_search.erl):

- a *word* is ``bytes`` (a binary level) or the atoms ``PLUS`` ('+') / ``HASH`` ('#');
- a *key* is ``(filter, (ID,))`` where ``filter`` is ``bytes`` (a topic without
  wildcards, kept as a binary) or a ``tuple`` of words (an Erlang word list);
  ``make_key/2`` decides which (:115-128);
- ``term_key`` orders Erlang terms the way the BEAM does (numbers < atoms <
  tuples < lists < binaries), so that list results can be put in the exact
  order the reference returns them.

Erlang atoms are Python ``str``; Erlang binaries are ``bytes``; Erlang tuples
are ``tuple``; Erlang lists are ``list`` (or ``tuple`` inside a key's filter).
"""
from __future__ import annotations


class BadArg(ValueError):
    """error(badarg) -- a topic level equal to '+' or '#' (emqx_trie_search.erl:374-375)."""


PLUS = "+"
HASH = "#"


def tokens(topic: bytes) -> list[bytes]:
    """emqx_topic:tokens/1 (emqx_topic.erl:318-319): split on '/', keep empty levels."""
    return bytes(topic).split(b"/")


def filter_words(topic) -> list:
    """filter_words/1 (emqx_trie_search.erl:358-366): '+'/'#' levels become atoms."""
    if isinstance(topic, (list, tuple)):
        return list(topic)
    return [PLUS if w == b"+" else HASH if w == b"#" else w for w in tokens(topic)]


def topic_words(topic) -> list[bytes]:
    """topic_words/1 + word/2 (emqx_trie_search.erl:368-378)."""
    if isinstance(topic, (list, tuple)):
        return list(topic)
    ws = tokens(topic)
    for w in ws:
        if w == b"+" or w == b"#":
            raise BadArg(topic)
    return ws


def wildcard(words) -> bool:
    """emqx_topic:wildcard/1 (emqx_topic.erl:65-77) on a word list."""
    return any(w == PLUS or w == HASH for w in words)


def filter(topic):  # noqa: A001 - reference name
    """filter/1 (emqx_trie_search.erl:136-140): word list if wildcard, else False."""
    ws = filter_words(topic)
    return ws if wildcard(ws) else False


def make_key(topic_or_words, ident):
    """make_key/2 (emqx_trie_search.erl:115-128)."""
    if isinstance(topic_or_words, (list, tuple)):
        return (tuple(topic_or_words), (ident,))
    t = bytes(topic_or_words)
    ws = filter(t)
    if ws is False:
        return (t, (ident,))
    return (tuple(ws), (ident,))


def get_id(key):
    """get_id/1 (emqx_trie_search.erl:142-145)."""
    return key[1][0]


def join(words) -> bytes:
    """emqx_topic:join/1 (emqx_topic.erl:351-363)."""
    out = []
    for i, w in enumerate(words):
        if w == HASH and i != len(words) - 1:
            raise ValueError("topic_invalid_#")
        out.append(w.encode() if isinstance(w, str) else bytes(w))
    return b"/".join(out)


def get_topic(key) -> bytes:
    """get_topic/1 (emqx_trie_search.erl:147-152)."""
    f = key[0]
    return join(f) if isinstance(f, tuple) else f


# ---------------------------------------------------------------- term order

def term_key(x):
    """Sort key giving Erlang's standard term order for the types used here."""
    if isinstance(x, bool):
        return (1, b"true" if x else b"false")
    if isinstance(x, (int, float)):
        return (0, x)
    if isinstance(x, str):
        return (1, x.encode())
    if isinstance(x, tuple):
        return (6, len(x), tuple(term_key(e) for e in x))
    if isinstance(x, list):
        return (8, tuple(term_key(e) for e in x))
    if isinstance(x, (bytes, bytearray, memoryview)):
        return (9, bytes(x))
    raise TypeError(f"no Erlang term order for {type(x).__name__}")


def key_order(key):
    """Term order of an index key {Filter, {ID}} (filter word lists are lists)."""
    f, (ident,) = key
    fk = (8, tuple(term_key(w) for w in f)) if isinstance(f, tuple) else (9, bytes(f))
    return (fk, term_key(ident))

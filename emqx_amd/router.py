"""Route table with the v2 schema of ``emqx_router`` on the MI355X index.

apps/emqx/src/emqx_router.erl: exact topics go to the bag table
(``emqx_route``, :431-432, :483-495), wildcard filters to the topic index
(``emqx_route_filters``, :489-490); ``match_routes/1`` (:205-212, :511-516) is
``lookup_routes(Topic) ++ [match_to_route(M) || M <- matches(Topic, Filters, [])]``
with ``match_to_route`` = ``#route{topic = get_topic(M), dest = get_id(M)}``
(:648-649).  ``match_routes_batch`` is the micro-batched form the broker
publish path hands over: one device launch per batch.
"""
from __future__ import annotations

from collections import namedtuple

from . import topic_index as ti
from .trie_search import filter as tfilter, make_key, term_key

Route = namedtuple("Route", "topic dest")


def route_order(r: Route):
    return (term_key(r.topic), term_key(r.dest))


class Router:
    def __init__(self, node="node", device: int = -1):
        self.node = node
        self._bag: dict[bytes, list] = {}       # emqx_route: Topic -> [Dest] (insertion order)
        self._filters = ti.Tab(device=device)   # emqx_route_filters

    # add_route/1,2 + do_add_route (emqx_router.erl:178-196, 483-495)
    def add_route(self, topic, dest=None):
        topic = bytes(topic)
        dest = self.node if dest is None else dest
        if tfilter(topic) is not False:
            self._filters.insert_key(make_key(topic, dest), [])
        else:
            dests = self._bag.setdefault(topic, [])
            if dest not in dests:
                dests.append(dest)

    # delete_route/1,2 (emqx_router.erl:218-234, 497-509)
    def delete_route(self, topic, dest=None):
        topic = bytes(topic)
        dest = self.node if dest is None else dest
        if tfilter(topic) is not False:
            self._filters.delete_key(make_key(topic, dest))
        else:
            dests = self._bag.get(topic, [])
            if dest in dests:
                dests.remove(dest)
            if not dests:
                self._bag.pop(topic, None)

    def lookup_routes(self, topic):
        return [Route(bytes(topic), d) for d in self._bag.get(bytes(topic), [])]

    def match_routes_batch(self, topics):
        topics = [bytes(t) for t in topics]
        matched = ti.matches_batch(topics, self._filters, ())
        return [self.lookup_routes(t) + [Route(ti.get_topic(m), ti.get_id(m)) for m in ms]
                for t, ms in zip(topics, matched)]

    def match_routes(self, topic):
        return self.match_routes_batch([topic])[0]

    def topics(self):
        """topics/0: distinct route topics (exact and wildcard)."""
        out = set(self._bag)
        out.update(ti.get_topic(k) for k in self._filters.keys())
        return list(out)

    def stats_n_routes(self):
        return sum(len(v) for v in self._bag.values()) + self._filters.size()

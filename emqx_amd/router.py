"""Route table with the v2 schema of ``emqx_router`` on the MI355X index.

apps/emqx/src/emqx_router.erl, schema v2 (:477-578): exact topics go to the bag
table ``emqx_route`` (:483-495), wildcard filters to the topic index
``emqx_route_filters`` (:489-490); ``match_routes/1`` (:205-212, :511-516) is

    lookup_route_tab(Topic) ++ [match_to_route(M) || M <- matches(Topic, Filters, [])]

with ``match_to_route`` = ``#route{topic = get_topic(M), dest = get_id(M)}``
(:648-649).

MI355X layout: both tables are mirrored into ONE device index
-- wildcard routes as word-list keys (trie terminals), exact routes as binary
keys (the index's exact table) -- so a publish batch is answered by one device
launch.  The device returns a topic's keys in traversal order: word-list keys
first, binary keys after them.  The binary keys of topic T are exactly T's bag
rows; the host puts them in the bag's insertion order (ets:lookup on a bag) and
the word-list keys in matches/3 order (reverse traversal), then concatenates.
The host dict of bag rows is the ETS table's stand-in (source of truth, for
lookup_routes/has_route/cleanup); matching reads it only for the insertion
order of the bag rows the device found.

Writes: ``add_route``/``delete_route`` (the single-op path, :178-196,
:218-234), ``do_batch`` (the router-syncer batch, :255-273), table events
replicated by mria from other nodes (``on_table_event``, the
``mnesia:subscribe({table, T, detailed})`` hook of SURVEY.md 8f.1), and
``cleanup_routes`` (node down, :535-578).  Every write becomes a delta of the
device index, shipped with one tm_apply_deltas before the next match.
"""
from __future__ import annotations

from collections import namedtuple

from . import topic_index as ti
from .trie_search import filter as tfilter, make_key, term_key

Route = namedtuple("Route", "topic dest")
RouteIdx = namedtuple("RouteIdx", "entry")      # #routeidx{entry = Key} of emqx_route_filters


def route_order(r: Route):
    return (term_key(r.topic), term_key(r.dest))


def get_dest_node(dest):
    """get_dest_node/1 (emqx_router.erl:580-585): the node a destination lives on."""
    if isinstance(dest, tuple) and len(dest) == 2:
        if dest[0] == "external":
            return dest
        return dest[1]
    return dest


class Router:
    def __init__(self, node="node", device: int = -1):
        self.node = node
        self._bag: dict[bytes, dict] = {}        # emqx_route: Topic -> {Dest: seq} (insertion order)
        self._seq = 0
        self._filters = ti.Tab(device=device)    # emqx_route_filters + the bag's device mirror

    # ---------------------------------------------------------------- writes
    def _bag_insert(self, topic, dest):
        dests = self._bag.setdefault(topic, {})
        if dest not in dests:
            self._seq += 1
            dests[dest] = self._seq
            self._filters.insert_key(make_key(topic, dest), [])

    def _bag_delete(self, topic, dest):
        dests = self._bag.get(topic)
        if dests and dest in dests:
            del dests[dest]
            self._filters.delete_key(make_key(topic, dest))
            if not dests:
                del self._bag[topic]

    # mria_insert_route_v2 (emqx_router.erl:483-490)
    def add_route(self, topic, dest=None):
        topic = bytes(topic)
        dest = self.node if dest is None else dest
        if tfilter(topic) is not False:
            self._filters.insert_key(make_key(topic, dest), [])
        else:
            self._bag_insert(topic, dest)
        return "ok"

    # mria_delete_route_v2 (emqx_router.erl:497-509)
    def delete_route(self, topic, dest=None):
        topic = bytes(topic)
        dest = self.node if dest is None else dest
        if tfilter(topic) is not False:
            self._filters.delete_key(make_key(topic, dest))
        else:
            self._bag_delete(topic, dest)
        return "ok"

    def do_batch(self, batch: dict) -> dict:
        """do_batch/1 (emqx_router.erl:255-273): apply a syncer batch
        {(Topic, Dest): (Action, Prio, Ctx)}; returns {(Topic, Dest): Error} for
        failed ops (empty on success).  The whole batch reaches the device as
        one tm_apply_deltas before the next match."""
        errors = {}
        for (topic, dest), op in batch.items():
            try:
                if op[0] == "add":
                    self.add_route(topic, dest)
                else:
                    self.delete_route(topic, dest)
            except Exception as e:   # reported per route, like mria_batch_run's results
                errors[(topic, dest)] = ("error", repr(e))
        return errors

    def on_table_event(self, event):
        """A replicated write seen through mnesia:subscribe({table, T, detailed}):
        ('write', Route | RouteIdx) or ('delete', Route | RouteIdx).  Keeps the
        device mirror in step with writes that bypass this node's router
        (SURVEY.md 3.2, 8f.1)."""
        op, rec = event
        if isinstance(rec, RouteIdx):
            (self._filters.insert_key if op == "write" else self._filters.delete_key)(*(
                (rec.entry, []) if op == "write" else (rec.entry,)))
        elif isinstance(rec, Route):
            (self._bag_insert if op == "write" else self._bag_delete)(bytes(rec.topic), rec.dest)
        else:
            raise TypeError(f"not a route table record: {rec!r}")

    def on_table_events(self, events):
        """A run of replicated table events -- everything the mirror's event
        process drained from its mailbox (src/emqx_router_gpu.erl) -- shipped
        to the device as ONE delta batch (emqx_topic_index_gpu:table_events/2).
        A node-down cleanup reaches the mirror this way: mria's match_delete
        on both tables (emqx_router.erl:535-550) produces a delete event per
        route, and the mirror never writes the mria-managed table itself."""
        for ev in events:
            self.on_table_event(ev)
        self._filters.flush()

    def attach(self, route_rows, filter_rows, batch_size: int = 1000) -> int:
        """Boot from existing route tables (emqx_router_gpu:attach/1 over
        ?ROUTE_TAB_FILTERS; the bag's rows as well, since its topics are binary
        keys of the same device index): route_rows are Route(topic, dest) in
        bag insertion order, filter_rows RouteIdx(entry) in key order; at most
        batch_size keys per tm_apply_deltas.  Returns the device calls made."""
        def rows():
            for r in route_rows:
                dests = self._bag.setdefault(bytes(r.topic), {})
                if r.dest not in dests:
                    self._seq += 1
                    dests[r.dest] = self._seq
                    yield make_key(bytes(r.topic), r.dest), []
            for r in filter_rows:
                yield r.entry, []
        return self._filters.attach(rows(), batch_size)

    def cleanup_routes(self, node):
        """cleanup_routes/1 (emqx_router.erl:535-578): drop every route whose
        destination lives on `node` (a dead node), wildcard and exact alike."""
        for key in self._filters.keys():
            if isinstance(key[0], tuple) and get_dest_node(key[1][0]) == node:
                self._filters.delete_key(key)
        for topic in list(self._bag):
            for dest in list(self._bag[topic]):
                if get_dest_node(dest) == node:
                    self._bag_delete(topic, dest)
        return "ok"

    # ----------------------------------------------------------------- reads
    def lookup_routes(self, topic):
        """lookup_routes/1 (emqx_router.erl:518-526)."""
        topic = bytes(topic)
        if tfilter(topic) is not False:
            return [Route(topic, key[1][0]) for key in self._filters.keys()
                    if isinstance(key[0], tuple) and key == make_key(topic, key[1][0])]
        dests = self._bag.get(topic, {})
        return [Route(topic, d) for d in sorted(dests, key=dests.get)]

    def has_route(self, topic, dest):
        """has_route/2 (emqx_router.erl:528-533)."""
        topic = bytes(topic)
        if tfilter(topic) is not False:
            return make_key(topic, dest) in self._filters._records
        return dest in self._bag.get(topic, {})

    def match_routes_batch(self, topics, errors: str = "raise"):
        """match_routes/1 over a batch of publish topics: one device launch.
        errors="return": a bad topic's slot holds its BadArg instead of
        failing the batch (topic_index.matches_batch)."""
        topics = [bytes(t) for t in topics]
        matched = ti.matches_batch(topics, self._filters, (), errors=errors)
        out = []
        for t, ms in zip(topics, matched):
            if isinstance(ms, Exception):
                out.append(ms)
                continue
            exact, wild = [], []
            for m in ms:
                (wild if isinstance(m[0], tuple) else exact).append(m)
            seq = self._bag.get(t, {})
            exact.sort(key=lambda m: seq[m[1][0]])          # bag insertion order
            out.append([Route(t, m[1][0]) for m in exact] +
                       [Route(ti.get_topic(m), ti.get_id(m)) for m in wild])
        return out

    def match_routes(self, topic):
        return self.match_routes_batch([topic])[0]

    def topics(self):
        """topics/0 = list_topics_v2 (emqx_router.erl:627-630): the bag's topics,
        then the topic of every wildcard key (one per route, in key order)."""
        wild = sorted((k for k in self._filters.keys() if isinstance(k[0], tuple)), key=ti.key_order)
        return sorted(self._bag) + [ti.get_topic(k) for k in wild]

    def stats_n_routes(self):
        """stats(n_routes) (emqx_router.erl:632-635)."""
        return self._filters.size()

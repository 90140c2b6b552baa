// workload.cpp -- deterministic synthetic filter / topic / delta sets for the
// benchmark configs of BASELINE.json.  Bench + test
// infrastructure (libtmwork.so), not part of the match path.
//
// Every item is a pure function of (config, seed, index): filter i is built
// from a splitmix64 stream seeded with mix(seed, i), so any shard or range can
// be generated on any rank or thread without the others (C4 generates only its
// own 1/N of 100M filters).  Level words are ASCII derived from the PRNG.
//
//  C1  10k filters: 70% exact, 20% one or two levels '+', 10% prefix(1..L-1)/'#';
//      depth 4-6, per-level vocabularies 16/64/256/1024/4096/16384.
//      Topics: depth 4-6; 50% instantiate a filter, 50% random words.
//  C2  1M 'fleet/{id}/sensor/+' (values = id) + 1k global rules, 250 values
//      each on '#', 'fleet/#', '+/+/sensor/#', 'fleet/+/sensor/#'
//      (variant 'nm': the globals are 'rules/{k}/#' and match nothing).
//      Topics 'fleet/{id}/sensor/{m}', id uniform in [0, 1.2M), m of 16 names.
//  C3  10M mixed: 60% exact, 25% '+', 10% '#' (prefix 2..L-1), 4% $share
//      (the group's real filter -- half of them re-subscribe an existing
//      filter -- with its own dest value, as emqx_shared_sub.erl:450 does),
//      1% '$SYS/...' filters, plus the globals '#' and '+/#' that '$SYS'
//      topics must not hit.  Vocabularies 16/4096/65536/65536/1024/256.
//      Topics: 2% '$SYS/...', 49% instantiate a filter, 49% random.
//  C4  = C3 at 100M, sharded by filter index mod N.
//  C3deep (cfg 30) = C3 filters; C3 topics of which 10% are extended with
//      random words to 33-64 levels (the deep-topic path).
//  C5  = C3 base + deltas: even delta k subscribes new filter F + k/2, odd
//      delta unsubscribes base filter (k/2 * P) mod F (P coprime to F), so
//      every unsubscribe removes a live key exactly once.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() { s += 0x9e3779b97f4a7c15ull; return mix64(s); }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

struct Cfg {
    int id;
    uint64_t cards[6];
    int hash_min;      // smallest '#' prefix length
    int pct_exact, pct_plus, pct_hash, pct_share, pct_sys;
};

const Cfg C1 = {1, {16, 64, 256, 1024, 4096, 16384}, 1, 70, 20, 10, 0, 0};
const Cfg C3 = {3, {16, 4096, 65536, 65536, 1024, 256}, 2, 60, 25, 10, 4, 1};

std::string level_word(uint64_t seed, int level, uint64_t idx) {
    static const char al[] = "abcdefghijklmnopqrstuvwxyz0123456789";
    uint64_t h = mix64(seed ^ 0x574f5244ull ^ ((uint64_t)level << 48) ^ (idx * 0x9e3779b97f4a7c15ull));
    int len = 3 + (int)(h % 6);
    std::string w;
    for (int k = 0; k < len; k++) {
        uint64_t r = mix64(h + (uint64_t)k + 1);
        w.push_back(al[r % 36]);
    }
    return w;
}

enum Kind { K_EXACT, K_PLUS, K_HASH };

// word list of a generated filter; "+" / "#" are the wildcard levels
void mixed_filter(const Cfg &c, uint64_t seed, uint64_t i, std::vector<std::string> &w, int *kind_out) {
    Rng r(mix64(seed ^ (i * 0x2545f4914f6cdd1dull)));
    w.clear();
    uint64_t pick = r.below(100);
    bool sys = false;
    int share_dup = -1;
    if ((int)pick >= c.pct_exact + c.pct_plus + c.pct_hash) {
        if ((int)pick < c.pct_exact + c.pct_plus + c.pct_hash + c.pct_share) {
            // $share/{g}/<real filter>: the index stores the real filter
            if (r.below(2) && i > 0) share_dup = 1;
        } else {
            sys = true;
        }
        pick = r.below(c.pct_exact + c.pct_plus + c.pct_hash);
    }
    if (share_dup == 1) {   // the group subscribes to a filter somebody already has
        uint64_t j = r.below(i);
        mixed_filter(c, seed, j, w, kind_out);
        return;
    }
    int kind = (int)pick < c.pct_exact ? K_EXACT : (int)pick < c.pct_exact + c.pct_plus ? K_PLUS : K_HASH;
    int L = 4 + (int)r.below(3);
    for (int l = 0; l < L; l++) w.push_back(level_word(seed, l, r.below(c.cards[l])));
    if (sys) w[0] = "$SYS";
    if (kind == K_PLUS) {
        int np = 1 + (int)r.below(2);
        for (int k = 0; k < np; k++) w[r.below(L)] = "+";
        if (sys && w[0] == "+") w[0] = "$SYS";
    } else if (kind == K_HASH) {
        int lo = c.hash_min, hi = L - 1;
        int k = lo + (int)r.below(hi - lo + 1);
        w.resize(k);
        w.push_back("#");
    }
    if (kind_out) *kind_out = kind;
}

void join(const std::vector<std::string> &w, std::string &out) {
    out.clear();
    for (size_t k = 0; k < w.size(); k++) { if (k) out.push_back('/'); out += w[k]; }
}

// topic j: instantiate filter u (replace '+' by a word, extend '#') or random
void mixed_topic(const Cfg &c, uint64_t seed, uint64_t nf, uint64_t j, std::string &out, std::vector<std::string> &w) {
    Rng r(mix64(seed ^ 0x544f504943ull ^ (j * 0x9e3779b97f4a7c15ull)));
    uint64_t pick = r.below(100);
    bool want_sys = c.pct_sys > 0 && pick < 2;
    if (want_sys || pick < 51) {
        uint64_t u = r.below(nf);
        if (want_sys) {   // find a '$SYS' filter near u (bounded search)
            for (int tries = 0; tries < 4096; tries++) {
                mixed_filter(c, seed, (u + tries) % nf, w, nullptr);
                if (w[0] == "$SYS") break;
            }
        } else {
            mixed_filter(c, seed, u, w, nullptr);
        }
        if (!w.empty() && w.back() == "#") {
            w.pop_back();
            int L = (int)w.size() + (int)r.below(7 - w.size());
            for (int l = (int)w.size(); l < L; l++) w.push_back(level_word(seed, l, r.below(c.cards[l < 6 ? l : 5])));
        }
        for (size_t l = 0; l < w.size(); l++)
            if (w[l] == "+") w[l] = level_word(seed, (int)l, r.below(c.cards[l < 6 ? l : 5]));
    } else {
        int L = 4 + (int)r.below(3);
        w.clear();
        for (int l = 0; l < L; l++) w.push_back(level_word(seed, l, r.below(c.cards[l])));
    }
    join(w, out);
}

void c2_filter(uint64_t i, uint64_t ndev, bool nonmatch, std::string &out) {
    if (i < ndev) { out = "fleet/" + std::to_string(i) + "/sensor/+"; return; }
    uint64_t g = i - ndev;
    if (nonmatch) { out = "rules/" + std::to_string(g) + "/#"; return; }
    static const char *glob[4] = {"#", "fleet/#", "+/+/sensor/#", "fleet/+/sensor/#"};
    out = glob[(g / 250) % 4];
}

void c2_topic(uint64_t seed, uint64_t ndev, uint64_t j, std::string &out) {
    static const char *m[16] = {"temp", "hum", "pres", "co2", "volt", "amp", "rpm", "lux",
                                "pm25", "pm10", "noise", "gps", "batt", "rssi", "door", "flow"};
    Rng r(mix64(seed ^ 0x4332ull ^ (j * 0x9e3779b97f4a7c15ull)));
    uint64_t id = r.below(ndev + ndev / 5);
    out = "fleet/" + std::to_string(id) + "/sensor/" + m[r.below(16)];
}

struct Out {
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offs;
    std::vector<uint32_t> vals;
    std::vector<uint8_t> flags;
};

template <class F>
void parallel_gen(uint64_t n, F &&gen_range, std::vector<Out> &parts) {
    unsigned T = std::thread::hardware_concurrency();
    if (T > 16) T = 16;
    if (T < 1) T = 1;
    if (n < 100000) T = 1;
    parts.assign(T, Out());
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; t++)
        th.emplace_back([&, t] { gen_range(n * t / T, n * (t + 1) / T, parts[t]); });
    for (auto &x : th) x.join();
}

}  // namespace

extern "C" {

typedef struct {
    uint8_t *bytes;     // concatenated items
    uint64_t *offs;     // n + 1
    uint32_t *vals;     // n (filters: key value; deltas: value)
    uint8_t *flags;     // n (deltas: 1 = subscribe, 0 = unsubscribe)
    uint64_t n, nbytes;
} tmw_set;

static void pack(std::vector<Out> &parts, tmw_set *o) {
    uint64_t n = 0, nb = 0;
    for (auto &p : parts) { n += p.vals.size(); nb += p.bytes.size(); }
    o->n = n; o->nbytes = nb;
    o->bytes = (uint8_t *)malloc(nb + 16);
    o->offs = (uint64_t *)malloc((n + 1) * 8);
    o->vals = (uint32_t *)malloc(n * 4 + 4);
    o->flags = (uint8_t *)malloc(n + 1);
    uint64_t i = 0, b = 0;
    for (auto &p : parts) {
        memcpy(o->bytes + b, p.bytes.data(), p.bytes.size());
        for (size_t k = 0; k < p.vals.size(); k++) {
            o->offs[i] = b + p.offs[k];
            o->vals[i] = p.vals[k];
            o->flags[i] = p.flags[k];
            i++;
        }
        b += p.bytes.size();
        std::vector<uint8_t>().swap(p.bytes);
    }
    o->offs[n] = b;
    memset(o->bytes + nb, 0, 16);
}

static void put(Out &o, const std::string &s, uint32_t v, uint8_t f) {
    o.offs.push_back(o.bytes.size());
    o.bytes.insert(o.bytes.end(), s.begin(), s.end());
    o.vals.push_back(v);
    o.flags.push_back(f);
}

// cfg: 1, 2 (C2), 20 (C2 non-matching globals), 3 (C3/C4/C5 base; topics: 30 = C3deep).
// Filters [lo, hi) of the config's full filter list, keeping index % nshards == shard.
int tmw_filters(int cfg, uint64_t seed, uint64_t nf, uint64_t shard, uint64_t nshards, tmw_set *out) {
    if (!out || nshards == 0) return -1;
    std::vector<Out> parts;
    const uint64_t total = cfg == 3 ? nf + 2 : (cfg == 2 || cfg == 20) ? nf + 1000 : nf;
    parallel_gen(total, [&](uint64_t lo, uint64_t hi, Out &o) {
        std::vector<std::string> w;
        std::string s;
        for (uint64_t i = lo; i < hi; i++) {
            if (i % nshards != shard) continue;
            if (cfg == 1 || cfg == 3) {
                const Cfg &c = cfg == 1 ? C1 : C3;
                if (i >= nf) s = (i == nf) ? "#" : "+/#";
                else { mixed_filter(c, seed, i, w, nullptr); join(w, s); }
            } else {
                c2_filter(i, nf, cfg == 20, s);
            }
            put(o, s, (uint32_t)i, 1);
        }
    }, parts);
    pack(parts, out);
    return 0;
}

// topics [first, first + n) of the config's topic stream
int tmw_topics(int cfg, uint64_t seed, uint64_t nf, uint64_t first, uint64_t n, tmw_set *out) {
    if (!out) return -1;
    std::vector<Out> parts;
    parallel_gen(n, [&](uint64_t lo, uint64_t hi, Out &o) {
        std::vector<std::string> w;
        std::string s;
        for (uint64_t j = first + lo; j < first + hi; j++) {
            if (cfg == 1 || cfg == 3 || cfg == 30) mixed_topic(cfg == 1 ? C1 : C3, seed, nf, j, s, w);
            else c2_topic(seed, nf, j, s);
            if (cfg == 30) {   // C3 topics, 10% of them extended to 33-64 levels
                Rng r(mix64(seed ^ 0x44454550ull ^ (j * 0x9e3779b97f4a7c15ull)));
                if (r.below(10) == 0) {
                    const size_t L = 33 + (size_t)r.below(32);
                    while (w.size() < L) w.push_back(level_word(seed, (int)(w.size() % 6), r.below(256)));
                    join(w, s);
                }
            }
            put(o, s, 0, 0);
        }
    }, parts);
    pack(parts, out);
    return 0;
}

// C5 churn deltas [first, first + n) against a C3 base of nf filters
int tmw_deltas(uint64_t seed, uint64_t nf, uint64_t first, uint64_t n, tmw_set *out) {
    if (!out || !nf) return -1;
    uint64_t P = 2654435761ull % nf;
    auto gcd = [](uint64_t a, uint64_t b) { while (b) { uint64_t t = a % b; a = b; b = t; } return a; };
    while (P == 0 || gcd(P, nf) != 1) P++;
    std::vector<Out> parts;
    parallel_gen(n, [&](uint64_t lo, uint64_t hi, Out &o) {
        std::vector<std::string> w;
        std::string s;
        for (uint64_t k = first + lo; k < first + hi; k++) {
            uint64_t i;
            uint8_t sub = (k & 1) == 0;
            if (sub) i = nf + 2 + k / 2;                       // brand-new key
            else i = (unsigned __int128)(k / 2) * P % nf;      // live base key
            mixed_filter(C3, seed, sub ? nf + k / 2 : i, w, nullptr);
            join(w, s);
            put(o, s, (uint32_t)i, sub);
        }
    }, parts);
    pack(parts, out);
    return 0;
}

void tmw_free(tmw_set *s) {
    if (!s) return;
    free(s->bytes); free(s->offs); free(s->vals); free(s->flags);
    memset(s, 0, sizeof *s);
}

}  // extern "C"

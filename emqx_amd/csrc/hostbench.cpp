// hostbench.cpp -- bench infrastructure (libtmbench.so), not part of the match
// path: the host-side measurements of bench.py done by native threads, as the
// NIF's dirty schedulers would drive libtmatch (c_src/emqx_tmatch_nif.c), so
// Python's GIL is not what is measured.
//
//   tmb_single     one caller: p50 / p99 of host-to-host batches of n topics
//                  (tm_host_alloc buffers: the batch runs in place)
//   tmb_callers    N caller threads (their own tm_host_alloc buffers) plus one
//                  thread applying subscribe/unsubscribe deltas, for a while:
//                  aggregate topics/s and per-batch p50 / p99 -- the reference's
//                  concurrent publishers (emqx_broker.erl:293-298)
//   tmb_writers    route writes one key at a time from many writer threads,
//                  group-committed by one mirror thread (emqx_router_gpu's
//                  process: every queued sync request in ONE tm_apply_deltas),
//                  while matcher threads run NIF-shaped batches: writes/s,
//                  write latency, the matchers' rate and p99, and each
//                  writer's read of its own write
//   tmb_pipeline   host-fed throughput: batches of topics in pinned host memory,
//                  H2D copy, match, D2H of offsets and values, overlapped on
//                  several streams -- the rate a caller that hands over host
//                  buffers sees, next to the PCIe bytes it moves
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tmatch.h"

// The C ABI of the libtmatch instance the caller loaded (tmb_bind: a bench or
// study may load an experimental build under another name; every tm_index*
// must go back to the library that made it).
namespace api {
int (*host_alloc)(tm_index *, uint64_t, void **);
int (*host_free)(tm_index *, void *);
int (*host_alloc_ex)(tm_index *, uint64_t, uint32_t, void **);   // optional (ABI 1.9)
int (*match_batch)(tm_index *, uint64_t, const uint8_t *, const uint64_t *, uint64_t *, uint32_t *, uint64_t, uint8_t *);
int (*match_batch_dev)(tm_index *, uint64_t, const uint8_t *, const uint64_t *, uint64_t *, uint32_t *, uint64_t,
                       uint8_t *, void *);
int (*apply_deltas)(tm_index *, uint64_t, const uint8_t *, const uint8_t *, const uint64_t *, const uint32_t *,
                    const uint8_t *);
int (*commit)(tm_index *, uint64_t, const uint8_t *, const uint8_t *, const uint64_t *, const uint32_t *,
              const uint8_t *, uint64_t *);   // optional (ABI 1.10)
int (*match_pairs)(tm_index *, uint64_t, const uint8_t *, const uint32_t *, uint32_t *, uint32_t *, uint64_t,
                   uint8_t *);                 // optional (ABI 1.10)
int (*stream_release)(tm_index *, void *);
int (*match_batch32)(tm_index *, uint64_t, const uint8_t *, const uint32_t *, uint32_t *, uint32_t *, uint64_t,
                     uint8_t *, uint32_t, uint32_t *);
int (*match_batch32_dev)(tm_index *, uint64_t, const uint8_t *, const uint32_t *, uint32_t *, uint32_t *, uint64_t,
                         uint8_t *, void *);
}  // namespace api

namespace {

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

double pct(std::vector<double> &v, double q) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q / 100.0 * (v.size() - 1) + 0.5))];
}

// one caller's pinned buffers for batches of `n` topics taken from a topic set
struct Caller {
    tm_index *h;
    uint64_t n, cap;
    uint8_t *blob = nullptr; uint64_t *offs = nullptr, *hit = nullptr; uint32_t *vals = nullptr; uint8_t *err = nullptr;
    uint32_t *offs32 = nullptr, *hit32 = nullptr;   // mode 4: tm_match_batch32_ex (u32 offsets)
    uint32_t *pairs32 = nullptr;                     // modes 6, 7: tm_match_batch32_pairs
    // mode 5: mode 4 with the inputs in TM_ALLOC_VRAM memory, written by the
    // caller before every batch (as a NIF packs each micro-batch)
    uint8_t *vblob = nullptr; uint32_t *voffs32 = nullptr; uint64_t nbytes = 0;
    int to_vram() {
        nbytes = offs[n];
        int rc;
        if (!api::host_alloc_ex) return TM_EINVAL;
        if ((rc = api::host_alloc_ex(h, nbytes + 16, TM_ALLOC_VRAM, (void **)&vblob)) ||
            (rc = api::host_alloc_ex(h, 4 * (n + 1), TM_ALLOC_VRAM, (void **)&voffs32)))
            return rc;
        return TM_OK;
    }
    int init(tm_index *ix, uint64_t nt, const uint8_t *tb, const uint64_t *to, uint64_t first, uint64_t cap_) {
        h = ix; n = nt; cap = cap_;
        const uint64_t b0 = to[first], nb = to[first + nt] - b0;
        int rc;
        if ((rc = api::host_alloc(h, nb + 16, (void **)&blob)) || (rc = api::host_alloc(h, 8 * (nt + 1), (void **)&offs)) ||
            (rc = api::host_alloc(h, 8 * (nt + 1), (void **)&hit)) || (rc = api::host_alloc(h, 4 * cap, (void **)&vals)) ||
            (rc = api::host_alloc(h, nt + 1, (void **)&err)) || (rc = api::host_alloc(h, 4 * (nt + 1), (void **)&offs32)) ||
            (rc = api::host_alloc(h, 4 * (nt + 1), (void **)&hit32)) ||
            (rc = api::host_alloc(h, 4 * (2 * nt + 1), (void **)&pairs32)))
            return rc;
        memcpy(blob, tb + b0, nb);
        for (uint64_t i = 0; i <= nt; i++) offs[i] = to[first + i] - b0;
        for (uint64_t i = 0; i <= nt; i++) offs32[i] = (uint32_t)offs[i];
        return TM_OK;
    }
    // device mode: the same batch copied into HBM once, run through the device
    // API on the caller's own stream (no PCIe traffic inside the batch)
    hipStream_t s = nullptr;
    uint8_t *dblob = nullptr, *derr = nullptr; uint64_t *doffs = nullptr, *dhit = nullptr; uint32_t *dvals = nullptr;
    int to_device() {
        const uint64_t nb = offs[n];
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&dblob, nb + 16) != hipSuccess || hipMalloc(&doffs, 8 * (n + 1)) != hipSuccess ||
            hipMalloc(&dhit, 8 * (n + 1)) != hipSuccess || hipMalloc(&dvals, 4 * cap) != hipSuccess ||
            hipMalloc(&derr, n + 1) != hipSuccess || hipMemcpy(dblob, blob, nb, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(doffs, offs, 8 * (n + 1), hipMemcpyHostToDevice) != hipSuccess)
            return TM_EDEVICE;
        return TM_OK;
    }
    // mode 2: inputs in HBM, outputs in the mapped host buffers; mode 3: the
    // reverse (which PCIe leg of an in-place batch costs what)
    int mode = 1;
    template <class T> static T *mapped(T *hp) {
        void *d = nullptr;
        return hipHostGetDevicePointer(&d, hp, 0) == hipSuccess ? static_cast<T *>(d) : nullptr;
    }
    int run() {
        if (mode == 4) return api::match_batch32(h, n, blob, offs32, hit32, vals, cap, err, TM_ORDER_TRAVERSAL, nullptr);
        if (mode == 5) {
            memcpy(vblob, blob, nbytes);
            memcpy(voffs32, offs32, 4 * (n + 1));
            return api::match_batch32(h, n, vblob, voffs32, hit32, vals, cap, err, TM_ORDER_TRAVERSAL, nullptr);
        }
        if (mode == 6 || mode == 7) {   // the NIF's pairs call; 6: inputs in TM_ALLOC_VRAM memory, 7: pinned
            if (!api::match_pairs) return TM_EINVAL;
            if (mode == 6) {
                memcpy(vblob, blob, nbytes);
                memcpy(voffs32, offs32, 4 * (n + 1));
                return api::match_pairs(h, n, vblob, voffs32, pairs32, vals, cap, err);
            }
            return api::match_pairs(h, n, blob, offs32, pairs32, vals, cap, err);
        }
        if (!s) return api::match_batch(h, n, blob, offs, hit, vals, cap, err);
        const bool hin = mode == 3, hout = mode == 2;
        int rc = api::match_batch_dev(h, n, hin ? mapped(blob) : dblob, hin ? mapped(offs) : doffs,
                                      hout ? mapped(hit) : dhit, hout ? mapped(vals) : dvals, cap,
                                      hout ? mapped(err) : derr, s);
        if (rc) return rc;
        return hipStreamSynchronize(s) == hipSuccess ? TM_OK : TM_EDEVICE;
    }
    void fini() {
        for (void *p : {(void *)blob, (void *)offs, (void *)hit, (void *)vals, (void *)err, (void *)offs32, (void *)hit32,
                        (void *)vblob, (void *)voffs32, (void *)pairs32})
            if (p) api::host_free(h, p);
        if (s) {
            for (void *p : {(void *)dblob, (void *)doffs, (void *)dhit, (void *)dvals, (void *)derr}) if (p) (void)hipFree(p);
            api::stream_release(h, s);
            (void)hipStreamDestroy(s);
        }
    }
};

}  // namespace

extern "C" {

// bind to the libtmatch the caller loaded (dlopen handle, e.g. ctypes' _handle)
int tmb_bind(void *lib) {
    api::host_alloc = reinterpret_cast<decltype(api::host_alloc)>(dlsym(lib, "tm_host_alloc"));
    api::host_free = reinterpret_cast<decltype(api::host_free)>(dlsym(lib, "tm_host_free"));
    api::host_alloc_ex = reinterpret_cast<decltype(api::host_alloc_ex)>(dlsym(lib, "tm_host_alloc_ex"));
    api::match_batch = reinterpret_cast<decltype(api::match_batch)>(dlsym(lib, "tm_match_batch"));
    api::match_batch_dev = reinterpret_cast<decltype(api::match_batch_dev)>(dlsym(lib, "tm_match_batch_dev"));
    api::apply_deltas = reinterpret_cast<decltype(api::apply_deltas)>(dlsym(lib, "tm_apply_deltas"));
    api::commit = reinterpret_cast<decltype(api::commit)>(dlsym(lib, "tm_commit"));
    api::match_pairs = reinterpret_cast<decltype(api::match_pairs)>(dlsym(lib, "tm_match_batch32_pairs"));
    api::stream_release = reinterpret_cast<decltype(api::stream_release)>(dlsym(lib, "tm_stream_release"));
    api::match_batch32 = reinterpret_cast<decltype(api::match_batch32)>(dlsym(lib, "tm_match_batch32_ex"));
    api::match_batch32_dev = reinterpret_cast<decltype(api::match_batch32_dev)>(dlsym(lib, "tm_match_batch32_dev"));
    return api::host_alloc && api::host_free && api::match_batch && api::match_batch_dev && api::apply_deltas &&
                   api::stream_release && api::match_batch32 && api::match_batch32_dev ? 0 : -1;
}

// out: [p50_ms, p99_ms, mean_ms]
// mode: as tmb_callers_ex (0: in place, u64 offsets; 4: u32; 5: u32 with the
// inputs in TM_ALLOC_VRAM memory written before every batch)
int tmb_single_ex(tm_index *h, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t cap, int iters, int mode,
                  double *out) {
    Caller c;
    int rc = c.init(h, n, tb, to, 0, cap);
    if (rc) return rc;
    if ((mode == 5 || mode == 6) && (rc = c.to_vram())) return rc;
    c.mode = mode ? mode : 1;
    std::vector<double> lat;
    for (int k = 0; k < iters + 3 && !rc; k++) {
        const double t0 = now_s();
        rc = c.run();
        if (k >= 3) lat.push_back((now_s() - t0) * 1e3);
    }
    double sum = 0;
    for (double x : lat) sum += x;
    c.fini();
    if (rc) return rc;
    out[2] = sum / std::max<size_t>(lat.size(), 1);
    out[0] = pct(lat, 50);
    out[1] = pct(lat, 99);
    return TM_OK;
}

int tmb_single(tm_index *h, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t cap, int iters, double *out) {
    return tmb_single_ex(h, n, tb, to, cap, iters, 0, out);
}

// nthreads callers, each with batches of n topics (caller k takes topics
// [k n, (k + 1) n) of the set, which must hold nthreads * n); one churn thread
// applies `churn_ops` deltas per millisecond (0: none).  device_buffers: each
// caller's batch lives in HBM and goes through tm_match_batch_dev on its own
// stream (what the device can take without the PCIe leg of in-place batches);
// 2: inputs in HBM, outputs written into the mapped host buffers; 3: inputs
// read from the mapped host buffers, outputs in HBM; 4: in place with u32
// offsets (tm_match_batch32_ex, what the NIF calls); 5: mode 4 with the inputs
// in TM_ALLOC_VRAM memory the caller writes before every batch; 6: mode 5
// through tm_match_batch32_pairs ((offset, count) pairs: what the NIF binds);
// 7: pairs with the inputs in pinned host memory.
// out: [batches, topics_per_s, p50_ms, p99_ms, deltas_per_s, seconds]
int tmb_callers_ex(tm_index *h, int nthreads, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t cap,
                   double seconds, int churn_ops, int device_buffers, double *out) {
    std::vector<Caller> cs(nthreads);
    for (int k = 0; k < nthreads; k++) {
        int rc = cs[k].init(h, n, tb, to, (uint64_t)k * n, cap);
        if (rc) return rc;
        if ((device_buffers == 5 || device_buffers == 6) && (rc = cs[k].to_vram())) return rc;
        if (device_buffers && device_buffers < 4 && (rc = cs[k].to_device())) return rc;
        cs[k].mode = device_buffers;
        if ((rc = cs[k].run())) return rc;   // warm: lane, workspace
    }
    std::atomic<bool> stop{false};
    std::atomic<int> err{0};
    std::vector<std::vector<double>> lat(nthreads);
    std::atomic<uint64_t> deltas{0};
    std::vector<std::thread> th;
    const double t0 = now_s();
    for (int k = 0; k < nthreads; k++)
        th.emplace_back([&, k] {
            while (!stop.load(std::memory_order_relaxed)) {
                const double a = now_s();
                const int rc = cs[k].run();
                if (rc) { err = rc; break; }
                lat[k].push_back((now_s() - a) * 1e3);
            }
        });
    if (churn_ops > 0)
        th.emplace_back([&] {
            std::vector<std::string> fs;
            std::vector<uint8_t> blob;
            std::vector<uint64_t> offs{0};
            std::vector<uint32_t> vals;
            for (int i = 0; i < churn_ops; i++) {
                std::string f = "bench/concurrent/" + std::to_string(i) + "/+";
                blob.insert(blob.end(), f.begin(), f.end());
                offs.push_back(blob.size());
                vals.push_back(0xF0000000u + i);
            }
            std::vector<uint8_t> ops(churn_ops, 1);
            while (!stop.load(std::memory_order_relaxed)) {
                if (api::apply_deltas(h, churn_ops, ops.data(), blob.data(), offs.data(), vals.data(), nullptr)) {
                    err = -1;
                    break;
                }
                deltas += churn_ops;
                for (auto &o : ops) o ^= 1;
                std::this_thread::sleep_for(std::chrono::milliseconds(1));
            }
        });
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (auto &t : th) t.join();
    const double el = now_s() - t0;
    for (auto &c : cs) c.fini();
    if (err) return err;
    std::vector<double> all;
    uint64_t nb = 0;
    for (auto &v : lat) { nb += v.size(); all.insert(all.end(), v.begin() + std::min<size_t>(2, v.size()), v.end()); }
    out[0] = (double)nb;
    out[1] = nb * (double)n / el;
    out[2] = pct(all, 50);
    out[3] = pct(all, 99);
    out[4] = deltas / el;
    out[5] = el;
    return TM_OK;
}

int tmb_callers(tm_index *h, int nthreads, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t cap,
                double seconds, int churn_ops, double *out) {
    return tmb_callers_ex(h, nthreads, n, tb, to, cap, seconds, churn_ops, 0, out);
}

// Route writes through a group-committing mirror.  The
// reference runs route writes in parallel in up to schedulers x 2 broker-pool
// workers (emqx_broker_sup.erl:36; emqx_broker.erl:778-808 -> emqx_router.erl
// :193-196, 492-493); with the device mirror each write also waits until the
// mirror has it (the read-your-writes hook, src/emqx_router_gpu.erl
// filters_written/1), and the mirror is ONE process: it takes every sync
// request queued when it wakes and ships them as ONE delta batch
// (mirror_batch/2), then replies to each.  Here: `nwriters` writer threads, each
// subscribing and unsubscribing its own keys one at a time (a binary key
// "bench/writer/<w>/<k>" -- the exact-topic path -- alternating with the word
// list "bench/writer/<w>/<k>/+"), one mirror thread committing the queue, and
// `nmatch` matcher threads running 4k-topic batches as the NIF does (u32
// offsets, inputs in TM_ALLOC_VRAM memory, through the combiner).  check:
// after each insert commit the writer matches its own topic (a one-topic
// batch) and counts a miss if its value is absent -- a publish right after the
// SUBACK must reach the subscriber.  commit: the mirror ships each group with
// tm_commit (published on a table copy no batch is reading), else with
// tm_apply_deltas.
// out: [writes_per_s, write_p50_ms, write_p99_ms, commits_per_s, topics_per_s, match_p50_ms, match_p99_ms,
//       ryw_checks, ryw_misses, seconds]
int tmb_writers(tm_index *h, int nwriters, int nmatch, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t cap,
                double seconds, int check, int commit, double *out) {
    if (commit && !api::commit) return TM_EINVAL;
    struct Req { uint8_t op; std::string key; uint32_t val; bool done = false; };
    std::mutex mu;
    std::condition_variable cv_mirror, cv_done;
    std::deque<Req *> q;
    std::atomic<bool> stop{false};
    bool mstop = false;   // (under mu) the mirror ends once every writer has
    std::atomic<int> err{0};
    std::atomic<uint64_t> commits{0}, ryw_checks{0}, ryw_miss{0};
    std::vector<Caller> cs(nmatch);
    for (int k = 0; k < nmatch; k++) {
        int rc = cs[k].init(h, n, tb, to, (uint64_t)k * n, cap);
        if (rc) return rc;
        cs[k].mode = api::match_pairs ? 7 : 4;   // the NIF's call: pairs, inputs in VRAM where it can
        if (cs[k].to_vram() == TM_OK) cs[k].mode = api::match_pairs ? 6 : 5;
        if ((rc = cs[k].run())) return rc;
    }
    std::vector<std::vector<double>> mlat(nmatch), wlat(nwriters);
    std::vector<std::thread> th;
    // the mirror process
    th.emplace_back([&] {
        std::vector<uint8_t> ops, blob, kinds;
        std::vector<uint64_t> offs;
        std::vector<uint32_t> vals;
        std::vector<Req *> batch;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv_mirror.wait(lk, [&] { return !q.empty() || mstop; });
            if (q.empty()) break;
            batch.assign(q.begin(), q.end());
            q.clear();
            lk.unlock();
            ops.clear(); blob.clear(); vals.clear(); kinds.clear(); offs.assign(1, 0);
            for (Req *r : batch) {
                ops.push_back(r->op);
                blob.insert(blob.end(), r->key.begin(), r->key.end());
                offs.push_back(blob.size());
                vals.push_back(r->val);
            }
            const int rc = commit ? api::commit(h, batch.size(), ops.data(), blob.data(), offs.data(), vals.data(), nullptr,
                                                nullptr)
                                  : api::apply_deltas(h, batch.size(), ops.data(), blob.data(), offs.data(), vals.data(),
                                                      nullptr);
            if (rc) err = -1;
            commits++;
            lk.lock();
            for (Req *r : batch) r->done = true;
            cv_done.notify_all();
        }
    });
    for (int k = 0; k < nmatch; k++)
        th.emplace_back([&, k] {
            while (!stop.load(std::memory_order_relaxed)) {
                const double a = now_s();
                const int rc = cs[k].run();
                if (rc) { err = rc; break; }
                mlat[k].push_back((now_s() - a) * 1e3);
            }
        });
    for (int w = 0; w < nwriters; w++)
        th.emplace_back([&, w] {
            // the one-topic batch a writer publishes after its subscribe: the
            // NIF's call (u32 offsets, pinned buffers: in place, through the
            // combiner -- it shares launches with the matchers' batches, as a
            // publish goes through the broker's micro-batcher)
            uint8_t *pb = nullptr; uint32_t *po = nullptr, *ph = nullptr; uint32_t *pv = nullptr; uint8_t *pe = nullptr;
            if (check && (api::host_alloc(h, 256, (void **)&pb) || api::host_alloc(h, 16, (void **)&po) ||
                          api::host_alloc(h, 16, (void **)&ph) || api::host_alloc(h, 4 * 4096, (void **)&pv) ||
                          api::host_alloc(h, 16, (void **)&pe))) { err = -2; return; }
            Req r;
            for (uint64_t k = 0; !stop.load(std::memory_order_relaxed); k++) {
                const std::string topic = "bench/writer/" + std::to_string(w) + "/" + std::to_string(k % 64);
                const bool words = (k / 64) & 1;   // the word-list key "<topic>/+" every other sweep
                r.key = words ? topic + "/+" : topic;
                r.val = 0xE0000000u + (uint32_t)w * 64 + (uint32_t)(k % 64);
                for (int op = 1; op >= 0; op--) {   // subscribe, (publish,) unsubscribe
                    r.op = (uint8_t)op;
                    r.done = false;
                    const double a = now_s();
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        q.push_back(&r);
                        cv_mirror.notify_one();
                        cv_done.wait(lk, [&] { return r.done; });
                    }
                    wlat[w].push_back((now_s() - a) * 1e3);
                    if (op == 1 && check) {
                        const std::string t = words ? topic + "/x" : topic;
                        memcpy(pb, t.data(), t.size());
                        po[0] = 0; po[1] = (uint32_t)t.size();
                        if (api::match_batch32(h, 1, pb, po, ph, pv, 4096, pe, TM_ORDER_TRAVERSAL, nullptr)) {
                            err = -3;
                            break;
                        }
                        bool seen = false;
                        for (uint64_t i = ph[0]; i < ph[1] && i < 4096; i++) seen |= pv[i] == r.val;
                        ryw_checks++;
                        if (!seen) ryw_miss++;
                    }
                }
            }
            for (void *p : {(void *)pb, (void *)po, (void *)ph, (void *)pv, (void *)pe}) if (p) api::host_free(h, p);
        });
    const double t0 = now_s();
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (size_t i = 1; i < th.size(); i++) th[i].join();
    {
        std::lock_guard<std::mutex> lk(mu);
        mstop = true;
        cv_mirror.notify_all();
    }
    th[0].join();
    const double el = now_s() - t0;
    for (auto &c : cs) c.fini();
    if (err) return err;
    std::vector<double> wa, ma;
    for (auto &v : wlat) wa.insert(wa.end(), v.begin(), v.end());
    uint64_t nb = 0;
    for (auto &v : mlat) { nb += v.size(); ma.insert(ma.end(), v.begin() + std::min<size_t>(2, v.size()), v.end()); }
    out[0] = wa.size() / el;
    out[1] = pct(wa, 50);
    out[2] = pct(wa, 99);
    out[3] = commits / el;
    out[4] = nb * (double)n / el;
    out[5] = pct(ma, 50);
    out[6] = pct(ma, 99);
    out[7] = (double)ryw_checks;
    out[8] = (double)ryw_miss;
    out[9] = el;
    return TM_OK;
}

// Host-fed pipeline.  R batches of n topics (batch k = topics [k n, (k + 1) n)
// of the set) are copied into pinned host memory (setup); a sizing pass
// records each batch's hit total.  Timed: `iters` batches rotate over the R
// host batches and over `nstreams` streams; per batch, on its stream: H2D of
// offsets + bytes, tm_match_batch_dev, D2H of the n + 1 offsets and of the
// values into pinned host buffers of that stream; before a stream's buffers
// are reused the host waits for its previous batch.
// out: [topics_per_s, ms_per_batch, h2d_bytes_per_batch, d2h_bytes_per_batch, seconds]
// u32 bit 0: the same with 32-bit offsets both ways (tm_match_batch32_dev):
// 4 B per topic less over PCIe in each direction.  Bit 1: every H2D on one
// upload stream and every D2H on one download stream, joined to the batches'
// compute streams by events (the arrangement tmb_pcie measures both directions
// at once with), instead of each batch's copies on its own stream.
int tmb_pipeline_ex(tm_index *h, int device, const uint8_t *tb, const uint64_t *to, uint64_t n, int R, int nstreams,
                    int iters, int u32, double *out) {
    if (hipSetDevice(device) != hipSuccess) return TM_EDEVICE;
    const bool sep = (u32 & 2) != 0;
    u32 &= 1;
    hipStream_t up = nullptr, down = nullptr;
    if (sep && (hipStreamCreateWithFlags(&up, hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&down, hipStreamNonBlocking) != hipSuccess))
        return TM_EDEVICE;
    struct HostBatch { uint8_t *p; uint64_t bytes, total; };
    std::vector<HostBatch> hb(R);
    uint64_t maxb = 0;
    const uint64_t ow = u32 ? 4 : 8;   // offset width
    const uint64_t boff = ((n + 1) * ow + 15) & ~15ull;
    for (int k = 0; k < R; k++) {
        const uint64_t b0 = to[(uint64_t)k * n], nb = to[(uint64_t)(k + 1) * n] - b0;
        hb[k].bytes = boff + nb;
        if (hipHostMalloc(&hb[k].p, hb[k].bytes + 16, hipHostMallocDefault) != hipSuccess) return TM_ENOMEM;
        for (uint64_t i = 0; i <= n; i++) {
            const uint64_t v = to[(uint64_t)k * n + i] - b0;
            if (u32) reinterpret_cast<uint32_t *>(hb[k].p)[i] = (uint32_t)v;
            else reinterpret_cast<uint64_t *>(hb[k].p)[i] = v;
        }
        memcpy(hb[k].p + boff, tb + b0, nb);
        maxb = std::max(maxb, hb[k].bytes);
    }
    auto match = [&](uint8_t *d_in, void *d_hit, uint32_t *d_vals, uint64_t cap, uint8_t *d_err, hipStream_t s) {
        return u32 ? api::match_batch32_dev(h, n, d_in + boff, reinterpret_cast<uint32_t *>(d_in),
                                            static_cast<uint32_t *>(d_hit), d_vals, cap, d_err, s)
                   : api::match_batch_dev(h, n, d_in + boff, reinterpret_cast<uint64_t *>(d_in),
                                          static_cast<uint64_t *>(d_hit), d_vals, cap, d_err, s);
    };
    struct Lane { hipStream_t s; hipEvent_t done, e_in, e_out; uint8_t *d_in; uint64_t *d_hit; uint32_t *d_vals;
                  uint8_t *d_err; uint64_t *h_hit; uint32_t *h_vals; bool busy; };
    std::vector<Lane> ls(nstreams);
    uint64_t cap = 0;
    for (auto &l : ls) {
        if (hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&l.done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&l.e_in, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&l.e_out, hipEventDisableTiming) != hipSuccess ||
            hipMalloc(&l.d_in, maxb + 16) != hipSuccess || hipMalloc(&l.d_hit, 8 * (n + 1)) != hipSuccess ||
            hipMalloc(&l.d_err, n + 1) != hipSuccess || hipHostMalloc(&l.h_hit, 8 * (n + 1), hipHostMallocDefault) != hipSuccess)
            return TM_EDEVICE;
        l.d_vals = nullptr; l.h_vals = nullptr; l.busy = false;
    }
    // sizing pass: every batch's hit total
    {
        Lane &l = ls[0];
        for (int k = 0; k < R; k++) {
            hipMemcpyAsync(l.d_in, hb[k].p, hb[k].bytes, hipMemcpyHostToDevice, l.s);
            int rc = match(l.d_in, l.d_hit, nullptr, 0, l.d_err, l.s);
            if (rc) return rc;
            hipMemcpyAsync(l.h_hit, l.d_hit, ow * (n + 1), hipMemcpyDeviceToHost, l.s);
            hipStreamSynchronize(l.s);
            hb[k].total = u32 ? reinterpret_cast<uint32_t *>(l.h_hit)[n] : l.h_hit[n];
            cap = std::max(cap, hb[k].total);
        }
    }
    for (auto &l : ls)
        if (hipMalloc(&l.d_vals, 4 * (cap + 16)) != hipSuccess ||
            hipHostMalloc(&l.h_vals, 4 * (cap + 16), hipHostMallocDefault) != hipSuccess)
            return TM_ENOMEM;
    double h2d = 0, d2h = 0;
    auto issue = [&](int k, Lane &l) -> int {
        const HostBatch &b = hb[k % R];
        hipStream_t si = sep ? up : l.s, so = sep ? down : l.s;
        if (hipMemcpyAsync(l.d_in, b.p, b.bytes, hipMemcpyHostToDevice, si) != hipSuccess) return TM_EDEVICE;
        if (sep && (hipEventRecord(l.e_in, up) != hipSuccess || hipStreamWaitEvent(l.s, l.e_in, 0) != hipSuccess))
            return TM_EDEVICE;
        int rc = match(l.d_in, l.d_hit, l.d_vals, cap, l.d_err, l.s);
        if (rc) return rc;
        if (sep && (hipEventRecord(l.e_out, l.s) != hipSuccess || hipStreamWaitEvent(down, l.e_out, 0) != hipSuccess))
            return TM_EDEVICE;
        if (hipMemcpyAsync(l.h_hit, l.d_hit, ow * (n + 1), hipMemcpyDeviceToHost, so) != hipSuccess ||
            hipMemcpyAsync(l.h_vals, l.d_vals, 4 * b.total, hipMemcpyDeviceToHost, so) != hipSuccess ||
            hipEventRecord(l.done, so) != hipSuccess)
            return TM_EDEVICE;
        h2d += b.bytes;
        d2h += (double)ow * (n + 1) + 4.0 * b.total;
        l.busy = true;
        return TM_OK;
    };
    for (int k = 0; k < 4 * nstreams; k++) {   // warm (the first rounds run slower)
        Lane &l = ls[k % nstreams];
        if (l.busy && hipEventSynchronize(l.done) != hipSuccess) return TM_EDEVICE;
        if (int rc = issue(k, l)) return rc;
    }
    for (auto &l : ls) { hipEventSynchronize(l.done); l.busy = false; }
    h2d = d2h = 0;
    const double t0 = now_s();
    for (int k = 0; k < iters; k++) {
        Lane &l = ls[k % nstreams];
        if (l.busy && hipEventSynchronize(l.done) != hipSuccess) return TM_EDEVICE;   // its results consumed
        int rc = issue(k, l);
        if (rc) return rc;
    }
    for (auto &l : ls) if (l.busy) hipEventSynchronize(l.done);
    const double el = now_s() - t0;
    for (auto &l : ls) {
        hipStreamSynchronize(l.s);
        api::stream_release(h, l.s);
        hipFree(l.d_in); hipFree(l.d_hit); hipFree(l.d_vals); hipFree(l.d_err);
        hipHostFree(l.h_hit); hipHostFree(l.h_vals);
        hipEventDestroy(l.done); hipEventDestroy(l.e_in); hipEventDestroy(l.e_out); hipStreamDestroy(l.s);
    }
    if (up) hipStreamDestroy(up);
    if (down) hipStreamDestroy(down);
    for (auto &b : hb) hipHostFree(b.p);
    out[0] = iters * (double)n / el;
    out[1] = el / iters * 1e3;
    out[2] = h2d / iters;
    out[3] = d2h / iters;
    out[4] = el;
    return TM_OK;
}

int tmb_pipeline(tm_index *h, int device, const uint8_t *tb, const uint64_t *to, uint64_t n, int R, int nstreams,
                 int iters, double *out) {
    return tmb_pipeline_ex(h, device, tb, to, n, R, nstreams, iters, 0, out);
}

// Launch noise (a study, tools/profile_walk.py --noise native): a thread that
// enqueues 4-byte hipMemsetAsync fills (one small kernel dispatch each) on a
// stream of its own as fast as the queue takes them, until tmb_noise_stop.
// Does another stream's dispatch rate slow a running walk?
static std::atomic<bool> g_noise_run{false};
static std::thread g_noise_th;
static std::atomic<uint64_t> g_noise_n{0};
static double g_noise_t0 = 0;

int tmb_noise_start(int device, int mode) {   // mode 0: 4-byte fills; 1: event records (no kernel)
    if (g_noise_run.exchange(true)) return TM_EINVAL;
    g_noise_n = 0;
    g_noise_t0 = now_s();
    g_noise_th = std::thread([device, mode] {
        if (hipSetDevice(device) != hipSuccess) return;
        hipStream_t s = nullptr;
        uint32_t *d = nullptr;
        hipEvent_t ev = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipMalloc(&d, 64) != hipSuccess ||
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
            return;
        while (g_noise_run.load(std::memory_order_relaxed)) {
            for (int k = 0; k < 64; k++) {
                if (mode == 1) (void)hipEventRecord(ev, s);
                else (void)hipMemsetAsync(d, 0, 4, s);
            }
            (void)hipStreamSynchronize(s);
            g_noise_n += 64;
        }
        (void)hipEventDestroy(ev);
        (void)hipStreamDestroy(s);
        (void)hipFree(d);
    });
    return TM_OK;
}

int tmb_noise_stop(double *per_s) {
    if (!g_noise_run.exchange(false)) return TM_EINVAL;
    g_noise_th.join();
    *per_s = (double)g_noise_n.load() / (now_s() - g_noise_t0);
    return TM_OK;
}

// The PCIe ceiling the host-fed pipeline runs against: pinned-host <-> HBM
// copies of `bytes` in `chunks` pieces, H2D alone, D2H alone, and both
// directions at once on two streams.  out: [h2d_GBps, d2h_GBps, both_h2d_GBps, both_d2h_GBps]
int tmb_pcie(int device, uint64_t bytes, int chunks, int reps, double *out) {
    if (hipSetDevice(device) != hipSuccess) return TM_EDEVICE;
    uint8_t *hin = nullptr, *hout = nullptr, *din = nullptr, *dout = nullptr;
    hipStream_t a = nullptr, b = nullptr;
    if (hipHostMalloc(&hin, bytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&hout, bytes, hipHostMallocDefault) != hipSuccess || hipMalloc(&din, bytes) != hipSuccess ||
        hipMalloc(&dout, bytes) != hipSuccess || hipStreamCreateWithFlags(&a, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&b, hipStreamNonBlocking) != hipSuccess)
        return TM_EDEVICE;
    memset(hin, 1, bytes);
    const uint64_t c = bytes / chunks;
    auto run = [&](bool up, bool down) -> double {
        const double t0 = now_s();
        for (int r = 0; r < reps; r++)
            for (int k = 0; k < chunks; k++) {
                if (up) (void)hipMemcpyAsync(din + k * c, hin + k * c, c, hipMemcpyHostToDevice, a);
                if (down) (void)hipMemcpyAsync(hout + k * c, dout + k * c, c, hipMemcpyDeviceToHost, b);
            }
        (void)hipStreamSynchronize(a);
        (void)hipStreamSynchronize(b);
        return (double)c * chunks * reps / (now_s() - t0) / 1e9;
    };
    run(true, true);   // warm
    out[0] = out[1] = out[2] = 0;
    for (int k = 0; k < 3; k++) {   // best of three (the simultaneous rate varies between runs)
        out[0] = std::max(out[0], run(true, false));
        out[1] = std::max(out[1], run(false, true));
        out[2] = std::max(out[2], run(true, true));   // each direction moved the same bytes in that time
    }
    out[3] = out[2];
    (void)hipStreamDestroy(a); (void)hipStreamDestroy(b);
    (void)hipFree(din); (void)hipFree(dout); (void)hipHostFree(hin); (void)hipHostFree(hout);
    return TM_OK;
}

}  // extern "C"

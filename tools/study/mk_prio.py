"""Study build (not product): the two-phase batch's short kernels (tails, scan,
emit, re-walk) on a high-priority stream of their own, forked from and joined
back to the caller's stream with events, so that with several batches in
flight a finished walk's follow-up kernels get workgroup slots ahead of other
batches' walk blocks.  PRIO=0 builds the same fork/join on a
normal-priority stream (the events' own cost).
Build: python tools/study/mk_prio.py [prio|fork]  ->  emqx_amd/variants/libtmatch_<name>.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
ST.mkdir(exist_ok=True)
name = sys.argv[1] if len(sys.argv) > 1 else "prio"
k = (CS / "tm_kernels.hip").read_text()
k = k.replace('#include "tm_dev.h"', '#include "tm_dev.h"\n#include <mutex>\n#include <unordered_map>', 1)
aux = r'''
// ---- study: fork/join of the short kernels onto a stream of their own
struct StAux { hipStream_t hp; hipEvent_t e1, e2; };
static StAux *st_aux(hipStream_t s) {
    static std::mutex mu;
    static std::unordered_map<hipStream_t, StAux> m;
    std::lock_guard<std::mutex> g(mu);
    auto it = m.find(s);
    if (it != m.end()) return &it->second;
    StAux a;
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStreamCreateWithPriority(&a.hp, hipStreamNonBlocking, %s);
    hipEventCreateWithFlags(&a.e1, hipEventDisableTiming);
    hipEventCreateWithFlags(&a.e2, hipEventDisableTiming);
    return &(m[s] = a);
}
''' % ("hi" if name == "prio" else "lo")
anchor = "hipError_t launch_match_phase1("
k = k.replace(anchor, aux + anchor, 1)
old = '''    hipError_t e = launch_match_phase1(ix, ws, n, bytes, offs, hit_offs, err, s, ev_walk0, ev_walk1);
    if (e != hipSuccess) return e;
    return launch_match_phase2(ix, ws, n, bytes, offs, hit_offs, out, cap, s);'''
assert old in k
new = '''    StAux *x = st_aux(s);
    hipError_t e = launch_match_phase1(ix, ws, n, bytes, offs, hit_offs, err, s, ev_walk0, ev_walk1, x);
    if (e != hipSuccess) return e;
    e = launch_match_phase2(ix, ws, n, bytes, offs, hit_offs, out, cap, x->hp);
    if (e != hipSuccess) return e;
    if ((e = hipEventRecord(x->e2, x->hp)) != hipSuccess) return e;
    return hipStreamWaitEvent(s, x->e2, 0);'''
k = k.replace(old, new, 1)
# phase 1: the walk on s, then fork: tails + scan on hp
old1 = '''                               hipEvent_t ev_walk0, hipEvent_t ev_walk1) {
    hipError_t e;'''
assert old1 in k
k = k.replace(old1, '''                               hipEvent_t ev_walk0, hipEvent_t ev_walk1, StAux *x = nullptr) {
    hipError_t e;
    const hipStream_t s0 = s;''', 1)
old2 = '''        if (ev_walk1 && (e = hipEventRecord(ev_walk1, s)) != hipSuccess) return e;
        // small batches: the tail kernel's last block also scans the (few) tile totals'''
assert old2 in k
k = k.replace(old2, '''        if (ev_walk1 && (e = hipEventRecord(ev_walk1, s)) != hipSuccess) return e;
        if (x) {
            if ((e = hipEventRecord(x->e1, s0)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(x->hp, x->e1, 0)) != hipSuccess) return e;
            s = x->hp;
        }
        // small batches: the tail kernel's last block also scans the (few) tile totals''', 1)
# the declaration in tm_dev.h has no StAux param: phase1 is also called elsewhere? keep default arg
(ST / f"{name}.hip").write_text(k)
from emqx_amd import build
print(build.build_variant(name, str(ST / f"{name}.hip"), force=True))

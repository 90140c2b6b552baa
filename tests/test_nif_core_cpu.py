"""The NIF's ERTS-free logic (c_src/tmatch_nif_core.c): buffer pool reuse,
topic packing, the TM_ECAP retry and the result rows, compiled here against a
stand-in libtmatch (tests/native/fake_tmatch.c: no device) -- the part of
c_src/emqx_tmatch_nif.c that does not need erl_nif.h."""
import ctypes as C
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
TM_OK, TM_EDEVICE, TM_ECAP = 0, -3, -4
TRAVERSAL, SORTED, UNIQUE = 0, 1, 2


@pytest.fixture(scope="module")
def core(tmp_path_factory):
    out = tmp_path_factory.mktemp("nifcore") / "libnifcore.so"
    subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-fPIC", "-shared", "-pthread",
                    f"-I{ROOT / 'include'}", f"-I{ROOT / 'c_src'}", "-o", str(out),
                    str(ROOT / "c_src" / "tmatch_nif_core.c"), str(ROOT / "tests" / "native" / "fake_tmatch.c")],
                   check=True)
    lib = C.CDLL(str(out))
    vp = C.c_void_p
    lib.fake_pool_new.restype = vp
    lib.fake_pool_free.argtypes = [vp]
    lib.fake_pool_size.argtypes = [vp]
    lib.fake_count.restype = C.c_long
    lib.tmn_take.restype = vp
    lib.tmn_take.argtypes = [vp]
    lib.tmn_give.argtypes = [vp, vp]
    lib.tmn_pack.argtypes = [vp, vp, C.c_uint32, vp, vp]
    lib.tmn_match.argtypes = [vp, vp, C.c_uint32, C.c_uint32]
    lib.tmn_first.argtypes = [vp, vp, C.c_uint32]
    lib.tmn_row.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    lib.tmn_first_row.argtypes = [vp, C.c_uint32, C.POINTER(C.c_uint32)]
    lib.fake_set_vals_cap.argtypes = [vp]
    lib.fake_set_vals_cap.restype = C.c_uint64
    lib.fake_set_reruns.argtypes = [vp]
    lib.fake_set_reruns.restype = C.c_uint64
    lib.fake_set_vals.argtypes = [vp]
    lib.fake_set_vals.restype = C.POINTER(C.c_uint32)
    lib.fake_ticket_new.restype = vp
    lib.fake_ticket_free.argtypes = [vp]
    lib.tmn_ticket_end.argtypes = [vp]
    return lib


H = C.c_void_p(1)


def pack(lib, s, topics):
    arr = (C.c_char_p * len(topics))(*topics)
    lens = (C.c_uint64 * len(topics))(*[len(t) for t in topics])
    return lib.tmn_pack(s, H, len(topics), C.cast(arr, C.c_void_p), C.cast(lens, C.c_void_p))


def rows(lib, s, n, order):
    vals = lib.fake_set_vals(s)
    out = []
    for i in range(n):
        b, e = C.c_uint64(), C.c_uint64()
        err = lib.tmn_row(s, n, order, i, C.byref(b), C.byref(e))
        out.append(err if err else [vals[k] for k in range(b.value, e.value)])
    return out


def test_rows_and_badarg(core):
    pool = core.fake_pool_new()
    s = core.tmn_take(pool)
    topics = [b"ab", b"+x", b"", b"xyz"]
    assert pack(core, s, topics) == TM_OK
    assert core.tmn_match(s, H, len(topics), TRAVERSAL) == TM_OK
    assert rows(core, s, 4, TRAVERSAL) == [[0, 1], 1, [], [3000, 3001, 3002]]
    assert core.tmn_match(s, H, len(topics), UNIQUE) == TM_OK
    assert rows(core, s, 4, UNIQUE) == [[0], 1, [], [3000, 3001]]
    assert core.tmn_first(s, H, len(topics)) == TM_OK
    found = []
    for i in range(4):
        v = C.c_uint32()
        found.append((core.tmn_first_row(s, i, C.byref(v)), v.value))
    assert found == [(1, 0), (2, 0), (0, 0), (1, 3000)]
    core.tmn_give(pool, s)
    core.fake_pool_free(pool)


def test_vram_inputs_same_rows_and_host_fallback(core):
    """A one-device NIF packs its inputs into TM_ALLOC_VRAM memory
    (tmn_pool.in_flags): topics and u32 offsets written once, in order, the
    u64 offsets for tm_first_batch kept on the host (the core never reads
    device memory back).  Rows equal the host-buffer ones; when the device
    allocation fails the set falls back to pinned host memory."""
    core.fake_vram_count.restype = C.c_long
    core.fake_pool_set_inputs.argtypes = [C.c_void_p, C.c_uint32]
    core.fake_vram_fail.argtypes = [C.c_int]
    topics = [b"ab", b"+x", b"", b"xyz"]
    for fail in (0, 1):
        core.fake_vram_fail(fail)
        pool = core.fake_pool_new()
        core.fake_pool_set_inputs(pool, 1)   # TM_ALLOC_VRAM
        s = core.tmn_take(pool)
        v0 = core.fake_vram_count()
        assert pack(core, s, topics) == TM_OK
        assert core.fake_vram_count() - v0 == (0 if fail else 2)   # blob + offsets
        assert core.tmn_match(s, H, len(topics), TRAVERSAL) == TM_OK
        assert rows(core, s, 4, TRAVERSAL) == [[0, 1], 1, [], [3000, 3001, 3002]]
        assert core.tmn_first(s, H, len(topics)) == TM_OK
        found = []
        for i in range(4):
            v = C.c_uint32()
            found.append((core.tmn_first_row(s, i, C.byref(v)), v.value))
        assert found == [(1, 0), (2, 0), (0, 0), (1, 3000)]
        core.tmn_give(pool, s)
        core.fake_pool_free(pool)
    core.fake_vram_fail(0)


def test_ecap_grows_the_set_and_reruns_once(core):
    """More values than the first guess (TMN_IDS_PER_TOPIC per topic + 1024):
    the batch is rerun once with room for the exact total, and the grown
    buffer stays with the set for the next batch."""
    pool = core.fake_pool_new()
    s = core.tmn_take(pool)
    topics = [b"x" * 3000, b"y" * 200]
    assert pack(core, s, topics) == TM_OK
    m0 = core.fake_count(2)
    assert core.tmn_match(s, H, 2, TRAVERSAL) == TM_OK
    assert core.fake_count(2) - m0 == 2 and core.fake_set_reruns(s) == 1
    r = rows(core, s, 2, TRAVERSAL)
    assert r[0] == list(range(3000)) and r[1] == list(range(1000, 1200))
    assert core.fake_set_vals_cap(s) >= 4 * 3200
    m0 = core.fake_count(2)
    assert core.tmn_match(s, H, 2, TRAVERSAL) == TM_OK
    assert core.fake_count(2) - m0 == 1 and core.fake_set_reruns(s) == 1   # sticky size: no rerun
    core.tmn_give(pool, s)
    core.fake_pool_free(pool)


def test_pool_reuses_sets_and_bounds_itself(core):
    pool = core.fake_pool_new()
    s1 = core.tmn_take(pool)
    assert pack(core, s1, [b"abc"]) == TM_OK
    core.tmn_give(pool, s1)
    a0 = core.fake_count(0)
    s2 = core.tmn_take(pool)
    assert s2 == s1                          # the pooled set, buffers and all
    assert pack(core, s2, [b"abd"]) == TM_OK
    assert core.fake_count(0) == a0          # no new pinned allocation
    sets = [core.tmn_take(pool) for _ in range(70)]
    assert core.fake_pool_size(pool) == 0
    f0 = core.fake_count(1)
    for x in sets:
        core.tmn_give(pool, x)
    core.tmn_give(pool, s2)
    assert core.fake_pool_size(pool) == 64   # TMN_POOL_MAX; the rest freed
    core.fake_pool_free(pool)
    assert core.fake_count(1) >= f0


def test_device_failure_is_never_a_badarg_row(core):
    """Err flag 4 (a batch the device failed) and TM_EDEVICE fail the whole
    call as a device error -- the NIF returns {error, device} -- and never
    become a per-topic badarg: the reference raises badarg only for a '+'/'#'
    level (emqx_trie_search.erl:374-375).  ADVICE r3 (tmatch_nif_core.c
    passed err 4 through as a row the NIF mapped to badarg)."""
    pool = core.fake_pool_new()
    s = core.tmn_take(pool)
    for topics in ([b"ab", b"!x", b"cd"], [b"ab", b"~x"]):
        assert pack(core, s, topics) == TM_OK
        assert core.tmn_match(s, H, len(topics), TRAVERSAL) == TM_EDEVICE
    # a row left with flag 4 (never after a TM_OK call) reads as the device code, not badarg (1)
    assert pack(core, s, [b"!x"]) == TM_OK
    core.tmn_match(s, H, 1, TRAVERSAL)
    b, e = C.c_uint64(), C.c_uint64()
    assert core.tmn_row(s, 1, TRAVERSAL, 0, C.byref(b), C.byref(e)) == 4
    # a well-formed batch after it is unaffected
    assert pack(core, s, [b"ab", b"+x"]) == TM_OK
    assert core.tmn_match(s, H, 2, TRAVERSAL) == TM_OK
    assert rows(core, s, 2, TRAVERSAL) == [[0, 1], 1]
    core.tmn_give(pool, s)
    core.fake_pool_free(pool)


def test_reader_ticket_ends_once_even_if_never_ended(core):
    """A reader's ticket is ended exactly once: read_end twice ends it once,
    and a ticket whose reader died before read_end (the NIF resource's term
    collected: its destructor) ends the read then, so the library's safe
    epoch is never pinned by a killed reader."""
    r0, e0 = core.fake_count(4), core.fake_count(5)
    a = core.fake_ticket_new()
    b = core.fake_ticket_new()
    assert core.fake_count(4) == r0 + 2
    core.tmn_ticket_end(a)
    core.tmn_ticket_end(a)                      # idempotent
    assert core.fake_count(4) == r0 + 1 and core.fake_count(5) == e0 + 1
    core.fake_ticket_free(a)                    # already ended: nothing more
    core.fake_ticket_free(b)                    # never ended: the destructor ends it
    assert core.fake_count(4) == r0 and core.fake_count(5) == e0 + 2

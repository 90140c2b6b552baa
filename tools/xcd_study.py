#!/usr/bin/env python3
"""Study (data only, no kernel change): does routing topics to XCDs by their
first two levels make the walk faster?  Workgroups go round-robin over the 8
XCDs (block b -> XCD b % 8), so a batch permuted so that block b holds only
topics of group b % 8 (group = CRC of the first two levels) gives each XCD's
L2 one eighth of the trie's top.  Times the isolated walk (HIP events, the
library's profile) over the C3 batch in its own order and permuted."""
import sys
import zlib
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def xcd_order(ts, groups=8, block=256):
    g = np.empty(len(ts), np.int64)
    for i in range(len(ts)):
        w = ts.item(i).split(b"/")
        g[i] = zlib.crc32(b"/".join(w[:2])) % groups
    lists = [list(np.nonzero(g == k)[0]) for k in range(groups)]
    order, b = [], 0
    while any(lists):
        src = lists[b % groups] or max(lists, key=len)
        order.extend(src[:block])
        del src[:block]
        b += 1
    return np.array(order, np.int64), np.bincount(g, minlength=groups)


def main():
    import torch
    from bench import CONFIGS
    from emqx_amd import _native, workload as wl
    gen, nf, _ = CONFIGS["c3"]
    fs = wl.filters(gen, nf)
    ix = _native.Index(device=0)
    for lo in range(0, len(fs), 2_000_000):
        p = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(p), np.uint8), p.blob, p.offs, p.vals)
    B = 1_000_000
    ts = wl.topics(gen, nf, B)
    perm, sizes = xcd_order(ts)
    print("group sizes", sizes.tolist(), flush=True)
    dev = torch.device("cuda:0")
    sets = {"own order": ts, "xcd-routed": wl.take(ts, perm)}
    hit = torch.zeros(B + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    res = {}
    for name, s in sets.items():
        blob = torch.from_numpy(s.blob).to(dev)
        offs = torch.from_numpy(s.offs.view(np.int64)).to(dev)
        tiny = torch.zeros(16, dtype=torch.int32, device=dev)
        ix.match_batch_dev(B, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), tiny.data_ptr(), 0, err.data_ptr())
        torch.cuda.synchronize()
        out = torch.zeros(int(hit[-1].item()) + 16, dtype=torch.int32, device=dev)
        cap = out.numel()
        for rep in range(3):
            ix.profile(False)
            ix.match_batch_dev(B, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), out.data_ptr(), cap, err.data_ptr())
            ix.profile(True)
            ix.profile_read(reset=True)
            for _ in range(20):
                ix.match_batch_dev(B, blob.data_ptr(), offs.data_ptr(), hit.data_ptr(), out.data_ptr(), cap,
                                   err.data_ptr())
            torch.cuda.synchronize()
            w, b, n = ix.profile_read(reset=True)
            res.setdefault(name, []).append((w / n, b / n))
        print(f"{name}: walk ms {[round(x[0], 4) for x in res[name]]} batch ms {[round(x[1], 4) for x in res[name]]}",
              flush=True)


if __name__ == "__main__":
    main()

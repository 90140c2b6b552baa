import sys, time
sys.path.insert(0, "/root/repo")
from emqx_amd import workload as wl
t = time.time()
fs = wl.filters(3, 10_000_000)
ex1, ex2, lens = set(), set(), set()
nex = 0
for i in range(len(fs)):
    f = fs.item(i)
    w = f.split(b"/")
    if b"+" in w or b"#" in w:
        continue
    nex += 1
    lens.add(len(w))
    ex1.add((len(w), w[0]))
    ex2.add((len(w), w[0], w[1] if len(w) > 1 else None))
ts = wl.topics(3, 10_000_000, 200_000)
a = b = c = 0
for i in range(len(ts)):
    w = ts.item(i).split(b"/")
    a += len(w) in lens
    b += (len(w), w[0]) in ex1
    c += (len(w), w[0], w[1] if len(w) > 1 else None) in ex2
n = len(ts)
print(f"exact keys {nex} of {len(fs)}; distinct (len,w0) {len(ex1)}, (len,w0,w1) {len(ex2)}")
print(f"topics needing the lookup: by length {a/n:.3f}, by (len,w0) {b/n:.3f}, by (len,w0,w1) {c/n:.3f}  ({time.time()-t:.0f}s)")

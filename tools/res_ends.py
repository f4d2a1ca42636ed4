"""Per-workgroup end stamps of the resident kernel (TSG_RES_DUMP=2 lines "[tsg] resident ends: ...",
0.01 us ticks after the first workgroup saw the query): is the spread systematic per workgroup /
XCD (w % 8) or random from query to query?"""
import sys

import numpy as np

rows = [list(map(int, l.split(":", 1)[1].split())) for l in open(sys.argv[1]) if "resident ends:" in l]
E = np.array(rows, dtype=float) / 100.0  # us
q, W = E.shape
print(f"{q} queries x {W} workgroups; end mean {E.mean():.2f} us, per-query spread (max-min) p50 "
      f"{np.median(E.max(1) - E.min(1)):.2f}")
Z = E - E.mean(1, keepdims=True)
print("per-workgroup mean deviation: std %.3f us (a random spread of the per-query std %.3f would give %.3f)"
      % (Z.mean(0).std(), Z.std(1).mean(), Z.std(1).mean() / np.sqrt(q)))
a, b = Z[::2].mean(0), Z[1::2].mean(0)
print("split-half correlation of workgroup deviations: %.3f" % np.corrcoef(a, b)[0, 1])
for name, key in (("w % 8", np.arange(W) % 8), ("w // 32", np.arange(W) // 32), ("w % 32", np.arange(W) % 32)):
    g = [Z[:, key == k].mean() for k in np.unique(key)]
    print(name, " ".join(f"{x:+.2f}" for x in g))
late = np.argsort(Z.mean(0))[-12:]
print("latest workgroups (mean dev us):", " ".join(f"{w}:{Z.mean(0)[w]:+.2f}" for w in late))
crow = [list(map(int, l.split(":", 1)[1].split())) for l in open(sys.argv[1]) if "resident counts:" in l]
if crow:
    C = np.array(crow, dtype=float)
    c = C.mean(0)
    print("records per workgroup: mean %.2f max %d; corr(records, mean end dev) %.3f"
          % (c.mean(), c.max(), np.corrcoef(c, Z.mean(0))[0, 1]))
    for k in range(int(c.max()) + 1):
        sel = np.round(c) == k
        if sel.any():
            print(f"  {k} records: {sel.sum()} workgroups, mean end dev {Z.mean(0)[sel].mean():+.2f} us")

"""Make inputs for / check outputs of tools/fe29_bench dump (dev tool, Python big ints)."""
import sys
import numpy as np
P = 2**255 - 19
def val(w): return sum(int(x) << (29 * i) for i, x in enumerate(w))
mode, n, path = sys.argv[1], int(sys.argv[2]), sys.argv[3]
if mode == "gen":
    rng = np.random.default_rng(5)
    a = rng.integers(0, 2**30, size=(n, 18), dtype=np.uint64)
    a[:, 8] %= 2**25; a[:, 17] %= 2**25
    a[:64] = 2**30 - 1; a[:64, 8] = 2**25 - 1; a[:64, 17] = 2**25 - 1   # worst case
    a[64:128] = 2**29 - 1; a[64:128, 8] = 2**23 - 1; a[64:128, 17] = 2**23 - 1
    a.astype(np.uint32).tofile(path); sys.exit(0)
inp = np.fromfile(path, np.uint32).reshape(n, 18)
out = np.fromfile(sys.argv[4], np.uint32).reshape(n, 36)
bad = 0
def tight(w): return all(int(x) < 2**29 for i, x in enumerate(w[:8]) if i != 1) and int(w[1]) < 2**29 + 2**17 and int(w[8]) < 2**23
for t in range(n):
    a, b = val(inp[t, :9]), val(inp[t, 9:])
    m, s, ch, sch = (out[t, 9 * k:9 * k + 9] for k in range(4))
    x = s_ = a * a % P
    for _ in range(100): x = x * b % P
    y = a
    for _ in range(100): y = y * y % P
    ok = (val(m) % P == a * b % P and tight(m) and val(s) % P == a * a % P and tight(s)
          and val(ch) % P == x and tight(ch) and val(sch) % P == y and tight(sch))
    if not ok:
        bad += 1
        if bad < 5: print("mismatch lane", t)
print("fe29 checks:", n - bad, "ok of", n)
sys.exit(1 if bad else 0)

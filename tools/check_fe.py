"""Check tools/fe_bench dump output against Python big-int arithmetic (dev tool)."""
import sys
import numpy as np
P = 2**255 - 19
n = int(sys.argv[1])
inp = np.fromfile(sys.argv[2], np.uint32).reshape(n, 16)
out = np.fromfile(sys.argv[3], np.uint32).reshape(n, 40)
def val(w): return sum(int(x) << (32 * i) for i, x in enumerate(w))
bad = 0
for t in range(n):
    a, b = val(inp[t, :8]), val(inp[t, 8:])
    m, ad, sb, bt, ch = (val(out[t, 8 * k:8 * k + 8]) for k in range(5))
    x = a
    for _ in range(100): x = x * b % P
    ok = (m % P == a * b % P and m < 2**255 + 2**43 and ad % P == (a + b) % P and ad < 2**255 + 2**43
          and bt % P == b % P and sb % P == (a - b) % P and sb < 2**256 and ch % P == x)
    if not ok:
        bad += 1
        if bad < 5: print("mismatch lane", t, hex(a), hex(b))
print("fe checks:", n - bad, "ok of", n)
sys.exit(1 if bad else 0)

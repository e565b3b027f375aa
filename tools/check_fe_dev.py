"""Check tools/fe_dev_check output (device fe_mul/fe_sq/fe_mul2/fe_sq2) with Python big ints (dev tool)."""
import sys
import numpy as np
P = 2**255 - 19
T = [2**29 - 1, 2**29 + 2**17] + [2**29 - 1] * 6 + [2**23 - 1]
def val(w): return sum(int(x) << (29 * i) for i, x in enumerate(w))
def tight(w): return all(int(x) <= t for x, t in zip(w, T))
n = int(sys.argv[1])
inp = np.fromfile(sys.argv[2], np.uint32).reshape(n, 18)
out = np.fromfile(sys.argv[3], np.uint32).reshape(n, 54)
bad = 0
for t in range(n):
    a, b = val(inp[t, :9]), val(inp[t, 9:])
    exp = [a * b, a * a, a * b, b * b, a * a, b * b]
    for k in range(6):
        w = out[t, 9 * k:9 * k + 9]
        if val(w) % P != exp[k] % P or not tight(w):
            bad += 1
            if bad < 5: print("mismatch lane", t, "op", k)
print("fe dev checks:", n * 6 - bad, "ok of", n * 6)
sys.exit(1 if bad else 0)

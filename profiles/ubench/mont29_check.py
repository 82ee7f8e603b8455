# Checks profiles/ubench/mont29.hip output: the 9x29-bit product (R = 2^261) against exact
# big-integer Montgomery products, and the production 8x32 product (R = 2^256).
import numpy as np
q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
n = 4096
raw = np.fromfile("gpurun_out/mont29_check.bin", dtype=np.uint32)
h = raw[:16 * n].reshape(n, 16)
o = raw[16 * n:].reshape(n, 17)
def num(ws, bits=32):
    return sum(int(w) << (bits * i) for i, w in enumerate(ws))
bad = 0
for i in range(n):
    a, b = num(h[i, :8]), num(h[i, 8:])
    c256 = num(o[i, :8])
    c29 = num(o[i, 8:], 29)
    assert all(int(x) < (1 << 29) for x in o[i, 8:])
    exp256 = a * b * pow(2, -256, q) % q
    assert c256 == exp256, i
    assert c29 < (1 << 258)
    if c29 % q != a * b * pow(2, -261, q) % q:
        bad += 1
print("checked", n, "bad", bad)

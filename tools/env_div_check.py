"""Exhaustive check behind env_fetch's multiplications (csrc/shade_ops.hpp): SphericalMap.cpp:17-29
forms u = 0.5 + atan2(x, z) / (2 pi) and v = 0.5 - asin(y) / pi in double and rounds them to float.
For EVERY float angle a in [-float(pi), float(pi)] (u) and [-float(pi/2), float(pi/2)] (v) this
compares (float)(0.5 +/- a / c) with (float)(0.5 +/- a * (1 / c)) in IEEE double (numpy, correctly
rounded like the GPU's v_div / v_mul sequences).  ~2.2e9 angles each, ~1 minute per check.
usage: python tools/env_div_check.py [stride]   (stride > 1: every stride-th float, for a quick run)"""
import sys
import time

import numpy as np

PI = 3.14159265358979323846


def mismatches(hi_f, c, sign, stride=1):
    inv = 1.0 / c
    hi = int(np.float32(hi_f).view(np.uint32))
    bad = n = 0
    step = 1 << 26
    for start in range(0, hi + 1, step):
        u = np.arange(start, min(start + step, hi + 1), stride, dtype=np.uint32)
        for neg in (False, True):
            a = u.view(np.float32).astype(np.float64)
            if neg:
                a = -a
            r1 = (0.5 + sign * (a / c)).astype(np.float32)
            r2 = (0.5 + sign * (a * inv)).astype(np.float32)
            bad += int(np.count_nonzero(r1.view(np.uint32) != r2.view(np.uint32)))
            n += a.size
    return bad, n


if __name__ == "__main__":
    stride = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    for name, hi, c, sign in (("u", PI, 2 * PI, 1.0), ("v", PI / 2, PI, -1.0)):
        t = time.time()
        bad, n = mismatches(hi, c, sign, stride)
        print(f"{name}: {bad} mismatches of {n} angles ({time.time() - t:.1f} s)", flush=True)

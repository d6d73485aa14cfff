"""env_fetch's products with the double reciprocals of 2 pi and pi (csrc/shade_ops.hpp) give the
float u / v of SphericalMap.cpp:17-29's divisions: a strided sample of every float angle here (the
exhaustive run is tools/env_div_check.py, log in profiles/r5/r5zy/env_div_check.txt)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import env_div_check  # noqa: E402


def test_env_division_products_sample():
    for hi, c, sign in ((env_div_check.PI, 2 * env_div_check.PI, 1.0), (env_div_check.PI / 2, env_div_check.PI, -1.0)):
        bad, n = env_div_check.mismatches(hi, c, sign, stride=31)
        assert n > 60_000_000 and bad == 0

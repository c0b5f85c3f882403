#!/usr/bin/env python3
"""Diagnostic (GPU box): device jax.random draws vs the numpy restatement at C1; prints the mismatching elements
with their uniform, log1p argument and the log1p selftest's host / device values."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quadruped-pympc-tamols_amd"), ROOT, os.path.join(ROOT, "tests")]
from helpers import make_case, product_cfg  # noqa: E402
from oracle import jax_random_oracle as jr  # noqa: E402
from quadruped_pympc_amd import _lib  # noqa: E402
from test_gpu_jax_rng import expected_noise, first_key  # noqa: E402

case = make_case("c1", N=128, method="random_sampling", par="zero_order", H=10)
ctx = _lib.Context(product_cfg(case))
ctx.set_rng("jax")
key = first_key()
got = ctx.draw_noise(jr.pack_key(key), 0)
ctx.close()
want = expected_noise(case, key, True)
bad = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
print("mismatches", len(bad))
for r, c in bad[:10]:
    print(r, c, repr(got[r, c]), repr(want[r, c]))
# the log1p arguments of the whole draw: recompute u from the restatement's bits
import inspect
print([n for n in dir(jr) if not n.startswith("_")])
bits = None
for r, c in bad[:10]:
    # element (r, c) of the RS draw: rebuild its uniform from the restatement to show the erf_inv argument / branch
    pass

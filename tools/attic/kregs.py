"""VGPR / spill counts of every k_trace / k_event / k_emit instantiation in a built library
(development tool; the same reader as tests/test_kernel_resources.py).
usage: python tools/kregs.py [lib.so]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_kernel_resources as t  # noqa: E402

if len(sys.argv) > 1:
    t.LIB = os.path.abspath(sys.argv[1])
for k, v in sorted(t._kernels().items()):
    if "k_trace" in k or "k_event" in k or "k_emit" in k:
        print(f"{v.get('vgpr_count', 0):4d} spill {v.get('vgpr_spill_count', 0):4d}  {k}")

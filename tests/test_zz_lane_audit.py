"""The cross-lane read audit (VERDICT r5 "next" #5): run last in a `-m gpu` session whose library is the
diagnostic build `microrts_amd/libmrts_audit.so` (`make -C microrts_amd/csrc audit`, selected with
MRTS_LIB_PATH).  In that build every readlane checks that its source lane is active where it executes, and
every DPP reduction / prefix sum and every ballot that the kernels treat as whole-wave checks that the whole
wave is active (mrts_kernels.hip, MRTS_LANE_AUDIT); a violation records its source line.  This test reads
the record after every other GPU test of the session has run and fails on any violation.  With the product
library (no mrts_lane_audit export) it skips.

Why: round 4's shipped bug was a readlane of a lane that was inactive at the read (the compiler had sunk the
source's LDS read into a divergent loop); the value is then whatever the register last held —
usually right, rarely not, so sampling steps could miss it.  The audit turns "usually right" into a check
over every path the suite executes; DESIGN.md §4 lists each site and why its source lane is active.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_no_cross_lane_read_of_an_inactive_lane():
    from microrts_amd import _lib

    L = _lib.load()
    fn = getattr(L, "mrts_lane_audit", None)
    if fn is None:
        pytest.skip(f"{os.path.basename(_lib.LIB_PATH)} is not the audit build (MRTS_LIB_PATH=microrts_amd/libmrts_audit.so)")
    out = np.zeros(256, np.int32)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(out.ctypes.data_as(ctypes.c_void_p), 0) == 0
    hits = sorted({(int(v) >> 24, int(v) & 0xFFFFFF) for v in out if v})
    kinds = {1: "readlane of an inactive lane", 2: "DPP reduction with inactive lanes", 3: "ballot with inactive lanes"}
    assert not hits, "mrts_kernels.hip: " + "; ".join(f"line {ln}: {kinds.get(k, k)}" for k, ln in hits)
    # the check can fail: the negative control reads lane 40 from a branch only lanes 0..31 take
    assert L.mrts_lane_audit_probe() == 0
    assert fn(out.ctypes.data_as(ctypes.c_void_p), 1) == 0
    assert any((int(v) >> 24) == 1 for v in out if v), "the audit missed its negative control"

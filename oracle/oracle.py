"""ctypes binding of the CPU oracle (oracle/artes_oracle.c) -- TEST INFRASTRUCTURE ONLY.

See the header of artes_oracle.c for what the oracle restates and how it is pinned.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from artes_amd.abi import (ARTES_NUM_COUNTERS, ARTES_NUM_ERR, ARTES_NUM_TOTALS, ARTES_TRACE_FIELDS, GridArrays, GridDesc,
                           RunParams)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.oracle_grid_create.restype = C.c_void_p
        L.oracle_grid_create.argtypes = [C.POINTER(GridDesc)]
        L.oracle_grid_destroy.argtypes = [C.c_void_p]
        L.oracle_cell_depth.restype = C.c_int
        L.oracle_cell_depth.argtypes = [C.c_void_p, C.c_int]
        L.oracle_run.restype = C.c_int
        L.oracle_run.argtypes = [C.c_void_p, C.POINTER(RunParams), C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                 C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
        L.oracle_run_flow.restype = C.c_int
        L.oracle_run_flow.argtypes = list(L.oracle_run.argtypes) + [C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.oracle_max_threads.restype = C.c_int
        dp = C.POINTER(C.c_double)
        L.oracle_thermal.restype = C.c_int
        L.oracle_thermal.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), dp, dp, dp, dp]
        _lib = L
    return _lib


class OracleGrid:
    def __init__(self, atm: dict, oblateness: float = 0.0):
        self.arrays = GridArrays(atm, oblateness)
        self.h = lib().oracle_grid_create(C.byref(self.arrays.desc))
        if not self.h:
            raise MemoryError("oracle_grid_create failed")

    def cell_depth(self, wl: int = 0) -> int:
        return lib().oracle_cell_depth(self.h, wl)

    def thermal(self, wl: int = 0, thermal_weight: bool = True, ring: bool = False):
        """grid_initialize(2), planet branch: (cell_depth, emissivity_total, cell_luminosity[nphi][ntheta][nr])."""
        cd = C.c_int()
        tot = C.c_double()
        a = self.arrays
        lum = np.zeros((a.nphi, a.ntheta, a.nr))
        dp = C.POINTER(C.c_double)
        rc = lib().oracle_thermal(self.h, wl, int(bool(thermal_weight)), int(bool(ring)), C.byref(cd), C.byref(tot),
                                  lum.ctypes.data_as(dp), None, None)
        if rc != 0:
            raise RuntimeError(f"oracle_thermal failed: {rc}")
        return cd.value, tot.value, lum

    def run(self, params: RunParams, first: int, n: int, seed: int, threads: int = 0, records: bool = False):
        det = np.zeros((4, 4, params.ny, params.nx))
        tot = np.zeros(ARTES_NUM_TOTALS)
        cnt = np.zeros(ARTES_NUM_COUNTERS, dtype=np.uint64)
        err = np.zeros(ARTES_NUM_ERR, dtype=np.uint64)
        rec = np.zeros((n, ARTES_TRACE_FIELDS)) if records else None
        rc = lib().oracle_run(self.h, C.byref(params), first, n, seed, threads,
                              det.ctypes.data_as(C.POINTER(C.c_double)), tot.ctypes.data_as(C.POINTER(C.c_double)),
                              cnt.ctypes.data_as(C.POINTER(C.c_uint64)), err.ctypes.data_as(C.POINTER(C.c_uint64)),
                              rec.ctypes.data_as(C.POINTER(C.c_double)) if rec is not None else None)
        if rc != 0:
            raise RuntimeError(f"oracle_run failed: {rc}")
        return det, tot, cnt, err, rec

    def run_flow(self, params: RunParams, first: int, n: int, seed: int, threads: int = 0):
        """``run`` plus the flow accumulators: (det, totals, counters, err, flow_global
        [nphi][ntheta][nr][3], flow_latitudinal [nphi][ntheta][nr][4])."""
        a = self.arrays
        det = np.zeros((4, 4, params.ny, params.nx))
        tot = np.zeros(ARTES_NUM_TOTALS)
        cnt = np.zeros(ARTES_NUM_COUNTERS, dtype=np.uint64)
        err = np.zeros(ARTES_NUM_ERR, dtype=np.uint64)
        fg = np.zeros((a.nphi, a.ntheta, a.nr, 3))
        ft = np.zeros((a.nphi, a.ntheta, a.nr, 4))
        dp, up = C.POINTER(C.c_double), C.POINTER(C.c_uint64)
        rc = lib().oracle_run_flow(self.h, C.byref(params), first, n, seed, threads, det.ctypes.data_as(dp),
                                   tot.ctypes.data_as(dp), cnt.ctypes.data_as(up), err.ctypes.data_as(up), None,
                                   fg.ctypes.data_as(dp), ft.ctypes.data_as(dp))
        if rc != 0:
            raise RuntimeError(f"oracle_run_flow failed: {rc}")
        return det, tot, cnt, err, fg, ft

    def close(self):
        if self.h:
            lib().oracle_grid_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def max_threads() -> int:
    return lib().oracle_max_threads()

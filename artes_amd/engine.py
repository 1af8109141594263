"""ctypes binding of the HIP transport engine (``artes_amd/lib/libartes_hip.so``).

This is the product path: every packet is transported by the gfx950 kernel behind
``include/artes_amd.h``.  There is deliberately no CPU fallback -- if the shared
library is missing or no device is visible, :class:`EngineUnavailable` is raised.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .abi import (ARTES_ABI_VERSION, ARTES_NUM_COUNTERS, ARTES_NUM_ERR, ARTES_NUM_TOTALS, ARTES_TRACE_FIELDS, COUNTER_NAMES,
                  GridArrays, GridDesc, RunParams)

HERE = os.path.dirname(os.path.abspath(__file__))
# ARTES_LIB_PATH selects another build of the engine (the A/B tools); a development build
# (ARTES_DEV_KNOBS: its schedule also follows ARTES_* environment variables) loads only with the
# explicit opt-in ARTES_DEV_LIB=1, so a stray path cannot bring environment-driven engine
# selection back into a production run
LIB_PATH = os.environ.get("ARTES_LIB_PATH") or os.path.join(HERE, "lib", "libartes_hip.so")

_lib = None


KERNEL_NAMES = ("trace", "event", "emit", "aux", "persistent")   # ARTES_K_* order
# artes_set_tuning keys (include/artes_amd.h; transport.hip, TUNE)
TUNING_KEYS = ("engine", "pool", "steps", "refill", "static", "dgrab", "batch", "batch_min", "hbatch", "gbatch", "defer",
               "backward", "emit_first", "late_append", "pix1", "det_lds", "event_lds", "event_ldsc", "event_block",
               "event_bpc", "trace_bpc", "wpe", "msym", "max_it", "verbose", "trace_gtab", "det_ordered", "event_ldsu")


class EngineUnavailable(RuntimeError):
    pass


class EngineError(RuntimeError):
    """A failed engine call; ``err`` holds the error-code counts the call returned, when it
    returned any (e.g. the ARTES_DEBUG invariant counters that made it fail)."""

    def __init__(self, msg: str, err=None):
        super().__init__(msg)
        self.err = err


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (soname
    # libamdhip64.so.7).  Loading torch first makes this library's DT_NEEDED resolve to
    # that same runtime, so torch tensors / RCCL and the engine share one HSA context.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    L.artes_abi_version.restype = C.c_int32
    L.artes_build_info.restype = C.c_char_p
    L.artes_last_error.restype = C.c_char_p
    L.artes_device_count.restype = C.c_int32
    L.artes_grid_create.restype = C.c_int32
    L.artes_grid_create.argtypes = [C.POINTER(GridDesc), C.c_int32, C.POINTER(C.c_void_p)]
    L.artes_grid_destroy.argtypes = [C.c_void_p]
    L.artes_grid_cell_depth.restype = C.c_int32
    L.artes_grid_cell_depth.argtypes = [C.c_void_p, C.c_int32]
    L.artes_grid_thermal.restype = C.c_int32
    L.artes_grid_thermal.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.artes_grid_num_matrices.restype = C.c_int32
    L.artes_grid_num_matrices.argtypes = [C.c_void_p]
    dp, up = C.POINTER(C.c_double), C.POINTER(C.c_uint64)
    L.artes_run.restype = C.c_int32
    L.artes_run.argtypes = [C.c_void_p, C.POINTER(RunParams), C.c_uint64, C.c_uint64, C.c_uint64, dp, dp, up, up]
    L.artes_run_device.restype = C.c_int32
    L.artes_run_device.argtypes = [C.c_void_p, C.POINTER(RunParams), C.c_uint64, C.c_uint64, C.c_uint64,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.artes_run_flow.restype = C.c_int32
    L.artes_run_flow.argtypes = [C.c_void_p, C.POINTER(RunParams), C.c_uint64, C.c_uint64, C.c_uint64, dp, dp, up, up,
                                 dp, dp]
    L.artes_run_device_flow.restype = C.c_int32
    L.artes_run_device_flow.argtypes = [C.c_void_p, C.POINTER(RunParams), C.c_uint64, C.c_uint64, C.c_uint64,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p]
    L.artes_run_trace.restype = C.c_int32
    L.artes_run_trace.argtypes = [C.c_void_p, C.POINTER(RunParams), C.c_uint64, C.c_uint64, C.c_uint64, dp]
    L.artes_last_kernel_ms.restype = C.c_double
    L.artes_last_kernel_ms.argtypes = [C.c_void_p]
    L.artes_set_profiling.restype = C.c_int32
    L.artes_set_profiling.argtypes = [C.c_void_p, C.c_int32]
    L.artes_kernel_times.restype = C.c_int32
    L.artes_kernel_times.argtypes = [C.c_void_p, dp, up]
    L.artes_set_tuning.restype = C.c_int32
    L.artes_set_tuning.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
    L.artes_get_tuning.restype = C.c_int64
    L.artes_get_tuning.argtypes = [C.c_void_p, C.c_char_p]
    L.artes_last_launch.restype = C.c_char_p
    L.artes_last_launch.argtypes = [C.c_void_p]
    if L.artes_abi_version() != ARTES_ABI_VERSION:
        raise EngineUnavailable("ABI version mismatch")
    if b"development build" in L.artes_build_info() and os.environ.get("ARTES_DEV_LIB") != "1":
        raise EngineUnavailable(f"{LIB_PATH} is a development build (tuning from the environment): "
                                "set ARTES_DEV_LIB=1 to load it deliberately")
    _lib = L
    return L


def build_info() -> str:
    """The loaded library's build string (``artes_build_info``)."""
    return lib().artes_build_info().decode()


def device_count() -> int:
    return lib().artes_device_count()


def _check(rc: int, what: str, err=None) -> None:
    if rc != 0:
        raise EngineError(f"{what} failed ({rc}): {lib().artes_last_error().decode(errors='replace')}", err)


class RunResult:
    """Raw (un-normalised) outputs of one transport call."""

    def __init__(self, det, totals, counters, err, flow_global=None, flow_latitudinal=None):
        self.det = det            # [4][4][ny][nx]
        self.totals = totals      # [ARTES_NUM_TOTALS]
        self.counters = counters  # [ARTES_NUM_COUNTERS]
        self.err = err            # [ARTES_NUM_ERR]
        self.flow_global = flow_global            # [nphi][ntheta][nr][3] or None
        self.flow_latitudinal = flow_latitudinal  # [nphi][ntheta][nr][4] or None

    def counter(self, name: str) -> int:
        return int(self.counters[COUNTER_NAMES.index(name)])

    def __iadd__(self, other: "RunResult"):
        self.det += other.det
        self.totals += other.totals
        self.counters += other.counters
        self.err += other.err
        for k in ("flow_global", "flow_latitudinal"):
            a, b = getattr(self, k), getattr(other, k)
            if b is not None:
                setattr(self, k, b.copy() if a is None else a + b)
        return self


class Grid:
    """Device-resident atmosphere tables (``artes_grid_create``)."""

    def __init__(self, atm: dict, device: int = 0, oblateness: float = 0.0):
        L = lib()
        n = L.artes_device_count()
        if n <= 0:
            raise EngineUnavailable("no HIP device visible")
        self.arrays = GridArrays(atm, oblateness)
        self.h = C.c_void_p()
        self.device = device
        _check(L.artes_grid_create(C.byref(self.arrays.desc), device, C.byref(self.h)), "artes_grid_create")
        # the host copies are not needed once the tables live in HBM
        self.nr, self.ntheta, self.nphi, self.nwav = (self.arrays.nr, self.arrays.ntheta, self.arrays.nphi,
                                                      self.arrays.nwav)
        self.arrays = None

    def cell_depth(self, wl: int = 0) -> int:
        return lib().artes_grid_cell_depth(self.h, wl)

    def thermal(self, wl: int = 0, thermal_weight: bool = True, ring: bool = False):
        """Thermal-source tables (``artes_grid_thermal``): (cell_depth, emissivity_total,
        cell_luminosity[nphi][ntheta][nr])."""
        cd = C.c_int32()
        tot = C.c_double()
        lum = np.zeros((self.nphi, self.ntheta, self.nr))
        _check(lib().artes_grid_thermal(self.h, int(wl), int(bool(thermal_weight)), int(bool(ring)), C.byref(cd),
                                        C.byref(tot), lum.ctypes.data_as(C.POINTER(C.c_double))), "artes_grid_thermal")
        return cd.value, tot.value, lum

    def num_matrices(self) -> int:
        return lib().artes_grid_num_matrices(self.h)

    def set_tuning(self, **kv) -> None:
        """Schedule overrides of this handle (``artes_set_tuning``; keys ``TUNING_KEYS``, a value
        of ``None`` or -1 restores the default, ``engine="persistent"`` selects the fused engine)."""
        for k, v in kv.items():
            if k == "engine" and isinstance(v, str):
                v = {"event": 0, "persistent": 1}[v]
            _check(lib().artes_set_tuning(self.h, k.encode(), -1 if v is None else int(v)), f"artes_set_tuning({k})")

    def last_launch(self) -> str:
        """The kernel instantiations of the last call (``artes_last_launch``)."""
        return lib().artes_last_launch(self.h).decode()

    def tuning(self) -> dict:
        """The keys this handle overrides ({} in production)."""
        out = {}
        for k in TUNING_KEYS:
            v = lib().artes_get_tuning(self.h, k.encode())
            if v >= 0:
                out[k] = int(v)
        return out

    def run(self, params: RunParams, first: int, n: int, seed: int, flow_global: bool = False,
            flow_latitudinal: bool = False) -> RunResult:
        """One transport call; with ``flow_global`` / ``flow_latitudinal`` also the energy-transport
        accumulators (``artes_run_flow``; output:flow_global / output:flow_latitudinal)."""
        det = np.zeros((4, 4, params.ny, params.nx))
        tot = np.zeros(ARTES_NUM_TOTALS)
        cnt = np.zeros(ARTES_NUM_COUNTERS, dtype=np.uint64)
        err = np.zeros(ARTES_NUM_ERR, dtype=np.uint64)
        dp, up = C.POINTER(C.c_double), C.POINTER(C.c_uint64)
        if not (flow_global or flow_latitudinal):
            _check(lib().artes_run(self.h, C.byref(params), int(first), int(n), int(seed), det.ctypes.data_as(dp),
                                   tot.ctypes.data_as(dp), cnt.ctypes.data_as(up), err.ctypes.data_as(up)),
                   "artes_run", err)
            return RunResult(det, tot, cnt, err)
        fg = np.zeros((self.nphi, self.ntheta, self.nr, 3)) if flow_global else None
        ft = np.zeros((self.nphi, self.ntheta, self.nr, 4)) if flow_latitudinal else None
        _check(lib().artes_run_flow(self.h, C.byref(params), int(first), int(n), int(seed), det.ctypes.data_as(dp),
                                    tot.ctypes.data_as(dp), cnt.ctypes.data_as(up), err.ctypes.data_as(up),
                                    fg.ctypes.data_as(dp) if fg is not None else None,
                                    ft.ctypes.data_as(dp) if ft is not None else None), "artes_run_flow")
        return RunResult(det, tot, cnt, err, fg, ft)

    def run_device(self, params: RunParams, first: int, n: int, seed: int, det_ptr: int, tot2_ptr: int = 0,
                   cnt_ptr: int = 0, err_ptr: int = 0, stream: int = 0) -> None:
        """Asynchronous launch accumulating into device buffers (e.g. torch tensors' data_ptr())."""
        _check(lib().artes_run_device(self.h, C.byref(params), int(first), int(n), int(seed), C.c_void_p(det_ptr),
                                      C.c_void_p(tot2_ptr or None), C.c_void_p(cnt_ptr or None),
                                      C.c_void_p(err_ptr or None), C.c_void_p(stream or None)), "artes_run_device")

    def run_device_flow(self, params: RunParams, first: int, n: int, seed: int, det_ptr: int, tot2_ptr: int = 0,
                        cnt_ptr: int = 0, err_ptr: int = 0, flow_global_ptr: int = 0, flow_latitudinal_ptr: int = 0,
                        stream: int = 0) -> None:
        """``run_device`` plus device flow accumulators ([nphi][ntheta][nr][3] / [..][4] doubles)."""
        _check(lib().artes_run_device_flow(self.h, C.byref(params), int(first), int(n), int(seed),
                                           C.c_void_p(det_ptr), C.c_void_p(tot2_ptr or None),
                                           C.c_void_p(cnt_ptr or None), C.c_void_p(err_ptr or None),
                                           C.c_void_p(flow_global_ptr or None),
                                           C.c_void_p(flow_latitudinal_ptr or None), C.c_void_p(stream or None)),
               "artes_run_device_flow")

    def trace(self, params: RunParams, first: int, n: int, seed: int) -> np.ndarray:
        """Per-packet records ``[n][ARTES_TRACE_FIELDS]`` (``artes_run_trace``): peeled I, scatterings,
        crossings, end state (1 exit, 2 absorbed, 3 dropped), peeled -Q, U, V, 0."""
        rec = np.zeros((n, ARTES_TRACE_FIELDS))
        _check(lib().artes_run_trace(self.h, C.byref(params), int(first), int(n), int(seed),
                                     rec.ctypes.data_as(C.POINTER(C.c_double))), "artes_run_trace")
        return rec

    def last_kernel_ms(self) -> float:
        return lib().artes_last_kernel_ms(self.h)

    def set_profiling(self, on: bool = True) -> None:
        _check(lib().artes_set_profiling(self.h, int(bool(on))), "artes_set_profiling")

    def kernel_times(self) -> dict:
        """{kernel class: (summed ms, launches)} since the last call (profiling on)."""
        ms = np.zeros(len(KERNEL_NAMES))
        n = np.zeros(len(KERNEL_NAMES), dtype=np.uint64)
        _check(lib().artes_kernel_times(self.h, ms.ctypes.data_as(C.POINTER(C.c_double)),
                                        n.ctypes.data_as(C.POINTER(C.c_uint64))), "artes_kernel_times")
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(KERNEL_NAMES)}

    def close(self) -> None:
        if getattr(self, "h", None) and self.h.value:
            lib().artes_grid_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

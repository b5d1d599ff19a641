"""ctypes binding of libfu.so (the C ABI in include/fu.h).

The product has no fallback. If libfu.so is missing this module raises at import time
(build it with `make -C simgrid-flow-updating-implementation_amd` or
`python -c "import __graft_entry__ as g; g.build()"`). If no GPU is visible, the device
entry points fail loudly with the library's own error message.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FU_LIBRARY", os.path.join(HERE, "libfu.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libfu.so not found at {LIB_PATH}: build it with "
        "`make -C simgrid-flow-updating-implementation_amd` (no CPU fallback exists)")

lib = ctypes.CDLL(LIB_PATH)


class FuError(RuntimeError):
    """A libfu call returned a negative status."""

    def __init__(self, func: str, code: int, msg: str):
        super().__init__(f"{func} failed ({code}): {msg}")
        self.code = code


i32 = ctypes.c_int32
i64 = ctypes.c_int64
u64 = ctypes.c_uint64
f64 = ctypes.c_double
f32 = ctypes.c_float
vp = ctypes.c_void_p
cp = ctypes.c_char_p
P = ctypes.POINTER

# (name, argtypes)
_SIGS = {
    "fu_last_error": ([], cp),
    "fu_version": ([], ctypes.c_int),
    "fu_device_count": ([P(i32)], ctypes.c_int),
    "fu_mem_info": ([i32, P(i64), P(i64)], ctypes.c_int),
    "fu_graph_from_edges": ([i32, i64, vp, vp, P(vp)], ctypes.c_int),
    "fu_graph_from_csr": ([i32, vp, vp, i32, P(vp)], ctypes.c_int),
    "fu_graph_gen_er": ([i32, i64, u64, P(vp)], ctypes.c_int),
    "fu_graph_gen_rr": ([i32, i32, u64, P(vp)], ctypes.c_int),
    "fu_graph_gen_rmat": ([i32, i32, f64, f64, f64, u64, P(vp)], ctypes.c_int),
    "fu_graph_gen_rgg": ([i32, f64, u64, P(vp)], ctypes.c_int),
    "fu_graph_info": ([vp, P(i32), P(i64), P(i32), P(i32)], ctypes.c_int),
    "fu_graph_export": ([vp, vp, vp, vp], ctypes.c_int),
    "fu_graph_free": ([vp], ctypes.c_int),
    "fu_graph_relabel": ([vp, i32, vp, P(vp)], ctypes.c_int),
    "fu_values_uniform": ([i64, u64, f64, f64, vp], ctypes.c_int),
    "fu_create": ([i32, i64, vp, vp, vp, vp, i32, P(vp)], ctypes.c_int),
    "fu_create_from_graph": ([vp, vp, i32, P(vp)], ctypes.c_int),
    "fu_create_from_graph_ex": ([vp, vp, i32, i32, P(vp)], ctypes.c_int),
    "fu_set_option": ([vp, cp, i64], ctypes.c_int),
    "fu_reset": ([vp], ctypes.c_int),
    "fu_set_targets": ([vp, vp], ctypes.c_int),
    "fu_run_collectall": ([vp, i32, i32, vp], ctypes.c_int),
    "fu_run_collectall_timed": ([vp, i32, P(f32)], ctypes.c_int),
    "fu_tune": ([vp], ctypes.c_int),
    "fu_run_collectall_marked": ([vp, i32, vp], ctypes.c_int),
    "fu_mark": ([vp, i32], ctypes.c_int),
    "fu_mark_elapsed": ([vp, i32, i32, P(f32)], ctypes.c_int),
    "fu_max_err": ([vp, P(f64)], ctypes.c_int),
    "fu_get_estimates": ([vp, vp], ctypes.c_int),
    "fu_get_flows": ([vp, vp], ctypes.c_int),
    "fu_get_round": ([vp, P(i64)], ctypes.c_int),
    "fu_get_info": ([vp, vp], ctypes.c_int),
    "fu_get_pack": ([vp, vp], ctypes.c_int),
    "fu_synchronize": ([vp], ctypes.c_int),
    "fu_destroy": ([vp], ctypes.c_int),
    "fu_copy_bandwidth": ([i32, i64, i32, P(f64)], ctypes.c_int),
    "fu_trace_build": ([i32, vp, vp, i32, i32, cp, P(vp)], ctypes.c_int),
    "fu_trace_build_ex": ([i32, vp, vp, i32, i32, cp, cp, P(vp)], ctypes.c_int),
    "fu_trace_build_routes": ([i32, vp, vp, i32, i32, cp, cp, vp, P(vp)], ctypes.c_int),
    "fu_trace_build_links": ([i32, vp, vp, i32, i32, cp, cp, i32, vp, vp, vp, vp, vp, f64, f64, f64, P(vp)],
                             ctypes.c_int),
    "fu_trace_build_links_ex": ([i32, vp, vp, i32, i32, cp, cp, i32, vp, vp, vp, vp, vp, f64, f64, f64, f64, f64,
                                 P(vp)], ctypes.c_int),
    "fu_trace_build_links_cross": ([i32, vp, vp, i32, i32, cp, cp, i32, vp, vp, vp, vp, vp, f64, f64, f64, f64, f64,
                                    f64, P(vp)], ctypes.c_int),
    "fu_trace_fault_stats": ([vp, P(i64), P(i64)], ctypes.c_int),
    "fu_trace_info": ([vp, vp], ctypes.c_int),
    "fu_trace_export": ([vp, vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
    "fu_trace_free": ([vp], ctypes.c_int),
    "fu_replay_create": ([i32, vp, vp, i32, vp, i64, vp, i64, vp, i64, vp, i64, i32, P(vp)],
                         ctypes.c_int),
    "fu_replay_create_from_trace": ([vp, vp, i32, P(vp)], ctypes.c_int),
    "fu_replay_run": ([vp, i32, i32, vp, vp], ctypes.c_int),
    "fu_replay_run_timed": ([vp, i32, P(f32)], ctypes.c_int),
    "fu_replay_get": ([vp, vp, vp, vp], ctypes.c_int),
    "fu_replay_destroy": ([vp], ctypes.c_int),
    "fu_replay_set_option": ([vp, cp, i64], ctypes.c_int),
    "fu_dist_create_local": ([i32, i64, vp, vp, vp, i32, i32, i32, vp, vp, vp, i32, P(vp)], ctypes.c_int),
    "fu_dist_exchange_local": ([vp, i32], ctypes.c_int),
    "fu_dist_run_local": ([vp, i32, i32], ctypes.c_int),
    "fu_dist_halo_time": ([vp, P(ctypes.c_float)], ctypes.c_int),
    "fu_part_gen_rgg": ([i64, f64, u64, i32, i32, P(vp)], ctypes.c_int),
    "fu_part_info": ([vp, vp], ctypes.c_int),
    "fu_part_export": ([vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
    "fu_part_free": ([vp], ctypes.c_int),
    "fu_values_uniform_range": ([i64, i64, u64, f64, f64, vp], ctypes.c_int),
    "fu_dist_unique_id": ([vp], ctypes.c_int),
    "fu_dist_create": ([i32, i64, vp, vp, vp, vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, vp,
                        vp, i32, P(vp)], ctypes.c_int),
}

EXPORTED = tuple(_SIGS)

for _name, (_args, _res) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.argtypes = _args
    _f.restype = _res


def last_error() -> str:
    msg = lib.fu_last_error()
    return msg.decode() if msg else ""


def check(func: str, code: int) -> int:
    if code < 0:
        raise FuError(func, code, last_error())
    return code


def call(name: str, *args) -> int:
    return check(name, getattr(lib, name)(*args))


def ptr(a: np.ndarray | None):
    """Raw data pointer of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data_as(vp)


def copy_bandwidth(device: int = 0, nbytes: int = 1 << 30, iters: int = 5) -> float:
    """The device's float4 copy rate in GB/s (read + write), best of `iters` copies."""
    g = f64(0.0)
    call("fu_copy_bandwidth", int(device), int(nbytes), int(iters), ctypes.byref(g))
    return float(g.value)


def mem_info(device: int = 0) -> tuple:
    """(free, total) bytes of HBM on the device."""
    fr, tot = i64(0), i64(0)
    call("fu_mem_info", int(device), ctypes.byref(fr), ctypes.byref(tot))
    return int(fr.value), int(tot.value)


def device_count() -> int:
    c = i32(0)
    call("fu_device_count", ctypes.byref(c))
    return int(c.value)

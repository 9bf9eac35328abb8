"""ctypes binding of libmsa.so (include/msa.h).

The library is built in-tree by ``__graft_entry__.build()`` /
``make -C cse305_parallel_sequence_alignment_amd/csrc``.  There is no CPU
fallback: if the library is missing, importing the compute API raises, and
on a machine without a gfx950 GPU every call returns MSA_ERR_NODEV, which
this module turns into ``MsaError``.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
# MSA_LIB_PATH: a diagnostic build (e.g. -DMSA_STAMPS) loaded instead of the in-tree library
LIB_PATH = Path(os.environ.get("MSA_LIB_PATH", str(PKG / "libmsa.so")))

MSA_OK = 0
STATUS = {
    0: "ok", -1: "invalid argument", -2: "more than 8 distinct symbols", -3: "HIP runtime error",
    -4: "no gfx950 device", -5: "unsupported parameters", -6: "cross-workgroup wait timed out",
    -7: "out of memory", -8: "output buffer too small", -9: "traceback found no predecessor",
}

# msa_alg_e / msa_out_e
SW_LINEAR, SW_AFFINE, NW_BANDED, REF_GOTOH, PARTIAL = 0, 1, 2, 3, 4
CELLS_NONE, CELLS_H, CELLS_DIR, CELLS_TAB = 0, 1, 2, 3


class MsaError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: msa status {status} ({STATUS.get(status, 'unknown')})")


def check(rc: int, what: str = "msa") -> None:
    if rc != MSA_OK:
        raise MsaError(rc, what)


class Node(C.Structure):
    _fields_ = [("i", C.c_uint64), ("j", C.c_uint64), ("t", C.c_int32), ("pad", C.c_int32)]


class PlanDesc(C.Structure):
    _fields_ = [
        ("alg", C.c_int32), ("cells", C.c_int32), ("match", C.c_int32), ("mismatch", C.c_int32),
        ("gap_open", C.c_int32), ("gap_extend", C.c_int32), ("start_type", C.c_int32), ("band", C.c_int32),
        ("track_end", C.c_int32), ("single", C.c_int32), ("n_pairs", C.c_int64),
        ("m", C.POINTER(C.c_int64)), ("n", C.POINTER(C.c_int64)),
        ("a_off", C.POINTER(C.c_int64)), ("b_off", C.POINTER(C.c_int64)),
    ]


class PairResult(C.Structure):
    _fields_ = [("score", C.c_int32), ("status", C.c_int32), ("end_i", C.c_int64), ("end_j", C.c_int64),
                ("fin", C.c_int32 * 3), ("pad", C.c_int32)]


_lib = None


def lib() -> C.CDLL:
    """Load libmsa.so (raises if it was not built: the product has no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = _Bind(C.CDLL(str(LIB_PATH)))
    P, sz, i32, i64, u64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_int64, C.c_uint64
    L.msa_status_string.restype = C.c_char_p
    L.msa_status_string.argtypes = [C.c_int]
    L.msa_version.restype = C.c_int
    L.msa_device_count.argtypes = [C.POINTER(C.c_int)]
    L.msa_set_device_budget.argtypes = [C.c_int64]
    L.msa_device_budget_info.argtypes = [C.POINTER(C.c_int64)]
    L.msa_device_memory_info.argtypes = [C.POINTER(C.c_int64)]
    L.msa_main_alignment.argtypes = [P, P, sz, sz, sz, C.c_double, C.c_double, P, sz, C.POINTER(sz),
                                     C.POINTER(C.c_double)]
    L.msa_subproblem.argtypes = [P, P, sz, sz, sz, sz, C.c_int, C.c_int, C.c_double, C.c_double, P, P, P, P, sz,
                                 C.POINTER(sz), P, C.POINTER(C.c_int)]
    L.msa_partial_partition.argtypes = [P, P, sz, sz, sz, C.c_double, C.c_double, C.c_int, C.c_int, P, sz,
                                        C.POINTER(sz)]
    L.msa_partial_tables.argtypes = [P, P, sz, sz, C.c_double, C.c_double, C.c_int, C.c_int, P, P, P, P, P, P]
    L.msa_partition_tables.argtypes = [P, P, P, P, P, P, sz, sz, sz, C.c_double, P, sz, C.POINTER(sz)]
    L.msa_non_parallel_tables.argtypes = [P, P, sz, sz, sz, sz, C.c_int, C.c_int, C.c_double, C.c_double, P, sz,
                                          C.POINTER(sz)]
    L.msa_subproblem_f64.argtypes = [P, P, sz, sz, sz, sz, C.c_int, C.c_double, C.c_double, C.c_int, P, P, P,
                                     C.POINTER(C.c_int)]
    L.msa_subproblem_row.argtypes = [C.c_int, P, P, sz, sz, sz, sz, C.c_int, C.c_double, C.c_double, sz, sz, P, P,
                                     P, P, P, P, P]
    L.msa_optimal_alignment.argtypes = [P, P, sz, sz, sz, C.c_double, C.c_double, P, sz, C.c_int, P, sz,
                                        C.POINTER(sz), P, sz, C.POINTER(sz)]
    L.msa_main_alignment_partitioned.argtypes = [P, P, sz, sz, sz, C.c_double, C.c_double, C.c_int, P, sz,
                                                 C.POINTER(sz)]
    L.msa_plan_create.argtypes = [C.POINTER(PlanDesc), C.POINTER(P)]
    L.msa_plan_destroy.argtypes = [P]
    L.msa_plan_destroy.restype = None
    L.msa_plan_cells_size.argtypes = [P, C.POINTER(i64)]
    L.msa_plan_run.argtypes = [P, P, P, P, P, P, P]
    L.msa_plan_results.argtypes = [P, P, P]
    L.msa_plan_error.argtypes = [P, C.POINTER(C.c_int), P]
    L.msa_plan_run_info.argtypes = [P, P, P]
    L.msa_plan_launch_info.argtypes = [P, P]
    L.msa_plan_clear_error.argtypes = [P, P]
    L.msa_plan_scores.argtypes = [P, P, P]
    L.msa_plan_stripe_meta.argtypes = [P, P, i64, P]
    L.msa_plan_stripes.argtypes = [P]
    L.msa_plan_stripes.restype = i64
    L.msa_plan_pair_layout.argtypes = [P, i64, C.POINTER(i64)]
    L.msa_plan_checksum.argtypes = [P, P, i64, C.POINTER(u64), P]
    L.msa_plan_traceback.argtypes = [P, i64, P, P, i64, P, P]
    L.msa_plan_traceback_gotoh.argtypes = [P, i64, C.c_int, P, P, i64, P, P]
    L.msa_plan_last_kernel_ms.argtypes = [P, C.POINTER(C.c_float)]
    L.msa_plan_set_timing.argtypes = [P, i32]
    L.msa_encode_pair.argtypes = [P, sz, P, sz, P, P]
    L.msa_sw_align.argtypes = [P, sz, P, sz, i32, i32, i32, i32, C.POINTER(i32), C.POINTER(i64), C.POINTER(i64),
                               C.POINTER(i64), C.POINTER(i64), P, sz]
    _lib = L.lib
    return _lib


class _Bind:
    """Attribute proxy used while declaring signatures (all symbols must exist)."""

    def __init__(self, lib):
        self.lib = lib

    def __getattr__(self, name):
        return getattr(self.lib, name)


# Every symbol include/msa.h declares (checked by the CPU test suite).
EXPORTED = [
    "msa_status_string", "msa_version", "msa_device_count", "msa_set_device_budget", "msa_device_budget_info", "msa_device_memory_info", "msa_main_alignment", "msa_subproblem",
    "msa_non_parallel_tables", "msa_optimal_alignment", "msa_main_alignment_partitioned",
    "msa_subproblem_f64", "msa_subproblem_row",
    "msa_partial_partition", "msa_partial_tables", "msa_partition_tables", "msa_plan_create", "msa_plan_destroy", "msa_plan_cells_size",
    "msa_plan_run", "msa_plan_results", "msa_plan_error", "msa_plan_run_info", "msa_plan_clear_error", "msa_plan_scores",
    "msa_plan_stripe_meta", "msa_plan_stripes", "msa_plan_pair_layout", "msa_plan_launch_info",
    "msa_plan_checksum", "msa_plan_traceback", "msa_plan_traceback_gotoh",
    "msa_plan_last_kernel_ms", "msa_plan_set_timing", "msa_encode_pair", "msa_sw_align",
]

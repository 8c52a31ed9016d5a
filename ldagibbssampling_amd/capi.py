"""ctypes binding of the C ABI in include/lda_mi355x.h (liblda_mi355x.so).

The library is built in-tree (ldagibbssampling_amd/lib/) by build.py /
__graft_entry__.build().  There is no CPU fallback: if the library is missing
or cannot be loaded, importing the sampler raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "liblda_mi355x.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "lda_mi355x.h")

LDA_OK = 0
STATUS_NAMES = {
    -1: "LDA_ERR_INVALID_ARG",
    -2: "LDA_ERR_DEVICE",
    -3: "LDA_ERR_OUT_OF_MEMORY",
    -4: "LDA_ERR_STATE",
    -5: "LDA_ERR_UNSUPPORTED",
    -6: "LDA_ERR_INTERNAL",
}
MAX_TOPICS = 4096
MAX_TOPICS_DENSE = 1024
MAX_DOC_TOKENS_BIGK = 65535
MAX_EXCHANGE_PARTS = 4
SAMPLERS = {"dense": 0, "sparse": 1}
COUNT_UPDATE = {"auto": 0, "recount": 1, "delta": 2}


class LdaError(RuntimeError):
    def __init__(self, status: int, where: str, message: str):
        self.status = status
        super().__init__(f"{where}: {STATUS_NAMES.get(status, status)}: {message}")


class lda_config(C.Structure):
    _fields_ = [
        ("num_topics", C.c_int32),
        ("num_types", C.c_int32),
        ("num_docs", C.c_int64),
        ("alpha", C.POINTER(C.c_double)),
        ("beta", C.c_double),
        ("seed", C.c_uint64),
        ("device", C.c_int32),
        ("sampler", C.c_int32),
        ("token_base", C.c_int64),
        ("tokens_per_range", C.c_int64),
    ]


_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_vp = C.c_void_p

# name -> (restype, argtypes); every symbol include/lda_mi355x.h declares.
SIGNATURES = {
    "lda_create": (C.c_int32, [C.POINTER(_vp), C.POINTER(lda_config), _i64p, _vp, _vp]),
    "lda_destroy": (None, [_vp]),
    "lda_sweep": (C.c_int32, [_vp, C.c_int32]),
    "lda_sample": (C.c_int32, [_vp]),
    "lda_delta_buffer": (C.c_int32, [_vp, C.POINTER(_vp), C.POINTER(C.c_size_t)]),
    "lda_apply": (C.c_int32, [_vp]),
    "lda_set_exchange_parts": (C.c_int32, [_vp, C.c_int32, C.c_int32]),
    "lda_get_exchange_parts": (C.c_int32, [_vp, C.POINTER(C.c_int32)]),
    "lda_sample_part": (C.c_int32, [_vp, C.c_int32]),
    "lda_delta_buffer_part": (C.c_int32, [_vp, C.c_int32, C.POINTER(_vp), C.POINTER(C.c_size_t)]),
    "lda_set_stream": (C.c_int32, [_vp, _vp]),
    "lda_get_stream": (C.c_int32, [_vp, C.POINTER(_vp)]),
    "lda_synchronize": (C.c_int32, [_vp]),
    "lda_get_sweep": (C.c_int32, [_vp, C.POINTER(C.c_uint32)]),
    "lda_set_sweep": (C.c_int32, [_vp, C.c_uint32]),
    "lda_padded_topics": (C.c_int32, [C.c_int32]),
    "lda_get_shape": (C.c_int32, [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                  C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "lda_get_z": (C.c_int32, [_vp, _i32p]),
    "lda_set_z": (C.c_int32, [_vp, _i32p]),
    "lda_get_counts": (C.c_int32, [_vp, _vp, _vp, _vp, _vp]),
    "lda_set_alpha_beta": (C.c_int32, [_vp, _f64p, C.c_double]),
    "lda_log_likelihood_parts": (C.c_int32, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "lda_log_likelihood": (C.c_int32, [_vp, C.POINTER(C.c_double)]),
    "lda_log_likelihood_enqueue": (C.c_int32, [_vp, C.POINTER(C.c_int64)]),
    "lda_log_likelihood_collect": (C.c_int32, [_vp, C.c_int64, C.POINTER(C.c_double),
                                               C.POINTER(C.c_double)]),
    "lda_infer": (C.c_int32, [_vp, C.c_int64, _i64p, _i32p, C.c_int32, C.c_int32, C.c_int32,
                              C.c_uint64, _f64p]),
    "lda_to_mallet_packed": (C.c_int32, [_vp, _vp, _i64p, C.POINTER(C.c_int32)]),
    "lda_max_doc_length": (C.c_int32, [_vp, C.POINTER(C.c_int32)]),
    "lda_doc_topic_histograms": (C.c_int32, [_vp, C.c_int32, _i32p, _i32p]),
    "lda_doc_topic_histograms_accumulate": (C.c_int32, [_vp, C.c_int32]),
    "lda_doc_topic_histograms_take": (C.c_int32, [_vp, C.c_int32, _i32p, _i32p]),
    "lda_doc_topic_histograms_clear": (C.c_int32, [_vp]),
    "lda_count_histogram": (C.c_int32, [_vp, C.c_int64, _i32p]),
    "lda_hyper_statistics": (C.c_int32, [_vp, C.c_int32, _vp, _vp, C.c_int64, _vp, _vp]),
    "lda_learn_parameters": (C.c_int32, [_f64p, C.c_int32, _i32p, _i32p, C.c_int32, C.c_double,
                                         C.c_double, C.c_int32, C.POINTER(C.c_double)]),
    "lda_learn_symmetric_concentration": (C.c_int32, [_i32p, C.c_int64, _i64p, _i32p, C.c_int64,
                                                      C.c_int32, C.c_double,
                                                      C.POINTER(C.c_double)]),
    "lda_digamma": (C.c_double, [C.c_double]),
    "lda_last_sample_ms": (C.c_int32, [_vp, C.POINTER(C.c_float)]),
    "lda_row_stats": (C.c_int32, [_vp, C.POINTER(C.c_double)]),
    "lda_sample_times": (C.c_int32, [_vp, C.c_int32, _vp, C.POINTER(C.c_int32)]),
    "lda_philox_draws": (C.c_int32, [C.c_uint64, C.c_uint32, C.c_uint32, _vp, C.c_int64, _vp]),
    "lda_recount_times": (C.c_int32, [_vp, C.c_int32, _vp, C.POINTER(C.c_int32)]),
    "lda_count_update_mode": (C.c_int32, [_vp, C.POINTER(C.c_int32)]),
    "lda_set_count_update": (C.c_int32, [_vp, C.c_int32, C.c_int32]),
    "lda_set_warm_start": (C.c_int32, [_vp, C.c_int32, C.c_int32, C.c_int64, C.c_int64]),
    "lda_get_warm_start": (C.c_int32, [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "lda_exchange_sizes": (C.c_int32, [_vp, C.c_int32, C.c_int64, C.POINTER(C.c_size_t),
                                       C.POINTER(C.c_size_t)]),
    "lda_exchange_pack": (C.c_int32, [_vp, C.c_int32, C.c_int32, C.c_int64, C.POINTER(_vp),
                                      C.POINTER(_vp)]),
    "lda_exchange_unpack": (C.c_int32, [_vp, C.c_int32, C.c_int32, C.c_int64, _vp]),
    "lda_exchange_unpack_lists": (C.c_int32, [_vp, C.c_int32, C.c_int32, C.c_int64, _vp, C.c_int32]),
    "lda_set_exchange_cells": (C.c_int32, [_vp, C.c_int32]),
    "lda_get_exchange_cells": (C.c_int32, [_vp, C.POINTER(C.c_int32)]),
    "lda_counts_checksum": (C.c_int32, [_vp, C.POINTER(C.c_uint64)]),
    "lda_set_sequential_sweeps": (C.c_int32, [_vp, C.c_int32, _vp, C.c_int64, C.c_int64]),
    "lda_get_sequential_sweeps": (C.c_int32, [_vp, C.POINTER(C.c_int32), _vp]),
    "lda_staleness_schedule": (C.c_int32, [C.c_int32, C.POINTER(C.c_int32), _vp]),
    "lda_warm_part_tokens": (C.c_int32, [_vp, C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.c_int64, _vp]),
    "lda_sweep_parts": (C.c_int32, [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "lda_get_count_update": (C.c_int32, [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "lda_abi_version": (C.c_int32, []),
    "lda_debug_fail_host_alloc": (None, [C.c_int32]),
    "lda_last_error": (C.c_char_p, []),
    "lda_version": (C.c_char_p, []),
}

_lib = None


def load(path: str | None = None):
    """Load liblda_mi355x.so; raises if it is missing (no CPU fallback).
    LDA_MI355X_LIB overrides the in-tree path (A/B runs of kernel variants)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("LDA_MI355X_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64
    # (soname libamdhip64.so.7, loaded by path through its $ORIGIN rpath).
    # Importing torch first makes our NEEDED libamdhip64.so.7 resolve to that
    # already-loaded copy; loading /opt/rocm's copy first would leave torch's
    # runtime without devices ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int, where: str):
    if status != LDA_OK:
        msg = load().lda_last_error()
        raise LdaError(status, where, msg.decode() if msg else "")


def padded_topics(K: int) -> int:
    return int(load().lda_padded_topics(K))

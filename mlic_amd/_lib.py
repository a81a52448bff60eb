"""ctypes binding of libmlic_hip.so (C ABI in include/mlic_hip.h).

The library is built in-tree (`python -m mlic_amd.build` or __graft_entry__.build()).  There is no
fallback: if the shared object is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MLIC_HIP_LIB", os.path.join(_HERE, "libmlic_hip.so"))

_lock = threading.Lock()
_lib = None


class MlicError(RuntimeError):
    pass


def _sig(lib):
    p, i, i64, f, sz = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_size_t
    P = C.POINTER
    lib.mlic_last_error.restype = C.c_char_p
    lib.mlic_version.restype = C.c_char_p
    sigs = {
        "mlic_create": [C.c_char_p, i, P(C.c_char_p), P(p), P(i64), P(i), p, P(p)],
        "mlic_destroy": [p],
        "mlic_forward": [p, p, p, i, i, i, p, p, p, f],
        "mlic_forward_v": [p, p, p, i, i, i, p, p, p, p],
        "mlic_compress_v": [p, p, p, i, i, i, p],
        "mlic_decompress_v": [p, p, P(p), P(sz), P(p), P(sz), i, i, i, p, p],
        "mlic_set_entropy_tables": [p, p, p, p, i, i, p, p, p, i, i],
        "mlic_compress": [p, p, p, i, i, i, f],
        "mlic_encoded_size": [p, i, P(sz), P(sz)],
        "mlic_encoded_copy": [p, i, p, p],
        "mlic_encoded_streams": [p, i, P(i64), P(i64), p, p, p],
        "mlic_decompress": [p, p, P(p), P(sz), P(p), P(sz), i, i, i, p, f],
        "mlic_run_module": [p, p, C.c_char_p, i, p, p, i, i, i, i, p],
        "mlic_workspace_bytes": [p, P(sz), P(sz)],
        "mlic_local_attn_mask": [p, p, i, i],
        "mlic_set_profiling": [p, i],
        "mlic_set_lanes": [p, i],
        "mlic_set_priority_base": [p, i],
        "mlic_set_precision": [p, i],
        "mlic_set_synthesis_precision": [p, i],
        "mlic_set_poison": [p, i],
        "mlic_set_kernel_option": [C.c_char_p, i],
        "mlic_ab_families": [P(i)],
        "mlic_batch_stream": [p, i, i, p, sz, P(sz)],
        "mlic_decompress_batch_stream": [p, p, p, sz, P(p), P(sz), i, i, i, p, p],
        "mlic_range_fallbacks": [p, P(i64), P(i64), P(i64), i],
        "mlic_profile_layers": [p, p, sz, P(sz)],
        "mlic_bench_conv": [i, i, i, i, i, i, i, i, i, i, P(C.c_double), P(C.c_double)],
        "mlic_profile_read": [p, i, P(i64), P(C.c_double), P(C.c_double), P(C.c_double)],
        "mlic_profile_categories": [P(i)],
        "mlic_host_stats": [p, P(C.c_double), P(C.c_double), P(C.c_double), i],
        "mlic_profile_category_name": [i, p, sz],
        "mlic_conv_run": [p, i, p, p, p, p, i, i, i, i, i, i, i, i, p, p],
        "mlic_conv_choice": [i, i, i, i, i, i, i, i, P(i)],
        "mlic_dw_run": [p, p, p, p, p, i, i, i, i, i, i],
        "mlic_dwpw_run": [p, p, p, p, p, p, p, i, i, i, i, i, i, p],
        "mlic_local_attn_run": [p, i, p, p, p, p, i, i, i, i, f],
        "mlic_local_attn_packed_run": [p, p, p, p, p, i, i, i, f],
        "mlic_local_attn_packed_half_run": [p, p, p, p, p, i, i, i, f, i],
        "mlic_image_sq_err_u8": [p, p, p, i, i64, p],
        "mlic_neglog2_sum": [p, p, i, i64, p],
        "mlic_gaussian_likelihood": [p, p, p, p, i64, f, p],
        "mlic_scale_indexes": [p, p, i64, p, i, p],
        "mlic_encoded_bits": [p, i, P(C.c_double), P(C.c_double)],
        "mlic_pmf_to_quantized_cdf": [p, i, i, p],
        "mlic_rans_encode": [p, p, i64, p, p, p, i, i, p, sz, P(sz)],
        "mlic_rans_decode": [p, sz, p, i64, p, p, p, i, i, p],
        "mlic_rans_decode_narrow": [p, sz, p, i64, i, p, p, p, i, i, p, P(i)],
    }
    for name, args in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    return lib


def _check_build_record():
    """The in-tree library must be the build of the sources in the tree (mlic_amd/build.py record)."""
    import json
    from . import build as _build
    if os.environ.get("MLIC_HIP_LIB"):
        return  # an explicitly chosen library (A/B builds): the caller vouches for it
    rec_path = _build.RECORD
    if not os.path.exists(rec_path):
        raise MlicError(f"{rec_path} missing: rebuild with `python -m mlic_amd.build` (records the sources the "
                        f"library was built from)")
    with open(rec_path) as f:
        rec = json.load(f)
    if rec.get("sources_sha256") != _build.source_digest():
        raise MlicError("libmlic_hip.so was built from other sources than the ones in this tree (stale build): "
                        "rebuild with `python -m mlic_amd.build`")


def lib():
    """The loaded library (raises if it was not built, or was built from other sources)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise MlicError(f"libmlic_hip.so not found at {LIB_PATH}: build it with "
                                f"`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            _check_build_record()
            _lib = _sig(C.CDLL(LIB_PATH))
    return _lib


def poison() -> bool:
    """$MLIC_POISON=1 (test switch): the executor NaN-fills its workspace blocks on allocation and the
    Python layer NaN-fills the output tensors it hands to the library, so any element a kernel does
    not write, or any read of memory its producer never wrote, shows up as NaN."""
    return os.environ.get("MLIC_POISON", "0") not in ("", "0")


def ab_families() -> bool:
    """True when the loaded library holds the A/B-only kernel families (make AB=1)."""
    v = C.c_int()
    call("mlic_ab_families", C.byref(v))
    return bool(v.value)


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().mlic_last_error().decode(errors="replace")
        raise MlicError(f"{what}: {msg}" if what else msg)


def call(name: str, *args):
    check(getattr(lib(), name)(*args), name)

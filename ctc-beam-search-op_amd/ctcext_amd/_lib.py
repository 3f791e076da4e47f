"""ctypes binding of libctcext.so (the C ABI declared in include/ctcext.h).

This is the Python-side FFI a maintainer of the reference would add in place
of ``load_library.load_op_library('_ctc_ext_beam_search_decoder_ops.so')``
(python/ops/ctc_ext_beam_search_decoder_ops.py:10-11).  The library is built
in-tree by ``__graft_entry__.build()`` (or ``make -C ctc-beam-search-op_amd/csrc``);
there is no fallback: if it is missing or cannot run, calls fail loudly.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CTCEXT_LIB_PATH") or os.path.join(_HERE, "lib", "libctcext.so")   # override: diagnostics builds

CTCEXT_OK = 0
CTCEXT_INVALID_ARGUMENT = 3
CTCEXT_FAILED_PRECONDITION = 9
CTCEXT_UNIMPLEMENTED = 12
CTCEXT_INTERNAL = 13
CTCEXT_F32 = 0
CTCEXT_F64 = 1
CTCEXT_FLAG_FORCE_LITERAL = 1
CTCEXT_FLAG_PROFILE = 2
CTCEXT_FLAG_PHASES = 4
CTCEXT_FLAG_GLOBAL_STATE = 8   # testing: the global-state tier whatever the shape
CTCEXT_FLAG_RECORD_RING = 16   # beam records kept in an LDS ring; only the reachable ones written to HBM
CTCEXT_FLAG_RING_MIN = 32      # testing: the record ring at 8 frames (short items flush); implies RECORD_RING
CTCEXT_FLAG_NO_RING = 64       # every beam record to HBM (the ring is the default for the score-table kernel)
CTCEXT_FLAG_HELPER_STRICT = 128     # a helper hand-over timeout fails the call instead of a one-wave re-decode
CTCEXT_FLAG_TEST_HELPER_DEAD = 256  # testing: the helper wave starts out timed out
CTCEXT_ABI_VERSION = 6
CTCEXT_SCORER_BASE = 0
CTCEXT_SCORER_BIGRAM = 1

# every symbol include/ctcext.h declares
EXPORTED_SYMBOLS = ("ctcext_create", "ctcext_create_sharded", "ctcext_destroy", "ctcext_validate",
                    "ctcext_decode", "ctcext_decode_sharded", "ctcext_fetch", "ctcext_get_stats",
                    "ctcext_last_error", "ctcext_max_beam_width", "ctcext_phase_counters", "ctcext_row_facts",
                    "ctcext_get_stats_sized", "ctcext_abi_version")


class DecodeArgs(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("inputs_on_device", ctypes.c_int32),
                ("inputs", ctypes.c_void_p), ("sequence_length", ctypes.c_void_p),
                ("max_time", ctypes.c_int64), ("batch_size", ctypes.c_int64),
                ("num_classes", ctypes.c_int64),
                ("beam_width", ctypes.c_int32), ("top_paths", ctypes.c_int32),
                ("merge_repeated", ctypes.c_int32), ("blank_index", ctypes.c_int32),
                ("blank_label", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("stream", ctypes.c_void_p),
                ("inputs_dims", ctypes.c_int32), ("sequence_length_dims", ctypes.c_int32),
                ("sequence_length_size", ctypes.c_int64),
                ("scorer", ctypes.c_int32), ("pad_", ctypes.c_int32), ("scorer_table", ctypes.c_void_p)]


class PathSizes(ctypes.Structure):
    _fields_ = [("num_decoded", ctypes.c_int64), ("max_decoded", ctypes.c_int64),
                ("num_alignment", ctypes.c_int64), ("max_alignment", ctypes.c_int64)]


class Outputs(ctypes.Structure):
    _fields_ = [("outputs_on_device", ctypes.c_int32),
                ("decoded_indices", ctypes.POINTER(ctypes.c_void_p)),
                ("decoded_values", ctypes.POINTER(ctypes.c_void_p)),
                ("decoded_shape", ctypes.POINTER(ctypes.c_void_p)),
                ("alignment_indices", ctypes.POINTER(ctypes.c_void_p)),
                ("alignment_values", ctypes.POINTER(ctypes.c_void_p)),
                ("alignment_shape", ctypes.POINTER(ctypes.c_void_p)),
                ("log_probability", ctypes.c_void_p)]


class Stats(ctypes.Structure):
    _fields_ = [("literal_frames", ctypes.c_int64), ("literal_nonfinite", ctypes.c_int64),
                ("literal_fill", ctypes.c_int64), ("duplicate_frames", ctypes.c_int64),
                ("no_label_paths", ctypes.c_int64),
                ("decode_kernel_ms", ctypes.c_double), ("norm_kernel_ms", ctypes.c_double),
                ("traceback_ms", ctypes.c_double), ("n_devices", ctypes.c_int32),
                ("tier", ctypes.c_int32), ("ring_frames", ctypes.c_int32),
                ("records_written", ctypes.c_int64), ("record_bytes", ctypes.c_int32),
                ("helper", ctypes.c_int32), ("helper_redecodes", ctypes.c_int32), ("pad_", ctypes.c_int32)]


_lib = None


def load():
    """Load libctcext.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError("libctcext.so not found at %s: run __graft_entry__.build() or "
                      "make -C ctc-beam-search-op_amd/csrc" % LIB_PATH)
    # PyTorch-ROCm wheels bundle their own libamdhip64.so.7 / libhsa-runtime64.so.1.
    # Two HIP runtimes in one process cannot share the GPU (whichever opens it
    # first wins).  Importing torch first maps its copies; libctcext.so's
    # NEEDED entries then bind to them by SONAME, so the process has one runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    lib.ctcext_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    lib.ctcext_create.restype = ctypes.c_int
    lib.ctcext_create_sharded.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    lib.ctcext_create_sharded.restype = ctypes.c_int
    lib.ctcext_validate.argtypes = [ctypes.POINTER(DecodeArgs)]
    lib.ctcext_validate.restype = ctypes.c_int
    lib.ctcext_decode_sharded.argtypes = [ctypes.c_void_p, ctypes.POINTER(DecodeArgs), ctypes.POINTER(PathSizes)]
    lib.ctcext_decode_sharded.restype = ctypes.c_int
    lib.ctcext_destroy.argtypes = [ctypes.c_void_p]
    lib.ctcext_destroy.restype = None
    lib.ctcext_decode.argtypes = [ctypes.c_void_p, ctypes.POINTER(DecodeArgs), ctypes.POINTER(PathSizes)]
    lib.ctcext_decode.restype = ctypes.c_int
    lib.ctcext_fetch.argtypes = [ctypes.c_void_p, ctypes.POINTER(Outputs)]
    lib.ctcext_fetch.restype = ctypes.c_int
    lib.ctcext_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(Stats)]
    lib.ctcext_get_stats.restype = ctypes.c_int
    if hasattr(lib, "ctcext_get_stats_sized"):   # (ABI 5; older builds stay loadable for A/B runs)
        lib.ctcext_get_stats_sized.argtypes = [ctypes.c_void_p, ctypes.POINTER(Stats), ctypes.c_size_t]
        lib.ctcext_get_stats_sized.restype = ctypes.c_int
        lib.ctcext_abi_version.argtypes = []
        lib.ctcext_abi_version.restype = ctypes.c_int32
    lib.ctcext_last_error.argtypes = []
    lib.ctcext_last_error.restype = ctypes.c_char_p
    lib.ctcext_max_beam_width.argtypes = [ctypes.c_int64, ctypes.c_int32]
    lib.ctcext_max_beam_width.restype = ctypes.c_int32
    lib.ctcext_phase_counters.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    lib.ctcext_phase_counters.restype = ctypes.c_int
    if hasattr(lib, "ctcext_row_facts"):   # (diagnostics; absent from builds before it, kept loadable for A/B)
        lib.ctcext_row_facts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        lib.ctcext_row_facts.restype = ctypes.c_int
    _lib = lib
    return lib


def get_stats(lib, handle, st):
    """Fill Stats st from the last decode on handle (only the prefix an older build knows)."""
    if hasattr(lib, "ctcext_get_stats_sized"):
        return lib.ctcext_get_stats_sized(handle, ctypes.byref(st), ctypes.sizeof(st))
    return lib.ctcext_get_stats(handle, ctypes.byref(st))

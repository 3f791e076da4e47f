"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product (ctc-beam-search-op_amd/ctcext_amd) never does.

``decode`` mirrors the reference op end to end: input validation
(kernels.cc:97-139), the sequential batch driver (kernels.cc:67-90) and the
SparseTensor packing of StoreAllDecodedSequences (kernels.cc:163-257), and
returns the same 7-field structure as the generated TF op
(``python/ops/ctc_ext_beam_search_decoder_ops.py:12``).
"""
import collections
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libctc_oracle.so")

OracleOutput = collections.namedtuple(
    "OracleOutput",
    ["decoded_indices", "decoded_values", "decoded_shape",
     "alignment_indices", "alignment_values", "alignment_shape",
     "log_probability"])


class OracleError(Exception):
    """Raised with the reference's status message verbatim."""


class _Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("no_label_events", ctypes.c_int32),
                ("total_dec", ctypes.c_int64), ("total_ali", ctypes.c_int64),
                ("dec_len", ctypes.POINTER(ctypes.c_int64)),
                ("ali_len", ctypes.POINTER(ctypes.c_int64)),
                ("dec_vals", ctypes.POINTER(ctypes.c_int32)),
                ("ali_vals", ctypes.POINTER(ctypes.c_int32)),
                ("log_prob", ctypes.POINTER(ctypes.c_double)),
                ("dup_frames", ctypes.c_int64),
                ("reclaims", ctypes.c_int64)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        lib.oracle_decode.restype = ctypes.POINTER(_Result)
        lib.oracle_decode.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.oracle_decode_scored.restype = ctypes.POINTER(_Result)
        lib.oracle_decode_scored.argtypes = lib.oracle_decode.argtypes + [ctypes.c_void_p]
        lib.oracle_decode_ex.restype = ctypes.POINTER(_Result)
        lib.oracle_decode_ex.argtypes = lib.oracle_decode_scored.argtypes + [ctypes.c_int, ctypes.c_int64]
        lib.oracle_free.argtypes = [ctypes.POINTER(_Result)]
        lib.oracle_row_norm.restype = None
        lib.oracle_row_norm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_void_p]
        _lib = lib
    return _lib


def row_norm(rows):
    """The softmax normaliser of each row of a [rows, C] float32/float64 array
    (ctc_ext_beam_search_decoder.h:72-80, ctc_oracle.cpp row_normaliser)."""
    x = np.ascontiguousarray(rows)
    assert x.ndim == 2 and x.dtype in (np.float32, np.float64)
    out = np.empty(x.shape[0], x.dtype)
    _load().oracle_row_norm(0 if x.dtype == np.float32 else 1, x.ctypes.data, x.shape[0], x.shape[1],
                            out.ctypes.data)
    return out


def raw_decode(inputs, sequence_length, beam_width, top_paths, merge_repeated=False,
               blank_index=0, blank_label=-1, mode="shared", stats=None, scorer_table=None,
               gc_threshold=0):
    """Returns (dec, ali, log_prob, no_label_events) with dec[b][p] / ali[b][p]
    python lists of ints and log_prob float64 [B, P].  ``stats`` (a dict), if
    given, receives ``duplicate_frames``: frames that started with one entry
    twice in the beam, and ``reclaims``: shared-mode node reclamation passes.
    ``scorer_table`` ([C + 1, C], the inputs' dtype): the bigram beam scorer
    (see ctc_oracle.cpp); None is the reference op's BaseBeamScorer.
    ``gc_threshold``: shared-mode node count that triggers reclamation (0: the
    library default; 1 reclaims every frame, for the tests)."""
    x = np.ascontiguousarray(inputs)
    if x.dtype not in (np.float32, np.float64):
        raise TypeError("inputs must be float32 or float64")
    if x.ndim != 3:
        raise OracleError("inputs is not a 3-Tensor")
    T, B, C = x.shape
    if T == 0:
        raise OracleError("max_time is 0")
    sl = np.ascontiguousarray(np.asarray(sequence_length, dtype=np.int32))
    if sl.ndim != 1:
        raise OracleError("sequence_length is not a vector")
    if sl.shape[0] != B:
        raise OracleError("len(sequence_length) != batch_size.  len(sequence_length):  %d batch_size: %d"
                          % (sl.shape[0], B))
    for b in range(B):
        if not sl[b] <= T:
            raise OracleError("sequence_length(%d) <= %d" % (b, T))
    if not 0 <= blank_index < C:
        raise OracleError("blank_index out of range")
    lib = _load()
    tab = None
    if scorer_table is not None:
        tab = np.ascontiguousarray(np.asarray(scorer_table, dtype=x.dtype))
        if tab.shape != (C + 1, C):
            raise ValueError("scorer_table must be [num_classes + 1, num_classes]")
    r = lib.oracle_decode_ex(0 if x.dtype == np.float32 else 1, 0 if mode == "faithful" else 1,
                             x.ctypes.data, sl.ctypes.data, T, B, C, int(beam_width),
                             int(top_paths), int(bool(merge_repeated)), int(blank_index),
                             int(blank_label), None if tab is None else tab.ctypes.data,
                             1 if stats is not None else 0, int(gc_threshold))
    try:
        res = r.contents
        if stats is not None:
            stats["duplicate_frames"] = int(res.dup_frames)
            stats["reclaims"] = int(res.reclaims)
        if res.status == 1:
            raise OracleError("requested more paths than the beam width.")
        if res.status == 2:
            raise OracleError("Less leaves in the beam search than requested.")
        P = int(top_paths)
        n = B * P
        dl = np.ctypeslib.as_array(res.dec_len, (n + 1,))[:n].copy()
        al = np.ctypeslib.as_array(res.ali_len, (n + 1,))[:n].copy()
        dv = np.ctypeslib.as_array(res.dec_vals, (int(res.total_dec) + 1,))[:res.total_dec].copy()
        av = np.ctypeslib.as_array(res.ali_vals, (int(res.total_ali) + 1,))[:res.total_ali].copy()
        lp = np.ctypeslib.as_array(res.log_prob, (n + 1,))[:n].copy().reshape(B, P)
        events = int(res.no_label_events)
    finally:
        lib.oracle_free(r)
    dec, ali = [], []
    od = oa = 0
    for b in range(B):
        db, ab = [], []
        for p in range(P):
            i = b * P + p
            db.append(dv[od:od + dl[i]].tolist()); od += dl[i]
            ab.append(av[oa:oa + al[i]].tolist()); oa += al[i]
        dec.append(db)
        ali.append(ab)
    return dec, ali, lp.astype(x.dtype), events


def pack_sparse(seqs, B, P):
    """StoreAllDecodedSequences (kernels.cc:163-257) for one kind of sequence:
    per path p -> (indices int64 [n,2], values int64 [n], shape int64 [2])."""
    idx_l, val_l, shp_l = [], [], []
    for p in range(P):
        rows, cols, vals = [], [], []
        mx = 0
        for b in range(B):
            s = seqs[b][p]
            mx = max(mx, len(s))
            rows.extend([b] * len(s))
            cols.extend(range(len(s)))
            vals.extend(s)
        idx = np.stack([np.asarray(rows, dtype=np.int64), np.asarray(cols, dtype=np.int64)], axis=1) \
            if rows else np.zeros((0, 2), dtype=np.int64)
        idx_l.append(idx.reshape(-1, 2))
        val_l.append(np.asarray(vals, dtype=np.int64))
        shp_l.append(np.asarray([B, mx], dtype=np.int64))
    return idx_l, val_l, shp_l


def decode(inputs, sequence_length, beam_width, top_paths, merge_repeated=False,
           blank_index=0, blank_label=-1, mode="shared", stats=None, scorer_table=None,
           gc_threshold=0):
    dec, ali, lp, _ = raw_decode(inputs, sequence_length, beam_width, top_paths,
                                 merge_repeated, blank_index, blank_label, mode, stats, scorer_table,
                                 gc_threshold)
    B = np.asarray(inputs).shape[1]
    di, dv, ds = pack_sparse(dec, B, top_paths)
    ai, av, ash = pack_sparse(ali, B, top_paths)
    return OracleOutput(di, dv, ds, ai, av, ash, lp)

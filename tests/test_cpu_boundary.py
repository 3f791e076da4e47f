"""CPU-side checks of the drop-in boundary (no GPU needed, no compute calls):

* libctcext.so loads and exports every function include/ctcext.h declares;
* the reference's validation (ops.cc:12-13 attr minimums, kernels.cc:111-139
  shape and length checks) runs behind the C ABI (ctcext_validate), with the
  reference's messages in its order, before any device work -- both called
  directly through ctypes and through the Python op;
* without a GPU the op fails loudly (no silent CPU fallback);
* the batch-sharded path (ctcext_amd.sharded) reassembles per-rank outputs
  into the single-device result: world_size 2 over gloo, with the oracle
  standing in for each rank's decoder.
"""
import ctypes
import os
import re
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

import ctcext_amd
from ctcext_amd import _lib
from ctcext_amd.sharded import gather_to_root, shard_bounds
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ctcext.h")


def _header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ctcext_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    declared = _header_functions()
    assert declared, "no functions parsed from include/ctcext.h"
    assert sorted(_lib.EXPORTED_SYMBOLS) == declared
    for name in declared:
        assert hasattr(lib, name), name
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_abi_structs_match_header(tmp_path):
    """The ctypes mirrors of ctcext_stats / ctcext_decode_args have the C
    header's size and field offsets (gcc on include/ctcext.h), and the library
    reports the header's ABI version."""
    import subprocess
    src = tmp_path / "abi.c"
    fields = {"ctcext_stats": _lib.Stats, "ctcext_decode_args": _lib.DecodeArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ctcext.h"', "int main(void) {"]
    for cname, py in fields.items():
        lines.append('printf("%%s size %%zu\\n", "%s", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%%s %%s %%zu\\n", "%s", "%s", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append('printf("abi %d\\n", CTCEXT_ABI_VERSION); return 0; }')
    src.write_text("\n".join(lines))
    exe = tmp_path / "abi"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)])
    got = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, py in fields.items():
        assert int(got["%s size" % cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got["%s %s" % (cname, f)]) == getattr(py, f).offset, (cname, f)
    assert int(got["abi"]) == _lib.CTCEXT_ABI_VERSION == _lib.load().ctcext_abi_version()


def test_every_shape_validates():
    # no shape limit of its own below the 32-bit indices: num_classes above the
    # 8-byte record (65535) and beams past the LDS tier validate (they decode
    # on the global-state tier)
    lib = _lib.load()
    for shape, W in (((3, 1, 70000), 8), ((3, 1, 29), 2048), ((3, 1, 200000), 600)):
        a, keep = _args(shape, [3], W=W)
        assert lib.ctcext_validate(ctypes.byref(a)) == _lib.CTCEXT_OK, lib.ctcext_last_error()
    assert lib.ctcext_max_beam_width(70000, _lib.CTCEXT_F32) == 0   # past the fast tier


def test_max_beam_width_is_host_only_and_monotone():
    lib = _lib.load()
    w29 = lib.ctcext_max_beam_width(29, _lib.CTCEXT_F32)
    assert w29 >= 256          # cfg3/cfg5 beam widths fit the LDS-resident state
    assert lib.ctcext_max_beam_width(29, _lib.CTCEXT_F64) <= w29
    assert lib.ctcext_max_beam_width(5000, _lib.CTCEXT_F32) <= w29


@pytest.mark.parametrize("bw,tp,msg", [
    (0, 1, "Value for attr 'beam_width' of 0 must be at least minimum 1"),
    (4, 0, "Value for attr 'top_paths' of 0 must be at least minimum 1"),
])
def test_attr_minimums(bw, tp, msg):
    x = np.zeros((3, 1, 4), np.float32)
    with pytest.raises(ctcext_amd.InvalidArgumentError) as e:
        ctcext_amd.ctc_ext_beam_search_decoder(x, [3], bw, tp)
    assert e.value.message == msg


def test_shape_errors_before_device_work():
    with pytest.raises(ctcext_amd.InvalidArgumentError) as e:
        ctcext_amd.ctc_ext_beam_search_decoder(np.zeros((3, 4), np.float32), [3], 2, 1)
    assert e.value.message == "inputs is not a 3-Tensor"
    with pytest.raises(ctcext_amd.InvalidArgumentError) as e:
        ctcext_amd.ctc_ext_beam_search_decoder(np.zeros((3, 1, 4), np.float32), [[3]], 2, 1)
    assert e.value.message == "sequence_length is not a vector"
    with pytest.raises(ctcext_amd.InvalidArgumentError) as e:
        ctcext_amd.ctc_ext_beam_search_decoder(np.zeros((0, 1, 4), np.float32), [0], 2, 1)
    assert e.value.message == "max_time is 0"
    with pytest.raises(ctcext_amd.FailedPreconditionError) as e:
        ctcext_amd.ctc_ext_beam_search_decoder(np.zeros((3, 2, 4), np.float32), [3], 2, 1)
    assert e.value.message == "len(sequence_length) != batch_size.  len(sequence_length):  1 batch_size: 2"


def _args(shape, sl, dims=None, sl_dims=1, sl_size=None, W=4, P=1, blank=0, dtype=_lib.CTCEXT_F32):
    a = _lib.DecodeArgs()
    a.dtype = dtype
    a.inputs_on_device = 0
    buf = (ctypes.c_float * 8)()
    a.inputs = ctypes.cast(buf, ctypes.c_void_p)
    sla = (ctypes.c_int32 * max(len(sl), 1))(*sl)
    a.sequence_length = ctypes.cast(sla, ctypes.c_void_p)
    d = list(shape) + [0, 0, 0]
    a.max_time, a.batch_size, a.num_classes = d[0], d[1], d[2]
    a.inputs_dims = len(shape) if dims is None else dims
    a.sequence_length_dims = sl_dims
    a.sequence_length_size = len(sl) if sl_size is None else sl_size
    a.beam_width, a.top_paths, a.blank_index, a.blank_label = W, P, blank, -1
    return a, (buf, sla)


@pytest.mark.parametrize("kw,code,msg", [
    # kernels.cc:111-113, 118-120, 122-124, 126-130, 134-139, in that order
    (dict(shape=(3, 4), sl=[3]), _lib.CTCEXT_INVALID_ARGUMENT, "inputs is not a 3-Tensor"),
    (dict(shape=(3, 4, 5, 6), sl=[3, 3, 3, 3]), _lib.CTCEXT_INVALID_ARGUMENT, "inputs is not a 3-Tensor"),
    (dict(shape=(0, 1, 4), sl=[0], sl_dims=2), _lib.CTCEXT_INVALID_ARGUMENT, "max_time is 0"),
    (dict(shape=(3, 1, 4), sl=[3], sl_dims=2), _lib.CTCEXT_INVALID_ARGUMENT, "sequence_length is not a vector"),
    (dict(shape=(3, 1, 4), sl=[3], sl_dims=0), _lib.CTCEXT_INVALID_ARGUMENT, "sequence_length is not a vector"),
    (dict(shape=(3, 2, 4), sl=[3]), _lib.CTCEXT_FAILED_PRECONDITION,
     "len(sequence_length) != batch_size.  len(sequence_length):  1 batch_size: 2"),
    (dict(shape=(3, 2, 4), sl=[3, 3, 3]), _lib.CTCEXT_FAILED_PRECONDITION,
     "len(sequence_length) != batch_size.  len(sequence_length):  3 batch_size: 2"),
    (dict(shape=(3, 2, 4), sl=[3, 4]), _lib.CTCEXT_FAILED_PRECONDITION, "sequence_length(1) <= 3"),
    # attr minimums (ops.cc:12-13), then this library's checks
    (dict(shape=(3, 1, 4), sl=[3], W=0), _lib.CTCEXT_INVALID_ARGUMENT,
     "Value for attr 'beam_width' of 0 must be at least minimum 1"),
    (dict(shape=(3, 1, 4), sl=[3], P=0), _lib.CTCEXT_INVALID_ARGUMENT,
     "Value for attr 'top_paths' of 0 must be at least minimum 1"),
    (dict(shape=(3, 1, 4), sl=[3], W=2, P=3), _lib.CTCEXT_INVALID_ARGUMENT,
     "requested more paths than the beam width."),
    (dict(shape=(3, 1, 4), sl=[3], blank=4), _lib.CTCEXT_INVALID_ARGUMENT,
     "blank_index out of range [0, num_classes)"),
    (dict(shape=(3, 1, 1 << 30), sl=[3]), _lib.CTCEXT_UNIMPLEMENTED,
     "num_classes or beam_width beyond this library's 32-bit indices"),
    (dict(shape=(3, 1, 4), sl=[3], dtype=7), _lib.CTCEXT_INVALID_ARGUMENT, "dtype must be float32 or float64"),
])
def test_c_abi_validation(kw, code, msg):
    # the reference's checks behind the C ABI, no GPU and no handle needed
    lib = _lib.load()
    a, keep = _args(**kw)
    assert lib.ctcext_validate(ctypes.byref(a)) == code
    assert lib.ctcext_last_error().decode() == msg
    del keep


def test_c_abi_validation_order_and_ok():
    lib = _lib.load()
    # rank is checked before everything else, length before the values
    a, keep = _args((3, 4), [9, 9], sl_dims=2)
    assert lib.ctcext_validate(ctypes.byref(a)) == _lib.CTCEXT_INVALID_ARGUMENT
    assert lib.ctcext_last_error().decode() == "inputs is not a 3-Tensor"
    a, keep = _args((3, 2, 4), [9])
    assert lib.ctcext_validate(ctypes.byref(a)) == _lib.CTCEXT_FAILED_PRECONDITION
    a, keep = _args((3, 2, 4), [3, 0])
    assert lib.ctcext_validate(ctypes.byref(a)) == _lib.CTCEXT_OK
    assert lib.ctcext_last_error().decode() == ""
    # an empty batch is valid (no item reaches TopPaths)
    a, keep = _args((3, 0, 4), [], W=1, P=5)
    assert lib.ctcext_validate(ctypes.byref(a)) == _lib.CTCEXT_OK
    del keep


def test_unsupported_dtypes_raise_type_error():
    # the op registers T in {float, double} only (ops.cc:17-18)
    with pytest.raises(TypeError, match="DataType int32 not in list of allowed values: float32, float64"):
        ctcext_amd.ctc_ext_beam_search_decoder(np.zeros((3, 1, 4), np.int32), [3], 2, 1)
    with pytest.raises(TypeError, match="float16"):
        ctcext_amd.ctc_ext_beam_search_decoder(np.zeros((3, 1, 4), np.float16), [3], 2, 1)
    with pytest.raises(TypeError, match="sequence_length"):
        ctcext_amd.ctc_ext_beam_search_decoder(np.zeros((3, 1, 4), np.float32), [3.0], 2, 1)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly():
    x = np.zeros((3, 1, 4), np.float32)
    with pytest.raises(ctcext_amd.OpError):
        ctcext_amd.ctc_ext_beam_search_decoder(x, [3], 2, 1)


def test_shard_bounds_cover_batch():
    for B in (0, 1, 7, 256, 1024):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(B, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _as_torch(o):
    t = lambda a: torch.as_tensor(np.asarray(a))
    return ctcext_amd.CTCExtBeamSearchDecoder([t(a) for a in o.decoded_indices], [t(a) for a in o.decoded_values],
                                              [t(a) for a in o.decoded_shape], [t(a) for a in o.alignment_indices],
                                              [t(a) for a in o.alignment_values], [t(a) for a in o.alignment_shape],
                                              t(o.log_probability))


def _rank_main(rank, world, port, x, sl, W, P, kw, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_bounds(x.shape[1], rank, world)
    part = oracle.decode(x[:, lo:hi], sl[lo:hi], W, P, **kw)
    got = gather_to_root(_as_torch(part), lo, P)
    if rank == 0:
        arrs = {"log_probability": got.log_probability.numpy()}
        for k in got._fields[:-1]:
            arrs.update({"%s_%d" % (k, p): v.numpy() for p, v in enumerate(getattr(got, k))})
        np.savez(path, **arrs)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B", [5, 2])
def test_sharded_gather_gloo_world2(tmp_path, B):
    rng = np.random.default_rng(B)
    T, C, W, P = 12, 5, 4, 2
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = rng.integers(1, T + 1, size=B).astype(np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    path = str(tmp_path / "gathered.npz")
    tmp.spawn(_rank_main, args=(2, _free_port(), x, sl, W, P, kw, path), nprocs=2, join=True)
    got = np.load(path)
    ref = oracle.decode(x, sl, W, P, **kw)
    for f in ("decoded_indices", "decoded_values", "decoded_shape",
              "alignment_indices", "alignment_values", "alignment_shape"):
        for p in range(P):
            np.testing.assert_array_equal(got["%s_%d" % (f, p)], np.asarray(getattr(ref, f)[p]),
                                          err_msg="%s[%d]" % (f, p))
    np.testing.assert_array_equal(got["log_probability"], np.asarray(ref.log_probability))

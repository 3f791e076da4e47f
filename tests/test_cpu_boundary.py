"""CPU-side checks of the drop-in boundary (no GPU needed, no compute calls):

* libctcext.so loads and exports every function include/ctcext.h declares;
* the host-side validation of ctc_ext_beam_search_decoder raises the
  reference's errors (ops.cc:12-13 attr minimums, kernels.cc:111-139 shape
  checks) before any device work;
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

"""Multi-device paths on the GPU (kernels.cc:68-90's batch loop split across
devices).

* ctcext_create_sharded (one process, several devices, peer-copy gather to
  the root) must give exactly the one-device outputs and the oracle's.  The
  box has one GPU, so the device list names it twice: the shards then run on
  two streams of the same GPU, which exercises the split, the strided input
  copies and the gather, not xGMI.
* one process per GPU (ctcext_amd.sharded.gather_to_root): two ranks started
  by torch.distributed.run as a child process (never an exec of this
  GPU-initialised process), each decoding its shard with the HIP decoder on
  cuda:0 and gathering over gloo (RCCL refuses two ranks on one device); rank 0
  writes the gathered outputs, compared here with the one-device decode.
* every entry point restores the caller's current device.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import ctcext_amd
import oracle
from parity_util import compare, to_numpy

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _same(a, b, P):
    for p in range(P):
        for k in a._fields[:-1]:
            np.testing.assert_array_equal(to_numpy(getattr(a, k)[p]), to_numpy(getattr(b, k)[p]),
                                          err_msg="%s[%d]" % (k, p))
    np.testing.assert_array_equal(to_numpy(a.log_probability), to_numpy(b.log_probability))


@pytest.mark.parametrize("B,device_in,ragged", [(5, True, True), (5, False, True), (1, True, False),
                                                (4, True, False), (7, False, False)])
def test_sharded_handle_matches_single_device(B, device_in, ragged):
    rng = np.random.default_rng(100 + B)
    T, C, W, P = 120, 29, 32, 2
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = (rng.integers(0, T + 1, size=B) if ragged else np.full(B, T)).astype(np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    xin = torch.as_tensor(x, device="cuda:0") if device_in else x
    slin = torch.as_tensor(sl, device="cuda:0") if device_in else sl
    one = ctcext_amd.ctc_ext_beam_search_decoder(xin, slin, W, P, **kw)
    for devs in ([0, 0], [0, 0, 0]):
        many = ctcext_amd.ctc_ext_beam_search_decoder(xin, slin, W, P, devices=devs, **kw)
        assert ctcext_amd.get_decoder(tuple(devs)).last_stats["n_devices"] == len(devs)
        _same(many, one, P)
    compare(one, oracle.decode(x, sl, W, P, **kw), P)


def test_sharded_handle_large_c_and_f64():
    rng = np.random.default_rng(7)
    x = rng.standard_normal((40, 6, 300))
    sl = np.array([40, 12, 1, 40, 33, 1], np.int32)
    kw = dict(merge_repeated=False, blank_index=5, blank_label=-1)
    one = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, 16, 3, **kw)
    many = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, 16, 3, devices=[0, 0, 0, 0], **kw)
    _same(many, one, 3)
    compare(one, oracle.decode(x, sl, 16, 3, **kw), 3)
    # zero-length items (top_paths 1: the root is the only leaf) in some shards
    sl0 = np.array([40, 0, 0, 40, 0, 7], np.int32)
    one = ctcext_amd.ctc_ext_beam_search_decoder(x, sl0, 16, 1, **kw)
    many = ctcext_amd.ctc_ext_beam_search_decoder(x, sl0, 16, 1, devices=[0, 0, 0, 0], **kw)
    _same(many, one, 1)
    compare(one, oracle.decode(x, sl0, 16, 1, **kw), 1)


def test_sharded_handle_errors_match():
    x = np.random.default_rng(0).standard_normal((5, 3, 4)).astype(np.float32)
    for devs in (None, [0, 0]):
        with pytest.raises(ctcext_amd.InvalidArgumentError) as e:
            ctcext_amd.ctc_ext_beam_search_decoder(x[:1], [1, 1, 1], 10, 5, devices=devs)
        assert e.value.message == "Less leaves in the beam search than requested."
        with pytest.raises(ctcext_amd.FailedPreconditionError) as e:
            ctcext_amd.ctc_ext_beam_search_decoder(x, [6, 1, 1], 4, 1, devices=devs)
        assert e.value.message == "sequence_length(0) <= 5"


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs: on one GPU the current "
                    "device and the library's device coincide, so restoration is not observable")
def test_current_device_is_restored():
    # the C ABI saves and restores the caller's HIP device (torch reads the
    # same runtime's current device)
    n = torch.cuda.device_count()
    x = np.random.default_rng(0).standard_normal((10, 2, 5)).astype(np.float32)
    for cur in range(min(n, 2)):
        torch.cuda.set_device(cur)
        ctcext_amd.ctc_ext_beam_search_decoder(torch.as_tensor(x, device="cuda:0"), [10, 10], 4, 1)
        assert torch.cuda.current_device() == cur
        ctcext_amd.ctc_ext_beam_search_decoder(x, [10, 10], 4, 1, devices=[0, 0])
        assert torch.cuda.current_device() == cur
    torch.cuda.set_device(0)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (the cross-device xGMI path: "
                    "peer access, strided shard copies out of the root's memory, peer-copy gather)")
def test_sharded_handle_two_distinct_devices():
    rng = np.random.default_rng(2)
    x = rng.standard_normal((80, 9, 29)).astype(np.float32)
    sl = rng.integers(0, 81, size=9).astype(np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    one = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, 32, 2, **kw)
    for xin, slin in ((x, sl), (torch.as_tensor(x, device="cuda:0"), torch.as_tensor(sl, device="cuda:0"))):
        many = ctcext_amd.ctc_ext_beam_search_decoder(xin, slin, 32, 2, devices=[0, 1], **kw)
        _same(many, one, 2)


@pytest.mark.parametrize("device_in", [False, True])
def test_sharded_root_shard_empty(device_in):
    # B < n_devices with every length <= 0: the split by count gives the root
    # no items; its input copies are skipped (ctcext_capi.hip run_decode)
    x = np.random.default_rng(3).standard_normal((4, 1, 6)).astype(np.float32)
    sl = np.array([0], np.int32)
    xin = torch.as_tensor(x, device="cuda:0") if device_in else x
    slin = torch.as_tensor(sl, device="cuda:0") if device_in else sl
    one = ctcext_amd.ctc_ext_beam_search_decoder(xin, slin, 4, 1)
    many = ctcext_amd.ctc_ext_beam_search_decoder(xin, slin, 4, 1, devices=[0, 0])
    _same(many, one, 1)
    compare(one, oracle.decode(x, sl, 4, 1), 1)


def test_cfg4_whole_workload_eight_shards():
    """BASELINE.json cfg4 as one call: B=1024, T=2000, C=1000 (BPE vocab),
    beam_width=64 -- kernels.cc:68-90's batch loop over the whole global batch
    -- through the sharded handle with eight shards (devices=[0]*8: eight
    streams and workspaces on the one GPU of this box, the strided shard
    copies and the peer-copy gather path; xGMI itself needs eight GPUs).
    Checks: bit-identical to the one-device call; the full_length.json cfg4
    items (oracle outputs at T=2000) placed at known batch positions -- across
    the shard boundary at 127/128 and in the last shard -- come back
    bit-exact; and the size-independent properties of test_gpu_properties."""
    import json
    from test_gpu_properties import _check_structure, _rows
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_fixtures_full
    B, T, C, W, P = 1024, 2000, 1000, 64, 1
    fixtures = json.load(open(os.path.join(ROOT, "tests", "golden", "full_length.json")))
    g = torch.Generator(device="cuda")
    g.manual_seed(4001)
    x = torch.randn((T, B, C), generator=g, device="cuda", dtype=torch.float32)   # 8.2 GB
    sl_np = np.random.default_rng(41).integers(T // 2, T + 1, size=B).astype(np.int32)
    placed = {}   # batch position -> (fixture, item)
    for name, pos in (("cfg4_T2000_B2", (127, 128)), ("cfg4_peaky_T2000", (1023,))):
        fx = fixtures[name]
        assert fx["case"][5:10] == [W, P, False, 0, -1], name
        xf, slf = make_fixtures_full.inputs(fx["case"])
        for item, b in enumerate(pos):
            x[:, b] = torch.as_tensor(xf[:, item], device="cuda")
            sl_np[b] = slf[item]
            placed[b] = (fx, item)
    sl = torch.as_tensor(sl_np, device="cuda")
    kw = dict(merge_repeated=False, blank_index=0, blank_label=-1)
    one = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, **kw)
    many = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, devices=[0] * 8, **kw)
    torch.cuda.synchronize()
    assert ctcext_amd.get_decoder(tuple([0] * 8)).last_stats["n_devices"] == 8
    del x
    torch.cuda.empty_cache()
    _same(many, one, P)
    dec = _rows(many.decoded_indices[0], many.decoded_values[0], B)
    ali = _rows(many.alignment_indices[0], many.alignment_values[0], B)
    lp = to_numpy(many.log_probability)
    for b, (fx, item) in placed.items():
        assert dec[b] == fx["decoded"][item][0], b
        assert ali[b] == fx["alignment"][item][0], b
        assert lp[b, 0] == np.float32(float.fromhex(fx["log_probability_hex"][item][0])), b
    _check_structure(many, sl_np, C, P, False)


def _memory_probe():
    import psutil
    free, _ = torch.cuda.mem_get_info(0)
    hs = torch.cuda.host_memory_stats() if hasattr(torch.cuda, "host_memory_stats") else {}
    return free, hs.get("reserved_bytes.current", hs.get("allocated_bytes.current", 0)), \
        psutil.Process().memory_info().rss


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_no_memory_growth_over_1000_calls(devices):
    """The reference's memory-leak test (python/ops/..._test.py:102-123: 1000
    calls, memory must not grow), on what this path allocates: device memory
    (the library's grow-only workspace, torch's caching allocator for device
    outputs), the pinned host pool behind host outputs, and this process's
    RSS.  After the first calls have sized every pool, 1000 more calls must
    not grow any of them."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((60, 6, 29)).astype(np.float32)
    sl = np.array([60, 41, 60, 7, 1, 60], np.int32)
    xd, sld = torch.as_tensor(x, device="cuda:0"), torch.as_tensor(sl, device="cuda:0")
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1, devices=devices)

    def call(i):
        if i % 2:
            out = ctcext_amd.ctc_ext_beam_search_decoder(xd, sld, 16, 2, **kw)
        else:
            out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, 16, 2, **kw)
        return out
    first = call(0)
    for i in range(1, 20):
        call(i)
    torch.cuda.synchronize()
    free0, pinned0, rss0 = _memory_probe()
    for i in range(1000):
        out = call(i)
    torch.cuda.synchronize()
    free1, pinned1, rss1 = _memory_probe()
    _same(out, ctcext_amd.ctc_ext_beam_search_decoder(xd, sld, 16, 2, **kw), 2)
    _same(first, out, 2)
    assert free1 >= free0, ("device memory shrank", free0, free1)
    assert pinned1 <= pinned0, ("pinned host pool grew", pinned0, pinned1)
    # RSS: the Python objects of 1000 calls come and go; a leak of the ~50 KB
    # of outputs per call would add ~50 MB
    assert rss1 - rss0 < 8 << 20, ("host RSS grew", rss0, rss1)


def test_two_ranks_hip_decoder_gather(tmp_path):
    out = str(tmp_path / "rank0.npz")
    port = 29500 + (os.getpid() % 2000)
    env = dict(os.environ, CTCX_ONE_DEVICE="1", PYTHONUNBUFFERED="1",
               HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % port,
           os.path.join(ROOT, "tests", "dist_worker.py"), out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = np.load(out)
    import dist_worker
    x, sl, W, P, kw = dist_worker.workload()
    one = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, **kw)
    for p in range(P):
        for k in one._fields[:-1]:
            np.testing.assert_array_equal(got["%s_%d" % (k, p)], to_numpy(getattr(one, k)[p]),
                                          err_msg="%s[%d]" % (k, p))
    np.testing.assert_array_equal(got["log_probability"], to_numpy(one.log_probability))

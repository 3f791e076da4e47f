"""``ctc_ext_beam_search_decoder`` — the reference's Python op, on MI355X.

Same signature, argument meaning, output structure and error messages as the
TF-generated wrapper the reference exports
(python/ops/ctc_ext_beam_search_decoder_ops.py:12, op definition
cc/ops/ctc_ext_beam_search_decoder_ops.cc:9-63):

    ctc_ext_beam_search_decoder(inputs, sequence_length, beam_width, top_paths,
                                merge_repeated=False, blank_index=0,
                                blank_label=-1, name=None)
      -> (decoded_indices, decoded_values, decoded_shape,
          alignment_indices, alignment_values, alignment_shape,
          log_probability)

The six list outputs are Python lists of ``top_paths`` int64 arrays (the
SparseTensor components of kernels.cc:163-257); ``log_probability`` is
[batch_size, top_paths] of the input dtype.  Host inputs (numpy, lists, CPU
torch tensors) give numpy outputs; device (HBM) torch tensors give device
torch tensors.  Decoding always runs on the GPU through libctcext.so.
"""
import collections
import ctypes
import threading
import warnings

import numpy as np

from . import _lib

CTCExtBeamSearchDecoder = collections.namedtuple(
    "CTCExtBeamSearchDecoder",
    ["decoded_indices", "decoded_values", "decoded_shape",
     "alignment_indices", "alignment_values", "alignment_shape",
     "log_probability"])


class OpError(Exception):
    """Mirror of tf.errors.OpError: ``.message`` holds the reference's text."""

    def __init__(self, message, code):
        super().__init__(message)
        self.message = message
        self.error_code = code


class InvalidArgumentError(OpError):
    pass


class FailedPreconditionError(OpError):
    pass


class UnimplementedError(OpError):
    pass


class InternalError(OpError):
    pass


_ERRORS = {_lib.CTCEXT_INVALID_ARGUMENT: InvalidArgumentError,
           _lib.CTCEXT_FAILED_PRECONDITION: FailedPreconditionError,
           _lib.CTCEXT_UNIMPLEMENTED: UnimplementedError,
           _lib.CTCEXT_INTERNAL: InternalError}

_tls = threading.local()


def _raise(lib, rc):
    msg = lib.ctcext_last_error().decode()
    raise _ERRORS.get(rc, InternalError)(msg, rc)


class Decoder:
    """One libctcext handle (device workspace + HIP stream per device) per
    device set and thread, like one OpKernel instance per device.  With more
    than one device the handle decodes contiguous batch shards on each and
    assembles the outputs on ``devices[0]`` (ctcext_create_sharded)."""

    def __init__(self, device=0):
        self.lib = _lib.load()
        devs = tuple(int(d) for d in (device if isinstance(device, (tuple, list)) else (device,)))
        h = ctypes.c_void_p()
        if len(devs) == 1:
            rc = self.lib.ctcext_create(devs[0], ctypes.byref(h))
        else:
            arr = (ctypes.c_int * len(devs))(*devs)
            rc = self.lib.ctcext_create_sharded(arr, len(devs), ctypes.byref(h))
        if rc != _lib.CTCEXT_OK:
            _raise(self.lib, rc)
        self.handle = h
        self.devices = devs
        self.device = devs[0]
        self.last_stats = None

    def close(self):
        if self.handle:
            self.lib.ctcext_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        s = _lib.Stats()
        _lib.get_stats(self.lib, self.handle, s)
        return {k: getattr(s, k) for k, _ in _lib.Stats._fields_ if k != "pad_"}

    # -- phase 1 ---------------------------------------------------------
    def decode(self, args):
        P = max(int(args.top_paths), 1)
        sizes = (_lib.PathSizes * P)()
        rc = self.lib.ctcext_decode_sharded(self.handle, ctypes.byref(args), sizes)
        if rc != _lib.CTCEXT_OK:
            _raise(self.lib, rc)
        self.last_stats = self.stats()
        if self.last_stats.get("helper_redecodes", 0) > 0:
            # a two-wave kernel's hand-over wait ran out of time (never in a
            # correct run): the outputs are right, decoded again by the
            # one-wave kernels, but the call took up to ~2x its time
            warnings.warn("ctc_ext_beam_search_decoder: a helper-wave hand-over wait timed out; the call was "
                          "decoded again with the one-wave kernels (ctcext_stats.helper_redecodes = %d)"
                          % self.last_stats["helper_redecodes"], RuntimeWarning, stacklevel=3)
        return [(s.num_decoded, s.max_decoded, s.num_alignment, s.max_alignment) for s in sizes]

    # -- phase 2 ---------------------------------------------------------
    def fetch(self, ptr_lists, log_prob_ptr, on_device):
        P = len(ptr_lists[0])
        arrs = [(ctypes.c_void_p * P)(*pl) for pl in ptr_lists]
        o = _lib.Outputs()
        o.outputs_on_device = 1 if on_device else 0
        o.decoded_indices, o.decoded_values, o.decoded_shape = arrs[0], arrs[1], arrs[2]
        o.alignment_indices, o.alignment_values, o.alignment_shape = arrs[3], arrs[4], arrs[5]
        o.log_probability = log_prob_ptr
        rc = self.lib.ctcext_fetch(self.handle, ctypes.byref(o))
        if rc != _lib.CTCEXT_OK:
            _raise(self.lib, rc)


def get_decoder(device=0):
    """The calling thread's handle for ``device`` (an ordinal, or a tuple of
    ordinals for a sharded multi-device handle)."""
    cache = getattr(_tls, "decoders", None)
    if cache is None:
        cache = _tls.decoders = {}
    key = tuple(device) if isinstance(device, (tuple, list)) else int(device)
    d = cache.get(key)
    if d is None:
        d = cache[key] = Decoder(key)
    return d


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _print_no_label(n):
    # ctc_beam_entry.h:148-150 prints once per path without any candidate
    for _ in range(int(n)):
        print("No label seq available")


def _type_error(name, got, allowed):
    # the message TF's op wrapper raises for a dtype outside the op's type list
    # (ops.cc:17-18: T in {float, double}; sequence_length: int32)
    raise TypeError("Value passed to parameter '%s' has DataType %s not in list of allowed values: %s"
                    % (name, got, allowed))


def _current_device():
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.current_device()
    except ImportError:
        pass
    return 0


def _args(x_ptr, shape, dtype_code, on_device, sl_ptr, sl_shape, beam_width, top_paths, merge_repeated,
          blank_index, blank_label, flags, stream):
    a = _lib.DecodeArgs()
    a.dtype = dtype_code
    a.inputs_on_device = 1 if on_device else 0
    a.inputs = x_ptr
    a.sequence_length = sl_ptr
    dims = list(shape) + [0, 0, 0]
    a.max_time, a.batch_size, a.num_classes = int(dims[0]), int(dims[1]), int(dims[2])
    a.inputs_dims = len(shape)
    a.sequence_length_dims = len(sl_shape)
    a.sequence_length_size = int(sl_shape[0]) if len(sl_shape) >= 1 else 0
    a.beam_width = int(beam_width)
    a.top_paths = int(top_paths)
    a.merge_repeated = 1 if merge_repeated else 0
    a.blank_index = int(blank_index)
    a.blank_label = int(blank_label)
    a.flags = int(flags)
    a.stream = stream
    return a


def ctc_ext_beam_search_decoder(inputs, sequence_length, beam_width, top_paths,
                                merge_repeated=False, blank_index=0, blank_label=-1,
                                name=None, *, flags=0, outputs="auto", devices=None, scorer_table=None):
    """Drop-in for the reference op.  See the module docstring.

    Keyword-only extensions (not in the reference):
      outputs: "auto" (device tensors for device inputs, numpy for host
        inputs), "host" (numpy, copied from the GPU into pinned host memory;
        the reference op's own output placement) or "device".
      devices: a list of device ordinals to decode contiguous batch shards on,
        in one process (ctcext_create_sharded); device inputs must live on
        devices[0], where the outputs are assembled.
      scorer_table: a [num_classes + 1, num_classes] table of log-probabilities
        (<= 0) for the decoder's beam-scorer hook (util/ctc_beam_scorer.h:31-65):
        expanding a beam that ends in label a (row 0: the empty beam) by label
        b adds table[a + 1, b] to the score it extends.  The reference op
        always uses the identity scorer (kernels.cc:260), which None selects.
      flags: CTCEXT_FLAG_* diagnostics.
    """
    del name
    if outputs not in ("auto", "host", "device"):
        raise ValueError("outputs must be 'auto', 'host' or 'device'")
    lib = _lib.load()
    keep = []   # arrays whose memory the C call reads
    on_device = _is_torch(inputs) and inputs.is_cuda
    if on_device:
        import torch
        if inputs.dtype not in (torch.float32, torch.float64):
            _type_error("inputs", str(inputs.dtype).replace("torch.", ""), "float32, float64")
        x = inputs.contiguous()
        dev = x.device
        if _is_torch(sequence_length):
            if sequence_length.dtype.is_floating_point:
                _type_error("sequence_length", str(sequence_length.dtype).replace("torch.", ""), "int32")
            sl = sequence_length.to(device=dev, dtype=torch.int32).contiguous()
        else:
            sl = torch.as_tensor(np.asarray(sequence_length, dtype=np.int32), device=dev)
        keep += [x, sl]
        shape, sl_shape = tuple(x.shape), tuple(sl.shape)
        code = _lib.CTCEXT_F32 if x.dtype == torch.float32 else _lib.CTCEXT_F64
        x_ptr, sl_ptr = x.data_ptr(), sl.data_ptr()
        index = dev.index if dev.index is not None else torch.cuda.current_device()
        stream = torch.cuda.current_stream(dev).cuda_stream
    else:
        if _is_torch(inputs):
            inputs = inputs.detach().cpu().numpy()
        if _is_torch(sequence_length):
            sequence_length = sequence_length.detach().cpu().numpy()
        if isinstance(inputs, np.ndarray):
            if inputs.dtype not in (np.float32, np.float64):
                _type_error("inputs", inputs.dtype.name, "float32, float64")
            x = np.ascontiguousarray(inputs)
        else:   # Python numbers convert to float32, as tf.convert_to_tensor does
            x = np.ascontiguousarray(np.asarray(inputs, dtype=np.float32))
        sl_arr = np.asarray(sequence_length)
        if sl_arr.dtype.kind == "f":
            _type_error("sequence_length", sl_arr.dtype.name, "int32")
        sl = np.ascontiguousarray(sl_arr.astype(np.int32))
        keep += [x, sl]
        shape, sl_shape = x.shape, sl.shape
        code = _lib.CTCEXT_F32 if x.dtype == np.float32 else _lib.CTCEXT_F64
        x_ptr, sl_ptr = x.ctypes.data, sl.ctypes.data
        index = None
        stream = None
    a = _args(x_ptr, shape, code, on_device, sl_ptr, sl_shape, beam_width, top_paths, merge_repeated,
              blank_index, blank_label, flags, stream)
    # the reference's shape/length checks run behind the C ABI, before any
    # device work (kernels.cc:97-139)
    rc = lib.ctcext_validate(ctypes.byref(a))
    if rc != _lib.CTCEXT_OK:
        _raise(lib, rc)
    if scorer_table is not None:
        C = int(shape[2]) if len(shape) == 3 else 0
        if on_device:
            import torch
            tab = torch.as_tensor(scorer_table, device=x.device, dtype=x.dtype).contiguous()
            a.scorer_table = tab.data_ptr()
        else:
            tab = np.ascontiguousarray(np.asarray(
                scorer_table.detach().cpu().numpy() if _is_torch(scorer_table) else scorer_table, dtype=x.dtype))
            a.scorer_table = tab.ctypes.data
        if tuple(tab.shape) != (C + 1, C):
            raise ValueError("scorer_table must be [num_classes + 1, num_classes] = [%d, %d], got %s"
                             % (C + 1, C, tuple(tab.shape)))
        keep.append(tab)
        a.scorer = _lib.CTCEXT_SCORER_BIGRAM
        # the library checks the table's entries (<= 0) before decoding
        rc = lib.ctcext_validate(ctypes.byref(a))
        if rc != _lib.CTCEXT_OK:
            _raise(lib, rc)
    if devices is not None:
        devs = tuple(int(d) for d in devices)
        if on_device and devs[0] != index:
            raise ValueError("device inputs must live on devices[0] (cuda:%d), not cuda:%d" % (devs[0], index))
        dec = get_decoder(devs if len(devs) > 1 else devs[0])
    else:
        dec = get_decoder(index if index is not None else _current_device())
    sizes = dec.decode(a)
    P = int(top_paths)
    B = int(shape[1])
    if outputs == "device" or (outputs == "auto" and on_device):
        import torch
        dev = torch.device("cuda", dec.device)
        i64 = dict(dtype=torch.int64, device=dev)
        di = [torch.empty((s[0], 2), **i64) for s in sizes]
        dv = [torch.empty((s[0],), **i64) for s in sizes]
        ds = [torch.empty((2,), **i64) for _ in sizes]
        ai = [torch.empty((s[2], 2), **i64) for s in sizes]
        av = [torch.empty((s[2],), **i64) for s in sizes]
        ash = [torch.empty((2,), **i64) for _ in sizes]
        lp = torch.empty((B, P), dtype=torch.float32 if code == _lib.CTCEXT_F32 else torch.float64, device=dev)
        lists = [[t.data_ptr() for t in lst] for lst in (di, dv, ds, ai, av, ash)]
        dec.fetch(lists, lp.data_ptr(), True)
    else:
        empty = _host_empty()
        fdt = np.float32 if code == _lib.CTCEXT_F32 else np.float64
        di = [empty((s[0], 2), np.int64) for s in sizes]
        dv = [empty((s[0],), np.int64) for s in sizes]
        ds = [empty((2,), np.int64) for _ in sizes]
        ai = [empty((s[2], 2), np.int64) for s in sizes]
        av = [empty((s[2],), np.int64) for s in sizes]
        ash = [empty((2,), np.int64) for _ in sizes]
        lp = empty((B, P), fdt)
        lists = [[t.ctypes.data for t in lst] for lst in (di, dv, ds, ai, av, ash)]
        dec.fetch(lists, lp.ctypes.data, False)
    del keep
    _print_no_label(dec.last_stats["no_label_paths"])
    return CTCExtBeamSearchDecoder(di, dv, ds, ai, av, ash, lp)


def _host_empty():
    """Host output allocator: numpy views of pinned torch CPU tensors (the
    caching host allocator reuses the pinned pages, so the GPU copies the
    components down at full PCIe rate without first-touch page faults), or
    plain numpy without torch."""
    try:
        import torch
        if torch.cuda.is_available():
            tdt = {np.dtype(np.int64): torch.int64, np.dtype(np.float32): torch.float32,
                   np.dtype(np.float64): torch.float64}

            def empty(shape, dt):
                return torch.empty(shape, dtype=tdt[np.dtype(dt)], pin_memory=True).numpy()
            return empty
    except ImportError:
        pass
    return np.empty

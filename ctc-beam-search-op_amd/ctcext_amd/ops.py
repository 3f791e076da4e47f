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
    """One libctcext handle (device workspace + HIP stream) per device and
    thread, like one OpKernel instance per device."""

    def __init__(self, device=0):
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        rc = self.lib.ctcext_create(int(device), ctypes.byref(h))
        if rc != _lib.CTCEXT_OK:
            _raise(self.lib, rc)
        self.handle = h
        self.device = int(device)
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
        self.lib.ctcext_get_stats(self.handle, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in _lib.Stats._fields_}

    # -- phase 1 ---------------------------------------------------------
    def decode(self, x_ptr, sl_ptr, T, B, C, dtype_code, on_device, beam_width, top_paths,
               merge_repeated, blank_index, blank_label, flags=0, stream=None):
        a = _lib.DecodeArgs()
        a.dtype = dtype_code
        a.inputs_on_device = 1 if on_device else 0
        a.inputs = x_ptr
        a.sequence_length = sl_ptr
        a.max_time, a.batch_size, a.num_classes = int(T), int(B), int(C)
        a.beam_width = int(beam_width)
        a.top_paths = int(top_paths)
        a.merge_repeated = 1 if merge_repeated else 0
        a.blank_index = int(blank_index)
        a.blank_label = int(blank_label)
        a.flags = int(flags)
        a.stream = stream
        P = max(int(top_paths), 1)
        sizes = (_lib.PathSizes * P)()
        rc = self.lib.ctcext_decode(self.handle, ctypes.byref(a), sizes)
        if rc != _lib.CTCEXT_OK:
            _raise(self.lib, rc)
        self.last_stats = self.stats()
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
    cache = getattr(_tls, "decoders", None)
    if cache is None:
        cache = _tls.decoders = {}
    d = cache.get(device)
    if d is None:
        d = cache[device] = Decoder(device)
    return d


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _validate_attrs(beam_width, top_paths):
    # attr constraints of the op definition (ops.cc:12-13)
    if int(beam_width) < 1:
        raise InvalidArgumentError("Value for attr 'beam_width' of %d must be at least minimum 1"
                                   % int(beam_width), _lib.CTCEXT_INVALID_ARGUMENT)
    if int(top_paths) < 1:
        raise InvalidArgumentError("Value for attr 'top_paths' of %d must be at least minimum 1"
                                   % int(top_paths), _lib.CTCEXT_INVALID_ARGUMENT)


def _print_no_label(n):
    # ctc_beam_entry.h:148-150 prints once per path without any candidate
    for _ in range(int(n)):
        print("No label seq available")


def ctc_ext_beam_search_decoder(inputs, sequence_length, beam_width, top_paths,
                                merge_repeated=False, blank_index=0, blank_label=-1,
                                name=None, flags=0):
    """Drop-in for the reference op.  See the module docstring."""
    del name
    _validate_attrs(beam_width, top_paths)
    if _is_torch(inputs) and inputs.is_cuda:
        return _decode_device(inputs, sequence_length, beam_width, top_paths, merge_repeated,
                              blank_index, blank_label, flags)
    return _decode_host(inputs, sequence_length, beam_width, top_paths, merge_repeated,
                        blank_index, blank_label, flags)


def _check_shapes(shape, sl_shape):
    if len(shape) != 3:
        raise InvalidArgumentError("inputs is not a 3-Tensor", _lib.CTCEXT_INVALID_ARGUMENT)
    if len(sl_shape) != 1:
        raise InvalidArgumentError("sequence_length is not a vector", _lib.CTCEXT_INVALID_ARGUMENT)
    if shape[0] == 0:
        raise InvalidArgumentError("max_time is 0", _lib.CTCEXT_INVALID_ARGUMENT)
    if sl_shape[0] != shape[1]:
        raise FailedPreconditionError(
            "len(sequence_length) != batch_size.  len(sequence_length):  %d batch_size: %d"
            % (sl_shape[0], shape[1]), _lib.CTCEXT_FAILED_PRECONDITION)


def _decode_host(inputs, sequence_length, beam_width, top_paths, merge_repeated, blank_index,
                 blank_label, flags, device=0):
    if _is_torch(inputs):
        inputs = inputs.detach().cpu().numpy()
    if _is_torch(sequence_length):
        sequence_length = sequence_length.detach().cpu().numpy()
    x = np.asarray(inputs)
    if x.dtype not in (np.float32, np.float64):
        x = x.astype(np.float32)
    x = np.ascontiguousarray(x)
    sl = np.ascontiguousarray(np.asarray(sequence_length, dtype=np.int32))
    _check_shapes(x.shape, sl.shape)
    T, B, C = x.shape
    dec = get_decoder(device)
    code = _lib.CTCEXT_F32 if x.dtype == np.float32 else _lib.CTCEXT_F64
    sizes = dec.decode(x.ctypes.data, sl.ctypes.data, T, B, C, code, False, beam_width, top_paths,
                       merge_repeated, blank_index, blank_label, flags)
    P = int(top_paths)
    di = [np.empty((s[0], 2), np.int64) for s in sizes]
    dv = [np.empty((s[0],), np.int64) for s in sizes]
    ds = [np.empty((2,), np.int64) for _ in sizes]
    ai = [np.empty((s[2], 2), np.int64) for s in sizes]
    av = [np.empty((s[2],), np.int64) for s in sizes]
    ash = [np.empty((2,), np.int64) for _ in sizes]
    lp = np.empty((B, P), x.dtype)
    lists = [[a.ctypes.data for a in lst] for lst in (di, dv, ds, ai, av, ash)]
    dec.fetch(lists, lp.ctypes.data, False)
    _print_no_label(dec.last_stats["no_label_paths"])
    return CTCExtBeamSearchDecoder(di, dv, ds, ai, av, ash, lp)


def _decode_device(inputs, sequence_length, beam_width, top_paths, merge_repeated, blank_index,
                   blank_label, flags):
    import torch
    dev = inputs.device
    if inputs.dtype not in (torch.float32, torch.float64):
        inputs = inputs.float()
    x = inputs.contiguous()
    if _is_torch(sequence_length):
        sl = sequence_length.to(device=dev, dtype=torch.int32).contiguous()
    else:
        sl = torch.as_tensor(np.asarray(sequence_length, dtype=np.int32), device=dev)
    _check_shapes(tuple(x.shape), tuple(sl.shape))
    T, B, C = x.shape
    index = dev.index if dev.index is not None else torch.cuda.current_device()
    dec = get_decoder(index)
    stream = torch.cuda.current_stream(dev).cuda_stream
    code = _lib.CTCEXT_F32 if x.dtype == torch.float32 else _lib.CTCEXT_F64
    sizes = dec.decode(x.data_ptr(), sl.data_ptr(), T, B, C, code, True, beam_width, top_paths,
                       merge_repeated, blank_index, blank_label, flags, stream)
    P = int(top_paths)
    i64 = dict(dtype=torch.int64, device=dev)
    di = [torch.empty((s[0], 2), **i64) for s in sizes]
    dv = [torch.empty((s[0],), **i64) for s in sizes]
    ds = [torch.empty((2,), **i64) for _ in sizes]
    ai = [torch.empty((s[2], 2), **i64) for s in sizes]
    av = [torch.empty((s[2],), **i64) for s in sizes]
    ash = [torch.empty((2,), **i64) for _ in sizes]
    lp = torch.empty((B, P), dtype=x.dtype, device=dev)
    lists = [[t.data_ptr() for t in lst] for lst in (di, dv, ds, ai, av, ash)]
    dec.fetch(lists, lp.data_ptr(), True)
    _print_no_label(dec.last_stats["no_label_paths"])
    return CTCExtBeamSearchDecoder(di, dv, ds, ai, av, ash, lp)

"""ctcext_amd — MI355X-native CTC beam search with per-beam best-alignment
tracking; a drop-in for prouast/ctc-beam-search-op's
``ctc_ext_beam_search_decoder`` (tensorflow_ctc_ext_beam_search_decoder/__init__.py:19).
"""
from .ops import (CTCExtBeamSearchDecoder, Decoder, FailedPreconditionError, InternalError,
                  InvalidArgumentError, OpError, UnimplementedError, ctc_ext_beam_search_decoder,
                  get_decoder)

__all__ = ["ctc_ext_beam_search_decoder", "CTCExtBeamSearchDecoder", "Decoder", "get_decoder",
           "OpError", "InvalidArgumentError", "FailedPreconditionError", "UnimplementedError",
           "InternalError"]

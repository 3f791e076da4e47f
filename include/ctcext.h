/* ctcext.h — C ABI of the MI355X CTC beam-search decoder with per-beam
 * best-alignment tracking (libctcext.so).
 *
 * This is the drop-in boundary for the reference TensorFlow op
 *   REGISTER_OP("CTCExtBeamSearchDecoder")
 *       cc/ops/ctc_ext_beam_search_decoder_ops.cc:9-63
 *   CTCExtBeamSearchDecoderOp<T>::Compute
 *       cc/kernels/ctc_ext_beam_search_decoder_kernels.cc:20-95
 * (paths relative to /root/reference/tensorflow_ctc_ext_beam_search_decoder/).
 * Plain pointers and sizes only; no framework types cross it.  A TF OpKernel
 *  or the ctypes binding in ctcext_amd/_lib.py calls it.
 *
 * Two phases, like the reference kernel which counts entries before
 * allocating its outputs (kernels.cc:170-213):
 *   1. ctcext_decode: validates, decodes the whole batch on the GPU and
 *      returns, per top path, the SparseTensor entry counts and dense widths.
 *   2. ctcext_fetch: writes the int64 SparseTensor components and the
 *      log-probabilities into caller-allocated buffers (device or host).
 * Status codes are TensorFlow's (error::Code); messages are the reference's
 * verbatim (kernels.cc:111-139, ctc_ext_beam_search_decoder.h:237-243).
 */
#ifndef CTCEXT_H_
#define CTCEXT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  CTCEXT_OK = 0,
  CTCEXT_INVALID_ARGUMENT = 3,   /* errors::InvalidArgument */
  CTCEXT_FAILED_PRECONDITION = 9,/* errors::FailedPrecondition */
  CTCEXT_UNIMPLEMENTED = 12,
  CTCEXT_INTERNAL = 13
};

enum { CTCEXT_F32 = 0, CTCEXT_F64 = 1 };   /* attr T: {float, double} (ops.cc:24) */

/* Beam scorer (util/ctc_beam_scorer.h:31-65).  The reference op always uses
 * BaseBeamScorer (kernels.cc:260), the identity; the decoder exposes the hook
 * (ctc_ext_beam_search_decoder.h:43-45, 103, 114, 171-182, 226).
 *   CTCEXT_SCORER_BIGRAM: ExpandState caches table[from_label + 1][to_label]
 *   (row 0: expansions of the root), GetStateExpansionScore adds it to the
 *   score it extends.  table is [num_classes + 1][num_classes] of dtype, in
 *   the memory inputs_on_device says; entries are log-probabilities (<= 0). */
enum { CTCEXT_SCORER_BASE = 0, CTCEXT_SCORER_BIGRAM = 1 };

enum {
  CTCEXT_FLAG_FORCE_LITERAL = 1,   /* testing: replay every frame through the literal TopN model */
  CTCEXT_FLAG_PROFILE = 2,         /* time the decode kernel with HIP events (ctcext_stats) */
  CTCEXT_FLAG_PHASES = 4,          /* diagnostics: per-item s_memtime phase counters */
  CTCEXT_FLAG_GLOBAL_STATE = 8,    /* testing: decode on the global-state tier whatever the shape */
  CTCEXT_FLAG_RECORD_RING = 16,    /* keep beam records in an LDS ring and write only those the
                                      traceback can reach (fewer HBM writes).  On by default
                                      where the score-table two-wave kernel runs (float,
                                      beam_width <= 128, num_classes <= 64); opt-in elsewhere */
  CTCEXT_FLAG_RING_MIN = 32,       /* testing: the record ring at its smallest (8 frames), so short
                                      items flush; implies CTCEXT_FLAG_RECORD_RING */
  CTCEXT_FLAG_NO_RING = 64,        /* write every beam record to HBM (no record ring) */
  CTCEXT_FLAG_HELPER_STRICT = 128, /* a two-wave kernel's hand-over wait that runs out of time
                                      (~1 s; never in a correct run) fails the call with
                                      CTCEXT_INTERNAL instead of decoding it again with the
                                      one-wave kernels (ctcext_stats.helper_redecodes) */
  CTCEXT_FLAG_TEST_HELPER_DEAD = 256 /* testing: the helper wave starts out as if its first
                                      wait had run out of time (the failure path, no hang) */
};

/* Version of this header's structs and entry points.  ctcext_stats only ever
 * grows at its end: callers built against an older header use
 * ctcext_get_stats_sized with their sizeof.
 *   4: ctcext_stats.record_bytes, .helper     5: .helper_redecodes,
 *      ctcext_get_stats_sized, ctcext_abi_version, the HELPER_STRICT flag
 *   6: ctcext_get_stats fills the ABI-4 prefix only (fields since: _sized);
 *      ctcext_phase_counters' layout is [batch][32] */
#define CTCEXT_ABI_VERSION 6

typedef struct ctcext_decoder ctcext_decoder;

/* Replaces the op's inputs + attrs (ops.cc:10-17).  The two input tensors
 * travel as (pointer, rank, sizes), the way an OpKernel sees them, so that the
 * reference's shape checks (kernels.cc:111-131) run behind this ABI. */
typedef struct {
  int32_t dtype;                   /* CTCEXT_F32 / CTCEXT_F64 */
  int32_t inputs_on_device;        /* 1: inputs/sequence_length are device (HBM) pointers
                                      on the decoder's (root) device */
  const void* inputs;              /* [max_time, batch_size, num_classes] row-major */
  const int32_t* sequence_length;  /* [batch_size] */
  int64_t max_time, batch_size, num_classes;   /* inputs.dim_size(0..2) (0 past the rank) */
  int32_t beam_width;              /* attr beam_width >= 1 */
  int32_t top_paths;               /* attr top_paths >= 1 */
  int32_t merge_repeated;          /* attr merge_repeated (default false) */
  int32_t blank_index;             /* attr blank_index (default 0) */
  int32_t blank_label;             /* attr blank_label (default -1) */
  int32_t flags;                   /* CTCEXT_FLAG_* */
  void* stream;                    /* hipStream_t; NULL = the decoder's own stream */
  int32_t inputs_dims;             /* inputs.dims(): must be 3 (kernels.cc:111-113) */
  int32_t sequence_length_dims;    /* sequence_length.dims(): must be 1 (kernels.cc:122-124) */
  int64_t sequence_length_size;    /* sequence_length.dim_size(0): must equal batch_size
                                      (kernels.cc:126-130); the number of int32 read */
  int32_t scorer;                  /* CTCEXT_SCORER_* (0: the reference op's BaseBeamScorer) */
  int32_t pad_;
  const void* scorer_table;        /* CTCEXT_SCORER_BIGRAM: [num_classes + 1][num_classes] */
} ctcext_decode_args;

/* Per top path p: sizes of decoded_indices[p] ([num_decoded, 2]),
 * decoded_values[p] ([num_decoded]), decoded_shape[p] = {batch, max_decoded},
 * and the same for the alignment outputs. */
typedef struct {
  int64_t num_decoded, max_decoded;
  int64_t num_alignment, max_alignment;
} ctcext_path_sizes;

/* Replaces the op's 6 * top_paths + 1 outputs (ops.cc:18-24).  Each list is an
 * array of top_paths pointers; shapes as in ctcext_path_sizes. */
typedef struct {
  int32_t outputs_on_device;       /* 1: all pointers below are device pointers */
  int64_t* const* decoded_indices;
  int64_t* const* decoded_values;
  int64_t* const* decoded_shape;
  int64_t* const* alignment_indices;
  int64_t* const* alignment_values;
  int64_t* const* alignment_shape;
  void* log_probability;           /* [batch_size, top_paths] of dtype */
} ctcext_outputs;

typedef struct {
  int64_t literal_frames;          /* frames replayed through the literal TopN model */
  int64_t literal_nonfinite;       /*   ... because a total or logit was not finite */
  int64_t literal_fill;            /*   ... because the beam filled up mid-frame */
  int64_t duplicate_frames;        /* frames whose beam held one entry twice (reachable
                                      with -inf logits: decoder.h:142 + 189-199) */
  int64_t no_label_paths;          /* paths whose alignment is empty: the reference prints
                                      "No label seq available" (ctc_beam_entry.h:148-150) */
  double decode_kernel_ms;         /* with CTCEXT_FLAG_PROFILE: last ctcx_beam_decode time
                                      (the slowest device of a sharded handle) */
  double norm_kernel_ms;
  double traceback_ms;             /* traceback + scan */
  int32_t n_devices;               /* devices of the handle */
  int32_t tier;                    /* last decode: 0 the LDS-resident fast tier, 1 the
                                      global-state tier (shapes past the LDS / record limits) */
  int32_t ring_frames;             /* last decode: frames of the LDS record ring (0: every
                                      record of every frame written to HBM) */
  int64_t records_written;         /* last decode: beam records written to HBM (all devices) */
  int32_t record_bytes;            /* last decode: bytes per record (8; 16 on the global-state
                                      tier; 4 in the two-wave kernel, beam_width <= 128 and
                                      num_classes <= 64) */
  int32_t helper;                  /* last decode: the two-wave kernel that ran (0: the one-wave
                                      kernel; 1: score-table helper; 2: gather-queue helper) */
  int32_t helper_redecodes;        /* last decode: 1 if a two-wave kernel's hand-over wait ran
                                      out of time and the call was decoded again with the
                                      one-wave kernels (helper is then 0) */
  int32_t pad_;
} ctcext_stats;

/* Handle lifetime.  A handle owns a HIP stream and a grow-only device
 * workspace; it is not thread-safe (use one per thread, like an OpKernel).
 * Every entry point restores the calling thread's current HIP device. */
int ctcext_create(int device, ctcext_decoder** out);
void ctcext_destroy(ctcext_decoder* dec);

/* Multi-device handle for one process driving several GPUs: the batch is split
 * into contiguous shards balanced by sum(sequence_length), one per device
 * (devices[0] is the root: inputs_on_device pointers live there, and the
 * outputs are assembled there).  Each device decodes its shard on its own
 * stream; the per-item walks are gathered to the root over peer copies (xGMI)
 * and packed there, so the outputs are identical to a one-device decode.  The
 * same device may be listed twice (its shards then share its CUs).  Use it
 * with ctcext_decode_sharded + ctcext_fetch. */
int ctcext_create_sharded(const int* devices, int n_devices, ctcext_decoder** out);

/* The reference's ValidateInputsGenerateOutputs (kernels.cc:97-139) plus this
 * library's attribute checks, on the host only (no HIP call, no handle): the
 * messages are the reference's verbatim and come in its order.  The
 * sequence_length values (kernels.cc:134-139) are checked here only when they
 * are host memory (inputs_on_device == 0); ctcext_decode checks them always. */
int ctcext_validate(const ctcext_decode_args* args);

/* Phase 1 (Compute up to the allocation of the outputs).  Synchronous. */
int ctcext_decode(ctcext_decoder* dec, const ctcext_decode_args* args, ctcext_path_sizes* sizes);

/* Phase 1 over a ctcext_create_sharded handle (kernels.cc:68-90's batch loop
 * split across devices).  On a one-device handle it is ctcext_decode. */
int ctcext_decode_sharded(ctcext_decoder* dec, const ctcext_decode_args* args, ctcext_path_sizes* sizes);

/* Phase 2 (StoreAllDecodedSequences + log_probability).  Synchronous. */
int ctcext_fetch(ctcext_decoder* dec, const ctcext_outputs* out);

/* Statistics of the last decode.  ctcext_get_stats fills the ABI-4 prefix
 * only (every field before helper_redecodes: callers built against that
 * header pass a struct of that size); ctcext_get_stats_sized fills the first
 * `size` bytes (pass sizeof(ctcext_stats) for every field of this header). */
int ctcext_get_stats(ctcext_decoder* dec, ctcext_stats* stats);
int ctcext_get_stats_sized(ctcext_decoder* dec, ctcext_stats* stats, size_t size);

/* CTCEXT_ABI_VERSION of the library. */
int32_t ctcext_abi_version(void);

/* Diagnostics: copies the [batch][32] phase counters of the last decode run
 * with CTCEXT_FLAG_PHASES, in the diagnostics build (make phases; the product
 * build leaves them 0).  [0, 24) the decoding wave (cycles: row load,
 * recursion, grow, extract, commit, literal frames; counts: grow events,
 * frames; ... see tools/diag_phases.py for every index), [24, 32) the helper
 * wave of the two-wave kernels. */
int ctcext_phase_counters(ctcext_decoder* dec, uint64_t* out, int64_t n);

/* Diagnostics (tests): the pre-pass of a decode alone, on device buffers and
 * the handle's stream, synchronously -- per (t, b) row of inputs
 * [max_time][batch][num_classes] (num_classes > 64) its record into prep
 * (*row_bytes each: RowHdr {max, largest non-blank value outside the top
 * set S, NaN/+inf flag, |S|}, the 64-class block maxima, S as (value bits,
 * label index) pairs in label order) and its softmax normaliser into norm.
 * With prep == NULL only *row_bytes is set.  Rows past seq_len are skipped. */
int ctcext_row_facts(ctcext_decoder* dec, const void* inputs, int32_t dtype, int64_t max_time, int64_t batch,
                     int64_t num_classes, int32_t blank_index, const int32_t* sequence_length, void* prep,
                     void* norm, int64_t* row_bytes);

/* Message of the last failing call on this thread ("" if none). */
const char* ctcext_last_error(void);

/* Widest beam the LDS-resident fast tier decodes for the given class count
 * and dtype (0: num_classes is past that tier).  Wider beams, and num_classes
 * above 65535 or the LDS row, decode on the global-state tier (beam state in
 * HBM, 16-byte records, the literal path every frame): any shape the
 * reference accepts, at a lower rate. */
int32_t ctcext_max_beam_width(int64_t num_classes, int32_t dtype);

#ifdef __cplusplus
}
#endif

#endif /* CTCEXT_H_ */

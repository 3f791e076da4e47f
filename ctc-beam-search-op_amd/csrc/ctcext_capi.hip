// ctcext_capi.hip — host side of libctcext.so: validation, workspace, kernel
// orchestration, multi-device sharding and output transfer behind the C ABI
// in include/ctcext.h.
//
// Mirrors the reference op kernel (cc/kernels/ctc_ext_beam_search_decoder_kernels.cc):
//   ValidateInputsGenerateOutputs  :97-139  -> validate_shapes / check_lengths (ctcext_validate)
//   Compute batch/time loop        :67-90   -> ctcx_row_norm + ctcx_beam_decode per shard
//   TopPaths errors                decoder.h:237-243
//   StoreAllDecodedSequences       :163-257 -> ctcx_traceback + ctcx_scan + ctcx_pack
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/ctcext.h"
#include "ctcx_kernels.h"

namespace ctcx {
template <typename T>
hipError_t launch_decode(const DecodeParams<T>& p, hipStream_t s);
template <typename T>
int ring_frames(const DecodeParams<T>& p, int cus, int cap, int hk);
template <typename T>
int use_helper_kernel(const DecodeParams<T>& p, int hk);
template <typename T>
int helper_kind(const DecodeParams<T>& p, int mode);
template <typename T>
hipError_t launch_row_norm(const T* x, const int32_t* sl, T* norm, int64_t T_, int64_t B, int64_t C,
                           int64_t xstride, hipStream_t s);
hipError_t launch_traceback(const TraceParams& tp, hipStream_t s);
template <typename T>
hipError_t launch_row_prep(const T* x, const int32_t* sl, char* prep, T* norm, int64_t T_, int64_t B, int64_t C,
                           int64_t xstride, int blank, hipStream_t s);
hipError_t launch_scan(const int32_t* len, int64_t* off, int64_t* res, int64_t B, int P, hipStream_t s);
hipError_t launch_pack(const PackParams& pp, hipStream_t s);
}  // namespace ctcx
// the global-state tier (ctcx_decode.hip compiled with CTCX_GSTATE)
hipError_t ctcx_gstate_launch_decode(const void* p, int is_f64, int scored, hipStream_t s);

static thread_local std::string g_err;

// the two-wave kernels a call runs by default (ctcx::helper_kind's mode): the
// scored gather queue for beams <= 128 (cfg3 decode 144.9 -> 126.8 ms, cfg4
// 164.9 -> 162.9 ms, same box: profiles/r5j_ab.txt), the gather queue above
constexpr int kDefaultHelperMode = ctcx::kHelperScored;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_OR_FAIL(expr)                                                             \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(CTCEXT_INTERNAL, std::string("HIP error: ") + hipGetErrorString(e_) \
                                       + " at " #expr);                              \
  } while (0)

namespace {

// Restores the calling thread's current HIP device on every exit path: the
// caller (e.g. torch in a per-rank process) reads the same runtime's device.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// One device of a handle: its stream, events and the per-shard workspace.
// The root (devs[0]) also holds the whole batch's walks, lengths and outputs.
struct Dev {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t s = nullptr;   // stream of the current call
  hipEvent_t ev[4] = {};
  DevBuf x, sl, norm, prep, rec, foff, item, top_pos, top_kind, logp, seq, len, phase, sctab, gstate;
  int64_t lo = 0, nb = 0;    // this call's shard [lo, lo + nb)
  int ring = 0;              // this call's record-ring frames (ctcx::ring_frames)
  int rec_bytes = 8;         // this call's record size (8, 16 or 4 bytes)
  int helper = 0;            // this call's two-wave kernel (ctcx::use_helper_kernel)
  int cus = 0;               // compute units of the device
};

}  // namespace

struct ctcext_decoder {
  std::vector<Dev> devs;
  // root-side: scan results and output staging
  DevBuf off, res, ptrs, out_idx, out_val;
  HostBuf h_item, h_res, h_kind;
  // state of the last successful decode (consumed by fetch)
  bool have = false;
  int dtype = 0;
  int64_t T = 0, B = 0, C = 0;
  int32_t W = 0, P = 0;
  std::vector<ctcext_path_sizes> sizes;
  ctcext_stats stats{};
};

static void release_dev(Dev& d) {
  (void)hipSetDevice(d.device);
  if (d.own_stream) (void)hipStreamSynchronize(d.own_stream);
  DevBuf* bufs[] = {&d.x, &d.sl, &d.norm, &d.prep, &d.rec, &d.foff, &d.item, &d.top_pos, &d.top_kind, &d.logp,
                    &d.seq, &d.len, &d.phase, &d.sctab, &d.gstate};
  for (DevBuf* b : bufs) b->release();
  for (auto& ev : d.ev)
    if (ev) (void)hipEventDestroy(ev);
  if (d.own_stream) (void)hipStreamDestroy(d.own_stream);
  d.own_stream = nullptr;
}

// The LDS-resident fast tier: the 8-byte record's limits and the LDS carve.
static int32_t max_beam_width(int64_t num_classes, int32_t dtype, bool scored) {
  const int ts = dtype == CTCEXT_F64 ? 8 : 4;
  if (num_classes > ctcx::kMaxRecClasses) return 0;
  int lo = 0;
  for (int w = 1; w <= ctcx::kMaxRecBeam; ++w)
    if (ctcx::decode_lds_bytes(w, num_classes, ts, scored) <= ctcx::kLdsBytes) lo = w;
  return lo;
}
static bool use_gstate(const ctcext_decode_args* a) {
  return (a->flags & CTCEXT_FLAG_GLOBAL_STATE) ||
         a->beam_width > max_beam_width(a->num_classes, a->dtype, a->scorer != CTCEXT_SCORER_BASE);
}

extern "C" int32_t ctcext_max_beam_width(int64_t num_classes, int32_t dtype) {
  return max_beam_width(num_classes, dtype, false);
}

extern "C" int ctcext_create_sharded(const int* devices, int n_devices, ctcext_decoder** out) {
  if (!out || !devices || n_devices < 1) return fail(CTCEXT_INVALID_ARGUMENT, "null argument or no devices");
  DeviceGuard guard;
  int n = 0;
  HIP_OR_FAIL(hipGetDeviceCount(&n));
  for (int i = 0; i < n_devices; ++i)
    if (devices[i] < 0 || devices[i] >= n) return fail(CTCEXT_INVALID_ARGUMENT, "invalid device ordinal");
  ctcext_decoder* d = new ctcext_decoder();
  d->devs.resize((size_t)n_devices);
  for (int i = 0; i < n_devices; ++i) {
    Dev& v = d->devs[(size_t)i];
    v.device = devices[i];
    hipError_t e = hipSetDevice(v.device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&v.own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      for (int j = 0; j < i; ++j) release_dev(d->devs[(size_t)j]);
      delete d;
      return fail(CTCEXT_INTERNAL, std::string("HIP error: ") + hipGetErrorString(e));
    }
    for (auto& ev : v.ev) (void)hipEventCreate(&ev);
    // the shard inputs and the gathered walks move between the root and this
    // device by peer copies (xGMI); "already enabled" is fine
    if (v.device != devices[0]) {
      int ok = 0;
      (void)hipDeviceCanAccessPeer(&ok, v.device, devices[0]);
      if (ok) {
        (void)hipDeviceEnablePeerAccess(devices[0], 0);
        (void)hipSetDevice(devices[0]);
        (void)hipDeviceEnablePeerAccess(v.device, 0);
      }
      (void)hipGetLastError();
    }
  }
  *out = d;
  g_err.clear();
  return CTCEXT_OK;
}

extern "C" int ctcext_create(int device, ctcext_decoder** out) { return ctcext_create_sharded(&device, 1, out); }

extern "C" void ctcext_destroy(ctcext_decoder* d) {
  if (!d) return;
  DeviceGuard guard;
  (void)hipSetDevice(d->devs[0].device);
  DevBuf* bufs[] = {&d->off, &d->res, &d->ptrs, &d->out_idx, &d->out_val};
  for (DevBuf* b : bufs) b->release();
  d->h_item.release();
  d->h_res.release();
  d->h_kind.release();
  for (Dev& v : d->devs) release_dev(v);
  delete d;
}

extern "C" const char* ctcext_last_error(void) { return g_err.c_str(); }

extern "C" int ctcext_phase_counters(ctcext_decoder* d, uint64_t* out, int64_t n) {
  if (!d || !out) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  Dev& r = d->devs[0];
  if (!r.phase.p) return fail(CTCEXT_FAILED_PRECONDITION, "no CTCEXT_FLAG_PHASES decode yet");
  if (n < 0 || 8 * (size_t)n > r.phase.cap) return fail(CTCEXT_INVALID_ARGUMENT, "n exceeds the counter buffer");
  DeviceGuard guard;
  HIP_OR_FAIL(hipSetDevice(r.device));
  HIP_OR_FAIL(hipMemcpy(out, r.phase.p, 8 * (size_t)n, hipMemcpyDeviceToHost));
  return CTCEXT_OK;
}

extern "C" int ctcext_row_facts(ctcext_decoder* d, const void* x, int32_t dtype, int64_t max_time, int64_t batch,
                                int64_t num_classes, int32_t blank_index, const int32_t* seq_len, void* prep,
                                void* norm, int64_t* row_bytes) {
  if (!d || !row_bytes) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  if (dtype != CTCEXT_F32 && dtype != CTCEXT_F64) return fail(CTCEXT_INVALID_ARGUMENT, "dtype");
  if (max_time < 0 || batch < 0 || num_classes <= 64 || blank_index < 0 || blank_index >= num_classes)
    return fail(CTCEXT_INVALID_ARGUMENT, "the pre-pass runs for num_classes > 64 and a blank index inside it");
  const int ts = dtype == CTCEXT_F64 ? 8 : 4;
  *row_bytes = (int64_t)ctcx::prep_row_bytes(num_classes, ts);
  if (!prep) return CTCEXT_OK;   // the size query
  if (!x || !seq_len || !norm) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  Dev& r = d->devs[0];
  DeviceGuard guard;
  HIP_OR_FAIL(hipSetDevice(r.device));
  const hipStream_t st = r.own_stream;
  if (dtype == CTCEXT_F64)
    HIP_OR_FAIL(ctcx::launch_row_prep<double>((const double*)x, seq_len, (char*)prep, (double*)norm, max_time, batch,
                                              num_classes, batch, blank_index, st));
  else
    HIP_OR_FAIL(ctcx::launch_row_prep<float>((const float*)x, seq_len, (char*)prep, (float*)norm, max_time, batch,
                                             num_classes, batch, blank_index, st));
  HIP_OR_FAIL(hipStreamSynchronize(st));
  return CTCEXT_OK;
}

// Frozen at the ABI-4 struct (every field before helper_redecodes): a binary
// built against that header passes a struct of that size, and a copy of the
// grown struct would write past it.  Fields added since are read through
// ctcext_get_stats_sized only.
extern "C" int ctcext_get_stats(ctcext_decoder* d, ctcext_stats* s) {
  return ctcext_get_stats_sized(d, s, offsetof(ctcext_stats, helper_redecodes));
}

// The struct has grown by appending fields (ctcext.h); a caller built against
// an older header passes its own sizeof and receives that prefix only.
extern "C" int ctcext_get_stats_sized(ctcext_decoder* d, ctcext_stats* s, size_t size) {
  if (!d || !s) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  ctcext_stats v = d->stats;
  v.n_devices = (int32_t)d->devs.size();
  memcpy(s, &v, std::min(size, sizeof(ctcext_stats)));
  return CTCEXT_OK;
}

extern "C" int32_t ctcext_abi_version(void) { return CTCEXT_ABI_VERSION; }

// ---------------------------------------------------------------------------
// Validation, in the reference's order (kernels.cc:97-139), host only.

// The op definition's attribute constraints (ops.cc:10-17) and the input
// shapes (kernels.cc:109-130).
static int validate_shapes(const ctcext_decode_args* a) {
  if (!a) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  if (a->dtype != CTCEXT_F32 && a->dtype != CTCEXT_F64)
    return fail(CTCEXT_INVALID_ARGUMENT, "dtype must be float32 or float64");
  if (a->beam_width < 1)
    return fail(CTCEXT_INVALID_ARGUMENT, "Value for attr 'beam_width' of " + std::to_string(a->beam_width) +
                                             " must be at least minimum 1");
  if (a->top_paths < 1)
    return fail(CTCEXT_INVALID_ARGUMENT, "Value for attr 'top_paths' of " + std::to_string(a->top_paths) +
                                             " must be at least minimum 1");
  if (a->inputs_dims != 3) return fail(CTCEXT_INVALID_ARGUMENT, "inputs is not a 3-Tensor");
  const int64_t T_ = a->max_time, B = a->batch_size, C = a->num_classes;
  if (T_ < 0 || B < 0 || C < 0) return fail(CTCEXT_INVALID_ARGUMENT, "inputs has a negative dimension");
  if (T_ == 0) return fail(CTCEXT_INVALID_ARGUMENT, "max_time is 0");
  if (a->sequence_length_dims != 1) return fail(CTCEXT_INVALID_ARGUMENT, "sequence_length is not a vector");
  if (a->sequence_length_size != B)
    return fail(CTCEXT_FAILED_PRECONDITION, "len(sequence_length) != batch_size.  len(sequence_length):  " +
                                                std::to_string(a->sequence_length_size) +
                                                " batch_size: " + std::to_string(B));
  if (B > 0 && (!a->inputs || !a->sequence_length)) return fail(CTCEXT_INVALID_ARGUMENT, "null input pointer");
  if (a->scorer != CTCEXT_SCORER_BASE && a->scorer != CTCEXT_SCORER_BIGRAM)
    return fail(CTCEXT_INVALID_ARGUMENT, "unknown beam scorer");
  if (a->scorer == CTCEXT_SCORER_BIGRAM && B > 0 && !a->scorer_table)
    return fail(CTCEXT_INVALID_ARGUMENT, "bigram beam scorer without a table");
  return CTCEXT_OK;
}

// The bigram table's entries must be log-probabilities: <= 0 and not NaN
// (exact_step's skipping bounds a child's score by its parent's total).
template <typename T>
static int check_table_t(const T* t, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    if (!(t[i] <= T(0)))
      return fail(CTCEXT_INVALID_ARGUMENT, "beam scorer table entries must be log-probabilities (<= 0)");
  return CTCEXT_OK;
}
static int check_table(const ctcext_decode_args* a, const void* host_table) {
  if (a->scorer != CTCEXT_SCORER_BIGRAM || a->batch_size == 0) return CTCEXT_OK;
  const int64_t n = (a->num_classes + 1) * a->num_classes;
  return a->dtype == CTCEXT_F64 ? check_table_t((const double*)host_table, n)
                                : check_table_t((const float*)host_table, n);
}

// kernels.cc:133-139
static int check_lengths(const int32_t* hsl, int64_t B, int64_t T_) {
  for (int64_t b = 0; b < B; ++b)
    if (!(hsl[b] <= T_))
      return fail(CTCEXT_FAILED_PRECONDITION, "sequence_length(" + std::to_string(b) + ") <= " + std::to_string(T_));
  return CTCEXT_OK;
}

// What the reference leaves unchecked or raises per item, and this library's
// own limits.
static int check_limits(const ctcext_decode_args* a) {
  const int64_t B = a->batch_size, C = a->num_classes;
  if (B == 0) return CTCEXT_OK;
  // the reference reads out of bounds here (no check); this library refuses
  if (a->blank_index < 0 || a->blank_index >= C)
    return fail(CTCEXT_INVALID_ARGUMENT, "blank_index out of range [0, num_classes)");
  // decoder.h:237-239 — raised by the first item's TopPaths
  if (a->top_paths > a->beam_width) return fail(CTCEXT_INVALID_ARGUMENT, "requested more paths than the beam width.");
  // every shape decodes (the global-state tier takes what the LDS tier cannot);
  // this library's int32 positions and labels bound it
  if (C > INT32_MAX / 2 || a->beam_width > (1 << 28))
    return fail(CTCEXT_UNIMPLEMENTED, "num_classes or beam_width beyond this library's 32-bit indices");
  return CTCEXT_OK;
}

extern "C" int ctcext_validate(const ctcext_decode_args* a) {
  int rc = validate_shapes(a);
  if (rc != CTCEXT_OK) return rc;
  if (!a->inputs_on_device) {
    rc = check_lengths(a->sequence_length, a->batch_size, a->max_time);
    if (rc != CTCEXT_OK) return rc;
  }
  rc = check_limits(a);
  if (rc == CTCEXT_OK && !a->inputs_on_device) rc = check_table(a, a->scorer_table);
  if (rc == CTCEXT_OK) g_err.clear();
  return rc;
}

// ---------------------------------------------------------------------------
// Decode.

// Contiguous shards balanced by sum(max(seq_len, 0)): shard i
// ends at the first item whose running sum reaches (i + 1) / n of the total.
static void shard_bounds(const std::vector<int32_t>& hsl, int n, std::vector<int64_t>& lo) {
  const int64_t B = (int64_t)hsl.size();
  lo.assign((size_t)n + 1, B);
  lo[0] = 0;
  int64_t tot = 0;
  for (int32_t v : hsl) tot += v > 0 ? v : 0;
  if (tot == 0) {   // no frames anywhere: split by count
    for (int i = 1; i < n; ++i) lo[(size_t)i] = B * i / n;
    return;
  }
  int64_t run = 0, b = 0;
  for (int i = 1; i < n; ++i) {
    const int64_t goal = (tot * i + n - 1) / n;
    while (b < B && run < goal) {
      const int32_t v = hsl[(size_t)b];
      run += v > 0 ? v : 0;
      ++b;
    }
    lo[(size_t)i] = b;
  }
}

// Enqueues norm + decode + traceback of one shard on its device's stream.
// x/sl point at the shard's first item; xstride is items per frame in x.
template <typename T>
static int enqueue_shard(ctcext_decoder* d, Dev& v, bool root, const ctcext_decode_args* a, const T* x,
                         int64_t xstride, const int32_t* sl, int helper_mode) {
  const int64_t T_ = a->max_time, C = a->num_classes, B = d->B, Bs = v.nb;
  const int W = a->beam_width, P = a->top_paths;
  const bool prof = (a->flags & CTCEXT_FLAG_PROFILE) != 0;
  const int64_t Bo = root ? B : Bs;   // the root's walk buffers hold the whole batch
  hipStream_t s = v.s;
  HIP_OR_FAIL(v.norm.ensure(sizeof(T) * (size_t)(T_ * Bs)));
  HIP_OR_FAIL(v.rec.ensure(sizeof(ctcx::Rec) * (size_t)(Bs * T_ * W)));
  HIP_OR_FAIL(v.item.ensure(sizeof(ctcx::ItemOut) * (size_t)Bo));
  HIP_OR_FAIL(v.top_pos.ensure(4 * (size_t)(Bs * P)));
  HIP_OR_FAIL(v.top_kind.ensure(4 * (size_t)(Bo * P)));
  HIP_OR_FAIL(v.logp.ensure(sizeof(T) * (size_t)(Bo * P)));
  HIP_OR_FAIL(v.seq.ensure(4 * (size_t)(Bo * P * 2 * T_)));
  HIP_OR_FAIL(v.len.ensure(4 * (size_t)(Bo * P * 2)));

  const bool gs = use_gstate(a);
  const bool scored = a->scorer != CTCEXT_SCORER_BASE;
  if (gs) {
    // the global-state tier: 16-byte records, the beam state in HBM
    HIP_OR_FAIL(v.rec.ensure(sizeof(ctcx::Rec16) * (size_t)(Bs * T_ * W)));
    HIP_OR_FAIL(v.gstate.ensure(ctcx::gstate_bytes(W, (int)sizeof(T), scored) * (size_t)Bs));
  } else if (C > 64) {
    HIP_OR_FAIL(v.prep.ensure(ctcx::prep_row_bytes(C, (int)sizeof(T)) * (size_t)(T_ * Bs)));
  }

  if (prof) HIP_OR_FAIL(hipEventRecord(v.ev[0], s));
  if (!gs && C > 64) {
    // large C: the normaliser and the row facts the decode kernel reads per
    // frame, one parallel pre-pass
    HIP_OR_FAIL(ctcx::launch_row_prep<T>(x, sl, (char*)v.prep.p, (T*)v.norm.p, T_, Bs, C, xstride,
                                         a->blank_index, s));
  } else {
    HIP_OR_FAIL(ctcx::launch_row_norm<T>(x, sl, (T*)v.norm.p, T_, Bs, C, xstride, s));
  }
  if (prof) HIP_OR_FAIL(hipEventRecord(v.ev[1], s));

  ctcx::DecodeParams<T> p{};
  p.x = x;
  p.norm = (const T*)v.norm.p;
  p.seq_len = sl;
  p.Tmax = T_; p.B = Bs; p.C = C; p.xstride = xstride;
  p.W = W; p.P = P; p.blank = a->blank_index; p.blank_label = a->blank_label;
  // num_classes == 1 (the blank alone): no label is ever offered, and the
  // fast paths' offer arithmetic divides by C - 1, so every frame takes the
  // literal path (the reference's own loops, decoder.h:146-209, then empty)
  p.force_literal = ((a->flags & CTCEXT_FLAG_FORCE_LITERAL) || C < 2) ? 1 : 0;
  p.rec = (ctcx::Rec*)v.rec.p;
  p.item = (ctcx::ItemOut*)v.item.p;
  p.top_pos = (int32_t*)v.top_pos.p;
  p.top_kind = (int32_t*)v.top_kind.p;
  p.log_prob = (T*)v.logp.p;
  p.prof = nullptr;
  p.scorer_tab = nullptr;
  p.prep = (const char*)v.prep.p;
  if (a->scorer == CTCEXT_SCORER_BIGRAM) {   // each device reads its own copy
    const size_t tb = (size_t)((C + 1) * C) * sizeof(T);
    HIP_OR_FAIL(v.sctab.ensure(tb));
    HIP_OR_FAIL(hipMemcpyAsync(v.sctab.p, a->scorer_table, tb, hipMemcpyDefault, s));
    p.scorer_tab = (const T*)v.sctab.p;
  }
  if (a->flags & CTCEXT_FLAG_PHASES) {
    HIP_OR_FAIL(v.phase.ensure(8 * ctcx::kPhaseN * (size_t)Bs));
    p.prof = (uint64_t*)v.phase.p;
  }
  // the host checked the shapes the kernel's grid and LDS carve assume
  if (Bs > 0x7fffffffLL || (!gs && (W > ctcx::kMaxRecBeam || C > ctcx::kMaxRecClasses)))
    return fail(CTCEXT_INTERNAL, "shard shape outside the kernel's limits");
  v.ring = 0;
  // the two-wave kernel: decided once here (the shape's kind, or none when
  // helper_off), then the ring, the kernel and the traceback's record format
  // all follow p.helper
  const int hk = gs ? 0 : ctcx::helper_kind<T>(p, helper_mode);
  p.test_flags = (a->flags & CTCEXT_FLAG_TEST_HELPER_DEAD) ? ctcx::kTestHelperDead : 0;
  // the record ring: asked for, or the default of the score-table two-wave kernel
  const bool ring = (a->flags & (CTCEXT_FLAG_RECORD_RING | CTCEXT_FLAG_RING_MIN)) ||
                    (!(a->flags & CTCEXT_FLAG_NO_RING) && ctcx::helper_rec32(hk, C));
  if (!gs && ring) {
    if (v.cus == 0 && hipDeviceGetAttribute(&v.cus, hipDeviceAttributeMultiprocessorCount, v.device) != hipSuccess)
      v.cus = 1;
    // ring frames: up to 128 (cfg3: 128 frames write 13.96M records per launch
    // instead of 64 frames' 20.86M, for +0.4% decode time, same box:
    // profiles/r5s_ring_frames.txt); CTCEXT_RING_FRAMES (diagnostics) another cap
    const char* rc = getenv("CTCEXT_RING_FRAMES");
    const int cap = (a->flags & CTCEXT_FLAG_RING_MIN) ? 8 : (rc && atoi(rc) >= 8) ? std::min(atoi(rc), 256) : 128;
    p.ring = v.ring = ctcx::ring_frames<T>(p, v.cus, cap, hk);
    if (p.ring > 0) {
      HIP_OR_FAIL(v.foff.ensure(4 * (size_t)(Bs * T_)));
      p.foff = (int32_t*)v.foff.p;
    }
  }
  p.helper = v.helper = ctcx::use_helper_kernel<T>(p, hk);
  if (gs) {
    p.gstate = (char*)v.gstate.p;
    p.gstate_stride = (int64_t)ctcx::gstate_bytes(W, (int)sizeof(T), scored);
    HIP_OR_FAIL(ctcx_gstate_launch_decode(&p, sizeof(T) == 8, scored, s));
  } else {
    HIP_OR_FAIL(ctcx::launch_decode<T>(p, s));
  }
  if (prof) HIP_OR_FAIL(hipEventRecord(v.ev[2], s));

  ctcx::TraceParams tp{};
  tp.rec = p.rec; tp.item = p.item; tp.seq_len = sl; tp.top_pos = p.top_pos; tp.top_kind = p.top_kind;
  tp.Tmax = T_; tp.B = Bs; tp.W = W; tp.P = P; tp.merge = a->merge_repeated ? 1 : 0;
  tp.blank_label = a->blank_label;
  tp.rec_fmt = gs ? ctcx::kRecFmt128 : ctcx::helper_rec32(v.helper, C) ? ctcx::kRecFmt32 : ctcx::kRecFmt64;
  v.rec_bytes = tp.rec_fmt == ctcx::kRecFmt128 ? 16 : tp.rec_fmt == ctcx::kRecFmt32 ? 4 : 8;
  tp.foff = p.foff;
  tp.seq = (int32_t*)v.seq.p;
  tp.len = (int32_t*)v.len.p;
  tp.len_stride = Bo;
  HIP_OR_FAIL(ctcx::launch_traceback(tp, s));
  if (prof) HIP_OR_FAIL(hipEventRecord(v.ev[3], s));
  return CTCEXT_OK;
}

template <typename T>
static int run_decode(ctcext_decoder* d, const ctcext_decode_args* a, const std::vector<int32_t>& hsl,
                      hipStream_t root_stream, int helper_mode) {
  const int64_t T_ = a->max_time, B = a->batch_size, C = a->num_classes;
  const int P = a->top_paths;
  const int ts = (int)sizeof(T);
  const int nd = (int)d->devs.size();
  Dev& root = d->devs[0];
  std::vector<int64_t> lo;
  shard_bounds(hsl, nd, lo);

  // 1. inputs to every device, then norm + decode + traceback, all async
  for (int i = 0; i < nd; ++i) {
    Dev& v = d->devs[(size_t)i];
    v.lo = lo[(size_t)i];
    v.nb = lo[(size_t)i + 1] - lo[(size_t)i];
    v.s = (i == 0) ? root_stream : v.own_stream;
    if (v.nb == 0 && i > 0) continue;
    HIP_OR_FAIL(hipSetDevice(v.device));
    const T* x;
    const int32_t* sl;
    int64_t xstride;
    if (i == 0 && a->inputs_on_device) {   // the root's shard is read in place
      x = (const T*)a->inputs;
      xstride = B;
      sl = a->sequence_length;
    } else if (v.nb == 0) {
      // an empty root shard (B < n_devices, no frames anywhere): nothing to
      // copy; enqueue_shard only sizes the root's whole-batch buffers and
      // launches no kernel over zero items
      x = nullptr;
      xstride = 0;
      sl = nullptr;
    } else {
      const size_t row = (size_t)v.nb * (size_t)C * ts;
      HIP_OR_FAIL(v.x.ensure(row * (size_t)T_ + 16));
      HIP_OR_FAIL(v.sl.ensure(4 * (size_t)v.nb + 16));
      const char* src = (const char*)a->inputs + (size_t)v.lo * (size_t)C * ts;
      if (v.nb == B) {
        HIP_OR_FAIL(hipMemcpyAsync(v.x.p, src, row * (size_t)T_, hipMemcpyDefault, v.s));
      } else {
        // a [T][nb][C] window of the [T][B][C] tensor: T rows of nb*C values
        HIP_OR_FAIL(hipMemcpy2DAsync(v.x.p, row, src, (size_t)B * (size_t)C * ts, row, (size_t)T_,
                                     hipMemcpyDefault, v.s));
      }
      HIP_OR_FAIL(hipMemcpyAsync(v.sl.p, hsl.data() + v.lo, 4 * (size_t)v.nb, hipMemcpyHostToDevice, v.s));
      x = (const T*)v.x.p;
      xstride = v.nb;
      sl = (const int32_t*)v.sl.p;
    }
    int rc = enqueue_shard<T>(d, v, i == 0, a, x, xstride, sl, helper_mode);
    if (rc != CTCEXT_OK) return rc;
  }

  // 2. wait for every shard; gather the per-item results to the root
  HIP_OR_FAIL(d->h_item.ensure(sizeof(ctcx::ItemOut) * (size_t)B + 16));
  HIP_OR_FAIL(d->h_res.ensure(8 * (size_t)(P * 4) + 16));
  for (int i = nd - 1; i >= 0; --i) {
    Dev& v = d->devs[(size_t)i];
    if (v.nb == 0 && i > 0) continue;
    HIP_OR_FAIL(hipSetDevice(v.device));
    HIP_OR_FAIL(hipStreamSynchronize(v.s));
  }
  HIP_OR_FAIL(hipSetDevice(root.device));
  hipStream_t s = root.s;
  for (int i = 1; i < nd; ++i) {   // peer copies (xGMI) into the root's whole-batch buffers
    Dev& v = d->devs[(size_t)i];
    if (v.nb == 0) continue;
    const size_t per = (size_t)P * 2 * (size_t)T_ * 4;
    HIP_OR_FAIL(hipMemcpyAsync((char*)root.seq.p + (size_t)v.lo * per, v.seq.p, (size_t)v.nb * per,
                               hipMemcpyDefault, s));
    for (int k = 0; k < 2 * P; ++k)
      HIP_OR_FAIL(hipMemcpyAsync((int32_t*)root.len.p + (size_t)k * B + v.lo, (int32_t*)v.len.p + (size_t)k * v.nb,
                                 4 * (size_t)v.nb, hipMemcpyDefault, s));
    HIP_OR_FAIL(hipMemcpyAsync((int32_t*)root.top_kind.p + (size_t)v.lo * P, v.top_kind.p, 4 * (size_t)(v.nb * P),
                               hipMemcpyDefault, s));
    HIP_OR_FAIL(hipMemcpyAsync((char*)root.logp.p + (size_t)(v.lo * P) * ts, v.logp.p, (size_t)(v.nb * P) * ts,
                               hipMemcpyDefault, s));
    HIP_OR_FAIL(hipMemcpyAsync((ctcx::ItemOut*)root.item.p + v.lo, v.item.p, sizeof(ctcx::ItemOut) * (size_t)v.nb,
                               hipMemcpyDefault, s));
  }
  // 3. SparseTensor sizes over the whole batch
  HIP_OR_FAIL(d->off.ensure(8 * (size_t)(B * P * 2)));
  HIP_OR_FAIL(d->res.ensure(8 * (size_t)(P * 4)));
  HIP_OR_FAIL(d->h_kind.ensure(4 * (size_t)(B * P) + 16));
  HIP_OR_FAIL(ctcx::launch_scan((const int32_t*)root.len.p, (int64_t*)d->off.p, (int64_t*)d->res.p, B, P, s));
  HIP_OR_FAIL(hipMemcpyAsync(d->h_item.p, root.item.p, sizeof(ctcx::ItemOut) * (size_t)B, hipMemcpyDeviceToHost, s));
  HIP_OR_FAIL(hipMemcpyAsync(d->h_res.p, d->res.p, 8 * (size_t)(P * 4), hipMemcpyDeviceToHost, s));
  HIP_OR_FAIL(hipMemcpyAsync(d->h_kind.p, root.top_kind.p, 4 * (size_t)(B * P), hipMemcpyDeviceToHost, s));
  HIP_OR_FAIL(hipStreamSynchronize(s));

  d->stats = ctcext_stats{};
  d->stats.tier = use_gstate(a) ? 1 : 0;
  d->stats.ring_frames = root.ring;
  d->stats.record_bytes = root.rec_bytes;
  d->stats.helper = root.helper;
  if (a->flags & CTCEXT_FLAG_PROFILE) {
    for (int i = 0; i < nd; ++i) {
      Dev& v = d->devs[(size_t)i];
      if (v.nb == 0) continue;
      float ms = 0;
      (void)hipEventElapsedTime(&ms, v.ev[0], v.ev[1]);
      d->stats.norm_kernel_ms = std::max(d->stats.norm_kernel_ms, (double)ms);
      (void)hipEventElapsedTime(&ms, v.ev[1], v.ev[2]);
      d->stats.decode_kernel_ms = std::max(d->stats.decode_kernel_ms, (double)ms);
      (void)hipEventElapsedTime(&ms, v.ev[2], v.ev[3]);
      d->stats.traceback_ms = std::max(d->stats.traceback_ms, (double)ms);
    }
  }
  const ctcx::ItemOut* io = (const ctcx::ItemOut*)d->h_item.p;
  for (int64_t b = 0; b < B; ++b) {
    d->stats.literal_frames += io[b].literal_steps;
    d->stats.literal_nonfinite += io[b].why_nonfinite;
    d->stats.literal_fill += io[b].why_fill;
    d->stats.duplicate_frames += io[b].dup_frames;
    d->stats.records_written += io[b].records;
  }
  bool dead = false;
  for (int64_t b = 0; b < B; ++b) dead |= io[b].pad != 0;
  if (dead) {
    // a two-wave kernel's hand-over wait ran out of time (~1 s; never in a
    // correct run): its items' results are incomplete.  The call is decoded
    // again with the one-wave kernels, unless the caller asked to fail
    if (helper_mode == ctcx::kHelperNone || (a->flags & CTCEXT_FLAG_HELPER_STRICT))
      return fail(CTCEXT_INTERNAL, "decode kernel: a helper-wave hand-over wait timed out");
    const int rc = run_decode<T>(d, a, hsl, root_stream, ctcx::kHelperNone);
    d->stats.helper_redecodes += 1;
    return rc;
  }
  // TopPaths (decoder.h:240-243) fails on the first item with too few leaves
  for (int64_t b = 0; b < B; ++b)
    if (io[b].n_leaves < P) return fail(CTCEXT_INVALID_ARGUMENT, "Less leaves in the beam search than requested.");
  const int32_t* kinds = (const int32_t*)d->h_kind.p;
  for (int64_t q = 0; q < B * P; ++q) d->stats.no_label_paths += (kinds[q] < 0) ? 1 : 0;
  (void)C;
  return CTCEXT_OK;
}

extern "C" int ctcext_decode_sharded(ctcext_decoder* d, const ctcext_decode_args* a, ctcext_path_sizes* sizes) {
  if (!d || !a) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  d->have = false;
  int rc = validate_shapes(a);
  if (rc != CTCEXT_OK) return rc;
  DeviceGuard guard;
  Dev& root = d->devs[0];
  HIP_OR_FAIL(hipSetDevice(root.device));
  const int64_t T_ = a->max_time, B = a->batch_size;
  hipStream_t s = a->stream ? (hipStream_t)a->stream : root.own_stream;

  // sequence_length is read on the host for validation (kernels.cc:134-139)
  // and for the shard split
  std::vector<int32_t> hsl((size_t)B);
  if (B > 0) {
    if (a->inputs_on_device) {
      HIP_OR_FAIL(hipMemcpyAsync(hsl.data(), a->sequence_length, 4 * (size_t)B, hipMemcpyDeviceToHost, s));
      HIP_OR_FAIL(hipStreamSynchronize(s));
    } else {
      memcpy(hsl.data(), a->sequence_length, 4 * (size_t)B);
    }
  }
  rc = check_lengths(hsl.data(), B, T_);
  if (rc == CTCEXT_OK) rc = check_limits(a);
  if (rc == CTCEXT_OK && a->scorer == CTCEXT_SCORER_BIGRAM && B > 0) {
    if (a->inputs_on_device) {
      const size_t tb = (size_t)((a->num_classes + 1) * a->num_classes) * (a->dtype == CTCEXT_F64 ? 8 : 4);
      std::vector<char> ht(tb);
      HIP_OR_FAIL(hipMemcpy(ht.data(), a->scorer_table, tb, hipMemcpyDeviceToHost));
      rc = check_table(a, ht.data());
    } else {
      rc = check_table(a, a->scorer_table);
    }
  }
  if (rc != CTCEXT_OK) return rc;

  const int P = a->top_paths;
  d->B = B;
  d->sizes.assign((size_t)P, ctcext_path_sizes{0, 0, 0, 0});
  d->stats = ctcext_stats{};
  if (B > 0) {
    // CTCEXT_HELPER (diagnostics, read once per call): 0 the one-wave kernels,
    // 1 the score table / unscored gather queue, 3 the scored gather queue
    // (beams <= 128; the default), 4 the scored queue for beams <= 256
    const char* hv = getenv("CTCEXT_HELPER");
    const int helper_mode = !hv || !hv[0] ? kDefaultHelperMode
                            : hv[0] == '0' ? ctcx::kHelperNone
                            : hv[0] == '3' ? ctcx::kHelperScored
                            : hv[0] == '4' ? ctcx::kHelperScoredWide : ctcx::kHelperLegacy;
    rc = (a->dtype == CTCEXT_F32) ? run_decode<float>(d, a, hsl, s, helper_mode)
                                  : run_decode<double>(d, a, hsl, s, helper_mode);
    if (rc != CTCEXT_OK) return rc;
    const int64_t* r = (const int64_t*)d->h_res.p;
    for (int p = 0; p < P; ++p) {
      d->sizes[p].num_decoded = r[(p * 2 + 0) * 2];
      d->sizes[p].max_decoded = r[(p * 2 + 0) * 2 + 1];
      d->sizes[p].num_alignment = r[(p * 2 + 1) * 2];
      d->sizes[p].max_alignment = r[(p * 2 + 1) * 2 + 1];
    }
  }
  d->have = true;
  d->dtype = a->dtype;
  d->T = T_; d->C = a->num_classes; d->W = a->beam_width; d->P = P;
  root.s = s;
  if (sizes)
    for (int p = 0; p < P; ++p) sizes[p] = d->sizes[p];
  g_err.clear();
  return CTCEXT_OK;
}

extern "C" int ctcext_decode(ctcext_decoder* d, const ctcext_decode_args* a, ctcext_path_sizes* sizes) {
  return ctcext_decode_sharded(d, a, sizes);
}

extern "C" int ctcext_fetch(ctcext_decoder* d, const ctcext_outputs* o) {
  if (!d || !o) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  if (!d->have) return fail(CTCEXT_FAILED_PRECONDITION, "ctcext_fetch without a successful ctcext_decode");
  DeviceGuard guard;
  Dev& root = d->devs[0];
  HIP_OR_FAIL(hipSetDevice(root.device));
  hipStream_t s = root.s;
  const int P = d->P;
  const int64_t B = d->B;
  const int ts = d->dtype == CTCEXT_F64 ? 8 : 4;

  // shapes: {batch_size, max length} (kernels.cc:236-237, 253-254)
  std::vector<int64_t> shapes((size_t)P * 4);
  for (int p = 0; p < P; ++p) {
    shapes[p * 4 + 0] = B; shapes[p * 4 + 1] = d->sizes[p].max_decoded;
    shapes[p * 4 + 2] = B; shapes[p * 4 + 3] = d->sizes[p].max_alignment;
  }

  std::vector<int64_t*> idx((size_t)P * 2), val((size_t)P * 2);
  std::vector<size_t> off_in_stage((size_t)P * 2);
  if (o->outputs_on_device) {
    for (int p = 0; p < P; ++p) {
      idx[p * 2] = o->decoded_indices[p]; val[p * 2] = o->decoded_values[p];
      idx[p * 2 + 1] = o->alignment_indices[p]; val[p * 2 + 1] = o->alignment_values[p];
    }
  } else {
    // stage on the device, then copy down
    size_t tot = 0;
    for (int p = 0; p < P; ++p) {
      off_in_stage[p * 2] = tot; tot += (size_t)d->sizes[p].num_decoded;
      off_in_stage[p * 2 + 1] = tot; tot += (size_t)d->sizes[p].num_alignment;
    }
    HIP_OR_FAIL(d->out_idx.ensure(16 * tot + 16));
    HIP_OR_FAIL(d->out_val.ensure(8 * tot + 16));
    for (int k = 0; k < P * 2; ++k) {
      idx[k] = (int64_t*)d->out_idx.p + 2 * off_in_stage[k];
      val[k] = (int64_t*)d->out_val.p + off_in_stage[k];
    }
  }
  std::vector<int64_t*> both((size_t)P * 4);   // must outlive the async copy below
  if (B > 0) {
    HIP_OR_FAIL(d->ptrs.ensure(sizeof(int64_t*) * (size_t)P * 4));
    int64_t** dp = (int64_t**)d->ptrs.p;
    for (int k = 0; k < P * 2; ++k) { both[k] = idx[k]; both[P * 2 + k] = val[k]; }
    HIP_OR_FAIL(hipMemcpyAsync(dp, both.data(), sizeof(int64_t*) * (size_t)P * 4, hipMemcpyHostToDevice, s));
    ctcx::PackParams pp{};
    pp.seq = (const int32_t*)root.seq.p;
    pp.len = (const int32_t*)root.len.p;
    pp.off = (const int64_t*)d->off.p;
    pp.Tmax = d->T; pp.B = B; pp.P = P;
    pp.idx = dp;
    pp.val = dp + P * 2;
    HIP_OR_FAIL(ctcx::launch_pack(pp, s));
  }
  const hipMemcpyKind to_dev = o->outputs_on_device ? hipMemcpyHostToDevice : hipMemcpyHostToHost;
  for (int p = 0; p < P; ++p) {
    HIP_OR_FAIL(hipMemcpyAsync(o->decoded_shape[p], &shapes[p * 4], 16, to_dev, s));
    HIP_OR_FAIL(hipMemcpyAsync(o->alignment_shape[p], &shapes[p * 4 + 2], 16, to_dev, s));
  }
  if (B > 0) {
    HIP_OR_FAIL(hipMemcpyAsync(o->log_probability, root.logp.p, (size_t)(B * P) * ts,
                               o->outputs_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
    if (!o->outputs_on_device) {
      for (int p = 0; p < P; ++p) {
        const size_t nd = (size_t)d->sizes[p].num_decoded, na = (size_t)d->sizes[p].num_alignment;
        if (nd) {
          HIP_OR_FAIL(hipMemcpyAsync(o->decoded_indices[p], idx[p * 2], 16 * nd, hipMemcpyDeviceToHost, s));
          HIP_OR_FAIL(hipMemcpyAsync(o->decoded_values[p], val[p * 2], 8 * nd, hipMemcpyDeviceToHost, s));
        }
        if (na) {
          HIP_OR_FAIL(hipMemcpyAsync(o->alignment_indices[p], idx[p * 2 + 1], 16 * na, hipMemcpyDeviceToHost, s));
          HIP_OR_FAIL(hipMemcpyAsync(o->alignment_values[p], val[p * 2 + 1], 8 * na, hipMemcpyDeviceToHost, s));
        }
      }
    }
  }
  HIP_OR_FAIL(hipStreamSynchronize(s));
  g_err.clear();
  return CTCEXT_OK;
}

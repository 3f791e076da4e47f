// ctcext_capi.hip — host side of libctcext.so: validation, workspace, kernel
// orchestration and output transfer behind the C ABI in include/ctcext.h.
//
// Mirrors the reference op kernel (cc/kernels/ctc_ext_beam_search_decoder_kernels.cc):
//   ValidateInputsGenerateOutputs  :97-160  -> validate()
//   Compute batch/time loop        :67-90   -> ctcx_row_norm + ctcx_beam_decode
//   TopPaths errors                decoder.h:237-243
//   StoreAllDecodedSequences       :163-257 -> ctcx_traceback + ctcx_scan + ctcx_pack
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/ctcext.h"
#include "ctcx_kernels.h"

namespace ctcx {
template <typename T>
hipError_t launch_decode(const DecodeParams<T>& p, hipStream_t s);
template <typename T>
hipError_t launch_row_norm(const T* x, const int32_t* sl, T* norm, int64_t T_, int64_t B, int64_t C, hipStream_t s);
hipError_t launch_traceback(const TraceParams& tp, hipStream_t s);
hipError_t launch_scan(const int32_t* len, int64_t* off, int64_t* res, int64_t B, int P, hipStream_t s);
hipError_t launch_pack(const PackParams& pp, hipStream_t s);
}  // namespace ctcx

static thread_local std::string g_err;

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

}  // namespace

struct ctcext_decoder {
  int device = 0;
  hipStream_t own_stream = nullptr;
  // workspace
  DevBuf x, sl, norm, rec, item, top_pos, top_kind, logp, seq, len, off, res, ptrs, out_idx, out_val, phase;
  HostBuf h_item, h_res;
  hipEvent_t ev[6] = {};
  // state of the last successful decode (consumed by fetch)
  bool have = false;
  int dtype = 0;
  int64_t T = 0, B = 0, C = 0;
  int32_t W = 0, P = 0;
  hipStream_t stream = nullptr;
  std::vector<ctcext_path_sizes> sizes;
  ctcext_stats stats{};
};

static size_t lds_limit() { return ctcx::kLdsBytes; }

extern "C" int32_t ctcext_max_beam_width(int64_t num_classes, int32_t dtype) {
  const int ts = dtype == CTCEXT_F64 ? 8 : 4;
  int lo = 0;
  for (int w = 1; w <= 512; ++w)
    if (ctcx::decode_lds_bytes(w, num_classes, ts) <= lds_limit()) lo = w;
  return lo;
}

extern "C" int ctcext_create(int device, ctcext_decoder** out) {
  if (!out) return fail(CTCEXT_INVALID_ARGUMENT, "null output handle");
  int n = 0;
  HIP_OR_FAIL(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(CTCEXT_INVALID_ARGUMENT, "invalid device ordinal");
  HIP_OR_FAIL(hipSetDevice(device));
  ctcext_decoder* d = new ctcext_decoder();
  d->device = device;
  hipError_t e = hipStreamCreateWithFlags(&d->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete d;
    return fail(CTCEXT_INTERNAL, std::string("HIP error: ") + hipGetErrorString(e));
  }
  for (auto& ev : d->ev) (void)hipEventCreate(&ev);
  *out = d;
  g_err.clear();
  return CTCEXT_OK;
}

extern "C" void ctcext_destroy(ctcext_decoder* d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->own_stream) (void)hipStreamSynchronize(d->own_stream);
  DevBuf* bufs[] = {&d->x, &d->sl, &d->norm, &d->rec, &d->item, &d->top_pos, &d->top_kind, &d->logp,
                    &d->seq, &d->len, &d->off, &d->res, &d->ptrs, &d->out_idx, &d->out_val, &d->phase};
  for (DevBuf* b : bufs) b->release();
  d->h_item.release();
  d->h_res.release();
  for (auto& ev : d->ev)
    if (ev) (void)hipEventDestroy(ev);
  if (d->own_stream) (void)hipStreamDestroy(d->own_stream);
  delete d;
}

extern "C" const char* ctcext_last_error(void) { return g_err.c_str(); }

extern "C" int ctcext_phase_counters(ctcext_decoder* d, uint64_t* out, int64_t n) {
  if (!d || !out) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  if (!d->phase.p) return fail(CTCEXT_FAILED_PRECONDITION, "no CTCEXT_FLAG_PHASES decode yet");
  if (n < 0 || 8 * (size_t)n > d->phase.cap) return fail(CTCEXT_INVALID_ARGUMENT, "n exceeds the counter buffer");
  HIP_OR_FAIL(hipSetDevice(d->device));
  HIP_OR_FAIL(hipMemcpy(out, d->phase.p, 8 * (size_t)n, hipMemcpyDeviceToHost));
  return CTCEXT_OK;
}

extern "C" int ctcext_get_stats(ctcext_decoder* d, ctcext_stats* s) {
  if (!d || !s) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  *s = d->stats;
  return CTCEXT_OK;
}

template <typename T>
static int run_decode(ctcext_decoder* d, const ctcext_decode_args* a, const T* x, const int32_t* sl,
                      hipStream_t s) {
  const int64_t T_ = a->max_time, B = a->batch_size, C = a->num_classes;
  const int W = a->beam_width, P = a->top_paths;
  const bool prof = (a->flags & CTCEXT_FLAG_PROFILE) != 0;
  HIP_OR_FAIL(d->norm.ensure(sizeof(T) * (size_t)(T_ * B)));
  HIP_OR_FAIL(d->rec.ensure(sizeof(ctcx::Rec) * (size_t)(B * T_ * W)));
  HIP_OR_FAIL(d->item.ensure(sizeof(ctcx::ItemOut) * (size_t)B));
  HIP_OR_FAIL(d->top_pos.ensure(4 * (size_t)(B * P)));
  HIP_OR_FAIL(d->top_kind.ensure(4 * (size_t)(B * P)));
  HIP_OR_FAIL(d->logp.ensure(sizeof(T) * (size_t)(B * P)));
  HIP_OR_FAIL(d->seq.ensure(4 * (size_t)(B * P * 2 * T_)));
  HIP_OR_FAIL(d->len.ensure(4 * (size_t)(B * P * 2)));
  HIP_OR_FAIL(d->off.ensure(8 * (size_t)(B * P * 2)));
  HIP_OR_FAIL(d->res.ensure(8 * (size_t)(P * 4)));
  HIP_OR_FAIL(d->h_item.ensure(sizeof(ctcx::ItemOut) * (size_t)B + 16));
  HIP_OR_FAIL(d->h_res.ensure(8 * (size_t)(P * 4) + 16));

  if (prof) HIP_OR_FAIL(hipEventRecord(d->ev[0], s));
  HIP_OR_FAIL(ctcx::launch_row_norm<T>(x, sl, (T*)d->norm.p, T_, B, C, s));
  if (prof) HIP_OR_FAIL(hipEventRecord(d->ev[1], s));

  ctcx::DecodeParams<T> p{};
  p.x = x;
  p.norm = (const T*)d->norm.p;
  p.seq_len = sl;
  p.Tmax = T_; p.B = B; p.C = C;
  p.W = W; p.P = P; p.blank = a->blank_index; p.blank_label = a->blank_label;
  p.force_literal = (a->flags & CTCEXT_FLAG_FORCE_LITERAL) ? 1 : 0;
  p.rec = (ctcx::Rec*)d->rec.p;
  p.item = (ctcx::ItemOut*)d->item.p;
  p.top_pos = (int32_t*)d->top_pos.p;
  p.top_kind = (int32_t*)d->top_kind.p;
  p.log_prob = (T*)d->logp.p;
  p.prof = nullptr;
  if (a->flags & CTCEXT_FLAG_PHASES) {
    HIP_OR_FAIL(d->phase.ensure(8 * ctcx::kPhaseN * (size_t)B));
    p.prof = (uint64_t*)d->phase.p;
  }
  HIP_OR_FAIL(ctcx::launch_decode<T>(p, s));
  if (prof) HIP_OR_FAIL(hipEventRecord(d->ev[2], s));

  ctcx::TraceParams tp{};
  tp.rec = p.rec; tp.item = p.item; tp.seq_len = sl; tp.top_pos = p.top_pos; tp.top_kind = p.top_kind;
  tp.Tmax = T_; tp.B = B; tp.W = W; tp.P = P; tp.merge = a->merge_repeated ? 1 : 0;
  tp.blank_label = a->blank_label;
  tp.seq = (int32_t*)d->seq.p;
  tp.len = (int32_t*)d->len.p;
  HIP_OR_FAIL(ctcx::launch_traceback(tp, s));
  HIP_OR_FAIL(ctcx::launch_scan(tp.len, (int64_t*)d->off.p, (int64_t*)d->res.p, B, P, s));
  if (prof) HIP_OR_FAIL(hipEventRecord(d->ev[3], s));

  HIP_OR_FAIL(hipMemcpyAsync(d->h_item.p, d->item.p, sizeof(ctcx::ItemOut) * (size_t)B, hipMemcpyDeviceToHost, s));
  HIP_OR_FAIL(hipMemcpyAsync(d->h_res.p, d->res.p, 8 * (size_t)(P * 4), hipMemcpyDeviceToHost, s));
  HIP_OR_FAIL(hipStreamSynchronize(s));

  d->stats = ctcext_stats{};
  if (prof) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, d->ev[0], d->ev[1]); d->stats.norm_kernel_ms = ms;
    (void)hipEventElapsedTime(&ms, d->ev[1], d->ev[2]); d->stats.decode_kernel_ms = ms;
    (void)hipEventElapsedTime(&ms, d->ev[2], d->ev[3]); d->stats.traceback_ms = ms;
  }
  const ctcx::ItemOut* io = (const ctcx::ItemOut*)d->h_item.p;
  for (int64_t b = 0; b < B; ++b) {
    if (io[b].error)
      return fail(CTCEXT_INTERNAL,
                  "beam reached a state holding the same entry twice (only reachable with -inf "
                  "totals); not supported on the device path");
    d->stats.literal_frames += io[b].literal_steps;
    d->stats.literal_nonfinite += io[b].why_nonfinite;
    d->stats.literal_evict_tie += io[b].why_evict_tie;
    d->stats.literal_order_tie += io[b].why_order_tie;
  }
  // TopPaths (decoder.h:240-243) fails on the first item with too few leaves
  for (int64_t b = 0; b < B; ++b)
    if (io[b].n_leaves < P) return fail(CTCEXT_INVALID_ARGUMENT, "Less leaves in the beam search than requested.");
  return CTCEXT_OK;
}

extern "C" int ctcext_decode(ctcext_decoder* d, const ctcext_decode_args* a, ctcext_path_sizes* sizes) {
  if (!d || !a) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  d->have = false;
  HIP_OR_FAIL(hipSetDevice(d->device));
  if (a->dtype != CTCEXT_F32 && a->dtype != CTCEXT_F64)
    return fail(CTCEXT_INVALID_ARGUMENT, "dtype must be float32 or float64");
  if (a->beam_width < 1) return fail(CTCEXT_INVALID_ARGUMENT, "Value for attr 'beam_width' must be >= 1");
  if (a->top_paths < 1) return fail(CTCEXT_INVALID_ARGUMENT, "Value for attr 'top_paths' must be >= 1");
  const int64_t T_ = a->max_time, B = a->batch_size, C = a->num_classes;
  if (T_ < 0 || B < 0 || C < 0) return fail(CTCEXT_INVALID_ARGUMENT, "inputs is not a 3-Tensor");
  // kernels.cc:118-120
  if (T_ == 0) return fail(CTCEXT_INVALID_ARGUMENT, "max_time is 0");
  hipStream_t s = a->stream ? (hipStream_t)a->stream : d->own_stream;
  const int ts = a->dtype == CTCEXT_F64 ? 8 : 4;
  (void)ts;

  // sequence_length must be read on the host for validation (kernels.cc:134-139)
  std::vector<int32_t> hsl((size_t)B);
  if (B > 0) {
    if (a->inputs_on_device) {
      HIP_OR_FAIL(hipMemcpyAsync(hsl.data(), a->sequence_length, 4 * (size_t)B, hipMemcpyDeviceToHost, s));
      HIP_OR_FAIL(hipStreamSynchronize(s));
    } else {
      memcpy(hsl.data(), a->sequence_length, 4 * (size_t)B);
    }
  }
  for (int64_t b = 0; b < B; ++b)
    if (!(hsl[b] <= T_))
      return fail(CTCEXT_FAILED_PRECONDITION,
                  "sequence_length(" + std::to_string(b) + ") <= " + std::to_string(T_));
  if (B > 0 && (a->blank_index < 0 || a->blank_index >= C))
    return fail(CTCEXT_INVALID_ARGUMENT, "blank_index out of range [0, num_classes)");
  // decoder.h:237-239 — raised by the first item's TopPaths
  if (B > 0 && a->top_paths > a->beam_width)
    return fail(CTCEXT_INVALID_ARGUMENT, "requested more paths than the beam width.");
  if (B > 0 && C > ctcx::kMaxRecClasses)
    return fail(CTCEXT_UNIMPLEMENTED, "num_classes " + std::to_string(C) + " exceeds the back-pointer record format (max " +
                                          std::to_string(ctcx::kMaxRecClasses) + ")");
  if (B > 0 && a->beam_width > ctcext_max_beam_width(C, a->dtype))
    return fail(CTCEXT_UNIMPLEMENTED, "beam_width " + std::to_string(a->beam_width) + " with num_classes " +
                                          std::to_string(C) + " exceeds the LDS-resident beam state (max " +
                                          std::to_string(ctcext_max_beam_width(C, a->dtype)) + ")");

  const void* x = a->inputs;
  const int32_t* sl = a->sequence_length;
  if (!a->inputs_on_device && B > 0) {
    const size_t xb = (size_t)(T_ * B * C) * ts;
    HIP_OR_FAIL(d->x.ensure(xb));
    HIP_OR_FAIL(d->sl.ensure(4 * (size_t)B));
    HIP_OR_FAIL(hipMemcpyAsync(d->x.p, a->inputs, xb, hipMemcpyHostToDevice, s));
    HIP_OR_FAIL(hipMemcpyAsync(d->sl.p, hsl.data(), 4 * (size_t)B, hipMemcpyHostToDevice, s));
    x = d->x.p;
    sl = (const int32_t*)d->sl.p;
  }

  const int P = a->top_paths;
  d->sizes.assign((size_t)P, ctcext_path_sizes{0, 0, 0, 0});
  if (B > 0) {
    int rc = (a->dtype == CTCEXT_F32) ? run_decode<float>(d, a, (const float*)x, sl, s)
                                      : run_decode<double>(d, a, (const double*)x, sl, s);
    if (rc != CTCEXT_OK) return rc;
    const int64_t* r = (const int64_t*)d->h_res.p;
    for (int p = 0; p < P; ++p) {
      d->sizes[p].num_decoded = r[(p * 2 + 0) * 2];
      d->sizes[p].max_decoded = r[(p * 2 + 0) * 2 + 1];
      d->sizes[p].num_alignment = r[(p * 2 + 1) * 2];
      d->sizes[p].max_alignment = r[(p * 2 + 1) * 2 + 1];
    }
    // paths whose alignment is empty although the item had frames or not:
    // the reference prints "No label seq available" for each (host side)
    std::vector<int32_t> kinds((size_t)(B * P));
    HIP_OR_FAIL(hipMemcpy(kinds.data(), d->top_kind.p, 4 * (size_t)(B * P), hipMemcpyDeviceToHost));
    for (int32_t k : kinds) d->stats.no_label_paths += (k < 0) ? 1 : 0;
  }
  d->have = true;
  d->dtype = a->dtype;
  d->T = T_; d->B = B; d->C = C; d->W = a->beam_width; d->P = P;
  d->stream = s;
  if (sizes)
    for (int p = 0; p < P; ++p) sizes[p] = d->sizes[p];
  g_err.clear();
  return CTCEXT_OK;
}

extern "C" int ctcext_fetch(ctcext_decoder* d, const ctcext_outputs* o) {
  if (!d || !o) return fail(CTCEXT_INVALID_ARGUMENT, "null argument");
  if (!d->have) return fail(CTCEXT_FAILED_PRECONDITION, "ctcext_fetch without a successful ctcext_decode");
  HIP_OR_FAIL(hipSetDevice(d->device));
  hipStream_t s = d->stream;
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
    pp.seq = (const int32_t*)d->seq.p;
    pp.len = (const int32_t*)d->len.p;
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
    HIP_OR_FAIL(hipMemcpyAsync(o->log_probability, d->logp.p, (size_t)(B * P) * ts,
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

// ctcx_kernels.h — shared declarations between the HIP kernels
// (ctcx_decode.hip) and the C-ABI host layer (ctcext_capi.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// LDS pointers are declared in address space 3 so that every access through
// them compiles to ds_read/ds_write (a generic pointer kept in a struct would
// become a flat access).  Debug harnesses that run device code on the host
// define CTCX_LDS as empty.
#ifndef CTCX_LDS
#define CTCX_LDS __attribute__((address_space(3)))
#endif

namespace ctcx {

// CTCEXT_FLAG_PHASES counters per item: 0 row load, 1 recursion, 2 grow,
// 3 extract, 4 commit, 5 literal frames, 6 grow events, 7 frames, 8 offer
// scoring, 9 event loops, 10 heap pushes, 11 offer chunks, 12 accepted
// events, 13 heap pushes (count)
constexpr int kPhaseN = 32;   // [0, 24): wave 0, [24, 32): the helper wave (CTCX_PHASES)

constexpr uint32_t kBpRestart = 0xFFFFFFFEu;  // candidate started a new chain
constexpr uint32_t kBpNone = 0xFFFFFFFFu;     // no candidate of that kind

// One record per (item, frame, surviving beam), written in the beam's sorted
// position k (= its branch index next frame): 8 bytes, packed
//   bits  0..10  link = (src branch << 1) | is_new_child   (src < 512)
//   bits 11..26  label + 1 (the beam's last label; -1 at the root)
//   bits 27..38  best blank-ending alignment back-pointer (pos << 1 | kind),
//   bits 39..50  best label-ending one; 4094 = restart, 4095 = none.
// Valid for beam_width <= 512 and num_classes <= 65535 (both checked).
typedef uint64_t Rec;
__host__ __device__ inline uint64_t rec_bp12(uint32_t q) {
  return q >= kBpRestart ? (uint64_t)(q - kBpRestart + 4094u) : (uint64_t)q;
}
__host__ __device__ inline uint32_t rec_unbp12(uint64_t v) {
  return v >= 4094u ? kBpRestart + (uint32_t)(v - 4094u) : (uint32_t)v;
}
__host__ __device__ inline Rec rec_pack(uint32_t link, int label, uint32_t bp_blank, uint32_t bp_nblank) {
  return (uint64_t)link | ((uint64_t)(uint32_t)(label + 1) << 11) | (rec_bp12(bp_blank) << 27) |
         (rec_bp12(bp_nblank) << 39);
}
__host__ __device__ inline uint32_t rec_link(Rec r) { return (uint32_t)(r & 0x7FFu); }
__host__ __device__ inline int rec_label(Rec r) { return (int)((r >> 11) & 0xFFFFu) - 1; }
__host__ __device__ inline uint32_t rec_bp_blank(Rec r) { return rec_unbp12((r >> 27) & 0xFFFu); }
__host__ __device__ inline uint32_t rec_bp_nblank(Rec r) { return rec_unbp12((r >> 39) & 0xFFFu); }
constexpr int kMaxRecClasses = 65535;
constexpr int kMaxRecBeam = 512;

// The 4-byte record of the two-wave kernel (beam_width <= 128, num_classes <=
// 64): the same fields, narrower:
//   bits  0..7   link = (src branch << 1) | is_new_child   (src < 128)
//   bits  8..13  label (0..63; the root's -1 is stored as 63 and never read:
//                the root is never a new child and has no label-ending candidate)
//   bits 14..22  best blank-ending alignment back-pointer (pos << 1 | kind),
//   bits 23..31  best label-ending one; 256 = restart or none (the traceback
//                stops at either and never follows a candidate that is absent)
typedef uint32_t Rec32;
__host__ __device__ inline uint32_t rec32_bp9(uint32_t q) { return q >= kBpRestart ? 256u : q; }
__host__ __device__ inline Rec32 rec32_pack(uint32_t link, int label, uint32_t bp_blank, uint32_t bp_nblank) {
  return link | ((uint32_t)(label & 63) << 8) | (rec32_bp9(bp_blank) << 14) | (rec32_bp9(bp_nblank) << 23);
}
__host__ __device__ inline uint32_t rec32_unbp9(uint32_t v) { return v >= 256u ? kBpRestart : v; }
constexpr int kRec32MaxBeam = 128;
constexpr int kRec32MaxClasses = 64;
// record formats (TraceParams::rec_fmt)
constexpr int kRecFmt64 = 0, kRecFmt128 = 1, kRecFmt32 = 2;

// The wide record of the global-state tier (any beam width and num_classes):
// the same four fields at full width, 16 bytes.
struct Rec16 {
  uint32_t link;    // (src branch << 1) | is_new_child
  int32_t label;    // the beam's last label (-1 at the root)
  uint32_t bpb;     // best blank-ending alignment back-pointer (pos << 1 | kind), kBpRestart / kBpNone
  uint32_t bpn;     // best label-ending one
};

// Per-item results of the decode kernel.
struct ItemOut {
  int32_t n_leaves;       // leaves_.size() after the last frame
  int32_t literal_steps;  // frames replayed through the literal TopN model
  int32_t dup_frames;     // frames whose beam held one entry twice (-inf logits)
  int32_t why_nonfinite;  // literal replays caused by a non-finite logit or total
  int32_t why_fill;       // ... by the beam filling up mid-frame
  int32_t pad;            // two-wave kernels: nonzero if a helper hand-over wait ran out of time
  int64_t records;        // records written to HBM (all of them without the record ring; T * W can pass 2^31)
};
static_assert(sizeof(ItemOut) == 32, "ItemOut layout");

// Large C (> 64): per-(t, b) row facts computed by the parallel pre-pass
// ctcx_row_prep before the decode kernel, which would otherwise derive them
// inside its T-serial chain (one wave per item): the row maximum, whether it
// holds a NaN / +inf, the maxima of its 64-class blocks, and (float rows) the
// row's top set S -- the non-blank labels whose value is >= tau for the
// smallest tau leaving at most kTopK of them -- in label-index order, with the
// largest value outside S.  All depend on x[t, b, :] only.
constexpr int kTopK = 64;
template <typename T>
struct RowHdr {
  T xmax;       // max over the row's C values
  T xout;       // largest non-blank value outside S (-inf: none; +inf: no top set)
  int32_t bad;  // the row holds a NaN or +inf
  int32_t ns;   // |S|
};
// One row's record: RowHdr, the nblk block maxima (T), then S as kTopK
// (float value, int32 label index) pairs (float rows only); 16-byte aligned.
__host__ __device__ inline size_t prep_row_bytes(int64_t C, int tsize) {
  const size_t hdr = tsize == 4 ? 16 : 32;
  size_t s = hdr + ((((size_t)(C + 63) / 64) * tsize + 15) & ~(size_t)15);
  if (tsize == 4) s += (size_t)kTopK * 8;
  return s;
}
__host__ __device__ inline size_t prep_bmax_offset(int tsize) { return tsize == 4 ? 16 : 32; }
__host__ __device__ inline size_t prep_top_offset(int64_t C, int tsize) {
  return prep_bmax_offset(tsize) + ((((size_t)(C + 63) / 64) * tsize + 15) & ~(size_t)15);
}

template <typename T>
struct DecodeParams {
  const T* x;               // row (t, b) at x + (t * xstride + b) * C
  const T* norm;            // [Tmax][B]  softmax normaliser per row
  const int32_t* seq_len;   // [B]
  int64_t Tmax, B, C;
  int64_t xstride;          // items per frame in x (B, or the full batch for a shard read in place)
  int32_t W, P, blank, blank_label;
  int32_t force_literal;    // testing knob: replay every frame literally
  Rec* rec;                 // [B][Tmax][W]
  ItemOut* item;            // [B]
  int32_t* top_pos;         // [B][P]  sorted position of path p at the last frame
  int32_t* top_kind;        // [B][P]  0 blank / 1 label-ending / -1 none
  T* log_prob;              // [B][P]
  uint64_t* prof;           // optional [B][8] phase cycle counters (diagnostics)
  const T* scorer_tab;      // bigram beam-scorer table [C + 1][C], or null (BaseBeamScorer)
  const char* prep;         // C > 64: [Tmax][B] row records of ctcx_row_prep (prep_row_bytes each)
  // global-state tier (ctcx_gs::ctcx_beam_decode): the beam state of item b
  // at gstate + b * gstate_stride (global memory instead of LDS), records
  // written as Rec16 through rec
  char* gstate;
  int64_t gstate_stride;
  // record ring (LDS tier, ring_frames): frames of records kept in LDS (0: every
  // record written to rec[b][t][k] directly); with it item b's records form a
  // compacted stream at rec + b * Tmax * W, frame t's from foff[b][t] on
  int32_t ring;
  int32_t* foff;            // [B][Tmax]
  // the two-wave kernel this launch runs (0: the one-wave kernel; 1: score
  // table; 2: gather queue), decided once per call on the host
  // (use_helper_kernel): the kernel, the ring's record size and the
  // traceback's record format all follow this one value
  int32_t helper;
  int32_t test_flags;       // kTestHelperDead: the helper wave starts out "timed out" (tests only)
};
constexpr int32_t kTestHelperDead = 1;
// helper_kind's modes and the record size of a two-wave kernel kind (4-byte
// Rec32 records: the score table, and the scored queue at C <= 64)
// (kHelperScoredWide: the scored queue for beams of 129..256 too -- measured
// neutral at cfg5, where the helper's gather alone nearly fills its wave;
// CTCEXT_HELPER=4, diagnostics)
constexpr int kHelperNone = 0, kHelperLegacy = 1, kHelperScored = 3, kHelperScoredWide = 4;
__host__ __device__ inline bool helper_rec32(int hk, int64_t C) { return hk == 1 || (hk == 3 && C <= kRec32MaxClasses); }

struct TraceParams {
  const Rec* rec;
  const ItemOut* item;
  const int32_t* seq_len;
  const int32_t* top_pos;
  const int32_t* top_kind;
  int64_t Tmax, B;
  int32_t W, P, merge, blank_label;
  int32_t rec_fmt;    // kRecFmt64 (Rec), kRecFmt128 (Rec16, global-state tier), kRecFmt32 (Rec32, two-wave kernel)
  const int32_t* foff;   // record ring: frame t of item b at rec + b * Tmax * W + foff[b][t] (null: [b][t][W])
  int32_t* seq;    // [B][P][2][Tmax]  walk output, reversed
  int32_t* len;    // [P][2][len_stride], this batch's items at [.][.][0, B)
  int64_t len_stride;
};

struct PackParams {
  const int32_t* seq;       // as TraceParams::seq
  const int32_t* len;       // [P][2][B]
  const int64_t* off;       // [P][2][B] exclusive prefix sums
  int64_t Tmax, B;
  int32_t P;
  int64_t* const* idx;      // [P*2] -> int64 [n][2]   (decoded p, alignment p)
  int64_t* const* val;      // [P*2] -> int64 [n]
};

// Size of the per-frame LDS hash table of new leaves (power of two >= 2W).
__host__ __device__ inline int htab_size(int W) {
  int n = 16;
  while (n < 2 * W) n <<= 1;
  return n;
}

// Bytes of one item's beam state in the global-state tier: the carve without
// the logit row and the large-C arrays (the row is read in place from the
// inputs; only the literal path runs there).
__host__ __device__ inline size_t decode_lds_bytes(int W, int64_t C, int tsize, bool scored);
__host__ __device__ inline size_t gstate_bytes(int W, int tsize, bool scored) {
  return (decode_lds_bytes(W, 1, tsize, scored) + 255) & ~(size_t)255;
}

// LDS bytes needed by the decode kernel (host + device agree on the carve).
constexpr size_t kLdsBytes = 160 * 1024;   // LDS per CU on gfx950 (one workgroup per item)

// Large C (> 64, the BIG kernels): one buffer of branch arrays, which the
// per-frame commit updates in place (the row of C values takes the room; two
// items then fit one CU at cfg5).  C <= 64: two buffers, by frame parity.
__host__ __device__ inline bool decode_inplace(int64_t C) { return C > 64; }

// LDS bytes of the record ring of R frames (after the decode layout, 16-byte
// aligned): the records [R][W], entries per frame [R], compacted positions by
// frame parity [2][W] and of the newest written frame by flush parity [2][W]
// (int16), reachability stamps by frame parity [2][W] (int32).
__host__ __device__ inline size_t ring_lds_bytes(int R, int W, int rec_bytes = 8) {
  auto a16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
  return a16((size_t)R * (size_t)W * rec_bytes) + a16(4 * (size_t)R) + 2 * a16(4 * (size_t)W) + a16(8 * (size_t)W);
}

// Bytes of the decode kernel's LDS layout for a beam capacity W (carve() in
// ctcx_decode.hip, same order and alignment).
__host__ __device__ inline size_t decode_lds_bytes(int W, int64_t C, int tsize, bool scored) {
  const size_t ENC = 3 * (size_t)W + 2;
  const size_t nbuf = decode_inplace(C) ? 1 : 2;
  auto a16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
  size_t s = 0;
  s += nbuf * a16(5 * (size_t)W * tsize);       // branch probs
  s += nbuf * a16(3 * (size_t)W * 4);           // branch label/parent/flags
  s += a16(4 * (size_t)W * 4);                  // child lists, state, new positions
  s += a16(5 * ENC * tsize);                    // entry probs
  s += a16(5 * ENC * 4);                        // entry bps/kind/label/flags
  s += a16(((size_t)W + 1) * 4) * 2;            // heap, top-paths scratch
  s += a16((size_t)W * 4);                      // sorted
  s += a16((size_t)W * 4);                      // alias (entries the beam holds twice)
  s += 64;                                      // scalars
  s += 32 * 8;                                  // expf's 2^(i/32) table
  s += nbuf * 2 * (size_t)W * 8;                // prefix hashes (two 64-bit chains)
  s += a16(4 * (size_t)htab_size(W));           // per-frame new-leaf hash table  } the free list / slot
  s += a16(8 * (size_t)W);                      // per-branch evicted-child bloom } map aliases these two
  s += ((size_t)(W > 256 ? W : W > 128 ? 256 : 128) + 2 + 64) * (tsize == 8 ? 16 : 8); // TopN elements (value, slot) + per-lane dummy slots
  if (scored) s += a16((nbuf * (size_t)W + ENC) * tsize); // beam-scorer states (branches, entries)
  s += a16((size_t)C * tsize);                  // logit row
  s += a16((size_t)((C + 63) / 64) * tsize);    // its per-64-label block maxima
  if (C > 64) {                                 // compacted chunk offers, child label bitmap + window summary, top set
    const size_t nw = (size_t)(C - 1 + 63) / 64;
    s += 64 * 4 + 8 * nw + 8 * ((nw + 63) / 64) + (size_t)kTopK * 8;   // + the row's top set (value, label index)
  }
  return s;
}

}  // namespace ctcx

// ctc_oracle.cpp — CPU restatement of the reference CTC beam search with
// per-beam best-alignment tracking.
//
// *** TEST INFRASTRUCTURE ONLY. ***  This file is the parity checker and the
// CPU-baseline workload.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it.  The product path (ctc-beam-search-op_amd/)
// never links, loads or calls it.
//
// Pinning: the reference (TF custom op) is unbuildable in this image (it needs
// TensorFlow and Eigen headers that are not installed), so this restatement is
// pinned by the reference's own golden vector — the Graves-paper example in
// python/ops/ctc_ext_beam_search_decoder_ops_test.py:20-100 — checked by
// tests/test_oracle_golden.py, for T=float and T=double.  Every other parity
// case is pinned only through this restatement.
//
// What is restated, with the reference lines it follows
// (paths relative to tensorflow_ctc_ext_beam_search_decoder/cc/):
//   * LogSumExp, kLogZero                    util/ctc_loss_util.h:19-41
//   * BeamProbability / alignment candidates util/ctc_beam_entry.h:32-100
//   * BeamEntry: Active/New/GetChild/LabelSeq/AlignmentLabelSeq/
//     AddAlignmentCandidate                   util/ctc_beam_entry.h:105-246
//   * BeamRoot arena, BeamComparer            util/ctc_beam_entry.h:248-280
//   * Step / Reset / TopPaths                 util/ctc_ext_beam_search_decoder.h:66-261
//   * Compute batch driver, validation, SparseTensor packing
//                                             kernels/ctc_ext_beam_search_decoder_kernels.cc:20-257
//   * beam scorer hook (BaseBeamScorer identity, or a bigram expansion-score
//     table)                                   util/ctc_beam_scorer.h:31-65, used at
//                                              ctc_ext_beam_search_decoder.h:103, 114, 171-182, 226
//   * gtl::TopN (third-party, TensorFlow tensorflow/core/lib/gtl/top_n.h,
//     TF 1.14-2.1 era per configure.sh:59-81): restated from its published
//     algorithm — UNORDERED -> BOTTOM_KNOWN -> HEAP_SORTED, libstdc++
//     make_heap/pop_heap/sort_heap/std::sort (the heap layout decides
//     tie order, so the real libstdc++ algorithms are used here).
//
// Two alignment stores (selected per call):
//   kFaithful: every candidate owns a std::vector<int> label sequence kept in a
//              std::priority_queue, copied on every AddAlignmentCandidate —
//              the reference's data structures and O(W*C*T^2) cost.  This is
//              the mode timed as bench.py's cpu_baseline ("port").
//   kShared:   a candidate is (prob, index into an append-only (label, prev)
//              arena) and only the first-pushed maximum is kept.  Same results
//              (only .top() of each queue is ever read, ctc_beam_entry.h:92-99),
//              O(W*C) time per frame.  Nodes that GetChild would create only to
//              be deactivated are never materialised, and unreachable
//              never-used nodes are reclaimed (Decoder::reclaim), so memory is
//              O(live prefixes): full-length cfg4/cfg5 items fit.  This is the
//              parity checker.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <limits>
#include <memory>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

namespace oracle {

template <class T>
constexpr T LogZero() { return -std::numeric_limits<T>::infinity(); }

// util/ctc_loss_util.h:29-41.  Float libm even when T is double.
template <class T>
inline T LSE(T a, T b) {
  if (a == LogZero<T>()) return b;
  if (b == LogZero<T>()) return a;
  return (a > b) ? a + log1pf(expf(b - a)) : b + log1pf(expf(a - b));
}

inline float NumExp(float x) { return expf(x); }
inline double NumExp(double x) { return exp(x); }
inline float NumLog(float x) { return logf(x); }
inline double NumLog(double x) { return log(x); }

// The softmax normaliser of one row (ctc_ext_beam_search_decoder.h:72-80):
// maxCoeff's loop, the sum of exp(x_j - max) in class order, max + log(sum).
template <typename T>
T row_normaliser(const T* x, int64_t C) {
  T mx = x[0];
  for (int64_t j = 1; j < C; ++j) mx = std::max(mx, x[j]);
  T s = T(0);
  for (int64_t j = 0; j < C; ++j) s += NumExp(x[j] - mx);
  return mx + NumLog(s);
}

// ---------------------------------------------------------------------------
// gtl::TopN restatement.
template <class E, class Greater>
class BoundedTop {
 public:
  explicit BoundedTop(size_t limit) : limit_(limit) {}
  size_t size() const { return std::min(v_.size(), limit_); }
  void push(E e) {
    if (limit_ == 0) return;
    if (state_ != kHeap) {
      v_.push_back(e);
      if (state_ != kUnordered && !gt_(v_.back(), v_.front())) std::swap(v_.front(), v_.back());
      if (v_.size() == limit_ + 1) {
        std::make_heap(v_.begin(), v_.end(), gt_);
        std::pop_heap(v_.begin(), v_.end(), gt_);
        state_ = kHeap;
      }
    } else if (gt_(e, v_.front())) {
      v_.back() = e;
      std::pop_heap(v_.begin(), v_.end(), gt_);
    }
  }
  E peek_bottom() {
    if (state_ == kUnordered) {
      size_t m = 0;
      for (size_t i = 1; i < v_.size(); ++i)
        if (gt_(v_[m], v_[i])) m = i;
      if (m != 0) std::swap(v_[0], v_[m]);
      state_ = kBottomKnown;
    }
    return v_.front();
  }
  // Destructive, descending order; caller calls reset() afterwards.
  std::vector<E> extract() {
    std::vector<E> out;
    out.swap(v_);
    if (state_ != kHeap) {
      std::sort(out.begin(), out.end(), gt_);
    } else {
      out.pop_back();
      std::sort_heap(out.begin(), out.end(), gt_);
    }
    return out;
  }
  void reset() { v_.clear(); state_ = kUnordered; }
  typename std::vector<E>::const_iterator ubegin() const { return v_.begin(); }
  typename std::vector<E>::const_iterator uend() const { return v_.begin() + size(); }

 private:
  enum { kUnordered, kBottomKnown, kHeap } state_ = kUnordered;
  std::vector<E> v_;
  size_t limit_;
  Greater gt_;
};

// ---------------------------------------------------------------------------
// Alignment candidate stores.
template <class T>
struct VecCand {             // reference-shaped candidate (ctc_beam_entry.h:46-63)
  T prob;
  std::vector<int> seq;
  VecCand() : prob(LogZero<T>()) {}
  VecCand(std::vector<int> s, T p) : prob(p), seq(s) {}   // by value, then copied: as the reference
};
// BeamAlignmentCandidateComparer (ctc_beam_entry.h:65-73): virtual, and it
// takes both candidates BY VALUE, so every heap comparison copies two label
// sequences.  Kept that way here: it is part of the reference's cost.
template <class T>
struct VecCandLess {
  virtual ~VecCandLess() {}
  virtual bool operator()(const VecCand<T> a, const VecCand<T> b) const { return a.prob < b.prob; }
};

template <class T>
struct FaithfulStore {
  using Queue = std::priority_queue<VecCand<T>, std::vector<VecCand<T>>, VecCandLess<T>>;
  struct Slots { Queue q[2]; };  // [0] = blank-ending, [1] = label-ending
  static bool has(const Slots& s, int k) { return !s.q[k].empty(); }
  static T prob(const Slots& s, int k) { return s.q[k].top().prob; }
  // BeamAlignment::Reset (ctc_beam_entry.h:84-91) pops every element
  static void clear(Slots& s) {
    while (!s.q[0].empty()) s.q[0].pop();
    while (!s.q[1].empty()) s.q[1].pop();
  }
  // old_cands = new_cands; new_cands.Reset()   (decoder.h:87-92)
  static void roll(Slots& old, Slots& nw) { old = nw; clear(nw); }
  // GetBlank / GetNBlank (ctc_beam_entry.h:92-99): a copy of top()
  static VecCand<T> top_copy(const Queue& q) { VecCand<T> r = q.top(); return r; }
  static constexpr bool kLazyNodes = false;
  // Same allocation/copy pattern as the reference's AddAlignmentCandidate
  // (ctc_beam_entry.h:190-228), so its O(t) copies per call are reproduced.
  void add(Slots& dst, int to_k, const Slots& src, int from_k, T base_if_none, T p, int label) {
    VecCand<T> old_cand;
    std::vector<int> old_seq;
    T base;
    if (!src.q[from_k].empty()) {
      old_cand = top_copy(src.q[from_k]);   // move-assigned from the returned copy
      base = old_cand.prob;
      old_seq = old_cand.seq;
    } else {
      base = base_if_none;
    }
    std::vector<int> grown(old_seq);
    grown.push_back(label);
    VecCand<T> nc = VecCand<T>(grown, base + p);
    dst.q[to_k].push(nc);
  }
  std::vector<int> sequence(const Slots& s, int k) const { return s.q[k].top().seq; }
  void reset_all() {}
};

// Shared store: a candidate is its probability plus a back-link into an
// append-only (label, prev) arena; only the first-pushed maximum of each kind
// is kept (only .top() is ever read, ctc_beam_entry.h:92-99).  A candidate
// of the current frame (new_c) is held unmaterialised as (label, prev) and
// enters the arena only when its entry rolls it into old_c as a branch
// (decoder.h:87-92), so the arena grows by <= 2 entries per branch per frame
// instead of one per AddAlignmentCandidate call: cost only, the candidate
// sequences are identical.
template <class T>
struct SharedStore {
  struct Slots {
    T p[2];
    int32_t label[2], prev[2];  // new_c form: appended label, arena id of the source (-1: none)
    int32_t id[2];              // old_c form: arena id of the whole sequence
    bool ok[2];
    Slots() { ok[0] = ok[1] = false; }
  };
  std::vector<std::pair<int32_t, int32_t>> arena;  // (label, prev id or -1)
  static constexpr bool kLazyNodes = true;
  static bool has(const Slots& s, int k) { return s.ok[k]; }
  static T prob(const Slots& s, int k) { return s.p[k]; }
  static void clear(Slots& s) { s.ok[0] = s.ok[1] = false; }
  void roll(Slots& old, Slots& nw) {
    for (int k = 0; k < 2; ++k) {
      old.ok[k] = nw.ok[k];
      if (!nw.ok[k]) continue;
      arena.emplace_back(nw.label[k], nw.prev[k]);
      old.p[k] = nw.p[k];
      old.id[k] = (int32_t)arena.size() - 1;
    }
    clear(nw);
  }
  void add(Slots& dst, int to_k, const Slots& src, int from_k, T base_if_none, T p, int label) {
    T base;
    int32_t prev;
    if (src.ok[from_k]) { base = src.p[from_k]; prev = src.id[from_k]; }
    else { base = base_if_none; prev = -1; }
    const T np = base + p;
    // first-pushed maximum == std::priority_queue::top() under a strict '<'
    if (dst.ok[to_k] && !(np > dst.p[to_k])) return;
    dst.p[to_k] = np;
    dst.label[to_k] = label;
    dst.prev[to_k] = prev;
    dst.ok[to_k] = true;
  }
  // sequence of a new_c candidate (TopPaths reads new_cands, ctc_beam_entry.h:137-152)
  std::vector<int> sequence(const Slots& s, int k) const {
    std::vector<int> out;
    out.push_back(s.label[k]);
    for (int32_t i = s.prev[k]; i >= 0; i = arena[i].second) out.push_back(arena[i].first);
    std::reverse(out.begin(), out.end());
    return out;
  }
  void reset_all() { arena.clear(); }
};

// ---------------------------------------------------------------------------
// Prefix-trie node (one per distinct label prefix) and the decoder.
template <class T, class Store>
struct Node {
  Node* parent;
  int label;
  std::unordered_map<int, Node*> kids;
  T old_t = LogZero<T>(), old_b = LogZero<T>(), old_l = LogZero<T>();
  T new_t = LogZero<T>(), new_b = LogZero<T>(), new_l = LogZero<T>();
  T state = T(0);   // beam-scorer state: the cached expansion score
  typename Store::Slots old_c, new_c;
  bool mark = false;  // reclamation: ancestor-or-self of a branch
  Node(Node* p, int l) : parent(p), label(l) {}
  bool active() const { return new_t != LogZero<T>(); }
  bool fresh() const { return old_t == LogZero<T>(); }
  void reset_new() { new_t = new_b = new_l = LogZero<T>(); }
  void reset_old() { old_t = old_b = old_l = LogZero<T>(); }
};

template <class T, class Store>
struct NodeGreater {
  bool operator()(const Node<T, Store>* a, const Node<T, Store>* b) const { return a->new_t > b->new_t; }
};

template <class T, class Store>
class Decoder {
  using N = Node<T, Store>;
  using Top = BoundedTop<N*, NodeGreater<T, Store>>;

 public:
  // tab: bigram scorer table [C + 1][C] (row from_label + 1), or null for
  // BaseBeamScorer (the identity the reference op uses, kernels.cc:260)
  Decoder(int C, int blank_index, int W, int blank_label, const T* tab = nullptr)
      : C_(C), blank_(blank_index), W_(W), blank_label_(blank_label), leaves_(W), tab_(tab),
        scratch_(nullptr, -1) { reset(); }

  void reset() {
    leaves_.reset();
    pool_.clear();
    store_.reset_all();
    gc_next_ = gc_threshold;
    pool_.emplace_back(new N(nullptr, -1));
    root_ = pool_.back().get();
    root_->new_t = T(0);
    root_->new_b = T(0);
    leaves_.push(root_);
    root_->state = T(0);   // InitializeState (decoder.h:226)
  }

  // ctc_ext_beam_search_decoder.h:69-210
  void step(const T* x) {
    const T norm = row_normaliser(x, C_);

    std::vector<N*> branches = leaves_.extract();
    leaves_.reset();
    if (count_dups) {
      // frames that start with one entry twice in the beam (reachable with -inf
      // logits: decoder.h:142 pushes every branch, :189-199 re-pushes a branch
      // that is not Active); counted only when the tests ask, so the timed
      // faithful mode does no work the reference does not
      std::vector<N*> sb(branches);
      std::sort(sb.begin(), sb.end());
      if (std::adjacent_find(sb.begin(), sb.end()) != sb.end()) ++dup_frames;
    }
    if (Store::kLazyNodes && (int64_t)pool_.size() > gc_next_) reclaim(branches);
    if (getenv("ORACLE_TRACE")) {   // debugging aid: frame-start beam, extract order
      printf("frame\n");
      for (N* b : branches) {
        std::vector<int> pre;
        for (N* c = b; c->parent; c = c->parent) pre.push_back(c->label);
        std::reverse(pre.begin(), pre.end());
        printf("  %a [", (double)b->new_t);
        for (int v : pre) printf("%d,", v);
        printf("]\n");
      }
    }
    for (N* b : branches) {
      b->old_t = b->new_t; b->old_b = b->new_b; b->old_l = b->new_l;
      store_.roll(b->old_c, b->new_c);
    }

    const T pblank = x[blank_] - norm;
    for (N* b : branches) {
      if (b->parent != nullptr) {
        const T p = x[b->label] - norm;
        N* P = b->parent;
        if (P->active()) {
          const bool same = (b->label == P->label);
          const T prev = same ? P->old_b : P->old_t;
          b->new_l = LSE(b->new_l, expansion_score(b, prev)) + x[b->label] - norm;
          cand(b, 1, P, 0, p, b->label);
          if (!same) cand(b, 1, P, 1, p, b->label);
          cand(b, 1, b, 1, p, b->label);
        } else {
          b->new_l += x[b->label] - norm;
          cand(b, 1, b, 1, p, b->label);
        }
      }
      b->new_b = b->old_t + x[blank_] - norm;
      cand(b, 0, b, 0, pblank, blank_label_);
      cand(b, 0, b, 1, pblank, blank_label_);
      b->new_t = LSE(b->new_b, b->new_l);
      leaves_.push(b);
    }

    for (N* b : branches) {
      if (!admissible(b->old_t)) continue;
      for (int l = 0; l < C_; ++l) {
        if (l == blank_) continue;
        N* c = Store::kLazyNodes ? find_child(b, l) : child(b, l);
        if (c->active()) continue;
        const T p = x[l] - norm;
        c->new_b = LogZero<T>();
        expand_state(b, c, l);
        if (l == b->label) {
          c->new_l = x[l] - norm + expansion_score(c, b->old_b);
          cand(c, 1, b, 0, p, l);
        } else {
          c->new_l = x[l] - norm + expansion_score(c, b->old_t);
          cand(c, 1, b, 0, p, l);
          cand(c, 1, b, 1, p, l);
        }
        c->new_t = c->new_l;
        if (admissible(c->new_t)) {
          if (c == &scratch_) c = adopt(b, l);
          if (leaves_.size() == (size_t)W_) {
            N* bottom = leaves_.peek_bottom();
            bottom->reset_new();
            Store::clear(bottom->new_c);
          }
          leaves_.push(c);
        } else {
          // deactivation (decoder.h:200-205); for the scratch node this
          // leaves it in the never-created state, as required below
          c->reset_old();
          c->reset_new();
          Store::clear(c->old_c);
          Store::clear(c->new_c);
        }
      }
    }
  }

  // ctc_ext_beam_search_decoder.h:230-261.  Returns 0, 1 (n > W) or 2 (n > leaves).
  int top_paths(int n, bool merge, std::vector<std::vector<int>>& paths,
                std::vector<std::vector<int>>& aligns, std::vector<T>& lps, int& no_label_events) {
    paths.clear(); aligns.clear(); lps.clear();
    if (n > W_) return 1;
    if ((size_t)n > leaves_.size()) return 2;
    Top best(n);
    for (auto it = leaves_.ubegin(); it != leaves_.uend(); ++it) best.push(*it);
    std::vector<N*> sel = best.extract();
    for (int i = 0; i < n; ++i) {
      N* e = sel[i];
      aligns.push_back(alignment(e, no_label_events));
      std::vector<int> labels;
      int prev = -1;
      for (const N* c = e; c->parent != nullptr; c = c->parent) {
        if (!merge || c->label != prev) labels.push_back(c->label);
        prev = c->label;
      }
      std::reverse(labels.begin(), labels.end());
      paths.push_back(labels);
      lps.push_back(e->new_t);
    }
    return 0;
  }

 private:
  // ctc_beam_scorer.h:41-56: ExpandState / GetStateExpansionScore
  void expand_state(const N* from, N* to, int to_label) {
    if (tab_) to->state = tab_[(int64_t)(from->label + 1) * C_ + to_label];
  }
  T expansion_score(const N* n, T prev) const { return tab_ ? prev + n->state : prev; }

  bool admissible(T total) {
    return total > LogZero<T>() &&
           (leaves_.size() < (size_t)W_ || total > leaves_.peek_bottom()->new_t);
  }
  N* child(N* b, int l) {
    auto it = b->kids.find(l);
    if (it != b->kids.end()) return it->second;
    pool_.emplace_back(new N(b, l));
    b->kids.emplace(l, pool_.back().get());
    return pool_.back().get();
  }

  // ---- cost-only node economy of the shared mode ------------------------
  // A node in the never-created state ("pristine": every probability -inf,
  // no candidate, no kids) is indistinguishable from one GetChild
  // (ctc_beam_entry.h:114-122) would build now:
  //   * new_t/new_b/new_l, new_c and old_c are pristine by definition;
  //   * old_t/old_b/old_l are pristine too (fresh() reads old_t);
  //   * `state` is written by ExpandState before every read (decoder.h:171-182
  //     writes it for an offered child; it is read only for that child and
  //     for branches, which are never reclaimed);
  //   * nothing compares node identity except TopN membership, and a reclaimed
  //     node is in no TopN (reclaim runs between Extract and the first push).
  // So (1) a child that does not exist yet is evaluated on one scratch node
  // and only materialised if the TopN accepts it (a rejected one is
  // deactivated, decoder.h:200-205, i.e. pristine again, exactly as if it had
  // been created), and (2) pristine nodes that are neither branches nor
  // ancestors of one are freed.  Results are unchanged; memory drops from
  // O(W*C*T) nodes to O(live prefixes).
  N* find_child(N* b, int l) {
    auto it = b->kids.find(l);
    if (it != b->kids.end()) return it->second;
    scratch_.parent = b;
    scratch_.label = l;
    return &scratch_;   // pristine (reset after every rejected offer)
  }
  N* adopt(N* b, int l) {
    N* n = new N(b, l);
    n->old_t = scratch_.old_t; n->old_b = scratch_.old_b; n->old_l = scratch_.old_l;
    n->new_t = scratch_.new_t; n->new_b = scratch_.new_b; n->new_l = scratch_.new_l;
    n->state = scratch_.state;
    n->old_c = scratch_.old_c;
    n->new_c = scratch_.new_c;
    pool_.emplace_back(n);
    b->kids.emplace(l, n);
    // scratch back to the never-created state
    scratch_.reset_old();
    scratch_.reset_new();
    Store::clear(scratch_.old_c);
    Store::clear(scratch_.new_c);
    return n;
  }
  static bool pristine(const N* n) {
    return n->kids.empty() && n->old_t == LogZero<T>() && n->old_b == LogZero<T>() &&
           n->old_l == LogZero<T>() && n->new_t == LogZero<T>() && n->new_b == LogZero<T>() &&
           n->new_l == LogZero<T>() && !Store::has(n->old_c, 0) && !Store::has(n->old_c, 1) &&
           !Store::has(n->new_c, 0) && !Store::has(n->new_c, 1);
  }
  void reclaim(const std::vector<N*>& branches) {
    for (N* b : branches)
      for (N* a = b; a != nullptr && !a->mark; a = a->parent) a->mark = true;
    // children are always created after their parent, so a reverse sweep
    // frees a node's reclaimable kids before the node itself is tested
    size_t live = 0;
    for (size_t i = pool_.size(); i-- > 1;) {
      N* n = pool_[i].get();
      if (!n->mark && pristine(n)) {
        n->parent->kids.erase(n->label);
        pool_[i].reset();
      }
    }
    for (size_t i = 0; i < pool_.size(); ++i) {
      if (!pool_[i]) continue;
      pool_[i]->mark = false;
      if (i != live) pool_[live] = std::move(pool_[i]);
      ++live;
    }
    pool_.resize(live);
    ++reclaims;
    gc_next_ = gc_threshold == 1 ? 1 : std::max<int64_t>(gc_threshold, 2 * (int64_t)live);
  }
  // ctc_beam_entry.h:190-228: receiver r gets a candidate built on
  // src's previous-step candidate of kind from_k (0 = blank-ending).
  void cand(N* r, int to_k, const N* src, int from_k, T p, int label) {
    T base_if_none = LogZero<T>();
    if (r->parent == nullptr || (r->parent->parent == nullptr && r->fresh()))
      base_if_none = (from_k == 0) ? T(0) : LogZero<T>();
    store_.add(r->new_c, to_k, src->old_c, from_k, base_if_none, p, label);
  }
  std::vector<int> alignment(N* e, int& no_label_events) {
    const bool hb = Store::has(e->new_c, 0), hn = Store::has(e->new_c, 1);
    if (hb && hn) return store_.sequence(e->new_c, Store::prob(e->new_c, 0) > Store::prob(e->new_c, 1) ? 0 : 1);
    if (hb) return store_.sequence(e->new_c, 0);
    if (hn) return store_.sequence(e->new_c, 1);
    ++no_label_events;   // reference prints "No label seq available"
    return {};
  }

  int C_, blank_, W_, blank_label_;
  Top leaves_;
  const T* tab_;

 public:
  int64_t dup_frames = 0;
  bool count_dups = false;
  int64_t gc_threshold = 1 << 20;   // nodes; tests force tiny values
  int64_t reclaims = 0;

 private:
  std::vector<std::unique_ptr<N>> pool_;
  N* root_ = nullptr;
  Store store_;
  N scratch_;
  int64_t gc_next_ = 1 << 20;
};

}  // namespace oracle

// ---------------------------------------------------------------------------
// C ABI used by oracle/oracle.py (ctypes).  Mirrors the Compute() batch
// driver (kernels.cc:20-95): items decoded one after another with one decoder
// that is reset between items; the first failing item aborts the call.
struct OracleResult {
  int32_t status;          // 0 ok; 1 "requested more paths than the beam width."
                           //      2 "Less leaves in the beam search than requested."
  int32_t no_label_events;
  int64_t total_dec, total_ali;
  int64_t* dec_len;        // [B*P]   (b-major)
  int64_t* ali_len;        // [B*P]
  int32_t* dec_vals;       // concatenation over (b, p) in b-major order
  int32_t* ali_vals;
  double* log_prob;        // [B*P]
  int64_t dup_frames;      // frames whose beam held one entry twice (flag 1)
  int64_t reclaims;        // shared-mode node reclamation passes
};

enum { kFlagCountDups = 1 };

template <class T, class Store>
static OracleResult* run(const T* x, const int32_t* seq_len, int64_t Tmax, int64_t B, int64_t C,
                         int W, int P, int merge, int blank_index, int blank_label, const T* tab,
                         int flags, int64_t gc_threshold) {
  OracleResult* r = new OracleResult();
  memset(r, 0, sizeof(*r));
  std::vector<std::vector<int>> dec_all, ali_all;
  std::vector<double> lp(B * P, 0.0);
  oracle::Decoder<T, Store> dec((int)C, blank_index, W, blank_label, tab);
  dec.count_dups = (flags & kFlagCountDups) != 0;
  if (gc_threshold > 0) dec.gc_threshold = gc_threshold;
  dec.reset();
  std::vector<T> row(C);
  for (int64_t b = 0; b < B; ++b) {
    for (int64_t t = 0; t < seq_len[b]; ++t) {
      memcpy(row.data(), x + (t * B + b) * C, sizeof(T) * C);
      dec.step(row.data());
    }
    std::vector<std::vector<int>> paths, aligns;
    std::vector<T> lps;
    int st = dec.top_paths(P, merge != 0, paths, aligns, lps, r->no_label_events);
    r->dup_frames = dec.dup_frames;
    r->reclaims = dec.reclaims;
    if (st != 0) { r->status = st; return r; }
    dec.reset();
    for (int p = 0; p < P; ++p) {
      lp[b * P + p] = (double)lps[p];
      dec_all.push_back(paths[p]);
      ali_all.push_back(aligns[p]);
    }
  }
  r->dec_len = new int64_t[B * P + 1];
  r->ali_len = new int64_t[B * P + 1];
  r->log_prob = new double[B * P + 1];
  for (int64_t i = 0; i < B * P; ++i) {
    r->dec_len[i] = (int64_t)dec_all[i].size();
    r->ali_len[i] = (int64_t)ali_all[i].size();
    r->total_dec += r->dec_len[i];
    r->total_ali += r->ali_len[i];
    r->log_prob[i] = lp[i];
  }
  r->dec_vals = new int32_t[r->total_dec + 1];
  r->ali_vals = new int32_t[r->total_ali + 1];
  int64_t od = 0, oa = 0;
  for (int64_t i = 0; i < B * P; ++i) {
    for (int v : dec_all[i]) r->dec_vals[od++] = v;
    for (int v : ali_all[i]) r->ali_vals[oa++] = v;
  }
  return r;
}

extern "C" {

// dtype 0 = float32, 1 = float64; mode 0 = faithful store, 1 = shared store;
// table: bigram beam-scorer table [C + 1][C] of dtype, or null (BaseBeamScorer);
// flags: kFlagCountDups; gc_threshold: shared-mode node count that triggers
// reclamation (<= 0: default 2^20; tests pass 1 to reclaim every frame).
OracleResult* oracle_decode_ex(int dtype, int mode, const void* x, const int32_t* seq_len,
                               int64_t T, int64_t B, int64_t C, int W, int P, int merge,
                               int blank_index, int blank_label, const void* table, int flags,
                               int64_t gc_threshold) {
  if (dtype == 0) {
    const float* xf = (const float*)x;
    const float* tf = (const float*)table;
    return mode == 0 ? run<float, oracle::FaithfulStore<float>>(xf, seq_len, T, B, C, W, P, merge, blank_index, blank_label, tf, flags, gc_threshold)
                     : run<float, oracle::SharedStore<float>>(xf, seq_len, T, B, C, W, P, merge, blank_index, blank_label, tf, flags, gc_threshold);
  }
  const double* xd = (const double*)x;
  const double* td = (const double*)table;
  return mode == 0 ? run<double, oracle::FaithfulStore<double>>(xd, seq_len, T, B, C, W, P, merge, blank_index, blank_label, td, flags, gc_threshold)
                   : run<double, oracle::SharedStore<double>>(xd, seq_len, T, B, C, W, P, merge, blank_index, blank_label, td, flags, gc_threshold);
}

OracleResult* oracle_decode_scored(int dtype, int mode, const void* x, const int32_t* seq_len,
                                   int64_t T, int64_t B, int64_t C, int W, int P, int merge,
                                   int blank_index, int blank_label, const void* table) {
  return oracle_decode_ex(dtype, mode, x, seq_len, T, B, C, W, P, merge, blank_index, blank_label, table, 0, 0);
}

OracleResult* oracle_decode(int dtype, int mode, const void* x, const int32_t* seq_len,
                            int64_t T, int64_t B, int64_t C, int W, int P, int merge,
                            int blank_index, int blank_label) {
  return oracle_decode_scored(dtype, mode, x, seq_len, T, B, C, W, P, merge, blank_index, blank_label, nullptr);
}

// the normaliser of each of rows consecutive rows of C values (dtype as above)
void oracle_row_norm(int dtype, const void* x, int64_t rows, int64_t C, void* out) {
  for (int64_t r = 0; r < rows; ++r) {
    if (dtype == 0) ((float*)out)[r] = oracle::row_normaliser((const float*)x + r * C, C);
    else ((double*)out)[r] = oracle::row_normaliser((const double*)x + r * C, C);
  }
}

void oracle_free(OracleResult* r) {
  if (!r) return;
  delete[] r->dec_len; delete[] r->ali_len; delete[] r->dec_vals; delete[] r->ali_vals;
  delete[] r->log_prob;
  delete r;
}

}  // extern "C"

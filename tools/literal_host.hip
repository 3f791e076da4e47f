// literal_host.hip — DEBUG HARNESS (not product, not shipped): runs the
// decode kernel's LITERAL path (literal_step + the commit + the traceback
// walks, restated here on the host) sequentially on the CPU, using the same
// source as the device build.  Lets the literal path be diffed against the
// oracle without a GPU:
//   hipcc -O1 -std=c++17 -ffp-contract=off -fPIC -shared --offload-arch=gfx950 \
//         tools/literal_host.hip -o /tmp/liblithost.so
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../ctc-beam-search-op_amd/csrc/ctcx_decode.hip"

using namespace ctcx;

extern "C" int lit_decode_f32(const float* x, const int32_t* seq_len, int64_t Tmax, int64_t B, int64_t C, int W,
                              int P, int merge, int blank, int blank_label, int32_t* out_len /*[B][P][2]*/,
                              int32_t* out_seq /*[B][P][2][Tmax]*/, float* out_lp /*[B][P]*/) {
  typedef float T;
  std::vector<char> lds(decode_lds_bytes(W, C, sizeof(T)) + 64);
  Ctx<T> cx;
  carve(cx, lds.data(), W, W, (int)C);
  cx.blank = blank;
  std::vector<Rec> rec((size_t)Tmax * W);
  for (int64_t b = 0; b < B; ++b) {
    const int sl = seq_len[b] > 0 ? seq_len[b] : 0;
    int buf = 0;
    cx.lab[0][0] = -1; cx.par[0][0] = -1; cx.flg[0][0] = F_ROOT;
    cx.ot[0][0] = 0; cx.ob[0][0] = 0; cx.ol[0][0] = ninf<T>();
    cx.ha[0][0] = kRootHa; cx.hb[0][0] = kRootHb;
    cx.head[0] = -1;
    int nb = 1, n_leaves = 1;
    for (int t = 0; t < sl; ++t) {
      const float* xr = x + ((int64_t)t * B + b) * C;
      for (int j = 0; j < C; ++j) cx.row[j] = xr[j];
      float m = xr[0];
      for (int j = 1; j < C; ++j) m = xr[j] > m ? xr[j] : m;
      float s = 0;
      for (int j = 0; j < C; ++j) s += gm::expf(xr[j] - m);
      const float norm = m + gm::logf(s);
      const bool last = (t == sl - 1);
      int err = 0;
      if (getenv("ORACLE_TRACE2")) {
        printf("branches t=%d\n", t);
        for (int i = 0; i < nb; ++i) printf("  i=%d lab=%d par=%d flg=%d ot=%a head=%d sib=%d\n", i, cx.lab[buf][i], cx.par[buf][i], cx.flg[buf][i], (double)cx.ot[buf][i], cx.head[i], cx.sib[i]);
      }
      const int n = literal_step(cx, buf, nb, norm, last, P, &err, &n_leaves);
      if (err) return -1;
      const int nx = buf ^ 1;
      for (int i = 0; i < nb; ++i) cx.newpos[i] = -1;
      for (int k = 0; k < n; ++k) {
        const uint32_t kd = cx.ekind[cx.sorted[k]];
        if (!(kd & 1u)) cx.newpos[kd >> 1] = k;
      }
      for (int q = 0; q < cx.hts; ++q) cx.htab[q] = -1;
      for (int k = 0; k < n; ++k) {
        const uint32_t kd = cx.ekind[cx.sorted[k]];
        const int src = (int)(kd >> 1);
        uint64_t ha, hb, pa, pb;
        if (kd & 1u) {
          pa = cx.ha[buf][src]; pb = cx.hb[buf][src];
          hmix(pa, pb, cx.elab[cx.sorted[k]], ha, hb);
          int q = (int)(ha & (uint64_t)(cx.hts - 1));
          while (cx.htab[q] != -1) q = (q + 1) & (cx.hts - 1);
          cx.htab[q] = k;
        } else {
          ha = cx.ha[buf][src]; hb = cx.hb[buf][src]; pa = cx.pha[buf][src]; pb = cx.phb[buf][src];
        }
        cx.ha[nx][k] = ha; cx.hb[nx][k] = hb; cx.pha[nx][k] = pa; cx.phb[nx][k] = pb;
      }
      for (int k = 0; k < n; ++k) {
        const int e = cx.sorted[k];
        const uint32_t kd = cx.ekind[e];
        const int src = (int)(kd >> 1);
        const bool isnew = (kd & 1u) != 0;
        const int pf = cx.flg[buf][src];
        int parent, fl;
        if (isnew) { parent = cx.newpos[src]; fl = (pf & F_ROOT) ? F_PROOT : 0; }
        else {
          const int pp = cx.par[buf][src]; parent = pp >= 0 ? cx.newpos[pp] : -1; fl = pf & (F_ROOT | F_PROOT);
          if (pp < 0 && !(pf & F_ROOT)) {
            const uint64_t pa = cx.pha[nx][k], pb = cx.phb[nx][k];
            for (int q = (int)(pa & (uint64_t)(cx.hts - 1));; q = (q + 1) & (cx.hts - 1)) {
              const int c = cx.htab[q];
              if (c < 0) break;
              if (cx.ha[nx][c] == pa && cx.hb[nx][c] == pb) { parent = c; break; }
            }
          }
        }
        const int ef = cx.eflg[e];
        fl |= ef & (F_HB | F_HN);
        cx.lab[nx][k] = cx.elab[e]; cx.par[nx][k] = parent; cx.flg[nx][k] = fl;
        cx.ot[nx][k] = cx.et[e]; cx.ob[nx][k] = cx.eb[e]; cx.ol[nx][k] = cx.el[e];
        cx.cb[nx][k] = cx.ecb[e]; cx.cn[nx][k] = cx.ecn[e];
        Rec rc{kd, cx.elab[e], (ef & F_HB) ? cx.ebpb[e] : kBpNone, (ef & F_HN) ? cx.ebpn[e] : kBpNone};
        rec[(size_t)t * W + k] = rc;
      }
      if (getenv("ORACLE_TRACE")) {
        printf("frame\n");
        for (int k = 0; k < n; ++k) {
          std::vector<int> pre;
          int kk = k;
          for (int tt = t; tt >= 0; --tt) {
            const Rec r = rec[(size_t)tt * W + kk];
            if (r.link & 1u) pre.push_back(r.label);
            kk = (int)(r.link >> 1);
          }
          printf("  %a [", (double)cx.ot[nx][k]);
          for (int i = (int)pre.size() - 1; i >= 0; --i) printf("%d,", pre[i]);
          printf("]\n");
        }
      }
      buf = nx;
      nb = n;
      for (int k = 0; k < nb; ++k) cx.head[k] = -1;
      for (int k = 0; k < nb; ++k) {
        const int pp = cx.par[buf][k];
        if (pp >= 0) { cx.sib[k] = cx.head[pp]; cx.head[pp] = k; }
      }
    }
    if (sl == 0) cx.tops[0] = 0;
    if (n_leaves < P) return -2;
    for (int q = 0; q < P; ++q) {
      const int pos = cx.tops[q];
      const int f = cx.flg[buf][pos];
      const bool hb = f & F_HB, hn = f & F_HN;
      int kind = -1;
      if (hb && hn) kind = (cx.cb[buf][pos] > cx.cn[buf][pos]) ? 0 : 1;
      else if (hb) kind = 0;
      else if (hn) kind = 1;
      out_lp[b * P + q] = cx.ot[buf][pos];
      for (int which = 0; which < 2; ++which) {
        int32_t* o = out_seq + ((b * P + q) * 2 + which) * Tmax;
        int len = 0, k = pos;
        if (sl > 0) {
          if (which == 0) {
            int prev = -1;
            for (int t = sl - 1; t >= 0; --t) {
              const Rec r = rec[(size_t)t * W + k];
              if (r.link & 1u) { if (!merge || r.label != prev) o[len++] = r.label; prev = r.label; }
              k = (int)(r.link >> 1);
            }
          } else {
            int kd = kind;
            for (int t = sl - 1; t >= 0 && kd >= 0; --t) {
              const Rec r = rec[(size_t)t * W + k];
              o[len++] = kd == 0 ? blank_label : r.label;
              const uint32_t qq = kd == 0 ? r.bp_blank : r.bp_nblank;
              if (qq >= kBpRestart) break;
              k = (int)(qq >> 1);
              kd = (int)(qq & 1u);
            }
          }
        }
        // reverse into order
        for (int i = 0; i < len / 2; ++i) { int32_t tmp = o[i]; o[i] = o[len - 1 - i]; o[len - 1 - i] = tmp; }
        out_len[(b * P + q) * 2 + which] = len;
      }
    }
  }
  return 0;
}

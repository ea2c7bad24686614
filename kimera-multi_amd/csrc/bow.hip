// bow.hip — the BoW candidate stage of Kimera-Multi-LCD on MI355X (gfx950).
//
// Replaces DBoW2 Database::queryL1 and L1Scoring::score as called by
// LoopClosureDetector::detectLoop / detectLoopWithRobot (drawio:2574-2580,
// 2612-2633) behind kmx_bow_* (include/kmx_abi.h).
//
//   * k_bow_query: one workgroup per query (grid-stride over the batch), with
//     a private dense accumulator acc[n_entries] and touched-list in HBM.
//     The query's words are visited in increasing word id; for each word the
//     workgroup streams the word's posting list in parallel — an entry occurs
//     at most once per posting list, so there are no write conflicts inside a
//     word — and a barrier separates words. Every entry therefore accumulates
//     |q - d| - |q| - |d| in exactly DBoW2's order (word, then entry), so the
//     scores are bit-identical to the CPU restatement (oracle/bow_oracle.c).
//   * Top-K (max_db_results) by (acc ascending, entry id ascending):
//     LDS histograms over the acc range narrow the candidates to <= SEL_CAP,
//     which are sorted in LDS (bitonic) — no pass over all n_entries.
//   * k_bow_pair_score: one thread per pair, the sorted-list merge of
//     L1Scoring::score (nss factor against the previous keyframe).
// Compiled with -ffp-contract=off (no FMA to contract here anyway).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "common.h"

namespace {

constexpr int BOW_BLOCK = 256;
constexpr int NBINS = 1024;
constexpr int SEL_CAP = 2048;
constexpr int MAX_RESULTS = 256;
constexpr int LEVELS = 6;

struct BowDb {
  const int* ptr;     // [n_words + 1]
  const int* ent;     // posting entry ids (increasing per word)
  const double* wt;   // posting weights
  int n_words, n_entries;
};

__device__ __forceinline__ bool key_less(double a, int ia, double b, int ib) {
  return a < b || (a == b && ia < ib);
}

// First histogram bin b at which the running count reaches `need` (the last
// bin if none does), and the count strictly before it: a block-wide prefix
// sum over NBINS bins (NBINS / BLOCK consecutive bins per thread), replacing
// a serial walk over the bins by one thread. Results in *sb, *scb; needs a
// __syncthreads() before they are read. `wsum` holds BLOCK / 64 ints.
template <int BLOCK>
__device__ __forceinline__ void find_bin(const int* hist, int need, int* wsum, int* sb, int* scb) {
  constexpr int PER = NBINS / BLOCK;
  static_assert(PER * BLOCK == NBINS, "NBINS must be a multiple of the block size");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int h[PER], mine = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) { h[k] = hist[tid * PER + k]; mine += h[k]; }
  int incl = mine;  // inclusive scan over the wave
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off, 64);
    if (lane >= off) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int base = 0;
  for (int k = 0; k < w; ++k) base += wsum[k];
  int cum = base + incl - mine;  // count before this thread's first bin
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int b = tid * PER + k;
    if (cum < need && cum + h[k] >= need) { *sb = b; *scb = cum; }
    else if (b == NBINS - 1 && cum + h[k] < need) { *sb = b; *scb = cum; }
    cum += h[k];
  }
}

// The workgroup's next query (workgroup-uniform): one atomic per query on a
// counter the launch starts at 0, so a workgroup that drew short posting lists
// takes more queries instead of every workgroup taking every gridDim-th one.
__device__ __forceinline__ int next_query(int* next, int nq) {
  __shared__ int s_q;
  __syncthreads();  // the previous query's readers of s_q are done
  if (threadIdx.x == 0) s_q = atomicAdd(next, 1);
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(min(s_q, nq));  // uniform: keep it in a scalar register
}

__global__ __launch_bounds__(BOW_BLOCK) void k_bow_query(BowDb db, int nq, const long long* qptr,
                                                         const unsigned* qw, const double* qv,
                                                         const int* max_id, int K, double* acc_all,
                                                         int* touched_all, int* out_n, int* out_id,
                                                         double* out_score, int* err, int* next) {
  __shared__ int s_nt, s_ns, s_b, s_cb, s_done;
  __shared__ int s_wsum[BOW_BLOCK / 64];
  __shared__ int hist[NBINS];
  __shared__ double c_val[SEL_CAP];
  __shared__ int c_id[SEL_CAP];
  const int tid = threadIdx.x;
  double* acc = acc_all + (size_t)blockIdx.x * db.n_entries;
  int* touched = touched_all + (size_t)blockIdx.x * db.n_entries;
  for (;;) {  // a work queue: the next query from a counter (queries differ in postings by 10x)
    const int q = next_query(next, nq);
    if (q >= nq) break;
    const int mid = max_id ? max_id[q] : -1;
    if (tid == 0) s_nt = 0;
    __syncthreads();
    // ---- phase 1: inverted-file accumulation, word by word
    for (long long i = qptr[q]; i < qptr[q + 1]; ++i) {
      const unsigned w = qw[i];
      if (w < (unsigned)db.n_words) {
        const double qval = qv[i];
        const int p0 = db.ptr[w], p1 = db.ptr[w + 1];
        for (int p = p0 + tid; p < p1; p += BOW_BLOCK) {
          const int e = db.ent[p];
          if (!(e < mid || mid == -1)) continue;
          const double d = db.wt[p];
          const double v = fabs(qval - d) - fabs(qval) - fabs(d);
          const double a = acc[e];
          if (a == 0.0) touched[atomicAdd(&s_nt, 1)] = e;  // values are < 0: 0 = untouched
          acc[e] = a + v;
        }
      }
      __syncthreads();
    }
    const int nt = s_nt;
    // ---- phase 2: top-K by (acc, id). Level l splits the current range into
    // NBINS bins; an entry stays in play while its bin equals the chosen bin
    // at every earlier level (bins recomputed from the same (lo, width) chain,
    // so membership is consistent), and is certain once its bin is below it.
    const int need0 = min(K, nt);
    int need = need0;
    double lvl_lo[LEVELS], lvl_w[LEVELS];
    int lvl_b[LEVELS];
    if (tid == 0) { s_ns = 0; s_done = 0; }
    __syncthreads();
    auto bin_of = [&](double a, int l) {
      int bb = (int)floor((a - lvl_lo[l]) / lvl_w[l]);
      return bb < 0 ? 0 : (bb >= NBINS ? NBINS - 1 : bb);
    };
    auto in_play = [&](double a, int level) {
      for (int l = 0; l < level; ++l)
        if (bin_of(a, l) != lvl_b[l]) return false;
      return true;
    };
    int level = 0;
    for (; level < LEVELS && need > 0; ++level) {
      lvl_lo[level] = level == 0 ? -2.0 : lvl_lo[level - 1] + lvl_b[level - 1] * lvl_w[level - 1];
      lvl_w[level] = (level == 0 ? 2.0 : lvl_w[level - 1]) / NBINS;
      for (int b = tid; b < NBINS; b += BOW_BLOCK) hist[b] = 0;
      __syncthreads();
      for (int i = tid; i < nt; i += BOW_BLOCK) {
        const double a = acc[touched[i]];
        if (in_play(a, level)) atomicAdd(&hist[bin_of(a, level)], 1);
      }
      __syncthreads();
      find_bin<BOW_BLOCK>(hist, need, s_wsum, &s_b, &s_cb);  // first bin reaching `need`
      __syncthreads();
      if (tid == 0) s_done = (s_ns + s_cb + hist[s_b] <= SEL_CAP) ? 1 : 0;
      __syncthreads();
      const int b = s_b, done = s_done, cb = s_cb;
      lvl_b[level] = b;
      for (int i = tid; i < nt; i += BOW_BLOCK) {
        const int e = touched[i];
        const double a = acc[e];
        if (!in_play(a, level)) continue;
        const int bb = bin_of(a, level);
        if (bb < b || (done && bb == b)) {
          const int slot = atomicAdd(&s_ns, 1);
          if (slot < SEL_CAP) { c_val[slot] = a; c_id[slot] = e; }
        }
      }
      __syncthreads();
      if (done) { need = 0; break; }
      need -= cb;
    }
    if (need > 0 && tid == 0) atomicExch(err, 1);  // > SEL_CAP exactly tied scores
    const int nc = min(s_ns, SEL_CAP);
    // bitonic sort of the candidates (padded to a power of two)
    int n2 = 1;
    while (n2 < nc) n2 <<= 1;
    for (int i = nc + tid; i < n2; i += BOW_BLOCK) { c_val[i] = 1.0; c_id[i] = 0x7fffffff; }
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < n2; i += BOW_BLOCK) {
          const int l = i ^ j;
          if (l > i) {
            const bool up = (i & k) == 0;
            const bool sw = up ? key_less(c_val[l], c_id[l], c_val[i], c_id[i])
                               : key_less(c_val[i], c_id[i], c_val[l], c_id[l]);
            if (sw) {
              const double tv = c_val[i]; c_val[i] = c_val[l]; c_val[l] = tv;
              const int ti = c_id[i]; c_id[i] = c_id[l]; c_id[l] = ti;
            }
          }
        }
        __syncthreads();
      }
    }
    const int nout = min(need0, nc);
    for (int i = tid; i < nout; i += BOW_BLOCK) {
      out_id[(size_t)q * K + i] = c_id[i];
      out_score[(size_t)q * K + i] = -c_val[i] / 2.0;
    }
    if (tid == 0) out_n[q] = nout;
    // ---- phase 3: clear the accumulator for the next query
    for (int i = tid; i < nt; i += BOW_BLOCK) acc[touched[i]] = 0.0;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_bow_query_lds: the same queryL1 with the accumulator in LDS.
//   * The database's entries are cut into chunks of `ch` (<= LCH) entries; a
//     chunk's accumulator is an LDS array, so the per-posting read-modify-write
//     that bounds k_bow_query (a dependent HBM round trip per word, then a
//     workgroup barrier) becomes an LDS one.
//   * Within a chunk, wave v of the LW_WAVES owns the entry sub-range
//     [v*sch, (v+1)*sch): it walks the query's words in order over its own
//     part of each posting list ([cptr[w][s], cptr[w][s+1]), s = sub-chunk;
//     lists ascend in entry id). No two waves touch an entry and a wave's LDS
//     operations complete in order, so every entry accumulates in DBoW2's
//     word order with no barrier at all. The wave applies several words'
//     pieces per step (collisions detected by LDS marks) and keeps three
//     steps of postings in flight (unconditional clamped loads, so the
//     compiler waits only for the step being applied).
//   * After each chunk, the chunk's K best (acc, id) are selected as in
//     k_bow_query (LDS histograms + bitonic sort) and merged with the running
//     list by merge-path ranks, so the result equals a top-K over all entries.
constexpr int LW_WAVES = 16;
constexpr int LW_BLOCK = 64 * LW_WAVES;
constexpr int LCH = 14336;     // max entries per chunk (112 KB of LDS), a multiple of LW_WAVES
constexpr int LSEL = 1024;     // candidate cap per chunk
constexpr int QW = 128;        // query words staged per batch
#ifndef KMX_BOW_PG
#define KMX_BOW_PG 8
#endif
constexpr int PG = KMX_BOW_PG;  // lanes per piece group: a step applies 64 / PG pieces of <= PG postings
constexpr int NGRP = 64 / PG;
constexpr int PC = 176;        // pieces per wave table

__global__ __launch_bounds__(LW_BLOCK) void k_bow_query_lds(BowDb db, const int* cptr, int nch, int ch, int nq,
                                                            const long long* qptr, const unsigned* qw,
                                                            const double* qv, const int* max_id, int K,
                                                            int* out_n, int* out_id, double* out_score,
                                                            int* err, int* next) {
  extern __shared__ __attribute__((aligned(16))) char bsm[];
  double* acc = reinterpret_cast<double*>(bsm);                   // [ch]
  double* c_val = acc + LCH;                                        // [LSEL]        \  selection scratch;
  double* m_val = c_val + LSEL;                                     // [MAX_RESULTS]  | the accumulation's
  int* c_id = reinterpret_cast<int*>(m_val + MAX_RESULTS);          // [LSEL]         | conflict marks
  int* m_id = c_id + LSEL;                                          // [MAX_RESULTS] /  alias it
  double* r_val = reinterpret_cast<double*>(m_id + MAX_RESULTS);    // [MAX_RESULTS] running best
  double* wq = r_val + MAX_RESULTS;                                 // [QW] query weights
  int* r_id = reinterpret_cast<int*>(wq + QW);                      // [MAX_RESULTS]
  int* pstart = r_id + MAX_RESULTS;                                 // [LW_WAVES][PC] piece: first posting
  unsigned short* pinfo = reinterpret_cast<unsigned short*>(pstart + LW_WAVES * PC);  // len-1 | word << 4
  int* hist = reinterpret_cast<int*>(pinfo + LW_WAVES * PC);        // [NBINS]
  __shared__ int s_ns, s_b, s_cb, s_done, s_nt, s_nr;
  __shared__ int s_wsum[LW_WAVES];
  const int tid = threadIdx.x, v = tid >> 6, lane = tid & 63;
  const int nsub = nch * LW_WAVES, sch = ch / LW_WAVES;
  for (;;) {  // a work queue: the next query from a counter (queries differ in postings by 10x)
    const int q = next_query(next, nq);
    if (q >= nq) break;
    const int mid = max_id ? max_id[q] : -1;
    const int lim = (mid < 0) ? db.n_entries : min(mid, db.n_entries);  // entries < lim are eligible
    const long long q0 = qptr[q], q1 = qptr[q + 1];
    if (tid == 0) s_nr = 0;
    for (int c = 0; c < nch && c * ch < lim; ++c) {
      const int lo = c * ch, n_here = min(ch, lim - lo);
      for (int i = tid; i < n_here; i += LW_BLOCK) acc[i] = 0.0;
      // ---- accumulation, query words in order, QW words staged at a time.
      // Each wave turns its sub-range of the batch's posting lists into pieces
      // of <= PG postings (a long list becomes consecutive pieces of the same
      // word) and applies 64 / PG pieces per step, one per PG-lane group
      // (PG = 8: 8 pieces; 16 and 32 measured 5 % and 29 % slower). Pieces of
      // different words may hit the same entry: the lanes mark their entries
      // with their group and read the marks back; on a collision the step's
      // pieces are applied one after another, so every entry still
      // accumulates in word order.
      int* my_start = pstart + v * PC;
      unsigned short* my_info = pinfo + v * PC;
      // volatile: the read-back must see other lanes' writes (no store-to-load forwarding)
      volatile unsigned char* mark = reinterpret_cast<unsigned char*>(c_val) + v * sch;
      const int g = lane / PG, j = lane - g * PG;
      const int sub = c * LW_WAVES + v;
      const bool sub_live = lo + v * sch < lim;
      const bool sub_cut = lo + (v + 1) * sch > lim;  // the sub-range holding max_id: drop entries >= lim
      const int mlo = lo + v * sch;
      auto run = [&](int np) {  // apply this wave's piece table [0, np)
        const int nst = (np + NGRP - 1) / NGRP;
        auto fetch = [&](int st, int& e, double& dv, int& wi, bool& ok) {
          const int pc = min(NGRP * st + g, max(np - 1, 0));
          const unsigned info = my_info[pc];
          ok = (NGRP * st + g < np) && (j <= (int)(info & 31u));
          wi = (int)(info >> 5);
          const int idx = ok ? my_start[pc] + j : 0;
          e = db.ent[idx];
          dv = db.wt[idx];
        };
        auto apply = [&](int e, double dv, int wi, bool ok) {
          const int el = e - mlo;
          if (ok) mark[el] = (unsigned char)g;
          bool clash = ok && mark[el] != (unsigned char)g;
          const double qval = wq[wi];
          const double val = fabs(qval - dv) - fabs(qval) - fabs(dv);
          if (!__any(clash)) {
            if (ok) acc[e - lo] += val;
          } else {  // one group at a time, in piece (= word) order
            volatile double* vacc = acc;
            for (int gg = 0; gg < NGRP; ++gg) {
              if (ok && g == gg) vacc[e - lo] = vacc[e - lo] + val;
              __builtin_amdgcn_wave_barrier();
              asm volatile("" ::: "memory");
            }
          }
        };
        int e0, e1, e2, e3, w0, w1, w2, w3;
        double d0, d1, d2, d3;
        bool k0, k1, k2, k3;
        fetch(0, e0, d0, w0, k0);
        fetch(1, e1, d1, w1, k1);
        fetch(2, e2, d2, w2, k2);
        for (int st = 0; st < nst; st += 4) {
          fetch(st + 3, e3, d3, w3, k3);
          apply(e0, d0, w0, k0);
          if (st + 1 >= nst) break;
          fetch(st + 4, e0, d0, w0, k0);
          apply(e1, d1, w1, k1);
          if (st + 2 >= nst) break;
          fetch(st + 5, e1, d1, w1, k1);
          apply(e2, d2, w2, k2);
          if (st + 3 >= nst) break;
          fetch(st + 6, e2, d2, w2, k2);
          apply(e3, d3, w3, k3);
        }
      };
      for (long long b0 = q0; b0 < q1; b0 += QW) {
        const int nw = (int)min((long long)QW, q1 - b0);
        __syncthreads();  // accumulator zeroed / previous batch's weights no longer read
        for (int i = tid; i < nw; i += LW_BLOCK) wq[i] = qv[b0 + i];
        __syncthreads();
        int np = 0;
        for (int w0 = 0; w0 < nw; w0 += 64) {
          // this lane's word: posting range in the wave's sub-range, piece count
          const int i = w0 + lane;
          int a = 0, b = 0;
          if (i < nw && sub_live) {
            const unsigned w = qw[b0 + i];
            if (w < (unsigned)db.n_words) {
              a = cptr[(size_t)w * (nsub + 1) + sub];
              b = cptr[(size_t)w * (nsub + 1) + sub + 1];
              if (sub_cut)
                while (a < b && db.ent[b - 1] >= lim) --b;
            }
          }
          const int cnt = (b - a + PG - 1) / PG;
          int incl = cnt;  // inclusive scan of the piece counts over the wave
#pragma unroll
          for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
          }
          const int gtot = __shfl(incl, 63, 64);
          if (np + gtot > PC) {  // table full: apply it first
            run(np);
            np = 0;
          }
          if (gtot > PC) {  // one 64-word group with very long lists: plain order-preserving loop
            for (int k = 0; k < 64 && w0 + k < nw; ++k) {
              const int ak = __shfl(a, k, 64), bk = __shfl(b, k, 64);
              const double qval = wq[w0 + k];
              for (int sl = ak + lane; sl < bk; sl += 64) {
                const double d = db.wt[sl];
                acc[db.ent[sl] - lo] += fabs(qval - d) - fabs(qval) - fabs(d);
              }
            }
            continue;
          }
          for (int k = 0, pos = np + incl - cnt; k < cnt; ++k, ++pos) {
            my_start[pos] = a + k * PG;
            my_info[pos] = (unsigned short)((min(PG, b - a - k * PG) - 1) | (i << 5));
          }
          np += gtot;
        }
        run(np);
      }
      __syncthreads();
      // ---- this chunk's best min(K, touched) by (acc, id): LDS histogram narrowing
      if (tid == 0) { s_nt = 0; s_ns = 0; s_done = 0; }
      __syncthreads();
      {
        int cnt = 0;
        for (int i = tid; i < n_here; i += LW_BLOCK) cnt += (acc[i] != 0.0) ? 1 : 0;
        if (cnt) atomicAdd(&s_nt, cnt);
      }
      __syncthreads();
      const int nt = s_nt;
      const int need0 = min(K, nt);
      int need = need0;
      double lvl_lo[LEVELS], lvl_w[LEVELS];
      int lvl_b[LEVELS];
      auto bin_of = [&](double a, int l) {
        int bb = (int)floor((a - lvl_lo[l]) / lvl_w[l]);
        return bb < 0 ? 0 : (bb >= NBINS ? NBINS - 1 : bb);
      };
      auto in_play = [&](double a, int level) {
        for (int l = 0; l < level; ++l)
          if (bin_of(a, l) != lvl_b[l]) return false;
        return true;
      };
      for (int level = 0; level < LEVELS && need > 0; ++level) {
        lvl_lo[level] = level == 0 ? -2.0 : lvl_lo[level - 1] + lvl_b[level - 1] * lvl_w[level - 1];
        lvl_w[level] = (level == 0 ? 2.0 : lvl_w[level - 1]) / NBINS;
        for (int b = tid; b < NBINS; b += LW_BLOCK) hist[b] = 0;
        __syncthreads();
        for (int i = tid; i < n_here; i += LW_BLOCK) {
          const double a = acc[i];
          if (a != 0.0 && in_play(a, level)) atomicAdd(&hist[bin_of(a, level)], 1);
        }
        __syncthreads();
        find_bin<LW_BLOCK>(hist, need, s_wsum, &s_b, &s_cb);  // first bin reaching `need`
        __syncthreads();
        if (tid == 0) s_done = (s_ns + s_cb + hist[s_b] <= LSEL) ? 1 : 0;
        __syncthreads();
        const int b = s_b, done = s_done, cb = s_cb;
        lvl_b[level] = b;
        for (int i = tid; i < n_here; i += LW_BLOCK) {
          const double a = acc[i];
          if (a == 0.0 || !in_play(a, level)) continue;
          const int bb = bin_of(a, level);
          if (bb < b || (done && bb == b)) {
            const int slot = atomicAdd(&s_ns, 1);
            if (slot < LSEL) { c_val[slot] = a; c_id[slot] = lo + i; }
          }
        }
        __syncthreads();
        if (done) { need = 0; break; }
        need -= cb;
      }
      if (need > 0 && tid == 0) atomicExch(err, 1);  // > LSEL exactly tied scores
      const int nc = min(s_ns, LSEL);
      int n2 = 1;
      while (n2 < nc) n2 <<= 1;
      for (int i = nc + tid; i < n2; i += LW_BLOCK) { c_val[i] = 1.0; c_id[i] = 0x7fffffff; }
      __syncthreads();
      for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = tid; i < n2; i += LW_BLOCK) {
            const int l = i ^ j;
            if (l > i) {
              const bool up = (i & k) == 0;
              const bool sw = up ? key_less(c_val[l], c_id[l], c_val[i], c_id[i])
                                 : key_less(c_val[i], c_id[i], c_val[l], c_id[l]);
              if (sw) {
                const double tv = c_val[i]; c_val[i] = c_val[l]; c_val[l] = tv;
                const int ti = c_id[i]; c_id[i] = c_id[l]; c_id[l] = ti;
              }
            }
          }
          __syncthreads();
        }
      }
      // ---- merge the chunk's sorted best (na) into the running best (nr) by ranks
      const int na = min(need0, nc), nr = s_nr;
      const int nm = min(K, na + nr);
      for (int i = tid; i < na + nr; i += LW_BLOCK) {
        const bool fromA = i < na;
        const int k = fromA ? i : i - na;
        const double val = fromA ? c_val[k] : r_val[k];
        const int id = fromA ? c_id[k] : r_id[k];
        int l = 0, h = fromA ? nr : na;  // elements of the other list ordered before (val, id)
        while (l < h) {
          const int m = (l + h) >> 1;
          const bool before = fromA ? key_less(r_val[m], r_id[m], val, id) : key_less(c_val[m], c_id[m], val, id);
          if (before) l = m + 1;
          else h = m;
        }
        const int pos = k + l;
        if (pos < nm) { m_val[pos] = val; m_id[pos] = id; }
      }
      __syncthreads();
      for (int i = tid; i < nm; i += LW_BLOCK) { r_val[i] = m_val[i]; r_id[i] = m_id[i]; }
      if (tid == 0) s_nr = nm;
      __syncthreads();
    }
    __syncthreads();
    const int nout = s_nr;
    for (int i = tid; i < nout; i += LW_BLOCK) {
      out_id[(size_t)q * K + i] = r_id[i];
      out_score[(size_t)q * K + i] = -r_val[i] / 2.0;
    }
    if (tid == 0) out_n[q] = nout;
    __syncthreads();
  }
}
constexpr size_t LDS_BOW = sizeof(double) * (LCH + LSEL + 2 * MAX_RESULTS + QW) +
                           sizeof(int) * (LSEL + 2 * MAX_RESULTS + LW_WAVES * PC + NBINS) +
                           sizeof(unsigned short) * LW_WAVES * PC;
static_assert(LW_WAVES * (LCH / LW_WAVES) <= sizeof(double) * (LSEL + MAX_RESULTS) + sizeof(int) * (LSEL + MAX_RESULTS),
              "conflict marks must fit the selection scratch");
static_assert(QW <= 2048 && PG <= 32 && 64 % PG == 0, "piece info packs len - 1 in 5 bits and the word in 11");
static_assert(LDS_BOW + 64 <= 160 * 1024, "k_bow_query_lds exceeds the 160 KiB of LDS per CU");

// L1Scoring::score of pairs (a_i, b_i): merge of the two sorted word lists.
__global__ void k_bow_pair_score(int n, const long long* aptr, const unsigned* aw, const double* av,
                                 const long long* bptr, const unsigned* bw, const double* bv, double* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  long long i = aptr[t], j = bptr[t];
  const long long ie = aptr[t + 1], je = bptr[t + 1];
  double s = 0.0;
  while (i < ie && j < je) {
    const unsigned x = aw[i], y = bw[j];
    if (x == y) {
      s += fabs(av[i] - bv[j]) - fabs(av[i]) - fabs(bv[j]);
      ++i;
      ++j;
    } else if (x < y) {
      ++i;
    } else {
      ++j;
    }
  }
  out[t] = -s / 2.0;
}

template <typename T>
int bow_alloc(T** p, size_t n) {
  *p = nullptr;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * std::max<size_t>(n, 1));
  if (e != hipSuccess) return kmx::fail(KMX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return 0;
}

}  // namespace

struct kmx_bow {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int n_words = 0, n_entries = 0;
  int *d_ptr = nullptr, *d_ent = nullptr;
  double* d_wt = nullptr;
  // query scratch
  int n_wg = 0;
  double* d_acc = nullptr;
  int* d_touched = nullptr;
  int* d_err = nullptr;
  // LDS-accumulator query (k_bow_query_lds): per-word chunk split points
  bool lds = true;
  int ch = 0, nch = 0;
  int* d_cptr = nullptr;
  size_t qcap = 0, wcap = 0;
  long long* d_qptr = nullptr;
  unsigned* d_qw = nullptr;
  double* d_qv = nullptr;
  int* d_maxid = nullptr;
  int *d_n = nullptr, *d_id = nullptr;
  double* d_score = nullptr;
  size_t rcap = 0;
  // pair-score scratch
  size_t pcap = 0, pwcap = 0;
  long long *d_aptr = nullptr, *d_bptr = nullptr;
  unsigned *d_aw = nullptr, *d_bw = nullptr;
  double *d_av = nullptr, *d_bv = nullptr, *d_pout = nullptr;
};

namespace {
void bow_free_db(kmx_bow* h) {
  for (void* p : {(void*)h->d_ptr, (void*)h->d_ent, (void*)h->d_wt, (void*)h->d_acc, (void*)h->d_touched,
                  (void*)h->d_cptr})
    if (p) (void)hipFree(p);
  h->d_ptr = h->d_ent = h->d_cptr = nullptr;
  h->d_wt = nullptr;
  h->d_acc = nullptr;
  h->d_touched = nullptr;
  h->n_wg = 0;
}
void bow_free_q(kmx_bow* h) {
  for (void* p : {(void*)h->d_qptr, (void*)h->d_qw, (void*)h->d_qv, (void*)h->d_maxid, (void*)h->d_n,
                  (void*)h->d_id, (void*)h->d_score})
    if (p) (void)hipFree(p);
  h->d_qptr = nullptr; h->d_qw = nullptr; h->d_qv = nullptr; h->d_maxid = nullptr;
  h->d_n = h->d_id = nullptr; h->d_score = nullptr;
  h->qcap = h->wcap = h->rcap = 0;
}
void bow_free_p(kmx_bow* h) {
  for (void* p : {(void*)h->d_aptr, (void*)h->d_bptr, (void*)h->d_aw, (void*)h->d_bw, (void*)h->d_av,
                  (void*)h->d_bv, (void*)h->d_pout})
    if (p) (void)hipFree(p);
  h->d_aptr = h->d_bptr = nullptr; h->d_aw = h->d_bw = nullptr;
  h->d_av = h->d_bv = h->d_pout = nullptr;
  h->pcap = h->pwcap = 0;
}
}  // namespace

extern "C" int kmx_bow_create(int device, kmx_bow** out) {
  KMX_GUARD_BEGIN
  KMX_CHECK(out, KMX_EINVAL, "null argument");
  int ndev = 0;
  KMX_HIP(hipGetDeviceCount(&ndev));
  KMX_CHECK(device >= 0 && device < ndev, KMX_EINVAL, "bad HIP device ordinal");
  KMX_HIP(hipSetDevice(device));
  kmx_bow* h = new kmx_bow();
  h->device = device;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return kmx::fail(KMX_EHIP, "hipStreamCreate failed");
  }
  h->own_stream = true;
  if (hipMalloc(reinterpret_cast<void**>(&h->d_err), 2 * sizeof(int)) != hipSuccess) {
    (void)hipStreamDestroy(h->stream);
    delete h;
    return kmx::fail(KMX_ENOMEM, "hipMalloc failed");
  }
  *out = h;
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_bow_destroy(kmx_bow* h) {
  if (!h) return KMX_OK;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  bow_free_db(h);
  bow_free_q(h);
  bow_free_p(h);
  if (h->d_err) (void)hipFree(h->d_err);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return KMX_OK;
}

extern "C" int kmx_bow_set_stream(kmx_bow* h, void* s) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  if (h->own_stream && h->stream) {
    KMX_HIP(hipStreamSynchronize(h->stream));
    KMX_HIP(hipStreamDestroy(h->stream));
  }
  h->own_stream = false;
  h->stream = reinterpret_cast<hipStream_t>(s);
  return KMX_OK;
}

extern "C" int kmx_bow_set_database(kmx_bow* h, int32_t n_words, int32_t n_entries, const int64_t* vptr,
                                    const uint32_t* words, const double* weights) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h && vptr && n_words > 0 && n_entries >= 0, KMX_EINVAL, "bad argument");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  const int64_t nnz = vptr[n_entries];
  KMX_CHECK(nnz >= 0 && nnz < INT32_MAX, KMX_EINVAL, "database too large (postings must fit int32)");
  std::vector<int> ptr((size_t)n_words + 1, 0);
  for (int e = 0; e < n_entries; ++e) {
    KMX_CHECK(vptr[e + 1] >= vptr[e], KMX_EINVAL, "vptr not monotone");
    for (int64_t k = vptr[e]; k < vptr[e + 1]; ++k) {
      KMX_CHECK(words[k] < (uint32_t)n_words, KMX_EINVAL, "word id >= n_words");
      KMX_CHECK(k == vptr[e] || words[k] > words[k - 1], KMX_EINVAL, "BowVector words must be strictly increasing");
      ptr[words[k] + 1]++;
    }
  }
  for (int w = 0; w < n_words; ++w) ptr[w + 1] += ptr[w];
  std::vector<int> fill(ptr.begin(), ptr.end() - 1), ent(std::max<int64_t>(nnz, 1));
  std::vector<double> wt(std::max<int64_t>(nnz, 1));
  for (int e = 0; e < n_entries; ++e)  // entries added in id order: posting lists ascending
    for (int64_t k = vptr[e]; k < vptr[e + 1]; ++k) {
      const int p = fill[words[k]]++;
      ent[p] = e;
      wt[p] = weights[k];
    }
  bow_free_db(h);
  h->n_words = n_words;
  h->n_entries = n_entries;
  // KMX_BOW_LDS=0 selects the HBM-accumulator kernel; KMX_BOW_CHUNK sets the
  // entries per LDS chunk (tests use small chunks to cover the merge)
  h->lds = true;
  if (const char* v = std::getenv("KMX_BOW_LDS")) h->lds = std::atoi(v) != 0;
  h->ch = LCH;
  if (const char* v = std::getenv("KMX_BOW_CHUNK")) h->ch = std::max(1, std::min(LCH, std::atoi(v)));
  h->ch = (h->ch + LW_WAVES - 1) / LW_WAVES * LW_WAVES;  // whole sub-ranges, one per wave
  h->nch = std::max(1, (n_entries + h->ch - 1) / h->ch);
  std::vector<int> cptr;
  if (h->lds) {  // first posting of each wave sub-range in every word's (ascending) list
    const int nsub = h->nch * LW_WAVES, sch = h->ch / LW_WAVES;
    cptr.assign((size_t)n_words * (nsub + 1), 0);
    for (int w = 0; w < n_words; ++w) {
      int p = ptr[w];
      for (int c = 0; c <= nsub; ++c) {
        const long long bound = (long long)c * sch;
        while (p < ptr[w + 1] && ent[p] < bound) ++p;
        cptr[(size_t)w * (nsub + 1) + c] = (c == nsub) ? ptr[w + 1] : p;
      }
    }
  }
  // persistent query workgroups: the HBM kernel gives each an acc / touched
  // scratch of n_entries; the LDS kernel runs one workgroup per CU
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
  h->n_wg = h->lds ? std::max(1, cus) : std::max(1, cus * 4);
  const size_t scratch = h->lds ? 1 : (size_t)h->n_wg * std::max(n_entries, 1);
  int rc;
  if ((rc = bow_alloc(&h->d_ptr, ptr.size())) || (rc = bow_alloc(&h->d_ent, ent.size())) ||
      (rc = bow_alloc(&h->d_wt, wt.size())) || (rc = bow_alloc(&h->d_acc, scratch)) ||
      (rc = bow_alloc(&h->d_touched, scratch)) || (h->lds && (rc = bow_alloc(&h->d_cptr, cptr.size())))) {
    bow_free_db(h);
    return rc;
  }
  if (h->lds) KMX_HIP(hipMemcpy(h->d_cptr, cptr.data(), sizeof(int) * cptr.size(), hipMemcpyHostToDevice));
  KMX_HIP(hipMemcpy(h->d_ptr, ptr.data(), sizeof(int) * ptr.size(), hipMemcpyHostToDevice));
  KMX_HIP(hipMemcpy(h->d_ent, ent.data(), sizeof(int) * ent.size(), hipMemcpyHostToDevice));
  KMX_HIP(hipMemcpy(h->d_wt, wt.data(), sizeof(double) * wt.size(), hipMemcpyHostToDevice));
  KMX_HIP(hipMemset(h->d_acc, 0, sizeof(double) * scratch));
  return KMX_OK;
  KMX_GUARD_END
}

namespace {
int bow_upload_queries(kmx_bow* h, int32_t nq, const int64_t* qptr, const uint32_t* words, const double* weights,
                       const int32_t* max_id, int32_t K) {
  const size_t nw = (size_t)qptr[nq];
  if ((size_t)nq + 1 > h->qcap || nw > h->wcap || (size_t)nq * K > h->rcap) {
    bow_free_q(h);
    h->qcap = std::max<size_t>(nq + 1, 1024);
    h->wcap = std::max<size_t>(nw, 1);
    h->rcap = std::max<size_t>((size_t)nq * K, 1);
    int rc;
    if ((rc = bow_alloc(&h->d_qptr, h->qcap)) || (rc = bow_alloc(&h->d_qw, h->wcap)) ||
        (rc = bow_alloc(&h->d_qv, h->wcap)) || (rc = bow_alloc(&h->d_maxid, h->qcap)) ||
        (rc = bow_alloc(&h->d_n, h->qcap)) || (rc = bow_alloc(&h->d_id, h->rcap)) ||
        (rc = bow_alloc(&h->d_score, h->rcap))) {
      bow_free_q(h);
      return rc;
    }
  }
  KMX_HIP(hipMemcpyAsync(h->d_qptr, qptr, sizeof(long long) * (nq + 1), hipMemcpyHostToDevice, h->stream));
  if (nw) {
    KMX_HIP(hipMemcpyAsync(h->d_qw, words, sizeof(unsigned) * nw, hipMemcpyHostToDevice, h->stream));
    KMX_HIP(hipMemcpyAsync(h->d_qv, weights, sizeof(double) * nw, hipMemcpyHostToDevice, h->stream));
  }
  if (max_id) KMX_HIP(hipMemcpyAsync(h->d_maxid, max_id, sizeof(int) * nq, hipMemcpyHostToDevice, h->stream));
  return KMX_OK;
}
}  // namespace

extern "C" int kmx_bow_query_async(kmx_bow* h, int32_t nq, const int64_t* qptr, const uint32_t* words,
                                   const double* weights, const int32_t* max_id, int32_t max_results) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h && h->d_ptr, KMX_ESTATE, "kmx_bow_set_database first");
  KMX_CHECK(nq >= 0 && qptr && max_results > 0 && max_results <= MAX_RESULTS, KMX_EINVAL,
            "bad argument (max_results in [1, 256])");
  KMX_HIP(hipSetDevice(h->device));
  for (int q = 0; q < nq; ++q) KMX_CHECK(qptr[q + 1] >= qptr[q], KMX_EINVAL, "qptr not monotone");
  if (int rc = bow_upload_queries(h, nq, qptr, words, weights, max_id, max_results)) return rc;
  if (nq == 0) return KMX_OK;
  KMX_HIP(hipMemsetAsync(h->d_err, 0, 2 * sizeof(int), h->stream));  // error flag, query counter
  BowDb db{h->d_ptr, h->d_ent, h->d_wt, h->n_words, h->n_entries};
  const int grid = std::min(nq, h->n_wg);
  if (h->lds) {
    hipLaunchKernelGGL(k_bow_query_lds, dim3(grid), dim3(LW_BLOCK), LDS_BOW, h->stream, db,
                       (const int*)h->d_cptr, h->nch, h->ch, nq, (const long long*)h->d_qptr,
                       (const unsigned*)h->d_qw, (const double*)h->d_qv,
                       max_id ? (const int*)h->d_maxid : nullptr, max_results, h->d_n, h->d_id, h->d_score,
                       h->d_err, h->d_err + 1);
    KMX_HIP(hipGetLastError());
    return KMX_OK;
  }
  hipLaunchKernelGGL(k_bow_query, dim3(grid), dim3(BOW_BLOCK), 0, h->stream, db, nq,
                     (const long long*)h->d_qptr, (const unsigned*)h->d_qw, (const double*)h->d_qv,
                     max_id ? (const int*)h->d_maxid : nullptr, max_results, h->d_acc, h->d_touched, h->d_n,
                     h->d_id, h->d_score, h->d_err, h->d_err + 1);
  KMX_HIP(hipGetLastError());
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_bow_query(kmx_bow* h, int32_t nq, const int64_t* qptr, const uint32_t* words,
                             const double* weights, const int32_t* max_id, int32_t max_results, int32_t* out_n,
                             int32_t* out_ids, double* out_scores) {
  KMX_GUARD_BEGIN
  KMX_CHECK(out_n && out_ids && out_scores, KMX_EINVAL, "null output");
  if (int rc = kmx_bow_query_async(h, nq, qptr, words, weights, max_id, max_results)) return rc;
  if (nq == 0) return KMX_OK;
  int err = 0;
  KMX_HIP(hipMemcpyAsync(out_n, h->d_n, sizeof(int) * nq, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipMemcpyAsync(out_ids, h->d_id, sizeof(int) * (size_t)nq * max_results, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipMemcpyAsync(out_scores, h->d_score, sizeof(double) * (size_t)nq * max_results, hipMemcpyDeviceToHost,
                         h->stream));
  KMX_HIP(hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  KMX_CHECK(!err, KMX_EUNSUP, "too many exactly tied scores at the max_results cut");
  return KMX_OK;
  KMX_GUARD_END
}

extern "C" int kmx_bow_sync(kmx_bow* h) {
  KMX_CHECK(h, KMX_EINVAL, "null handle");
  KMX_HIP(hipSetDevice(h->device));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
}

extern "C" int kmx_bow_score_pairs(kmx_bow* h, int32_t n, const int64_t* aptr, const uint32_t* aw,
                                   const double* av, const int64_t* bptr, const uint32_t* bw, const double* bv,
                                   double* out) {
  KMX_GUARD_BEGIN
  KMX_CHECK(h && n >= 0 && aptr && bptr && out, KMX_EINVAL, "bad argument");
  if (n == 0) return KMX_OK;
  KMX_HIP(hipSetDevice(h->device));
  const size_t na = (size_t)aptr[n], nb = (size_t)bptr[n];
  if ((size_t)n + 1 > h->pcap || std::max(na, nb) > h->pwcap) {
    bow_free_p(h);
    h->pcap = std::max<size_t>(n + 1, 1024);
    h->pwcap = std::max<size_t>(std::max(na, nb), 1);
    int rc;
    if ((rc = bow_alloc(&h->d_aptr, h->pcap)) || (rc = bow_alloc(&h->d_bptr, h->pcap)) ||
        (rc = bow_alloc(&h->d_aw, h->pwcap)) || (rc = bow_alloc(&h->d_bw, h->pwcap)) ||
        (rc = bow_alloc(&h->d_av, h->pwcap)) || (rc = bow_alloc(&h->d_bv, h->pwcap)) ||
        (rc = bow_alloc(&h->d_pout, h->pcap))) {
      bow_free_p(h);
      return rc;
    }
  }
  KMX_HIP(hipMemcpyAsync(h->d_aptr, aptr, sizeof(long long) * (n + 1), hipMemcpyHostToDevice, h->stream));
  KMX_HIP(hipMemcpyAsync(h->d_bptr, bptr, sizeof(long long) * (n + 1), hipMemcpyHostToDevice, h->stream));
  if (na) {
    KMX_HIP(hipMemcpyAsync(h->d_aw, aw, sizeof(unsigned) * na, hipMemcpyHostToDevice, h->stream));
    KMX_HIP(hipMemcpyAsync(h->d_av, av, sizeof(double) * na, hipMemcpyHostToDevice, h->stream));
  }
  if (nb) {
    KMX_HIP(hipMemcpyAsync(h->d_bw, bw, sizeof(unsigned) * nb, hipMemcpyHostToDevice, h->stream));
    KMX_HIP(hipMemcpyAsync(h->d_bv, bv, sizeof(double) * nb, hipMemcpyHostToDevice, h->stream));
  }
  hipLaunchKernelGGL(k_bow_pair_score, dim3((n + 255) / 256), dim3(256), 0, h->stream, n,
                     (const long long*)h->d_aptr, (const unsigned*)h->d_aw, (const double*)h->d_av,
                     (const long long*)h->d_bptr, (const unsigned*)h->d_bw, (const double*)h->d_bv, h->d_pout);
  KMX_HIP(hipGetLastError());
  KMX_HIP(hipMemcpyAsync(out, h->d_pout, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
  KMX_HIP(hipStreamSynchronize(h->stream));
  return KMX_OK;
  KMX_GUARD_END
}

/*
 * oracle/bow_oracle.c — CPU restatement of the BoW candidate stage of
 * Kimera-Multi-LCD. TEST INFRASTRUCTURE ONLY (parity
 * checker + cpu_baseline of bench.py); never linked into the product.
 *
 * PARITY STATUS: DBoW2 (dbow2_catkin@master, kimera_multi.repos:14-17) and
 * kimera_multi_lcd are not vendored => "parity unpinned" against upstream.
 * This file restates DBoW2's published L1 scoring (Nister & Stewenius 2006 as
 * implemented by DBoW2 L1Scoring / Database::queryL1) and the detection
 * filters named by the call flow (drawio:1565, 2574-2580, 2612-2633) with the
 * constants of params/D455/LcdParams.yaml:3-12. It is pinned by an independent
 * dense numpy restatement (tests/test_oracle_bow.py).
 *
 *   BowVector ........... sorted (word id, weight) pairs, L1-normalised.
 *   L1 score ............ s(v, w) = -1/2 sum_{i in v and w} (|v_i - w_i| - |v_i| - |w_i|)
 *                         over common words in increasing word id (L1Scoring::score).
 *   queryL1 ............. inverted file: per word, (entry id, weight) in entry
 *                         order. For every query word (increasing id) and every
 *                         posting entry with id < max_id (or max_id == -1):
 *                         acc[id] += |q - d| - |q| - |d|; results sorted by acc
 *                         ascending (ties: lower entry id first [U: DBoW2 uses
 *                         an unstable std::sort]), cut to max_results,
 *                         score = -acc / 2.
 *   detectLoopWithRobot . nss = s(query, previous keyframe of the query robot);
 *                         reject if nss < min_nss_factor (0.05); query the
 *                         robot's DB (max_db_results 50); keep results with
 *                         score >= alpha * nss (alpha 0.4); best = first.
 *   islands / temporal .. computeIslands + checkTemporalConstraint of the
 *                         single-robot detectLoop (max_intraisland_gap 3,
 *                         min_matches_per_island 1, max_nrFrames_between_islands 3,
 *                         max_nrFrames_between_queries 2, min_temporal_matches 1).
 */
#define _GNU_SOURCE /* qsort_r */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ scoring -- */
double orc_bow_score(const uint32_t* w1, const double* v1, int n1, const uint32_t* w2, const double* v2,
                     int n2) {
  double s = 0.0;
  int i = 0, j = 0;
  while (i < n1 && j < n2) {
    if (w1[i] == w2[j]) {
      s += fabs(v1[i] - v2[j]) - fabs(v1[i]) - fabs(v2[j]);
      ++i;
      ++j;
    } else if (w1[i] < w2[j]) {
      ++i;
    } else {
      ++j;
    }
  }
  return -s / 2.0;
}

/* ---------------------------------------------------------- database ---- */
typedef struct {
  int n_words, n_entries;
  int* ptr;       /* [n_words + 1] */
  int* ent;       /* posting entry ids, increasing per word */
  double* wt;     /* posting weights */
  double* acc;    /* [n_entries] scratch (zero between queries) */
  int* touched;   /* [n_entries] list scratch */
} orc_bowdb;

/* Build the inverted file of entries 0..n-1 (entry i = frame i of the CSR). */
void* orc_bowdb_create(int n_words, int n, const int64_t* vptr, const uint32_t* words, const double* weights) {
  orc_bowdb* db = (orc_bowdb*)calloc(1, sizeof(orc_bowdb));
  db->n_words = n_words;
  db->n_entries = n;
  db->ptr = (int*)calloc((size_t)n_words + 1, sizeof(int));
  for (int64_t k = 0; k < vptr[n]; ++k) db->ptr[words[k] + 1]++;
  for (int w = 0; w < n_words; ++w) db->ptr[w + 1] += db->ptr[w];
  const int64_t nnz = vptr[n];
  db->ent = (int*)malloc(sizeof(int) * (size_t)(nnz > 0 ? nnz : 1));
  db->wt = (double*)malloc(sizeof(double) * (size_t)(nnz > 0 ? nnz : 1));
  int* fill = (int*)malloc(sizeof(int) * (size_t)n_words);
  memcpy(fill, db->ptr, sizeof(int) * (size_t)n_words);
  for (int e = 0; e < n; ++e)
    for (int64_t k = vptr[e]; k < vptr[e + 1]; ++k) {
      const int p = fill[words[k]]++;
      db->ent[p] = e;
      db->wt[p] = weights[k];
    }
  free(fill);
  db->acc = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  db->touched = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  return db;
}

void orc_bowdb_destroy(void* h) {
  orc_bowdb* db = (orc_bowdb*)h;
  if (!db) return;
  free(db->ptr);
  free(db->ent);
  free(db->wt);
  free(db->acc);
  free(db->touched);
  free(db);
}

static int cmp_res(const void* a, const void* b, void* ctx) {
  const double* acc = (const double*)ctx;
  const int x = *(const int*)a, y = *(const int*)b;
  if (acc[x] < acc[y]) return -1;
  if (acc[x] > acc[y]) return 1;
  return (x > y) - (x < y);
}

/* queryL1: returns the number of results (<= max_results); ids / scores out. */
int orc_bowdb_query(void* h, const uint32_t* words, const double* weights, int n, int max_results, int max_id,
                    int* out_id, double* out_score) {
  orc_bowdb* db = (orc_bowdb*)h;
  int nt = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t w = words[i];
    if ((int)w >= db->n_words) continue;
    const double q = weights[i];
    for (int p = db->ptr[w]; p < db->ptr[w + 1]; ++p) {
      const int e = db->ent[p];
      if (!(e < max_id || max_id == -1)) continue;
      const double d = db->wt[p];
      const double value = fabs(q - d) - fabs(q) - fabs(d);
      if (db->acc[e] == 0.0) db->touched[nt++] = e; /* values are < 0: 0 means untouched */
      db->acc[e] += value;
    }
  }
  qsort_r(db->touched, (size_t)nt, sizeof(int), cmp_res, db->acc);
  const int k = (max_results > 0 && nt > max_results) ? max_results : nt;
  for (int i = 0; i < k; ++i) {
    out_id[i] = db->touched[i];
    out_score[i] = -db->acc[db->touched[i]] / 2.0;
  }
  for (int i = 0; i < nt; ++i) db->acc[db->touched[i]] = 0.0;
  return k;
}

/* ---------------------------------------------- inter-robot detection --- */
/* detectLoopWithRobot for a batch of queries against one robot's database:
 * query q has BowVector qv[q], previous keyframe pv[q] (n_prev[q] == 0: none).
 * out_match[q] = best entry id or -1; out_score = its score; out_nss = nss. */
void orc_bow_detect_batch(void* h, int nq, const int64_t* qptr, const uint32_t* qw, const double* qv,
                          const int64_t* pptr, const uint32_t* pw, const double* pv, int max_results,
                          double alpha, double min_nss, int* out_match, double* out_score, double* out_nss) {
  int* ids = (int*)malloc(sizeof(int) * (size_t)(max_results > 0 ? max_results : 1));
  double* sc = (double*)malloc(sizeof(double) * (size_t)(max_results > 0 ? max_results : 1));
  for (int q = 0; q < nq; ++q) {
    out_match[q] = -1;
    out_score[q] = 0.0;
    out_nss[q] = 0.0;
    const int nqv = (int)(qptr[q + 1] - qptr[q]), npv = (int)(pptr[q + 1] - pptr[q]);
    if (npv == 0) continue;
    const double nss = orc_bow_score(qw + qptr[q], qv + qptr[q], nqv, pw + pptr[q], pv + pptr[q], npv);
    out_nss[q] = nss;
    if (nss < min_nss) continue;
    const int k = orc_bowdb_query(h, qw + qptr[q], qv + qptr[q], nqv, max_results, -1, ids, sc);
    if (k > 0 && sc[0] >= alpha * nss) {
      out_match[q] = ids[0];
      out_score[q] = sc[0];
    }
  }
  free(ids);
  free(sc);
}

/* ------------------------------------------------ islands / temporal ---- */
typedef struct {
  int start, end, best_id;
  double score, best_score;
} orc_island;

/* computeIslands over query results (id, score), visited in increasing id. */
static int cmp_id(const void* a, const void* b) {
  const int* x = (const int*)a;
  const int* y = (const int*)b;
  return (x[0] > y[0]) - (x[0] < y[0]);
}

int orc_bow_islands(int n, const int* ids, const double* scores, int max_gap, int min_matches, orc_island* out) {
  if (n == 0) return 0;
  if (n == 1) {
    out[0].start = out[0].end = out[0].best_id = ids[0];
    out[0].score = out[0].best_score = scores[0];
    return 1;
  }
  /* sort (id, index) by id; ties impossible (entry ids unique) */
  int* ord = (int*)malloc(sizeof(int) * 2 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    ord[2 * i] = ids[i];
    ord[2 * i + 1] = i;
  }
  qsort(ord, (size_t)n, 2 * sizeof(int), cmp_id);
  int ni = 0;
  int first = ord[0], last = ord[0], i_first = 0, i_last = 0;
  double best_score = scores[ord[1]];
  int best_entry = ord[0];
  for (int idx = 1; idx <= n; ++idx) {
    const int have = idx < n;
    const int id = have ? ord[2 * idx] : 0;
    const double sc = have ? scores[ord[2 * idx + 1]] : 0.0;
    if (have && id - last < max_gap) {
      last = id;
      i_last = idx;
      if (sc > best_score) {
        best_score = sc;
        best_entry = id;
      }
      continue;
    }
    if (last - first + 1 >= min_matches) {
      double s = 0.0;
      for (int k = i_first; k <= i_last; ++k) s += scores[ord[2 * k + 1]];
      out[ni].start = first;
      out[ni].end = last;
      out[ni].score = s;
      out[ni].best_score = best_score;
      out[ni].best_id = best_entry;
      ++ni;
    }
    if (have) {
      first = last = id;
      i_first = i_last = idx;
      best_score = sc;
      best_entry = id;
    }
  }
  free(ord);
  return ni;
}

/* checkTemporalConstraint: state = {temporal_entries, latest_query_id,
 * latest island start, latest island end}; returns 1 when the island passes. */
int orc_bow_temporal(int* state, int query_id, int island_start, int island_end, int max_between_queries,
                     int max_between_islands, int min_temporal_matches) {
  int* te = &state[0];
  if (*te == 0 || query_id - state[1] > max_between_queries) {
    *te = 1;
  } else {
    const int a1 = state[2], a2 = state[3], b1 = island_start, b2 = island_end;
    if ((b1 <= a1 && a1 <= b2) || (a1 <= b1 && b1 <= a2) || (b1 <= a2 && a2 <= b2) || (a1 <= b2 && b2 <= a2)) {
      *te += 1;
    } else {
      const int d1 = a1 - b2, d2 = b1 - a2;
      const int gap = d1 > d2 ? d1 : d2;
      *te = (gap <= max_between_islands) ? *te + 1 : 1;
    }
  }
  state[1] = query_id;
  state[2] = island_start;
  state[3] = island_end;
  return *te > min_temporal_matches;
}

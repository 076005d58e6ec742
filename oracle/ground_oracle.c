/* TEST INFRASTRUCTURE ONLY — C restatement of the reference's path counter.
 *
 * Semantics follow KnowledgeGraph::rule_destination (reference
 * miner/rnnlogic.cpp:412-442) and, equivalently, grounding/propagate
 * (src/data.py:136-173): per (query h, rule body) the number of paths from h
 * along the body, with the query's own edge (rm_src -rel r-> rm_dst) skipped
 * at every hop whose relation is the query relation r.  An empty body yields
 * the one-hot of h (data.py:139-147).
 *
 * Only tests/ and bench.py's cpu_baseline leg call this (via ctypes).  It
 * is pinned against the reference miner (oracle/_ref/libref_miner.so) and the
 * golden COO counts in tests/test_oracle_c.py.
 *
 * Graph layout: vertex-major CSR, edges of (v, rel) are col[off[v*R+rel] ..
 * off[v*R+rel+1]).  Rules: CSR by head relation: rules of head r are
 * positions rh_ptr[r] .. rh_ptr[r+1]-1 (file order), body tokens of position i
 * are body[bptr[i] .. bptr[i+1]) and its global (file) rule id is rid[i].
 *
 * Per query it produces, for every candidate t (total count > 0):
 *   sum[t] = sum_rho count_rho(t)                          (int64)
 *   fp[t]  = sum_rho count_rho(t) * mix64(rho)  mod 2^64    (rule-identity fingerprint)
 * and the order-independent digest  sum_t mix64(t ^ mix64(sum ^ mix64(fp))) mod 2^64,
 * which the HIP path reproduces exactly (tests/test_gpu_*.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

uint64_t oracle_mix64(uint64_t x) { return mix64(x); }

typedef struct {
  const int64_t *off;
  const int32_t *col;
  int R, E;
  const int32_t *rh_ptr, *bptr, *body;
  const int32_t *rid;       /* position in the head-sorted table -> global rule id */
} graph_t;

typedef struct {
  int64_t *cur_c, *nxt_c;   /* dense counts, |E| */
  int32_t *cur_v, *nxt_v;   /* touched lists */
  int64_t *sum;
  uint64_t *fp;
  int32_t *cand;            /* touched candidates */
  int n_cand;
  int64_t F, T, P;          /* frontier expansions, edge traversals, (rule, dest) pairs */
} scratch_t;

static int scratch_init(scratch_t *s, int E) {
  s->cur_c = calloc(E, 8);
  s->nxt_c = calloc(E, 8);
  s->cur_v = malloc((size_t)E * 4);
  s->nxt_v = malloc((size_t)E * 4);
  s->sum = calloc(E, 8);
  s->fp = calloc(E, 8);
  s->cand = malloc((size_t)E * 4);
  s->n_cand = 0;
  s->F = s->T = s->P = 0;
  return s->cur_c && s->nxt_c && s->cur_v && s->nxt_v && s->sum && s->fp && s->cand;
}

static void scratch_free(scratch_t *s) {
  free(s->cur_c); free(s->nxt_c); free(s->cur_v); free(s->nxt_v);
  free(s->sum); free(s->fp); free(s->cand);
}

/* Per-rule statistics of one query (Predictor, reference predictors.py:53-119):
 * for rule position k of the head's list, pos[k] = count at the true tail t,
 * tot[k] = sum of counts over all destinations; wsum[t] += count * w[rule id]
 * accumulates the EM Predictor's score in double. */
typedef struct {
  int t;
  int64_t *pos, *tot;
  const double *w;
  double *wsum;             /* |E|, cleared by the caller */
} rule_stats_t;

/* Ground every rule of head r from h; accumulate sum/fp per candidate
 * (and, when st != NULL, the per-rule statistics). */
static void ground_query_st(const graph_t *g, scratch_t *s, int h, int r, int rm_src, int rm_dst,
                            rule_stats_t *st);

static void ground_query(const graph_t *g, scratch_t *s, int h, int r, int rm_src, int rm_dst) {
  ground_query_st(g, s, h, r, rm_src, rm_dst, NULL);
}

static void ground_query_st(const graph_t *g, scratch_t *s, int h, int r, int rm_src, int rm_dst,
                            rule_stats_t *st) {
  const int R = g->R;
  s->n_cand = 0;
  for (int rule = g->rh_ptr[r]; rule < g->rh_ptr[r + 1]; ++rule) {
    int ncur = 1;
    s->cur_v[0] = h;
    s->cur_c[h] = 1;
    for (int k = g->bptr[rule]; k < g->bptr[rule + 1]; ++k) {
      const int rel = g->body[k];
      int nnxt = 0;
      for (int i = 0; i < ncur; ++i) {
        const int v = s->cur_v[i];
        const int64_t c = s->cur_c[v];
        s->cur_c[v] = 0;
        const int64_t b = g->off[(int64_t)v * R + rel], e = g->off[(int64_t)v * R + rel + 1];
        s->F += 1;
        s->T += e - b;
        for (int64_t j = b; j < e; ++j) {
          const int t = g->col[j];
          if (rel == r && v == rm_src && t == rm_dst) continue;
          if (s->nxt_c[t] == 0) s->nxt_v[nnxt++] = t;
          s->nxt_c[t] += c;
        }
      }
      /* swap */
      int64_t *tc = s->cur_c; s->cur_c = s->nxt_c; s->nxt_c = tc;
      int32_t *tv = s->cur_v; s->cur_v = s->nxt_v; s->nxt_v = tv;
      ncur = nnxt;
    }
    const uint64_t m = mix64((uint64_t)g->rid[rule]);
    const int k = rule - g->rh_ptr[r];
    if (st) {
      st->pos[k] = s->cur_c[st->t];
      st->tot[k] = 0;
    }
    for (int i = 0; i < ncur; ++i) {
      const int t = s->cur_v[i];
      const int64_t c = s->cur_c[t];
      s->cur_c[t] = 0;
      if (c == 0) continue;
      if (st) {
        st->tot[k] += c;
        if (st->w) st->wsum[t] += (double)c * st->w[g->rid[rule]];
      }
      s->P += 1;
      if (s->sum[t] == 0) s->cand[s->n_cand++] = t;
      s->sum[t] += c;
      s->fp[t] += (uint64_t)c * m;
    }
  }
}

static uint64_t digest_and_clear(scratch_t *s, int *n_out) {
  uint64_t d = 0;
  for (int i = 0; i < s->n_cand; ++i) {
    const int t = s->cand[i];
    d += mix64((uint64_t)t ^ mix64((uint64_t)s->sum[t] ^ mix64(s->fp[t])));
    s->sum[t] = 0;
    s->fp[t] = 0;
  }
  *n_out = s->n_cand;
  return d;
}

static int cmp_int(const void *a, const void *b) {
  const int x = *(const int *)a, y = *(const int *)b;
  return (x > y) - (x < y);
}

/* One query, full candidate list sorted by t.  Returns #candidates, or
 * -needed if cap is too small, or -1 on allocation failure. */
int oracle_query_candidates(const int64_t *off, const int32_t *col, int R, int E, const int32_t *rh_ptr,
                            const int32_t *bptr, const int32_t *body, const int32_t *rid, int h, int r,
                            int rm_src, int rm_dst, int32_t *out_t, int64_t *out_sum, uint64_t *out_fp, int cap) {
  graph_t g = {off, col, R, E, rh_ptr, bptr, body, rid};
  scratch_t s;
  if (!scratch_init(&s, E)) { scratch_free(&s); return -1; }
  ground_query(&g, &s, h, r, rm_src, rm_dst);
  const int n = s.n_cand;
  if (n > cap) { scratch_free(&s); return -n; }
  qsort(s.cand, n, sizeof(int32_t), cmp_int);
  for (int i = 0; i < n; ++i) {
    const int t = s.cand[i];
    out_t[i] = t;
    out_sum[i] = s.sum[t];
    out_fp[i] = s.fp[t];
  }
  scratch_free(&s);
  return n;
}

typedef struct {
  const graph_t *g;
  const int32_t *qh, *qr, *qrs, *qrd;
  int nq, nthreads, tid;
  uint64_t *digest;
  int32_t *ncand;
  int64_t *work;    /* optional (F, T, P) per query */
  int ok;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  scratch_t s;
  if (!scratch_init(&s, j->g->E)) { scratch_free(&s); j->ok = 0; return NULL; }
  for (int q = j->tid; q < j->nq; q += j->nthreads) {
    ground_query(j->g, &s, j->qh[q], j->qr[q], j->qrs ? j->qrs[q] : -1, j->qrd ? j->qrd[q] : -1);
    int n;
    j->digest[q] = digest_and_clear(&s, &n);
    j->ncand[q] = n;
    if (j->work) {
      j->work[3 * q] = s.F;
      j->work[3 * q + 1] = s.T;
      j->work[3 * q + 2] = s.P;
      s.F = s.T = s.P = 0;
    }
  }
  scratch_free(&s);
  j->ok = 1;
  return NULL;
}

/* Many queries over `nthreads` pthreads: per-query digest + candidate count.
 * rm_src/rm_dst may be NULL (no edge removal); work (3 x nq) may be NULL.
 * Returns 0 on success. */
int oracle_digests(const int64_t *off, const int32_t *col, int R, int E, const int32_t *rh_ptr,
                   const int32_t *bptr, const int32_t *body, const int32_t *rid, const int32_t *qh,
                   const int32_t *qr,
                   const int32_t *rm_src, const int32_t *rm_dst, int nq, int nthreads, uint64_t *digest,
                   int32_t *ncand, int64_t *work) {
  graph_t g = {off, col, R, E, rh_ptr, bptr, body, rid};
  if (nthreads < 1) nthreads = 1;
  pthread_t *th = malloc(sizeof(pthread_t) * nthreads);
  job_t *jobs = malloc(sizeof(job_t) * nthreads);
  for (int i = 0; i < nthreads; ++i) {
    jobs[i] = (job_t){&g, qh, qr, rm_src, rm_dst, nq, nthreads, i, digest, ncand, work, 0};
    pthread_create(&th[i], NULL, worker, &jobs[i]);
  }
  int ok = 1;
  for (int i = 0; i < nthreads; ++i) {
    pthread_join(th[i], NULL);
    ok &= jobs[i].ok;
  }
  free(th);
  free(jobs);
  return ok ? 0 : 1;
}

typedef struct {
  const graph_t *g;
  const int32_t *qh, *qr, *qrs, *qrd, *qt;
  int nq, nthreads, tid;
  const double *w;
  const int64_t *rq_ptr, *cand_ptr;
  int64_t *pos, *tot;
  int32_t *out_t;
  double *out_score;
  int ok;
} stats_job_t;

static void *stats_worker(void *arg) {
  stats_job_t *j = (stats_job_t *)arg;
  scratch_t s;
  double *wsum = calloc(j->g->E, sizeof(double));
  if (!scratch_init(&s, j->g->E) || !wsum) { scratch_free(&s); free(wsum); j->ok = 0; return NULL; }
  j->ok = 1;
  for (int q = j->tid; q < j->nq; q += j->nthreads) {
    rule_stats_t st = {j->qt[q], j->pos + j->rq_ptr[q], j->tot + j->rq_ptr[q], j->w, wsum};
    ground_query_st(j->g, &s, j->qh[q], j->qr[q], j->qrs ? j->qrs[q] : -1, j->qrd ? j->qrd[q] : -1, &st);
    const int n = s.n_cand;
    if (j->out_t && j->cand_ptr[q + 1] - j->cand_ptr[q] != n) { j->ok = 0; }
    qsort(s.cand, n, sizeof(int32_t), cmp_int);
    for (int i = 0; i < n; ++i) {
      const int t = s.cand[i];
      if (j->ok && j->out_t) {
        j->out_t[j->cand_ptr[q] + i] = t;
        j->out_score[j->cand_ptr[q] + i] = wsum[t];
      }
      wsum[t] = 0.0;
      s.sum[t] = 0;
      s.fp[t] = 0;
    }
  }
  scratch_free(&s);
  free(wsum);
  return NULL;
}

/* The EM Predictor's integer work per query, over `nthreads` pthreads:
 * per rule position k of the query relation's rules (file order),
 * pos[rq_ptr[q] + k] = paths h -> t along the rule, tot[...] = paths h -> any
 * destination (compute_H's inputs, predictors.py:82-119); and, when out_t is
 * not NULL, the candidates sorted by entity with their score
 * sum_rho count_rho * w[rho] in double (predictors.py:53-80) at cand_ptr[q]
 * (cand_ptr from the candidate counts of oracle_digests).  Returns 0 on
 * success. */
int oracle_query_stats(const int64_t *off, const int32_t *col, int R, int E, const int32_t *rh_ptr,
                       const int32_t *bptr, const int32_t *body, const int32_t *rid, const int32_t *qh,
                       const int32_t *qr, const int32_t *rm_src, const int32_t *rm_dst, const int32_t *qt,
                       int nq, int nthreads, const double *w, const int64_t *rq_ptr, int64_t *pos,
                       int64_t *tot, const int64_t *cand_ptr, int32_t *out_t, double *out_score) {
  graph_t g = {off, col, R, E, rh_ptr, bptr, body, rid};
  if (nthreads < 1) nthreads = 1;
  pthread_t *th = malloc(sizeof(pthread_t) * nthreads);
  stats_job_t *jobs = malloc(sizeof(stats_job_t) * nthreads);
  for (int i = 0; i < nthreads; ++i) {
    jobs[i] = (stats_job_t){&g, qh, qr, rm_src, rm_dst, qt, nq, nthreads, i, w, rq_ptr, cand_ptr, pos, tot,
                            out_t, out_score, 0};
    pthread_create(&th[i], NULL, stats_worker, &jobs[i]);
  }
  int ok = 1;
  for (int i = 0; i < nthreads; ++i) {
    pthread_join(th[i], NULL);
    ok &= jobs[i].ok;
  }
  free(th);
  free(jobs);
  return ok ? 0 : 1;
}

/*
 * anomod_oracle.c — CPU restatement of the AnoMod hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the timed CPU port — never as part of the product path.
 *
 * Written from scratch in plain C, one function per hot-path stage, each
 * citing the reference code (paths relative to /root/reference) it restates:
 *
 *  - parent resolution: the parent of a span is the span of the SAME trace
 *    whose id equals the span's parent reference — jaeger_to_csv.py:34-38
 *    (first CHILD_OF ref, '' when none) and trace_collector.py:424-443
 *    (same segment / refs[0]; a parent that is not in the trace makes the
 *    span a root).  First match in trace order wins.
 *  - edge table / histogram / quantiles: absent in the reference (SURVEY.md
 *    §0.3, §8a a10-a11); nearest-rank index (n*q)//100 follows
 *    monitor_http_responses.py:180-190.
 *  - EWMA/z: absent in the reference (§8a a12); pinned by pandas
 *    Series.ewm(alpha, adjust=False) in tests/golden.
 *  - PageRank: absent in the reference (§8a a13); networkx 3.4.2
 *    _pagerank_scipy convention, pinned by networkx in tests/golden.
 *
 * Parity status: the decode rules are pinned by golden vectors produced by
 * the reference's own code (tests/golden/gen/make_goldens.py); the
 * build-defined stages are pinned against pandas / networkx goldens.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_SUB_BITS 5u
#define OR_BINS 896u

uint32_t oracle_hist_bin(uint32_t v) {
  if (v < 64u) return v;
  uint32_t lg = 31u - (uint32_t)__builtin_clz(v);
  uint32_t e = lg - OR_SUB_BITS;
  return (e << OR_SUB_BITS) + (v >> e);
}

void oracle_hist_bounds(uint32_t bin, uint32_t* lo, uint32_t* hi) {
  if (bin < 64u) {
    *lo = *hi = bin;
    return;
  }
  uint32_t e = (bin >> OR_SUB_BITS) - 1u;
  uint64_t m = (uint64_t)(bin & ((1u << OR_SUB_BITS) - 1u)) + (1u << OR_SUB_BITS);
  *lo = (uint32_t)(m << e);
  *hi = (uint32_t)(((m + 1) << e) - 1);
}

/* Accumulate traces [t0, t1) into the caller's tables (E = (S+2)*S rows:
 * row = p*S + c, p = S for ROOT, S+1 for ORPHAN).  The caller zeroes
 * count/err/sum/hist/mx and sets mn to UINT32_MAX. */
void oracle_edge_aggregate(uint32_t S, const uint64_t* span_id, const uint64_t* parent,
                           const uint16_t* svc, const uint16_t* flags, const uint32_t* dur,
                           const uint64_t* trace_ptr, uint64_t t0, uint64_t t1, uint64_t* count,
                           uint64_t* err, uint64_t* sum, uint32_t* mn, uint32_t* mx,
                           uint64_t* hist) {
  for (uint64_t t = t0; t < t1; ++t) {
    const uint64_t a = trace_ptr[t], b = trace_ptr[t + 1];
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t pid = parent[i];
      uint32_t p = S;
      if (pid != 0) {
        p = S + 1;
        for (uint64_t q = a; q < b; ++q) {
          if (span_id[q] == pid) {
            p = svc[q];
            break;
          }
        }
      }
      const uint64_t e = (uint64_t)p * S + svc[i];
      const uint32_t d = dur[i];
      count[e] += 1;
      if (flags[i] & 1u) err[e] += 1;
      sum[e] += d;
      if (d < mn[e]) mn[e] = d;
      if (d > mx[e]) mx[e] = d;
      hist[e * OR_BINS + oracle_hist_bin(d)] += 1;
    }
  }
}

/* The edge row of every span of traces [t0, t1) (the same first-match
 * parent rule as oracle_edge_aggregate), for exact per-edge order
 * statistics. */
void oracle_span_edges(uint32_t S, const uint64_t* span_id, const uint64_t* parent,
                       const uint16_t* svc, const uint64_t* trace_ptr, uint64_t t0, uint64_t t1,
                       uint32_t* edge) {
  for (uint64_t t = t0; t < t1; ++t) {
    const uint64_t a = trace_ptr[t], b = trace_ptr[t + 1];
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t pid = parent[i];
      uint32_t p = S;
      if (pid != 0) {
        p = S + 1;
        for (uint64_t q = a; q < b; ++q) {
          if (span_id[q] == pid) {
            p = svc[q];
            break;
          }
        }
      }
      edge[i] = p * S + svc[i];
    }
  }
}

/* Nearest-rank quantile from a histogram row: rank r = (n*q_pct)//100
 * (monitor_http_responses.py:187-189), value = midpoint of the bin that
 * holds the r-th (0-based) sample; NaN when the row is empty. */
void oracle_quantiles(const uint64_t* hist, uint64_t E, uint32_t q_pct, double* out) {
  for (uint64_t e = 0; e < E; ++e) {
    const uint64_t* h = hist + e * OR_BINS;
    uint64_t n = 0;
    for (uint32_t b = 0; b < OR_BINS; ++b) n += h[b];
    if (n == 0) {
      out[e] = NAN;
      continue;
    }
    const uint64_t r = n * q_pct / 100u;
    uint64_t c = 0;
    for (uint32_t b = 0; b < OR_BINS; ++b) {
      c += h[b];
      if (r < c) {
        uint32_t lo, hi;
        oracle_hist_bounds(b, &lo, &hi);
        out[e] = 0.5 * ((double)lo + (double)hi);
        break;
      }
    }
  }
}

/* Windowed EWMA/z-score (f64 state and f64 z).  X is [T][S]; Z is [T/W][S]. */
void oracle_ewma_z(const float* X, uint64_t T, uint64_t S, double alpha, uint32_t W, double eps,
                   float* Z) {
  const double beta = 1.0 - alpha;
  for (uint64_t s = 0; s < S; ++s) {
    double m = 0.0, v = 0.0;
    uint64_t n = 0;
    double wmax = 0.0;
    uint32_t wpos = 0;
    uint64_t w = 0;
    for (uint64_t t = 0; t < T; ++t) {
      const float x = X[t * S + s];
      double z = 0.0;
      if (x == x) {
        if (n == 0) {
          m = x;
          v = 0.0;
        } else {
          const double d = (double)x - m;
          z = d / sqrt(v + eps);
          m = m + alpha * d;
          v = beta * (v + alpha * d * d);
        }
        ++n;
      }
      if (fabs(z) > wmax) wmax = fabs(z);
      if (++wpos == W) {
        Z[w * S + s] = (float)wmax;
        ++w;
        wpos = 0;
        wmax = 0.0;
      }
    }
  }
}

/* Personalized PageRank, networkx 3.4.2 _pagerank_scipy convention, push
 * form over the out-edge CSR.  p must already sum to 1.  Returns iterations
 * executed; stops when ||x - xlast||_1 < N*tol (tol > 0) or after iters. */
uint32_t oracle_pagerank(const uint32_t* row_ptr, const uint32_t* col, const float* w, uint32_t N,
                         const double* p, double alpha, uint32_t iters, double tol,
                         double* x_out) {
  double* outw = (double*)calloc(N, sizeof(double));
  double* x = (double*)malloc(N * sizeof(double));
  double* y = (double*)malloc(N * sizeof(double));
  for (uint32_t u = 0; u < N; ++u) {
    for (uint32_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k) outw[u] += (double)w[k];
    x[u] = 1.0 / N;
  }
  uint32_t it = 0;
  for (; it < iters;) {
    double dsum = 0.0;
    for (uint32_t u = 0; u < N; ++u) {
      y[u] = 0.0;
      if (outw[u] == 0.0) dsum += x[u];
    }
    for (uint32_t u = 0; u < N; ++u) {
      if (outw[u] == 0.0) continue;
      for (uint32_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k)
        y[col[k]] += x[u] * ((double)w[k] / outw[u]);
    }
    double err = 0.0;
    for (uint32_t u = 0; u < N; ++u) {
      y[u] = alpha * (y[u] + dsum * p[u]) + (1.0 - alpha) * p[u];
      err += fabs(y[u] - x[u]);
    }
    double* tmp = x;
    x = y;
    y = tmp;
    ++it;
    if (tol > 0.0 && err < (double)N * tol) break;
  }
  memcpy(x_out, x, N * sizeof(double));
  free(outw);
  free(x);
  free(y);
  return it;
}

/* Trace structure of traces [t0, t1): restatement of _build_span_records
 * (trace_collector.py:401-481) on id columns.  Per trace of L spans:
 *   first/last(i) : first / last span of the trace with span i's id
 *   own parent    : first span whose id equals parent[i] (0 = no reference),
 *                   every such span counts as a child of that node (:438-439)
 *   node parent   : own parent of last(i) — parents[node_id] keeps the last
 *                   span's value (:437)
 *   depth         : BFS deepest visit = longest path from a root (:441-449);
 *                   unreached or fed by a reached cycle -> 0 (:477)
 *   roots         : first spans whose node parent is missing (:443)
 * parent_pos is trace-local; 0xFFFFFFFF = no parent.  n_children, svc_mask
 * must be zeroed by the caller. */
static long or_first(const uint64_t* id, uint64_t a, uint64_t b, uint64_t x) {
  if (x == 0) return -1;
  for (uint64_t q = a; q < b; ++q)
    if (id[q] == x) return (long)(q - a);
  return -1;
}

void oracle_trace_structure(const uint64_t* span_id, const uint64_t* parent, const uint16_t* svc,
                            const uint64_t* trace_ptr, uint64_t t0, uint64_t t1, uint32_t words,
                            uint32_t* parent_pos, uint32_t* depth, uint32_t* n_children,
                            uint8_t* flags, uint32_t* n_roots, uint64_t* svc_mask) {
  for (uint64_t t = t0; t < t1; ++t) {
    const uint64_t a = trace_ptr[t], b = trace_ptr[t + 1], L = b - a;
    uint32_t roots = 0;
    long* F = (long*)malloc((L ? L : 1) * sizeof(long));   /* node: first span with the id */
    long* PF = (long*)malloc((L ? L : 1) * sizeof(long));  /* own parent reference resolved */
    long* D = (long*)malloc((L ? L : 1) * sizeof(long));   /* node depth, -1 = not reached */
    for (uint64_t i = a; i < b; ++i) {
      long f = -1, l = -1;
      for (uint64_t q = a; q < b; ++q)
        if (span_id[q] == span_id[i]) {
          if (f < 0) f = (long)(q - a);
          l = (long)(q - a);
        }
      const long pf = or_first(span_id, a, b, parent[i]);
      const long np = (l == (long)(i - a)) ? pf : or_first(span_id, a, b, parent[a + l]);
      if (pf >= 0) n_children[a + pf] += 1;
      parent_pos[i] = np >= 0 ? (uint32_t)np : 0xFFFFFFFFu;
      flags[i] = (uint8_t)((np < 0 ? 1u : 0u) | (f == (long)(i - a) ? 2u : 0u));
      if (np < 0 && f == (long)(i - a)) ++roots;
      svc_mask[t * words + (svc[i] >> 6)] |= 1ull << (svc[i] & 63u);
      F[i - a] = f;
      PF[i - a] = pf;
      D[i - a] = -1;
    }
    /* Depth (trace_collector.py:441-449): the BFS from the roots enqueues a
       node once per child-list entry — one per span whose own parent
       reference resolves (:438-439) — and keeps its LAST visit, the deepest:
       the longest path from a root (a node whose last span's parent does not
       resolve) along those edges.  Relaxed to the fixpoint; a node still
       growing after 2L + 2 rounds sits on or after a cycle the BFS reaches
       (the reference never terminates there) and, like unreachable nodes,
       gets 0.  Without duplicate ids this is the walk up the parent chain. */
    for (uint64_t k = 0; k < L; ++k)
      if (F[k] == (long)k && (flags[a + k] & 1u)) D[k] = 0;
    for (uint64_t round = 0; round < 2 * L + 2; ++round) {
      int changed = 0;
      for (uint64_t k = 0; k < L; ++k) {
        if (PF[k] < 0 || D[PF[k]] < 0) continue;
        if (D[PF[k]] + 1 > D[F[k]]) {
          D[F[k]] = D[PF[k]] + 1;
          changed = 1;
        }
      }
      if (!changed) break;
    }
    for (uint64_t i = a; i < b; ++i) {
      const long f = F[i - a];
      if (f != (long)(i - a)) n_children[i] = n_children[a + f];
      const long d = D[f];
      depth[i] = (d >= 0 && d < (long)L) ? (uint32_t)d : 0u;
    }
    free(F);
    free(PF);
    free(D);
    n_roots[t] = roots;
  }
}

/* ---- grouping of spans that arrive interleaved (north_star (2)) ----------
 * The CPU side of anomod_edge_aggregate_ungrouped / anomod_spans_group: the
 * Elasticsearch path pulls sw_segment-* hits sorted by start_time over all
 * traces (enhanced_trace_collector.py:80-90), so a trace's spans are known
 * only by trace_hash.  Output: order[] such that spans taken in that order are
 * grouped — traces by k = mix64(trace_hash) ascending, the spans of a trace in
 * arrival order (stable) — and trace_ptr over them; the same result as
 * oracle/spec.py group_by_trace (a numpy stable argsort), here as a parallel
 * two-level MSD radix partition (pthreads) so that bench.py can time the
 * ungrouped step on every usable host core.  Level 1 scatters (k, arrival)
 * pairs stably by the top 11 bits of k (per-thread chunk counts, one prefix);
 * level 2 counting-sorts each level-1 bucket by the next 11 bits, then a
 * stable insertion sort by k finishes each (tiny) sub-bucket. */
#include <pthread.h>

typedef struct {
  uint64_t k, i;
} or_pair;

static uint64_t or_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

#define OR_G_BITS 11u
#define OR_G_DIG (1u << OR_G_BITS)

typedef struct {
  const uint64_t* h;
  uint64_t n;
  uint32_t threads;
  or_pair* a; /* pairs in arrival order, then the result */
  or_pair* b; /* level-1 output */
  uint64_t* cnt; /* [threads][OR_G_DIG] chunk counts, then scatter cursors */
  uint64_t* bs;  /* [OR_G_DIG + 1] level-1 bucket starts */
  uint64_t next; /* level-2 bucket ticket */
  uint64_t* chg; /* [threads] trace starts per chunk, then their prefix */
  uint64_t* order;
  uint64_t* tptr;
  int phase;
} or_group;

typedef struct {
  or_group* g;
  uint32_t t;
} or_job;

static void or_chunk(const or_group* g, uint32_t t, uint64_t* lo, uint64_t* hi) {
  *lo = g->n * t / g->threads;
  *hi = g->n * (t + 1) / g->threads;
}

static void* or_group_worker(void* arg) {
  or_job* j = (or_job*)arg;
  or_group* g = j->g;
  const uint32_t t = j->t;
  uint64_t lo, hi;
  or_chunk(g, t, &lo, &hi);
  if (g->phase == 0) { /* keys + chunk counts of the top bits */
    uint64_t* c = g->cnt + (uint64_t)t * OR_G_DIG;
    for (uint64_t i = lo; i < hi; ++i) {
      const uint64_t k = or_mix64(g->h[i]);
      g->a[i].k = k;
      g->a[i].i = i;
      c[k >> (64u - OR_G_BITS)]++;
    }
  } else if (g->phase == 1) { /* stable level-1 scatter */
    uint64_t* c = g->cnt + (uint64_t)t * OR_G_DIG;
    for (uint64_t i = lo; i < hi; ++i) g->b[c[g->a[i].k >> (64u - OR_G_BITS)]++] = g->a[i];
  } else if (g->phase == 2) { /* level 2 per bucket, then insertion sort */
    uint64_t sc[OR_G_DIG];
    for (;;) {
      const uint64_t d = __atomic_fetch_add(&g->next, 1ull, __ATOMIC_RELAXED);
      if (d >= OR_G_DIG) break;
      const uint64_t s = g->bs[d], e = g->bs[d + 1];
      if (e - s <= 1) {
        if (e > s) g->a[s] = g->b[s];
        continue;
      }
      memset(sc, 0, sizeof(sc));
      for (uint64_t i = s; i < e; ++i) sc[(g->b[i].k >> (64u - 2u * OR_G_BITS)) & (OR_G_DIG - 1u)]++;
      uint64_t run = s;
      for (uint32_t x = 0; x < OR_G_DIG; ++x) {
        const uint64_t c = sc[x];
        sc[x] = run;
        run += c;
      }
      for (uint64_t i = s; i < e; ++i)
        g->a[sc[(g->b[i].k >> (64u - 2u * OR_G_BITS)) & (OR_G_DIG - 1u)]++] = g->b[i];
      /* sub-bucket x now ends at sc[x]: stable insertion sort by k */
      uint64_t ss = s;
      for (uint32_t x = 0; x < OR_G_DIG; ++x) {
        const uint64_t se = sc[x];
        for (uint64_t i = ss + 1; i < se; ++i) {
          const or_pair v = g->a[i];
          uint64_t q = i;
          while (q > ss && g->a[q - 1].k > v.k) {
            g->a[q] = g->a[q - 1];
            --q;
          }
          g->a[q] = v;
        }
        ss = se;
      }
    }
  } else if (g->phase == 3) { /* order, trace starts per chunk */
    uint64_t c = 0;
    for (uint64_t i = lo; i < hi; ++i) {
      g->order[i] = g->a[i].i;
      c += (i == 0 || g->a[i].k != g->a[i - 1].k) ? 1u : 0u;
    }
    g->chg[t] = c;
  } else { /* trace_ptr */
    uint64_t w = g->chg[t];
    for (uint64_t i = lo; i < hi; ++i)
      if (i == 0 || g->a[i].k != g->a[i - 1].k) g->tptr[w++] = i;
  }
  return NULL;
}

static int or_run(or_group* g, int phase) {
  pthread_t th[256];
  or_job jobs[256];
  g->phase = phase;
  for (uint32_t t = 0; t < g->threads; ++t) {
    jobs[t].g = g;
    jobs[t].t = t;
    if (pthread_create(&th[t], NULL, or_group_worker, &jobs[t]) != 0) {
      for (uint32_t q = 0; q < t; ++q) pthread_join(th[q], NULL);
      return -1;
    }
  }
  for (uint32_t t = 0; t < g->threads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* order[n], tptr[n + 1] (caller-sized); returns the trace count, or -1. */
int64_t oracle_group_by_trace(const uint64_t* trace_hash, uint64_t n, uint32_t threads,
                              uint64_t* order, uint64_t* tptr) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  if (n == 0) {
    tptr[0] = 0;
    return 0;
  }
  or_group g;
  memset(&g, 0, sizeof(g));
  g.h = trace_hash;
  g.n = n;
  g.threads = threads;
  g.order = order;
  g.tptr = tptr;
  g.a = (or_pair*)malloc(n * sizeof(or_pair));
  g.b = (or_pair*)malloc(n * sizeof(or_pair));
  g.cnt = (uint64_t*)calloc((size_t)threads * OR_G_DIG, sizeof(uint64_t));
  g.bs = (uint64_t*)malloc((OR_G_DIG + 1) * sizeof(uint64_t));
  g.chg = (uint64_t*)malloc((threads + 1) * sizeof(uint64_t));
  int64_t rc = -1;
  if (g.a && g.b && g.cnt && g.bs && g.chg && or_run(&g, 0) == 0) {
    uint64_t run = 0;
    for (uint32_t d = 0; d < OR_G_DIG; ++d) { /* digit-major, thread-minor: stable */
      g.bs[d] = run;
      for (uint32_t t = 0; t < threads; ++t) {
        const uint64_t c = g.cnt[(uint64_t)t * OR_G_DIG + d];
        g.cnt[(uint64_t)t * OR_G_DIG + d] = run;
        run += c;
      }
    }
    g.bs[OR_G_DIG] = run;
    if (or_run(&g, 1) == 0 && or_run(&g, 2) == 0 && or_run(&g, 3) == 0) {
      uint64_t tot = 0;
      for (uint32_t t = 0; t < threads; ++t) {
        const uint64_t c = g.chg[t];
        g.chg[t] = tot;
        tot += c;
      }
      if (or_run(&g, 4) == 0) {
        tptr[tot] = n;
        rc = (int64_t)tot;
      }
    }
  }
  free(g.a);
  free(g.b);
  free(g.cnt);
  free(g.bs);
  free(g.chg);
  return rc;
}

/* The span columns taken in `order` (rows [lo, hi) of the output), for one
 * thread's share of the gather after oracle_group_by_trace. */
void oracle_take_spans(const uint64_t* order, uint64_t lo, uint64_t hi, const uint64_t* h,
                       const uint64_t* sid, const uint64_t* pid, const uint16_t* svc,
                       const uint16_t* flags, const uint32_t* dur, uint64_t* oh, uint64_t* osid,
                       uint64_t* opid, uint16_t* osvc, uint16_t* oflags, uint32_t* odur) {
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t s = order[i];
    oh[i] = h[s];
    osid[i] = sid[s];
    opid[i] = pid[s];
    osvc[i] = svc[s];
    oflags[i] = flags[s];
    odur[i] = dur[s];
  }
}

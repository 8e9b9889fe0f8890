/*
 * gossip_oracle.c -- CPU restatement of the gossip hot path.  TEST INFRASTRUCTURE:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * library, and only as the checker / the timed CPU baseline -- never as the
 * product path (the product is libgossip_hip.so, which has no CPU fallback).
 *
 * Parity status:
 *  - overlay selection: pinned by the reference's own outputs
 *    (tests/golden/powerlaw_join.npz, c1_overlay.json); the Chung-Lu builder below
 *    is the build's own definition (the reference has no large-graph generator,
 *    SURVEY.md §0 finding 2) and is pinned against an independent numpy
 *    restatement (oracle/graph_ref.py).
 *  - propagation: the reference never forwards (SURVEY.md §0 finding 1: Peer.py
 *    sends each message once to direct out-links, Peer.py:402-404, receivers only
 *    log, Peer.py:206,286).  Round 1 of a directed run IS the reference's direct
 *    delivery matrix (tests/golden/c1_wire.json).  Multi-hop forward-once semantics
 *    are the build's spec and are cross-checked against the
 *    per-peer Message-List harness oracle/harness.py (sha256 dedup).
 *
 * Written as straightforward scalar loops (no bitmap tricks beyond the u64 packing
 * that defines the Message-List), OpenMP over vertices: the expansion, the
 * per-message forwards (fused into the expansion pass) and the coverage count
 * all run on every thread, so the full 2^24 x 4096 run (BASELINE config 4)
 * finishes in about a minute on 16 host cores.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- integer mixing ----------------------------------- */
static inline uint64_t or_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static inline uint64_t or_key(uint64_t seed, uint64_t stream) {
  return or_splitmix64(seed ^ or_splitmix64(stream));
}
static inline uint64_t or_draw(uint64_t key, uint64_t idx) {
  return or_splitmix64(key + idx * 0x9E3779B97F4A7C15ULL);
}
static inline uint64_t or_below(uint64_t r, uint64_t n) {
  return (uint64_t)(((unsigned __int128)r * (unsigned __int128)n) >> 64);
}
static inline uint64_t or_fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
static inline uint64_t or_term(uint32_t rr, uint32_t w, uint64_t bits) {
  return or_fmix64(bits ^ or_fmix64(((uint64_t)(rr + 1) << 32) | (uint64_t)w));
}
#define OR_INJ 0x80000000u

uint64_t or_digest_term(uint32_t rr, uint32_t w, uint64_t bits) { return or_term(rr, w, bits); }
uint64_t or_draw_export(uint64_t seed, uint64_t stream, uint64_t idx) {
  return or_draw(or_key(seed, stream), idx);
}

/* ---- Chung-Lu overlay ---------------------------------- */
static int cmp_u64(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}

/* Returns nnz; row_ptr (n+1) and col (nnz) are malloc'ed, free with or_free. */
int64_t or_chung_lu(int64_t n, double dbar, double gamma, uint64_t seed, int64_t** row_ptr_out,
                    int32_t** col_out) {
  const double alpha = 1.0 / (gamma - 1.0);
  uint64_t* q = (uint64_t*)malloc((size_t)n * 8);
  uint64_t T = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t qi = (uint64_t)floor(ldexp(pow((double)(i + 1), -alpha), 32));
    if (qi < 1) qi = 1;
    q[i] = qi;
    T += qi;
  }
  /* integer Vose alias table; small/large stacks filled in index order */
  uint64_t* prob = (uint64_t*)malloc((size_t)n * 8);
  int32_t* alias = (int32_t*)malloc((size_t)n * 4);
  uint64_t* p = (uint64_t*)malloc((size_t)n * 8);
  int32_t* small = (int32_t*)malloc((size_t)n * 4);
  int32_t* large = (int32_t*)malloc((size_t)n * 4);
  int64_t ns = 0, nl = 0;
  for (int64_t i = 0; i < n; ++i) {
    prob[i] = T;
    alias[i] = (int32_t)i;
    p[i] = q[i] * (uint64_t)n;
    if (p[i] < T) small[ns++] = (int32_t)i;
    else large[nl++] = (int32_t)i;
  }
  while (ns > 0 && nl > 0) {
    int32_t s = small[--ns], l = large[--nl];
    prob[s] = p[s];
    alias[s] = l;
    p[l] -= T - p[s];
    if (p[l] < T) small[ns++] = l;
    else large[nl++] = l;
  }
  free(q); free(p); free(small); free(large);

  /* random relabel: rank of (hash32(i) << 32 | i) */
  uint64_t* rk = (uint64_t*)malloc((size_t)n * 8);
  const uint64_t krel = or_key(seed, 2);
  for (int64_t i = 0; i < n; ++i) rk[i] = ((or_draw(krel, (uint64_t)i) >> 32) << 32) | (uint64_t)i;
  qsort(rk, (size_t)n, 8, cmp_u64);
  int32_t* new_id = (int32_t*)malloc((size_t)n * 4);
  for (int64_t k = 0; k < n; ++k) new_id[(uint32_t)rk[k]] = (int32_t)k;
  free(rk);

  const int64_t E = (int64_t)floor(dbar * (double)n / 2.0);
  uint64_t* keys = (uint64_t*)malloc((size_t)(2 * E > 0 ? 2 * E : 1) * 8);
  int64_t K = 0;
  const uint64_t kedge = or_key(seed, 1);
  for (int64_t e = 0; e < E; ++e) {
    uint64_t b = 4ull * (uint64_t)e;
    uint64_t i0 = or_below(or_draw(kedge, b + 0), (uint64_t)n);
    uint64_t x0 = or_below(or_draw(kedge, b + 1), T);
    int32_t u = x0 < prob[i0] ? (int32_t)i0 : alias[i0];
    uint64_t i1 = or_below(or_draw(kedge, b + 2), (uint64_t)n);
    uint64_t x1 = or_below(or_draw(kedge, b + 3), T);
    int32_t v = x1 < prob[i1] ? (int32_t)i1 : alias[i1];
    if (u == v) continue;
    uint64_t a = (uint32_t)new_id[u], c = (uint32_t)new_id[v];
    keys[K++] = (a << 32) | c;
    keys[K++] = (c << 32) | a;
  }
  free(prob); free(alias); free(new_id);
  qsort(keys, (size_t)K, 8, cmp_u64);
  int64_t A = 0;
  for (int64_t k = 0; k < K; ++k)
    if (k == 0 || keys[k] != keys[k - 1]) keys[A++] = keys[k];
  int64_t* rp = (int64_t*)calloc((size_t)n + 1, 8);
  int32_t* col = (int32_t*)malloc((size_t)(A > 0 ? A : 1) * 4);
  for (int64_t k = 0; k < A; ++k) {
    rp[(keys[k] >> 32) + 1]++;
    col[k] = (int32_t)(uint32_t)keys[k];
  }
  for (int64_t v = 0; v < n; ++v) rp[v + 1] += rp[v];
  free(keys);
  *row_ptr_out = rp;
  *col_out = col;
  return A;
}

void or_free(void* p) { free(p); }

/* ---- gossip rounds --------------------------------- */
typedef struct or_round_stats {
  int64_t injected, lost, new_bits, receivers, sends, active, crashed, reports, removals, dup_reports;
} or_round_stats;

enum { ST_CRASHED = 1, ST_REMOVED = 2, ST_DOWN = 3 };

static inline int popc64(uint64_t x) { return __builtin_popcountll(x); }

/*
 * Full run.  In-CSR: In(v) = col[row_ptr[v] .. row_ptr[v+1]) (senders to v).
 * directed: out-CSR (the other end of every heartbeat link); deg_out from it.
 * crash_vert/crash_round: explicit crashes (silent mode) applied in L_round.
 * Outputs may be NULL.  Returns the number of rounds run, or <0 on bad input.
 */
int32_t or_run(int64_t n, const int64_t* row_ptr, const int32_t* col, int32_t directed,
               const int64_t* out_row_ptr, const int32_t* out_col, int32_t m, const int32_t* origin,
               const int32_t* inject_round, int32_t churn, double p_fail, uint64_t churn_seed,
               int32_t miss_thr, int32_t n_crash, const int32_t* crash_vert, const int32_t* crash_round,
               int32_t max_rounds, int32_t nthreads, uint64_t* seen_out, uint8_t* first_out,
               uint64_t* digest_out, uint64_t* coverage_out, uint64_t* forwards_out,
               or_round_stats* stats_out, int32_t* report_out, int64_t report_cap,
               int64_t* n_reports_out) {
  if (n <= 0 || m < 1 || m > 4096 || max_rounds < 1) return -1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  int W = 1;
  while (W * 64 < m) W <<= 1;
  uint64_t* front = (uint64_t*)calloc((size_t)n * W, 8);
  uint64_t* next = (uint64_t*)calloc((size_t)n * W, 8);
  /* seen_out, when given, IS the Message-List array (no second n x W copy:
     32 GiB at 2^26 x 4096) */
  uint64_t* seen = seen_out;
  if (seen) memset(seen, 0, (size_t)n * W * 8);
  else seen = (uint64_t*)calloc((size_t)n * W, 8);
  uint64_t* digest = (uint64_t*)calloc((size_t)n, 8);
  uint8_t* state = (uint8_t*)calloc((size_t)n, 1);
  uint8_t* miss = (uint8_t*)calloc((size_t)n, 1);
  int32_t* deg_live = (int32_t*)malloc((size_t)n * 4);
  int32_t* cand = (int32_t*)malloc((size_t)n * 4);
  uint64_t* fwd = (uint64_t*)calloc((size_t)W * 64, 8);
  /* fz[v]: frontier row of v non-zero (senders with an empty frontier are skipped:
     OR-ing a zero row changes nothing) */
  uint8_t* fz = (uint8_t*)calloc((size_t)n, 1);
  uint8_t* fz_next = (uint8_t*)calloc((size_t)n, 1);
  int nth = 1;
#ifdef _OPENMP
  nth = omp_get_max_threads();
#endif
  /* per-thread per-message accumulators (forwards, coverage), summed after each pass */
  uint64_t* acc_t = (uint64_t*)calloc((size_t)nth * W * 64, 8);
  if (first_out) memset(first_out, 0xFF, (size_t)n * m);
  const int64_t* drp = directed ? out_row_ptr : row_ptr;
  for (int64_t v = 0; v < n; ++v) deg_live[v] = (int32_t)(drp[v + 1] - drp[v]);
  int32_t last_inject = -1;
  for (int32_t k = 0; k < m; ++k)
    if (inject_round[k] > last_inject) last_inject = inject_round[k];
  int liveness = churn || n_crash > 0;
  int64_t nrep = 0;
  int32_t r = 0, rounds = 0;
  const uint64_t p_thresh = (p_fail > 0.0 && p_fail < 1.0) ? (uint64_t)ldexp(p_fail, 64) : 0;
  /* GP_ORACLE_PROGRESS=1: one stderr line per round (long full-size runs) */
  const char* prog_env = getenv("GP_ORACLE_PROGRESS");
  const int progress = prog_env && prog_env[0] == '1';
  for (r = 0; r < max_rounds; ++r) {
    or_round_stats st;
    memset(&st, 0, sizeof(st));
    /* L_r: crash draws, miss counters, 3-miss detection, removal (Peer.py:298-313, Seed.py:358-391) */
    if (liveness) {
      const uint64_t key = or_key(churn_seed, 0x100 + (uint64_t)r);
      int64_t nc = 0;
      for (int64_t v = 0; v < n; ++v) {
        if (!(state[v] & ST_DOWN)) {
          int crash = 0;
          for (int32_t k = 0; k < n_crash; ++k)
            if (crash_vert[k] == v && crash_round[k] == r) crash = 1;
          if (!crash && churn && p_fail >= 1.0) crash = 1;
          if (!crash && churn && p_thresh && or_draw(key, (uint64_t)v) < p_thresh) crash = 1;
          if (crash) {
            state[v] |= ST_CRASHED;
            memset(front + (size_t)v * W, 0, (size_t)W * 8);
            fz[v] = 0;
            st.crashed++;
          }
        }
        if (state[v] & ST_CRASHED) {
          if (miss[v] < 255) miss[v]++;
          if (miss[v] == miss_thr && !(state[v] & ST_REMOVED)) cand[nc++] = (int32_t)v;
        }
      }
      for (int64_t k = 0; k < nc; ++k) {
        const int32_t v = cand[k];
        int64_t live = 0;
        for (int64_t j = row_ptr[v]; j < row_ptr[v + 1]; ++j) live += !(state[col[j]] & ST_DOWN);
        if (directed)
          for (int64_t j = out_row_ptr[v]; j < out_row_ptr[v + 1]; ++j) live += !(state[out_col[j]] & ST_DOWN);
        if (live == 0) continue;
        st.reports += live;
        st.removals += 1;
        st.dup_reports += live - 1;
        for (int pass = 0; pass < 1 + (directed != 0); ++pass) {
          const int64_t* rp = pass ? out_row_ptr : row_ptr;
          const int32_t* cl = pass ? out_col : col;
          for (int64_t j = rp[v]; j < rp[v + 1]; ++j) {
            if (state[cl[j]] & ST_DOWN) continue;
            if (report_out && nrep < report_cap) {
              report_out[3 * nrep + 0] = v;
              report_out[3 * nrep + 1] = cl[j];
              report_out[3 * nrep + 2] = r;
            }
            nrep++;
          }
        }
        state[v] |= ST_REMOVED;
        for (int64_t j = row_ptr[v]; j < row_ptr[v + 1]; ++j) deg_live[col[j]]--;
      }
    }
    /* I_r: injection (Peer.py:397-400) -- one digest term per (origin, word) */
    for (int32_t k = 0; k < m; ++k) {
      if (inject_round[k] != r) continue;
      const int32_t o = origin[k];
      if (state[o] & ST_DOWN) {
        st.lost++;
        continue;
      }
      front[(size_t)o * W + (k >> 6)] |= 1ull << (k & 63);
      fz[o] = 1;
      seen[(size_t)o * W + (k >> 6)] |= 1ull << (k & 63);
      if (first_out) first_out[(size_t)o * m + k] = (uint8_t)r;
      st.injected++;
    }
    for (int32_t k = 0; k < m; ++k) {   /* digest: group this round's injections per (o, word) */
      if (inject_round[k] != r || (state[origin[k]] & ST_DOWN)) continue;
      const int32_t o = origin[k];
      int dup = 0;   /* first message of its (o, word) group in this round? */
      for (int32_t j = 0; j < k; ++j)
        if (inject_round[j] == r && origin[j] == o && (j >> 6) == (k >> 6)) { dup = 1; break; }
      if (dup) continue;
      uint64_t bits = 0;
      for (int32_t j = k; j < m; ++j)
        if (inject_round[j] == r && origin[j] == o && (j >> 6) == (k >> 6)) bits |= 1ull << (j & 63);
      digest[o] ^= or_term((uint32_t)r, (uint32_t)(k >> 6) | OR_INJ, bits);
    }
    /* E_r: pull expansion with forward-once dedup against the Message-List `seen`;
       the same pass adds round r's per-message forwards: every holder of message k
       in its frontier sends it to its live links (thread-local, summed below) */
    int64_t s_new = 0, s_recv = 0, s_sends = 0, s_active = 0;
    const int want_fwd = forwards_out != NULL;
#pragma omp parallel reduction(+ : s_new, s_recv, s_sends, s_active)
    {
      int tid = 0;
#ifdef _OPENMP
      tid = omp_get_thread_num();
#endif
      uint64_t* my_fwd = acc_t + (size_t)tid * W * 64;
#pragma omp for schedule(dynamic, 512)
      for (int64_t v = 0; v < n; ++v) {
        const uint64_t* fv = front + (size_t)v * W;
        const uint64_t dl = (uint64_t)(deg_live[v] > 0 ? deg_live[v] : 0);
        int64_t pc = 0;
        if (fz[v]) {
          for (int w = 0; w < W; ++w) {
            uint64_t x = fv[w];
            pc += popc64(x);
            if (want_fwd)
              while (x) {
                my_fwd[w * 64 + __builtin_ctzll(x)] += dl;
                x &= x - 1;
              }
          }
        }
        if (pc) {
          s_sends += pc * (int64_t)dl;
          s_active++;
        }
        uint64_t* nx = next + (size_t)v * W;
        fz_next[v] = 0;
        if (state[v] & ST_DOWN) {
          memset(nx, 0, (size_t)W * 8);
          continue;
        }
        int64_t newc = 0;
        uint64_t acc[64];
        for (int w = 0; w < W; ++w) acc[w] = 0;
        for (int64_t j = row_ptr[v]; j < row_ptr[v + 1]; ++j) {
          if (!fz[col[j]]) continue;
          const uint64_t* fu = front + (size_t)col[j] * W;
          for (int w = 0; w < W; ++w) acc[w] |= fu[w];
        }
        for (int w = 0; w < W; ++w) {
          uint64_t nw = acc[w] & ~seen[(size_t)v * W + w];
          nx[w] = nw;
          if (!nw) continue;
          seen[(size_t)v * W + w] |= nw;
          newc += popc64(nw);
          digest[v] ^= or_term((uint32_t)(r + 1), (uint32_t)w, nw);
          if (first_out) {
            uint64_t x = nw;
            while (x) {
              int b = __builtin_ctzll(x);
              first_out[(size_t)v * m + w * 64 + b] = (uint8_t)(r + 1);
              x &= x - 1;
            }
          }
        }
        fz_next[v] = newc > 0;
        s_new += newc;
        s_recv += newc > 0;
      }
    }
    if (want_fwd)
      for (int t = 0; t < nth; ++t)
        for (int k = 0; k < W * 64; ++k) {
          fwd[k] += acc_t[(size_t)t * W * 64 + k];
          acc_t[(size_t)t * W * 64 + k] = 0;
        }
    st.new_bits = s_new;
    st.receivers = s_recv;
    st.sends = s_sends;
    st.active = s_active;
    if (stats_out) stats_out[r] = st;
    uint64_t* t = front;
    front = next;
    next = t;
    uint8_t* tz = fz;
    fz = fz_next;
    fz_next = tz;
    rounds = r + 1;
    if (progress) {
      fprintf(stderr, "[oracle] round %d: new_bits %lld receivers %lld crashed %lld removals %lld\n", (int)r,
              (long long)s_new, (long long)s_recv, (long long)st.crashed, (long long)st.removals);
      fflush(stderr);
    }
    if (s_new == 0 && r >= last_inject) break;
  }
  if (digest_out) memcpy(digest_out, digest, (size_t)n * 8);
  if (coverage_out) {   /* holders of each message: thread-local counts over vertex blocks */
#pragma omp parallel
    {
      int tid = 0;
#ifdef _OPENMP
      tid = omp_get_thread_num();
#endif
      uint64_t* my = acc_t + (size_t)tid * W * 64;
#pragma omp for schedule(static)
      for (int64_t v = 0; v < n; ++v)
        for (int w = 0; w < W; ++w) {
          uint64_t x = seen[(size_t)v * W + w];
          while (x) {
            my[w * 64 + __builtin_ctzll(x)]++;
            x &= x - 1;
          }
        }
    }
    for (int32_t k = 0; k < m; ++k) {
      uint64_t c = 0;
      for (int t = 0; t < nth; ++t) c += acc_t[(size_t)t * W * 64 + k];
      coverage_out[k] = c;
    }
  }
  if (forwards_out)
    for (int32_t k = 0; k < m; ++k) forwards_out[k] = fwd[k];
  if (n_reports_out) *n_reports_out = nrep;
  if (seen != seen_out) free(seen);
  free(front); free(next); free(digest); free(state); free(miss);
  free(deg_live); free(cand); free(fwd); free(fz); free(fz_next); free(acc_t);
  return rounds;
}

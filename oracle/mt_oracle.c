/*
 * ORACLE — test infrastructure only (see bcount_oracle.c header for the usage rule).
 *
 * All-cores CPU baseline (SURVEY §8(d) CPU timing plan, item 2): the same restatements as
 * oracle_bcount (count.cpp:7-99) and oracle_stats (main.py:10-79), spread over host threads.
 * The reference itself is single-threaded (count.cpp:22-97 is one loop, no threads); this is the
 * strongest CPU version of the same arithmetic that bench.py's cpu_baseline reports next to it.
 *   bcount: threads take contiguous read ranges into private histograms (integer sums: order-free,
 *           bit-exact), then add them position-parallel; the first out-of-range read is the
 *           smallest over the threads' first ones.
 *   stats:  threads take contiguous position ranges (positions are independent).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_bcount(int64_t ref_len, uint32_t mbq, int64_t n, const int32_t* pos, const uint32_t* cig_beg,
                  const uint32_t* cig_n, const uint32_t* seq_nib, const uint32_t* cigar, const uint8_t* seq,
                  const uint8_t* qual, uint32_t* out, int64_t* bad_read, int64_t* bad_pos);
void oracle_stats_range(const uint32_t* counts6, int64_t p0, int64_t p1, int64_t L, int show_n, double nf,
                        double nf2, int32_t* cov_out, double* pc, double* ent, double* sec);

typedef struct {
    int64_t ref_len, r0, r1, p0, p1;
    uint32_t mbq;
    const int32_t* pos;
    const uint32_t *cig_beg, *cig_n, *seq_nib, *cigar;
    const uint8_t *seq, *qual;
    uint32_t* priv;  /* this thread's [ref_len][6] */
    uint32_t** all;  /* every thread's */
    int nt;
    uint32_t* out;
    int64_t bad_read, bad_pos;
} CountJob;

static void* count_range(void* a) {
    CountJob* j = (CountJob*)a;
    int64_t br = -1, bp = -1;
    if (oracle_bcount(j->ref_len, j->mbq, j->r1 - j->r0, j->pos + j->r0, j->cig_beg + j->r0, j->cig_n + j->r0,
                      j->seq_nib + j->r0, j->cigar, j->seq, j->qual, j->priv, &br, &bp))
        br += j->r0;
    j->bad_read = br;
    j->bad_pos = bp;
    return NULL;
}

static void* reduce_range(void* a) {
    CountJob* j = (CountJob*)a;
    const int64_t e0 = j->p0 * 6, e1 = j->p1 * 6;
    for (int64_t e = e0; e < e1; ++e) {
        uint32_t s = 0;
        for (int t = 0; t < j->nt; ++t) s += j->all[t][e];
        j->out[e] = s;
    }
    return NULL;
}

int oracle_bcount_mt(int64_t ref_len, uint32_t mbq, int64_t n, const int32_t* pos, const uint32_t* cig_beg,
                     const uint32_t* cig_n, const uint32_t* seq_nib, const uint32_t* cigar, const uint8_t* seq,
                     const uint8_t* qual, uint32_t* out, int64_t* bad_read, int64_t* bad_pos, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    CountJob jobs[256];
    pthread_t th[256];
    uint32_t* priv[256];
    const size_t hb = (size_t)(ref_len > 0 ? ref_len : 0) * 6 * sizeof(uint32_t);
    for (int t = 0; t < nthreads; ++t) {
        priv[t] = (uint32_t*)malloc(hb ? hb : 4);
        if (!priv[t]) {
            for (int u = 0; u < t; ++u) free(priv[u]);
            return -1;
        }
    }
    for (int t = 0; t < nthreads; ++t) {
        CountJob* j = &jobs[t];
        memset(j, 0, sizeof *j);
        j->ref_len = ref_len;
        j->mbq = mbq;
        j->r0 = n * t / nthreads;
        j->r1 = n * (t + 1) / nthreads;
        j->pos = pos;
        j->cig_beg = cig_beg;
        j->cig_n = cig_n;
        j->seq_nib = seq_nib;
        j->cigar = cigar;
        j->seq = seq;
        j->qual = qual;
        j->priv = priv[t];
        j->all = priv;
        j->nt = nthreads;
        j->out = out;
        pthread_create(&th[t], NULL, count_range, j);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    *bad_read = -1;
    *bad_pos = -1;
    for (int t = 0; t < nthreads; ++t)  /* ranges are in read order: the first thread with one */
        if (jobs[t].bad_read >= 0) {
            *bad_read = jobs[t].bad_read;
            *bad_pos = jobs[t].bad_pos;
            break;
        }
    if (*bad_read < 0) {
        for (int t = 0; t < nthreads; ++t) {
            jobs[t].p0 = ref_len * t / nthreads;
            jobs[t].p1 = ref_len * (t + 1) / nthreads;
            pthread_create(&th[t], NULL, reduce_range, &jobs[t]);
        }
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    }
    for (int t = 0; t < nthreads; ++t) free(priv[t]);
    return *bad_read >= 0;
}

typedef struct {
    const uint32_t* counts6;
    int64_t p0, p1, L;
    int show_n;
    double nf, nf2;
    int32_t* cov;
    double *pc, *ent, *sec;
} StatsJob;

static void* stats_range(void* a) {
    StatsJob* j = (StatsJob*)a;
    oracle_stats_range(j->counts6, j->p0, j->p1, j->L, j->show_n, j->nf, j->nf2, j->cov, j->pc, j->ent, j->sec);
    return NULL;
}

void oracle_stats_mt(const uint32_t* counts6, int64_t L, int show_n, double nf, double nf2, int32_t* cov_out,
                     double* pc, double* ent, double* sec, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    StatsJob jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        StatsJob j = {counts6, L * t / nthreads, L * (t + 1) / nthreads, L, show_n, nf, nf2, cov_out, pc, ent, sec};
        jobs[t] = j;
        pthread_create(&th[t], NULL, stats_range, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

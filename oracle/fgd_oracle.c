/*
 * fgd_oracle.c -- TEST INFRASTRUCTURE ONLY (see fgd_oracle.h).
 *
 * A plain-C restatement of the reference's per-pod Filter+Score path.  Each
 * function names the Go source it follows (paths relative to the reference
 * tree).  Floating-point expressions keep Go's evaluation order; the file is
 * compiled with -ffp-contract=off so that no a*b+c is fused (Go on amd64,
 * GOAMD64=v1, emits no FMA).
 */
#include "fgd_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* Go math.Exp, portable algorithm (Go src/math/exp.go, FreeBSD e_exp.c). */
/* Parity unpinned: on amd64 the reference binary dispatches to an         */
/* assembly routine; no reference test pins the difference.    */
/* ------------------------------------------------------------------ */
static double go_ldexp_small(double y, int k) {
    /* y in [0.5, 2], |k| < 1000: scale by an exact power of two, in two steps so
     * the intermediate stays normal.  Exact for every result that is normal. */
    int k1 = k / 2, k2 = k - k1;
    union { uint64_t u; double d; } a, b;
    a.u = (uint64_t)(1023 + k1) << 52;
    b.u = (uint64_t)(1023 + k2) << 52;
    return (y * a.d) * b.d;
}

double orc_go_exp(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01;
    const double Ln2Lo = 1.90821492927058770002e-10;
    const double Log2e = 1.44269504088896338700e+00;
    const double Overflow = 7.09782712893383973096e+02;
    const double Underflow = -7.45133219101941108420e+02;
    const double NearZero = 1.0 / (double)(1 << 28);
    const double P1 = 1.66666666666666657415e-01;
    const double P2 = -2.77777777770155933842e-03;
    const double P3 = 6.61375632143793436117e-05;
    const double P4 = -1.65339022054652515390e-06;
    const double P5 = 4.13813679705723846039e-08;
    if (isnan(x) || (isinf(x) && x > 0)) return x;
    if (isinf(x) && x < 0) return 0;
    if (x > Overflow) return INFINITY;
    if (x < Underflow) return 0;
    if (-NearZero < x && x < NearZero) return 1 + x;
    int k = 0;
    if (x < 0) k = (int)(Log2e * x - 0.5);
    else if (x > 0) k = (int)(Log2e * x + 0.5);
    double hi = x - (double)k * Ln2Hi;
    double lo = (double)k * Ln2Lo;
    /* expmulti */
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
    return go_ldexp_small(y, k);
}

/* plugin_utils.go:76-78.  g_exp_nudge != 0 (census runs only) moves exp's result by that many ulps:
 * a stand-in for a different math.Exp (Go's amd64 assembly) within a few ulps of the portable one. */
static int g_exp_nudge = 0;
static double nudge_ulps(double e, int j) {
    for (; j > 0; --j) e = nextafter(e, HUGE_VAL);
    for (; j < 0; ++j) e = nextafter(e, -HUGE_VAL);
    return e;
}
static int g_exp_mode = 0;  /* 0: the portable algorithm; 1: exp in x87 extended precision rounded to double */
static double exp_cr(double x) { return (double)expl((long double)x); }
static double census_exp(double x) {
    const double e = g_exp_mode ? exp_cr(x) : orc_go_exp(x);
    return g_exp_nudge ? nudge_ulps(e, g_exp_nudge) : e;
}
double orc_sigmoid(double x) {
    return 1.0 / (1.0 + ((g_exp_nudge | g_exp_mode) ? census_exp(-x) : orc_go_exp(-x)));
}
void orc_set_exp_nudge(int ulps) { g_exp_nudge = ulps; }
void orc_set_exp_mode(int mode) { g_exp_mode = mode; }

/* ------------------------------------------------------------------ */
/* math.Exp census (tests/golden/make_exp_census.py).     */
/* fgd_score.go:123,144 score = int64(sigmoid((cur-new)/1000)*100) is a */
/* step function of delta = cur - new: score >= k iff delta >= th[k].   */
/* A different exp (Go's amd64 assembly) moves each th[k] by about      */
/* 1000 * 2^-52 per ulp of exp; the census records how close any delta  */
/* the path evaluates comes to any th[k].                               */
/* ------------------------------------------------------------------ */
static int score_of_delta(double delta) { return (int)(int64_t)(orc_sigmoid(delta / 1000) * (double)100); }
static long long ord_key(double d) {
    long long b;
    memcpy(&b, &d, 8);
    return b >= 0 ? b : (long long)(0x8000000000000000ULL - (unsigned long long)b);
}
static double ord_dbl(long long k) {
    long long b = k >= 0 ? k : (long long)(0x8000000000000000ULL - (unsigned long long)k);
    double d;
    memcpy(&d, &b, 8);
    return d;
}
int orc_score_thresholds(double* th) {
    th[0] = -HUGE_VAL;
    th[101] = HUGE_VAL;
    if (score_of_delta(-1.0e9) != 0 || score_of_delta(1.0e9) != 100) return -1;
    for (int k = 1; k <= 100; k++) {
        long long lo = ord_key(-1.0e9), hi = ord_key(1.0e9); /* score(lo) < k <= score(hi) */
        while ((unsigned long long)hi - (unsigned long long)lo > 1ULL) {
            long long mid = (long long)((unsigned long long)lo + ((unsigned long long)hi - (unsigned long long)lo) / 2);
            if (score_of_delta(ord_dbl(mid)) >= k) hi = mid;
            else lo = mid;
        }
        th[k] = ord_dbl(hi);
        if (k > 1 && !(th[k] > th[k - 1])) return -1;
    }
    return 0;
}
static double g_th[102];
#define ORC_CENSUS_NEAR 1.0e-10  /* > 400 x the step shift of one exp ulp (1000 * 2^-52) */
#define ORC_CENSUS_KEEP 16
static long long g_census_near, g_census_sens, g_census_crdiff, g_census_nkept;
static double g_census_sens_max;  /* largest |delta| whose score a one-ulp move of exp changes */
static orc_census_case g_census_cases[ORC_CENSUS_KEEP];       /* portable != correctly rounded */
static orc_census_case g_census_sens_cases[ORC_CENSUS_KEEP];  /* a one-ulp move of exp changes the score */
static int g_census_on = 0;
static pthread_mutex_t g_census_mu = PTHREAD_MUTEX_INITIALIZER;
static double g_census_min;
static double g_census_delta;
static int g_census_step, g_census_node, g_census_k;
static long long g_census_n;
static int g_census_cur_step = -1;
static __thread int tl_census_node = -1;

/* Diagnostics: the raw PWR min / max of every PWR / PWR+FGD cycle scored (step -> {lo, hi}; the step's entry stays
 * {1, 0} when no normalisation ran).  Used to size a speculative NormalizeScore range. */
static int64_t* g_pwr_lohi = NULL;
static int g_pwr_lohi_cap = 0;
void orc_pwr_lohi_trace(int64_t* buf, int cap) {
    g_pwr_lohi = buf;
    g_pwr_lohi_cap = cap;
}

int orc_census_begin(void) {
    if (orc_score_thresholds(g_th)) return -1;
    g_census_min = HUGE_VAL;
    g_census_delta = 0;
    g_census_step = g_census_node = g_census_k = -1;
    g_census_n = 0;
    g_census_near = g_census_sens = g_census_crdiff = g_census_nkept = 0;
    g_census_sens_max = 0;
    memset(g_census_cases, 0, sizeof g_census_cases);
    memset(g_census_sens_cases, 0, sizeof g_census_sens_cases);
    g_census_on = 1;
    return 0;
}
void orc_census_near(long long* near, long long* crdiff, long long* sensitive, double* sens_max,
                     orc_census_case* cr_cases, orc_census_case* sens_cases) {
    *near = g_census_near;
    *crdiff = g_census_crdiff;
    *sensitive = g_census_sens;
    if (sens_max) *sens_max = g_census_sens_max;
    memcpy(cr_cases, g_census_cases, sizeof g_census_cases);
    memcpy(sens_cases, g_census_sens_cases, sizeof g_census_sens_cases);
}
void orc_census_end(double* min_dist, double* delta_at, int* step_at, int* node_at, int* k_at, long long* n,
                    double* th) {
    g_census_on = 0;
    *min_dist = g_census_min;
    *delta_at = g_census_delta;
    *step_at = g_census_step;
    *node_at = g_census_node;
    *k_at = g_census_k;
    *n = g_census_n;
    if (th) memcpy(th, g_th, sizeof g_th);
}
static void census(double delta) {
    if (!g_census_on) return;
    const int s = score_of_delta(delta);
    const double dlo = delta - g_th[s], dhi = g_th[s + 1] - delta;
    const double d = dlo < dhi ? dlo : dhi;
    __atomic_add_fetch(&g_census_n, 1, __ATOMIC_RELAXED);
    if (d < ORC_CENSUS_NEAR) {
        /* near a step: is the score the one a correctly rounded exp gives (ulps = 0 in the record),
         * and does it survive exp's result moving by one ulp either way (ulps = -1 / +1)? */
        __atomic_add_fetch(&g_census_near, 1, __ATOMIC_RELAXED);
        const double x = -(delta / 1000);
        const double e = orc_go_exp(x), ecr = exp_cr(x);
        int j = 0, sj = (int)(int64_t)((1.0 / (1.0 + ecr)) * (double)100);
        if (sj == s) {
            for (j = -1; j <= 1; j += 2) {
                sj = (int)(int64_t)((1.0 / (1.0 + nudge_ulps(e, j))) * (double)100);
                if (sj != s) break;
            }
        }
        if (sj != s) {
            const long long i = __atomic_fetch_add(j == 0 ? &g_census_crdiff : &g_census_sens, 1, __ATOMIC_RELAXED);
            if (j == 0 && i < ORC_CENSUS_KEEP) {
                orc_census_case c = {delta, g_census_cur_step, tl_census_node, s, sj, j};
                g_census_cases[i] = c;
            } else if (j != 0) {
                pthread_mutex_lock(&g_census_mu);
                if (fabs(delta) > g_census_sens_max) g_census_sens_max = fabs(delta);
                pthread_mutex_unlock(&g_census_mu);
                const long long k = __atomic_fetch_add(&g_census_nkept, 1, __ATOMIC_RELAXED);
                if (k < ORC_CENSUS_KEEP) {
                    orc_census_case c = {delta, g_census_cur_step, tl_census_node, s, sj, j};
                    g_census_sens_cases[k] = c;
                }
            }
        }
    }
    double cur;
    __atomic_load(&g_census_min, &cur, __ATOMIC_RELAXED);
    if (d < cur) {
        pthread_mutex_lock(&g_census_mu);
        if (d < g_census_min) {
            __atomic_store(&g_census_min, &d, __ATOMIC_RELAXED);
            g_census_delta = delta;
            g_census_step = g_census_cur_step;
            g_census_node = tl_census_node;
            g_census_k = dlo < dhi ? s : s + 1;
        }
        pthread_mutex_unlock(&g_census_mu);
    }
}

/* ------------------------------------------------------------------ */
/* utils.go:957-1006 IsNodeAccessibleToPodByType                        */
/* ------------------------------------------------------------------ */
int orc_is_node_accessible_to_pod_by_type(const char* node_type, const char* pod_type) {
    if (pod_type[0] == '\0') return 1;
    int cnt = 0, check = 0;
    const char* s = pod_type;
    for (;;) {
        const char* e = strchr(s, '|');
        size_t len = e ? (size_t)(e - s) : strlen(s);
        if (len > 0) {
            cnt++;
            if (strlen(node_type) == len && strncmp(s, node_type, len) == 0) check = 1;
        }
        if (!e) break;
        s = e + 1;
    }
    if (!check && cnt == 0) check = 1;
    return check;
}

/* frag.go:224-229 */
int64_t orc_get_gpu_milli_left_total(const orc_node_resource* n) {
    int64_t t = 0;
    for (int i = 0; i < n->n_gpu_left; i++) t += n->milli_gpu_left[i];
    return t;
}

/* frag.go:205-213 */
int64_t orc_get_gpu_frag_milli(const orc_node_resource* n, const orc_pod_resource* p) {
    int64_t f = 0;
    for (int i = 0; i < n->n_gpu_left; i++)
        if (n->milli_gpu_left[i] < p->milli_gpu) f += n->milli_gpu_left[i];
    return f;
}

/* frag.go:447-458 */
int orc_can_node_host_pod_on_gpu_memory(const orc_node_resource* n, const orc_pod_resource* p) {
    int req = p->gpu_number;
    for (int i = 0; i < n->n_gpu_left; i++) {
        if (n->milli_gpu_left[i] >= p->milli_gpu) {
            req -= 1;
            if (req <= 0) return 1;
        }
    }
    return 0;
}

/* frag.go:460-493 */
int orc_get_node_pod_frag(const orc_node_resource* n, const orc_pod_resource* p) {
    if (p->milli_gpu == 0) return n->milli_cpu_left >= p->milli_cpu ? ORC_XL : ORC_XR;
    if (!orc_is_node_accessible_to_pod_by_type(n->gpu_type, p->gpu_type)) return ORC_NA;
    if (orc_can_node_host_pod_on_gpu_memory(n, p))
        return n->milli_cpu_left >= p->milli_cpu ? ORC_Q3 : ORC_Q4;
    return n->milli_cpu_left >= p->milli_cpu ? ORC_Q2 : ORC_Q1;
}

/* frag.go:148-188 NodeGpuShareFragAmount (bins accumulated in typical-pod order) */
void orc_node_gpu_share_frag_amount(const orc_node_resource* n, const orc_target_pod* tp, int nt,
                                   double out[ORC_NBINS]) {
    for (int k = 0; k < ORC_NBINS; k++) out[k] = 0.0;
    for (int t = 0; t < nt; t++) {
        double freq = tp[t].percentage;
        if (freq < 0 || freq > 1) continue;
        int ft = orc_get_node_pod_frag(n, &tp[t].res);
        int64_t left = orc_get_gpu_milli_left_total(n);
        if (ft == ORC_Q3) {
            int64_t fm = orc_get_gpu_frag_milli(n, &tp[t].res);
            double a = freq * (double)fm;              /* AddByFragType(Q2, ...) */
            if (!(a < 0)) out[ORC_Q2] += a;
            double b = freq * (double)(left - fm);     /* AddByFragType(Q3, ...) */
            if (!(b < 0)) out[ORC_Q3] += b;
        } else {
            double a = freq * (double)left;
            if (!(a < 0)) out[ft] += a;
        }
    }
}

/* frag.go:411-418 */
double orc_frag_amount_sum_except_q3(const double b[ORC_NBINS]) {
    double out = 0;
    for (int i = 0; i < ORC_NBINS; i++)
        if (i != ORC_Q3) out += b[i];
    return out;
}

/* frag.go:420-425 */
double orc_frag_amount_sum_q1q2q4(const double b[ORC_NBINS]) {
    double out = 0;
    out += b[ORC_Q1];
    out += b[ORC_Q2];
    out += b[ORC_Q4];
    return out;
}

/* frag.go:200-203 */
double orc_node_gpu_share_frag_amount_score(const orc_node_resource* n, const orc_target_pod* tp, int nt) {
    double b[ORC_NBINS];
    orc_node_gpu_share_frag_amount(n, tp, nt, b);
    return orc_frag_amount_sum_except_q3(b);
}

/* ------------------------------------------------------------------ */
/* resource.go helpers                                                  */
/* ------------------------------------------------------------------ */

/* resource.go:179-197 SortedMilliGpuLeftIndexList (sort.SliceStable) */
static void sorted_index(const orc_node_resource* n, int ascending, int* idx) {
    for (int i = 0; i < n->n_gpu_left; i++) idx[i] = i;
    /* insertion sort == stable */
    for (int i = 1; i < n->n_gpu_left; i++) {
        int v = idx[i], j = i - 1;
        while (j >= 0) {
            int64_t a = n->milli_gpu_left[idx[j]], b = n->milli_gpu_left[v];
            int before = ascending ? (b < a) : (b > a);
            if (!before) break;
            idx[j + 1] = idx[j];
            j--;
        }
        idx[j + 1] = v;
    }
}

/* resource.go:199-215 Flatten: MilliGpu field */
void orc_flatten_milli_gpu(const orc_node_resource* n, char* out, int cap) {
    int idx[ORC_MAX_GPU_LIST];
    sorted_index(n, 0, idx);
    int pos = 0;
    out[0] = '\0';
    for (int i = 0; i < 8; i++) {
        long long v = i < n->n_gpu_left ? (long long)n->milli_gpu_left[idx[i]] : 0;
        int w = snprintf(out + pos, (size_t)(cap - pos), "%lld,", v);
        if (w < 0 || w >= cap - pos) return;
        pos += w;
    }
}

/* resource.go:454-480 Sub (returns 0 ok, -1 error; out is the partially-updated copy either way) */
int orc_node_sub(const orc_node_resource* n, const orc_pod_resource* p, orc_node_resource* out) {
    *out = *n;
    if (out->milli_cpu_left < p->milli_cpu || out->gpu_number < p->gpu_number) return -1;
    out->milli_cpu_left -= p->milli_cpu;
    int req = p->gpu_number;
    if (req == 0) return 0;
    int idx[ORC_MAX_GPU_LIST];
    sorted_index(out, 1, idx);
    for (int i = 0; i < out->n_gpu_left; i++) {
        if (p->milli_gpu <= out->milli_gpu_left[idx[i]]) {
            req -= 1;
            out->milli_gpu_left[idx[i]] -= p->milli_gpu;
            if (req <= 0) return 0;
        }
    }
    return -1;
}

/* resource.go:482-534 Add (valid idl branch; the reference's condition is
 * `len(idl) > 0 || len(idl) != gpuRequest`) */
int orc_node_add(const orc_node_resource* n, const orc_pod_resource* p, const int* idl, int nidl,
                 orc_node_resource* out) {
    *out = *n;
    out->milli_cpu_left += p->milli_cpu;
    if (out->milli_cpu_left > out->milli_cpu_capacity) {
        out->milli_cpu_left -= p->milli_cpu;
        return -1;
    }
    int req = p->gpu_number;
    if (p->gpu_number == 0) return 0;
    if (nidl > 0 || nidl != req) {
        for (int i = 0; i < nidl; i++) {
            if (idl[i] > out->n_gpu_left - 1 || idl[i] < 0) return -1;
            if (out->milli_gpu_left[idl[i]] + p->milli_gpu > ORC_MILLI) return -1;
            out->milli_gpu_left[idl[i]] += p->milli_gpu;
            req -= 1;
        }
        return 0;
    }
    int idx[ORC_MAX_GPU_LIST];
    sorted_index(out, 1, idx);
    for (int i = 0; i < out->n_gpu_left; i++) {
        if (p->milli_gpu + out->milli_gpu_left[idx[i]] <= ORC_MILLI) {
            req -= 1;
            out->milli_gpu_left[idx[i]] += p->milli_gpu;
            if (req <= 0) return 0;
        }
    }
    return -1;
}

/* resource.go:383-403 AllocateExclusiveGpuId -> GPU bitmask (-1: would panic) */
int orc_allocate_exclusive_gpu_id(const orc_node_resource* n, const orc_pod_resource* p) {
    int64_t req = p->milli_gpu * (int64_t)p->gpu_number;
    int mask = 0;
    for (int i = 0; i < n->n_gpu_left; i++) {
        if (req <= 0) break;
        if (n->milli_gpu_left[i] == ORC_MILLI) {
            mask |= 1 << i;
            req -= ORC_MILLI;
        }
    }
    if (req > 0) return -1;
    return mask;
}

/* ------------------------------------------------------------------ */
/* score plugins                                                        */
/* ------------------------------------------------------------------ */

/* fgd_score.go:99-149 calculateGpuShareFragExtendScore */
int64_t orc_fgd_score(const orc_node_resource* n, const orc_pod_resource* p, const orc_target_pod* tp, int nt,
                      int* gpu_mask) {
    double cur = orc_node_gpu_share_frag_amount_score(n, tp, nt);
    if (p->gpu_number == 1 && p->milli_gpu < ORC_MILLI) {
        int64_t score = 0;
        int gid = -1;
        for (int i = 0; i < n->n_gpu_left; i++) {
            if (n->milli_gpu_left[i] >= p->milli_gpu) {
                orc_node_resource c = *n;
                c.milli_cpu_left -= p->milli_cpu;
                c.milli_gpu_left[i] -= p->milli_gpu;
                double nw = orc_node_gpu_share_frag_amount_score(&c, tp, nt);
                census(cur - nw);
                int64_t fs = (int64_t)(orc_sigmoid((cur - nw) / 1000) * (double)100);
                if (gid == -1 || fs > score) {
                    score = fs;
                    gid = i;
                }
            }
        }
        if (gpu_mask) *gpu_mask = gid < 0 ? 0 : (1 << gid);
        return score;
    }
    orc_node_resource c;
    (void)orc_node_sub(n, p, &c); /* error ignored, as in the reference */
    double nw = orc_node_gpu_share_frag_amount_score(&c, tp, nt);
    census(cur - nw);
    int64_t fs = (int64_t)(orc_sigmoid((cur - nw) / 1000) * (double)100);
    if (gpu_mask) {
        /* AllocateExclusiveGpuId; for CPU-only pods it returns "" (req = 0) */
        int m = orc_allocate_exclusive_gpu_id(n, p);
        *gpu_mask = m < 0 ? 0 : m;
    }
    return fs;
}

/* best_fit_score.go:66-97 getBestFitScore */
int64_t orc_best_fit_score(const orc_node_resource* n, const orc_pod_resource* p) {
    double freeVec[2] = {(double)n->milli_cpu_left, (double)orc_get_gpu_milli_left_total(n)};
    double reqVec[2] = {(double)p->milli_cpu, (double)(p->milli_gpu * (int64_t)p->gpu_number)};
    double maxSpec[2] = {(double)ORC_MAX_SPEC_CPU, (double)ORC_MAX_SPEC_GPU};
    double w[2] = {0.5, 0.5};
    double score = 0;
    for (int i = 0; i < 2; i++) {
        if (freeVec[i] < reqVec[i]) return -1;
        score += (freeVec[i] - reqVec[i]) / maxSpec[i] * w[i];
    }
    score = (1.0 - score) * (double)100;
    return (int64_t)score;
}

/* Go math.Tanh, portable algorithm (src/math/tanh.go) */
double orc_go_tanh(double x) {
    static const double P[3] = {-9.64399179425052238628e-1, -9.92877231001918586564e1, -1.61468768441708447952e3};
    static const double Q[3] = {1.12811678491632931402e2, 2.23548839060100448583e3, 4.84406305325125486048e3};
    const double MAXLOG = 8.8029691931113054295988e+01; /* log(2**127) */
    double z = fabs(x);
    if (z > 0.5 * MAXLOG) return x < 0 ? -1 : 1;
    if (z >= 0.625) {
        double e = orc_go_exp(2 * z);
        z = 1 - 2 / (e + 1);
        if (x < 0) z = -z;
        return z;
    }
    if (x == 0) return x;
    double s = x * x;
    return x + x * s * ((P[0] * s + P[1]) * s + P[2]) / (((s + Q[0]) * s + Q[1]) * s + Q[2]);
}

/* A virtual node / pod resource of GenerateSchedulingMatchGroups: a vector and a GPU id (bitmask;
 * 0 = "", -1 = "" from a panicking AllocateExclusiveGpuId, which the callers never reach). */
typedef struct { double v[ORC_MAX_GPU_LIST + 1]; int len; int gid; } orc_vres;

/* resource.go:217-244 ToFormalizedGpuResourceList: partly used GPUs in index order, then all idle ones */
static int formalized_gpus(const orc_node_resource* n, int64_t* left, int* ids) {
    int k = 0, idle = 0, idle_ids = 0;
    for (int id = 0; id < n->n_gpu_left; id++) {
        int64_t l = n->milli_gpu_left[id];
        if (l == ORC_MILLI) { idle++; idle_ids |= 1 << id; }
        else if (l > 0) { left[k] = l; ids[k] = 1 << id; k++; }
    }
    if (idle > 0) { left[k] = (int64_t)idle * ORC_MILLI; ids[k] = idle_ids; k++; }
    return k;
}

static int fully_free(const orc_node_resource* n) {
    int c = 0;
    for (int id = 0; id < n->n_gpu_left; id++) c += n->milli_gpu_left[id] == ORC_MILLI;
    return c;
}

/* resource.go:296-381 ToVirtualNodeResourceList */
static int virtual_nodes(const orc_node_resource* n, const orc_pod_resource* p, int dim, orc_vres* out) {
    if (n->milli_cpu_left < p->milli_cpu) return 0;
    int64_t req = p->milli_gpu * (int64_t)p->gpu_number;
    int64_t tot = orc_get_gpu_milli_left_total(n);
    int c = 0;
    if (dim == ORC_DIM_MERGE) {
        out[0].v[0] = (double)n->milli_cpu_left;
        out[0].v[1] = (double)tot;
        out[0].len = 2;
        out[0].gid = 0;
        return 1;
    }
    if (dim == ORC_DIM_SHARE || dim == ORC_DIM_DIVIDE) {
        if (req < ORC_MILLI) {
            for (int id = 0; id < n->n_gpu_left; id++) {
                int64_t l = n->milli_gpu_left[id];
                if (l >= ORC_MILLI) continue;
                if (l < req) continue;
                out[c].v[0] = dim == ORC_DIM_SHARE ? (double)n->milli_cpu_left
                                                   : (double)(n->milli_cpu_left * l) / (double)tot;
                out[c].v[1] = (double)l;
                out[c].len = 2;
                out[c].gid = 1 << id;
                c++;
            }
        }
        int idle = fully_free(n);
        if (req <= (int64_t)idle * ORC_MILLI) {
            out[c].gid = orc_allocate_exclusive_gpu_id(n, p);
            out[c].v[0] = dim == ORC_DIM_SHARE ? (double)n->milli_cpu_left
                                               : (double)(n->milli_cpu_left * (int64_t)(idle * ORC_MILLI)) / (double)tot;
            out[c].v[1] = (double)(idle * ORC_MILLI);
            out[c].len = 2;
            c++;
        }
        return c;
    }
    /* extend */
    int64_t left[ORC_MAX_GPU_LIST + 1];
    int ids[ORC_MAX_GPU_LIST + 1];
    int k = formalized_gpus(n, left, ids);
    out[0].v[0] = (double)n->milli_cpu_left;
    for (int i = 0; i < k; i++) out[0].v[1 + i] = (double)left[i];
    out[0].len = 1 + k;
    out[0].gid = 0;
    return 1;
}

/* resource.go:246-294 ToVirtualPodResourceList */
static int virtual_pods(const orc_pod_resource* p, int dim, const orc_node_resource* n, orc_vres* out) {
    int64_t req = p->milli_gpu * (int64_t)p->gpu_number;
    if (dim != ORC_DIM_EXTEND) {
        out[0].v[0] = (double)p->milli_cpu;
        out[0].v[1] = (double)req;
        out[0].len = 2;
        out[0].gid = 0;
        return 1;
    }
    int64_t left[ORC_MAX_GPU_LIST + 1];
    int ids[ORC_MAX_GPU_LIST + 1];
    int k = formalized_gpus(n, left, ids), c = 0;
    for (int i = 0; i < k; i++) {
        if (left[i] < req) continue;
        out[c].v[0] = (double)p->milli_cpu;
        for (int j = 0; j < k; j++) out[c].v[1 + j] = j == i ? (double)req : 0;
        out[c].len = 1 + k;
        out[c].gid = left[i] < ORC_MILLI ? ids[i] : orc_allocate_exclusive_gpu_id(n, p);
        c++;
    }
    return c;
}

/* utils.go:1220-1236 NormalizeVector (in place) */
void orc_normalize_vector(double* v, int len, const double* nv, int nlen) {
    if (nlen == 0 || len == 0 || nlen != len) return;
    for (int i = 0; i < len; i++) v[i] = nv[i] > 0 ? v[i] / nv[i] : 0;
}

/* utils.go:1238-1248 CalculateVectorDotProduct */
double orc_vector_dot_product(const double* a, int la, const double* b, int lb) {
    if (la == 0 || lb == 0 || la != lb) return -1;
    double ip = 0;
    for (int i = 0; i < la; i++) ip += a[i] * b[i];
    return ip;
}

/* dot_product_score.go:64-100 calculateDotProductScore over GenerateSchedulingMatchGroups
 * (utils.go:1274-1342); *gid: the best group's GpuId (bitmask, 0 = "") */
int64_t orc_dot_product_score_cfg(const orc_node_resource* n, const orc_pod_resource* p, int dim, int norm,
                                  int* gid) {
    orc_vres vn[ORC_MAX_GPU_LIST + 2], vp[ORC_MAX_GPU_LIST + 2];
    int nn = virtual_nodes(n, p, dim, vn);
    int np = virtual_pods(p, dim, n, vp);
    double score = -1;
    *gid = 0;
    for (int a = 0; a < nn; a++) {
        for (int b = 0; b < np; b++) {
            double nv[ORC_MAX_GPU_LIST + 1], pv[ORC_MAX_GPU_LIST + 1];
            memcpy(nv, vn[a].v, sizeof nv);
            memcpy(pv, vp[b].v, sizeof pv);
            int ln = vn[a].len, lp = vp[b].len;
            int g = 0;
            if (dim == ORC_DIM_SHARE || dim == ORC_DIM_DIVIDE) g = vn[a].gid;
            else if (dim == ORC_DIM_EXTEND) g = vp[b].gid;
            double cv[ORC_MAX_GPU_LIST + 1];
            int lc = dim == ORC_DIM_EXTEND ? ln : 2;
            double c0, cg;
            if (norm == ORC_NORM_NODE) { c0 = (double)n->milli_cpu_capacity; cg = (double)(n->gpu_number * ORC_MILLI); }
            else if (norm == ORC_NORM_POD) { c0 = (double)p->milli_cpu; cg = (double)(p->milli_gpu * (int64_t)p->gpu_number); }
            else { c0 = (double)ORC_MAX_SPEC_CPU; cg = (double)ORC_MAX_SPEC_GPU; }
            cv[0] = c0;
            for (int i = 1; i < lc; i++) cv[i] = cg;
            orc_normalize_vector(nv, ln, cv, lc);
            orc_normalize_vector(pv, lp, cv, lc);
            double cur = orc_vector_dot_product(nv, ln, pv, lp);
            if (cur == -1) continue;
            cur /= (double)lp;
            if (norm == ORC_NORM_POD) cur = orc_go_tanh(cur / 10);
            cur = 1 - cur;
            if (score < cur) { score = cur; *gid = g; }
        }
    }
    if (score == -1) { *gid = 0; return 0; }
    return (int64_t)((double)100 * score);
}

int64_t orc_dot_product_score(const orc_node_resource* n, const orc_pod_resource* p) {
    int g = 0;
    return orc_dot_product_score_cfg(n, p, ORC_DIM_MERGE, ORC_NORM_MAX, &g);
}

/* gpu_packing_score.go:71-117 getPackingScore */
int64_t orc_packing_score(const orc_node_resource* n, const orc_pod_resource* p, int* err) {
    *err = 0;
    int ff = 0;
    for (int i = 0; i < n->n_gpu_left; i++)
        if (n->milli_gpu_left[i] == ORC_MILLI) ff++;
    if (ff == n->gpu_number) {
        int64_t s = 100 / 3 - (int64_t)ff;
        return s > (int64_t)ff ? s : (int64_t)ff;
    }
    int idx[ORC_MAX_GPU_LIST];
    sorted_index(n, 1, idx);
    int req = p->gpu_number, ffuse = 0, nuse = 0, use[ORC_MAX_GPU_LIST];
    for (int k = 0; k < n->n_gpu_left; k++) {
        if (req == 0) break;
        int64_t left = n->milli_gpu_left[idx[k]];
        if (p->milli_gpu <= left) {
            req--;
            use[nuse++] = idx[k];
            if (left == ORC_MILLI) ffuse++;
        }
    }
    if (req != 0) { *err = 1; return 0; }
    if (ffuse > 0) {
        int64_t s = 100 / 2 - (int64_t)ffuse;
        return s > 100 / 3 ? s : 100 / 3;
    }
    int64_t r = 0;
    for (int k = 0; k < nuse; k++) r += n->milli_gpu_left[use[k]] * 100 / ORC_MILLI;
    int64_t s = 100 - r / 10;
    return s > 100 / 2 ? s : 100 / 2;
}

/* gpu_clustering_score.go:32-56.  pod_tag: -1 = no-gpu, 0 = share-gpu, k = "k-gpu".
 * node_tag_counts[0..8]: pods per tag currently on the node (utils.go:1056-1063). */
int64_t orc_clustering_score(const orc_node_resource* n, const orc_pod_resource* p, int pod_tag,
                             const int32_t* node_tag_counts) {
    (void)p;
    if (pod_tag < 0) return 0;
    int distinct = 0;
    for (int k = 0; k < 9; k++)
        if (node_tag_counts[k] > 0) distinct++;
    int64_t left = orc_get_gpu_milli_left_total(n);
    int64_t base = (int64_t)(100 / 4) * ((int64_t)ORC_MAX_SPEC_GPU - left) / (int64_t)ORC_MAX_SPEC_GPU;
    if (node_tag_counts[pod_tag] > 0) {
        if (distinct == 1) return base + 100 * 3 / 4;
        return base + 100 * 2 / 4;
    }
    if (distinct == 0) return base + 100 / 4;
    return base;
}

/* plugin_utils.go:48-74 NormalizeScore */
void orc_normalize_score(int64_t* s, int n) {
    int64_t hi = -INT64_MAX, lo = INT64_MAX;
    for (int i = 0; i < n; i++) {
        if (s[i] > hi) hi = s[i];
        if (s[i] < lo) lo = s[i];
    }
    int64_t oldRange = hi - lo, newRange = 100 - 0;
    for (int i = 0; i < n; i++) s[i] = oldRange == 0 ? 0 : ((s[i] - lo) * newRange / oldRange) + 0;
}

/* ---- PWR (pwr_score.go; energy model resource.go:536-563, const.go:41-124) ---- */

/* const.go:48-55 MapCpuTypeEnergyConsumption: idle / full watts and cores per CPU */
static const struct { const char* name; double idle, full, ncores; } CPU_ENERGY[] = {
    {"", 15, 120, 16},
    {"Intel-Xeon-8269CY", 20, 205, 26},
    {"Intel-Xeon-8163", 20, 165, 24},
    {"Intel-Xeon-ES-2682-V4", 15, 120, 16},
    {"Intel-Xeon-6326", 20, 185, 16},
    {"Intel-Xeon-8369B", 20, 270, 32},
};
/* const.go:62-69 MapGpuTypeEnergyConsumption through const.go:115-124 MapGpuTypeModelEnergy
 * (G2 uses the A10 profile, G3 the A100 profile) */
static const struct { const char* name; double idle, full; } GPU_ENERGY[] = {
    {"T4", 10, 70}, {"A10", 30, 150}, {"P100", 25, 250}, {"V100M16", 30, 300},
    {"V100M32", 30, 300}, {"A100", 50, 400}, {"G2", 30, 150}, {"G3", 50, 400},
};

/* resource.go:536-563 GetEnergyConsumptionNode */
int orc_energy_node(const orc_node_resource* n, double* cpu_power, double* gpu_power) {
    *cpu_power = 0;
    *gpu_power = 0;
    if (n->gpu_type[0] != '\0') {
        int k = -1;
        for (int i = 0; i < (int)(sizeof GPU_ENERGY / sizeof GPU_ENERGY[0]); i++)
            if (strcmp(GPU_ENERGY[i].name, n->gpu_type) == 0) k = i;
        if (k < 0) return -1;
        int free_gpus = 0; /* GetFullyFreeGpuNum, resource.go:170-177 */
        for (int g = 0; g < n->n_gpu_left; g++)
            if (n->milli_gpu_left[g] == ORC_MILLI) free_gpus++;
        double num_idle = (double)free_gpus;
        double num_working = (double)n->gpu_number - num_idle;
        *gpu_power = (GPU_ENERGY[k].idle * num_idle) + (GPU_ENERGY[k].full * num_working);
    }
    int c = -1;
    for (int i = 0; i < (int)(sizeof CPU_ENERGY / sizeof CPU_ENERGY[0]); i++)
        if (strcmp(CPU_ENERGY[i].name, n->cpu_type) == 0) c = i;
    if (c < 0) return -2;
    double real_cores = ceil((double)n->milli_cpu_capacity / ORC_MILLI / 2);
    double idle_cores = floor((double)n->milli_cpu_left / ORC_MILLI / 2);
    double working_cores = real_cores - idle_cores;
    double ncores = CPU_ENERGY[c].ncores;
    double num_cpus = ceil(real_cores / ncores);
    double num_active = ceil(working_cores / ncores);
    double num_idle_cpus = num_cpus - num_active;
    *cpu_power = (CPU_ENERGY[c].idle * num_idle_cpus) + (CPU_ENERGY[c].full * num_active);
    return 0;
}

/* pwr_score.go:143-212 calculatePWRShareExtendScore */
int64_t orc_pwr_score(const orc_node_resource* n, const orc_pod_resource* p, int* gpu_mask, int* err) {
    double oc, og, nc, ng;
    *gpu_mask = 0;
    *err = 0;
    if (orc_energy_node(n, &oc, &og)) { *err = 1; return 0; }
    double old_energy = oc + og;
    if (p->gpu_number == 1 && p->milli_gpu < ORC_MILLI) {
        int64_t score = INT64_MIN;
        int gid = -1;
        for (int i = 0; i < n->n_gpu_left; i++) {
            if (n->milli_gpu_left[i] >= p->milli_gpu) {
                orc_node_resource c = *n;
                c.milli_cpu_left -= p->milli_cpu;
                c.milli_gpu_left[i] -= p->milli_gpu;
                (void)orc_energy_node(&c, &nc, &ng);
                int64_t s = (int64_t)(old_energy - (nc + ng));
                if (gid == -1 || s > score) { /* first fitting GPU, then strictly better */
                    score = s;
                    gid = i;
                }
            }
        }
        *gpu_mask = gid < 0 ? 0 : (1 << gid);
        return score;
    }
    orc_node_resource c;
    (void)orc_node_sub(n, p, &c); /* error ignored, as in the reference */
    (void)orc_energy_node(&c, &nc, &ng);
    int64_t s = (int64_t)(old_energy - (nc + ng));
    int m = orc_allocate_exclusive_gpu_id(n, p);
    *gpu_mask = m < 0 ? 0 : m;
    return s;
}

/* pwr_score.go:104-141 NormalizeScore: all equal -> 100, else (s - min) * 100 / (max - min) */
void orc_normalize_score_pwr(int64_t* s, int n) {
    if (n <= 0) return;
    int64_t lo = s[0], hi = s[0];
    for (int i = 0; i < n; i++) {
        if (s[i] < lo) lo = s[i];
        if (s[i] > hi) hi = s[i];
    }
    for (int i = 0; i < n; i++) s[i] = lo == hi ? 100 : (s[i] - lo) * 100 / (hi - lo);
}

/* open_gpu_share.go:285-303 allocateGpuIdBasedOnBestFit */
int orc_alloc_gpu_best_fit(const orc_node_resource* n, const orc_pod_resource* p) {
    if (p->milli_gpu < ORC_MILLI) {
        int cand = -1;
        for (int i = 0; i < n->n_gpu_left; i++) {
            if (n->milli_gpu_left[i] >= p->milli_gpu) {
                if (cand == -1 || n->milli_gpu_left[i] < n->milli_gpu_left[cand]) cand = i;
            }
        }
        return cand < 0 ? -1 : (1 << cand);
    }
    return orc_allocate_exclusive_gpu_id(n, p);
}

/* open_gpu_share.go:305-323 allocateGpuIdBasedOnWorstFit */
static int alloc_gpu_worst_fit(const orc_node_resource* n, const orc_pod_resource* p) {
    if (p->milli_gpu < ORC_MILLI) {
        int cand = -1;
        for (int i = 0; i < n->n_gpu_left; i++) {
            if (n->milli_gpu_left[i] >= p->milli_gpu) {
                if (cand == -1 || n->milli_gpu_left[i] > n->milli_gpu_left[cand]) cand = i;
            }
        }
        return cand < 0 ? -1 : (1 << cand);
    }
    return orc_allocate_exclusive_gpu_id(n, p);
}

/* ------------------------------------------------------------------ */
/* typical pods: frag.go:285-380, SortTargetPodInDecreasingCount :436-445, */
/* TargetPodList.Less resource.go:24-42                                  */
/* ------------------------------------------------------------------ */
static int pod_res_less(const orc_pod_resource* a, const orc_pod_resource* b) {
    if (a->milli_cpu != b->milli_cpu) return a->milli_cpu < b->milli_cpu;
    if (a->milli_gpu != b->milli_gpu) return a->milli_gpu < b->milli_gpu;
    if (a->gpu_number != b->gpu_number) return a->gpu_number < b->gpu_number;
    return strcmp(a->gpu_type, b->gpu_type) < 0;
}
static int pod_res_eq(const orc_pod_resource* a, const orc_pod_resource* b) {
    return a->milli_cpu == b->milli_cpu && a->milli_gpu == b->milli_gpu && a->gpu_number == b->gpu_number &&
           strcmp(a->gpu_type, b->gpu_type) == 0;
}
static int target_less(const orc_target_pod* a, const orc_target_pod* b) {
    if (a->percentage != b->percentage) return a->percentage < b->percentage;
    return pod_res_less(&a->res, &b->res);
}
static int cmp_reverse(const void* x, const void* y) {
    const orc_target_pod* a = (const orc_target_pod*)x;
    const orc_target_pod* b = (const orc_target_pod*)y;
    /* sort.Reverse: a before b iff b.Less(a) */
    if (target_less(b, a)) return -1;
    if (target_less(a, b)) return 1;
    return 0;
}

int orc_get_typical_pods(const orc_workload_pod* pods, int n, orc_typical_cfg cfg, orc_target_pod* out, int cap) {
    orc_target_pod* m = (orc_target_pod*)calloc((size_t)(n > 0 ? n : 1), sizeof(orc_target_pod));
    int nm = 0;
    double total = 0;
    for (int i = 0; i < n; i++) {
        orc_pod_resource r;
        memset(&r, 0, sizeof r);
        r.milli_cpu = pods[i].has_cpu ? pods[i].cpu_milli : 100; /* GetNonzeroRequests */
        r.milli_gpu = pods[i].gpu_milli;
        r.gpu_number = pods[i].gpu_number;
        strncpy(r.gpu_type, pods[i].gpu_type, ORC_TYPE_LEN - 1);
        if (!cfg.is_involved_cpu_pods && r.gpu_number == 0) continue;
        double w = 1;
        if (cfg.gpu_res_weight > 0 && r.milli_gpu == ORC_MILLI) w = 1 + (double)r.gpu_number * cfg.gpu_res_weight;
        int j;
        for (j = 0; j < nm; j++)
            if (pod_res_eq(&m[j].res, &r)) break;
        if (j < nm) m[j].percentage = m[j].percentage + w;
        else { m[nm].res = r; m[nm].percentage = w; nm++; }
        total += w;
    }
    qsort(m, (size_t)nm, sizeof(orc_target_pod), cmp_reverse);
    double expected = (double)(cfg.pod_popularity_threshold > 0 ? cfg.pod_popularity_threshold : 60) * total / 100.0;
    int step = cfg.pod_increase_step > 0 ? cfg.pod_increase_step : 10;
    int i = 0, podResNum = 0;
    double cum = 0;
    while (cum < expected) {
        podResNum += step;
        while (i < podResNum && i < nm) {
            double num = m[i].percentage;
            cum += num;
            m[i].percentage = m[i].percentage / total;
            i += 1;
        }
        if (i >= nm && cum < expected) break; /* guard: the Go loop would spin forever */
    }
    int nout = i;
    if (i < nm) {
        for (int j = 0; j < i; j++) m[j].percentage /= cum / total;
    } else {
        nout = nm;
    }
    if (nout > cap) nout = -1;
    else memcpy(out, m, (size_t)nout * sizeof(orc_target_pod));
    free(m);
    return nout;
}

/* ------------------------------------------------------------------ */
/* replay driver                                                        */
/* ------------------------------------------------------------------ */
uint64_t orc_mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}
/* Random contract: node key and GPU key */
static uint64_t rand_node_key(uint64_t seed, int step, uint32_t rank) {
    return orc_mix64(orc_mix64(seed ^ 0xA0761D6478BD642FULL) ^ (((uint64_t)(uint32_t)step << 32) | rank));
}
static uint64_t rand_gpu_key(uint64_t node_key, int g) { return orc_mix64(node_key ^ (uint64_t)(0x100 + g)); }

/* Go math/rand (Go stdlib src/math/rand, outside the reference tree; go.mod:4 go 1.15): the global
 * source the Random draw structure consumes.  rng.go rngSource: Seed expands the seed with the
 * Park-Miller step seedrand and XORs rngCooked; Uint64 is the additive lagged Fibonacci generator
 * (length 607, tap 273).  rand.go: Int63 = Uint64 masked to 63 bits, Int31 = Int63 >> 32, Int31n
 * by rejection above the largest multiple of n (a power of two masks Int31, n = 1 included: it
 * still draws), Intn(n <= 2^31-1) = Int31n.  The rngCooked data table is the one
 * tools/gen_go_rng_cooked.c recomputes (tests/test_go_rand.py pins it against Go's published
 * rand.Seed(1) outputs, for this restatement too). */
static const int64_t orc_rng_cooked[ORC_GO_LEN] = {
#include "../kubernetes-scheduler-simulator_amd/csrc/go_rng_cooked.inc"
};
static int32_t go_seedrand(int32_t x) { /* rng.go seedrand: x * 48271 mod (2^31 - 1), Schrage */
    const int32_t a = 48271, q = 44488, r = 3399;
    int32_t hi = x / q, lo = x % q;
    x = a * lo - r * hi;
    if (x < 0) x += 2147483647;
    return x;
}
void orc_go_seed(orc_go_rng* g, int64_t seed) {
    g->tap = 0;
    g->feed = ORC_GO_LEN - ORC_GO_TAP;
    seed %= 2147483647;
    if (seed < 0) seed += 2147483647;
    if (seed == 0) seed = 89482311;
    int32_t x = (int32_t)seed;
    for (int i = -20; i < ORC_GO_LEN; i++) {
        x = go_seedrand(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << 40;
            x = go_seedrand(x);
            u ^= (uint64_t)(int64_t)x << 20;
            x = go_seedrand(x);
            u ^= (uint64_t)(int64_t)x;
            u ^= (uint64_t)orc_rng_cooked[i];
            g->vec[i] = u;
        }
    }
}
uint64_t orc_go_uint64(orc_go_rng* g) {
    if (--g->tap < 0) g->tap += ORC_GO_LEN;
    if (--g->feed < 0) g->feed += ORC_GO_LEN;
    g->vec[g->feed] += g->vec[g->tap];
    return g->vec[g->feed];
}
static int32_t go_int31(orc_go_rng* g) { return (int32_t)((orc_go_uint64(g) & 0x7fffffffffffffffULL) >> 32); }
int32_t orc_go_int31n(orc_go_rng* g, int32_t n) {
    if (n <= 0) return -1; /* Go panics */
    if ((n & (n - 1)) == 0) return go_int31(g) & (n - 1);
    const int32_t max = (int32_t)((1u << 31) - 1 - (1u << 31) % (uint32_t)n);
    int32_t v = go_int31(g);
    while (v > max) v = go_int31(g);
    return v % n;
}

typedef struct {
    int64_t cpu_req, mem_req;  /* nodeInfo.Requested */
    int32_t pods;
    int64_t gpu_used[8];
    int32_t tag_counts[9];
} node_dyn;

static int pod_tag_of(const orc_event* e) {
    /* open-gpu-share/utils/pod.go:111-123 GetGpuAffinityFromPodAnnotation */
    if (e->gpu_number == 0) return -1;
    if (e->gpu_number == 1 && e->gpu_milli < ORC_MILLI) return 0;
    if (e->gpu_number >= 1 && e->gpu_milli == ORC_MILLI) return e->gpu_number <= 8 ? e->gpu_number : -2;
    return -2; /* the reference panics */
}

/* GetNodeResourceViaNodeInfo (utils.go:1053-1075) */
static void node_res_of(const orc_node_spec* s, const node_dyn* d, orc_node_resource* r) {
    memset(r, 0, sizeof *r);
    r->milli_cpu_left = s->cpu_alloc - d->cpu_req;
    r->milli_cpu_capacity = s->cpu_alloc;
    r->gpu_number = s->gpu_count;
    strncpy(r->gpu_type, s->gpu_type, ORC_TYPE_LEN - 1);
    strncpy(r->cpu_type, s->cpu_type, ORC_TYPE_LEN - 1);
    r->n_gpu_left = s->gpu_count > 0 ? s->gpu_count : 0; /* getGpuMilliLeftListOnNode: nil for non-GPU */
    for (int g = 0; g < r->n_gpu_left && g < 8; g++) r->milli_gpu_left[g] = ORC_MILLI - d->gpu_used[g];
}

static orc_pod_resource pod_res_of(const orc_event* e) {
    orc_pod_resource p;
    memset(&p, 0, sizeof p);
    p.milli_cpu = e->cpu_nz;
    p.milli_gpu = e->gpu_milli;
    p.gpu_number = e->gpu_number;
    strncpy(p.gpu_type, e->gpu_type, ORC_TYPE_LEN - 1);
    return p;
}

/* Filter: fit.go:230-290 fitsRequest ∧ open_gpu_share.go:81-118 Filter ∧ gpunodeinfo.go:136-204 */
static int filter_node(const orc_node_spec* s, const node_dyn* d, const orc_event* e) {
    if (d->pods + 1 > s->pods_alloc) return 0;
    if (!(e->cpu_req == 0 && e->mem_req == 0)) {
        if (s->cpu_alloc < e->cpu_req + d->cpu_req) return 0;
        if (s->mem_alloc < e->mem_req + d->mem_req) return 0;
    }
    if (e->gpu_milli <= 0) return 1;
    if (s->gpu_count == 0) return 0;
    if (!orc_is_node_accessible_to_pod_by_type(s->gpu_type, e->gpu_type)) return 0;
    /* AllocateGpuId */
    if (e->gpu_milli <= 0 || e->gpu_number <= 0) return 0;
    int64_t idle[8];
    int ndev = s->gpu_count < 8 ? s->gpu_count : 8;
    for (int g = 0; g < ndev; g++) idle[g] = ORC_MILLI - d->gpu_used[g];
    if (ndev <= 0) return 0;
    if (e->gpu_number == 1) {
        for (int g = 0; g < ndev; g++)
            if (idle[g] >= e->gpu_milli) return 1;
        return 0;
    }
    int dev = 0, got = 0;
    while (dev < ndev && got < e->gpu_number) {
        if (idle[dev] >= e->gpu_milli) { idle[dev] -= e->gpu_milli; got++; }
        else dev++;
    }
    return got == e->gpu_number;
}

typedef struct {
    const orc_node_spec* nodes;
    const node_dyn* dyn;
    const orc_target_pod* tp;
    int nt;
    orc_policy pol;
    const orc_event* e;
    int step;
    const uint32_t* rank;
    int lo, hi;
    uint8_t* feasible;
    int64_t* raw;
    int32_t* gmask;
    int32_t* err;
    int64_t* raw2;   /* ORC_POL_PWR_FGD: the FGD score (raw holds the PWR score) */
} work_t;

static int64_t score_one(const work_t* w, int i, int32_t* gm, int32_t* err) {
    orc_node_resource nr;
    node_res_of(&w->nodes[i], &w->dyn[i], &nr);
    orc_pod_resource pr = pod_res_of(w->e);
    int accessible = orc_is_node_accessible_to_pod_by_type(nr.gpu_type, pr.gpu_type);
    *gm = 0;
    switch (w->pol.policy) {
    case ORC_POL_FGD: {
        /* fgd_score.go:60-63 (a pod with no resource requests scores 100) never
         * applies to trace pods: pod_csv_to_yaml.py always sets cpu and memory.
         * fgd_score.go:74-77: inaccessible -> error */
        if (!accessible) { *err = 1; return 0; }
        int m = 0;
        tl_census_node = i;
        int64_t s = orc_fgd_score(&nr, &pr, w->tp, w->nt, &m);
        *gm = m;
        return s;
    }
    case ORC_POL_BESTFIT: {
        if (!accessible) { *err = 1; return 0; }
        int64_t s = orc_best_fit_score(&nr, &pr);
        if (s == -1) { *err = 1; return 0; }
        return s;
    }
    case ORC_POL_DOTPROD: {
        int g = 0;
        int64_t sc = orc_dot_product_score_cfg(&nr, &pr, w->pol.dim_ext, w->pol.norm, &g);
        *gm = g;
        return sc;
    }
    case ORC_POL_PACKING: {
        if (w->e->gpu_milli <= 0) return 0;
        if (!accessible) { *err = 1; return 0; }
        int er = 0;
        int64_t s = orc_packing_score(&nr, &pr, &er);
        if (er) { *err = 1; return 0; }
        return s;
    }
    case ORC_POL_CLUSTERING: {
        if (!accessible) { *err = 1; return 0; }
        int tag = pod_tag_of(w->e);
        if (tag == -2) { *err = 1; return 0; }
        return orc_clustering_score(&nr, &pr, tag, w->dyn[i].tag_counts);
    }
    case ORC_POL_PWR:
    case ORC_POL_PWR_FGD: {
        /* pwr_score.go:87-89: inaccessible -> error */
        if (!accessible) { *err = 1; return 0; }
        int m = 0, er = 0;
        int64_t s = orc_pwr_score(&nr, &pr, &m, &er);
        if (er) { *err = 1; return 0; }
        *gm = m;
        if (w->pol.policy == ORC_POL_PWR_FGD) w->raw2[i] = orc_fgd_score(&nr, &pr, w->tp, w->nt, NULL);
        return s;
    }
    default:
        return 0; /* Random: handled by the pre-score pick */
    }
}

static void* work_fn(void* arg) {
    work_t* w = (work_t*)arg;
    for (int i = w->lo; i < w->hi; i++) {
        w->feasible[i] = (uint8_t)filter_node(&w->nodes[i], &w->dyn[i], w->e);
        if (!w->feasible[i]) continue;
        int32_t er = 0;
        w->raw[i] = score_one(w, i, &w->gmask[i], &er);
        if (er) w->err[i] = 1;
    }
    return NULL;
}

/* Exact accumulation for the cluster report: x * 2^80 as a 128-bit integer (x >= 0, finite),
 * via frexp/ldexp.  The reference sums the per-node bins in Go map order, which is not
 * reproducible (client-go/testing/fixture.go:201); the exact sum rounded once is order free and
 * within a few ulps of any ordered sum of these non-negative terms. */
static __int128 orc_fix80(double x) {
    if (x == 0.0) return 0;
    int ex = 0;
    double m = frexp(x, &ex);                 /* x = m * 2^ex, 0.5 <= |m| < 1 */
    int64_t mant = (int64_t)ldexp(m, 53);     /* exact: 53 significant bits */
    int sh = ex - 53 + 80;
    if (sh >= 0) return (__int128)mant << sh;
    if (sh <= -64) return 0;
    return (__int128)(mant >> (-sh));
}

static const orc_node_spec* g_sort_nodes;
static int cmp_name_idx(const void* a, const void* b) {
    int i = *(const int*)a, j = *(const int*)b;
    return strcmp(g_sort_nodes[i].name, g_sort_nodes[j].name);
}

int orc_run_events_state(const orc_node_spec* nodes, int n_nodes, const orc_target_pod* tp, int nt,
                         orc_policy pol, const orc_event* ev, int n_ev, orc_result* res, orc_report* rep,
                         orc_node_state* final_state) {
    /* A deletion names an earlier creation, at most once (the reference deletes a pod once). */
    {
        uint8_t* gone = (uint8_t*)calloc((size_t)(n_ev > 0 ? n_ev : 1), 1);
        int bad = 0;
        for (int s = 0; s < n_ev && !bad; s++) {
            if (!ev[s].is_delete) continue;
            const int ref = ev[s].ref;
            bad = ref < 0 || ref >= s || ev[ref].is_delete || gone[ref];
            if (!bad) gone[ref] = 1;
        }
        free(gone);
        if (bad) return -1;
    }
    node_dyn* dyn = (node_dyn*)calloc((size_t)n_nodes, sizeof(node_dyn));
    uint8_t* feas = (uint8_t*)calloc((size_t)n_nodes, 1);
    int64_t* raw = (int64_t*)calloc((size_t)n_nodes, sizeof(int64_t));
    int32_t* gm = (int32_t*)calloc((size_t)n_nodes, sizeof(int32_t));
    int32_t* err = (int32_t*)calloc((size_t)n_nodes, sizeof(int32_t));
    int* fidx = (int*)calloc((size_t)n_nodes, sizeof(int));
    int64_t* fs = (int64_t*)calloc((size_t)n_nodes, sizeof(int64_t));
    int64_t* raw2 = (int64_t*)calloc((size_t)n_nodes, sizeof(int64_t));
    int64_t* fs2 = (int64_t*)calloc((size_t)n_nodes, sizeof(int64_t));
    uint32_t* rank = (uint32_t*)calloc((size_t)n_nodes, sizeof(uint32_t));
    int* order = (int*)calloc((size_t)n_nodes, sizeof(int));
    for (int i = 0; i < n_nodes; i++) order[i] = i;
    g_sort_nodes = nodes;
    qsort(order, (size_t)n_nodes, sizeof(int), cmp_name_idx);
    for (int r = 0; r < n_nodes; r++) rank[order[r]] = (uint32_t)r;

    int64_t arrived_gpu = 0, arrived_cpu = 0;
    int threads = pol.threads > 1 ? pol.threads : 1;
    /* the Random draw structure: a private copy of the Go stream (orc_policy.go_stream) */
    orc_go_rng* go = NULL;
    if (pol.go_stream) {
        go = (orc_go_rng*)malloc(sizeof *go);
        *go = *pol.go_stream;
    }
    for (int s = 0; s < n_ev; s++) {
        const orc_event* e = &ev[s];
        orc_result* R = &res[s];
        memset(R, 0, sizeof *R);
        R->node = -1;
        g_census_cur_step = s;
        if (e->is_delete) {
            /* simulator.go:416-422 deletePod -> informer DeleteFunc -> removePod */
            int ref = e->ref;
            R->status = 3; /* deleted */
            if (ref >= 0 && ref < s && res[ref].node >= 0) {
                const orc_event* c = &ev[ref];
                node_dyn* d = &dyn[res[ref].node];
                d->cpu_req -= c->cpu_req;
                d->mem_req -= c->mem_req;
                d->pods -= 1;
                for (int g = 0; g < 8; g++)
                    if (res[ref].gpu_mask & (1 << g)) d->gpu_used[g] -= c->gpu_milli;
                int tag = pod_tag_of(c);
                if (tag >= 0) d->tag_counts[tag] -= 1;
                R->node = res[ref].node;
                R->gpu_mask = res[ref].gpu_mask;
            }
        } else {
            orc_pod_resource pr = pod_res_of(e);
            if (go) (void)orc_go_int31n(go, 100); /* scheduler.go:464 SetRecordPluginMetrics(rand.Intn(100) < ..) */
            arrived_gpu += pr.milli_gpu * pr.gpu_number;  /* simulator.go:401-402 */
            arrived_cpu += pr.milli_cpu;
            memset(err, 0, (size_t)n_nodes * sizeof(int32_t));
            work_t w[64];
            pthread_t th[64];
            if (threads > 64) threads = 64;
            int chunk = (n_nodes + threads - 1) / threads;
            for (int t = 0; t < threads; t++) {
                w[t] = (work_t){nodes, dyn, tp, nt, pol, e, s, rank, t * chunk,
                                (t + 1) * chunk < n_nodes ? (t + 1) * chunk : n_nodes, feas, raw, gm, err, raw2};
                if (w[t].lo > w[t].hi) w[t].lo = w[t].hi;
                if (threads > 1) pthread_create(&th[t], NULL, work_fn, &w[t]);
                else work_fn(&w[t]);
            }
            if (threads > 1)
                for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
            int nf = 0;
            for (int i = 0; i < n_nodes; i++)
                if (feas[i]) fidx[nf++] = i;
            R->n_feasible = nf;
            int winner = -1;
            int64_t wscore = 0;
            if (nf == 0) {
                R->status = 1;
                /* scheduler.go:474-480 PostFilter -> DefaultPreemption.FindCandidates: every node is
                 * Unschedulable (not ...AndUnresolvable), so the offset draw is over all of them
                 * (default_preemption.go:197-212,183) */
                if (go && n_nodes > 0) (void)orc_go_int31n(go, n_nodes);
            } else if (nf == 1) {
                winner = fidx[0]; /* generic_scheduler.go:158-164 */
            } else {
                int anyerr = 0;
                for (int k = 0; k < nf; k++) {
                    fs[k] = raw[fidx[k]];
                    fs2[k] = raw2[fidx[k]];
                    if (err[fidx[k]]) anyerr = 1;
                }
                /* random_score.go:42-51: RandomScorePlugin.PreScore is enabled for every policy
                 * (utils.go:241-248) and runs after Filter when two or more nodes are feasible */
                const int go_pick = go ? (int)orc_go_int31n(go, nf) : -1;
                if (pol.policy == ORC_POL_RANDOM && go) {
                    /* random_score.go:53-68: MaxNodeScore for the PreScore pick, MinNodeScore else; the
                     * feasible list in node order (one filter worker: parallelize.Until's order) */
                    for (int k = 0; k < nf; k++) fs[k] = k == go_pick ? 100 : 0;
                } else if (pol.policy == ORC_POL_RANDOM) {
                    /* random_score.go:42-68: PreScore picks one feasible node (Random contract) */
                    int pick = -1;
                    uint64_t best = 0;
                    for (int k = 0; k < nf; k++) {
                        /* 24-bit key (the device packs it into the score field), ties -> smaller rank */
                        uint64_t key = rand_node_key(pol.seed, s, rank[fidx[k]]) >> 40;
                        if (pick < 0 || key > best || (key == best && rank[fidx[k]] < rank[fidx[pick]])) {
                            best = key;
                            pick = k;
                        }
                    }
                    for (int k = 0; k < nf; k++) fs[k] = k == pick ? 100 : 0;
                }
                if (anyerr) {
                    R->status = 2; /* framework.go:656-667: a Score error aborts the cycle */
                } else {
                    if (pol.policy == ORC_POL_BESTFIT) orc_normalize_score(fs, nf);
                    if (pol.policy == ORC_POL_PWR || pol.policy == ORC_POL_PWR_FGD) {
                        if (g_pwr_lohi && s < g_pwr_lohi_cap) {
                            int64_t lo = fs[0], hi = fs[0];
                            for (int k = 1; k < nf; k++) { lo = fs[k] < lo ? fs[k] : lo; hi = fs[k] > hi ? fs[k] : hi; }
                            g_pwr_lohi[2 * s] = lo;
                            g_pwr_lohi[2 * s + 1] = hi;
                        }
                        orc_normalize_score_pwr(fs, nf);
                    }
                    /* framework.go:686-704: range check, then x plugin weight; prioritizeNodes sums the
                     * plugins (generic_scheduler.go:511-519) */
                    const int64_t w1 = pol.policy == ORC_POL_PWR_FGD ? pol.w_pwr : 1000;
                    for (int k = 0; k < nf; k++) {
                        if (fs[k] > 100 || fs[k] < 0) anyerr = 1;
                        fs[k] *= w1;
                        if (pol.policy == ORC_POL_PWR_FGD) {
                            if (fs2[k] > 100 || fs2[k] < 0) anyerr = 1;
                            fs[k] += fs2[k] * pol.w_fgd;
                        }
                    }
                    if (anyerr) R->status = 2;
                    else {
                        /* selectHost, generic_scheduler.go:187-212 */
                        winner = fidx[0];
                        wscore = fs[0];
                        for (int k = 1; k < nf; k++) {
                            if (fs[k] > wscore) { wscore = fs[k]; winner = fidx[k]; }
                            else if (fs[k] == wscore && strcmp(nodes[fidx[k]].name, nodes[winner].name) < 0)
                                winner = fidx[k];
                        }
                    }
                }
            }
            if (winner >= 0) {
                /* Reserve: open_gpu_share.go:178-205, allocateGpuId :252-283 */
                int mask = 0;
                if (e->gpu_milli > 0) {
                    orc_node_resource nr;
                    node_res_of(&nodes[winner], &dyn[winner], &nr);
                    switch (pol.gpu_sel) {
                    case ORC_SEL_FGD: {
                        int m = 0;
                        (void)orc_fgd_score(&nr, &pr, tp, nt, &m);
                        mask = m == 0 ? -1 : m;
                        break;
                    }
                    case ORC_SEL_PWR: { /* pwr_score.go:214-219 allocateGpuIdBasedOnPWRScore */
                        int m = 0, er = 0;
                        (void)orc_pwr_score(&nr, &pr, &m, &er);
                        mask = (m == 0 || er) ? -1 : m;
                        break;
                    }
                    case ORC_SEL_WORST: mask = alloc_gpu_worst_fit(&nr, &pr); break;
                    case ORC_SEL_DOTPROD: { /* dot_product_score.go:102-107 allocateGpuIdBasedOnDotProduct */
                        if (pr.milli_gpu < ORC_MILLI && pr.gpu_number > 1) { mask = -1; break; } /* :266-268 panic */
                        int g = 0;
                        (void)orc_dot_product_score_cfg(&nr, &pr, pol.dim_ext, pol.norm, &g);
                        mask = g <= 0 ? -1 : g;
                        break;
                    }
                    case ORC_SEL_RANDOM:
                        if (go && pr.milli_gpu < ORC_MILLI) {
                            /* open_gpu_share.go:274-276 panic first; :325-343 reservoir draw per fitting GPU */
                            int pick = -1, cnt = 0;
                            if (pr.gpu_number > 1) { mask = -1; break; }
                            for (int g = 0; g < nr.n_gpu_left; g++)
                                if (nr.milli_gpu_left[g] >= pr.milli_gpu && orc_go_int31n(go, ++cnt) == 0) pick = g;
                            mask = pick < 0 ? -1 : (1 << pick);
                        } else if (pr.milli_gpu < ORC_MILLI) {
                            uint64_t nk = rand_node_key(pol.seed, s, rank[winner]);
                            int pick = -1;
                            uint64_t best = 0;
                            for (int g = 0; g < nr.n_gpu_left; g++) {
                                if (nr.milli_gpu_left[g] >= pr.milli_gpu) {
                                    uint64_t k = rand_gpu_key(nk, g);
                                    if (pick < 0 || k > best) { best = k; pick = g; }
                                }
                            }
                            mask = pick < 0 ? -1 : (1 << pick);
                        } else {
                            mask = orc_allocate_exclusive_gpu_id(&nr, &pr);
                        }
                        break;
                    default: mask = orc_alloc_gpu_best_fit(&nr, &pr); break;
                    }
                    if (mask <= 0) { R->status = 2; winner = -1; }
                }
                if (winner >= 0) {
                    node_dyn* d = &dyn[winner];
                    d->cpu_req += e->cpu_req;
                    d->mem_req += e->mem_req;
                    d->pods += 1;
                    for (int g = 0; g < 8; g++)
                        if (mask & (1 << g)) d->gpu_used[g] += e->gpu_milli;
                    int tag = pod_tag_of(e);
                    if (tag >= 0) d->tag_counts[tag] += 1;
                    R->node = winner;
                    R->gpu_mask = mask;
                    R->score = wscore;
                }
            }
        }
        if (rep) {
            /* analysis.go:59-119 ClusterGpuFragReport (node order: input order) */
            orc_report* P = &rep[s];
            memset(P, 0, sizeof *P);
            __int128 ex[ORC_NBINS] = {0};
            for (int i = 0; i < n_nodes; i++) {
                orc_node_resource nr;
                node_res_of(&nodes[i], &dyn[i], &nr);
                double b[ORC_NBINS];
                orc_node_gpu_share_frag_amount(&nr, tp, nt, b);
                for (int k = 0; k < ORC_NBINS; k++) {
                    P->frag_bins[k] += 1.0 * b[k];
                    ex[k] += orc_fix80(b[k]);
                }
                double pc = 0, pg = 0;
                if (orc_energy_node(&nr, &pc, &pg) == 0) {
                    P->power_cpu += pc;  /* analysis.go:48-49 */
                    P->power_gpu += pg;
                } else {
                    P->power_invalid += 1;
                }
                P->total_gpus += nr.gpu_number;
                int ff = 0;
                for (int g = 0; g < nr.n_gpu_left; g++)
                    if (nr.milli_gpu_left[g] == ORC_MILLI) ff++;
                if (ff < nr.gpu_number || nr.milli_cpu_left < nr.milli_cpu_capacity) {
                    P->used_nodes += 1;
                    P->used_gpus += nr.gpu_number;
                    P->used_gpu_milli += (int64_t)nr.gpu_number * ORC_MILLI - orc_get_gpu_milli_left_total(&nr);
                    P->used_cpu_milli += nr.milli_cpu_capacity - nr.milli_cpu_left;
                }
            }
            for (int k = 0; k < ORC_NBINS; k++) P->frag_bins_exact[k] = ldexp((double)ex[k], -80);
            P->arrived_gpu_milli = arrived_gpu;
            P->arrived_cpu_milli = arrived_cpu;
        }
    }
    if (final_state) {
        for (int i = 0; i < n_nodes; i++) {
            final_state[i].cpu_left = nodes[i].cpu_alloc - dyn[i].cpu_req;
            final_state[i].mem_left = nodes[i].mem_alloc - dyn[i].mem_req;
            final_state[i].pods = dyn[i].pods;
            for (int g = 0; g < 8; g++)
                final_state[i].gpu_left[g] = g < nodes[i].gpu_count ? (int32_t)(ORC_MILLI - dyn[i].gpu_used[g]) : 0;
        }
    }
    free(dyn); free(feas); free(raw); free(gm); free(err); free(fidx); free(fs); free(rank); free(order); free(raw2); free(fs2);
    free(go);
    return 0;
}

int orc_run_events(const orc_node_spec* nodes, int n_nodes, const orc_target_pod* tp, int nt, orc_policy pol,
                   const orc_event* ev, int n_ev, orc_result* res, orc_report* rep) {
    return orc_run_events_state(nodes, n_nodes, tp, nt, pol, ev, n_ev, res, rep, NULL);
}

/*
 * fgd_oracle.h -- CPU restatement of the reference's per-pod Filter+Score path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the
 * `cpu_baseline` leg of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may load it.  The product (libksim_hip.so) never
 * links, loads or calls anything in oracle/.
 *
 * It restates, function by function, the Go code of
 * Fr4nz83/kubernetes-scheduler-simulator @ 2024_08_07 (paths relative to that
 * tree; every function in fgd_oracle.c cites the file:line it follows):
 *   pkg/utils/frag.go                       (FGD fragmentation math)
 *   pkg/simulator/plugin/{fgd,...}_score.go         (FGD, BestFit, DotProduct, GpuPacking,
 *                                             GpuClustering, Random, PWR)
 *   pkg/type/open-gpu-share/utils/const.go   (PWR energy model constants)
 *   pkg/simulator/plugin/open_gpu_share.go   (Filter, Reserve, GPU selectors)
 *   pkg/type/resource.go                     (NodeResource/PodResource helpers)
 *   pkg/type/open-gpu-share/cache/gpunodeinfo.go (AllocateGpuId fit test)
 *   vendor/.../noderesources/fit.go          (fitsRequest)
 *   vendor/.../core/generic_scheduler.go     (single-feasible shortcut, selectHost)
 *
 * Types are kept as strings (GPU models, node names) exactly as the reference
 * keeps them, so the product's integer encodings (type bitmasks, name ranks)
 * are checked rather than shared.
 *
 * Parity pins: the Go unit-test known answers (pkg/utils/frag_test.go,
 * pkg/simulator/plugin/gpu_packing_score_test.go, pkg/type/resource_test.go)
 * are checked in tests/test_oracle_golden.py.  Go's math.Exp (used by the FGD
 * sigmoid) and math/rand are outside the reference tree and no reference test
 * pins them: "parity unpinned" for those two.
 */
#ifndef FGD_ORACLE_H
#define FGD_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MILLI 1000              /* open-gpu-share/utils/const.go:14 */
#define ORC_MAX_SPEC_CPU 128000     /* const.go:16 */
#define ORC_MAX_SPEC_GPU 8000       /* const.go:18 */
#define ORC_MAX_GPU_LIST 16         /* NodeResource.MilliGpuLeftList capacity (tests use 9) */
#define ORC_TYPE_LEN 64

/* frag.go:17-35 FragRatioDataMap indices */
enum { ORC_Q1 = 0, ORC_Q2 = 1, ORC_Q3 = 2, ORC_Q4 = 3, ORC_XL = 4, ORC_XR = 5, ORC_NA = 6, ORC_NBINS = 7 };

/* resource.go:51-58 PodResource (CpuType is always "" in the traces; kept out) */
typedef struct {
    int64_t milli_cpu;                 /* non-zero default applied (utils.go:1008-1029) */
    int64_t milli_gpu;                 /* per GPU, 0..1000 */
    int32_t gpu_number;
    char    gpu_type[ORC_TYPE_LEN];    /* pipe-separated model list; "" = any */
} orc_pod_resource;

/* resource.go:61-72 NodeResource */
typedef struct {
    int64_t milli_cpu_left;
    int64_t milli_cpu_capacity;
    int64_t milli_gpu_left[ORC_MAX_GPU_LIST];
    int32_t n_gpu_left;                /* len(MilliGpuLeftList) */
    int32_t gpu_number;
    char    gpu_type[ORC_TYPE_LEN];
    char    cpu_type[ORC_TYPE_LEN];    /* CpuType (alibabacloud.com/cpu-model label; "" when absent) */
} orc_node_resource;

/* resource.go:14-17 TargetPod */
typedef struct {
    orc_pod_resource res;
    double percentage;
} orc_target_pod;

/* ---- leaf math (frag.go) ---- */
int     orc_get_node_pod_frag(const orc_node_resource* n, const orc_pod_resource* p);
int     orc_can_node_host_pod_on_gpu_memory(const orc_node_resource* n, const orc_pod_resource* p);
int     orc_is_node_accessible_to_pod_by_type(const char* node_type, const char* pod_type);
int64_t orc_get_gpu_milli_left_total(const orc_node_resource* n);
int64_t orc_get_gpu_frag_milli(const orc_node_resource* n, const orc_pod_resource* p);
void    orc_node_gpu_share_frag_amount(const orc_node_resource* n, const orc_target_pod* tp, int nt,
                                       double out_bins[ORC_NBINS]);
double  orc_frag_amount_sum_except_q3(const double bins[ORC_NBINS]);
double  orc_frag_amount_sum_q1q2q4(const double bins[ORC_NBINS]);
double  orc_node_gpu_share_frag_amount_score(const orc_node_resource* n, const orc_target_pod* tp, int nt);

/* ---- Go math restated ---- */
double  orc_go_exp(double x);          /* Go src/math/exp.go (portable algorithm) */
double  orc_sigmoid(double x);         /* plugin_utils.go:76-78 */
/* The FGD score as a step function of delta = cur - new: th[k] = smallest delta with score >= k
 * (th[0] = -inf, th[101] = +inf); 0, or -1 if the steps are not monotone. */
int     orc_score_thresholds(double* th /* [102] */);
/* math.Exp census: while on, every FGD score delta the path evaluates is compared with th[];
 * end returns the smallest distance |delta - th[k]|, where it happened (event, node, k) and the
 * number of deltas seen. */
typedef struct { double delta; int event, node, score, score_nudged, ulps; } orc_census_case;
void    orc_pwr_lohi_trace(int64_t* buf, int cap); /* diagnostics: per-step raw PWR min / max */
int     orc_census_begin(void);
/* deltas within 1e-10 of a step; of those, the ones whose score differs from the one a correctly
 * rounded exp gives (crdiff) and, of the rest, the ones whose score changes when exp's result moves
 * by one ulp (sensitive); the first 16 cases of each kept */
void    orc_census_near(long long* near, long long* crdiff, long long* sensitive, double* sens_max /* max |delta| */,
                        orc_census_case* cr_cases /* [16] */, orc_census_case* sens_cases /* [16] */);
/* census runs only: move every exp result by `ulps` ulps; mode 1 = exp in x87 extended precision
 * rounded to double (a stand-in for a correctly rounded exp); 0 / 0 = the portable algorithm */
void    orc_set_exp_nudge(int ulps);
void    orc_set_exp_mode(int mode);
void    orc_census_end(double* min_dist, double* delta_at, int* step_at, int* node_at, int* k_at, long long* n,
                       double* th /* [102] or NULL */);

/* ---- resource.go helpers ---- */
int     orc_node_sub(const orc_node_resource* n, const orc_pod_resource* p, orc_node_resource* out);
int     orc_node_add(const orc_node_resource* n, const orc_pod_resource* p, const int* idl, int nidl,
                     orc_node_resource* out);
/* AllocateExclusiveGpuId -> bitmask of GPU indices; -1 when it would panic */
int     orc_allocate_exclusive_gpu_id(const orc_node_resource* n, const orc_pod_resource* p);
/* Flatten("x").MilliGpu string, e.g. "600,350,200,0,0,0,0,0," */
void    orc_flatten_milli_gpu(const orc_node_resource* n, char* out, int cap);

/* ---- score plugins ---- */
/* fgd_score.go:99-149: returns score; *gpu_mask = chosen GPU set (0 = "") */
int64_t orc_fgd_score(const orc_node_resource* n, const orc_pod_resource* p, const orc_target_pod* tp, int nt,
                      int* gpu_mask);
int64_t orc_best_fit_score(const orc_node_resource* n, const orc_pod_resource* p);      /* -1 = error */
int64_t orc_dot_product_score(const orc_node_resource* n, const orc_pod_resource* p);   /* merge/max */
/* dimExtMethod / normMethod (config.go:3-55); *gid = the best match group's GpuId as a bitmask */
enum { ORC_DIM_MERGE = 0, ORC_DIM_SHARE = 1, ORC_DIM_DIVIDE = 2, ORC_DIM_EXTEND = 3 };
enum { ORC_NORM_MAX = 0, ORC_NORM_NODE = 1, ORC_NORM_POD = 2 };
int64_t orc_dot_product_score_cfg(const orc_node_resource* n, const orc_pod_resource* p, int dim, int norm, int* gid);
double  orc_vector_dot_product(const double* a, int la, const double* b, int lb);
void    orc_normalize_vector(double* v, int len, const double* nv, int nlen);
double  orc_go_tanh(double x);
int64_t orc_packing_score(const orc_node_resource* n, const orc_pod_resource* p, int* err);
int64_t orc_clustering_score(const orc_node_resource* n, const orc_pod_resource* p, int pod_tag,
                             const int32_t* node_tag_counts);
void    orc_normalize_score(int64_t* scores, int n);                                     /* plugin_utils.go:48-74 */
/* resource.go:536-563 GetEnergyConsumptionNode; 0 ok, -1 GPU model without an energy model
 * (the reference calls a nil func), -2 CPU model unknown (its map lookup yields NaN power) */
int     orc_energy_node(const orc_node_resource* n, double* cpu_power, double* gpu_power);
/* pwr_score.go:143-212 calculatePWRShareExtendScore: returns score; *gpu_mask = chosen GPU set;
 * *err = 1 when orc_energy_node fails */
int64_t orc_pwr_score(const orc_node_resource* n, const orc_pod_resource* p, int* gpu_mask, int* err);
void    orc_normalize_score_pwr(int64_t* scores, int n);                                 /* pwr_score.go:104-141 */
int     orc_alloc_gpu_best_fit(const orc_node_resource* n, const orc_pod_resource* p);   /* mask, -1 none */

/* ---- typical pods (frag.go:285-380) ---- */
typedef struct {
    int64_t cpu_milli;     /* container cpu request (milli); used for MilliCpu non-zero default */
    int32_t has_cpu;       /* 0 -> non-zero default 100m */
    int64_t gpu_milli;
    int32_t gpu_number;
    char    gpu_type[ORC_TYPE_LEN];
} orc_workload_pod;

typedef struct {
    int32_t is_involved_cpu_pods;
    int32_t pod_popularity_threshold;
    int32_t pod_increase_step;
    double  gpu_res_weight;
} orc_typical_cfg;

int orc_get_typical_pods(const orc_workload_pod* pods, int n, orc_typical_cfg cfg, orc_target_pod* out, int cap);

/* ---- replay driver (scheduleOne semantics) ---- */
enum { ORC_POL_FGD = 0, ORC_POL_BESTFIT = 1, ORC_POL_DOTPROD = 2, ORC_POL_PACKING = 3,
       ORC_POL_CLUSTERING = 4, ORC_POL_RANDOM = 5,
       ORC_POL_PWR = 6,       /* PWRScore alone */
       ORC_POL_PWR_FGD = 7 }; /* PWRScore + FGDScore, weights orc_policy.w_pwr / w_fgd */
enum { ORC_SEL_BEST = 0, ORC_SEL_WORST = 1, ORC_SEL_RANDOM = 2, ORC_SEL_FGD = 3, ORC_SEL_PWR = 4, ORC_SEL_DOTPROD = 5 };

typedef struct {
    char    name[64];              /* full node name, e.g. "0042-openb-node-0001" (tie-break key) */
    int64_t cpu_alloc;             /* milli */
    int64_t mem_alloc;             /* MiB */
    int32_t pods_alloc;
    int32_t gpu_count;
    char    gpu_type[ORC_TYPE_LEN];
    char    cpu_type[ORC_TYPE_LEN];    /* alibabacloud.com/cpu-model ("" when absent) */
} orc_node_spec;

typedef struct {
    int64_t cpu_req;               /* actual container request, milli (fitsRequest / Requested) */
    int64_t cpu_nz;                /* GetNonzeroRequests value (Score) */
    int64_t mem_req;               /* MiB */
    int64_t gpu_milli;
    int32_t gpu_number;
    int32_t is_delete;             /* deletion event */
    int32_t ref;                   /* deletion: index of the creation event */
    char    gpu_type[ORC_TYPE_LEN];
} orc_event;

typedef struct {
    int32_t node;                  /* winning node index, -1 = failed */
    int32_t gpu_mask;              /* GPUs assigned (Reserve) */
    int64_t score;                 /* winning total score (0 if single-feasible shortcut) */
    int32_t n_feasible;
    int32_t status;                /* 0 ok, 1 unschedulable, 2 error */
} orc_result;

typedef struct {
    double  frag_bins[ORC_NBINS];  /* cluster sum of NodeGpuShareFragAmount (analysis.go:81-85) */
    int64_t used_nodes, used_gpus, used_gpu_milli, total_gpus, arrived_gpu_milli;
    int64_t used_cpu_milli, arrived_cpu_milli;
    double  frag_bins_exact[ORC_NBINS]; /* the same sums, exact, rounded once to nearest (see
                                           orc_fix80 in fgd_oracle.c; the product's contract) */
    /* analysis.go:24-56 ClusterPowerConsumptionReport: Σ over nodes (input order) of
     * orc_energy_node's CPU and GPU terms; nodes where it fails are counted, not summed */
    double  power_cpu, power_gpu;
    int64_t power_invalid;
} orc_report;

/* Go math/rand's global source (rng.go rngSource), for the Random draw structure */
#define ORC_GO_LEN 607
#define ORC_GO_TAP 273
typedef struct {
    int32_t tap, feed;
    uint64_t vec[ORC_GO_LEN];
} orc_go_rng;
void     orc_go_seed(orc_go_rng* g, int64_t seed);      /* rand.Seed */
uint64_t orc_go_uint64(orc_go_rng* g);                  /* rngSource.Uint64 */
int32_t  orc_go_int31n(orc_go_rng* g, int32_t n);       /* Rand.Int31n (= Intn for n < 2^31) */

typedef struct {
    int32_t policy;
    int32_t gpu_sel;
    uint64_t seed;                 /* Random policy: see DESIGN.md "Random contract" */
    int32_t threads;               /* >1: parallelize.Until-style worker fan-out over nodes */
    int32_t w_pwr, w_fgd;          /* ORC_POL_PWR_FGD plugin weights (scheduler config score weights) */
    int32_t dim_ext, norm;         /* ORC_POL_DOTPROD GpuPluginCfg (ORC_DIM_*, ORC_NORM_*) */
    /* non-NULL: the Random draw structure on Go's global math/rand stream, starting from this
     * state (the stream after the replay's own draws; copied, not modified).  Per creation event:
     * scheduler.go:464 Intn(100); no feasible node: default_preemption.go:183 Int31n(#nodes);
     * two or more: random_score.go:44 Intn(#feasible), the node at that index of the feasible list
     * in node order (PreScore runs for every policy; Random's Score picks that node); Reserve with
     * the random GPU selector: open_gpu_share.go:333 Intn(k) at the k-th fitting GPU. */
    const orc_go_rng* go_stream;
} orc_policy;

/* Replays n events on a fresh cluster.  results[n]; reports[n] may be NULL. */
int orc_run_events(const orc_node_spec* nodes, int n_nodes, const orc_target_pod* tp, int nt,
                   orc_policy pol, const orc_event* ev, int n_ev, orc_result* results, orc_report* reports);

/* Final per-node state after orc_run_events (call with the same inputs). */
typedef struct {
    int64_t cpu_left, mem_left;
    int32_t pods;
    int32_t gpu_left[8];
} orc_node_state;
int orc_run_events_state(const orc_node_spec* nodes, int n_nodes, const orc_target_pod* tp, int nt,
                         orc_policy pol, const orc_event* ev, int n_ev, orc_result* results,
                         orc_report* reports, orc_node_state* final_state);

/* Random-policy hash (DESIGN.md "Random contract"); exported for tests. */
uint64_t orc_mix64(uint64_t x);

#ifdef __cplusplus
}
#endif
#endif

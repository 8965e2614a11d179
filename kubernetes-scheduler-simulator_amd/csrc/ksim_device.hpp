// ksim_device.hpp -- device-side data layout and the per-node math of the
// Filter+Score path (gfx950).  Every function cites the reference Go code it
// restates (paths relative to Fr4nz83/kubernetes-scheduler-simulator @ 2024_08_07).
//
// Compiled with -ffp-contract=off: Go (amd64, GOAMD64=v1) never fuses a*b+c,
// and every fp64 expression below keeps Go's evaluation order so that the
// fragmentation amounts are bit-identical to the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KSIM_HD __host__ __device__ __forceinline__

namespace ksim {

constexpr int kMaxGpu = 8;
constexpr int kMilli = 1000;         // open-gpu-share/utils/const.go:14
constexpr int kMaxSpecCpu = 128000;  // const.go:16
constexpr int kMaxSpecGpu = 8000;    // const.go:18
constexpr int kNumTags = 9;
constexpr int kMaxTypical = 256;

// One node of one replica in HBM: 32 B, read once per pod step.
struct __align__(16) NodeRec {
  int32_t cpu_left;    // Allocatable.MilliCPU - Requested.MilliCPU
  int32_t mem_left;    // MiB
  uint16_t gl[kMaxGpu];  // milli-GPU left per device (0 beyond gpu_cnt)
  int16_t pods_left;   // AllowedPodNumber - len(Pods)
  uint8_t gpu_cnt;
  uint8_t gpu_type;    // model id, 0..31
  uint32_t name_rank;  // byte-wise rank of the node name
};
static_assert(sizeof(NodeRec) == 32, "NodeRec must stay 32 B");

// Register image of a NodeRec: eight dwords, fields extracted with shifts so
// that no per-lane array ever lands in scratch (gl(g) is only called with
// compile-time g inside unrolled loops).
struct NodeV {
  int32_t cpu_left;
  int32_t mem_left;
  uint32_t g[4];     // two u16 milli-left values per dword
  uint32_t meta;     // pods_left (i16) | gpu_cnt << 16 | gpu_type << 24
  uint32_t name_rank;
  KSIM_HD int gl(int i) const {
    const uint32_t w = i < 2 ? g[0] : (i < 4 ? g[1] : (i < 6 ? g[2] : g[3]));
    return (int)((i & 1) ? (w >> 16) : (w & 0xffffu));
  }
  KSIM_HD int pods_left() const { return (int)(int16_t)(meta & 0xffffu); }
  KSIM_HD int gpu_cnt() const { return (int)((meta >> 16) & 0xffu); }
  KSIM_HD int gpu_type() const { return (int)(meta >> 24); }
  // The eight milli-left lanes as packed 16-bit pairs (v_pk_* on gfx950).  Every record keeps 0 <= gl <= 1000 and
  // gl = 0 on the lanes past gpu_cnt (set_nodes; a Bind touches only the node's own GPUs), which the packed
  // reductions below rely on: they fold all eight lanes with no per-lane `g < gpu_cnt` test.
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  KSIM_HD static u16x2 pk(uint32_t w) {
    u16x2 v;
    __builtin_memcpy(&v, &w, 4);
    return v;
  }
  KSIM_HD int total() const {  // (<= 8000: no packed lane overflows)
    const u16x2 t = (pk(g[0]) + pk(g[1])) + (pk(g[2]) + pk(g[3]));
    return (int)t.x + (int)t.y;
  }
  KSIM_HD int gl_max() const {  // the most milli left on one GPU (0 with no GPU)
    const u16x2 m = __builtin_elementwise_max(__builtin_elementwise_max(pk(g[0]), pk(g[1])),
                                              __builtin_elementwise_max(pk(g[2]), pk(g[3])));
    return m.x > m.y ? (int)m.x : (int)m.y;
  }
  KSIM_HD int gl_full() const {  // GPUs with all 1000 milli left: gl - 999 saturated at 0 is 1 there and 0 below
    const u16x2 k = {(unsigned short)999, (unsigned short)999};
    const u16x2 t = (__builtin_elementwise_sub_sat(pk(g[0]), k) + __builtin_elementwise_sub_sat(pk(g[1]), k)) +
                    (__builtin_elementwise_sub_sat(pk(g[2]), k) + __builtin_elementwise_sub_sat(pk(g[3]), k));
    return (int)t.x + (int)t.y;
  }
};

KSIM_HD NodeV load_node(const NodeRec* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  NodeV n;
  n.cpu_left = (int32_t)a.x;
  n.mem_left = (int32_t)a.y;
  n.g[0] = a.z; n.g[1] = a.w; n.g[2] = b.x; n.g[3] = b.y;
  n.meta = b.z;
  n.name_rank = b.w;
  return n;
}
KSIM_HD void store_node(NodeRec* p, const NodeV& n) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4((uint32_t)n.cpu_left, (uint32_t)n.mem_left, n.g[0], n.g[1]);
  q[1] = make_uint4(n.g[2], n.g[3], n.meta, n.name_rank);
}

// tags[tag] += sign on a node's u16 tag counts in HBM without reading them back: one fire-and-forget atomic on
// the u32 word holding the pair (a count stays within its half), so no load latency sits on the Bind's path.
// For the tag counts no kernel reads during the run (every policy but GpuClustering, whose counts sit in LDS).
__device__ __forceinline__ void tag_add(uint16_t* tags, int tag, int sign) {
  unsigned* w = reinterpret_cast<unsigned*>(tags + (tag & ~1));
  const unsigned one = 1u << (16 * (tag & 1));
  atomicAdd(w, sign > 0 ? one : 0u - one);
}

// One event of one replica: 32 B.
struct __align__(16) PodDev {
  int32_t cpu_req;   // Filter / Requested
  int32_t cpu_nz;    // Score (non-zero default)
  int32_t mem;       // MiB
  int16_t milli;     // per-GPU milli
  int8_t num;        // GPU count
  int8_t tag;        // -1 no-gpu, 0 share-gpu, k "k-gpu", -2 invalid (reference panics)
  uint32_t tmask;    // accepted model bitmask
  int32_t ref;       // deletion: creation index
  uint32_t flags;    // kPodDelete
  int32_t pad;
};
static_assert(sizeof(PodDev) == 32, "PodDev must stay 32 B");
constexpr uint32_t kPodDelete = 1u;

// Typical-pod table entry: 32 B, read with scalar loads (uniform across the workgroup).
// Per replica the table is split, order preserved within each part:
//   [0, ncpu)   typical pods with MilliGpu == 0   (feed only bins XL, XR)
//   [ncpu, nt)  typical pods with MilliGpu  > 0   (feed only bins Q1, Q2, Q4, NA)
// Each bin is a sequential sum over its own subsequence, so the split keeps
// every bin bit-identical to the reference's single pass (frag.go:153-186).
struct __align__(32) TypDev {
  int32_t cpu;
  int32_t milli;
  int32_t num_eff;  // max(GpuNumber, 1): CanNodeHostPodOnGpuMemory (frag.go:447-458)
  uint32_t tmask;
  double freq;
  int32_t pad[2];
};
static_assert(sizeof(TypDev) == 32, "TypDev must stay 32 B");

struct ResultDev {  // == ksim_result
  int32_t node;
  int32_t gpu_mask;
  int64_t score;
  int32_t n_feasible;
  int32_t status;
};
static_assert(sizeof(ResultDev) == 24, "ResultDev must match ksim_result");

struct ReplicaDev {
  int32_t policy;
  int32_t gpusel;
  uint64_t seed;
  int32_t n_events;
  int32_t nt;    // typical entries: [0, ncpu) CPU-only, [ncpu, nt) GPU
  int32_t ncpu;
  int32_t typed; // some GPU entry names a model (NA bin reachable)
  const TypDev* tp;
  const PodDev* ev;
  ResultDev* res;
  NodeRec* nodes;
  uint16_t* tags;  // [N][16]
  // cluster report (null when disabled): the state a Bind / delete left on the node it changed,
  // the previous event that changed the same node (-1: none since the run started), the
  // per-event exact report, the static allocatable CPU per node and the run's initial state
  NodeRec* snap;         // [E]
  int32_t* prev;         // [E]
  struct RepAcc* rep;    // [E]
  const int32_t* cap;    // [N] MilliCpuCapacity (utils.go:1101)
  const NodeRec* init;   // [N]
  int32_t* last;         // [N] k_step: last event that changed each node
  int32_t node_off;      // node-sharded cluster: global index (= name rank) of local node 0, else 0
  int32_t dpcfg;         // DotProduct GpuPluginCfg: dimExtMethod | normMethod << 4 (dp_dim / dp_norm)
  // PWR (pwr_score.go): energy model, CPU model id per node, per-node PWR scratch of the
  // two-phase k_step cycle (raw PWR score | packed FGD score and GPU choices), plugin weights
  const struct PowerDev* pw;
  const uint8_t* cpum;   // [N]
  int2* pws;             // [N]
  int32_t w_pwr, w_fgd;
  int32_t has_pw;        // an energy model was given: the cluster report adds the [Power] terms
  int32_t n_local;       // the replica's node count (a node-sharded k_replay group: each shard's own)
  const int32_t* mcap;   // [N] allocatable memory, MiB (the Unreserve guard)
};

// Per-event cluster report, exact (fixed point 2^-80 for the fp64 terms; see fix80).
// fx: the 7 frag bins, then the cluster's CPU and GPU power (ClusterPowerConsumptionReport, W).
// cnt: used nodes, used GPUs, used GPU milli, used CPU milli, arrived GPU milli, arrived CPU milli,
//      nodes without an energy model (the reference's power report would fail on them), pad.
struct __align__(16) RepAcc {
  __int128 fx[9];
  long long cnt[8];
};
static_assert(sizeof(RepAcc) == 208, "RepAcc layout");

// Per-replica cross-workgroup accumulators for one step (reset by the last block).
struct __align__(64) Accum {
  unsigned long long best;  // packed argmax key
  int32_t nfeas;
  int32_t err;
  int32_t lo;               // BestFit NormalizeScore: min raw score
  int32_t hi;               // max raw score
  uint32_t ticket;
  int32_t pad[9];
};

enum : int { POL_FGD = 0, POL_BESTFIT = 1, POL_DOTPROD = 2, POL_PACKING = 3, POL_CLUSTERING = 4, POL_RANDOM = 5,
             POL_PWR = 6, POL_PWR_FGD = 7 };
enum : int { SEL_BEST = 0, SEL_WORST = 1, SEL_RANDOM = 2, SEL_FGD = 3, SEL_PWR = 4, SEL_DOTPROD = 5 };
KSIM_HD bool is_pwr_policy(int pol) { return pol == POL_PWR || pol == POL_PWR_FGD; }

// PWR energy model (== ksim_power_model): resource.go:536-563 GetEnergyConsumptionNode with the
// const.go:41-124 tables, indexed by GPU model id and CPU model id
constexpr int kMaxCpuModels = 8;
struct PowerDev {
  double gidle[32], gfull[32];
  double cidle[kMaxCpuModels], cfull[kMaxCpuModels], cnc[kMaxCpuModels];
  uint32_t gvalid;  // GPU model ids with an energy model (MapGpuTypeModelEnergy)
  uint32_t gnone;   // GPU model ids standing for "no gpu-card-model label" (GpuType == "": no GPU term)
  uint32_t cvalid;
  uint32_t pad;
};
enum : int { ST_OK = 0, ST_UNSCHED = 1, ST_ERROR = 2, ST_DELETED = 3 };

// ---------------------------------------------------------------------------
// Go math.Exp, portable algorithm (Go src/math/exp.go).  Identical operation
// sequence to oracle/fgd_oracle.c orc_go_exp.
// ---------------------------------------------------------------------------
KSIM_HD double go_exp(double x) {
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
  if (x != x) return x;
  if (x > Overflow) return __builtin_bit_cast(double, 0x7ff0000000000000LL);
  if (x < Underflow) return 0.0;
  if (-NearZero < x && x < NearZero) return 1 + x;
  int k = 0;
  if (x < 0) k = (int)(Log2e * x - 0.5);
  else if (x > 0) k = (int)(Log2e * x + 0.5);
  double hi = x - (double)k * Ln2Hi;
  double lo = (double)k * Ln2Lo;
  double r = hi - lo;
  double t = r * r;
  double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
  int k1 = k / 2, k2 = k - k1;
  double a = __builtin_bit_cast(double, (long long)(1023 + k1) << 52);
  double b = __builtin_bit_cast(double, (long long)(1023 + k2) << 52);
  return (y * a) * b;
}

// plugin_utils.go:76-78
KSIM_HD double go_sigmoid(double x) { return 1.0 / (1.0 + go_exp(-x)); }

// Go math.Tanh, portable algorithm (Go src/math/tanh.go: the Cephes rational form below 0.625,
// 1 - 2 / (exp(2|x|) + 1) above), operation for operation; the oracle's orc_go_tanh is the same
// sequence.  Used by DotProduct's normMethod "pod" (dot_product_score.go:79).
KSIM_HD double go_tanh(double x) {
  const double P0 = -9.64399179425052238628e-1, P1 = -9.92877231001918586564e1, P2 = -1.61468768441708447952e3;
  const double Q0 = 1.12811678491632931402e2, Q1 = 2.23548839060100448583e3, Q2 = 4.84406305325125486048e3;
  const double kMaxLog = 8.8029691931113054295988e+01;  // log(2**127)
  double z = x < 0 ? -x : x;
  if (z > 0.5 * kMaxLog) return x < 0 ? -1.0 : 1.0;
  if (z >= 0.625) {
    const double s = go_exp(2 * z);
    z = 1 - 2 / (s + 1);
    return x < 0 ? -z : z;
  }
  if (x == 0) return x;
  const double s = x * x;
  return x + x * s * ((P0 * s + P1) * s + P2) / (((s + Q0) * s + Q1) * s + Q2);
}

// fgd_score.go:123 fragScore = int64(sigmoid((cur-new)/1000) * MaxNodeScore)
KSIM_HD int fgd_frag_score(double cur, double nw) {
  return (int)(go_sigmoid((cur - nw) / 1000) * (double)100);
}
// The same score as a function of delta = cur - new (the first operation of the expression above).
KSIM_HD int fgd_score_of_delta(double delta) { return (int)(go_sigmoid(delta / 1000) * (double)100); }

// fgd_score_of_delta is a step function of delta: every step of it (delta/1000, negation, go_exp,
// 1 + e, 1 / x, * 100, truncation) is monotone, so the score is #{k in 1..100 : delta >= th[k]}
// where th[k] is the smallest double delta with score >= k.  build_score_thresholds finds every
// th[k] by bisection over the ordered integer image of the doubles, then checks the step on
// +-kScoreCheckUlps doubles around each threshold (the only place where a rounding blip of
// go_exp could matter); it returns false if any check fails, and the table must not be used.
// th[0] = -inf, th[101] = +inf.
constexpr int kScoreCheckUlps = 4096;
inline long long score_key_of(double d) {
  const long long b = __builtin_bit_cast(long long, d);
  return b >= 0 ? b : (long long)(0x8000000000000000ull - (unsigned long long)b);  // order preserving
}
inline double score_double_of(long long k) {
  return __builtin_bit_cast(double, k >= 0 ? k : (long long)(0x8000000000000000ull - (unsigned long long)k));
}
inline bool build_score_thresholds(double* th /* [102] */) {
  th[0] = -__builtin_huge_val();
  th[101] = __builtin_huge_val();
  const long long lo0 = score_key_of(-1.0e9), hi0 = score_key_of(1.0e9);
  if (fgd_score_of_delta(-1.0e9) != 0 || fgd_score_of_delta(1.0e9) != 100) return false;
  for (int k = 1; k <= 100; ++k) {
    long long lo = lo0, hi = hi0;  // score(lo) < k <= score(hi)
    while ((unsigned long long)hi - (unsigned long long)lo > 1ull) {  // the span exceeds INT64_MAX
      const long long mid = (long long)((unsigned long long)lo + ((unsigned long long)hi - (unsigned long long)lo) / 2);
      if (fgd_score_of_delta(score_double_of(mid)) >= k) hi = mid;
      else lo = mid;
    }
    th[k] = score_double_of(hi);
    for (long long j = -kScoreCheckUlps; j <= kScoreCheckUlps; ++j) {
      const int s = fgd_score_of_delta(score_double_of(hi + j));
      if ((j < 0 && s >= k) || (j >= 0 && s < k)) return false;
    }
    if (k > 1 && !(th[k] > th[k - 1])) return false;
  }
  return true;
}
// The score from the table: an fp32 estimate (error far below one score unit), corrected by the
// two thresholds around it.  Equal to fgd_score_of_delta(delta) for every finite delta.
KSIM_HD int fgd_score_lookup(double delta, const double* th) {
  const float e = __builtin_expf((float)delta * -0.001f);
  int a = (int)(100.0f / (1.0f + e));
  a = a < 0 ? 0 : (a > 100 ? 100 : a);
  if (delta >= th[a + 1]) ++a;
  else if (delta < th[a]) --a;
  return a;
}

// ---------------------------------------------------------------------------
// F(state) = NodeGpuShareFragAmountScore (frag.go:200-203)
//          = FragAmountSumExceptQ3 (frag.go:411-418) of NodeGpuShareFragAmount
//            (frag.go:148-188) with GetNodePodFrag (frag.go:460-493).
// Each bin is a sequential fp64 sum in typical-pod order; a bin a typical pod
// does not touch receives +0.0, which leaves every non-negative sum bit-exact.
// Bin Q3 (index 2) is not part of F and is not accumulated here.
// kTyped = some GPU typical pod names a GPU model (else the NA bin stays 0).
// ---------------------------------------------------------------------------
template <bool kTyped>
KSIM_HD double frag_F(int cpuL, const int (&gl)[kMaxGpu], uint32_t typebit, const TypDev* __restrict__ tp,
                      int ncpu, int nt) {
  int total = 0;
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) total += gl[g];  // GetGpuMilliLeftTotal (frag.go:224-229)
  const double dtot = (double)total;
  // CPU-only typical pods: XL / XR (frag.go:463-469)
  double b4 = 0.0, b5 = 0.0;
#pragma unroll 2
  for (int t = 0; t < ncpu; ++t) {
    const double x = tp[t].freq * dtot;  // freq * float64(gpuMilliLeftTotal)
    const bool cpu_ok = cpuL >= tp[t].cpu;
    b4 += cpu_ok ? x : 0.0;
    b5 += cpu_ok ? 0.0 : x;
  }
  double b0 = 0.0, b1 = 0.0, b3 = 0.0, b6 = 0.0;
#pragma unroll 2
  for (int t = ncpu; t < nt; ++t) {
    const int m = tp[t].milli;
    const double f = tp[t].freq;
    const double x = f * dtot;
    const bool cpu_ok = cpuL >= tp[t].cpu;
    int cnt = 0, frag = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      const bool ge = gl[g] >= m;
      cnt += ge ? 1 : 0;               // CanNodeHostPodOnGpuMemory (frag.go:447-458)
      frag += ge ? 0 : gl[g];          // GetGpuFragMilliByNodeResAndPodRes (frag.go:205-213)
    }
    const bool gpu_ok = cnt >= tp[t].num_eff;
    const double y = f * (double)frag;  // freq * float64(gpuFragMilli)
    if (kTyped) {
      const bool acc = (tp[t].tmask & typebit) != 0u;  // IsNodeAccessibleToPod (utils.go:957-1006)
      b0 += (acc && !gpu_ok && !cpu_ok) ? x : 0.0;        // Q1
      b1 += (acc && cpu_ok) ? (gpu_ok ? y : x) : 0.0;     // Q2 (Q3 adds its frag part here)
      b3 += (acc && gpu_ok && !cpu_ok) ? x : 0.0;         // Q4
      b6 += acc ? 0.0 : x;                                // NA
    } else {
      b0 += (!gpu_ok && !cpu_ok) ? x : 0.0;
      b1 += cpu_ok ? (gpu_ok ? y : x) : 0.0;
      b3 += (gpu_ok && !cpu_ok) ? x : 0.0;
    }
  }
  double out = 0.0;
  out += b0;
  out += b1;
  out += b3;
  out += b4;
  out += b5;
  out += b6;
  return out;
}

// NodeGpuShareFragAmount (frag.go:148-188): all 7 bins of one node state (Q1, Q2, Q3, Q4, XL,
// XR, NA; frag.go:27-35), the per-node term of the cluster report (analysis.go:81-85).  Every
// bin is a sequential fp64 sum in typical-pod order: the table split of TypDev keeps the
// order of each bin, since CPU-only pods only touch XL/XR and GPU pods only Q1-Q4/NA.
KSIM_HD void frag_bins7(int cpuL, const int (&gl)[kMaxGpu], uint32_t typebit, const TypDev* __restrict__ tp,
                        int ncpu, int nt, double (&b)[7]) {
  int total = 0;
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) total += gl[g];  // GetGpuMilliLeftTotal (frag.go:224-229)
  const double dtot = (double)total;
#pragma unroll
  for (int k = 0; k < 7; ++k) b[k] = 0.0;
  for (int t = 0; t < ncpu; ++t) {  // GetNodePodFrag case 1 (frag.go:463-469)
    const double x = tp[t].freq * dtot;
    if (cpuL >= tp[t].cpu) b[4] += x;
    else b[5] += x;
  }
  for (int t = ncpu; t < nt; ++t) {
    const double f = tp[t].freq;
    const int m = tp[t].milli;
    int cnt = 0, frag = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      cnt += gl[g] >= m ? 1 : 0;   // CanNodeHostPodOnGpuMemory (frag.go:447-458)
      frag += gl[g] < m ? gl[g] : 0;  // GetGpuFragMilliByNodeResAndPodRes (frag.go:205-213)
    }
    const bool cpu_ok = cpuL >= tp[t].cpu;
    const bool gpu_ok = cnt >= tp[t].num_eff;
    if ((tp[t].tmask & typebit) == 0u) {
      b[6] += f * dtot;                      // NA (frag.go:472-474)
    } else if (gpu_ok && cpu_ok) {           // Q3: frag part to Q2, the rest to Q3 (frag.go:174-181)
      b[1] += f * (double)frag;
      b[2] += f * (double)(total - frag);
    } else if (gpu_ok) {
      b[3] += f * dtot;                      // Q4
    } else if (cpu_ok) {
      b[1] += f * dtot;                      // Q2
    } else {
      b[0] += f * dtot;                      // Q1
    }
  }
}

// Exact fixed-point image of a non-negative fp64 value: x * 2^80 as a 128-bit integer
// (truncated below 2^-80).  Cluster sums of these are exact and order independent, so the
// report's cluster bins are the correctly rounded exact sum of the per-node fp64 bins
// (DESIGN.md "Cluster report"); the reference sums them in Go map order (analysis.go:80-98).
KSIM_HD __int128 fix80(double x) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  const int ex = (int)((b >> 52) & 0x7ff);
  if (ex == 0) return 0;  // zero / subnormal (< 2^-1022): far below 2^-80
  const unsigned long long m = (b & ((1ull << 52) - 1)) | (1ull << 52);
  const int sh = ex - 1075 + 80;  // x = m * 2^(ex-1075)
  __int128 v = sh >= 0 ? ((__int128)m << sh) : (sh > -64 ? (__int128)(m >> (-sh)) : (__int128)0);
  return (b >> 63) ? -v : v;
}

KSIM_HD void unpack_gl(const NodeV& n, int (&gl)[kMaxGpu]) {
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) gl[g] = n.gl(g);
}

// Filter: fitsRequest (fit.go:230-290) ∧ GpuSharePlugin.Filter (open_gpu_share.go:81-118)
//         ∧ GpuNodeInfo.AllocateGpuId (gpunodeinfo.go:136-204).
KSIM_HD bool filter_node(const NodeV& n, const PodDev& p) {
  if (n.pods_left() < 1) return false;
  if (!(p.cpu_req == 0 && p.mem == 0)) {
    if (n.cpu_left < p.cpu_req) return false;
    if (n.mem_left < p.mem) return false;
  }
  if (p.milli <= 0) return true;
  const int cnt = n.gpu_cnt();
  if (cnt == 0) return false;
  if ((p.tmask & (1u << n.gpu_type())) == 0u) return false;
  if (p.num <= 0) return false;
  if (p.num == 1) {
    bool any = false;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) any |= (g < cnt) && (n.gl(g) >= p.milli);
    return any;
  }
  // multi-GPU two-pointer greedy: a device can host floor(idle/milli) slots
  int slots = 0;
  if (p.milli == kMilli) {  // whole GPUs (every multi-GPU pod of the traces): floor(idle/1000) = idle == 1000
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) slots += (g < cnt && n.gl(g) == kMilli) ? 1 : 0;
    return slots >= p.num;
  }
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g)
    if (g < cnt) slots += n.gl(g) / p.milli;
  return slots >= p.num;
}

// filter_node's decisions without its early returns (k_scan1's per-slot scan: there the return chain diverged per
// lane, each exit an exec-mask branch).  The pod's fields are uniform in a scan, so only its branches remain.
KSIM_HD bool filter_scan(const NodeV& n, const PodDev& p) {
  bool ok = n.pods_left() >= 1;
  const bool zero = p.cpu_req == 0 && p.mem == 0;
  ok = ok & (zero | ((n.cpu_left >= p.cpu_req) & (n.mem_left >= p.mem)));
  if (p.milli > 0) {
    const int cnt = n.gpu_cnt();
    bool dev = (cnt != 0) & (((p.tmask >> n.gpu_type()) & 1u) != 0u) & (p.num > 0);
    if (p.num == 1) {  // some GPU holds the share (packed max over the lanes; p.milli >= 1)
      dev = dev & (n.gl_max() >= p.milli);
    } else if (p.milli == kMilli) {  // enough whole GPUs
      dev = dev & (n.gl_full() >= p.num);
    } else {
      dev = dev & filter_node(n, p);  // a partial multi-GPU request (no trace has one)
    }
    ok = ok & dev;
  }
  return ok;
}

KSIM_HD bool is_share_pod(const PodDev& p) { return p.num == 1 && p.milli < kMilli; }

// GPUs selected by NodeResource.Sub (resource.go:454-480): ascending stable
// order of milli left, first `num` devices with left >= milli.  Returns mask;
// *ok=false when Sub would return its early error (state left unchanged).
KSIM_HD unsigned sub_gpu_mask(const int (&gl)[kMaxGpu], int gpu_cnt, int cpuL, const PodDev& p,
                                                 bool* ok) {
  *ok = !(cpuL < p.cpu_nz || gpu_cnt < p.num);
  if (!*ok || p.num <= 0) return 0u;
  unsigned taken = 0u;
  if (p.milli == kMilli) {
    // whole GPUs: only fully free devices qualify; the stable ascending order keeps them in index order
    int need = p.num;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      if (need > 0 && g < gpu_cnt && gl[g] == kMilli) {
        taken |= 1u << g;
        --need;
      }
    }
    return taken;
  }
  for (int k = 0; k < p.num; ++k) {
    int best = -1, bv = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      const bool cand = g < gpu_cnt && !((taken >> g) & 1u) && gl[g] >= p.milli;
      if (cand && (best < 0 || gl[g] < bv)) { best = g; bv = gl[g]; }
    }
    if (best < 0) break;
    taken |= 1u << best;
  }
  return taken;
}

// AllocateExclusiveGpuId (resource.go:383-403): lowest-index fully free GPUs.
// Returns -1 where the reference panics.
KSIM_HD int exclusive_gpu_mask(const NodeV& n, const PodDev& p) {
  int req = (int)p.milli * (int)p.num;
  int mask = 0;
  const int cnt = n.gpu_cnt();
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) {
    if (req > 0 && g < cnt && n.gl(g) == kMilli) {
      mask |= 1 << g;
      req -= kMilli;
    }
  }
  return req > 0 ? -1 : mask;
}

// GetEnergyConsumptionNode (resource.go:536-563) of a node state; false when the reference would
// fail (a GPU model without an energy model: nil func call; an unknown CPU model).  Go's
// operation order; every term is an exact small integer in fp64.
KSIM_HD bool node_energy(int cpuL, int cap, int cm, const int (&gl)[kMaxGpu], int cnt, int gtype, const PowerDev& pw,
                         double* energy) {
  double gpu = 0;
  if (!((pw.gnone >> gtype) & 1u)) {
    if (!((pw.gvalid >> gtype) & 1u)) return false;
    int free_gpus = 0;  // GetFullyFreeGpuNum (resource.go:170-177)
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) free_gpus += (g < cnt && gl[g] == kMilli) ? 1 : 0;
    const double num_idle = (double)free_gpus;
    const double num_working = (double)cnt - num_idle;
    gpu = (pw.gidle[gtype] * num_idle) + (pw.gfull[gtype] * num_working);
  }
  if (!((pw.cvalid >> cm) & 1u)) return false;
  const double real_cores = ceil((double)cap / (double)kMilli / 2);
  const double idle_cores = floor((double)cpuL / (double)kMilli / 2);
  const double working_cores = real_cores - idle_cores;
  const double nc = pw.cnc[cm];
  const double num_cpus = ceil(real_cores / nc);
  const double num_active = ceil(working_cores / nc);
  const double num_idle_cpus = num_cpus - num_active;
  const double cpu = (pw.cidle[cm] * num_idle_cpus) + (pw.cfull[cm] * num_active);
  *energy = cpu + gpu;  // pwr_score.go:147 old_CPU_energy + old_GPU_energy
  return true;
}

// GetEnergyConsumptionNode (resource.go:536-563) split into its CPU and GPU terms, for the per-event
// [Power] report (analysis.go:24-56 ClusterPowerConsumptionReport sums each over the nodes).  Same
// expressions as node_energy; false where the reference would fail (no energy model for the node's
// GPU model: a nil func call; an unknown CPU model).
KSIM_HD bool node_power(int cpuL, int cap, int cm, const int (&gl)[kMaxGpu], int cnt, int gtype, const PowerDev& pw,
                        double* cpu_w, double* gpu_w) {
  double gpu = 0;
  if (!((pw.gnone >> gtype) & 1u)) {
    if (!((pw.gvalid >> gtype) & 1u)) return false;
    int free_gpus = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) free_gpus += (g < cnt && gl[g] == kMilli) ? 1 : 0;
    const double num_idle = (double)free_gpus;
    const double num_working = (double)cnt - num_idle;
    gpu = (pw.gidle[gtype] * num_idle) + (pw.gfull[gtype] * num_working);
  }
  if (!((pw.cvalid >> cm) & 1u)) return false;
  const double real_cores = ceil((double)cap / (double)kMilli / 2);
  const double idle_cores = floor((double)cpuL / (double)kMilli / 2);
  const double working_cores = real_cores - idle_cores;
  const double nc = pw.cnc[cm];
  const double num_cpus = ceil(real_cores / nc);
  const double num_active = ceil(working_cores / nc);
  const double num_idle_cpus = num_cpus - num_active;
  *cpu_w = (pw.cidle[cm] * num_idle_cpus) + (pw.cfull[cm] * num_active);
  *gpu_w = gpu;
  return true;
}

// calculatePWRShareExtendScore (pwr_score.go:143-212): int64(old - new) energy; share pods try every
// fitting GPU (first, then strictly better; *gpu = its index), others take NodeResource.Sub
// (resource.go:454-480).  *err when the energy model fails.
KSIM_HD int pwr_score(const NodeV& n, const PodDev& p, int cap, int cm, const PowerDev& pw, int* gpu, bool* err) {
  int gl[kMaxGpu];
  unpack_gl(n, gl);
  const int cnt = n.gpu_cnt(), gt = n.gpu_type();
  double old_e = 0, new_e = 0;
  *gpu = -1;
  *err = !node_energy(n.cpu_left, cap, cm, gl, cnt, gt, pw, &old_e);
  if (*err) return 0;
  if (is_share_pod(p)) {
    int score = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      if (g < cnt && gl[g] >= p.milli) {
        int c[kMaxGpu];
#pragma unroll
        for (int h = 0; h < kMaxGpu; ++h) c[h] = gl[h] - (h == g ? (int)p.milli : 0);
        (void)node_energy(n.cpu_left - p.cpu_nz, cap, cm, c, cnt, gt, pw, &new_e);
        const int s = (int)(long long)(old_e - new_e);
        if (*gpu < 0 || s > score) { score = s; *gpu = g; }
      }
    }
    return score;
  }
  bool ok = false;
  int cpuL = n.cpu_left;
  const unsigned sm = sub_gpu_mask(gl, cnt, cpuL, p, &ok);
  if (ok) {
    cpuL -= p.cpu_nz;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g)
      if ((sm >> g) & 1u) gl[g] -= p.milli;
  }
  (void)node_energy(cpuL, cap, cm, gl, cnt, gt, pw, &new_e);
  return (int)(long long)(old_e - new_e);
}

// PWRScorePlugin.NormalizeScore (pwr_score.go:104-141)
KSIM_HD int pwr_normalize(int s, int lo, int hi) { return lo == hi ? 100 : (int)((long long)(s - lo) * 100 / (hi - lo)); }

// x / 125 correctly rounded for every integer-valued x with |x| < 2^31, without a division: the product
// with RN(1/125), its exact remainder by an fma, one fma correction.  Checked against IEEE division for
// every x in [0, 2^31) (tests/native/div125_check.c; the formula is odd in x); 3 fp64 operations instead
// of the ~11 of a division.  kMaxSpecCpu = 125 x 2^10 and kMaxSpecGpu = 125 x 2^6, and scaling by a power
// of two is exact, so x / kMaxSpec* = div125(x) x 2^-k bit for bit (const.go:16-18).
KSIM_HD double div125(double x) {
  const double r = 1.0 / 125.0;
  const double q = x * r;
  const double e = __builtin_fma(-q, 125.0, x);
  return __builtin_fma(e, r, q);
}
KSIM_HD double div_spec_cpu(double x) { return div125(x) * 0x1p-10; }  // x / kMaxSpecCpu, |x| < 2^31 integer
KSIM_HD double div_spec_gpu(double x) { return div125(x) * 0x1p-6; }   // x / kMaxSpecGpu, |x| < 2^31 integer
static_assert(kMaxSpecCpu == 125 * 1024 && kMaxSpecGpu == 125 * 64, "div_spec_* assume these");

// getBestFitScore (best_fit_score.go:66-97); -1 = error
KSIM_HD int bestfit_score(const NodeV& n, const PodDev& p, int total) {
  const double f0 = (double)n.cpu_left, r0 = (double)p.cpu_nz;
  const double f1 = (double)total, r1 = (double)((int)p.milli * (int)p.num);
  double s = 0;
  if (f0 < r0) return -1;
  s += div_spec_cpu(f0 - r0) * 0.5;  // (f0 - r0) / MaxSpecCpu: an integer in [0, 2^31)
  if (f1 < r1) return -1;
  s += div_spec_gpu(f1 - r1) * 0.5;
  s = (1.0 - s) * (double)100;
  return (int)s;
}

// DotProduct's GpuPluginCfg (config.go:3-55): dimExtMethod, normMethod; packed in ReplicaDev.dpcfg
enum : int { DIM_MERGE = 0, DIM_SHARE = 1, DIM_DIVIDE = 2, DIM_EXTEND = 3 };
enum : int { NORM_MAX = 0, NORM_NODE = 1, NORM_POD = 2 };
KSIM_HD int dp_dim(int cfg) { return cfg & 15; }
KSIM_HD int dp_norm(int cfg) { return (cfg >> 4) & 15; }

// One match group of calculateDotProductScore (dot_product_score.go:70-92): node (n0, n1) and pod
// (p0, p1) normalized by (c0, c1) (NormalizeVector, utils.go:1220-1236: / c, or 0 when c <= 0),
// CalculateVectorDotProduct in order (utils.go:1238-1248), / len(podVec), tanh(x / 10) for "pod",
// 1 - x; the group replaces the best when strictly larger (the first max keeps its GPU id).  The
// extend method's pod vectors are zero except at one GPU dimension, so their dot product is
// exactly n0 p0 + nj pj (adding +0.0 to a non-negative sum changes nothing): the same two terms.
KSIM_HD void dp_group(double n0, double n1, double p0, double p1, double c0, double c1, int len, int norm, int gid,
                      double* best, int* best_gid) {
  const double a0 = c0 > 0 ? n0 / c0 : 0, a1 = c1 > 0 ? n1 / c1 : 0;
  const double b0 = c0 > 0 ? p0 / c0 : 0, b1 = c1 > 0 ? p1 / c1 : 0;
  double cur = 0;
  cur += a0 * b0;
  cur += a1 * b1;
  if (cur == -1) return;
  cur /= (double)len;
  if (norm == NORM_POD) cur = go_tanh(cur / 10);
  cur = 1 - cur;
  if (*best < cur) {
    *best = cur;
    *best_gid = gid;
  }
}

// calculateDotProductScore for every dimExtMethod / normMethod (dot_product_score.go:64-100 over
// GenerateSchedulingMatchGroups, utils.go:1274-1342; ToVirtualNodeResourceList /
// ToVirtualPodResourceList / ToFormalizedGpuResourceList, resource.go:217-381).  cap: the node's
// MilliCpuCapacity (normMethod "node").  *gid: the best group's GpuId as a GPU mask (0 = "", the
// merge method's and no group's) -- allocateGpuIdBasedOnDotProduct (:102-107).
KSIM_HD int dotprod_cfg_score(const NodeV& n, const PodDev& p, int cap, int cfg, int* gid) {
  const int dim = dp_dim(cfg), norm = dp_norm(cfg);
  double best = -1;
  *gid = 0;
  const int cpuL = n.cpu_left, cpu = p.cpu_nz;  // MilliCpuLeft; PodResource.MilliCpu (non-zero default)
  const int req = (int)p.milli * (int)p.num;    // podMilliGpuReq / TotalMilliGpu
  const int cnt = n.gpu_cnt();
  if (cpuL >= cpu) {  // ToVirtualNodeResourceList: nil when the CPU left is short
    const int tot = n.total();
    int idle = 0, part = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      idle += (g < cnt && n.gl(g) == kMilli) ? 1 : 0;
      part += (g < cnt && n.gl(g) > 0 && n.gl(g) < kMilli) ? 1 : 0;
    }
    const int excl = req <= idle * kMilli ? exclusive_gpu_mask(n, p) : -1;  // AllocateExclusiveGpuId
    const double c0 = norm == NORM_NODE ? (double)cap : norm == NORM_POD ? (double)cpu : (double)kMaxSpecCpu;
    const double c1 = norm == NORM_NODE ? (double)(cnt * kMilli) : norm == NORM_POD ? (double)req : (double)kMaxSpecGpu;
    // extend: ToFormalizedGpuResourceList = the partly used GPUs (0 < left < 1000) in index order, then
    // one entry of all idle GPUs, and one pod vector per entry that holds the request (its length
    // 1 + entries); share / divide: a share pod on each partly used GPU that holds it (divide: the CPU
    // left scaled by that GPU's share of the GPU left), then the idle GPUs; merge: one group.
    // Candidates j = 0..7 are GPU j, j = 8 the idle group (merge: j = 8 is the merged node).
    const int len = dim == DIM_EXTEND ? 1 + part + (idle > 0 ? 1 : 0) : 2;
    // GPU j's milli left is the low half of w0 at iteration j (the words shift down by 16 bits per
    // iteration: a runtime index into the packed words would put them in scratch)
    uint32_t w0 = n.g[0], w1 = n.g[1], w2 = n.g[2], w3 = n.g[3];
#pragma unroll 1
    for (int j = (dim == DIM_MERGE ? kMaxGpu : 0); j <= kMaxGpu; ++j) {
      bool use;
      int v1, g_id;
      if (j < kMaxGpu) {
        const int l = (int)(w0 & 0xffffu);
        w0 = (w0 >> 16) | (w1 << 16);
        w1 = (w1 >> 16) | (w2 << 16);
        w2 = (w2 >> 16) | (w3 << 16);
        w3 >>= 16;
        use = j < cnt && l < kMilli && l >= req && (dim == DIM_EXTEND ? l > 0 : req < kMilli);
        v1 = l;
        g_id = 1 << j;
      } else if (dim == DIM_MERGE) {
        use = true;
        v1 = tot;
        g_id = 0;
      } else {
        use = dim == DIM_EXTEND ? (idle > 0 && idle * kMilli >= req) : req <= idle * kMilli;
        v1 = idle * kMilli;
        g_id = excl;
      }
      if (!use) continue;
      const double v0 = dim == DIM_DIVIDE ? (double)((long long)cpuL * v1) / (double)tot : (double)cpuL;
      dp_group(v0, (double)v1, (double)cpu, (double)req, c0, c1, len, norm, g_id, &best, gid);
    }
  }
  if (best == -1) {
    *gid = 0;
    return 0;
  }
  return (int)((double)100 * best);
}

// The paper's configuration (merge / max) in closed form: one match group, the same operations as
// dotprod_cfg_score's (the fast path of the scanning kernels; tests check the two agree).
KSIM_HD int dotprod_merge_max(const NodeV& n, const PodDev& p) {
  if (n.cpu_left < p.cpu_nz) return 0;
  // the quotients by div_spec_* (integers below 2^31: the same bits as the divisions)
  const double a0 = div_spec_cpu((double)n.cpu_left);
  const double a1 = div_spec_gpu((double)n.total());
  const double c0 = div_spec_cpu((double)p.cpu_nz);
  const double c1 = div_spec_gpu((double)((int)p.milli * (int)p.num));
  double cur = 0;
  cur += a0 * c0;
  cur += a1 * c1;
  cur /= (double)2;
  cur = 1 - cur;
  return (int)((double)100 * cur);
}

// getPackingScore (gpu_packing_score.go:71-117); *err on allocation failure
KSIM_HD int packing_score(const NodeV& n, const PodDev& p, bool* err) {
  *err = false;
  const int cnt = n.gpu_cnt();
  const int ff = n.gl_full();
  if (ff == cnt) {
    const int s = 100 / 3 - ff;
    return s > ff ? s : ff;
  }
  // The two request shapes of the traces in closed form over the packed lanes (the loop below is the general one):
  if (p.milli == kMilli && p.num >= 1) {  // num whole GPUs: each pick is a full GPU (the least milli >= 1000): ffuse = num
    if (ff < p.num) {
      *err = true;
      return 0;
    }
    const int s = 100 / 2 - p.num;
    return s > 100 / 3 ? s : 100 / 3;
  }
  if (p.num == 1) {  // one share: the least milli left >= p.milli (lanes below it, and the absent ones, map high)
    const NodeV::u16x2 k = {(unsigned short)(0x8000 - p.milli), (unsigned short)(0x8000 - p.milli)};
    const NodeV::u16x2 f = {(unsigned short)0x8000, (unsigned short)0x8000};
    auto w = [&](uint32_t x) { return (NodeV::pk(x) + k) ^ f; };  // gl - milli if gl >= milli, else >= 0x8000
    const NodeV::u16x2 m = __builtin_elementwise_min(__builtin_elementwise_min(w(n.g[0]), w(n.g[1])),
                                                     __builtin_elementwise_min(w(n.g[2]), w(n.g[3])));
    const int d = m.x < m.y ? (int)m.x : (int)m.y;
    if (d > kMilli) {
      *err = true;
      return 0;
    }
    const int bv = d + p.milli;
    if (bv == kMilli) return 100 / 2 - 1 > 100 / 3 ? 100 / 2 - 1 : 100 / 3;
    const int s = 100 - (bv * 100 / kMilli) / 10;
    return s > 100 / 2 ? s : 100 / 2;
  }
  unsigned taken = 0u;
  int ffuse = 0, req = p.num, r = 0;
  for (int k = 0; k < kMaxGpu && req > 0; ++k) {
    int best = -1, bv = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      const int v = n.gl(g);
      const bool cand = g < cnt && !((taken >> g) & 1u) && v >= p.milli;
      if (cand && (best < 0 || v < bv)) { best = g; bv = v; }
    }
    if (best < 0) break;
    taken |= 1u << best;
    --req;
    if (bv == kMilli) ++ffuse;
    r += bv * 100 / kMilli;
  }
  if (req != 0) {
    *err = true;
    return 0;
  }
  if (ffuse > 0) {
    const int s = 100 / 2 - ffuse;
    return s > 100 / 3 ? s : 100 / 3;
  }
  const int s = 100 - r / 10;
  return s > 100 / 2 ? s : 100 / 2;
}

// GpuClusteringScorePlugin.Score (gpu_clustering_score.go:32-56)
KSIM_HD int clustering_score(const uint16_t* tags, int pod_tag, int total) {
  if (pod_tag < 0) return 0;
  int distinct = 0;
#pragma unroll
  for (int k = 0; k < kNumTags; ++k) distinct += tags[k] > 0 ? 1 : 0;
  const int base = (100 / 4) * (kMaxSpecGpu - total) / kMaxSpecGpu;
  if (tags[pod_tag] > 0) return distinct == 1 ? base + 100 * 3 / 4 : base + 100 * 2 / 4;
  return distinct == 0 ? base + 100 / 4 : base;
}

// clustering_score on a node whose non-zero tag counts are the bits of `m` (bit k: tags[k] > 0): the
// score reads nothing else of the counts, so on a create-only stream (counts only grow) a presence mask
// per node is all a scan needs (k_scan1)
KSIM_HD int clustering_score_mask(unsigned m, int pod_tag, int total) {
  if (pod_tag < 0) return 0;
  const int distinct = __builtin_popcount(m & ((1u << kNumTags) - 1u));
  const int base = (100 / 4) * (kMaxSpecGpu - total) / kMaxSpecGpu;
  if ((m >> pod_tag) & 1u) return distinct == 1 ? base + 100 * 3 / 4 : base + 100 * 2 / 4;
  return distinct == 0 ? base + 100 / 4 : base;
}

// Random contract: splitmix64 finaliser.
KSIM_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}
KSIM_HD uint64_t rand_node_key(uint64_t seed, int step, uint32_t rank) {
  return mix64(mix64(seed ^ 0xA0761D6478BD642FULL) ^ (((uint64_t)(uint32_t)step << 32) | rank));
}
KSIM_HD uint64_t rand_gpu_key(uint64_t node_key, int g) { return mix64(node_key ^ (uint64_t)(0x100 + g)); }

// Packed argmax key: [63:40] score (24 b) | [39:16] ~name_rank (24 b) | [15:12] gpu index + 1 |
// [11:0] the node's slot in its workgroup slice (k_replay; 0 elsewhere).  Ranks are unique,
// so max over keys = max score, ties to the byte-wise smallest name (selectHost).
KSIM_HD unsigned long long pack_key(unsigned score, uint32_t rank, int gpu, int loc = 0) {
  return ((unsigned long long)(score & 0xFFFFFFu) << 40) | ((unsigned long long)((0xFFFFFFu - rank) & 0xFFFFFFu) << 16) |
         ((unsigned long long)((gpu + 1) & 0xF) << 12) | (unsigned long long)(loc & 0xFFF);
}
KSIM_HD int key_score(unsigned long long k) { return (int)(k >> 40); }
KSIM_HD uint32_t key_rank(unsigned long long k) { return 0xFFFFFFu - (uint32_t)((k >> 16) & 0xFFFFFFu); }
KSIM_HD int key_gpu(unsigned long long k) { return (int)((k >> 12) & 0xFu) - 1; }
KSIM_HD int key_loc(unsigned long long k) { return (int)(k & 0xFFFu); }
constexpr int kMaxRank = 0xFFFFFF;  // name ranks must stay below (N < 2^24)
// BestFit's raw score leaves [0, 100] downwards on a node with more CPU left than MaxSpecCpu, and only -1 is a
// Score error (best_fit_score.go:48-51,76-96).  Its raw scores travel biased by kBfKeyBias (> -2^23 for CPU below
// 2^31), so the key field and the min / max accumulators see non-negative values.  NormalizeScore maps only the
// max raw score to 100 whatever the range (plugin_utils.go:48-74), so the raw argmax is the normalized one.
constexpr int kBfKeyBias = 1 << 23;
constexpr int kMaxSlice = 0xFFF;    // slots per k_replay workgroup

}  // namespace ksim

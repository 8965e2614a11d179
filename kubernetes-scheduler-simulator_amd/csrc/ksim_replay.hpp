// ksim_replay.hpp -- persistent whole-trace replay kernel (k_replay).
//
// One launch replays every replica to completion (1024-thread workgroups).  Replica r is owned by K
// co-resident workgroups; workgroup w keeps the node records of its slice
// [w*S, min(N,(w+1)*S)) in LDS for the whole run, so the per-pod loop touches
// no node record in HBM.  Per pod step:
// Pipelining: a Bind changes ONE node, and the only node of a slice that can win a
// step is the slice's own best.  So right after publishing step s a workgroup
// evaluates pod s+1 on its slice with its step-s best node b excluded from the
// aggregate, evaluating b twice: as it is (pre) and in the virtual slot with step
// s's Bind applied (post).  When step s's exchange completes it commits (owner ->
// the virtual slot becomes b) and combines the aggregate with post (owner) or pre
// (everyone else) -- the exchange latency overlaps the next step's Filter+Score.
// Per pod step:
//   1. Filter + Score of the slice on LDS records.  FGD: eight lanes per node,
//      lane g owning GPU g -- Filter, the candidate placements (one per distinct
//      milli-left value among the fitting GPUs) and the final sigmoid scores are
//      per-lane; the work list is compacted with ballot + mbcnt.  F of the node's current
//      state is cached per node in LDS (it does not depend on the pod; a Bind or a
//      delete invalidates it), and every candidate state is evaluated by a QUAD of
//      lanes -- lane q classifies typical pod tb+q, then the quad folds the four
//      (bin, value) pairs in typical-pod order with lane q owning bin q, so every
//      bin stays the reference's sequential fp64 sum;
//   2. the workgroup publishes its best packed key and its counters as three
//      8-byte {tag = step+1, value} granules (agent-scope relaxed stores);
//   3. one wave polls the replica's 3K granules (agent-scope relaxed loads)
//      until every tag equals step+1, then every workgroup reduces the same K
//      values to the same winner -- an all-gather with no fence and no second
//      phase (MI355X_MICROARCH.md "granule" hand-off, R2 form);
//   4. the workgroup owning the winner runs Reserve's GPU selector and applies
//      the Bind scatter to its LDS record, and writes the result.
// Granule slots alternate by step parity: a workgroup can only publish step
// s+2 after every workgroup has published s+1, which each does only after
// reading step s.  Every spin is bounded; a timeout sets *fail and ends the
// replica's loop on every workgroup.
#pragma once

namespace ksim_replay {

using namespace ksim;

constexpr int kRBlock = 1024;
constexpr int kRWaves = kRBlock / 64;
constexpr int kChunk = kRBlock;      // nodes per chunk, one lane per node (non-FGD policies)
constexpr int kFChunk = kRBlock / 8; // nodes per chunk, 8 lanes per node -- lane g <-> GPU g (FGD)
constexpr int kRMaxCand = 9;         // FGD items per node: stale current state + up to 8 candidates
constexpr int kMaxK = 256;         // workgroups per replica (<= 64: one granule column per polling lane)
constexpr int kGran = 3;           // granules per workgroup per step (the key exchange)
constexpr int kGranW = 10;         // granule words per workgroup per parity: key round 0-2; PWR+FGD's round 0-6, its miss round 7-8
constexpr int kPfGuess = 256;      // PWR+FGD: entries of the guessed-range table (class id mod 256)
constexpr unsigned kSpinLimit = 1u << 22;  // ~seconds: only a non-resident workgroup can stall a poll
constexpr int kEvBuf = 128;        // events staged in LDS per refill (4 KB)

struct ReplayArgs {
  ReplicaDev* reps;
  const int* rep_list;  // replica of each group of K workgroups (one policy per launch)
  int N;
  int K;            // workgroups per replica
  int S;            // slice size (nodes per workgroup)
  unsigned long long* gran;  // [launch replica][2][K][kGranW]
  int2* hist;       // [R][K][hist_stride]: (node, mask+1) of pods this workgroup bound
  int hist_stride;
  int* fail;
  unsigned long long* prof;  // optional [R*K][8] s_memrealtime phase sums (KSIM_PROFILE=1), else null
  int skip;                  // the dead-class skip (create-only streams; class ids < 1024)
  int pm_c;                  // PWR+FGD: class stride of the per-(class, slot) memo in LDS, 0 = no memo
  unsigned pm_ver0;          // the slots' first version (KSIM_TEST pf_memo_ver0: tests start near the wrap)
  int pf_guess;              // PWR+FGD: learn each class's ranges (KSIM_TEST pf_guess=0: never -- every scored step misses)
  // A node-sharded group in one launch (ksim_shard_group_run, lean cheap policies): rep_list / reps name one
  // replica per shard, a.K slices each; xK = every shard's slices together, the exchange's columns (0: a.K, one
  // replica's), and results carry global name ranks -- the owner of the winner reports, every other shard's
  // first workgroup names the winner (ksim.shard.merge_results)
  int xK;
  int group;
};
constexpr int kProfPhases = 12;  // 0-7 phases, 8 poll spins, 10 core cycles, 11 wall ticks

// Per-workgroup state at the start of the dynamic LDS region (16-B aligned); after it, only what the
// launch's policy reads (replay_layout): the FGD evaluation scratch, NodeRec nodes[S+1], u16
// tags[S+1][16] (GpuClustering; the other policies keep the tag counts in HBM), double F0[S+1]
// (FGD: cached F of the current state, < 0 = stale), double E0[S+1] + int2 pe[S+1] (PWR: cached
// energy, static energy terms), i32 last[S+1] (cluster report), i32 praw[S+1] + i32 pinf[S+1]
// (PWR+FGD: the raw PWR score and packed FGD score / GPU choices of every slot, two steps' worth) + int4
// gtab[kPfGuess] (PWR+FGD: each class's two most recent cluster-wide raw PWR ranges).  A lean
// BestFit / DotProd / GpuPacking / Random workgroup of C2 / C4 is about 44 KB, so several share a
// CU.  Slot ns (one past the slice) is the VIRTUAL node: the pending step's local best node with
// that step's Bind already applied (see the pipelining note).
struct __align__(16) ReplayShared {
  PodDev ev[kEvBuf];
  // the step's local aggregate (LDS atomics), the pending best node b and the virtual node excluded
  unsigned long long agg_key;
  unsigned long long agg_key1, agg_pad;  // PWR+FGD: the slice's key under the class's second guessed range
  int agg_cnt, agg_err, agg_lo, agg_hi;
  // the excluded real node (pre-Bind) and the virtual node (post-Bind) of the current step
  unsigned long long pre_key, post_key;
  int pre_feas, pre_err, post_feas, post_err;
  // the pending exchange as the other waves need it (wave 0 keeps the rest in registers)
  int pend_valid, pend_b;
  int stop;
  int nitems;                   // FGD work-list length of the current chunk
  int pf_redo;                  // PWR+FGD: this workgroup re-evaluates the step (its winner was not the virtual node)
  int pad0, pad1;
  unsigned long long prof[kProfPhases];  // KSIM_PROFILE phase sums (thread 0)
  unsigned long long prof_pad[4];
  // PWR+FGD, the pending step (kept here, not in wave 0's registers): its pod, the class's guessed ranges
  // {lo0, hi0, lo1, hi1} and this slice's key under the second one
  PodDev pf_pod;
  int4 pf_g;
  unsigned long long pf_key1, pf_pad2;
  PowerDev pw;                  // PWR policies: the replica's energy model
  unsigned dead[32];            // classes with no feasible node (create-only streams: for good)
};
static_assert(sizeof(ReplayShared) % 16 == 0, "keep the node records 16-B aligned");

// FGD evaluation scratch (FGD, PWR+FGD launches only).
struct __align__(16) ReplayFgd {
  TypDev tp[kMaxTypical];  // the replica's typical table (per-lane reads in the quad evaluator)
  double F[kFChunk * kRMaxCand];
  uint16_t item_node[kFChunk * kRMaxCand];
  uint8_t item_code[kFChunk * kRMaxCand];
  uint8_t pad_[(16 - (kFChunk * kRMaxCand * 3) % 16) % 16];
};
static_assert(sizeof(ReplayFgd) % 16 == 0, "keep the node records 16-B aligned");

// The dynamic LDS layout of one k_replay workgroup (host and device).
struct RLayout {
  size_t fgd, nodes, tags, F0, E0, pe, last, praw, pinf, gtab, pver, pm, total;
};
// pm_c > 0 (PWR+FGD): u32 pver[S+1] (each slot's state version) and uint2 pm[pm_c][S] (every class's
// memoised Filter + Score of every real slot, valid while its version matches; pf_memo_* below)
__host__ __device__ inline RLayout replay_layout(int S, int pol, bool general, int pm_c = 0) {
  const bool tags = pol == POL_CLUSTERING, fgd = pol == POL_FGD || pol == POL_PWR_FGD;
  const bool pwr = pol == POL_PWR || pol == POL_PWR_FGD, pf = pol == POL_PWR_FGD;
  const size_t S1 = (size_t)S + 1;
  RLayout L;
  size_t o = sizeof(ReplayShared);
  L.fgd = o;   o += fgd ? sizeof(ReplayFgd) : 0;
  L.nodes = o; o += S1 * sizeof(NodeRec);
  L.tags = o;  o += tags ? S1 * kTagStride * sizeof(uint16_t) : 0;
  L.F0 = o;    o += fgd ? S1 * sizeof(double) : 0;
  L.E0 = o;    o += pwr ? S1 * sizeof(double) : 0;
  L.pe = o;    o += pwr ? S1 * sizeof(int2) : 0;
  L.last = o;  o += general ? S1 * sizeof(int) : 0;
  L.praw = o;  o += pf ? 2 * S1 * sizeof(int) : 0;  // by step parity: the pending step's stays intact
  L.pinf = o;  o += pf ? 2 * S1 * sizeof(int) : 0;
  o = (o + 15) / 16 * 16;
  L.gtab = o;  o += pf ? kPfGuess * sizeof(int4) : 0;
  L.pver = o;  o += (pf && pm_c > 0) ? (S1 * sizeof(unsigned) + 15) / 16 * 16 : 0;
  L.pm = o;    o += (pf && pm_c > 0) ? (size_t)pm_c * S * sizeof(uint2) : 0;
  L.total = o;
  return L;
}

// PWR+FGD memo entry of one (class, slot): x = the raw PWR score, y = the packed FGD score / GPU choices
// (pinf's low 16 bits), Filter's verdict (16), the Score error (17) and the slot version it was computed
// at (18-31; kPmInvalid: never).  A slot's version advances whenever its node record changes.
constexpr unsigned kPmInvalid = 0x3fffu;
__device__ __forceinline__ bool pf_memo_hit(const uint2& e, unsigned ver) { return (e.y >> 18) == ver; }
__device__ __forceinline__ uint2 pf_memo_pack(int praw, int pinf, unsigned ver) {
  return make_uint2((unsigned)praw, ((unsigned)pinf & 0xffffu) | ((pinf & (1 << 30)) ? 1u << 16 : 0u) |
                                        ((pinf & (1 << 29)) ? 1u << 17 : 0u) | (ver << 18));
}
__device__ __forceinline__ int pf_memo_pinf(const uint2& e) {  // back to pinf's layout (kPfFeas 30, kPfErr 29)
  return (int)((e.y & 0xffffu) | ((e.y >> 16) & 1u) << 30 | ((e.y >> 17) & 1u) << 29);
}

__device__ __forceinline__ unsigned long long gload(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- wave reductions over all 64 lanes with DPP row ops + 4 readlanes (call with every lane active) ----
template <int kCtrl>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, kCtrl, 0xF, 0xF, false);
}
template <int kCtrl>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v) {
  const int lo = dpp_i<kCtrl>((int)(unsigned)v), hi = dpp_i<kCtrl>((int)(unsigned)(v >> 32));
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror: every lane of a
// 16-lane row ends with the row's reduction; the four rows are then combined uniformly.
__device__ __forceinline__ unsigned long long wave_max_u64_dpp(unsigned long long v) {
  unsigned long long w;
  w = dpp_u64<0xB1>(v); v = w > v ? w : v;
  w = dpp_u64<0x4E>(v); v = w > v ? w : v;
  w = dpp_u64<0x141>(v); v = w > v ? w : v;
  w = dpp_u64<0x140>(v); v = w > v ? w : v;
  const unsigned long long a = readlane_u64(v, 0), b = readlane_u64(v, 16), c = readlane_u64(v, 32),
                           d = readlane_u64(v, 48);
  const unsigned long long x = a > b ? a : b, y = c > d ? c : d;
  return x > y ? x : y;
}
__device__ __forceinline__ int wave_sum_dpp(int v) {
  v += dpp_i<0xB1>(v);
  v += dpp_i<0x4E>(v);
  v += dpp_i<0x141>(v);
  v += dpp_i<0x140>(v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ int wave_min_dpp(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  v = min(v, dpp_i<0x141>(v));
  v = min(v, dpp_i<0x140>(v));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ int wave_max_dpp(int v) {
  v = max(v, dpp_i<0xB1>(v));
  v = max(v, dpp_i<0x4E>(v));
  v = max(v, dpp_i<0x141>(v));
  v = max(v, dpp_i<0x140>(v));
  return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// Max over each group of 8 lanes (8k .. 8k+7): xor 1, xor 2, then row_half_mirror.
__device__ __forceinline__ int group8_max(int v) {
  v = max(v, dpp_i<0xB1>(v));
  v = max(v, dpp_i<0x4E>(v));
  v = max(v, dpp_i<0x141>(v));
  return v;
}

// milli left on GPU g (0..7, lane-varying) without dynamic register indexing.
__device__ __forceinline__ int gl_dyn(const NodeV& n, int g) {
  const uint32_t w01 = (g & 2) ? n.g[1] : n.g[0];
  const uint32_t w23 = (g & 2) ? n.g[3] : n.g[2];
  const uint32_t w = (g & 4) ? w23 : w01;
  return (int)((g & 1) ? (w >> 16) : (w & 0xffffu));
}

// Bit h set iff GPU h has exactly v milli left.
__device__ __forceinline__ unsigned gl_equal_mask(const NodeV& n, int v) {
  const uint32_t vv = (uint32_t)v * 0x10001u;
  unsigned m = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = n.g[i] ^ vv;
    m |= ((x & 0xffffu) == 0u ? 1u : 0u) << (2 * i);
    m |= ((x >> 16) == 0u ? 1u : 0u) << (2 * i + 1);
  }
  return m;
}

// An LDS-staged event as wave-uniform values (readfirstlane keeps it in SGPRs).
__device__ __forceinline__ PodDev uniform_pod(const PodDev* s) {
  const uint4* q = reinterpret_cast<const uint4*>(s);
  uint4 x = q[0], y = q[1];
  x.x = __builtin_amdgcn_readfirstlane(x.x); x.y = __builtin_amdgcn_readfirstlane(x.y);
  x.z = __builtin_amdgcn_readfirstlane(x.z); x.w = __builtin_amdgcn_readfirstlane(x.w);
  y.x = __builtin_amdgcn_readfirstlane(y.x); y.y = __builtin_amdgcn_readfirstlane(y.y);
  y.z = __builtin_amdgcn_readfirstlane(y.z); y.w = __builtin_amdgcn_readfirstlane(y.w);
  PodDev p;
  uint4* o = reinterpret_cast<uint4*>(&p);
  o[0] = x;
  o[1] = y;
  return p;
}

// An LDS node record as wave-uniform values.
__device__ __forceinline__ NodeV uniform_node(const NodeRec* s) {
  NodeV n = load_node(s);
  n.cpu_left = __builtin_amdgcn_readfirstlane(n.cpu_left);
  n.mem_left = __builtin_amdgcn_readfirstlane(n.mem_left);
#pragma unroll
  for (int i = 0; i < 4; ++i) n.g[i] = __builtin_amdgcn_readfirstlane(n.g[i]);
  n.meta = __builtin_amdgcn_readfirstlane(n.meta);
  n.name_rank = __builtin_amdgcn_readfirstlane(n.name_rank);
  return n;
}

// ---- quad (4-lane) broadcasts: every lane of a quad gets lane J's value ----
template <int J>
__device__ __forceinline__ int qbc(int v) {
  return __builtin_amdgcn_mov_dpp(v, J * 0x55, 0xF, 0xF, true);
}
template <int J>
__device__ __forceinline__ double qbc_d(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)qbc<J>((int)(unsigned)u), hi = (unsigned)qbc<J>((int)(unsigned)(u >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// 1.0 or +0.0 from a flag: the high word selected, the low word a constant 0 (one v_cndmask)
__device__ __forceinline__ double sel01(bool f) {
  return __builtin_bit_cast(double, (unsigned long long)(f ? 0x3FF00000u : 0u) << 32);
}

// Candidate state of `code` on node m: 0 current, 1..8 share pod on GPU code-1
// (fgd_score.go:111-118), 9 NodeResource.Sub (fgd_score.go:137-141, resource.go:454-480).
// g: packed u16 milli-left per GPU; *total: GetGpuMilliLeftTotal of the state.
__device__ __forceinline__ void fgd_candidate(const NodeV& m, int code, const PodDev& p, int* cpuL,
                                              uint32_t (&g)[4], int* total) {
  *cpuL = m.cpu_left;
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = m.g[i];
  unsigned mask = 0u;
  if (code >= 1 && code <= 8) {
    mask = 1u << (code - 1);
  } else if (code == 9) {
    int gl[kMaxGpu];
    unpack_gl(m, gl);
    bool ok = false;
    mask = sub_gpu_mask(gl, m.gpu_cnt(), *cpuL, p, &ok);
    if (!ok) mask = 0u;
    if (ok) *cpuL -= p.cpu_nz;
  }
  if (code >= 1 && code <= 8) *cpuL -= p.cpu_nz;
  const uint32_t d = (uint32_t)(uint16_t)p.milli;
#pragma unroll
  for (int i = 0; i < 4; ++i)  // u16 lanes never borrow: a selected GPU has left >= milli
    g[i] -= (((mask >> (2 * i)) & 1u) ? d : 0u) + (((mask >> (2 * i + 1)) & 1u) ? (d << 16) : 0u);
  uint32_t t = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) t = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, g[i]), (u16x2){1, 1}, t, false);
  *total = (int)t;
}

// F = NodeGpuShareFragAmountScore of one state (frag.go:148-203, 411-418, 460-493),
// evaluated by the 4 lanes of a quad (q = lane & 3); every lane returns the same F.
//   Rounds of four typical pods: lane q classifies t = tb+q from the LDS table `ltp`, the
//   quad then folds t = tb..tb+3 in order (DPP quad broadcasts) and lane q keeps bin q.
//   CPU-only typical pods [0, ncpu): lane 0 keeps XL, lane 1 XR.
//   GPU typical pods [ncpu, nt): cnt / frag over the 8 packed GPUs with v_pk_sub_i16 +
//     v_pk_lshrrev_b16 + v_dot2_u32_u16, bins 0 = Q1, 1 = Q2 + Q3's frag part, 2 = Q4,
//     3 = NA; two rounds per loop iteration, so both rounds' LDS loads are in flight at once.
//   `tp` (the global copy of the table) is unused.
// Every bin is the same sequence of fp64 adds as frag_F's (adding +0.0 for the
// typical pods that do not touch it), so F is bit-identical.
template <bool kTyped>
__device__ __forceinline__ double frag_F_quad(int cpuL, const uint32_t (&g)[4], int total, uint32_t typebit,
                                              const TypDev* __restrict__ tp, const TypDev* ltp, int ncpu, int nt,
                                              int q) {
  (void)tp;
  const double dtot = (double)total;
  // CPU-only typical pods, four per round like the GPU ones below: lane q classifies t = tb+q from
  // the LDS table, the quad folds the round in order, lane 0 keeps XL and lane 1 XR
  double bc = 0.0;
  for (int tb = 0; tb < ncpu; tb += 4) {
    const int t = min(tb + q, max(nt - 1, 0));
    const double x = ltp[t].freq * dtot;  // freq * float64(gpuMilliLeftTotal)
    int code = cpuL >= ltp[t].cpu ? 0 : 1;
    code = tb + q < ncpu ? code : 4;
    int cj;
    double vj;
    cj = qbc<0>(code); vj = qbc_d<0>(x); bc = __builtin_fma(vj, sel01(cj == q), bc);
    cj = qbc<1>(code); vj = qbc_d<1>(x); bc = __builtin_fma(vj, sel01(cj == q), bc);
    cj = qbc<2>(code); vj = qbc_d<2>(x); bc = __builtin_fma(vj, sel01(cj == q), bc);
    cj = qbc<3>(code); vj = qbc_d<3>(x); bc = __builtin_fma(vj, sel01(cj == q), bc);
  }
  double bg = 0.0;
  // two rounds per iteration: both rounds' table entries are loaded before the first is classified
  const int tmax = max(nt - 1, 0);
  for (int tb0 = ncpu; tb0 < nt; tb0 += 8) {
    const TypDev e2[2] = {ltp[min(tb0 + q, tmax)], ltp[min(tb0 + 4 + q, tmax)]};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int tb = tb0 + 4 * h;
      const TypDev e = e2[h];
      const uint32_t mp = (uint32_t)e.milli * 0x10001u;
      uint32_t frag = 0u, nlt = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u16x2 gv = __builtin_bit_cast(u16x2, g[i]);
        const u16x2 lt = (u16x2)(gv - __builtin_bit_cast(u16x2, mp)) >> (u16x2){15, 15};  // left < milli
        frag = __builtin_amdgcn_udot2(gv, lt, frag, false);  // GetGpuFragMilliByNodeResAndPodRes (frag.go:205-213)
        nlt = __builtin_amdgcn_udot2(lt, (u16x2){1, 1}, nlt, false);
      }
      const bool gpu_ok = kMaxGpu - (int)nlt >= e.num_eff;  // CanNodeHostPodOnGpuMemory (frag.go:447-458)
      const bool cpu_ok = cpuL >= e.cpu;
      const bool acc = !kTyped || (e.tmask & typebit) != 0u;  // IsNodeAccessibleToPod (utils.go:957-1006)
      const double x = e.freq * dtot;
      const double y = e.freq * (double)(int)frag;           // freq * float64(gpuFragMilli)
      int code = acc ? (cpu_ok ? 1 : (gpu_ok ? 2 : 0)) : 3;
      code = tb + q < nt ? code : 4;
      const double v = (acc && cpu_ok && gpu_ok) ? y : x;
      // bin q += (cj == q) ? vj : 0.0 as one fma with a 0 / 1 selector: vj * 1.0 and vj * 0.0 = +0.0 are exact
      // (vj finite, >= 0), so fma(vj, sel, bin) rounds exactly as the add does, with one instruction less per
      // typical pod than selecting both halves of vj (the fold's issue count bounds the large tables)
      double vj;
      int cj;
      cj = qbc<0>(code); vj = qbc_d<0>(v); bg = __builtin_fma(vj, sel01(cj == q), bg);
      cj = qbc<1>(code); vj = qbc_d<1>(v); bg = __builtin_fma(vj, sel01(cj == q), bg);
      cj = qbc<2>(code); vj = qbc_d<2>(v); bg = __builtin_fma(vj, sel01(cj == q), bg);
      cj = qbc<3>(code); vj = qbc_d<3>(v); bg = __builtin_fma(vj, sel01(cj == q), bg);
    }
  }
  const double b0 = qbc_d<0>(bg), b1 = qbc_d<1>(bg), b3 = qbc_d<2>(bg), b6 = qbc_d<3>(bg);
  const double b4 = qbc_d<0>(bc), b5 = qbc_d<1>(bc);
  double out = 0.0;
  out += b0;
  out += b1;
  out += b3;
  out += b4;
  out += b5;
  out += b6;
  return out;
}

// getEnergyConsumptionNode (pwr_score.go:147) with the node's static terms precomputed:
// rc = ceil(MilliCpuCapacity / 1000 / 2) and ncpus = ceil(rc / cores per CPU) are integer-valued
// doubles computed by the same expressions as node_energy's, so the energy is bit-identical.
__device__ __forceinline__ bool energy_rc(int cpuL, double rc, double ncpus, int cm, int free_gpus, int cnt, int gt,
                                          const PowerDev& pw, double* energy) {
  double gpu = 0;
  if (!((pw.gnone >> gt) & 1u)) {
    if (!((pw.gvalid >> gt) & 1u)) return false;
    const double num_idle = (double)free_gpus;
    const double num_working = (double)cnt - num_idle;
    gpu = (pw.gidle[gt] * num_idle) + (pw.gfull[gt] * num_working);
  }
  if (!((pw.cvalid >> cm) & 1u)) return false;
  const double idle_cores = floor((double)cpuL / (double)kMilli / 2);
  const double working_cores = rc - idle_cores;
  const double num_active = ceil(working_cores / pw.cnc[cm]);
  const double num_idle_cpus = ncpus - num_active;
  const double cpu = (pw.cidle[cm] * num_idle_cpus) + (pw.cfull[cm] * num_active);
  *energy = cpu + gpu;
  return true;
}

// The static terms of a node (host of energy_rc): {rc, ncpus << 3 | cpu model}.
__device__ __forceinline__ int2 energy_static(int cap, int cm, const PowerDev& pw) {
  const double rc = ceil((double)cap / (double)kMilli / 2);
  const double nc = ((pw.cvalid >> cm) & 1u) ? ceil(rc / pw.cnc[cm]) : 0.0;
  return make_int2((int)rc, (int)nc << 3 | cm);
}

// Fully free GPUs (GetFullyFreeGpuNum, resource.go:170-177) of packed milli-left words, GPU `g`
// reduced by `d` first (g < 0: none), or the GPUs of `sub` reduced by `d`.
__device__ __forceinline__ int free_gpus_after(const NodeV& n, int cnt, unsigned sub, int d) {
  int f = 0;
#pragma unroll
  for (int h = 0; h < kMaxGpu; ++h) {
    const int v = (int)((n.g[h >> 1] >> (16 * (h & 1))) & 0xffffu) - (((sub >> h) & 1u) ? d : 0);
    f += (h < cnt && v == kMilli) ? 1 : 0;
  }
  return f;
}

// PWR score of a node by the 8 lanes of its group (lane g <-> GPU g), first half: lane g's packed
// candidate (calculatePWRShareExtendScore, pwr_score.go:143-212).  Share pods: lane g evaluates the
// pod on GPU g when it fits, v = (score + kBias) << 4 | (14 - g), so the group max (pwr8_finish,
// after a uniform group8_max) is the first GPU reaching the max score, as the sequential loop keeps
// it.  Other pods: the NodeResource.Sub state on every lane (v carries the score, GPU none).
// old_e: the node's current energy (cached per slot; kEnergyErr when the model fails -> *err).
// *ovf: a score outside the packed range.
constexpr int kPwrVBias = 1 << 23;
constexpr double kEnergyStale = -1.0, kEnergyErr = -2.0;
__device__ __forceinline__ double node_energy_now(const NodeV& n, int2 pe, const PowerDev& pw) {
  double e = 0;
  const int cnt = n.gpu_cnt();
  if (!energy_rc(n.cpu_left, (double)pe.x, (double)(pe.y >> 3), pe.y & 7, free_gpus_after(n, cnt, 0u, 0), cnt,
                 n.gpu_type(), pw, &e))
    return kEnergyErr;
  return e;
}
__device__ __forceinline__ int pwr_cand8(const NodeV& n, const PodDev& p, int2 pe, double old_e, const PowerDev& pw,
                                         int g, bool* err, bool* ovf) {
  const int cnt = n.gpu_cnt(), gt = n.gpu_type(), cm = pe.y & 7;
  const double rc = (double)pe.x, ncpus = (double)(pe.y >> 3);
  double new_e = 0;
  *ovf = false;
  *err = old_e == kEnergyErr;
  if (*err) return -1;
  int s = 0, gsel = 15;
  if (is_share_pod(p)) {
    if (!(g < cnt && gl_dyn(n, g) >= p.milli)) return -1;
    (void)energy_rc(n.cpu_left - p.cpu_nz, rc, ncpus, cm, free_gpus_after(n, cnt, 1u << g, p.milli), cnt, gt, pw,
                    &new_e);
    s = (int)(long long)(old_e - new_e);
    gsel = 14 - g;
  } else {
    int gl[kMaxGpu];
    unpack_gl(n, gl);
    bool ok = false;
    int cpuL = n.cpu_left;
    const unsigned sm = sub_gpu_mask(gl, cnt, cpuL, p, &ok);
    if (ok) cpuL -= p.cpu_nz;
    (void)energy_rc(cpuL, rc, ncpus, cm, free_gpus_after(n, cnt, ok ? sm : 0u, p.milli), cnt, gt, pw, &new_e);
    s = (int)(long long)(old_e - new_e);
  }
  if (s <= -kPwrVBias || s >= kPwrVBias) { *ovf = true; return -1; }
  return ((s + kPwrVBias) << 4) | gsel;
}
// Second half, on the group max: the score and the GPU (-1: none / not a share pod).
__device__ __forceinline__ int pwr8_finish(int v, int* gpu) {
  if (v < 0) { *gpu = -1; return 0; }
  *gpu = (v & 15) == 15 ? -1 : 14 - (v & 15);
  return (v >> 4) - kPwrVBias;
}

// Workgroup-wide exclusive scan of one int per thread (kRBlock threads), total in *tot.
__device__ __forceinline__ int block_excl_scan(int v, int* s_tmp, int* tot) {
  const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(incl, o, 64);
    if (lane >= o) incl += x;
  }
  if (lane == 63) s_tmp[w] = incl;
  __syncthreads();
  int base = 0, t = 0;
#pragma unroll
  for (int i = 0; i < kRWaves; ++i) {
    base += i < w ? s_tmp[i] : 0;
    t += s_tmp[i];
  }
  *tot = t;
  __syncthreads();
  return base + incl - v;
}

}  // namespace ksim_replay

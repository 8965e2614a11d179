// ksim_memo.hpp -- memoised whole-trace FGD replay (k_memo).
//
// Why: a pod step changes ONE node (the Bind of the winner, or a delete), and the FGD score of a
// node for a pod depends only on that node's state and on the pod's request.  A trace has few
// distinct requests (openb default: 151 pod classes over ~10.9k events), so the score of every
// (pod class, node) pair is kept as a packed 32-bit key and only the changed node's keys are
// recomputed per step; the per-pod argmax over all N nodes reads memoised keys instead of
// re-running Filter + Score on N nodes (fgd_score.go:44-156, frag.go:148-203).  Results are the
// same bits as k_replay / k_step / the oracle (the same device functions produce every key).
//
// Layout: replica r is run by K co-resident 1024-thread workgroups.  EVERY workgroup keeps the
// whole cluster state in LDS (N x 32 B, node slot = name rank) and owns Cw of the replica's pod
// classes (host assignment, classes with the same score request kept together), with the key of
// every node for each owned class in LDS (Cw x N x 4 B).
//
// Per pod step s (class c_s, owner workgroup o_s), with d = the node changed by event s-1:
//   1. every workgroup refreshes the keys of d for its classes: wave 0 lists the states to
//      evaluate (d's current state + one candidate per GPU value class / the Sub state, per
//      distinct score request that some owned class finds feasible; c_s's first), every wave
//      evaluates one state's F (wave_F: lane t classifies typical pod t, lanes 0-5 fold the six
//      bins of F in typical-pod order), wave 0 turns them into keys and updates counts;
//   2. o_s takes the winner = max(top-2 of c_s's keys with d excluded, d's fresh key), runs
//      Reserve's GPU selector and publishes {node, mask} as one 4-byte granule win[s] (written
//      once per run, so no slot reuse and no tag), and writes the result;
//   3. the owner of the NEXT create event's class computes that class's top-2 keys (all fresh
//      but the node step s will change -- the exclusion in 2 handles it);
//   4. every workgroup reads win[s] (relaxed agent-scope poll) and applies the Bind to its LDS
//      copy of the cluster; that node is the next step's d.
// Delete events need no exchange: every workgroup reads the creation's granule and unbinds.
// Every spin is bounded; a timeout sets *fail and stops the replica on every workgroup.
#pragma once

namespace ksim_memo {

using namespace ksim;

constexpr int kMBlock = 1024;
constexpr int kMWaves = kMBlock / 64;
constexpr int kMaxCw = 64;                 // class slots per workgroup (one wave-0 lane each)
constexpr int kMaxItems = 1 + 8 * kMaxCw;  // F evaluations per refresh: current + 8 per request
constexpr int kFoldRows = 6;               // Q1, Q2 (+Q3 frag), Q4, XL, XR, NA
constexpr int kCritWaves = 9;              // owner: waves 1..9 evaluate the step's class on d
// fold-buffer rows 66 doubles apart: lanes 0-5 fold rows 0-5 with ds_read_b128, whose bank is
// (a/4) % 64; a 64-double (2 x 256 B) stride put all six rows on the same banks (6-way conflict),
// 66 puts row b on banks 4b..4b+3
constexpr int kFoldStride = 66;
constexpr int kFoldBuf = kFoldRows * kFoldStride;  // doubles per evaluating wave
constexpr int kEvBuf = 128;
constexpr unsigned kSpinLimit = 1u << 22;
constexpr int kMaxDeadWords = 32;  // dead-class bitmask: class ids < 1024
// Decider mode (MemoArgs::decider): class owners publish, for event s, the top kTopN keys of its
// class and its feasible count as of kLag events earlier; the decider adds the <= kLag nodes
// changed since.
constexpr int kLag = 3;
constexpr int kTopN = kLag + 1;
constexpr int kTopWords = 8;  // per event: kTopN keys | 1, (count << 8) | 1 (nonzero once written)
constexpr int kDItems = kLag * 9;

struct MemoArgs {
  ReplicaDev* reps;
  const int* rep_list;   // replica of each launch position
  // launch position << 8 | workgroup index within the replica, per block: a replica's workgroups are consecutive
  // blocks, K of them (r06: K may differ per replica -- the paper sweep's widened FGD replicas, MemoPlan::Kr)
  const int* wg_map;
  int N, K, Cw;          // K: the most workgroups of a replica
  int nfw;               // waves with a fold buffer (F evaluators)
  int Cmax;              // class table stride
  const PodDev* cls_pod;     // [launch replica][Cmax] representative request of each class
  const int* cls_owner;      // [launch replica][Cmax] (workgroup << 8) | slot
  const int* wg_cls;         // [block][Cw] class of each slot, -1 empty
  const int* wg_ref;         // [block][Cw] first slot with the same score request
  const unsigned long long* wg_grp;  // [block][Cw] slots sharing the request (on the first)
  const int* ev_owner;       // [launch replica][win_stride] owner code of each event's class, -1 delete
  const double* th;          // [102] FGD score steps, or null: the direct sigmoid expression
  unsigned* win;             // [launch replica][win_stride] winner granules, zeroed before launch
  int win_stride;
  int* fail;
  unsigned long long* prof;  // optional [R*K][kProfPhases] (KSIM_PROFILE=1)
  unsigned long long* trace; // optional [R*K][trace_steps][2] (KSIM_PROFILE=2): step start, publish / receive
  int trace_steps;
  // decider mode: workgroup 0 decides every event, workgroups 1..K-1 own the classes
  int decider;
  const int* ev_cls;         // [launch replica][win_stride] class of each event, -1 delete
  unsigned* topg;            // [launch replica][win_stride][kTopWords] top granules, zeroed before launch
  int skip;                  // lean launches: the dead-class skip (KSIM_VARIANT skip=0: off)
  int delay;                 // the hdelay test knob (general and stress instantiations): 1 every wave before the end-of-step
                             // barrier (wave 0 before it receives the step's granule), 2 the owner's critical waves
                             // before their F, 4 every wave at the step start
  unsigned* hkeys;           // kHKeys: [block][Cw][N] the keys in HBM instead of LDS
  // Residency gate (a concurrent run's wide FGD group, launched before the other groups): each workgroup stores
  // `gate_epoch` into started[its block] once it holds its LDS state; the host launches the next group when all
  // have (ksim_engine.hip run_persistent).  Null: no gate.
  int* started;
  int gate_epoch;
};
constexpr int kTrace = 4;  // KSIM_PROFILE=2 trace words per workgroup and step
constexpr int kProfPhases = 24;  // 0-9 phases (thread 0), 10 clock, 11 wall, 12-13 list wave A / C,
                                 // 14 step-start loads, 15 owner's A, 16-20 owner's A split (wave 0)

struct __align__(16) MemoShared {
  PodDev ev[kEvBuf];
  int evo[kEvBuf + 8];  // owner code of each staged event (+ the next window's first): workgroup << 16 |
                        // first slot of its group << 8 | slot; -1 delete
  unsigned dead[kMaxDeadWords];  // lean launches: classes with no feasible node (create-only: for good)
  PodDev cls[kMaxCw];
  TypDev tp[kMaxTypical];
  NodeRec dnode;      // the record of the node the previous event changed (d)
  unsigned dfirst;    // first_of_class(dnode, 0): GPUs holding the first occurrence of their milli-left value
  unsigned pad_dfirst[3];
  double th[104];     // FGD score steps (build_score_thresholds), th[0] = -inf, th[101] = +inf
  unsigned long long grp[kMaxCw];
  int cls_id[kMaxCw];
  int sc_ref[kMaxCw];
  int cnt[kMaxCw];
  unsigned ikey[kMaxItems + 3];
  double F[kMaxItems + 1];
  double Fc[10];      // the step's own class: F of d's current state and of its candidates (waves 0-8)
  uint8_t item_code[kMaxItems + 7];
  uint8_t item_slot[kMaxItems + 7];
  unsigned wtop[kMWaves][2];
  unsigned wtop4[kMWaves][kTopN];  // decider mode: per-wave top keys of an upcoming event's class
  unsigned t2a, t2b;  // top-2 keys of the next create event's class (its owner only)
  int nitems;
  int crit_done;      // owner: critical F evaluations finished (waves 1-9 count up, wave 0 waits)
  int dirty;          // node (rank) changed by the previous event, -1 none
  int stop;
  unsigned pay;       // this step's granule (its owner)
  unsigned long long prof[kProfPhases];
};
static_assert(sizeof(MemoShared) % 16 == 0, "keep the node records 16-B aligned");

// Packed 32-bit key of (pod class, node): [30:24] score + 1 | [23:12] 4095 - rank | [11:8] gpu
// field (15 - g for a share pod placed on GPU g, 0 otherwise) | 0.  0 = infeasible.  Max key =
// max score, ties to the smallest name (selectHost, generic_scheduler.go:187-212); for one node
// the max over its candidates keeps the lowest GPU index (fgd_score.go:128).
constexpr int kMemoMaxRank = 0xFFF;
KSIM_HD unsigned pack_key32(int score, int rank, int gf) {
  return ((unsigned)(score + 1) << 24) | ((unsigned)(kMemoMaxRank - rank) << 12) | ((unsigned)gf << 8);
}
KSIM_HD int key32_score(unsigned k) { return (int)(k >> 24) - 1; }
KSIM_HD int key32_rank(unsigned k) { return kMemoMaxRank - (int)((k >> 12) & 0xFFFu); }
KSIM_HD int key32_gpu(unsigned k) {
  const int gf = (int)((k >> 8) & 0xFu);
  return gf ? 15 - gf : -1;
}

// Granule of step s: bit 0 written | bit 1 no feasible node | [23:8] rank + 1 (0: nothing bound) |
// [31:24] GPU mask.
KSIM_HD unsigned pack_pay(int rank, int mask) {
  return 1u | ((unsigned)(rank + 1) << 8) | ((unsigned)(mask & 0xff) << 24);
}

// Global-memory access through address-space-1 pointers: ReplicaDev's pointers are generic, and a
// flat_store counts in lgkmcnt as well as vmcnt, so every later LDS wait (s_waitcnt lgkmcnt(0))
// would stall until the store is acknowledged by memory.  global_* stores count in vmcnt only.
template <typename T>
__device__ __forceinline__ void gput(T* p, const T& v) {
  static_assert(sizeof(T) % 4 == 0, "word-sized records");
  const unsigned* src = reinterpret_cast<const unsigned*>(&v);
  __attribute__((address_space(1))) unsigned* dst = (__attribute__((address_space(1))) unsigned*)(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = src[i];
}
template <typename T>
__device__ __forceinline__ T gget(const T* p) {
  static_assert(sizeof(T) % 4 == 0, "word-sized records");
  T v;
  unsigned* dst = reinterpret_cast<unsigned*>(&v);
  const __attribute__((address_space(1))) unsigned* src = (const __attribute__((address_space(1))) unsigned*)(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = src[i];
  return v;
}
__device__ __forceinline__ void gput_node(NodeRec* p, const NodeV& n) {
  uint4* q = reinterpret_cast<uint4*>(p);
  gput(q, make_uint4((uint32_t)n.cpu_left, (uint32_t)n.mem_left, n.g[0], n.g[1]));
  gput(q + 1, make_uint4(n.g[2], n.g[3], n.meta, n.name_rank));
}

__device__ __forceinline__ unsigned gload32(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore32(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// Bit g set iff GPU g has at least m milli left (packed u16 compares; the GPUs beyond gpu_cnt hold 0).
// first_of_class(n, m) == first_of_class(n, 0) & ge_mask(n, m).
__device__ __forceinline__ unsigned ge_mask(const NodeV& n, int m) {
  using ksim_replay::u16x2;
  const uint32_t mp = (uint32_t)m * 0x10001u;
  unsigned lt = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u16x2 d = (u16x2)(__builtin_bit_cast(u16x2, n.g[i]) - __builtin_bit_cast(u16x2, mp)) >> (u16x2){15, 15};
    const uint32_t x = __builtin_bit_cast(uint32_t, d);
    lt |= ((x & 1u) | ((x >> 15) & 2u)) << (2 * i);
  }
  return ~lt & 0xFFu;
}

// fgd_score_lookup with the hardware's fast exp2 / reciprocal for the estimate (error ~1e-6
// relative, far below the one score unit the two threshold compares correct).
__device__ __forceinline__ int score_lookup_dev(double delta, const double* th) {
  const float e = __builtin_amdgcn_exp2f((float)delta * -0.0014426950408889634f);  // exp(-delta/1000)
  int a = (int)(100.0f * __builtin_amdgcn_rcpf(1.0f + e));
  a = a < 0 ? 0 : (a > 100 ? 100 : a);
  if (delta >= th[a + 1]) ++a;
  else if (delta < th[a]) --a;
  return a;
}

// first_of_class(n, 0) computed lane-parallel (lane g < 8 tests GPU g): a few VALU instructions
// and one ballot instead of 28 scalar compares.  Every lane must be active.
__device__ __forceinline__ unsigned first_mask_lanes(const NodeV& n, int lane) {
  const int g = lane & 7;
  const int v = ksim_replay::gl_dyn(n, g);
  const bool first = lane < 8 && g < n.gpu_cnt() && (ksim_replay::gl_equal_mask(n, v) & ((1u << g) - 1u)) == 0u;
  return (unsigned)__ballot(first) & 0xFFu;
}

// Top-2 merge of two disjoint sets of distinct keys.
__device__ __forceinline__ void merge2(unsigned& a1, unsigned& a2, unsigned b1, unsigned b2) {
  const unsigned lo = a1 < b1 ? a1 : b1, hi2 = a2 > b2 ? a2 : b2;
  a1 = a1 > b1 ? a1 : b1;
  a2 = lo > hi2 ? lo : hi2;
}
template <int kCtrl>
__device__ __forceinline__ void merge2_dpp(unsigned& a1, unsigned& a2) {
  merge2(a1, a2, (unsigned)ksim_replay::dpp_i<kCtrl>((int)a1), (unsigned)ksim_replay::dpp_i<kCtrl>((int)a2));
}
// Top-2 over the 64 lanes (every lane active): quad xor 1, xor 2, row half mirror, row mirror, then
// the four rows -- the same DPP pattern as wave_max_dpp.
__device__ __forceinline__ void wave_top2(unsigned& a1, unsigned& a2) {
  merge2_dpp<0xB1>(a1, a2);
  merge2_dpp<0x4E>(a1, a2);
  merge2_dpp<0x141>(a1, a2);
  merge2_dpp<0x140>(a1, a2);
  unsigned r1 = (unsigned)__builtin_amdgcn_readlane((int)a1, 0), r2 = (unsigned)__builtin_amdgcn_readlane((int)a2, 0);
  merge2(r1, r2, (unsigned)__builtin_amdgcn_readlane((int)a1, 16), (unsigned)__builtin_amdgcn_readlane((int)a2, 16));
  merge2(r1, r2, (unsigned)__builtin_amdgcn_readlane((int)a1, 32), (unsigned)__builtin_amdgcn_readlane((int)a2, 32));
  merge2(r1, r2, (unsigned)__builtin_amdgcn_readlane((int)a1, 48), (unsigned)__builtin_amdgcn_readlane((int)a2, 48));
  a1 = r1;
  a2 = r2;
}

// Key of one (node, class) pair, one thread (initial fill).  Same functions, same order as the
// k_replay evaluation: Filter, then F of the current state and of each candidate state.
__device__ __forceinline__ unsigned memo_key_scalar(const NodeV& n, const PodDev& p, double F0, int rank,
                                                    const ReplicaDev& rp, const TypDev* __restrict__ tp) {
  if (!filter_node(n, p)) return 0u;
  if (!is_share_pod(p)) {
    const double Fk = eval_fgd_item(n, 9, p, rp, tp);  // fgd_score.go:137-141 NodeResource.Sub
    return pack_key32(fgd_frag_score(F0, Fk), rank, 0);
  }
  unsigned bk = pack_key32(0, rank, 0);  // feasible with no fitting GPU (milli 0, GPU-less node)
  const unsigned fm = first_of_class(n, p.milli);
  for (int g = 0; g < kMaxGpu; ++g) {
    if ((fm >> g) & 1u) {
      const double Fk = eval_fgd_item(n, 1 + g, p, rp, tp);  // fgd_score.go:111-118
      const unsigned k = pack_key32(fgd_frag_score(F0, Fk), rank, 15 - g);
      bk = k > bk ? k : bk;
    }
  }
  return bk;
}

// F = NodeGpuShareFragAmountScore of one state (frag.go:148-203, 411-418, 460-493) by ONE wave:
// lane t classifies typical pod t (64 per round) into (row, value) exactly as frag_F does, writes
// its value into its row of the wave's fold buffer (zeros elsewhere), and lane b < 6 then folds
// row b in typical-pod order.  Rows: 0 Q1, 1 Q2 (+ Q3's frag part), 2 Q4, 3 XL, 4 XR, 5 NA.
// Every bin receives the same sequence of fp64 adds as frag_F's (+0.0 for the typical pods that
// do not touch it, the identity on these non-negative sums), and F adds the bins in index order
// 0,1,3,4,5,6, so F is bit-identical.  All lanes return F.
__device__ __forceinline__ double wave_F(int cpuL, const uint32_t (&g)[4], int total, uint32_t typebit, bool typed,
                                         const TypDev* ltp, int ncpu, int nt, int lane, double* buf) {
  using ksim_replay::u16x2;
  const double dtot = (double)total;
  double acc = 0.0;
  for (int t0 = 0; t0 < nt; t0 += 64) {
    const int t = t0 + lane;
    // branch free: every lane reads a valid entry (clamped) and classifies it both ways
    const int tc = t < nt ? t : nt - 1;
    const uint4 e4 = reinterpret_cast<const uint4*>(ltp)[2 * tc];  // cpu, milli, num_eff, tmask
    const double fr = ltp[tc].freq;
    asm volatile("" ::"v"(e4.y), "v"(e4.z), "v"(e4.w));  // one LDS round trip for the whole entry
    const bool cpu_ok = cpuL >= (int)e4.x;
    const double x = fr * dtot;  // freq * float64(gpuMilliLeftTotal)
    const uint32_t mp = e4.y * 0x10001u;
    uint32_t frag = 0u, nlt = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u16x2 gv = __builtin_bit_cast(u16x2, g[i]);
      const u16x2 lt = (u16x2)(gv - __builtin_bit_cast(u16x2, mp)) >> (u16x2){15, 15};  // left < milli
      frag = __builtin_amdgcn_udot2(gv, lt, frag, false);  // GetGpuFragMilliByNodeResAndPodRes (frag.go:205-213)
      nlt = __builtin_amdgcn_udot2(lt, (u16x2){1, 1}, nlt, false);
    }
    const bool gpu_ok = kMaxGpu - (int)nlt >= (int)e4.z;       // CanNodeHostPodOnGpuMemory (frag.go:447-458)
    const bool acc_ok = !typed || (e4.w & typebit) != 0u;  // IsNodeAccessibleToPod (utils.go:957-1006)
    const bool is_cpu = t < ncpu;                          // GetNodePodFrag case 1 (frag.go:463-469): XL / XR
    int row = is_cpu ? (cpu_ok ? 3 : 4) : (!acc_ok ? 5 : (cpu_ok ? 1 : (gpu_ok ? 2 : 0)));
    row = t < nt ? row : -1;
    const double y = fr * (double)(int)frag;  // Q3: frag part to Q2
    const double val = (!is_cpu && acc_ok && cpu_ok && gpu_ok) ? y : x;
#pragma unroll
    for (int b = 0; b < kFoldRows; ++b) buf[b * kFoldStride + lane] = row == b ? val : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // lane b < 6 folds row b in typical-pod order; columns past the chunk's last typical pod hold
    // +0.0, so the uniform 8-pair batches only ever add exact zeros beyond it
    const int np = (min(64, nt - t0) + 1) >> 1;
    if (lane < kFoldRows) {
      const double2* rw = reinterpret_cast<const double2*>(buf + lane * kFoldStride);
      int k0 = 0;
      for (; k0 + 8 <= np; k0 += 8) {
        double2 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = rw[k0 + i];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc += v[i].x;
          acc += v[i].y;
        }
      }
      // the chunk's last pairs two at a time (openb: 18 pairs -> 8 + 8 + 2, not 24 with 12 +0.0 adds)
      for (; k0 < np; k0 += 2) {
        const double2 v0 = rw[k0], v1 = rw[k0 + 1];
        acc += v0.x;
        acc += v0.y;
        acc += v1.x;
        acc += v1.y;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // FragAmountSumExceptQ3 (frag.go:411-418): Q1 + Q2 + Q4 + XL + XR + NA, in this order
  double out = 0.0;
  out += readlane_d(acc, 0);
  out += readlane_d(acc, 1);
  out += readlane_d(acc, 2);
  out += readlane_d(acc, 3);
  out += readlane_d(acc, 4);
  out += readlane_d(acc, 5);
  return out;
}

// the hdelay test knob stress delays at the hand-over points of a step (the memoised kernels' general
// instantiations and k_memo's stress instantiation only): a wave about to read something another wave of
// the same step may be writing sleeps 0-3 x ~3.4 us on about half the steps (a hash of step, wave and
// workgroup), so the late-reader orders that are rare on an idle chip happen thousands of times per run.
// The bits name the points (k_hmemo, k_memo).
__device__ __forceinline__ void hdelay(int mask, int bit, int step, int wave, int wg) {
  if (!(mask & bit)) return;
  unsigned h = (unsigned)step * 0x9E3779B1u ^ (unsigned)(wave * 0x85EBCA77) ^ (unsigned)(wg * 0xC2B2AE3D) ^ (unsigned)bit;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  if (h & 1u) return;
  for (int i = (int)((h >> 1) & 3u); i > 0; --i) __builtin_amdgcn_s_sleep(127);
}

// ---------------------------------------------------------------------------
// Decider mode.  Workgroup 0 of a replica owns no class: it keeps the cluster and, per event,
// decides the winner itself instead of waiting for a class owner to publish it:
//   W = max( top kTopN keys of the event's class as its owner saw them after event s-1-kLag, minus
//            the nodes changed since,  fresh keys of those <= kLag changed nodes )
// (the snapshot's top list holds the best unchanged node because at most kLag entries are
// removed), n_feasible = snapshot count - their snapshot feasibility + their current one.  The
// owners (workgroups 1..K-1) refresh their keys behind it and publish each top list kLag events
// ahead, so the decider's chain per event is its own F evaluations, no cross-CU hand-off.
// ---------------------------------------------------------------------------
constexpr int kRing = 16;  // top lists the prefetch wave may hold ahead of the coordinator

struct __align__(16) DeciderScratch {
  PodDev cq[kEvBuf];      // class request (Filter + Score) of each staged create event
  PodDev cp;              // this create event's class request, for the F waves
  NodeRec xcur[kLag];     // this event's changed nodes: current records
  NodeRec hprev[kLag], hafter[kLag];  // event t's change (slot t % kLag): record before / after
  int hnode[kLag];                    // node (rank) event t changed, -1 none
  double F[kDItems + 1];
  unsigned ring[kRing][kTopWords];
  int ring_tag[kRing];    // step + 1 once the slot holds that step's top list
  int xn, nitems;
  int cflag;              // create events whose work list is posted (monotonic)
  int fdone;              // F-wave completions (monotonic)
  int consumed;           // last step the coordinator finished
  int finished;
  uint8_t item_x[kDItems + 5], item_code[kDItems + 5];
};

__device__ __forceinline__ int lds_load(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Hand-offs between the decider's waves go through LDS only.  A wave's LDS operations execute in
// issue order, so the data stores before a flag store are seen by a wave that has seen the flag;
// the release only drains the wave's LDS queue (a workgroup-scope fence would also wait for every
// outstanding global store -- the previous event's result and granule -- about a microsecond).
__device__ __forceinline__ void lds_release() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_acquire() { asm volatile("" ::: "memory"); }

// A bounded LDS wait: past the limit the replica stops with a failure (no silent hang).
__device__ __forceinline__ bool lds_spin(unsigned& spins, int* stop, int* fail) {
  if (++spins > 4 * kSpinLimit) {
    __hip_atomic_store(stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    atomicOr(fail, 1);
    return false;
  }
  __builtin_amdgcn_s_sleep(0);
  return true;
}
__device__ __forceinline__ NodeV sel3(int j, const NodeV& a0, const NodeV& a1, const NodeV& a2) {
  return j == 0 ? a0 : (j == 1 ? a1 : a2);
}

// The decider workgroup.  No workgroup barrier inside the event loop: three roles hand work over
// through LDS counters (release / acquire at workgroup scope), so the prefetch wave can run ahead.
//   wave 0        coordinator: the changed nodes and their F work list (history kept in
//                 registers), then the keys, the winner, Reserve, the granule, the result, Bind;
//   waves 1..nF   F evaluations of the posted work list;
//   wave 15       prefetch: polls each create event's top list (global memory, published kLag
//                 events ahead by the class owner) into an LDS ring.
__device__ void memo_decider(const MemoArgs& a, const ReplicaDev& rp, MemoShared& sh, NodeRec* s_nodes,
                             DeciderScratch& ds, double* s_fold, int* s_last, int gi, int tid) {
  const int lane = tid & 63, wv = tid >> 6;
  const size_t gbase = (size_t)gi * a.win_stride;
  unsigned* win = a.win + gbase;
  const int E = rp.n_events;
  constexpr int kPW = kMWaves - 1;
  const int nfw = min(a.nfw, kPW);  // waves with a fold buffer, the prefetch wave excluded
  const int nF = nfw - 1;           // F waves 1 .. nfw-1
  if (tid == 0) { ds.cflag = 0; ds.fdone = 0; ds.consumed = -1; ds.finished = 0; }
  for (int i = tid; i < kRing; i += kMBlock) ds.ring_tag[i] = 0;
  for (int i = tid; i < kLag; i += kMBlock) ds.hnode[i] = -1;
  __syncthreads();
  // KSIM_PROFILE=1 (coordinator): prof[20] work list, [21] top-list wait, [22] F wait, [23] decision + bind
  const bool prof = a.prof != nullptr && tid == 0;
  unsigned long long tp0 = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
  auto dmark = [&](int ph) {
    if (prof) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      sh.prof[ph] += t - tp0;
      tp0 = t;
    }
  };

  if (wv == 0) {
    // ---------------- coordinator
    const PodDev* cls_pod = a.cls_pod + (size_t)gi * a.Cmax;
    const bool use_th = a.th != nullptr;
    auto score_of = [&](double delta) { return use_th ? score_lookup_dev(delta, sh.th) : fgd_score_of_delta(delta); };
    // the last kLag events' changes, newest first: node (rank, -1 none), record before, record after
    static_assert(kLag == 3, "the history registers are unrolled for kLag == 3");
    // (the records before live in the LDS ring ds.hprev, slot = event % kLag)
    int hn0 = -1, hn1 = -1, hn2 = -1;
    NodeV ha0{}, ha1{}, ha2{};
    unsigned hf0 = 0u, hf1 = 0u, hf2 = 0u;  // first_of_class(after, 0), lane-parallel at Bind time
    int ncreate = 0;
    for (int step = 0; step < E; ++step) {
      const int eb = step & (kEvBuf - 1);
      if (eb == 0) {
        const int ne = min(kEvBuf, E - step);
        const uint4* src = reinterpret_cast<const uint4*>(rp.ev + step);
        for (int i = lane; i < ne * 2; i += 64) reinterpret_cast<uint4*>(sh.ev)[i] = gget(src + i);
        for (int i = lane; i < ne; i += 64) {
          const int c = gget(a.ev_cls + gbase + step + i);
          ds.cq[i] = c >= 0 ? gget(cls_pod + c) : PodDev{};
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      const PodDev p = ksim_replay::uniform_pod(&sh.ev[eb]);
      const bool del = (p.flags & kPodDelete) != 0u;
      int rk = -1;
      NodeV before{}, after{};
      if (!del) {
        const PodDev cp = ksim_replay::uniform_pod(&ds.cq[eb]);
        const bool share = is_share_pod(cp);
        // changed nodes X from the register history, oldest change first (the snapshot state of a
        // node changed twice is the one before its first change; its current state the one after
        // its last)
        int xn = 0, x0 = -1, x1 = -1, x2 = -1;
        bool s0 = false, s1 = false, s2 = false;
        NodeV c0{}, c1{}, c2{};
        unsigned f0 = 0u, f1 = 0u, f2 = 0u;
#define KSIM_XADD(R, PRE, POST, FM)                         \
        if ((R) >= 0) {                                     \
          if ((R) == x0) {                                  \
            c0 = (POST); f0 = (FM);                         \
          } else if ((R) == x1) {                           \
            c1 = (POST); f1 = (FM);                         \
          } else {                                          \
            const bool f_ = filter_node((PRE), cp);         \
            if (xn == 0) { x0 = (R); s0 = f_; c0 = (POST); f0 = (FM); } \
            else if (xn == 1) { x1 = (R); s1 = f_; c1 = (POST); f1 = (FM); } \
            else { x2 = (R); s2 = f_; c2 = (POST); f2 = (FM); } \
            ++xn;                                           \
          }                                                 \
        }
        KSIM_XADD(hn2, ksim_replay::uniform_node(&ds.hprev[(step + 0) % kLag]), ha2, hf2)  // event step-3
        KSIM_XADD(hn1, ksim_replay::uniform_node(&ds.hprev[(step + 1) % kLag]), ha1, hf1)  // event step-2
        KSIM_XADD(hn0, ksim_replay::uniform_node(&ds.hprev[(step + 2) % kLag]), ha0, hf0)  // event step-1
#undef KSIM_XADD
        // F work list: per changed node its current state, then one candidate per GPU value class
        // (share pod) or the Sub state; written lane-parallel.  first_of_class(c, m) ==
        // first_of_class(c, 0) & ge_mask(c, m): packed compares instead of 64 scalar ones
        const unsigned cm0 = xn > 0 && share ? (f0 & ge_mask(c0, cp.milli)) : 0u;
        const unsigned cm1 = xn > 1 && share ? (f1 & ge_mask(c1, cp.milli)) : 0u;
        const unsigned cm2 = xn > 2 && share ? (f2 & ge_mask(c2, cp.milli)) : 0u;
        const int n0 = xn > 0 ? 1 + (share ? __popc(cm0) : 1) : 0;
        const int n1 = xn > 1 ? 1 + (share ? __popc(cm1) : 1) : 0;
        const int n2 = xn > 2 ? 1 + (share ? __popc(cm2) : 1) : 0;
        const int xf1 = n0, xf2 = n0 + n1, nit = n0 + n1 + n2;
        if (lane < nit) {
          const int j = lane < xf1 ? 0 : (lane < xf2 ? 1 : 2);
          const int k = lane - (j == 0 ? 0 : (j == 1 ? xf1 : xf2));
          unsigned m = j == 0 ? cm0 : (j == 1 ? cm1 : cm2);
          for (int q = 1; q < k; ++q) m &= m - 1u;
          ds.item_x[lane] = (uint8_t)j;
          ds.item_code[lane] = (uint8_t)(k == 0 ? 0 : (share ? 1 + __builtin_ctz(m) : 9));
        }
        if (lane < xn) store_node(&ds.xcur[lane], sel3(lane, c0, c1, c2));
        if (lane == 0) {
          ds.cp = cp;
          ds.nitems = nit;
        }
        lds_release();
        ++ncreate;
        if (lane == 0) lds_store(&ds.cflag, ncreate);
        dmark(20);
        // the class owner's top list (the prefetch wave's LDS ring; the words before the tag)
        const int slot = step % kRing;
        unsigned rw = 0u, spins = 0;
        for (;;) {
          const int tg = lds_load(&ds.ring_tag[slot]);
          rw = lane <= kTopN ? ds.ring[slot][lane] : 0u;
          if (tg == step + 1) break;
          if (lds_load(&sh.stop) || !lds_spin(spins, &sh.stop, a.fail)) break;
        }
        dmark(21);
        // the F values
        spins = 0;
        while (lds_load(&ds.fdone) < nF * ncreate) {
          if (lds_load(&sh.stop) || !lds_spin(spins, &sh.stop, a.fail)) break;
        }
        lds_acquire();
        if (lds_load(&sh.stop)) break;
        dmark(22);
        // fresh key of changed node j on lane j (memo_key_scalar's key from the F values)
        unsigned fresh = 0u;
        bool fnow = false, fsnap = false;
        const int xr = lane == 0 ? x0 : (lane == 1 ? x1 : x2);
        if (lane < xn) {
          const NodeV cur = sel3(lane, c0, c1, c2);
          fsnap = lane == 0 ? s0 : (lane == 1 ? s1 : s2);
          if (filter_node(cur, cp)) {
            fnow = true;
            const int nj = lane == 0 ? n0 : (lane == 1 ? n1 : n2);
            const int xfj = lane == 0 ? 0 : (lane == 1 ? xf1 : xf2);
            double Fv[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) Fv[k] = k < nj ? ds.F[xfj + k] : 0.0;
            unsigned bk = pack_key32(0, xr, 0);
            if (share) {
              unsigned m = lane == 0 ? cm0 : (lane == 1 ? cm1 : cm2);
#pragma unroll
              for (int k = 1; k < 9; ++k) {
                if (m) {
                  const int g = __builtin_ctz(m);
                  m &= m - 1u;
                  const unsigned key = pack_key32(score_of(Fv[0] - Fv[k]), xr, 15 - g);
                  bk = key > bk ? key : bk;
                }
              }
            } else {
              const unsigned key = pack_key32(score_of(Fv[0] - Fv[1]), xr, 0);
              bk = key > bk ? key : bk;
            }
            fresh = bk;
          }
        }
        unsigned tk = 0u;
        if (lane < kTopN) {
          const unsigned k = rw & ~0xffu;
          const int kr = key32_rank(k);
          const bool inx = k != 0u && ((xn > 0 && kr == x0) || (xn > 1 && kr == x1) || (xn > 2 && kr == x2));
          tk = inx ? 0u : k;
        }
        const unsigned W = (unsigned)ksim_replay::wave_max_dpp((int)(fresh > tk ? fresh : tk));
        const int cnt = (int)((unsigned)__builtin_amdgcn_readlane((int)rw, kTopN) >> 8);
        const int nfeas = cnt + __popcll(__ballot(fnow)) - __popcll(__ballot(lane < xn && fsnap));
        if (lane == 0) lds_store(&ds.consumed, step);
        ResultDev out{-1, 0, 0, nfeas, ST_UNSCHED};
        unsigned pay = 1u;
        if (W != 0u) {
          const int wr = key32_rank(W);
          const NodeV wn = wr == x0 ? c0 : (wr == x1 ? c1 : (wr == x2 ? c2 : ksim_replay::uniform_node(&s_nodes[wr])));
          const int mask = select_gpus(wn, p, rp.gpusel, key32_gpu(W), rp.seed, step);
          if (mask < 0) {  // Reserve failed: allocateGpuId returned "" / panicked
            out.status = ST_ERROR;
          } else {
            out.status = ST_OK;
            out.score = result_score(rp, nfeas, key32_score(W), 0, 0);
            out.node = wr;  // name rank; k_memo_finish maps it to the node index
            out.gpu_mask = mask;
            pay = pack_pay(wr, mask);
            rk = wr;
            before = wn;
            after = wn;
            bind_node(after, p, mask, +1);
          }
        }
        if (lane == 0) {
          gstore32(win + step, pay);
          gput(rp.res + step, out);
        }
      } else {
        // simulator.go:416-422 deletePod: undo the creation's Bind (the coordinator wrote its granule)
        unsigned pay = 0u;
        PodDev bp = p;
        if (p.ref >= 0 && p.ref < step) {
          pay = __builtin_amdgcn_readfirstlane(gload32(win + p.ref));
          const uint4* q = reinterpret_cast<const uint4*>(rp.ev + p.ref);
          uint4 u0 = gget(q), u1 = gget(q + 1);
          uint32_t* o = reinterpret_cast<uint32_t*>(&bp);
          o[0] = __builtin_amdgcn_readfirstlane(u0.x); o[1] = __builtin_amdgcn_readfirstlane(u0.y);
          o[2] = __builtin_amdgcn_readfirstlane(u0.z); o[3] = __builtin_amdgcn_readfirstlane(u0.w);
          o[4] = __builtin_amdgcn_readfirstlane(u1.x); o[5] = __builtin_amdgcn_readfirstlane(u1.y);
          o[6] = __builtin_amdgcn_readfirstlane(u1.z); o[7] = __builtin_amdgcn_readfirstlane(u1.w);
        }
        const int wr = (int)((pay >> 8) & 0xffffu) - 1;
        const int mask = (int)(pay >> 24);
        if (wr >= 0) {
          rk = wr;
          before = ksim_replay::uniform_node(&s_nodes[wr]);
          after = before;
          bind_node(after, bp, mask, -1);
        }
        if (lane == 0) gput(rp.res + step, ResultDev{wr, wr >= 0 ? mask : 0, 0, 0, ST_DELETED});
        if (lane == 0) lds_store(&ds.consumed, step);
      }
      if (rk >= 0) {
        if (lane == 0) store_node(&s_nodes[rk], after);
        if (rp.snap && lane == 0) {  // cluster report: the state this event left
          gput_node(rp.snap + step, after);
          gput(rp.prev + step, s_last[rk]);
        }
        if (lane == 0) s_last[rk] = step;
      }
      if (rk >= 0 && lane == 0) store_node(&ds.hprev[step % kLag], before);
      const unsigned fa = rk >= 0 ? first_mask_lanes(after, lane) : 0u;
      hn2 = hn1; ha2 = ha1; hf2 = hf1;
      hn1 = hn0; ha1 = ha0; hf1 = hf0;
      hn0 = rk; ha0 = after; hf0 = fa;
      dmark(23);
    }
    if (lane == 0) lds_store(&ds.finished, 1);
  } else if (wv == kPW) {
    // ---------------- prefetch wave: the top list of every create event, in order, kRing ahead
    int chunk = 0, my_cls = -1;
    for (int step = 0; step < E; ++step) {
      if (step == 0 || step - chunk >= 64) {
        chunk = step;
        my_cls = step + lane < E ? gget(a.ev_cls + gbase + step + lane) : -1;
      }
      if (__builtin_amdgcn_readlane(my_cls, step - chunk) < 0) continue;  // deletes: no top list
      unsigned cspins = 0;
      while (lds_load(&ds.consumed) < step - kRing) {
        if (lds_load(&sh.stop) || lds_load(&ds.finished) || !lds_spin(cspins, &sh.stop, a.fail)) break;
      }
      if (lds_load(&sh.stop) || lds_load(&ds.finished)) break;
      unsigned v = 0u;
      bool ok = true;
      if (lane <= kTopN) {
        const unsigned* tw = a.topg + (gbase + step) * kTopWords;
        unsigned spins = 0;
        while ((v = gload32(tw + lane)) == 0u) {
          if (++spins > kSpinLimit || lds_load(&sh.stop)) { ok = false; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (__ballot(!ok) != 0ull) {
        if (lane == 0) { lds_store(&sh.stop, 1); atomicOr(a.fail, 1); }
        break;
      }
      const int slot = step % kRing;
      if (lane <= kTopN) ds.ring[slot][lane] = v;
      lds_release();
      if (lane == 0) lds_store(&ds.ring_tag[slot], step + 1);
    }
  } else if (wv <= nF) {
    // ---------------- F waves: the posted work list of each create event
    int seen = 0;
    for (;;) {
      int cf;
      unsigned spins = 0;
      while ((cf = lds_load(&ds.cflag)) == seen) {  // (backs off: 14 polling waves would crowd the LDS)
        if (lds_load(&ds.finished) || lds_load(&sh.stop) || !lds_spin(spins, &sh.stop, a.fail)) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if (cf == seen) break;
      seen = cf;
      lds_acquire();
      const int nit = __builtin_amdgcn_readfirstlane(ds.nitems);
      const PodDev cp = ksim_replay::uniform_pod(&ds.cp);
      for (int it = wv - 1; it < nit; it += nF) {
        const NodeV cur = ksim_replay::uniform_node(&ds.xcur[ds.item_x[it]]);
        int cpuL, total;
        uint32_t gs[4];
        ksim_replay::fgd_candidate(cur, ds.item_code[it], cp, &cpuL, gs, &total);
        const double F = wave_F(cpuL, gs, total, 1u << cur.gpu_type(), rp.typed != 0, sh.tp, rp.ncpu, rp.nt, lane,
                                s_fold + (size_t)wv * kFoldBuf);
        if (lane == 0) ds.F[it] = F;
      }
      lds_release();
      if (lane == 0) __hip_atomic_fetch_add(&ds.fdone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// k_memo.  Dynamic LDS: MemoShared | NodeRec nodes[N] (slot = name rank) | u32 keys[Cw][N] |
// f64 fold buffers [nfw][6][64] (the initial F of every node at start-up) | i32 last[N] (cluster
// report: the last event that changed each node).
// Per step the phases are (barriers between):
//   A  owner of the step's class: waves 0-8 evaluate F of d's current state and of its candidate
//      states for that class (no list: wave k <-> candidate k) -- the critical path;
//      list wave (15): the work list of d's other requests;
//   B  owner: wave 0 scores, updates the class group's keys, takes the winner and publishes;
//      the other waves evaluate the listed states;
//   C  list wave: the listed requests' keys; then (next step's owner) top-2; then wave 0 reads
//      the step's granule and applies the Bind.
// ---------------------------------------------------------------------------
// kDecider: decider mode (MemoArgs::decider), a separate instantiation so that the classic
// kernel's register allocation does not carry the decider's code.
// kGeneral: the KSIM_PROFILE phase timers and step trace, the per-event cluster report stores,
// delete events and the direct sigmoid expression when the host has no score table.  The lean
// instantiation (kGeneral = false: no profile, no report, no delete event, score table present --
// the bench and the paper sweeps)
// compiles them out of the step loop: this kernel's critical path is sensitive to code size and
// scalar-register pressure (39.1 -> 35.8 ms per C2 launch for the profile hooks alone).
// kStress: the lean instantiation plus the hdelay test knob's delays (tests only: the dead-class skip is lean-only).
// kReport (r06): the lean instantiation plus the cluster report's stores (the paper sweep's wide FGD replicas:
// with the general kernel the report cost them 25 %).  kHKeys (r06): the (class, node) keys in HBM (MemoArgs::hkeys,
// L2-resident) instead of LDS, for replicas whose classes' keys do not fit beside the cluster (the gpuspec traces:
// 457 classes); only the key array moves, every other access is the LDS kernel's.
template <bool kDecider, bool kGeneral, bool kStress = false, bool kReport = false, bool kHKeys = false>
__global__ __launch_bounds__(kMBlock) void k_memo(MemoArgs a, const TypDev* __restrict__ tp_all) {
  static_assert(!(kDecider && kHKeys), "the decider's scratch aliases the LDS keys");
  constexpr bool kDelays = kGeneral || kStress;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  MemoShared& sh = *reinterpret_cast<MemoShared*>(smem);
  constexpr int kLW = kMWaves - 1;  // the list wave
  const int gw = a.wg_map[blockIdx.x];
  const int gi = gw >> 8;  // replica position in this launch
  const int r = a.rep_list[gi];
  const int w = gw & 0xff;
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const ReplicaDev rp = a.reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  const int N = a.N, Cw = a.Cw;
  const int* rank2idx = reinterpret_cast<const int*>(rp.tags + (size_t)N * kTagStride);
  NodeRec* s_nodes = reinterpret_cast<NodeRec*>(smem + sizeof(MemoShared));
  unsigned* s_keys = kHKeys ? a.hkeys + (size_t)blockIdx.x * Cw * N : reinterpret_cast<unsigned*>(s_nodes + N);
  double* s_fold = reinterpret_cast<double*>(
      reinterpret_cast<char*>(s_nodes + N) + (kHKeys ? 0 : (std::max((size_t)Cw * N * 4, sizeof(DeciderScratch)) + 15) & ~(size_t)15));
  int* s_last = reinterpret_cast<int*>(reinterpret_cast<char*>(s_fold) +
                                       std::max((size_t)a.nfw * kFoldBuf * 8, ((size_t)N * 8 + 15) & ~(size_t)15));
  const PodDev* cls_pod = a.cls_pod + (size_t)gi * a.Cmax;
  const size_t wgo = (size_t)blockIdx.x * Cw;
  unsigned* win = a.win + (size_t)gi * a.win_stride;
  const int* evo = a.ev_owner + (size_t)gi * a.win_stride;
  const bool is_w0 = w == 0;
  constexpr bool kSkip = !kDecider && !kGeneral;  // the dead-class skip (create-only streams)
  const bool skip_ok = kSkip && a.skip && a.Cmax <= kMaxDeadWords * 32;

  // ---- start-up: the cluster in rank order, the owned classes, the typical table
  for (int i = tid; i < N; i += kMBlock) {
    store_node(&s_nodes[i], load_node(rp.nodes + rank2idx[i]));
    s_last[i] = -1;
  }
  for (int j = tid; j < kMaxCw; j += kMBlock) {
    const int cid = j < Cw ? a.wg_cls[wgo + j] : -1;
    sh.cls_id[j] = cid;
    sh.sc_ref[j] = j < Cw ? a.wg_ref[wgo + j] : j;
    sh.grp[j] = j < Cw ? a.wg_grp[wgo + j] : 0ull;
    sh.cnt[j] = 0;
    if (cid >= 0) sh.cls[j] = cls_pod[cid];
    else reinterpret_cast<uint4*>(&sh.cls[j])[0] = reinterpret_cast<uint4*>(&sh.cls[j])[1] = make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < rp.nt * 2; i += kMBlock)
    reinterpret_cast<uint4*>(sh.tp)[i] = reinterpret_cast<const uint4*>(tp)[i];
  if (tid == 0) { sh.dirty = -1; sh.stop = 0; sh.nitems = 0; sh.t2a = 0u; sh.t2b = 0u; sh.pay = 0u; sh.crit_done = 0; }
  // the residency gate: this workgroup has started (a vector store to host memory, system scope)
  if (a.started != nullptr && tid == 0)
    __hip_atomic_store(a.started + blockIdx.x, a.gate_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int i = tid; i < kMaxDeadWords; i += kMBlock) sh.dead[i] = 0u;
  // phase timer (wall clock, 100 MHz): only with a profile buffer, thread 0 of each workgroup
  const bool prof = kGeneral && a.prof != nullptr;
  unsigned long long* const trace = kGeneral ? a.trace : nullptr;
  if (prof && tid < kProfPhases) sh.prof[tid] = 0ull;
  unsigned long long t_last = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const unsigned long long t_start = t_last, c_start = prof ? __builtin_amdgcn_s_memtime() : 0ull;
  auto mark = [&](int ph) {
    if (prof && tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      sh.prof[ph] += t - t_last;
      t_last = t;
    }
  };
  __syncthreads();
  // F of every node's initial state, then the key of every (owned class, node) pair
  double* s_F0 = s_fold;
  for (int i = tid; i < N; i += kMBlock) s_F0[i] = eval_fgd_item(load_node(&s_nodes[i]), 0, PodDev{}, rp, tp);
  __syncthreads();
  for (int x = tid; x < Cw * N; x += kMBlock) {
    const int j = x / N, i = x - j * N;
    unsigned k = 0u;
    if (sh.cls_id[j] >= 0) k = memo_key_scalar(load_node(&s_nodes[i]), sh.cls[j], s_F0[i], i, rp, tp);
    s_keys[x] = k;
  }
  __syncthreads();
  for (int j = wv; j < Cw; j += kMWaves) {  // feasible nodes per class
    int c = 0;
    for (int i0 = 0; i0 < N; i0 += 64) c += __popcll(__ballot(i0 + lane < N && s_keys[(size_t)j * N + i0 + lane] != 0u));
    if (lane == 0) sh.cnt[j] = c;
  }

  // top-2 keys of class slot `slot` over all nodes (every thread of the workgroup calls it)
  auto top2 = [&](int slot) {
    const unsigned* kr = s_keys + (size_t)slot * N;
    unsigned a1 = 0u, a2 = 0u;
    for (int i = tid; i < N; i += kMBlock) {
      const unsigned k = kr[i];
      if (k > a1) { a2 = a1; a1 = k; } else if (k > a2) { a2 = k; }
    }
    wave_top2(a1, a2);
    if (lane == 0) { sh.wtop[wv][0] = a1; sh.wtop[wv][1] = a2; }
    __syncthreads();
    if (wv == 0) {
      a1 = lane < kMWaves ? sh.wtop[lane][0] : 0u;
      a2 = lane < kMWaves ? sh.wtop[lane][1] : 0u;
      wave_top2(a1, a2);
      if (lane == 0) { sh.t2a = a1; sh.t2b = a2; }
    }
  };
  const bool use_th = !kGeneral || a.th != nullptr;  // the lean instantiation is launched with a table
  if (use_th)
    for (int i = tid; i < 102; i += kMBlock) sh.th[i] = a.th[i];
  // decider mode: the top kTopN keys of class slot `slot` and its feasible count, published for
  // event sp (every thread of the workgroup calls it)
  const size_t gbase = (size_t)gi * a.win_stride;
  auto publish_top = [&](int slot, int sp) {
    const unsigned* kr = s_keys + (size_t)slot * N;
    unsigned k4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) k4[q] = tid + q * kMBlock < N ? kr[tid + q * kMBlock] : 0u;
    unsigned prev = 0xFFFFFFFFu;
#pragma unroll
    for (int r = 0; r < kTopN; ++r) {  // keys are distinct (they carry the rank): next smaller each round
      unsigned c = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) c = (k4[q] < prev && k4[q] > c) ? k4[q] : c;
      const unsigned m = (unsigned)ksim_replay::wave_max_dpp((int)c);
      if (lane == 0) sh.wtop4[wv][r] = m;
      prev = m;
    }
    __syncthreads();
    if (wv == 0) {
      const unsigned v = lane < kMWaves * kTopN ? sh.wtop4[lane / kTopN][lane % kTopN] : 0u;
      unsigned pv = 0xFFFFFFFFu, out = 0u;
#pragma unroll
      for (int r = 0; r < kTopN; ++r) {
        const unsigned m = (unsigned)ksim_replay::wave_max_dpp((int)(v < pv ? v : 0u));
        out = lane == r ? m : out;
        pv = m;
      }
      unsigned* tw = a.topg + (gbase + sp) * kTopWords;
      if (lane < kTopN) gstore32(tw + lane, out | 1u);
      else if (lane == kTopN) gstore32(tw + lane, ((unsigned)sh.cnt[slot] << 8) | 1u);
    }
  };
  if constexpr (kDecider) {
    // the first kLag events see the initial state
    for (int sp = 0; sp < kLag && sp < rp.n_events; ++sp) {
      const int o = evo[sp];
      __syncthreads();
      if (o >= 0 && (o >> 16) == w) publish_top(o & 0xff, sp);
    }
  } else {
    // the first create event's class
    int s0 = 0;
    while (s0 < rp.n_events && evo[s0] < 0) ++s0;
    __syncthreads();
    if (s0 < rp.n_events && (evo[s0] >> 16) == w) top2(evo[s0] & 0xff);
  }
  __syncthreads();
  mark(0);
  auto score_of = [&](double delta) { return use_th ? score_lookup_dev(delta, sh.th) : fgd_score_of_delta(delta); };

  // list wave, lane j <-> class slot j: the slot's request and group, kept in registers
  PodDev lq{};
  bool l_valid = false, l_rep = false, l_share = false;
  int l_ref = 0;
  unsigned long long l_grp = 0ull;
  if (wv == kLW) {
    l_valid = lane < Cw && sh.cls_id[lane] >= 0;
    if (l_valid) lq = sh.cls[lane];
    l_ref = sh.sc_ref[lane];
    l_grp = sh.grp[lane];
    l_rep = l_valid && l_ref == lane;
    l_share = is_share_pod(lq);
  }
  // list-wave state of the current refresh
  bool r_feas = false, r_need = false, r_skip = false;
  int r_base = 0, r_ni = 0;

  const bool decider = kDecider && w == 0;
  if constexpr (kDecider)
    if (decider) memo_decider(a, rp, sh, s_nodes, *reinterpret_cast<DeciderScratch*>(s_keys), s_fold, s_last, gi, tid);
  for (int step = 0; step < (decider ? 0 : rp.n_events); ++step) {
    const int eb = step & (kEvBuf - 1);
    if (eb == 0) {
      const int ne = min(kEvBuf, rp.n_events - step);
      const uint4* src = reinterpret_cast<const uint4*>(rp.ev + step);
      for (int i = tid; i < ne * 2; i += kMBlock) reinterpret_cast<uint4*>(sh.ev)[i] = gget(src + i);
      for (int i = tid; i <= ne + kLag; i += kMBlock) sh.evo[i] = step + i < rp.n_events ? gget(evo + step + i) : -1;
      __syncthreads();
    }
    // Dead-class skip (lean launches, create-only streams): Filter is monotone in a node's resources and a
    // creation only takes resources, so once an event found no feasible node (its granule says so), every
    // later event of its class finds none either -- unscheduled, 0 feasible, nothing changes.  Every
    // workgroup holds the same dead set (updated from the same granules), so all skip the same steps;
    // the dirty node is carried to the next decided step, and the owner of the next event's class
    // still precomputes its top-2 (with the dirty node excluded there, as on any step).
    if constexpr (kSkip) {
      const int cls = __builtin_amdgcn_readfirstlane(sh.ev[eb].pad);  // the event's class (load_events)
      if (skip_ok && ((sh.dead[cls >> 5] >> (cls & 31)) & 1u)) {
        // the whole run of dead events up to the next live one (or the window's end) at once: the dead
        // set cannot change inside the run; every wave finds the same run
        const int wend = min(kEvBuf, rp.n_events - (step - eb));
        int run = wend - eb;
        for (int j0 = eb + 1; j0 < wend; j0 += 64) {
          const int j = j0 + lane;
          const int c = j < wend ? sh.ev[j].pad : 0;
          const unsigned long long lb = __ballot(j < wend && !((sh.dead[c >> 5] >> (c & 31)) & 1u));
          if (lb) {
            run = j0 + (int)__builtin_ctzll(lb) - eb;
            break;
          }
        }
        if (is_w0)
          for (int i = tid; i < run; i += kMBlock) gput(rp.res + step + i, ResultDev{-1, 0, 0, 0, ST_UNSCHED});
        if (step + run < rp.n_events) {  // the next event's owner precomputes its class's top-2
          const int ocn = __builtin_amdgcn_readfirstlane(sh.evo[eb + run]);
          if (ocn >= 0 && (ocn >> 16) == w) {
            __syncthreads();
            top2(ocn & 0xff);
          }
        }
        __syncthreads();
        step += run - 1;
        continue;
      }
    }
    if (trace && tid == 0 && step < a.trace_steps)
      trace[((size_t)blockIdx.x * a.trace_steps + step) * kTrace] = __builtin_amdgcn_s_memrealtime();
    if constexpr (kDelays) hdelay(a.delay, 4, step, wv, (int)blockIdx.x);
    // one LDS round trip: the event, its owner code, d and d's record
    const PodDev p = ksim_replay::uniform_pod(&sh.ev[eb]);
    const int oc = __builtin_amdgcn_readfirstlane(sh.evo[eb]);
    const int d = __builtin_amdgcn_readfirstlane(sh.dirty);
    const NodeV dn = ksim_replay::uniform_node(&sh.dnode);
    const unsigned dfirst = __builtin_amdgcn_readfirstlane(sh.dfirst);
    const bool del = kGeneral && (p.flags & kPodDelete) != 0u;  // lean: launched on create-only streams
    const bool own = !kDecider && oc >= 0 && (oc >> 16) == w;  // decider mode: workgroup 0 decides
    const int oslot = own ? (oc & 0xff) : -1;
    const int crep = own ? ((oc >> 8) & 0xff) : -1;
    const unsigned long long t_loaded = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (prof && tid == 0) sh.prof[14] += t_loaded - t_last;  // step start: the event / d loads

    // ---- A: the step's own class on d (owner, waves 0-8) | the list of d's other requests (list wave)
    if (d >= 0) {
      if (own && wv >= 1 && wv <= kCritWaves) {
        if constexpr (kDelays) hdelay(a.delay, 2, step, wv, (int)blockIdx.x);
        // wave 1 + c evaluates candidate c of d for the step's class: 0 = d's current state,
        // 1..8 = the share pod on GPU c-1 (first GPU of its milli-left value), 1 = the Sub state
        // otherwise.  Nine waves over four SIMDs; wave 0 is left to the owner's bookkeeping.
        const PodDev cp = ksim_replay::uniform_pod(&sh.cls[crep]);
        const int c = wv - 1;
        int code = -1;
        if (c == 0) code = 0;
        else if (is_share_pod(cp)) code = (((dfirst & ge_mask(dn, cp.milli)) >> (c - 1)) & 1u) ? c : -1;
        else if (c == 1) code = 9;
        if (code >= 0) {
          int cpuL, total;
          uint32_t gs[4];
          ksim_replay::fgd_candidate(dn, code, cp, &cpuL, gs, &total);
          const double F = wave_F(cpuL, gs, total, 1u << dn.gpu_type(), rp.typed != 0, sh.tp, rp.ncpu, rp.nt, lane,
                                  s_fold + (size_t)wv * kFoldBuf);
          if (lane == 0) sh.Fc[c] = F;
        }
        if (lane == 0) {  // hand the candidate's F to wave 0 without a workgroup barrier
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __hip_atomic_fetch_add(&sh.crit_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      if (wv == kLW) {
        const unsigned long long tl0 = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
        r_skip = own && l_valid && l_ref == crep;  // the step's own group: its keys are set in B
        r_feas = l_valid && !r_skip && filter_node(dn, lq);
        const unsigned long long FM = __ballot(r_feas);
        r_need = l_rep && !r_skip && (FM & l_grp) != 0ull;
        unsigned cm = 0u;
        if (r_need) cm = l_share ? (dfirst & ge_mask(dn, lq.milli)) : 0x100u;
        r_ni = __popc(cm);
        // exclusive prefix of r_ni over the lanes (r_ni <= 8: four bit planes)
        int excl = 0, tot = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const unsigned long long m = __ballot((r_ni >> b) & 1);
          excl += __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
          tot += __popcll(m) << b;
        }
        const int i0 = own ? 0 : 1;  // item 0 = d's current state unless the owner evaluated it (Fc[0])
        r_base = i0 + excl;
        int o = r_base;
        unsigned mm = cm;
        while (mm) {
          const int g = __builtin_ctz(mm);
          mm &= mm - 1u;
          sh.item_code[o] = (uint8_t)(l_share ? 1 + g : 9);
          sh.item_slot[o] = (uint8_t)lane;
          ++o;
        }
        if (lane == 0) {
          if (!own) {
            sh.item_code[0] = 0;
            sh.item_slot[0] = 0;
          }
          sh.nitems = tot > 0 ? i0 + tot : 0;
          if (prof) sh.prof[12] += __builtin_amdgcn_s_memrealtime() - tl0;
        }
      }
    }
    // ---- the owner publishes the step's winner (wave 0, as soon as waves 1-9 have their F).
    // Everything that does not depend on this step's F values -- the precomputed best of the other
    // nodes (ex) and Reserve's GPU choice on it, the class requests, d's feasibility and old key --
    // is loaded while waves 1-9 evaluate F; after the wait only d's key, the max and the granule store
    // remain before the winner is out.
    unsigned gk_crit = 0u;
    if (own && wv == 0) {
      const unsigned t2a = sh.t2a, t2b = sh.t2b;
      const unsigned ex = (d >= 0 && t2a != 0u && key32_rank(t2a) == d) ? t2b : t2a;
      const int cnt_o = sh.cnt[oslot];
      unsigned old_own = 0u, fresh = 0u;
      bool ofeas = false;
      PodDev cp{};
      if (d >= 0) {
        old_own = s_keys[(size_t)oslot * N + d];
        cp = ksim_replay::uniform_pod(&sh.cls[crep]);
        ofeas = filter_node(dn, ksim_replay::uniform_pod(&sh.cls[oslot]));
      }
      const int mask_ex =
          ex != 0u ? select_gpus(load_node(&s_nodes[key32_rank(ex)]), p, rp.gpusel, key32_gpu(ex), rp.seed, step) : -1;
      // Reserve on d: only the FGD / PWR selectors of a share pod depend on the key's GPU
      const bool d_gpu_from_key = is_share_pod(p) && p.milli > 0 && (rp.gpusel == SEL_FGD || rp.gpusel == SEL_PWR);
      const int mask_d_pre = d >= 0 && !d_gpu_from_key ? select_gpus(dn, p, rp.gpusel, -1, rp.seed, step) : -1;
      if (prof && tid == 0) sh.prof[16] += __builtin_amdgcn_s_memrealtime() - t_loaded;
      if (d >= 0) {
        if (lane == 0) {  // wait for waves 1-9 (LDS counter; every one of them arrives after its own F, nothing
                          // else: the lean kernel's wait is r03's tight loop, the delayed ones are bounded)
          if constexpr (kDelays) {
            unsigned spins = 0;
            while (__hip_atomic_load(&sh.crit_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < kCritWaves) {
              if (++spins > 4 * kSpinLimit) {
                sh.stop = 1;
                atomicOr(a.fail, 32);  // (bit 2 is PWR's key-field overflow)
                break;
              }
              __builtin_amdgcn_s_sleep(0);
            }
          } else {
            while (__hip_atomic_load(&sh.crit_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < kCritWaves)
              __builtin_amdgcn_s_sleep(0);
          }
          sh.crit_done = 0;
          if (prof) sh.prof[17] += __builtin_amdgcn_s_memrealtime() - t_loaded;
          if (trace && step < a.trace_steps)
            trace[((size_t)blockIdx.x * a.trace_steps + step) * kTrace + 3] = __builtin_amdgcn_s_memrealtime();
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        const bool cshare = is_share_pod(cp);
        const unsigned fm = cshare ? (dfirst & ge_mask(dn, cp.milli)) : 0u;
        const bool has = lane >= 1 && lane <= 8 && (cshare ? ((fm >> (lane - 1)) & 1u) != 0u : lane == 1);
        int k = 0;
        if (has) k = (int)pack_key32(score_of(sh.Fc[0] - sh.Fc[lane]), d, cshare ? 15 - (lane - 1) : 0);
        const unsigned gk = (unsigned)ksim_replay::wave_max_dpp(k);
        const unsigned z = pack_key32(0, d, 0);  // feasible with no fitting GPU
        gk_crit = gk > z ? gk : z;
        fresh = ofeas ? gk_crit : 0u;
        if (prof && tid == 0) sh.prof[18] += __builtin_amdgcn_s_memrealtime() - t_loaded;
        if (trace && lane == 0 && step < a.trace_steps)
          trace[((size_t)blockIdx.x * a.trace_steps + step) * kTrace + 2] = __builtin_amdgcn_s_memrealtime();
      }
      const unsigned W = fresh > ex ? fresh : ex;
      const int rk = W != 0u ? key32_rank(W) : -1;
      // Reserve (open_gpu_share.go:178-205) on the winner: d's record is in registers
      const int gW = key32_gpu(W);
      const int mask = W == 0u ? -1 : (W == ex ? mask_ex : (d_gpu_from_key ? (gW < 0 ? -1 : 1 << gW) : mask_d_pre));
      // bit 1: no feasible node at all (W == 0), as opposed to a Reserve failure on the winner
      const unsigned pay = (W != 0u && mask >= 0) ? pack_pay(rk, mask) : (W == 0u ? 3u : 1u);
      if (lane == 0) {
        gstore32(win + step, pay);
        asm volatile("" ::: "memory");
        if (prof) sh.prof[20] += __builtin_amdgcn_s_memrealtime() - t_loaded;
        if (trace && step < a.trace_steps)
          trace[((size_t)blockIdx.x * a.trace_steps + step) * kTrace + 1] = __builtin_amdgcn_s_memrealtime();
        const int nfeas = cnt_o + (d >= 0 ? (fresh != 0u ? 1 : 0) - (old_own != 0u ? 1 : 0) : 0);
        ResultDev out{-1, 0, 0, nfeas, ST_UNSCHED};
        if (W != 0u) {
          if (mask < 0) {  // Reserve failed: allocateGpuId returned "" / panicked
            out.status = ST_ERROR;
          } else {
            out.status = ST_OK;
            out.score = result_score(rp, nfeas, key32_score(W), 0, 0);
            out.node = rk;  // name rank; k_memo_finish maps it to the node index
            out.gpu_mask = mask;
          }
        }
        gput(rp.res + step, out);
        sh.pay = pay;
        if (prof) sh.prof[19] += __builtin_amdgcn_s_memrealtime() - t_loaded;
      }
      if (d >= 0) {  // every class of the step's score group on d (its own included)
        const int j = lane;
        if (j < Cw && ((sh.grp[crep] >> j) & 1ull)) {
          const PodDev q = sh.cls[j];
          const unsigned nk = filter_node(dn, q) ? gk_crit : 0u;
          unsigned* kp = s_keys + (size_t)j * N + d;
          const unsigned old = *kp;
          *kp = nk;
          sh.cnt[j] += (nk != 0u ? 1 : 0) - (old != 0u ? 1 : 0);
        }
      }
    }
    if (prof && tid == 0 && own) sh.prof[15] += __builtin_amdgcn_s_memrealtime() - t_loaded;  // owner's A
    mark(1);
    __syncthreads();
    mark(2);
    mark(3);
    if (d >= 0) {
      const int nit = __builtin_amdgcn_readfirstlane(sh.nitems);
      if (wv < a.nfw) {
        double* fb = s_fold + (size_t)wv * kFoldBuf;
        for (int it = wv; it < nit; it += a.nfw) {
          const int code = sh.item_code[it];
          const PodDev q = ksim_replay::uniform_pod(&sh.cls[sh.item_slot[it]]);
          int cpuL, total;
          uint32_t gs[4];
          ksim_replay::fgd_candidate(dn, code, q, &cpuL, gs, &total);
          const double F = wave_F(cpuL, gs, total, 1u << dn.gpu_type(), rp.typed != 0, sh.tp, rp.ncpu, rp.nt, lane, fb);
          if (lane == 0) sh.F[it] = F;
        }
      }
    }
    mark(4);
    __syncthreads();
    mark(5);
    // ---- C: the listed requests' keys (list wave)
    if (d >= 0 && wv == kLW) {
      const unsigned long long tl0 = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
      const int nit = __builtin_amdgcn_readfirstlane(sh.nitems);
      const double F0 = own ? sh.Fc[0] : sh.F[0];
      for (int it = (own ? 0 : 1) + lane; it < nit; it += 64) {
        const int code = sh.item_code[it];
        sh.ikey[it] = pack_key32(score_of(F0 - sh.F[it]), d, code <= 8 ? 15 - (code - 1) : 0);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      unsigned gk = r_need ? pack_key32(0, d, 0) : 0u;
      for (int k = 0; k < r_ni; ++k) {
        const unsigned x = sh.ikey[r_base + k];
        gk = x > gk ? x : gk;
      }
      const unsigned gkj = __shfl(gk, l_valid ? l_ref : 0, 64);
      if (l_valid && !r_skip) {
        const unsigned nk = r_feas ? gkj : 0u;
        unsigned* kp = s_keys + (size_t)lane * N + d;
        const unsigned old = *kp;
        *kp = nk;
        sh.cnt[lane] += (nk != 0u ? 1 : 0) - (old != 0u ? 1 : 0);
      }
      if (prof && lane == 0) sh.prof[13] += __builtin_amdgcn_s_memrealtime() - tl0;
    }
    mark(6);
    // ---- top-2 of the next create event's class (its owner), on keys fresh but for this step's node;
    // decider mode: the top list of event step + kLag on keys fresh up to event step - 1
    if constexpr (kDecider) {
      if (step + kLag < rp.n_events) {
        const int ocn = __builtin_amdgcn_readfirstlane(sh.evo[eb + kLag]);
        if (ocn >= 0 && (ocn >> 16) == w) {
          __syncthreads();
          publish_top(ocn & 0xff, step + kLag);
        }
      }
    } else if (step + 1 < rp.n_events) {
      const int ocn = __builtin_amdgcn_readfirstlane(sh.evo[eb + 1]);
      if (ocn >= 0 && (ocn >> 16) == w) {
        __syncthreads();
        top2(ocn & 0xff);
      }
    }
    mark(7);
    if constexpr (kDelays) hdelay(a.delay, 1, step, wv, (int)blockIdx.x);
    // ---- this step's outcome on every workgroup: the Bind (or the delete) on the LDS cluster
    if (wv == 0) {
      int nd_w = -1;
      NodeV nn{};
      if (lane == 0) {
      unsigned pay = 0u;
      int sign = +1;
      PodDev bp = p;
      bool ok = true;
      if (del) {
        sign = -1;
        if (p.ref >= 0 && p.ref < step) {
          pay = gload32(win + p.ref);  // written before this workgroup passed step p.ref
          bp = gget(rp.ev + p.ref);
        }
      } else if (own) {
        pay = sh.pay;
      } else {
        unsigned spins = 0;
        while ((pay = gload32(win + step)) == 0u) {
          if (++spins > kSpinLimit) { ok = false; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        if (trace && step < a.trace_steps)
          trace[((size_t)blockIdx.x * a.trace_steps + step) * kTrace + 1] = __builtin_amdgcn_s_memrealtime();
      }
      int nd = -1;
      if (kSkip && skip_ok && ok && (pay & 2u))  // this event's class has no feasible node, for good
        sh.dead[p.pad >> 5] |= 1u << (p.pad & 31);
      if (!ok) {
        sh.stop = 1;
        atomicOr(a.fail, 1);
      } else {
        const int rk = (int)((pay >> 8) & 0xffffu) - 1;
        const int mask = (int)(pay >> 24);
        if (rk >= 0) {
          NodeV n = load_node(&s_nodes[rk]);
          bind_node(n, bp, mask, sign);
          store_node(&s_nodes[rk], n);
          store_node(&sh.dnode, n);
          nn = n;
          // (results carry name ranks and the affinity tags are applied by k_memo_finish: nothing
          // here waits on global memory)
          if (del && is_w0) gput(rp.res + step, ResultDev{rk, mask, 0, 0, ST_DELETED});
          if ((kGeneral || kReport) && rp.snap && (del ? is_w0 : own)) {  // cluster report: the state this event left
            gput_node(rp.snap + step, n);
            gput(rp.prev + step, s_last[rk]);
          }
          s_last[rk] = step;
          nd = rk;
        } else if (del && is_w0) {
          gput(rp.res + step, ResultDev{-1, 0, 0, 0, ST_DELETED});
        }
      }
      sh.dirty = nd;
      nd_w = nd;
      }  // lane 0
      // the first-occurrence GPU mask of the changed node, for the next step's candidate lists
      nd_w = __builtin_amdgcn_readfirstlane(nd_w);
      if (nd_w >= 0) {
        NodeV u;
        u.cpu_left = __builtin_amdgcn_readfirstlane(nn.cpu_left);
        u.mem_left = __builtin_amdgcn_readfirstlane(nn.mem_left);
#pragma unroll
        for (int i = 0; i < 4; ++i) u.g[i] = __builtin_amdgcn_readfirstlane(nn.g[i]);
        u.meta = __builtin_amdgcn_readfirstlane(nn.meta);
        u.name_rank = __builtin_amdgcn_readfirstlane(nn.name_rank);
        const unsigned fmk = first_mask_lanes(u, lane);
        if (lane == 0) sh.dfirst = fmk;
      }
    }
    mark(8);
    __syncthreads();
    mark(9);
    if (sh.stop) break;
  }
  if (prof && tid == 0) {
    sh.prof[10] = __builtin_amdgcn_s_memtime() - c_start;
    sh.prof[11] = __builtin_amdgcn_s_memrealtime() - t_start;
  }
  __syncthreads();
  if (prof && tid < kProfPhases) a.prof[(size_t)blockIdx.x * kProfPhases + tid] = sh.prof[tid];
  // final cluster state
  if (is_w0 && !sh.stop)
    for (int i = tid; i < N; i += kMBlock) store_node(rp.nodes + rank2idx[i], load_node(&s_nodes[i]));
}

// After k_memo: results carry name ranks -> node indices, and every Bind / delete adds its pod's
// affinity tag (pod.go:111-123) to the node's counts (commutative u32 atomics on the packed u16
// pairs: any transient borrow between the halves cancels, the final counts are exact).
__global__ void k_memo_finish(ReplicaDev* reps, const int* rep_list, int N) {
  const ReplicaDev rp = reps[rep_list[blockIdx.y]];
  const int e = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (e >= rp.n_events) return;
  const int* rank2idx = reinterpret_cast<const int*>(rp.tags + (size_t)N * kTagStride);
  ResultDev r = rp.res[e];
  if (r.node < 0) return;
  const int idx = rank2idx[r.node];
  rp.res[e].node = idx;
  const PodDev p = rp.ev[e];
  const bool del = (p.flags & kPodDelete) != 0u;
  if (!(del ? r.status == ST_DELETED : r.status == ST_OK)) return;
  const int tag = del ? rp.ev[p.ref].tag : p.tag;
  if (tag < 0) return;
  const size_t h = (size_t)idx * kTagStride + tag;
  unsigned* word = reinterpret_cast<unsigned*>(rp.tags) + (h >> 1);
  atomicAdd(word, (unsigned)(del ? -1 : 1) << (16 * (h & 1)));
}

// LDS bytes of k_memo's dynamic region (must match the carving in the kernel).
inline size_t memo_lds(int N, int Cw, int nfw, bool hkeys = false) {
  const size_t keys = hkeys ? 0 : (std::max((size_t)Cw * N * 4, sizeof(DeciderScratch)) + 15) & ~(size_t)15;
  const size_t fold = std::max((size_t)nfw * kFoldBuf * 8, ((size_t)N * 8 + 15) & ~(size_t)15);
  return sizeof(MemoShared) + (size_t)N * sizeof(NodeRec) + keys + fold + (size_t)N * 4;
}

}  // namespace ksim_memo

// ksim_hmemo.hpp -- memoised FGD replay with the (pod class, node) keys in HBM (k_hmemo).
//
// k_memo (ksim_memo.hpp) keeps every (class, node) key of a replica in LDS, spread over K
// co-resident workgroups, so it only fits when the replica's classes x nodes fit K x 160 KB and
// K x replicas <= CUs.  The paper sweep's 170 FGD replicas (one workgroup each) and the 100k-node
// C5 cluster do not, and fell back to k_replay, which re-scores every node per pod.
//
// k_hmemo runs ONE workgroup per replica (no cross-workgroup exchange, hence no co-residency
// requirement) and keeps:
//   HBM   key[c][rank]            the packed key of every (class, node) pair (hkey below)
//   LDS   L1[c][b] = max key[c][64b .. 64b+63]    (a max tree of fan-out 64, one level: N <= 4096)
//         the cluster (node slot = name rank), the class table, the typical table.
// Per pod step, with d = the node changed by the previous event (its Bind or a delete):
//   1. wave 0 lists the F evaluations: d's current state + every score group's candidates (groups:
//      same cpu_nz, milli, num, hence the same candidate states, fgd_score.go:99-149; one candidate
//      per distinct milli-left value among the fitting GPUs, or the NodeResource.Sub state), while
//      waves 1-15 run the class pass: Filter on d's new and old records (feasible counts) and which
//      classes had d as the max of d's block (flagged);
//   2. every quarter-wave issues the HBM load of one flagged class's 64-key block (held in
//      registers), every quad of lanes evaluates one state's F (frag_F_quad, bit-exact with
//      frag.go), then the quarter-waves take their blocks' maxima without d (DPP);
//   3. class pass: the class's group key on d (score steps of its candidates), key[c][d] (HBM
//      store), L1[c][d/64] (max with the new key, or the block max without d when d was the block
//      max), the feasible count;
//   4. wave 0: the winner of the event's class = max over L1[class][*] (selectHost: max score, ties
//      to the smallest name), Reserve's GPU selector on it, the Bind in LDS, the result.
// Every key of every class is fresh at step 4, so the decision is the one k_replay / k_step / the
// oracle make (same device functions: filter_node, fgd_candidate + frag_F_quad, the score table).
//
// Keys are produced before the run by k_hinit_gk / k_hinit_keys: one evaluation per (group,
// distinct initial node state), then key = Filter ? that score with the node's rank : 0.
//
// Wide clusters (C5: 100k nodes; one level of L1 covers 4096): K > 1 co-resident workgroups per
// replica, workgroup w owning the ranks [w S, w S + S) (S a multiple of 64, so no L1 block straddles
// two workgroups) -- their records and the L1 of their blocks in LDS; the keys stay in HBM.  Per
// pod step only the owner of d refreshes (steps 1-3); at step 4 every workgroup takes its slice's
// max key and feasible count of the event's class, publishes them as two {tag, value} granules,
// polls all K (k_replay's exchange), and the owner of the global winner runs Reserve + Bind.  A
// delete is undone by the workgroup that bound the creation (a per-workgroup bind history).
#pragma once

namespace ksim_hmemo {

using namespace ksim;

constexpr int kHBlock = 1024;
constexpr int kHWaves = kHBlock / 64;
constexpr int kFan = 64;              // keys per L1 block (one wave / one quarter-wave dwordx4 row)
constexpr int kMaxNb = 64;            // L1 blocks per class (N <= 4096)
constexpr int kMaxClasses = 1024;     // one class-pass thread each
constexpr int kMaxGroups = 128;
constexpr int kMaxItems = 1 + 8 * kMaxGroups;
constexpr int kEvBuf = 128;
constexpr int kQuarters = kHBlock / 16;
constexpr int kMaxPeers = 16;  // shard processes of a device exchange (ksim_engine_set_shard: world <= 16)
constexpr int kFW = 7;                 // F waves of the bulk refresh (1..kFW: 112 quads, one listed state each)
constexpr int kCW = kHWaves - 1 - kFW; // class waves (kFW+1..15)

// Packed key of (class, node): [30:24] score + 1 | [23:4] kHRankMax - rank | [3:0] gpu field
// (15 - g for a share pod placed on GPU g, 0 otherwise).  0 = infeasible.  Max key = max score,
// ties to the smallest name (selectHost, generic_scheduler.go:187-212); over one node's candidates
// the max keeps the lowest GPU index reaching the max (fgd_score.go:128).  Non-negative as int32.
constexpr int kHRankMax = (1 << 20) - 1;
KSIM_HD unsigned hkey(int score, int rank, int gf) {
  return ((unsigned)(score + 1) << 24) | ((unsigned)(kHRankMax - rank) << 4) | (unsigned)gf;
}
// The key without its rank field (k_hinit_gk); hkey(s, r, g) == hkey_norank(s, g) | hkey_rankbits(r).
KSIM_HD unsigned hkey_norank(int score, int gf) { return ((unsigned)(score + 1) << 24) | (unsigned)gf; }
KSIM_HD unsigned hkey_rankbits(int rank) { return (unsigned)(kHRankMax - rank) << 4; }
KSIM_HD int hkey_score(unsigned k) { return (int)(k >> 24) - 1; }
KSIM_HD int hkey_rank(unsigned k) { return kHRankMax - (int)((k >> 4) & (unsigned)kHRankMax); }
KSIM_HD int hkey_gpu(unsigned k) {
  const int gf = (int)(k & 15u);
  return gf ? 15 - gf : -1;
}

struct HMemoArgs {
  ReplicaDev* reps;
  const int* rep_list;      // replica of each launch workgroup
  int N, Npad, nb;          // nodes, padded to kFan, L1 blocks per class
  int Cmax, Gmax;           // class / group table strides
  const int* cg;            // [Rg][2] classes, groups
  const PodDev* cls;        // [Rg][Cmax] class requests, sorted by group
  const uint16_t* cgrp;     // [Rg][Cmax] group of each class
  const PodDev* gpod;       // [Rg][Gmax] a request of each group (the score part is the group's)
  const int* evc;           // [Rg][stride] class of each event, -1 delete
  int stride;
  unsigned* keys;           // [Rg][Cmax][Npad]
  const unsigned* l1;       // [Rg][Cmax][nb] initial L1 (k_hinit_keys)
  const unsigned* l2;       // [Rg][Cmax][nb] initial second maxima, or null: no L2 (it does not fit in LDS)
  const int* cnt0;          // [Rg][Cmax] initial feasible counts
  const double* th;         // [102] FGD score steps
  unsigned long long* prof; // optional [Rg * K][kHProf] (KSIM_PROFILE=1)
  int K, S, nbw;            // workgroups per replica, ranks per workgroup, L1 blocks per workgroup
  unsigned long long* gran; // K > 1: [Rg][2][K][2] exchange granules {tag, value}
  uint8_t* hist;            // K > 1 with deletes: [Rg][K][stride] 1 bound here, 2 Reserve failed here, 3 no winner,
                            // 4 bound in another shard
  int* fail;                // K > 1: a granule poll timed out
  // Node-sharded cluster (several engines, one per shard, in one exchange): every launch workgroup is
  // workgroup w of its shard, granule column wbase + w of Ktot; the shard's ranks are global rank - roff
  // (keys carry the global rank, so selectHost's tie-break spans the shards).  Unsharded: 0, 0, K.
  int roff, wbase, Ktot;
  const TypDev* tp;         // the typical tables (k_hmemo_group: per shard; k_hmemo: the kernel argument)
  // One shard per process / GPU (ksim_engine_set_shard_peers): `gran` is this shard's own exchange buffer
  // (uncached device memory), peer[q] shard q's buffer mapped here (IPC; own included); each step's
  // granules are stored into every peer's buffer (system scope, over xGMI) and polled in the own one.
  // epoch (24 bits, never 0 with peers) tags a run's granules (no reset between runs, so no rank can clear
  // a granule a peer already wrote).  npeer = 0: the exchange buffer is shared in place (one launch).
  int npeer, epoch;
  unsigned long long* peer[kMaxPeers];
  int skip;                 // the dead-class skip (create-only streams; class slots < 1024)
  int pf;                   // one workgroup per replica: 1 (default) = wave 0 lists the next refresh's F evaluations after its
                            // Bind, 2 = it also touches the next refresh's flagged key rows (KSIM_VARIANT hpf)
  int delay;                // the hdelay test knob (general instantiation only): hand-over stress delays, hdelay() below
  int prune_t;              // list only the score groups some class of which may pass Filter on d (the group's
                            // PodDev holds the least demanding request: min CPU / memory, every accepted GPU
                            // model) for replicas with more than prune_t typical pods (KSIM_VARIANT hprune)
  // Residency gate (a concurrent run's FGD group): each workgroup stores `gate_epoch` into started[its
  // index] (host memory) as it starts, so the host launches the short groups only once every long replay
  // holds its CU.  Null: no gate.
  int* started;
  int gate_epoch;
  // Per-model tables (typed replicas, null otherwise): mtoff[gi][model] = kMtPresent | slot << 21 | entries << 12 |
  // offset into mtab[gi][.] (typical-table indices: the CPU-only pods, then the GPU pods accepting the model, in
  // table order); na[gi][slot][total] = the NA bin of every state of that model with `total` milli-GPU left
  // (k_hinit_na).  Mtab: mtab's stride; Mslots: na's.
  const int* mtoff;
  const uint8_t* mtab;
  const double* na;
  int Mtab, Mslots;
};
constexpr uint32_t kMtPresent = 1u << 31;
constexpr int kNaStride = 8008;  // totals 0 .. 8 x 1000 (kMaxGpu x kMilli), padded
constexpr int kHProf = 16;  // 0-6 phase sums, 7 items, 8 flagged classes, 9 refresh steps, 10 clock, 11 wall

struct __align__(16) HShared {
  PodDev ev[kEvBuf];
  int evc[kEvBuf];
  TypDev tp[kMaxTypical];
  double th[104];
  // The node the previous decided event changed (record before / after, its rank or -1, first_of_class
  // of the new record), double-buffered: the bulk reads [cur] while wave 0's decision writes [cur ^ 1].
  NodeRec dold[2], dnew[2];
  int d[2];
  unsigned dfirst[2];
  int nitems[2];       // the F list's length (double-buffered)
  int nflag;
  int stop;            // K > 1: a poll timed out, every workgroup leaves its loop
  int bar;             // the bulk waves' barrier counter
  int cbar;            // the class waves' barrier counter
  int lseq;            // the F list's hand-over: refreshes listed so far
  // The class the last decided step found dead (-1 none), double-buffered like d: wave 0's decision runs
  // while slower waves may still be reading this step's skip condition, so it writes [cur ^ 1] and folds
  // [cur] into `dead`; every reader checks dead | pdead[cur] (the same answer before and after the fold).
  int pdead[2];
  int f0seq;           // refreshes whose item 0 (d's current state) has its F in s_F[0] (the item keys' reference)
  int pad_[2];
  unsigned long long prof[kHProf];
  unsigned dead[32];   // class slots with no feasible node (create-only streams: for good)
};
static_assert(sizeof(HShared) % 16 == 0, "keep the dynamic regions 16-B aligned");

// Dynamic LDS after HShared (16-B aligned regions).
struct HLayout {
  size_t cls, gpod, F, l1, l2, nodes, last, cnt, bx, bx2, cgrp, flist, code, igrp, fnew, fold, gbase, gkey, ctp, mto, total;
};
KSIM_HD size_t halign(size_t x) { return (x + 15) & ~(size_t)15; }
KSIM_HD HLayout hmemo_layout(int N, int Cmax, int Gmax, int nb, bool l2, int Mtab) {
  HLayout L;
  size_t o = sizeof(HShared);
  L.cls = o;   o = halign(o + (size_t)Cmax * sizeof(PodDev));
  L.gpod = o;  o = halign(o + (size_t)Gmax * sizeof(PodDev));
  L.F = o;     o = halign(o + (size_t)kMaxItems * sizeof(double));
  L.l1 = o;    o = halign(o + (size_t)Cmax * nb * 4);
  L.l2 = o;    o = halign(o + (l2 ? (size_t)Cmax * nb * 4 : 0));
  L.nodes = o; o = halign(o + (size_t)N * sizeof(NodeRec));
  L.last = o;  o = halign(o + (size_t)N * 4);
  L.cnt = o;   o = halign(o + (size_t)Cmax * 4);
  L.bx = o;    o = halign(o + (size_t)Cmax * 4);
  L.bx2 = o;   o = halign(o + (l2 ? (size_t)Cmax * 4 : 0));
  L.cgrp = o;  o = halign(o + (size_t)Cmax * 2);
  L.flist = o; o = halign(o + (size_t)Cmax * 2);
  L.code = o;  o = halign(o + (size_t)2 * kMaxItems);  // the F list, double-buffered like d's records
  L.igrp = o;  o = halign(o + (size_t)2 * kMaxItems);
  L.fnew = o;  o = halign(o + (size_t)Cmax);
  L.fold = o;  o = halign(o + (size_t)Cmax);
  L.gbase = o; o = halign(o + (size_t)Gmax * 2 * 2);
  L.gkey = o;  o = halign(o + (size_t)Gmax * 2 * 4);  // every score group's key on d, double-buffered like the list
  L.ctp = o;   o = halign(o + (size_t)Mtab * sizeof(TypDev));  // the per-model tables (typed replicas)
  L.mto = o;   o = halign(o + (Mtab > 0 ? (size_t)KSIM_MAX_TYPES * 4 : 0));
  L.total = o;
  return L;
}

// Global-address-space access (flat loads / stores also count in lgkmcnt, so every later LDS wait
// would stall on them; global_* ones count in vmcnt only).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld4(const unsigned* p) {
  const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gst1(unsigned* p, unsigned v) {
  *(__attribute__((address_space(1))) unsigned*)(p) = v;
}

// A node record reduced to what filter_node reads per class (computed once per refresh), and the
// Filter from it: the same decisions as filter_node (ksim_device.hpp; fit.go:230-290,
// open_gpu_share.go:81-118) with the per-GPU scans done once instead of once per class.  The
// multi-GPU request with a partial milli (no trace has one) takes filter_node itself.
struct NodeSum {
  int pods_left, cpu_left, mem_left, cnt, type_bit, max_left, free_cnt;
};
__device__ __forceinline__ NodeSum node_sum(const NodeV& n) {
  NodeSum s;
  s.pods_left = n.pods_left();
  s.cpu_left = n.cpu_left;
  s.mem_left = n.mem_left;
  s.cnt = n.gpu_cnt();
  s.type_bit = 1 << n.gpu_type();
  int mx = 0, fr = 0;
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) {
    const int l = g < s.cnt ? n.gl(g) : 0;
    mx = l > mx ? l : mx;
    fr += l == kMilli ? 1 : 0;
  }
  s.max_left = mx;
  s.free_cnt = fr;
  return s;
}
// Branch-free except for the partial-milli multi-GPU request (the class pass runs it for every class
// of the replica, one class per thread, so a divergent early-return chain would serialise the wave).
__device__ __forceinline__ bool filter_sum(const NodeSum& s, const NodeV& n, const PodDev& p) {
  const bool res_ok = (p.cpu_req == 0 && p.mem == 0) || (s.cpu_left >= p.cpu_req && s.mem_left >= p.mem);
  const bool dev_ok = s.cnt != 0 && (p.tmask & (unsigned)s.type_bit) != 0u && p.num > 0;
  const bool fits = p.num == 1 ? s.max_left >= p.milli : s.free_cnt >= p.num;  // whole GPUs when num > 1
  bool ok = s.pods_left >= 1 && res_ok && (p.milli <= 0 || (dev_ok && fits));
  if (p.milli > 0 && p.num > 1 && p.milli != kMilli) ok = filter_node(n, p);  // partial multi-GPU: no trace has one
  return ok;
}

// Row (16-lane) max of unsigned values below 2^31: every lane of the row ends with it.
__device__ __forceinline__ int row_max16(int v) {
  using ksim_replay::dpp_i;
  v = max(v, dpp_i<0xB1>(v));
  v = max(v, dpp_i<0x4E>(v));
  v = max(v, dpp_i<0x141>(v));
  v = max(v, dpp_i<0x140>(v));
  return v;
}

// Max of a 64-key block row held as one uint4 per lane of a 16-lane row, the key of node `d`
// excluded (lane l16 holds nodes base + 4 l16 .. base + 4 l16 + 3).
__device__ __forceinline__ unsigned block_max_excl(const uint4& v, int base, int l16, int d) {
  const int n0 = base + 4 * l16;
  unsigned m = 0u;
  m = (n0 + 0 != d && v.x > m) ? v.x : m;
  m = (n0 + 1 != d && v.y > m) ? v.y : m;
  m = (n0 + 2 != d && v.z > m) ? v.z : m;
  m = (n0 + 3 != d && v.w > m) ? v.w : m;
  return (unsigned)row_max16((int)m);
}

// the hdelay test knob stress delays (ksim_memo::hdelay).  Bits here: 1 waves 1-15 before reading the step's
// skip condition (the r03 dead-set race: wave 0 decides and marks the class dead first), 2 wave 1 before
// its F list (the F waves wait on the list hand-over), 4 wave 0 before its decision (the bulk finishes the
// step first), 8 the class waves before the class pass.  Results must not change (tests/test_gpu_hdelay.py).
using ksim_memo::hdelay;

// The top two keys of a 64-key block row (one uint4 per lane of a 16-lane row), node d's excluded: every
// lane of the row ends with them (the quad / half-row / row DPP merges of wave_top2: disjoint halves).
__device__ __forceinline__ void block_top2_excl(const uint4& v, int base, int l16, int d, unsigned& m1, unsigned& m2) {
  const int n0 = base + 4 * l16;
  const unsigned x[4] = {n0 + 0 != d ? v.x : 0u, n0 + 1 != d ? v.y : 0u, n0 + 2 != d ? v.z : 0u, n0 + 3 != d ? v.w : 0u};
  unsigned a1 = 0u, a2 = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (x[i] > a1) { a2 = a1; a1 = x[i]; } else if (x[i] > a2) { a2 = x[i]; }
  }
  ksim_memo::merge2_dpp<0xB1>(a1, a2);
  ksim_memo::merge2_dpp<0x4E>(a1, a2);
  ksim_memo::merge2_dpp<0x141>(a1, a2);
  ksim_memo::merge2_dpp<0x140>(a1, a2);
  m1 = a1;
  m2 = a2;
}

// L2: the second-largest key of each (class, block) beside L1's largest, so that the block's new maximum
// is known without reloading its 64 keys when the node d that held the maximum changes (the flagged rows
// of the class pass).  kL2Stale: unknown -- set when d held the maximum and dropped below the second, or
// held the second and dropped (the new second is then max(d's key, the third)); a reload (the flagged row)
// is needed only when d holds the maximum of a block whose second is unknown.  dr: d's key rank; k its new
// key; x1, x2: the reloaded row's top two without d (used only when m2 is stale and d held the max).
constexpr unsigned kL2Stale = 0xFFFFFFFFu;  // (keys are below 2^31)
__device__ __forceinline__ void l12_update(unsigned& m1, unsigned& m2, unsigned k, int dr, unsigned x1, unsigned x2) {
  const unsigned o1 = m1, o2 = m2;
  const bool stale = o2 == kL2Stale;
  if (o1 != 0u && hkey_rank(o1) == dr) {  // d held the maximum
    if (stale) { m1 = k > x1 ? k : x1; m2 = k > x1 ? x1 : (k > x2 ? k : x2); }
    else if (k >= o2) { m1 = k; }
    else { m1 = o2; m2 = kL2Stale; }
  } else if (!stale && o2 != 0u && hkey_rank(o2) == dr) {  // d held the second
    if (k > o1) { m1 = k; m2 = o1; }
    else if (k >= o2) { m2 = k; }
    else { m2 = kL2Stale; }
  } else {
    if (k > o1) { m1 = k; m2 = o1; }  // (the old maximum is the largest of the others: exact even when stale)
    else if (!stale && k > o2) { m2 = k; }
  }
}

// kSub = ceil(K / 64): the granule columns one polling lane reads (K > 1); kSub = 0: the lean one-
// workgroup form (K = 1, the exchange compiled out).  kProf: the general instantiation -- the
// KSIM_PROFILE phase timers and the the hdelay test knob stress delays (compiled out of the lean launches, as
// k_memo's: the step loop's scalar registers are what it runs short of).
// kModel: the instantiation for large typical tables -- the per-model tables (typed replicas) and the F-list
// pruning (one workgroup per replica)
template <int kSub, bool kProf, bool kModel = false>
__device__ __forceinline__ void hmemo_body(const HMemoArgs& a, const TypDev* __restrict__ tp_all, const int wg) {
  using namespace ksim_replay;
  using ksim_memo::gget;
  using ksim_memo::gput;
  using ksim_memo::gput_node;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  HShared& sh = *reinterpret_cast<HShared*>(smem);
  constexpr int kS = kSub > 0 ? kSub : 1;
  const int K = kSub == 0 ? 1 : a.K;
  const int Kt = kSub == 0 ? 1 : a.Ktot;  // granule columns of the exchange (every shard's workgroups)
  const int roff = kSub == 0 ? 0 : a.roff;
  const bool sharded = Kt > K;
  const int gi = wg / K, w = wg % K;
  const int r = a.rep_list[gi];
  const ReplicaDev rp = a.reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = a.N, nb = a.nbw;  // nb: L1 blocks of this workgroup's slice
  const int lo = w * a.S, ns = min(a.S, N - lo), b0 = lo / kFan;
  const int C = a.cg[2 * gi], G = a.cg[2 * gi + 1];
  // L2 is compiled into the one-workgroup instantiations only (KSIM_VARIANT hl2=1): in the wide form its code alone cost C5
  // 4.09 -> 4.22 s (r04 bisect, profiles/r05/hmemo/c5_bisect_r05c26.txt), on or off
  constexpr bool kL2Code = kSub == 0;
  const bool use_l2 = kL2Code && a.l2 != nullptr;
  const HLayout L = hmemo_layout(a.S, a.Cmax, a.Gmax, nb, use_l2, a.Mtab);
  PodDev* s_cls = reinterpret_cast<PodDev*>(smem + L.cls);
  PodDev* s_gpod = reinterpret_cast<PodDev*>(smem + L.gpod);
  double* s_F = reinterpret_cast<double*>(smem + L.F);
  unsigned* s_l1 = reinterpret_cast<unsigned*>(smem + L.l1);
  unsigned* s_l2 = reinterpret_cast<unsigned*>(smem + L.l2);   // use_l2 only
  unsigned* s_bx2 = reinterpret_cast<unsigned*>(smem + L.bx2); // use_l2 only
  NodeRec* s_nodes = reinterpret_cast<NodeRec*>(smem + L.nodes);
  int* s_last = reinterpret_cast<int*>(smem + L.last);
  int* s_cnt = reinterpret_cast<int*>(smem + L.cnt);
  unsigned* s_bx = reinterpret_cast<unsigned*>(smem + L.bx);
  uint16_t* s_cgrp = reinterpret_cast<uint16_t*>(smem + L.cgrp);
  uint8_t* const s_code_b = reinterpret_cast<uint8_t*>(smem + L.code);
  uint8_t* const s_igrp_b = reinterpret_cast<uint8_t*>(smem + L.igrp);
  uint8_t* s_fnew = reinterpret_cast<uint8_t*>(smem + L.fnew);
  uint8_t* s_fold = reinterpret_cast<uint8_t*>(smem + L.fold);
  int16_t* const s_gbase_b = reinterpret_cast<int16_t*>(smem + L.gbase);
  unsigned* const s_gkey_b = reinterpret_cast<unsigned*>(smem + L.gkey);
  uint16_t* s_flist = reinterpret_cast<uint16_t*>(smem + L.flist);
  TypDev* s_ctp = reinterpret_cast<TypDev*>(smem + L.ctp);
  int* s_mto = reinterpret_cast<int*>(smem + L.mto);
  const int* rank2idx = reinterpret_cast<const int*>(rp.tags + (size_t)N * kTagStride);
  unsigned* keys = a.keys + (size_t)gi * a.Cmax * a.Npad;
  const int* evc = a.evc + (size_t)gi * a.stride;
  unsigned long long* gr = Kt > 1 ? a.gran + (size_t)gi * 2 * Kt * 2 : nullptr;
  const int col = (kSub == 0 ? 0 : a.wbase) + w;  // this workgroup's granule column
  uint8_t* hist = (Kt > 1 && a.hist) ? a.hist + ((size_t)gi * K + w) * a.stride : nullptr;

  // ---- start-up: the slice (slot = rank - lo), classes, groups, typical table, score steps, L1, counts
  for (int i = tid; i < ns; i += kHBlock) {
    store_node(&s_nodes[i], load_node(rp.nodes + rank2idx[lo + i]));
    s_last[i] = -1;
  }
  for (int c = tid; c < C; c += kHBlock) {
    s_cls[c] = a.cls[(size_t)gi * a.Cmax + c];
    s_cgrp[c] = a.cgrp[(size_t)gi * a.Cmax + c];
    if (K == 1) s_cnt[c] = a.cnt0[(size_t)gi * a.Cmax + c];
  }
  if (K > 1) {  // the slice's feasible count of every class (the initial keys hold the Filter)
    for (int c = wv; c < C; c += kHWaves) {
      int n = 0;
      for (int i = lane; i < ns; i += 64) n += gget(keys + (size_t)c * a.Npad + lo + i) != 0u ? 1 : 0;
      n = wave_sum_dpp(n);
      if (lane == 0) s_cnt[c] = n;
    }
  }
  for (int g = tid; g < G; g += kHBlock) {
    s_gpod[g] = a.gpod[(size_t)gi * a.Gmax + g];
  }
  for (int i = tid; i < C * nb; i += kHBlock) {
    const bool in = b0 + i % nb < a.nb;
    const size_t gix = ((size_t)gi * a.Cmax + i / nb) * a.nb + b0 + i % nb;
    s_l1[i] = in ? a.l1[gix] : 0u;
    if (use_l2) s_l2[i] = in ? a.l2[gix] : 0u;
  }
  for (int i = tid; i < rp.nt * 2; i += kHBlock) reinterpret_cast<uint4*>(sh.tp)[i] = reinterpret_cast<const uint4*>(tp)[i];
  if (kModel && a.Mtab > 0) {  // the per-model tables: copies of the entries they name (the table in HBM, as above)
    for (int i = tid; i < a.Mtab * 2; i += kHBlock)
      reinterpret_cast<uint4*>(s_ctp)[i] = reinterpret_cast<const uint4*>(tp + a.mtab[(size_t)gi * a.Mtab + i / 2])[i & 1];
    for (int m = tid; m < KSIM_MAX_TYPES; m += kHBlock) s_mto[m] = rp.typed ? a.mtoff[(size_t)gi * KSIM_MAX_TYPES + m] : 0;
  }
  for (int i = tid; i < 102; i += kHBlock) sh.th[i] = a.th[i];
  if (tid == 0) { sh.d[0] = sh.d[1] = -1; sh.nitems[0] = sh.nitems[1] = 0; sh.nflag = 0; sh.dfirst[0] = sh.dfirst[1] = 0u; sh.stop = 0; sh.bar = 0; sh.cbar = 0; sh.lseq = 0; sh.pdead[0] = sh.pdead[1] = -1; sh.f0seq = 0; }
  // the residency gate (C4): this workgroup has started -- a vector store to host memory, system scope.  In the
  // one-workgroup instantiations it is stored here, not at the kernel's entry: there it took them from 8 to 57
  // VGPR spills (C2 run_mode 5 48.7 -> 47.2 ms here); the wide form keeps it at the entry (C5 measured no better
  // with it here, profiles/r05/hmemo/ab_r05c30_gate_store.txt)
  if (kSub == 0 && a.started != nullptr && tid == 0)
    __hip_atomic_store(a.started + blockIdx.x, a.gate_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int i = tid; i < 32; i += kHBlock) sh.dead[i] = 0u;
  const bool prof = kProf && a.prof != nullptr;
  if (prof && tid < kHProf) sh.prof[tid] = 0ull;
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
  // the bulk waves' phase timer (thread 64)
  unsigned long long tb_last = t_last;
  auto bmark = [&](int ph) {
    if (prof && tid == 64) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      sh.prof[ph] += t - tb_last;
      tb_last = t;
    }
  };
  const bool typed = rp.typed != 0;
  int cur = 0;         // the d-record buffer of this step (toggled at the end of every decided step)
  int bar_target = 0;  // the bulk barrier's count so far (waves 1-15)
  int cbar_target = 0; // the class waves' barrier count so far
  int list_seq = 0;    // refreshes whose F list wave 1 handed over (waves 1..fw)
  // F waves (1..fw) and class waves (fw+1..15); r04 measured 8-10 F waves for the large tables (KSIM_HFW, removed
  // in r05) within C4's spread
  const int fw = kFW, cw = kHWaves - 1 - fw;
  // (the instantiations for large tables only: compiled into the wide form it measured slower at C5, and into
  // the lean untyped one it cost C2 run_mode 5 registers)
  const bool prune = kModel && rp.nt > a.prune_t;
  // F of a candidate state of node n (fgd_candidate's cpuL / gs / total) by the quad of lane q.  A typed replica
  // with per-model tables evaluates only the CPU-only pods and the GPU pods that accept n's model: every other
  // GPU pod adds its freq x total to the NA bin and nothing else (GetNodePodFrag, frag.go:460-493), so the NA
  // bin -- added last in FragAmountSumExceptQ3 (frag.go:411-418) -- is the same sequential sum for every state
  // of the model with that total: na[slot][total] (k_hinit_na).  Same bits as the whole table.
  auto state_F = [&](const NodeV& n, int cpuL, const uint32_t (&gs)[4], int total, int q) -> double {
    const uint32_t tb = 1u << n.gpu_type();
    if constexpr (kModel) {  // (the instantiations without it -- the wide form, C5 -- keep r04's registers)
      // (a launch of this instantiation for the pruning alone has no tables: s_mto is then not allocated)
      const unsigned mw = a.Mtab > 0 ? (unsigned)s_mto[n.gpu_type()] : 0u;
      if (mw & kMtPresent) {
        const double nav = a.na[((size_t)gi * a.Mslots + ((mw >> 21) & 31u)) * kNaStride + total];
        const double F = frag_F_quad<false>(cpuL, gs, total, tb, tp, s_ctp + (mw & 0xfffu), rp.ncpu, (int)((mw >> 12) & 0x1ffu), q);
        return F + nav;
      }
    }
    return typed ? frag_F_quad<true>(cpuL, gs, total, tb, tp, sh.tp, rp.ncpu, rp.nt, q)
                 : frag_F_quad<false>(cpuL, gs, total, tb, tp, sh.tp, rp.ncpu, rp.nt, q);
  };
  // wave 0 lists the next refresh's F evaluations (one workgroup per replica; the wide form too with bit 4)
  const bool w0list = (kSub == 0 || (a.pf & 4) != 0) && (a.pf & 1) != 0;
  const bool w0pf = kSub == 0 && (a.pf & 2) != 0;    // and touches its flagged key rows
  // A bounded wait on one of the bulk's LDS counters (lane 0 of a wave): past the limit the workgroup
  // stops with a failure bit (4 bulk barrier, 8 class barrier, 16 list hand-over, 32 item 0's F hand-over)
  // instead of hanging.
  auto spin_until = [&](int* ctr, int target, int bit, int step_, int d_) {
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
      if (++spins > 4 * ksim_replay::kSpinLimit) {
        printf("ksim hmemo wait timeout: blk %d wave %d bit %d step %d d %d cur %d target %d ctr %d | bar %d cbar %d lseq %d "
               "nflag %d nitems %d %d d[] %d %d\n",
               (int)blockIdx.x, wv, bit, step_, d_, cur, target, *ctr, sh.bar, sh.cbar, sh.lseq, sh.nflag, sh.nitems[0],
               sh.nitems[1], sh.d[0], sh.d[1]);
        atomicOr(a.fail, bit);
        __hip_atomic_store(&sh.stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      __builtin_amdgcn_s_sleep(0);
    }
  };
  int seq = 0;  // K > 1: exchanges so far (wave 0; every workgroup sees the same events)

  for (int step = 0; step < rp.n_events; ++step) {
    const int eb = step & (kEvBuf - 1);
    if (eb == 0) {
      const int ne = min(kEvBuf, rp.n_events - step);
      const uint4* src = reinterpret_cast<const uint4*>(rp.ev + step);
      for (int i = tid; i < ne * 2; i += kHBlock) reinterpret_cast<uint4*>(sh.ev)[i] = gget(src + i);
      for (int i = tid; i < ne; i += kHBlock) sh.evc[i] = gget(evc + step + i);
      __syncthreads();
    }
    // Dead-class skip (create-only streams): Filter is monotone in the resources a creation takes, so an
    // event whose class found no feasible node before finds none now -- unscheduled, 0 feasible, nothing
    // changes.  Every workgroup (every shard) holds the same dead set, taken from the same exchanges, so
    // all skip the same steps; the changed node d is carried to the next decided step's refresh.
    {
      if constexpr (kProf)
        if (wv != 0) hdelay(a.delay, 1, step, wv, wg);
      const int cs0 = __builtin_amdgcn_readfirstlane(sh.evc[eb]);
      const int pd = __builtin_amdgcn_readfirstlane(sh.pdead[cur]);
      if (a.skip && cs0 >= 0 && (cs0 == pd || ((sh.dead[cs0 >> 5] >> (cs0 & 31)) & 1u))) {
        // the whole run of dead events up to the next live one (or the window's end) at once
        const int wend = min(kEvBuf, rp.n_events - (step - eb));
        int run = wend - eb;
        for (int j0 = eb + 1; j0 < wend; j0 += 64) {
          const int j = j0 + lane;
          const int c = j < wend ? sh.evc[j] : 0;
          const unsigned long long lb = __ballot(j < wend && (c < 0 || (c != pd && !((sh.dead[c >> 5] >> (c & 31)) & 1u))));
          if (lb) {
            run = j0 + (int)__builtin_ctzll(lb) - eb;
            break;
          }
        }
        if (w == 0)
          for (int i = tid; i < run; i += kHBlock) gput(rp.res + step + i, ResultDev{-1, 0, 0, 0, ST_UNSCHED});
        __syncthreads();
        step += run - 1;
        continue;
      }
    }
    const int d = __builtin_amdgcn_readfirstlane(sh.d[cur]);  // changed rank in this slice, -1 none
    const int cs = __builtin_amdgcn_readfirstlane(sh.evc[eb]);  // the event's class, -1 delete
    const int own = d >= 0 ? cs : -1;                            // the class wave 0 refreshes itself
    uint8_t* const s_code = s_code_b + cur * kMaxItems;          // this step's F list
    uint8_t* const s_igrp = s_igrp_b + cur * kMaxItems;
    int16_t* const s_gbase = s_gbase_b + cur * a.Gmax;
    unsigned* const s_gkey = s_gkey_b + cur * a.Gmax;
    if (d >= 0 && wv != 0) {
      // ===== the bulk (waves 1-15): every class but the event's own on d, beside wave 0's critical path;
      //       needed from the next decision on.  Three phases, joined by LDS-counter barriers of these
      //       15 waves (wave 0 does not stop for them).
      const NodeV dn = uniform_node(&sh.dnew[cur]);
      const int b = d / kFan - b0;  // the slice's L1 block of d
      const int bt = tid - 64;      // bulk thread
      if (prof && tid == 64) tb_last = __builtin_amdgcn_s_memrealtime();
      auto bulk_bar = [&]() {
        bar_target += kHWaves - 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) {
          __hip_atomic_fetch_add(&sh.bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          spin_until(&sh.bar, bar_target, 4, step, d);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      };
      // ---- 1+2. waves 1..kFW: F of every listed state -- wave 1 lists them (d's current state + each
      //      score group's candidates; a group no class admits just goes unused) and hands the list over
      //      through an LDS counter, then every quad of these waves evaluates one state (frag_F_quad) --
      //      beside waves kFW+1..15: the class pass (Filter on d's new and old records; which classes
      //      had d as the max of d's block: flagged), then the flagged blocks' loads (one quarter-wave
      //      each) and their maxima without d
      if (wv <= fw) {
        ++list_seq;
        if (w0list) {
          // listed by wave 0 after the previous decided step's Bind
        } else if (wv == 1) {
          if constexpr (kProf) hdelay(a.delay, 2, step, wv, wg);
          const unsigned dfirst = __builtin_amdgcn_readfirstlane(sh.dfirst[cur]);
          const NodeSum sd = node_sum(dn);
          int base = 1;  // item 0: d's current state
          for (int g0 = 0; g0 < G; g0 += 64) {
            const int g = g0 + lane;
            unsigned cm = 0u;
            bool share = false;
            if (g < G) {
              const PodDev gp = s_gpod[g];
              share = is_share_pod(gp);
              cm = share ? (dfirst & ksim_memo::ge_mask(dn, gp.milli)) : 0x100u;
              if (prune && !filter_sum(sd, dn, gp)) cm = 0u;  // no class of the group passes Filter on d
            }
            const int nc = __popc(cm);
            int excl = 0, tot = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const unsigned long long m = __ballot((nc >> k) & 1);
              excl += __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << k;
              tot += __popcll(m) << k;
            }
            int o = base + excl;
            if (g < G) {
              s_gbase[g] = (int16_t)o;
              s_gkey[g] = share ? hkey(0, roff + d, 0) : 0u;  // feasible with no fitting GPU; the items max into it
            }
            unsigned mm = cm;
            while (mm) {
              const int x = __builtin_ctz(mm);
              mm &= mm - 1u;
              s_code[o] = (uint8_t)(share ? 1 + x : 9);
              s_igrp[o] = (uint8_t)g;
              ++o;
            }
            base += tot;
          }
          if (lane == 0) {
            s_code[0] = 0;
            s_igrp[0] = 0;
            sh.nitems[cur] = base;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __hip_atomic_store(&sh.lseq, list_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          bmark(0);
        } else {
          if (lane == 0) spin_until(&sh.lseq, list_seq, 16, step, d);
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        const int nit = __builtin_amdgcn_readfirstlane(sh.nitems[cur]);
        const int q = bt & 3;
        // (r05 tried the items round robin over the F waves, so that a short list keeps every SIMD busy: C5
        // 4.25 -> 4.57 s, C2 run_mode 5 48.7 -> 52.6 ms -- the class waves beside the idle F waves lost their
        // issue slots; profiles/r05/hmemo/ab_r05c18_round_robin.txt)
        const int j0 = bt >> 2;
        for (int j = j0; j < nit; j += fw * 16) {
          const int code = s_code[j];
          const PodDev gp = s_gpod[s_igrp[j]];
          int cpuL, total;
          uint32_t gs[4];
          fgd_candidate(dn, code, gp, &cpuL, gs, &total);
          const double F = state_F(dn, cpuL, gs, total, q);
          if (q == 0) s_F[j] = F;
        }
        // every listed candidate's key into its score group's max (LDS atomics), against item 0's F (d's
        // current state: quad 0 of wave 1 publishes it; the other F waves wait for it) -- the class update
        // below then reads one key per class instead of scoring its group's candidates itself
        if (wv == 1 && lane == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __hip_atomic_store(&sh.f0seq, list_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr (kProf) hdelay(a.delay, 16, step, wv, wg);
        if (lane == 0) spin_until(&sh.f0seq, list_seq, 32, step, d);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (q == 0) {
          const double F0k = s_F[0];
          for (int j = j0; j < nit; j += fw * 16) {  // (the items this quad evaluated)
            if (j == 0) continue;
            const int code = s_code[j];
            const unsigned x =
                hkey(ksim_memo::score_lookup_dev(F0k - s_F[j], sh.th), roff + d, code <= 8 ? 15 - (code - 1) : 0);
            atomicMax(&s_gkey[s_igrp[j]], x);
          }
        }
        if (prof && tid == 64) { sh.prof[7] += (unsigned long long)nit; sh.prof[9] += 1ull; }
        bmark(2);
      } else {
        const int ct = tid - (fw + 1) * 64;  // class-wave thread
        const unsigned long long tc0 = (prof && ct == 0) ? __builtin_amdgcn_s_memrealtime() : 0ull;
        if constexpr (kProf) hdelay(a.delay, 8, step, wv, wg);
        const NodeV dold = uniform_node(&sh.dold[cur]);
        const NodeSum sn = node_sum(dn), so = node_sum(dold);
        for (int c = ct; c < C; c += cw * 64) {
          const PodDev q = s_cls[c];
          s_fnew[c] = filter_sum(sn, dn, q) ? 1 : 0;
          s_fold[c] = filter_sum(so, dold, q) ? 1 : 0;
          const unsigned old = c != own ? s_l1[c * nb + b] : 0u;  // the own class's row is wave 0's
          // d held the block's maximum and (with L2) its second is unknown: reload the block's keys
          const bool fl = old != 0u && hkey_rank(old) == roff + d && (!use_l2 || s_l2[c * nb + b] == kL2Stale);
          const unsigned long long fm = __ballot(fl);
          if (fm) {
            int o = 0;
            if (lane == __builtin_ctzll(fm)) o = atomicAdd(&sh.nflag, (int)__popcll(fm));
            o = __builtin_amdgcn_readlane(o, __builtin_ctzll(fm));
            if (fl)
              s_flist[o + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(fm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)fm, 0u))] =
                  (uint16_t)c;
          }
        }
        // the class waves' own barrier (LDS counter): every flag is listed
        cbar_target += cw;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) {
          __hip_atomic_fetch_add(&sh.cbar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          spin_until(&sh.cbar, cbar_target, 8, step, d);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int nflag = __builtin_amdgcn_readfirstlane(sh.nflag);
        const int qid = ct >> 4, l16 = ct & 15;
        const int kCQ = cw * 4;  // quarter-waves of the class waves
        // two rows per quarter-wave in flight at once, then any further ones one by one
        uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
        const size_t boff = (size_t)(b0 + b) * kFan + 4 * l16;
        if (qid < nflag) v0 = gld4(keys + (size_t)s_flist[qid] * a.Npad + boff);
        if (qid + kCQ < nflag) v1 = gld4(keys + (size_t)s_flist[qid + kCQ] * a.Npad + boff);
        auto reduce_row = [&](const uint4& v, int c) {
          if (use_l2) {
            unsigned m1, m2;
            block_top2_excl(v, (b0 + b) * kFan, l16, d, m1, m2);
            if (l16 == 0) { s_bx[c] = m1; s_bx2[c] = m2; }
          } else {
            const unsigned m = block_max_excl(v, (b0 + b) * kFan, l16, d);
            if (l16 == 0) s_bx[c] = m;
          }
        };
        if (qid < nflag) reduce_row(v0, s_flist[qid]);
        if (qid + kCQ < nflag) reduce_row(v1, s_flist[qid + kCQ]);
        for (int i = 2 * kCQ + qid; i < nflag; i += kCQ) {
          const int c = s_flist[i];
          const uint4 v = gld4(keys + (size_t)c * a.Npad + boff);
          reduce_row(v, c);
        }
        if (prof && ct == 0) { sh.prof[8] += (unsigned long long)nflag; sh.prof[4] += __builtin_amdgcn_s_memrealtime() - tc0; }
      }
      bulk_bar();
      if (tid == 64) sh.nflag = 0;  // (read above, before the barrier; the next class pass adds to it)
      // ---- 3. every other class's key on d (its score group's, scored by the F waves above: the max over the
      //         group's candidates, fgd_score.go:100-141), key[c][d] (HBM store), L1[c][d/64] (max with the new
      //         key, or the block max without d when d was the block max), the feasible count
      for (int c = bt; c < C; c += kHBlock - 64) {
        if (c == own) continue;
        const bool fn = s_fnew[c] != 0;
        const unsigned k = fn ? s_gkey[s_cgrp[c]] : 0u;
        gst1(keys + (size_t)c * a.Npad + d, k);
        s_cnt[c] += (fn ? 1 : 0) - (s_fold[c] ? 1 : 0);
        unsigned* l = &s_l1[c * nb + b];
        if (use_l2) {
          unsigned m1 = *l, m2 = s_l2[c * nb + b];
          const bool rl = m1 != 0u && hkey_rank(m1) == roff + d && m2 == kL2Stale;  // reloaded in the class pass
          l12_update(m1, m2, k, roff + d, rl ? s_bx[c] : 0u, rl ? s_bx2[c] : 0u);
          *l = m1;
          s_l2[c * nb + b] = m2;
        } else {
          const unsigned old = *l;
          if (k > old) *l = k;
          else if (old != 0u && hkey_rank(old) == roff + d) *l = k > s_bx[c] ? k : s_bx[c];
        }
      }
      bmark(3);
    } else if (wv == 0 && own >= 0) {
      // ===== the critical path (wave 0): the event's own class on d -- its Filter on d's new and old
      //       records, its group's candidates (one quad each: quad 0 = d's current state, quad 1 + i = the
      //       i-th candidate), its key, L1 entry and feasible count -- then the decision below reads it
      const NodeV dn = uniform_node(&sh.dnew[cur]);
      const NodeV dold = uniform_node(&sh.dold[cur]);
      const int b = d / kFan - b0;
      const PodDev q = uniform_pod(&s_cls[own]);
      const bool fn = filter_node(dn, q), fo = filter_node(dold, q);
      unsigned* l = &s_l1[own * nb + b];
      const unsigned old = __builtin_amdgcn_readfirstlane(*l);
      const unsigned old2 = use_l2 ? (unsigned)__builtin_amdgcn_readfirstlane((int)s_l2[own * nb + b]) : 0u;
      // d was the max of its block (and, with L2, the block's second is unknown): reload the block's keys
      const bool flag = old != 0u && hkey_rank(old) == roff + d && (!use_l2 || old2 == kL2Stale);
      uint4 bv = make_uint4(0u, 0u, 0u, 0u);
      if (flag && lane < 16) bv = gld4(keys + (size_t)own * a.Npad + (size_t)(b0 + b) * kFan + 4 * lane);
      unsigned k = 0u;
      if (fn) {
        const PodDev gp = uniform_pod(&s_gpod[s_cgrp[own]]);
        const bool share = is_share_pod(gp);
        const unsigned dfirst = __builtin_amdgcn_readfirstlane(sh.dfirst[cur]);
        const unsigned cm = share ? (dfirst & ksim_memo::ge_mask(dn, gp.milli)) : 0x100u;
        const int qd = lane >> 2, qq = lane & 3;
        int code = -1;
        if (qd == 0) {
          code = 0;
        } else {
          unsigned mm = cm;
          for (int i = 1; i < qd && mm; ++i) mm &= mm - 1u;
          if (mm) code = share ? 1 + __builtin_ctz(mm) : 9;
        }
        double F = 0.0;
        if (code >= 0) {
          int cpuL, total;
          uint32_t gs[4];
          fgd_candidate(dn, code, gp, &cpuL, gs, &total);
          F = state_F(dn, cpuL, gs, total, qq);
        }
        const long long fb = __builtin_bit_cast(long long, F);
        const double F0 = __builtin_bit_cast(double, ((long long)(unsigned)__builtin_amdgcn_readlane((int)(fb >> 32), 0) << 32) |
                                                         (long long)(unsigned)__builtin_amdgcn_readlane((int)fb, 0));
        unsigned x = 0u;
        if (code > 0 && qq == 0)
          x = hkey(ksim_memo::score_lookup_dev(F0 - F, sh.th), roff + d, share ? 15 - (code - 1) : 0);
        k = (unsigned)wave_max_dpp((int)x);
        if (share) {
          const unsigned z = hkey(0, roff + d, 0);  // feasible with no fitting GPU
          k = k > z ? k : z;
        }
      }
      unsigned bx = 0u, bx2 = 0u;
      if (flag) {
        if (use_l2) {
          unsigned m1, m2;
          block_top2_excl(bv, (b0 + b) * kFan, lane & 15, d, m1, m2);
          bx = (unsigned)__builtin_amdgcn_readfirstlane((int)m1);
          bx2 = (unsigned)__builtin_amdgcn_readfirstlane((int)m2);
        } else {
          bx = (unsigned)__builtin_amdgcn_readfirstlane((int)block_max_excl(bv, (b0 + b) * kFan, lane & 15, d));
        }
      }
      if (lane == 0) {
        gst1(keys + (size_t)own * a.Npad + d, k);
        s_cnt[own] += (fn ? 1 : 0) - (fo ? 1 : 0);
        if (use_l2) {
          unsigned m1 = old, m2 = old2;
          l12_update(m1, m2, k, roff + d, bx, bx2);
          *l = m1;
          s_l2[own * nb + b] = m2;
        } else {
          if (k > old) *l = k;
          else if (flag) *l = k > bx ? k : bx;
        }
      }
      // the decision below reads this class's L1 row and count: the wave's LDS operations in order
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      mark(1);
    }
    // ---- 4. the event: the winner of its class (create) or the unbind (delete); wave 0
    if (wv == 0) {
      if constexpr (kProf) hdelay(a.delay, 4, step, wv, wg);
      const PodDev p = uniform_pod(&sh.ev[eb]);
      int rk = -1, mask = 0, ndead = -1;
      bool write = false;
      NodeV before{}, after{};
      ResultDev out{-1, 0, 0, 0, ST_DELETED};
      if (cs >= 0) {
        const unsigned lv = lane < nb ? s_l1[cs * nb + lane] : 0u;
        unsigned W = (unsigned)wave_max_dpp((int)lv);
        int nfeas = __builtin_amdgcn_readfirstlane(s_cnt[cs]);
        if (Kt > 1) {
          // the slices' maxima and feasible counts: granules {tag, key}, {tag, count} (k_replay's exchange)
          const size_t so = (size_t)(seq & 1) * Kt * 2;
          unsigned long long* slot = gr + so;
          // tag: {epoch (24 bits) | seq mod 256} across processes (a peer is at most one exchange ahead,
          // so a slot holds this exchange or the one two before: 8 bits of seq tell them apart, and a
          // 24-bit epoch keeps the previous runs' granules out); {seq + 1 (24 bits)} in one launch, whose
          // buffer is zeroed before it (never a zero tag)
          const unsigned long long tag =
              (unsigned long long)(a.epoch ? (((unsigned)a.epoch << 8) | ((unsigned)(seq + 1) & 0xffu))
                                           : ((unsigned)(seq + 1) & 0xffffffu)) << 32;
          const int np = a.npeer;
          if (np > 0) {  // lane q -> shard q's buffer
            if (lane < np) {
              unsigned long long* ps = a.peer[lane] + so + (size_t)col * 2;
              __hip_atomic_store(ps, tag | W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(ps + 1, tag | (unsigned)nfeas, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
          } else if (lane == 0) {
            ksim_replay::gstore(slot + (size_t)col * 2 + 0, tag | W);
            ksim_replay::gstore(slot + (size_t)col * 2 + 1, tag | (unsigned)nfeas);
          }
          unsigned long long x0[kS], x1[kS];
          auto load = [&]() {
#pragma unroll
            for (int j = 0; j < kS; ++j) {
              const int k = lane + 64 * j;
              if (k < Kt) {
                if (np > 0) {
                  x0[j] = __hip_atomic_load(slot + (size_t)k * 2 + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                  x1[j] = __hip_atomic_load(slot + (size_t)k * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                } else {
                  x0[j] = ksim_replay::gload(slot + (size_t)k * 2 + 0);
                  x1[j] = ksim_replay::gload(slot + (size_t)k * 2 + 1);
                }
              }
            }
          };
          auto ready = [&]() {
            bool ok = true;
#pragma unroll
            for (int j = 0; j < kS; ++j)
              ok = ok && (lane + 64 * j >= Kt || ((x0[j] & ~0xffffffffull) == tag && (x1[j] & ~0xffffffffull) == tag));
            return ok;
          };
          load();
          unsigned spins = 0;
          while (!__all(ready())) {
            if (++spins > ksim_replay::kSpinLimit) {
              if (lane == 0) { atomicOr(a.fail, 1); sh.stop = 1; }
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            load();
          }
          unsigned m = 0u;
          int c = 0;
#pragma unroll
          for (int j = 0; j < kS; ++j) {
            if (lane + 64 * j < Kt) {
              const unsigned kj = (unsigned)(x0[j] & 0xffffffffull);
              m = kj > m ? kj : m;
              c += (int)(unsigned)(x1[j] & 0xffffffffull);
            }
          }
          W = (unsigned)wave_max_dpp((int)m);
          nfeas = wave_sum_dpp(c);
          ++seq;
        }
        out = ResultDev{-1, 0, 0, nfeas, ST_UNSCHED};
        write = W == 0u && w == 0;  // nobody feasible: workgroup 0 reports
        if (a.skip && W == 0u) ndead = cs;  // for good (create-only); published through pdead below
        uint8_t h = 3;
        if (W != 0u) {
          const int wr = hkey_rank(W) - roff;  // the winner's rank in this shard
          h = 0;
          if (sharded && (wr < 0 || wr >= N)) {
            // the winner is in another shard (history 4): this shard's first workgroup writes a provisional
            // record naming it (the owner's record is authoritative; ksim/shard.py merge_results)
            h = 4;
            if (w == 0) {
              out = ResultDev{wr + roff, 0, result_score(rp, nfeas, hkey_score(W), 0, 0), nfeas, ST_OK};
              write = true;
            }
          }
          if (wr >= lo && wr < lo + ns) {  // the winner is in this slice
            const NodeV wn = uniform_node(&s_nodes[wr - lo]);
            mask = select_gpus(wn, p, rp.gpusel, hkey_gpu(W), rp.seed, step);
            write = true;
            if (mask < 0) {  // Reserve failed: allocateGpuId returned "" / panicked
              out.status = ST_ERROR;
              h = 2;
            } else {
              out.status = ST_OK;
              out.score = result_score(rp, nfeas, hkey_score(W), 0, 0);
              out.node = wr + roff;  // name rank (global); k_memo_finish maps it to the node index
              out.gpu_mask = mask;
              rk = wr;
              before = wn;
              after = wn;
              bind_node(after, p, mask, +1);
              h = 1;
            }
          }
        }
        if (hist && lane == 0) hist[step] = h;
      } else if (p.ref >= 0 && p.ref < step) {
        // simulator.go:416-422 deletePod: undo the creation's Bind (its result holds the rank and mask);
        // with K > 1 only the workgroup that bound it (its own history) reads that result
        // (every value read here was written by this workgroup: a record another workgroup -- possibly on
        // another XCD, another L2 -- wrote is never read back)
        const int hh = hist ? (int)hist[p.ref] : 1;
        if (hh == 1) {
          const ResultDev cr = gget(rp.res + p.ref);
          const int crk = __builtin_amdgcn_readfirstlane(cr.node) - roff;
          const int cst = __builtin_amdgcn_readfirstlane(cr.status);
          const int cmask = __builtin_amdgcn_readfirstlane(cr.gpu_mask);
          if (crk >= 0 && cst == ST_OK) {
            const PodDev bp = uniform_pod(reinterpret_cast<const PodDev*>(rp.ev + p.ref));
            rk = crk;
            before = uniform_node(&s_nodes[rk - lo]);
            after = before;
            bind_node(after, bp, cmask, -1);
            out = ResultDev{rk + roff, cmask, 0, 0, ST_DELETED};
          }
          write = true;
        } else {
          write = hh == 2 || (hh == 3 && w == 0);
          if (hh == 4 && w == 0) {  // bound in another shard: name it, from this workgroup's own record
            const ResultDev cr = gget(rp.res + p.ref);
            out = ResultDev{__builtin_amdgcn_readfirstlane(cr.node), 0, 0, 0, ST_DELETED};
            write = true;
          }
        }
        if (hist && lane == 0) hist[step] = 0;
      } else {
        write = w == 0;
      }
      if (lane == 0) {
        if (write) gput(rp.res + step, out);
        if (rk >= 0) {
          store_node(&s_nodes[rk - lo], after);
          store_node(&sh.dold[cur ^ 1], before);
          store_node(&sh.dnew[cur ^ 1], after);
          if (rp.snap) {  // cluster report: the state this event left
            gput_node(rp.snap + step, after);
            gput(rp.prev + step, s_last[rk - lo]);
          }
          s_last[rk - lo] = step;
        }
        sh.d[cur ^ 1] = rk;
        {  // the dead set: fold the previous decided step's class in, publish this one's for the next step
          const int pc = sh.pdead[cur];
          if (pc >= 0) sh.dead[pc >> 5] |= 1u << (pc & 31);
          sh.pdead[cur ^ 1] = ndead;
        }
      }
      if (rk >= 0) {
        const unsigned fm = ksim_memo::first_mask_lanes(after, lane);
        if (lane == 0) sh.dfirst[cur ^ 1] = fm;
        if (w0list) {  // the next refresh's F list (wave 0 waits for the bulk at the end barrier anyway)
          const unsigned dfirst = (unsigned)__builtin_amdgcn_readfirstlane((int)fm);
          const NodeSum sd = node_sum(after);
          uint8_t* const ncode = s_code_b + (cur ^ 1) * kMaxItems;
          uint8_t* const nigrp = s_igrp_b + (cur ^ 1) * kMaxItems;
          int16_t* const ngbase = s_gbase_b + (cur ^ 1) * a.Gmax;
          unsigned* const ngkey = s_gkey_b + (cur ^ 1) * a.Gmax;
          int base = 1;  // item 0: the node's current state
          for (int g0 = 0; g0 < G; g0 += 64) {
            const int g = g0 + lane;
            unsigned cm = 0u;
            bool share = false;
            if (g < G) {
              const PodDev gp = s_gpod[g];
              share = is_share_pod(gp);
              cm = share ? (dfirst & ksim_memo::ge_mask(after, gp.milli)) : 0x100u;
              if (prune && !filter_sum(sd, after, gp)) cm = 0u;  // no class of the group passes Filter on d
            }
            const int nc = __popc(cm);
            int excl = 0, tot = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const unsigned long long m = __ballot((nc >> k) & 1);
              excl += __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << k;
              tot += __popcll(m) << k;
            }
            int o = base + excl;
            if (g < G) {
              ngbase[g] = (int16_t)o;
              ngkey[g] = share ? hkey(0, roff + rk, 0) : 0u;
            }
            unsigned mm = cm;
            while (mm) {
              const int x = __builtin_ctz(mm);
              mm &= mm - 1u;
              ncode[o] = (uint8_t)(share ? 1 + x : 9);
              nigrp[o] = (uint8_t)g;
              ++o;
            }
            base += tot;
          }
          if (lane == 0) {
            ncode[0] = 0;
            nigrp[0] = 0;
            sh.nitems[cur ^ 1] = base;
          }
        }
        if (w0pf) {
          // touch the key rows of the classes whose block max is the node just bound: the next refresh
          // reloads most of them (its flagged blocks), and this workgroup's L1 then holds them.  A hint
          // only: the L1 values read here may be mid-update by the bulk.
          const int nb2 = (rk - lo) / kFan;
          unsigned acc = 0u;
          for (int c = lane; c < C; c += 64) {
            const unsigned o = s_l1[c * nb + nb2];
            if (o != 0u && hkey_rank(o) == roff + rk) {
              const unsigned* row = keys + (size_t)c * a.Npad + (size_t)(b0 + nb2) * kFan;
              acc ^= row[0] ^ row[16] ^ row[32] ^ row[48];
            }
          }
          asm volatile("" ::"v"(acc));
        }
      }
    }
    __syncthreads();
    mark(5);
    cur ^= 1;
    if (sh.stop) break;  // K > 1: a poll timed out; any K: a bulk wait timed out
  }
  if (prof && tid == 0) {
    sh.prof[10] = __builtin_amdgcn_s_memtime() - c_start;
    sh.prof[11] = __builtin_amdgcn_s_memrealtime() - t_start;
  }
  __syncthreads();
  if (prof && tid < kHProf) a.prof[(size_t)blockIdx.x * kHProf + tid] = sh.prof[tid];
  // final cluster state
  for (int i = tid; i < ns; i += kHBlock) store_node(rp.nodes + rank2idx[lo + i], load_node(&s_nodes[i]));
}

template <int kSub, bool kProf, bool kModel = false>
__global__ __launch_bounds__(kHBlock) void k_hmemo(HMemoArgs a, const TypDev* __restrict__ tp_all) {
  if (kSub != 0 && a.started != nullptr && threadIdx.x == 0)  // (the one-workgroup forms store it in the body)
    __hip_atomic_store(a.started + blockIdx.x, a.gate_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  hmemo_body<kSub, kProf, kModel>(a, tp_all, (int)blockIdx.x);
}

// One launch over the shards of a node-sharded cluster on one device (ksim_shard_group_run): workgroup
// blockIdx.x is workgroup blockIdx.x % K of shard blockIdx.x / K, with that shard engine's arguments.
template <int kSub, bool kProf>
__global__ __launch_bounds__(kHBlock) void k_hmemo_group(const HMemoArgs* __restrict__ sa, int K) {
  const HMemoArgs a = sa[blockIdx.x / K];
  hmemo_body<kSub, kProf>(a, a.tp, (int)blockIdx.x % K);
}

// ---------------------------------------------------------------------------
// Initial keys.  k_hinit_gk: per (launch replica, group, distinct initial node state) the group's
// best (score, GPU) on that state -- memo_key_scalar's evaluation without the Filter and the rank.
// k_hinit_keys: per (launch replica, class, rank) the key = Filter ? that with the rank : 0, the
// feasible counts and the L1 maxima (one wave = one block of 64 ranks).
// ---------------------------------------------------------------------------
struct HInitArgs {
  ReplicaDev* reps;
  const int* rep_list;
  int N, Npad, nb, Cmax, Gmax, Smax;
  const int* cg;           // [Rg][2]
  const PodDev* cls;       // [Rg][Cmax]
  const uint16_t* cgrp;    // [Rg][Cmax]
  const PodDev* gpod;      // [Rg][Gmax]
  int roff;                // node-sharded: the shard's first global rank (keys carry global ranks)
  const NodeRec* st;       // [Rg][Smax] distinct initial node states
  const int* ns;           // [Rg] distinct states
  const int* nstate;       // [Rg][Npad] state of each rank (-1 padding)
  unsigned* gsc;           // [Rg][Gmax][Smax] hkey(score, 0, gf) without the rank field
  unsigned* keys;          // [Rg][Cmax][Npad]
  unsigned* l1;            // [Rg][Cmax][nb]
  unsigned* l2;            // [Rg][Cmax][nb] second maxima, or null
  int* cnt;                // [Rg][Cmax], zeroed before k_hinit_keys
  const double* th;
  const int* mtoff;        // [Rg][KSIM_MAX_TYPES] the per-model tables (HMemoArgs), null: none
  double* na;              // [Rg][Mslots][kNaStride]
  int Mslots;
};

// grid (kNaStride / 256, Mslots, Rg): the NA bin of every (model, total) of a typed replica -- the sequential
// sum, in table order, of freq x total over the GPU typical pods that do not accept the model (frag_F_quad's
// bin 3: x = freq * dtot, then bin += x)
__global__ __launch_bounds__(256) void k_hinit_na(HInitArgs a, const TypDev* __restrict__ tp_all) {
  const int gi = (int)blockIdx.z, slot = (int)blockIdx.y;
  const int total = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (total >= kNaStride) return;
  const int r = a.rep_list[gi];
  const ReplicaDev& rp = a.reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  int m = -1;
  for (int k = 0; k < KSIM_MAX_TYPES; ++k) {
    const unsigned w = (unsigned)a.mtoff[(size_t)gi * KSIM_MAX_TYPES + k];
    if ((w & kMtPresent) && (int)((w >> 21) & 31u) == slot) m = k;
  }
  if (m < 0) return;
  const double dtot = (double)total;
  double na = 0.0;
  for (int t = rp.ncpu; t < rp.nt; ++t) {
    if ((tp[t].tmask >> m) & 1u) continue;
    const double x = tp[t].freq * dtot;
    na += x;
  }
  a.na[((size_t)gi * a.Mslots + slot) * kNaStride + total] = na;
}

__global__ __launch_bounds__(256) void k_hinit_gk(HInitArgs a, const TypDev* __restrict__ tp_all) {
  const int gi = (int)blockIdx.z, g = (int)blockIdx.y;
  const int s = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g >= a.cg[2 * gi + 1] || s >= a.ns[gi]) return;
  const int r = a.rep_list[gi];
  const ReplicaDev& rp = a.reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  const NodeV n = load_node(a.st + (size_t)gi * a.Smax + s);
  const PodDev p = a.gpod[(size_t)gi * a.Gmax + g];
  const double F0 = eval_fgd_item(n, 0, PodDev{}, rp, tp);
  unsigned k;
  if (!is_share_pod(p)) {
    k = hkey_norank(fgd_score_lookup(F0 - eval_fgd_item(n, 9, p, rp, tp), a.th), 0);  // fgd_score.go:137-141
  } else {
    k = hkey_norank(0, 0);
    const unsigned fm = first_of_class(n, p.milli);
    for (int x = 0; x < kMaxGpu; ++x) {
      if ((fm >> x) & 1u) {  // fgd_score.go:111-118
        const unsigned c = hkey_norank(fgd_score_lookup(F0 - eval_fgd_item(n, 1 + x, p, rp, tp), a.th), 15 - x);
        k = c > k ? c : k;
      }
    }
  }
  a.gsc[((size_t)gi * a.Gmax + g) * a.Smax + s] = k;
}

__global__ __launch_bounds__(256) void k_hinit_keys(HInitArgs a) {
  const int gi = (int)blockIdx.z, c = (int)blockIdx.y;
  const int rank = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (c >= a.cg[2 * gi] || rank >= a.Npad) return;  // uniform per workgroup (Npad % 256 == 0 not required: waves stay whole)
  const int s = a.nstate[(size_t)gi * a.Npad + rank];
  unsigned k = 0u;
  if (s >= 0) {
    const NodeV n = load_node(a.st + (size_t)gi * a.Smax + s);
    const PodDev q = a.cls[(size_t)gi * a.Cmax + c];
    if (filter_node(n, q)) {
      const int g = a.cgrp[(size_t)gi * a.Cmax + c];
      k = a.gsc[((size_t)gi * a.Gmax + g) * a.Smax + s] | hkey_rankbits(a.roff + rank);
    }
  }
  a.keys[((size_t)gi * a.Cmax + c) * a.Npad + rank] = k;
  const int lane = (int)(threadIdx.x & 63);
  const unsigned long long fb = __ballot(k != 0u);
  unsigned m = k, m2 = 0u;
  ksim_memo::wave_top2(m, m2);  // (every lane active: one wave = one block of 64 ranks)
  if (lane == 0) {
    a.l1[((size_t)gi * a.Cmax + c) * a.nb + rank / kFan] = m;
    if (a.l2) a.l2[((size_t)gi * a.Cmax + c) * a.nb + rank / kFan] = m2;
    if (fb) atomicAdd(&a.cnt[(size_t)gi * a.Cmax + c], (int)__popcll(fb));
  }
}

}  // namespace ksim_hmemo

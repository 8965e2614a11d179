// ksim_pmemo.hpp -- pipelined memoised FGD replay (k_pmemo).
//
// k_memo (ksim_memo.hpp) runs every pod step through one serial chain: the owner of the step's class
// learns the previous winner (a cross-CU granule), evaluates that node's F for the class, decides
// and publishes -- the hand-off and the critical F in series, ~3.15 us per step at C2.  k_pmemo puts
// k_replay's pipelining (ksim_replay.hpp) on memoised keys, so the hand-off overlaps the step's work:
//
//   - node slices: replica r is run by K co-resident workgroups, workgroup w owning the name ranks
//     [w S, w S + S) with S <= 64: wave-0 lane n holds slot n's record, its stale bits and (LDS) the
//     F of its current state.  LDS holds the packed key of every (score group, slot) pair:
//     gk[g][slot] = the group's best (score, GPU) on that node with the rank (hkey), the Filter NOT
//     applied -- groups share the candidate states (same cpu_nz, milli, num: fgd_score.go:99-149),
//     and the per-class Filter is evaluated when a step reads the key (one lane per slot);
//   - the only slot of a slice that step s can change is the slice's own candidate b (its best key
//     for step s).  Right after publishing step s a workgroup works on step s+1 with b excluded,
//     and evaluates b twice: as it is (pre) and in a VIRTUAL slot holding b with step s's Reserve +
//     Bind applied (post).  When step s's exchange completes it publishes step s+1 with post (it
//     owned the winner) or pre -- selectHost over the union (generic_scheduler.go:187-212) -- and
//     commits (the virtual slot becomes b);
//   - staleness: a committed slot's keys are stale in every group but the step's (one bit per (slot,
//     group), in wave 0's registers).  Each step's critical list holds the virtual slot's F0 and the
//     step group's candidates on it, and the step group's candidates on every slot still stale in
//     it; a bulk batch of other stale (slot, group) pairs of one focus slot is evaluated by waves
//     1-15 while wave 0 runs the next step's decision (their keys land one step later), so a changed
//     node's keys become fresh within a few steps, no step waits on a key it does not read, and the
//     refresh stays off the chain.  A batch listed at step t leaves out step t+1's group and the
//     slot pending after step t (the only one step t+1 can commit).
//
// Per pod step s (every workgroup of the replica):
//   F   one wave per critical item: fgd_candidate + wave_F (frag.go's sequential fp64 bins, the same
//       bits as frag_F);                                                                  | barrier
//   D   wave 0: the group keys of the critical jobs and of the bulk batch listed at step s-2 (one
//       lane per item: the score steps; one lane per job: the max, ties to the lowest GPU,
//       fgd_score.go:128), the slice's best key for step s with b excluded (Filter per lane), b's
//       versions, the exchange of step s-1 (granules polled since the F round), the granule of step
//       s, the result and commit of step s-1, Reserve + Bind of the new candidate into the virtual
//       slot, the critical list of step s+1 and the next bulk batch;
//       waves 1-15: the bulk batch listed at step s-1.                                     | barrier
// Every key read in D is fresh, and b's versions are the same keys k_hmemo / k_replay / the oracle
// compute (the same device functions), so the decisions are theirs.
//
// Scope: FGD replicas on create-only streams (no report), N <= 64 K, K <= 64 co-resident workgroups,
// <= 128 score groups, the FGD / best / worst / random GPU selectors.  The host takes k_memo /
// k_hmemo / k_replay otherwise.
#pragma once

namespace ksim_pmemo {

using namespace ksim;
using ksim_hmemo::hkey;
using ksim_hmemo::hkey_gpu;
using ksim_hmemo::hkey_rank;
using ksim_hmemo::hkey_rankbits;
using ksim_hmemo::hkey_score;

constexpr int kPBlock = 1024;
constexpr int kPWaves = kPBlock / 64;
constexpr int kSlots = 64;                       // slots per workgroup (one wave-0 lane each)
constexpr int kVirt = kSlots;                    // job slot code of the virtual node
constexpr int kMaxGroups = 128;                  // two u64 stale words per slot
constexpr int kBulk = kPWaves - 1;               // bulk items (and jobs) per step: waves 1-15, one each
constexpr int kMaxJobs = 1 + kSlots;             // critical jobs: the virtual slot + every slot
constexpr int kMaxItems = 9 + 8 * kSlots;        // critical items
constexpr int kEvBuf = 128;
constexpr int kTagBits = 19;                     // granule: key << 32 | count << 19 | (step + 1) tag
constexpr unsigned kTagMask = (1u << kTagBits) - 1u;
constexpr int kCntMask = (1 << (32 - kTagBits)) - 1;
constexpr unsigned kSpinLimit = 1u << 22;

struct PMemoArgs {
  ReplicaDev* reps;
  const int* rep_list;      // replica of each group of K workgroups
  int N, K, S;              // nodes, workgroups per replica, slots per workgroup
  int Gmax, Smax, Npad;     // k_hmemo plan strides
  const int* cg;            // [Rg][2] classes, groups
  const PodDev* gpod;       // [Rg][Gmax] score request of each group
  const int* evg;           // [Rg][stride] group of each event
  int stride;
  const unsigned* gsc;      // [Rg][Gmax][Smax] k_hinit_gk: group key of each distinct initial state, no rank
  const int* nstate;        // [Rg][Npad] distinct initial state of each rank
  const double* th;         // [102] FGD score steps
  unsigned long long* gran; // [Rg][2][K] exchange granules
  int* fail;                // a granule poll timed out
  unsigned long long* prof; // k_pmemo<true>: [Rg * K][kPProf] phase sums (KSIM_PROFILE=1)
  unsigned long long* trace; // k_pmemo<true>: [Rg * K][trace_steps][kTr] times of step s (see kTr)
  int trace_steps;
};
// 0 F round, 1 D: job keys, 2 D: slice max + b's versions, 3 exchange wait, 4 publish + result +
// commit + virtual, 5 next lists, 6 end barrier; 7 critical items, 8 critical jobs, 9 bulk items,
// 10 shader clock, 11 wall ticks
constexpr int kPProf = 12;
// trace of step s: 0 F round start, 1 D start, 2 wait start, 3 exchange(s-1) done, 4 publish(s), 5 lists done
constexpr int kTr = 6;

// Item descriptor: slot (kVirt: the virtual slot) | fgd_candidate code << 8 | group << 16.
__device__ __forceinline__ unsigned pdesc(int slot, int code, int g) {
  return (unsigned)slot | ((unsigned)code << 8) | ((unsigned)g << 16);
}

struct __align__(16) PShared {
  PodDev ev[kEvBuf];
  int evg[kEvBuf];
  TypDev tp[kMaxTypical];
  double th[104];
  NodeRec nodes[kSlots + 1];                    // wave 0's records (slot kVirt: the virtual slot) for the F waves
  double F0[kSlots];                            // F of every slot's current state
  double F[kMaxItems];                          // critical items
  unsigned desc[kMaxItems];
  unsigned kbuf[kMaxItems];                     // the items' keys (D)
  double bF[2][kBulk + 1];                      // bulk batches (by listing step parity)
  unsigned bdesc[2][kBulk + 1];
  unsigned bkbuf[kBulk + 1];
  uint8_t job_slot[kMaxJobs];
  uint8_t job_grp[kMaxJobs];
  uint8_t job_n[kMaxJobs];
  uint8_t bjob_n[2][kBulk + 1];
  uint8_t bjob_grp[2][kBulk + 1];
  uint8_t bjob_o[2][kBulk + 1];
  uint8_t pad_[(16 - (3 * kMaxJobs + 6 * (kBulk + 1)) % 16) % 16];
  uint16_t job_o[kMaxJobs];
  uint16_t pad2_[(8 - kMaxJobs % 8) % 8];
  int nitems, njobs, ncrit, stop;
  int nbitems[2], nbjobs[2], bslot[2], pad3_[2];
  unsigned long long prof[kPProf];
};
static_assert(sizeof(PShared) % 16 == 0, "keep the dynamic regions 16-B aligned");

// Dynamic LDS: PShared | PodDev gpod[Gmax] | u32 gk[Gmax][kSlots] | f64 fold[kPWaves][kFoldBuf].
inline size_t pmemo_lds(int Gmax) {
  return sizeof(PShared) + (size_t)Gmax * sizeof(PodDev) + (size_t)Gmax * kSlots * 4 +
         (size_t)kPWaves * ksim_memo::kFoldBuf * 8;
}

// Exclusive prefix and total of a per-lane count 0..15 over the wave (four ballot bit planes).
__device__ __forceinline__ int lane_prefix(int v, int* tot) {
  int excl = 0, t = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const unsigned long long m = __ballot((v >> b) & 1);
    excl += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
    t += __popcll(m) << b;
  }
  *tot = t;
  return excl;
}
__device__ __forceinline__ int lanes_before(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
// Workgroup barrier for LDS hand-offs only: __syncthreads() is a release fence as well, which makes
// every wave wait for its outstanding global stores (here: the granule and result stores, whose
// acknowledgement takes about a hand-off latency) before the barrier.  Nothing in the step loop
// hands global memory between waves of one workgroup, so the wave's LDS queue is all it drains.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A lane's record as wave-uniform values (v_readlane).
__device__ __forceinline__ NodeV readlane_node(const NodeV& n, int l) {
  NodeV u;
  u.cpu_left = __builtin_amdgcn_readlane(n.cpu_left, l);
  u.mem_left = __builtin_amdgcn_readlane(n.mem_left, l);
#pragma unroll
  for (int i = 0; i < 4; ++i) u.g[i] = (uint32_t)__builtin_amdgcn_readlane((int)n.g[i], l);
  u.meta = (uint32_t)__builtin_amdgcn_readlane((int)n.meta, l);
  u.name_rank = (uint32_t)__builtin_amdgcn_readlane((int)n.name_rank, l);
  return u;
}

// F of one listed item (one wave): the candidate state of its slot's LDS record for its group's request.
__device__ __forceinline__ double item_F(unsigned d, const NodeRec* nodes, const PodDev* gpod, bool typed, const TypDev* ltp,
                                        int ncpu, int nt, int lane, double* fold) {
  const int slot = (int)(d & 0xffu), code = (int)((d >> 8) & 0xfu), g = (int)(d >> 16);
  const NodeV m = ksim_replay::uniform_node(&nodes[slot]);
  const PodDev gp = ksim_replay::uniform_pod(&gpod[g]);
  int cpuL, total;
  uint32_t gs[4];
  ksim_replay::fgd_candidate(m, code, gp, &cpuL, gs, &total);
  return ksim_memo::wave_F(cpuL, gs, total, 1u << m.gpu_type(), typed, ltp, ncpu, nt, lane, fold);
}

template <bool kProf>
__global__ __launch_bounds__(kPBlock) void k_pmemo(PMemoArgs a, const TypDev* __restrict__ tp_all) {
  using namespace ksim_replay;
  using ksim_memo::gget;
  using ksim_memo::gput;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  PShared& sh = *reinterpret_cast<PShared*>(smem);
  const int gi = (int)blockIdx.x / a.K, w = (int)blockIdx.x % a.K;
  const int r = a.rep_list[gi];
  const ReplicaDev rp = a.reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = a.N, K = a.K;
  const int lo = w * a.S, ns = max(0, min(a.S, N - lo));
  const int G = a.cg[2 * gi + 1];
  PodDev* s_gpod = reinterpret_cast<PodDev*>(smem + sizeof(PShared));
  unsigned* s_gk = reinterpret_cast<unsigned*>(s_gpod + a.Gmax);
  double* s_fold = reinterpret_cast<double*>(s_gk + (size_t)a.Gmax * kSlots);
  double* fold = s_fold + (size_t)wv * ksim_memo::kFoldBuf;
  const int* rank2idx = reinterpret_cast<const int*>(rp.tags + (size_t)N * kTagStride);
  const int* evg = a.evg + (size_t)gi * a.stride;
  unsigned long long* gr = a.gran + (size_t)gi * 2 * K;
  const int E = rp.n_events;
  const bool typed = rp.typed != 0;

  // ---- start-up: the groups, the initial keys, the tables; wave 0 lane n: slot n's record
  for (int g = tid; g < G; g += kPBlock) s_gpod[g] = a.gpod[(size_t)gi * a.Gmax + g];
  for (int x = tid; x < G * ns; x += kPBlock) {
    const int g = x / ns, i = x - g * ns;
    const int st = a.nstate[(size_t)gi * a.Npad + lo + i];
    s_gk[g * kSlots + i] = a.gsc[((size_t)gi * a.Gmax + g) * a.Smax + st] | hkey_rankbits(lo + i);
  }
  for (int i = tid; i < rp.nt * 2; i += kPBlock) reinterpret_cast<uint4*>(sh.tp)[i] = reinterpret_cast<const uint4*>(tp)[i];
  for (int i = tid; i < 102; i += kPBlock) sh.th[i] = a.th[i];
  for (int i = tid; i < ns; i += kPBlock) {
    const NodeV n = load_node(rp.nodes + rank2idx[lo + i]);
    store_node(&sh.nodes[i], n);
    sh.F0[i] = eval_fgd_item(n, 0, PodDev{}, rp, tp);
  }
  if (tid == 0) {
    sh.stop = 0; sh.nitems = 0; sh.njobs = 0; sh.ncrit = 0;
    sh.nbitems[0] = sh.nbitems[1] = 0; sh.nbjobs[0] = sh.nbjobs[1] = 0; sh.bslot[0] = sh.bslot[1] = 0;
  }
  if (kProf && tid < kPProf) sh.prof[tid] = 0ull;
  NodeV rec{};                                 // wave 0, lane n < ns: slot n's record
  unsigned long long st0 = 0ull, st1 = 0ull;   // wave 0, lane n: slot n's stale groups
  if (wv == 0 && lane < ns) rec = load_node(rp.nodes + rank2idx[lo + lane]);
  __syncthreads();
  const bool prof = kProf && a.prof != nullptr;
  unsigned long long t_last = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const unsigned long long t_start = t_last, c_start = prof ? __builtin_amdgcn_s_memtime() : 0ull;
  auto tr = [&](int s, int k) {  // KSIM_PROFILE=2: thread 0's timestamps of step s
    if (kProf && a.trace && tid == 0 && s < a.trace_steps)
      a.trace[((size_t)blockIdx.x * a.trace_steps + s) * kTr + k] = __builtin_amdgcn_s_memrealtime();
  };
  auto mark = [&](int ph) {  // thread 0 (wave 0 lane 0)
    if (prof && tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      sh.prof[ph] += t - t_last;
      t_last = t;
    }
  };

  // wave 0's pending step (published, not committed): candidate slot, key, Reserve mask, count, and
  // the candidate with the pending Bind applied (the virtual slot; uniform)
  int pb = -1, pmask = -1, pcnt = 0;
  unsigned pkey = 0u;
  bool pend = false;
  NodeV vrec{};
  const unsigned long long all0 = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
  const unsigned long long all1 = G > 64 ? (G >= 128 ? ~0ull : ((1ull << (G - 64)) - 1ull)) : 0ull;

  // ---- wave 0: the critical list of the step in event-window slot eb1 (the virtual slot if `virt`,
  // then every slot stale in the step's group) and the bulk batch `bb` (other stale groups of one
  // focus slot other than `excl`, the step's group left out); listed pairs leave the stale set now
  auto build_lists = [&](int eb1, bool virt, int excl, int bb) {
    const int g1 = __builtin_amdgcn_readfirstlane(sh.evg[eb1]);
    const PodDev gp = uniform_pod(&s_gpod[g1]);
    const bool share = is_share_pod(gp);
    int o = 0, nj = 0;
    if (virt) {  // item 0: the virtual slot's current state (its F0), then its candidates
      const unsigned f0 = ksim_memo::first_mask_lanes(vrec, lane);
      const unsigned cm = share ? (f0 & ksim_memo::ge_mask(vrec, gp.milli)) : 0x100u;
      const int nc = __popc(cm);
      if (lane <= nc) {
        unsigned m = cm;
        for (int q = 1; q < lane; ++q) m &= m - 1u;
        sh.desc[lane] = pdesc(kVirt, lane == 0 ? 0 : (share ? 1 + __builtin_ctz(m) : 9), g1);
      }
      if (lane == 0) {
        sh.job_slot[0] = (uint8_t)kVirt;
        sh.job_grp[0] = (uint8_t)g1;
        sh.job_o[0] = 0;
        sh.job_n[0] = (uint8_t)(1 + nc);
      }
      o = 1 + nc;
      nj = 1;
    }
    // critical: every slot stale in the step's group
    const unsigned long long gbit = 1ull << (g1 & 63);
    const bool crit = lane < ns && ((g1 < 64 ? st0 : st1) & gbit) != 0ull;
    const unsigned cm = crit ? (share ? first_of_class(rec, gp.milli) : 0x100u) : 0u;
    int tot = 0;
    const int nc = __popc(cm);
    const int ex = lane_prefix(nc, &tot);
    const unsigned long long cb = __ballot(crit);
    if (crit) {
      const int j = nj + lanes_before(cb), io = o + ex;
      sh.job_slot[j] = (uint8_t)lane;
      sh.job_grp[j] = (uint8_t)g1;
      sh.job_o[j] = (uint16_t)io;
      sh.job_n[j] = (uint8_t)nc;
      unsigned m = cm;
      for (int k = 0; k < nc; ++k) {
        sh.desc[io + k] = pdesc(lane, share ? 1 + __builtin_ctz(m) : 9, g1);
        m &= m - 1u;
      }
      if (g1 < 64) st0 &= ~gbit;
      else st1 &= ~gbit;
    }
    nj += __popcll(cb);
    o += tot;
    if (lane == 0) {
      sh.nitems = o;
      sh.njobs = nj;
      if (kProf) sh.ncrit = nj;
    }
    // bulk batch: the lowest slot (not `excl`) with stale groups, its groups in order, one item per wave
    int bo = 0, bj = 0, fs = -1;
    const unsigned long long ob = __ballot(lane < ns && lane != excl && (st0 | st1) != 0ull);
    if (ob != 0ull) {
      fs = __builtin_ctzll(ob);
      const NodeV fn = readlane_node(rec, fs);
      const unsigned f0 = ksim_memo::first_mask_lanes(fn, lane);
      const unsigned long long fw0 = readlane_u64(st0, fs), fw1 = readlane_u64(st1, fs);
      unsigned long long took0 = 0ull, took1 = 0ull;
      for (int half = 0; half < 2; ++half) {
        const int gg = half * 64 + lane;
        const unsigned long long fw = half ? fw1 : fw0;
        const bool want = ((fw >> lane) & 1ull) != 0ull && gg != g1;
        int bc = 0;
        unsigned bm = 0u;
        bool bshare = false;
        if (want) {
          const PodDev q = s_gpod[gg];
          bshare = is_share_pod(q);
          bm = bshare ? (f0 & ksim_memo::ge_mask(fn, q.milli)) : 0x100u;
          bc = __popc(bm);
        }
        int btot = 0;
        const int bex = lane_prefix(bc, &btot);
        const unsigned long long wb = __ballot(want);
        const bool take = want && bo + bex + bc <= kBulk && bj + lanes_before(wb) < kBulk;
        const unsigned long long tb = __ballot(take);
        if (take) {
          const int j = bj + lanes_before(tb), io = bo + bex;
          sh.bjob_grp[bb][j] = (uint8_t)gg;
          sh.bjob_o[bb][j] = (uint8_t)io;
          sh.bjob_n[bb][j] = (uint8_t)bc;
          unsigned m = bm;
          for (int k = 0; k < bc; ++k) {
            sh.bdesc[bb][io + k] = pdesc(fs, bshare ? 1 + __builtin_ctz(m) : 9, gg);
            m &= m - 1u;
          }
        }
        if (half == 0) took0 = tb;
        else took1 = tb;
        bo += wave_sum_dpp(take ? bc : 0);
        bj += __popcll(tb);
        if ((wb & ~tb) != 0ull) break;  // the batch is full
      }
      if (lane == fs) {
        st0 &= ~took0;
        st1 &= ~took1;
      }
    }
    if (lane == 0) {
      sh.nbitems[bb] = bo;
      sh.nbjobs[bb] = bj;
      sh.bslot[bb] = fs;
    }
  };
  // wave 0: stage the event window starting at step s0
  auto refill = [&](int s0) {
    const int ne = min(kEvBuf, E - s0);
    const uint4* src = reinterpret_cast<const uint4*>(rp.ev + s0);
    for (int i = lane; i < ne * 2; i += 64) reinterpret_cast<uint4*>(sh.ev)[i] = gget(src + i);
    for (int i = lane; i < ne; i += 64) sh.evg[i] = gget(evg + s0 + i);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  // wave 0, lane k < K: step ps's granule of workgroup k
  auto poll = [&](int ps) -> unsigned long long {
    return lane < K ? gload(gr + (size_t)(ps & 1) * K + lane) : 0ull;
  };
  // wave 0: the exchange of the pending step ps (every workgroup's granule), from an earlier poll
  auto finish_exchange = [&](int ps, unsigned long long pv, unsigned* W, int* cnt) -> bool {
    if (K == 1) {
      *W = pkey;
      *cnt = pcnt;
      return true;
    }
    const unsigned tag = (unsigned)(ps + 1) & kTagMask;
    unsigned spins = 0;
    bool ok = true;
    while (!__all(lane >= K || ((unsigned)pv & kTagMask) == tag)) {
      if (++spins > kSpinLimit) { ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
      pv = poll(ps);
    }
    const unsigned kk = lane < K ? (unsigned)(pv >> 32) : 0u;
    const int cc = lane < K ? (int)((pv >> kTagBits) & (unsigned long long)kCntMask) : 0;
    *W = (unsigned)wave_max_dpp((int)kk);
    *cnt = wave_sum_dpp(cc);
    return ok;
  };
  // wave 0: the pending step's result and, if this workgroup owned the winner and it bound, the commit
  // (the virtual slot becomes the slot; kg >= 0: its key in group kg is vgk, every other group stale)
  auto commit = [&](int ps, unsigned W, int wcnt, int kg, unsigned vgk, double F0v) {
    const bool owner = pb >= 0 && W != 0u && W == pkey;
    if (lane == 0) {
      ResultDev out{-1, 0, 0, wcnt, ST_UNSCHED};
      bool write = W == 0u && w == 0;  // nobody feasible: workgroup 0 reports
      if (owner) {
        write = true;
        if (pmask < 0) {  // Reserve failed: allocateGpuId returned "" / panicked
          out.status = ST_ERROR;
        } else {
          out.status = ST_OK;
          out.score = result_score(rp, wcnt, hkey_score(W), 0, 0);
          out.node = lo + pb;  // name rank; k_memo_finish maps it to the node index
          out.gpu_mask = pmask;
        }
      }
      if (write) gput(rp.res + ps, out);
    }
    if (owner && pmask >= 0 && lane == pb) {
      rec = vrec;
      store_node(&sh.nodes[pb], vrec);
      sh.F0[pb] = F0v;
      if (kg >= 0) s_gk[kg * kSlots + pb] = vgk;
      st0 = all0 & ((kg >= 0 && kg < 64) ? ~(1ull << kg) : ~0ull);
      st1 = all1 & ((kg >= 64) ? ~(1ull << (kg - 64)) : ~0ull);
    }
  };
  // wave 0: the group keys of a job list -- lane i scores item i (F0 - F through the score steps,
  // keyed with the rank and the item's GPU field), lane j takes job j's max.  fvirt: the virtual
  // slot's F0 (item 0).
  auto item_keys = [&](const unsigned* desc, const double* F, unsigned* kb, int nit, int vrank, double fvirt) {
    for (int i0 = 0; i0 < nit; i0 += 64) {
      const int i = i0 + lane;
      if (i < nit) {
        const unsigned d = desc[i];
        const int slot = (int)(d & 0xffu), code = (int)((d >> 8) & 0xfu);
        const bool virt = slot == kVirt;
        const double F0 = virt ? fvirt : sh.F0[slot];
        const int rank = virt ? vrank : lo + slot;
        kb[i] = code == 0 ? 0u
                          : hkey(ksim_memo::score_lookup_dev(F0 - F[i], sh.th), rank, code <= 8 ? 15 - (code - 1) : 0);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  auto job_key = [&](const unsigned* kb, int o, int n, int rank, bool share) -> unsigned {
    unsigned k = share ? hkey(0, rank, 0) : 0u;  // share: feasible with no fitting GPU
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c < n) k = kb[o + c] > k ? kb[o + c] : k;
    return k;
  };

  __syncthreads();
  if (wv == 0 && E > 0) {
    refill(0);
    build_lists(0, false, -1, 1);  // (an empty-step-parity batch: nothing in flight yet)
    if (lane == 0) { sh.nbitems[1] = 0; sh.nbjobs[1] = 0; }
  }
  __syncthreads();

  for (int s = 0; s < E; ++s) {
    const int eb = s & (kEvBuf - 1);
    // ---- F: one wave per critical item (wave 0 first issues the pending exchange's loads)
    unsigned long long pv = 0ull;
    tr(s, 0);
    if (wv == 0 && pend && K > 1) pv = poll(s - 1);
    {
      const int nit = __builtin_amdgcn_readfirstlane(sh.nitems);
      for (int it = wv; it < nit; it += kPWaves) {
        const double F = item_F(sh.desc[it], sh.nodes, s_gpod, typed, sh.tp, rp.ncpu, rp.nt, lane, fold);
        if (lane == 0) sh.F[it] = F;
      }
    }
    lds_barrier();
    mark(0);
    if (wv != 0) {
      // ---- waves 1-15: the bulk batch listed at step s-1 (its slot is not the one D commits now)
      const int bb = (s - 1) & 1;
      const int nb = __builtin_amdgcn_readfirstlane(sh.nbitems[bb]);
      if (s >= 1 && wv - 1 < nb) {
        const double F = item_F(sh.bdesc[bb][wv - 1], sh.nodes, s_gpod, typed, sh.tp, rp.ncpu, rp.nt, lane, fold);
        if (lane == 0) sh.bF[bb][wv - 1] = F;
      }
    } else {
      // ---- D: wave 0
      tr(s, 1);
      const PodDev p = uniform_pod(&sh.ev[eb]);
      const int g = __builtin_amdgcn_readfirstlane(sh.evg[eb]);
      // 1. keys: the critical jobs (the virtual job, job 0, kept in registers) and the bulk batch of step s-2
      const bool vjob = pend && pb >= 0 && pmask >= 0;
      const double F0v = vjob ? sh.F[0] : 0.0;
      unsigned vgk = 0u;
      {
        const int nit = __builtin_amdgcn_readfirstlane(sh.nitems), nj = __builtin_amdgcn_readfirstlane(sh.njobs);
        item_keys(sh.desc, sh.F, sh.kbuf, nit, lo + pb, F0v);
        for (int j0 = 0; j0 < nj; j0 += 64) {
          const int j = j0 + lane;
          unsigned k = 0u;
          if (j < nj) {
            const int slot = sh.job_slot[j], jg = sh.job_grp[j], o = sh.job_o[j], n = sh.job_n[j];
            const bool virt = slot == kVirt;
            k = job_key(sh.kbuf, virt ? o + 1 : o, virt ? n - 1 : n, virt ? lo + pb : lo + slot,
                        is_share_pod(s_gpod[jg]));
            if (!virt) s_gk[jg * kSlots + slot] = k;
          }
          if (j0 == 0 && vjob) vgk = (unsigned)__builtin_amdgcn_readlane((int)k, 0);
        }
        const int bb = s & 1;
        const int nbi = __builtin_amdgcn_readfirstlane(sh.nbitems[bb]), nbj = __builtin_amdgcn_readfirstlane(sh.nbjobs[bb]);
        if (s >= 2 && nbj > 0) {
          const int fs = __builtin_amdgcn_readfirstlane(sh.bslot[bb]);
          item_keys(sh.bdesc[bb], sh.bF[bb], sh.bkbuf, nbi, 0, 0.0);
          if (lane < nbj) {
            const int jg = sh.bjob_grp[bb][lane];
            const unsigned k = job_key(sh.bkbuf, sh.bjob_o[bb][lane], sh.bjob_n[bb][lane], lo + fs, is_share_pod(s_gpod[jg]));
            s_gk[jg * kSlots + fs] = k;
          }
        }
      }
      mark(1);
      // 2. the slice's best key over the fresh keys, the pending slot excluded (Filter per lane), and the
      //    pending slot as it is (pre) and with the pending Bind applied (post)
      const bool fa = lane < ns && filter_node(rec, p);
      const unsigned ka = fa ? s_gk[g * kSlots + lane] : 0u;
      const bool fx = fa && lane != pb;
      int A = wave_max_dpp((int)(fx ? ka : 0u));
      int cnt = (int)__popcll(__ballot(fx));
      bool fpre = false, fpost = false;
      unsigned kpre = 0u, kpost = 0u;
      if (pb >= 0) {
        fpre = ((__ballot(fa) >> pb) & 1ull) != 0ull;
        kpre = (unsigned)__builtin_amdgcn_readlane((int)ka, pb);
        fpost = fpre;
        kpost = kpre;
        if (pmask >= 0) {
          fpost = filter_node(vrec, p);
          kpost = fpost ? vgk : 0u;
        }
      }
      mark(2);
      tr(s, 2);
      bool ok = true;
      unsigned W = 0u;
      int wcnt = 0;
      if (pend) ok = finish_exchange(s - 1, pv, &W, &wcnt);
      mark(3);
      tr(s, 3);
      if (ok) {
        const bool bound = pend && pb >= 0 && W != 0u && W == pkey && pmask >= 0;
        if (pb >= 0) {
          const unsigned kb = bound ? kpost : kpre;
          A = (int)((unsigned)A > kb ? (unsigned)A : kb);
          cnt += (bound ? fpost : fpre) ? 1 : 0;
        }
        // publish step s first, then the pending step's result and commit
        if (K > 1 && lane == 0)
          gstore(gr + (size_t)(s & 1) * K + w, ((unsigned long long)(unsigned)A << 32) |
                                                   ((unsigned long long)(unsigned)(cnt & kCntMask) << kTagBits) |
                                                   (unsigned long long)((unsigned)(s + 1) & kTagMask));
        tr(s, 4);
        if (pend) commit(s - 1, W, wcnt, g, vgk, F0v);
        // Reserve + Bind of the new candidate into the virtual slot
        int nb = -1, nmask = -1;
        if (A != 0) {
          nb = hkey_rank((unsigned)A) - lo;
          NodeV bn = readlane_node(rec, nb);
          nmask = select_gpus(bn, p, rp.gpusel, hkey_gpu((unsigned)A), rp.seed, s);
          if (nmask >= 0) {
            bind_node(bn, p, nmask, +1);
            if (lane == 0) store_node(&sh.nodes[kVirt], bn);
          }
          vrec = bn;
        }
        pend = true;
        pb = nb;
        pkey = (unsigned)A;
        pmask = nmask;
        pcnt = cnt;
        mark(4);
        if (s + 1 < E) {
          const int eb1 = (s + 1) & (kEvBuf - 1);
          if (eb1 == 0) refill(s + 1);
          build_lists(eb1, nb >= 0 && nmask >= 0, nb, s & 1);
          if (prof && lane == 0) {
            sh.prof[7] += (unsigned long long)sh.nitems;
            sh.prof[8] += (unsigned long long)sh.ncrit;
            sh.prof[9] += (unsigned long long)sh.nbitems[s & 1];
          }
        }
        mark(5);
        tr(s, 5);
      } else if (lane == 0) {
        sh.stop = 1;
        atomicOr(a.fail, 1);
      }
    }
    lds_barrier();
    mark(6);
    if (sh.stop) break;
  }
  // the last step's exchange and commit (no key is read any more)
  if (wv == 0 && pend && !sh.stop) {
    unsigned W;
    int wcnt;
    const unsigned long long pv = K > 1 ? poll(E - 1) : 0ull;
    if (finish_exchange(E - 1, pv, &W, &wcnt)) commit(E - 1, W, wcnt, -1, 0u, 0.0);
    else if (lane == 0) { sh.stop = 1; atomicOr(a.fail, 1); }
  }
  if (prof && tid == 0) {
    sh.prof[10] = __builtin_amdgcn_s_memtime() - c_start;
    sh.prof[11] = __builtin_amdgcn_s_memrealtime() - t_start;
  }
  __syncthreads();
  if (prof && tid < kPProf) a.prof[(size_t)blockIdx.x * kPProf + tid] = sh.prof[tid];
  // final cluster state (wave 0's registers)
  if (wv == 0 && !sh.stop && lane < ns) store_node(rp.nodes + rank2idx[lo + lane], rec);
}

}  // namespace ksim_pmemo

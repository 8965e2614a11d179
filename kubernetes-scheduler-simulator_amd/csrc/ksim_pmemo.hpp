// ksim_pmemo.hpp -- pipelined memoised FGD replay (k_pmemo).
//
// k_memo (ksim_memo.hpp) runs every pod step through one serial chain: the owner of the step's class
// learns the previous winner (a cross-CU granule), evaluates that node's F for the class, decides
// and publishes -- the hand-off and the critical F in series, ~3.15 us per step at C2.  k_pmemo puts
// k_replay's pipelining (ksim_replay.hpp) on memoised keys, so the hand-off overlaps the step's work:
//
//   - node slices: replica r is run by K co-resident workgroups, workgroup w owning the name ranks
//     [w S, w S + S) with S <= 64 (one wave-0 lane per slot).  LDS holds the slice's records, the F
//     of every slot's current state and the packed key of every (score group, slot) pair:
//     gk[g][slot] = the group's best (score, GPU) on that node with the rank (hkey), the Filter NOT
//     applied -- groups share the candidate states (same cpu_nz, milli, num: fgd_score.go:99-149),
//     and the per-class Filter is evaluated when a step reads the key (one lane per slot);
//   - the only slot of a slice that step s can change is the slice's own candidate b (its best key
//     for step s).  Right after publishing step s a workgroup works on step s+1 with b excluded,
//     and evaluates b twice: as it is (pre) and in a VIRTUAL slot holding b with step s's Reserve +
//     Bind applied (post).  When step s's exchange completes it commits (it owned the winner: the
//     virtual slot becomes b) and publishes step s+1 with post or pre (selectHost over the union,
//     generic_scheduler.go:187-212);
//   - staleness: a committed slot's keys are stale in every group but the step's (bit per (slot,
//     group)).  Each step's work list holds the critical items -- the virtual slot's F0 and the
//     step group's candidates on it, the step group's candidates on every slot still stale in it --
//     and fills the rest of the round's 16 wave slots with stale (slot, group) pairs of one focus
//     slot (bulk), so a changed node's keys become fresh within a few steps while no step waits on
//     a key it does not read.
//
// Per pod step s (every workgroup of the replica):
//   F   one wave per listed item: fgd_candidate + wave_F (frag.go's sequential fp64 bins, the same
//       bits as frag_F);                                                                  | barrier
//   K   one wave per job (slot, group): the candidates' score steps (score_lookup_dev), the group key
//       = max (ties: lowest GPU, fgd_score.go:128), the stale bit cleared;               | barrier
//   D   wave 0: the slice's best key for step s over the fresh keys with b excluded (Filter per
//       lane), the exchange of step s-1 (granules polled since the F round), the commit and the
//       result of step s-1, b's version, the granule of step s, Reserve + Bind of the new candidate
//       into the virtual slot, and the work list of step s+1.                           | barrier
// Every key read in D is fresh, and b's versions are the same keys k_hmemo / k_replay / the oracle
// compute (the same device functions), so the decisions are theirs.
//
// Scope: FGD replicas on create-only streams (no report, no profile), N <= 64 K, K <= 64 co-resident
// workgroups, <= 128 score groups, the FGD / best / worst / random GPU selectors.  The host takes
// k_memo / k_hmemo / k_replay otherwise.
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
constexpr int kVirt = kSlots;                    // slot index of the virtual node
constexpr int kMaxGroups = 128;                  // two u64 stale words per slot
constexpr int kBulkJobs = kPWaves;               // bulk jobs per step (one K round)
constexpr int kMaxJobs = 1 + kSlots + kBulkJobs;
constexpr int kMaxItems = 9 + 8 * kSlots + kPWaves + 15;
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
};

struct __align__(16) PShared {
  PodDev ev[kEvBuf];
  int evg[kEvBuf];
  TypDev tp[kMaxTypical];
  double th[104];
  NodeRec nodes[kSlots + 1];                    // slot kVirt: the pending candidate after its Bind
  double F0[kSlots + 2];                        // F of every slot's current state (kVirt: the virtual's)
  unsigned long long stale[kSlots + 1][2];      // bit g: gk[g][slot] is stale
  double F[kMaxItems];
  uint8_t item_job[kMaxItems];
  uint8_t item_code[kMaxItems];                 // fgd_candidate: 0 current, 1..8 GPU, 9 Sub
  uint8_t job_slot[kMaxJobs];
  uint8_t job_grp[kMaxJobs];
  uint8_t job_n[kMaxJobs];
  uint8_t pad_[(16 - (2 * kMaxItems + 3 * kMaxJobs) % 16) % 16];
  uint16_t job_o[kMaxJobs];
  uint16_t pad2_[(8 - kMaxJobs % 8) % 8];
  int nitems, njobs, vslot, stop;
  unsigned vgk;                                 // the virtual slot's key in the step's group
  int pad3_[3];
};
static_assert(sizeof(PShared) % 16 == 0, "keep the dynamic regions 16-B aligned");

// Dynamic LDS: PShared | PodDev gpod[Gmax] | u32 gk[Gmax][kSlots] | f64 fold[kPWaves][kFoldBuf].
inline size_t pmemo_lds(int Gmax) {
  return sizeof(PShared) + (size_t)Gmax * sizeof(PodDev) + (size_t)Gmax * kSlots * 4 +
         (size_t)kPWaves * ksim_memo::kFoldBuf * 8;
}

// Wave-uniform 64-bit readlane.
__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
  return ksim_replay::readlane_u64(v, l);
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
  const int* rank2idx = reinterpret_cast<const int*>(rp.tags + (size_t)N * kTagStride);
  const int* evg = a.evg + (size_t)gi * a.stride;
  unsigned long long* gr = a.gran + (size_t)gi * 2 * K;
  const int E = rp.n_events;
  const bool typed = rp.typed != 0;

  // ---- start-up: the slice (slot = rank - lo), the groups, the initial keys, the tables
  for (int i = tid; i < ns; i += kPBlock) store_node(&sh.nodes[i], load_node(rp.nodes + rank2idx[lo + i]));
  for (int g = tid; g < G; g += kPBlock) s_gpod[g] = a.gpod[(size_t)gi * a.Gmax + g];
  for (int x = tid; x < G * ns; x += kPBlock) {
    const int g = x / ns, i = x - g * ns;
    const int st = a.nstate[(size_t)gi * a.Npad + lo + i];
    s_gk[g * kSlots + i] = a.gsc[((size_t)gi * a.Gmax + g) * a.Smax + st] | hkey_rankbits(lo + i);
  }
  for (int i = tid; i < rp.nt * 2; i += kPBlock) reinterpret_cast<uint4*>(sh.tp)[i] = reinterpret_cast<const uint4*>(tp)[i];
  for (int i = tid; i < 102; i += kPBlock) sh.th[i] = a.th[i];
  for (int i = tid; i < 2 * (kSlots + 1); i += kPBlock) (&sh.stale[0][0])[i] = 0ull;
  if (tid == 0) { sh.stop = 0; sh.nitems = 0; sh.njobs = 0; sh.vslot = -1; sh.vgk = 0u; }
  __syncthreads();
  for (int i = tid; i < ns; i += kPBlock) sh.F0[i] = eval_fgd_item(load_node(&sh.nodes[i]), 0, PodDev{}, rp, tp);

  // ---- wave 0: the work list of step s1 (event window slot eb1): virtual slot vb (or -1), then the
  // slots stale in the step's group, then bulk pairs of one focus slot while the round has room.
  auto build_list = [&](int eb1, int vb) {
    const int g1 = __builtin_amdgcn_readfirstlane(sh.evg[eb1]);
    const PodDev gp = uniform_pod(&s_gpod[g1]);
    const bool share = is_share_pod(gp);
    int o = 0, nj = 0;
    if (vb >= 0) {  // item 0: F0 of the virtual slot, then its candidates in the step's group
      const NodeV vn = uniform_node(&sh.nodes[kVirt]);
      const unsigned f0 = ksim_memo::first_mask_lanes(vn, lane);
      const unsigned cm = share ? (f0 & ksim_memo::ge_mask(vn, gp.milli)) : 0x100u;
      const int nc = __popc(cm);
      if (lane == 0) {
        sh.job_slot[0] = (uint8_t)kVirt;
        sh.job_grp[0] = (uint8_t)g1;
        sh.job_o[0] = 0;
        sh.job_n[0] = (uint8_t)(1 + nc);
        sh.item_job[0] = 0;
        sh.item_code[0] = 0;
        sh.vslot = vb;
      }
      if (lane < nc) {
        unsigned m = cm;
        for (int q = 0; q < lane; ++q) m &= m - 1u;
        sh.item_job[1 + lane] = 0;
        sh.item_code[1 + lane] = (uint8_t)(share ? 1 + __builtin_ctz(m) : 9);
      }
      o = 1 + nc;
      nj = 1;
    }
    // critical: every slot stale in the step's group
    const unsigned long long st0 = lane < ns ? sh.stale[lane][0] : 0ull, st1 = lane < ns ? sh.stale[lane][1] : 0ull;
    const unsigned long long gbit = 1ull << (g1 & 63);
    const bool crit = ((g1 < 64 ? st0 : st1) & gbit) != 0ull;
    unsigned cm = 0u;
    if (crit) {
      const NodeV nd = load_node(&sh.nodes[lane]);
      cm = share ? first_of_class(nd, gp.milli) : 0x100u;
    }
    int tot = 0;
    const int nc = __popc(cm);
    const int excl = lane_prefix(nc, &tot);
    const unsigned long long cb = __ballot(crit);
    if (crit) {
      const int j = nj + lanes_before(cb), io = o + excl;
      sh.job_slot[j] = (uint8_t)lane;
      sh.job_grp[j] = (uint8_t)g1;
      sh.job_o[j] = (uint16_t)io;
      sh.job_n[j] = (uint8_t)nc;
      unsigned m = cm;
      for (int k = 0; k < nc; ++k) {
        sh.item_job[io + k] = (uint8_t)j;
        sh.item_code[io + k] = (uint8_t)(share ? 1 + __builtin_ctz(m) : 9);
        m &= m - 1u;
      }
    }
    nj += __popcll(cb);
    o += tot;
    // bulk: the lowest slot with other stale groups, its groups in order while the round has room
    const bool other = lane < ns && ((st0 & (g1 < 64 ? ~gbit : ~0ull)) | (st1 & (g1 < 64 ? ~0ull : ~gbit))) != 0ull;
    const unsigned long long ob = __ballot(other);
    int cap = kPWaves - o, jcap = kBulkJobs - nj;
    if (ob != 0ull && cap > 0 && jcap > 0) {
      const int fs = __builtin_ctzll(ob);
      const NodeV fn = uniform_node(&sh.nodes[fs]);
      const unsigned f0 = ksim_memo::first_mask_lanes(fn, lane);
      const unsigned long long fw0 = readlane64(st0, fs), fw1 = readlane64(st1, fs);
      for (int half = 0; half < 2; ++half) {
        const int gg = half * 64 + lane;
        const unsigned long long fw = half ? fw1 : fw0;
        const bool want = gg < G && gg != g1 && ((fw >> lane) & 1ull) != 0ull;
        int bc = 0;
        bool bshare = false;
        if (want) {
          const PodDev q = s_gpod[gg];
          bshare = is_share_pod(q);
          bc = bshare ? __popc(f0 & ksim_memo::ge_mask(fn, q.milli)) : 1;
        }
        int btot = 0;
        const int bex = lane_prefix(bc, &btot);
        const unsigned long long wb = __ballot(want);
        const bool take = want && bex + bc <= cap && lanes_before(wb) < jcap;
        const unsigned long long tb = __ballot(take);
        if (take) {
          const int j = nj + lanes_before(tb), io = o + bex;
          sh.job_slot[j] = (uint8_t)fs;
          sh.job_grp[j] = (uint8_t)gg;
          sh.job_o[j] = (uint16_t)io;
          sh.job_n[j] = (uint8_t)bc;
          unsigned m = bshare ? (f0 & ksim_memo::ge_mask(fn, s_gpod[gg].milli)) : 0x100u;
          for (int k = 0; k < bc; ++k) {
            sh.item_job[io + k] = (uint8_t)j;
            sh.item_code[io + k] = (uint8_t)(bshare ? 1 + __builtin_ctz(m) : 9);
            m &= m - 1u;
          }
        }
        const int used = wave_sum_dpp(take ? bc : 0);
        nj += __popcll(tb);
        o += used;
        cap -= used;
        jcap -= __popcll(tb);
        if ((wb & ~tb) != 0ull || cap <= 0 || jcap <= 0) break;  // the round is full
      }
    }
    if (lane == 0) {
      sh.nitems = o;
      sh.njobs = nj;
      if (vb < 0) sh.vslot = -1;
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

  // wave 0's pending step (published, not committed): candidate slot, key, Reserve mask, count
  int pb = -1, pmask = -1, pcnt = 0;
  unsigned pkey = 0u;
  bool pend = false;
  const unsigned long long all0 = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
  const unsigned long long all1 = G > 64 ? (G >= 128 ? ~0ull : ((1ull << (G - 64)) - 1ull)) : 0ull;
  __syncthreads();
  if (wv == 0 && E > 0) {
    refill(0);
    build_list(0, -1);
  }
  __syncthreads();

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
  // wave 0: the pending step's result and, if this workgroup owned the winner, its commit (the virtual
  // slot becomes the slot; kg >= 0: the virtual's key in group kg is fresh, every other group stale)
  auto commit = [&](int ps, unsigned W, int wcnt, int kg) {
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
    if (owner && pmask >= 0) {
      if (lane < 2) reinterpret_cast<uint4*>(&sh.nodes[pb])[lane] = reinterpret_cast<const uint4*>(&sh.nodes[kVirt])[lane];
      else if (lane == 2) sh.F0[pb] = sh.F0[kVirt];
      else if (lane == 3 && kg >= 0) s_gk[kg * kSlots + pb] = sh.vgk;
      else if (lane == 4) sh.stale[pb][0] = all0 & ((kg >= 0 && kg < 64) ? ~(1ull << kg) : ~0ull);
      else if (lane == 5) sh.stale[pb][1] = all1 & ((kg >= 64) ? ~(1ull << (kg - 64)) : ~0ull);
    }
    return owner && pmask >= 0;
  };

  for (int s = 0; s < E; ++s) {
    const int eb = s & (kEvBuf - 1);
    // ---- F: one wave per item (wave 0 first issues the pending exchange's loads)
    unsigned long long pv = 0ull;
    if (wv == 0 && pend && K > 1) pv = poll(s - 1);
    {
      const int nit = __builtin_amdgcn_readfirstlane(sh.nitems);
      for (int it = wv; it < nit; it += kPWaves) {
        const int j = __builtin_amdgcn_readfirstlane((int)sh.item_job[it]);
        const int code = __builtin_amdgcn_readfirstlane((int)sh.item_code[it]);
        const int slot = __builtin_amdgcn_readfirstlane((int)sh.job_slot[j]);
        const int g = __builtin_amdgcn_readfirstlane((int)sh.job_grp[j]);
        const NodeV m = uniform_node(&sh.nodes[slot]);
        const PodDev gp = uniform_pod(&s_gpod[g]);
        int cpuL, total;
        uint32_t gs[4];
        fgd_candidate(m, code, gp, &cpuL, gs, &total);
        const double F = ksim_memo::wave_F(cpuL, gs, total, 1u << m.gpu_type(), typed, sh.tp, rp.ncpu, rp.nt, lane,
                                           s_fold + (size_t)wv * ksim_memo::kFoldBuf);
        if (lane == 0) sh.F[it] = F;
      }
    }
    __syncthreads();
    // ---- K: one wave per job, the group key from its candidates' score steps
    {
      const int nj = __builtin_amdgcn_readfirstlane(sh.njobs);
      for (int j = wv; j < nj; j += kPWaves) {
        const int slot = __builtin_amdgcn_readfirstlane((int)sh.job_slot[j]);
        const int g = __builtin_amdgcn_readfirstlane((int)sh.job_grp[j]);
        const int o = __builtin_amdgcn_readfirstlane((int)sh.job_o[j]);
        const int m = __builtin_amdgcn_readfirstlane((int)sh.job_n[j]);
        const bool virt = slot == kVirt;
        const int vs = virt ? __builtin_amdgcn_readfirstlane(sh.vslot) : slot;
        const double F0 = virt ? sh.F[o] : sh.F0[slot];
        const int c0 = virt ? o + 1 : o, nc = virt ? m - 1 : m;
        const int rank = lo + vs;
        const bool share = is_share_pod(uniform_pod(&s_gpod[g]));
        int k = 0;
        if (lane < nc) {
          const int code = sh.item_code[c0 + lane];
          k = (int)hkey(ksim_memo::score_lookup_dev(F0 - sh.F[c0 + lane], sh.th), rank, share ? 15 - (code - 1) : 0);
        }
        unsigned gkey = (unsigned)wave_max_dpp(k);
        if (share) {
          const unsigned z = hkey(0, rank, 0);  // feasible with no fitting GPU
          gkey = gkey > z ? gkey : z;
        }
        if (lane == 0) {
          if (virt) {
            sh.vgk = gkey;
            sh.F0[kVirt] = F0;
          } else {
            s_gk[g * kSlots + slot] = gkey;
            __hip_atomic_fetch_and(&sh.stale[slot][g >> 6], ~(1ull << (g & 63)), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    }
    __syncthreads();
    // ---- D: wave 0
    if (wv == 0) {
      const PodDev p = uniform_pod(&sh.ev[eb]);
      const int g = __builtin_amdgcn_readfirstlane(sh.evg[eb]);
      // the slice's best key over the fresh keys, the pending slot excluded (Filter per lane)
      bool f = false;
      if (lane < ns && lane != pb) f = filter_node(load_node(&sh.nodes[lane]), p);
      int A = (int)(f ? s_gk[g * kSlots + lane] : 0u);
      A = wave_max_dpp(A);
      int cnt = (int)__popcll(__ballot(f));
      // the pending slot as it is (pre) and with the pending Bind applied (post)
      bool fpre = false, fpost = false;
      unsigned kpre = 0u, kpost = 0u;
      if (pb >= 0) {
        fpre = filter_node(uniform_node(&sh.nodes[pb]), p);
        kpre = fpre ? s_gk[g * kSlots + pb] : 0u;
        fpost = fpre;
        kpost = kpre;
        if (pmask >= 0) {
          fpost = filter_node(uniform_node(&sh.nodes[kVirt]), p);
          kpost = fpost ? sh.vgk : 0u;
        }
      }
      bool ok = true, bound = false;
      if (pend) {
        unsigned W;
        int wcnt;
        ok = finish_exchange(s - 1, pv, &W, &wcnt);
        if (ok) bound = commit(s - 1, W, wcnt, g);
      }
      if (ok) {
        if (pb >= 0) {
          const unsigned kb = bound ? kpost : kpre;
          A = (int)((unsigned)A > kb ? (unsigned)A : kb);
          cnt += (bound ? fpost : fpre) ? 1 : 0;
        }
        // publish step s
        if (K > 1 && lane == 0)
          gstore(gr + (size_t)(s & 1) * K + w, ((unsigned long long)(unsigned)A << 32) |
                                                   ((unsigned long long)(unsigned)(cnt & kCntMask) << kTagBits) |
                                                   (unsigned long long)((unsigned)(s + 1) & kTagMask));
        // Reserve + Bind of the new candidate into the virtual slot
        int nb = -1, nmask = -1;
        if (A != 0) {
          nb = hkey_rank((unsigned)A) - lo;
          NodeV bn = uniform_node(&sh.nodes[nb]);
          nmask = select_gpus(bn, p, rp.gpusel, hkey_gpu((unsigned)A), rp.seed, s);
          if (nmask >= 0) {
            bind_node(bn, p, nmask, +1);
            if (lane == 0) store_node(&sh.nodes[kVirt], bn);
          }
        }
        pend = true;
        pb = nb;
        pkey = (unsigned)A;
        pmask = nmask;
        pcnt = cnt;
        if (s + 1 < E) {
          const int eb1 = (s + 1) & (kEvBuf - 1);
          if (eb1 == 0) refill(s + 1);
          build_list(eb1, (nb >= 0 && nmask >= 0) ? nb : -1);
        }
      } else if (lane == 0) {
        sh.stop = 1;
        atomicOr(a.fail, 1);
      }
    }
    __syncthreads();
    if (sh.stop) break;
  }
  // the last step's exchange and commit (no key is read any more)
  if (wv == 0 && pend && !sh.stop) {
    unsigned W;
    int wcnt;
    const unsigned long long pv = K > 1 ? poll(E - 1) : 0ull;
    if (finish_exchange(E - 1, pv, &W, &wcnt)) (void)commit(E - 1, W, wcnt, -1);
    else if (lane == 0) { sh.stop = 1; atomicOr(a.fail, 1); }
  }
  __syncthreads();
  // final cluster state
  if (!sh.stop)
    for (int i = tid; i < ns; i += kPBlock) store_node(rp.nodes + rank2idx[lo + i], load_node(&sh.nodes[i]));
}

}  // namespace ksim_pmemo

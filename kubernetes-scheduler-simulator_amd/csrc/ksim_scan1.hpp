// ksim_scan1.hpp -- single-workgroup replay of a cheap-policy replica (k_scan1<policy>).
//
// The paper sweep (C4) runs 170 replicas per policy, one workgroup each (K = 1), beside the FGD
// group; the whole sweep is bound by how many replicas the CUs hold at once, not by one chain.
// k_replay's K = 1 workgroup is 1024 threads (16 waves) with a pipelined exchange it does not need
// at K = 1.  k_scan1 is the K = 1 form for BestFit, DotProduct, GpuPacking, GpuClustering and the
// hash-contract Random: 256 threads (4 waves), so a CU holds as many replicas as its LDS allows,
// and ONE workgroup barrier per pod step:
//   - thread t scans the node slots t, t + 256, ... (Filter, the policy's Score, the packed key
//     max-score / smallest-name, the feasible count, Score errors, BestFit's raw min / max) into
//     registers, each wave reduces them (DPP) into its slot of a double-buffered partial table;
//   - barrier;
//   - every wave reads the four partials and takes the same cycle decision (selectHost over the
//     packed keys, the single-feasible shortcut, the Score-error abort: k_replay's commit);
//   - the wave whose threads scan the winner's slot runs Reserve's GPU selector and the Bind on it
//     and reports; slot s is only ever read by thread s % 256, so the Bind needs no second barrier.
// GpuClustering keeps one presence bit per affinity tag and node (u16 in LDS) instead of the tag counts:
// on a create-only stream a count only grows, and the score reads only which counts are non-zero
// (clustering_score_mask); the counts themselves change in HBM by fire-and-forget atomics, as for the
// other policies.
// k_scan1_mix<kReport, kReg> runs replicas of all five policies in ONE launch (the policy is chosen per
// workgroup, DotProduct in the paper's merge / max configuration only): the paper sweep's cheap groups
// then need one stream beside the FGD group's instead of five (streams and queues).
// Create-only streams without a profile (the host takes k_replay for anything else); with the
// per-event cluster report (kReport) the Bind also records the node's new record and the previous
// event that changed it (snap / prev, ksim_report.hpp), as k_replay's general form does.  Same
// device functions as k_replay / k_step / the oracle, so the same bits.
#pragma once

namespace ksim_scan1 {

using namespace ksim;

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kEvBuf = 128;
constexpr int kRegSlots = 5;  // kReg: node slots per thread held in VGPRs (N <= 1280, the openb clusters)

struct Scan1Args {
  ReplicaDev* reps;
  const int* rep_list;  // replica of each workgroup
  int N;
  int skip;             // the dead-class skip (every replica's classes fit kDeadWords x 32 bits)
  // The overlapped report's queue (ksim_report.hpp k_report_overlap; null: none): once a workgroup's replay --
  // results, report records, final state -- is visible device-wide, it takes the next slot (done[0], a ticket zeroed
  // before the run) and stores epoch << 32 | its position in the launch there (done[2 + slot]); the report takes
  // replicas in that order, while the longer ones still run.
  unsigned long long* done;
  unsigned epoch;
};
constexpr int kDeadWords = 32;  // dead-class bitmask: class ids < 1024

struct __align__(16) Scan1Part {
  unsigned long long key;  // the wave's best packed key (0: nothing feasible)
  int cnt;                 // feasible nodes
  int err;                 // a feasible node's Score failed
  int lo, hi;              // raw score min / max over the feasible nodes (BestFit's NormalizeScore)
  int pad[2];
};

struct __align__(16) Scan1Shared {
  PodDev ev[kEvBuf];
  Scan1Part part[2][kWaves];  // by decided-step parity: a wave may write step s+1's while another reads step s's
  unsigned dead[kWaves][kDeadWords];  // each wave's copy of the dead classes (every wave decides alike)
};
static_assert(sizeof(Scan1Shared) % 16 == 0, "keep the node records 16-B aligned");

// Dynamic LDS: Scan1Shared | NodeRec nodes[N] (not with kReg) | u16 tag presence[N] rounded up to 16 B
// (GpuClustering, and every k_scan1_mix launch) | i32 last[N] (report)
constexpr int kPolMix = 65;  // scan1_lds's policy id of a k_scan1_mix launch (the presence bits always present)
__host__ __device__ inline size_t scan1_tm_bytes(int N) { return ((size_t)N * sizeof(uint16_t) + 15) & ~(size_t)15; }
__host__ __device__ inline size_t scan1_lds(int N, int pol, bool report, bool reg = false) {
  return sizeof(Scan1Shared) + (reg ? 0 : (size_t)N * sizeof(NodeRec)) +
         (pol == POL_CLUSTERING || pol == kPolMix ? scan1_tm_bytes(N) : 0) + (report ? (size_t)N * 4 : 0);
}

// x = c ? y : x field by field (a select of whole structs would take the array's address)
__device__ __forceinline__ void sel_node(NodeV& x, const NodeV& y, bool c) {
  x.cpu_left = c ? y.cpu_left : x.cpu_left;
  x.mem_left = c ? y.mem_left : x.mem_left;
#pragma unroll
  for (int i = 0; i < 4; ++i) x.g[i] = c ? y.g[i] : x.g[i];
  x.meta = c ? y.meta : x.meta;
  x.name_rank = c ? y.name_rank : x.name_rank;
}

// kReg: thread t keeps the records of its slots t + 256 k (k < kRegSlots) in VGPRs instead of LDS, so
// a workgroup needs only a few KB of LDS and a CU holds as many replicas as its registers allow.
// kDpMM: DotProduct in the merge / max configuration only (k_scan1_mix): the closed form, and the
// DotProduct selector's group mask is the merge method's "" (0).  kLdsPol: the policy id the launch's
// LDS layout was sized for (kPol, or kPolMix).
template <int kPol, bool kReport, bool kReg, bool kDpMM = false, int kLdsPol = kPol>
__device__ __forceinline__ void scan1_body(const Scan1Args& a, const ReplicaDev& rp, char* smem) {
  using namespace ksim_replay;
  constexpr bool kTags = kPol == POL_CLUSTERING;  // GpuClustering reads the tag presence per pod step
  constexpr bool kMinMax = kPol == POL_BESTFIT;
  Scan1Shared& sh = *reinterpret_cast<Scan1Shared*>(smem);
  NodeRec* s_nodes = reinterpret_cast<NodeRec*>(smem + sizeof(Scan1Shared));
  uint16_t* s_tm = reinterpret_cast<uint16_t*>(smem + sizeof(Scan1Shared) + (kReg ? 0 : (size_t)a.N * sizeof(NodeRec)));
  int* s_last = reinterpret_cast<int*>(smem + scan1_lds(a.N, kLdsPol, false, kReg));  // report: last event per slot
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = a.N;
  NodeV rn[kReg ? kRegSlots : 1];  // kReg: the records of slots tid + 256 k
  if (kReg) {
#pragma unroll
    for (int k = 0; k < kRegSlots; ++k) {
      rn[k] = NodeV{};
      if (tid + kBlock * k < N) rn[k] = load_node(rp.nodes + tid + kBlock * k);
    }
  } else {
    for (int i = tid; i < N; i += kBlock) store_node(&s_nodes[i], load_node(rp.nodes + i));
  }
  if (kTags)
    for (int i = tid; i < N; i += kBlock) {
      unsigned m = 0u;
#pragma unroll
      for (int k = 0; k < kNumTags; ++k) m |= rp.tags[(size_t)i * kTagStride + k] > 0 ? 1u << k : 0u;
      s_tm[i] = (uint16_t)m;
    }
  if (kReport)
    for (int i = tid; i < N; i += kBlock) s_last[i] = -1;
  for (int i = tid; i < kWaves * kDeadWords; i += kBlock) (&sh.dead[0][0])[i] = 0u;
  unsigned* dead = sh.dead[wv];
  int nd = 0;  // decided (not skipped) steps so far: the partial table's parity
  __syncthreads();

  for (int step = 0; step < rp.n_events; ++step) {
    const int eb = step & (kEvBuf - 1);
    if (eb == 0) {
      // skipped steps have no barrier: wait until no wave reads the old window any more
      if (step > 0) __syncthreads();
      const int nl = min(kEvBuf, rp.n_events - step) * 2;
      const uint4* src = reinterpret_cast<const uint4*>(rp.ev + step);
      for (int i = tid; i < nl; i += kBlock) reinterpret_cast<uint4*>(sh.ev)[i] = src[i];
      __syncthreads();
    }
    const PodDev p = uniform_pod(&sh.ev[eb]);
    // Dead-class skip (create-only streams): Filter is monotone in the resources a creation takes, so an
    // event whose class found no feasible node before finds none now -- unscheduled, 0 feasible, nothing
    // changes.  Every wave keeps its own copy of the dead set and decides alike, so no barrier is needed.
    if (a.skip && ((dead[p.pad >> 5] >> (p.pad & 31)) & 1u)) {
      if (tid == 0) rp.res[step] = ResultDev{-1, 0, 0, 0, ST_UNSCHED};
      continue;
    }
    // ---- scan: Filter + Score of this thread's slots
    unsigned long long best = 0ull;
    int cnt = 0, lo = 0x7fffffff, hi = -1;
    bool err = false;
    auto visit = [&](const NodeV& n, int i) {
      if (filter_scan(n, p)) {
        bool e1 = false;
        int raw;
        if constexpr (kTags) {
          e1 = p.tag == -2;
          raw = e1 ? 0 : clustering_score_mask(s_tm[i], p.tag, n.total());
        } else if constexpr (kPol == POL_DOTPROD && kDpMM) {
          raw = dotprod_merge_max(n, p);
          e1 = raw < 0;  // the framework's range check (<= 100 always)
        } else {
          const int cap = (kPol == POL_DOTPROD && dp_norm(rp.dpcfg) == NORM_NODE) ? rp.cap[i] : 0;
          raw = cheap_score<kPol>(n, p, rp.seed, nullptr, step, &e1, rp.dpcfg, cap);
        }
        const unsigned long long k = pack_key((unsigned)raw, n.name_rank, -1, i);
        best = k > best ? k : best;
        ++cnt;
        err = err || e1;
        if (kMinMax) { lo = min(lo, raw); hi = max(hi, raw); }
      }
    };
    if (kReg) {
#pragma unroll
      for (int k = 0; k < kRegSlots; ++k)
        if (tid + kBlock * k < N) visit(rn[k], tid + kBlock * k);
    } else {
      for (int i = tid; i < N; i += kBlock) visit(load_node(&s_nodes[i]), i);
    }
    best = wave_max_u64_dpp(best);
    cnt = wave_sum_dpp(cnt);
    const bool werr = __any(err);
    if (kMinMax) { lo = wave_min_dpp(lo); hi = wave_max_dpp(hi); }
    Scan1Part* pt = sh.part[nd & 1];
    ++nd;
    if (lane == 0) pt[wv] = Scan1Part{best, cnt, werr ? 1 : 0, lo, hi, {0, 0}};
    __syncthreads();
    // ---- the cycle decision, by every wave (the same values): k_replay's commit at K = 1
    unsigned long long W = 0ull;
    int nfeas = 0, gerr = 0, glo = 0x7fffffff, ghi = -1;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
      const Scan1Part q = pt[k];
      W = q.key > W ? q.key : W;
      nfeas += q.cnt;
      gerr |= q.err;
      if (kMinMax) { glo = min(glo, q.lo); ghi = max(ghi, q.hi); }
    }
    if (a.skip && nfeas == 0 && lane == 0) dead[p.pad >> 5] |= 1u << (p.pad & 31);
    const int loc = key_loc(W);
    const int owner = W != 0ull ? (loc % kBlock) / 64 : 0;  // the wave that scans the winner's slot
    if (wv == owner) {
      ResultDev out{-1, 0, 0, nfeas, ST_UNSCHED};
      if (nfeas > 0) {
        out.status = (nfeas > 1 && gerr) ? ST_ERROR : ST_OK;  // a Score error aborts the cycle
        if (out.status == ST_OK) {
          out.score = result_score(rp, nfeas, key_score(W), glo, ghi);
          NodeV bn;
          if (kReg) {  // the record from the register slot loc / 256 of lane loc % 64
            const int ks = loc / kBlock, src = loc & 63;
            NodeV x = rn[0];
#pragma unroll
            for (int k = 1; k < kRegSlots; ++k) sel_node(x, rn[k], ks == k);  // field-wise: rn stays in VGPRs
            bn.cpu_left = __builtin_amdgcn_readlane(x.cpu_left, src);
            bn.mem_left = __builtin_amdgcn_readlane(x.mem_left, src);
#pragma unroll
            for (int i = 0; i < 4; ++i) bn.g[i] = (uint32_t)__builtin_amdgcn_readlane((int)x.g[i], src);
            bn.meta = (uint32_t)__builtin_amdgcn_readlane((int)x.meta, src);
            bn.name_rank = (uint32_t)__builtin_amdgcn_readlane((int)x.name_rank, src);
          } else {
            bn = uniform_node(&s_nodes[loc]);
          }
          const int sarg = (kPol == POL_DOTPROD && kDpMM) ? (rp.gpusel == SEL_DOTPROD ? 0 : key_gpu(W))
                                                          : sel_arg<kPol == POL_DOTPROD>(rp, bn, p, loc, key_gpu(W));
          const int mask = select_gpus(bn, p, rp.gpusel, sarg, rp.seed, step);
          if (mask < 0) {  // Reserve failed: allocateGpuId returned "" / panicked
            out.status = ST_ERROR;
            out.score = 0;
          } else {
            bind_node(bn, p, mask, +1);
            if (kReg) {
              if (tid == loc % kBlock) {
#pragma unroll
                for (int k = 0; k < kRegSlots; ++k)
                  if (loc / kBlock == k) rn[k] = bn;
              }
            }
            if (lane == 0) {
              if (!kReg) store_node(&s_nodes[loc], bn);
              if (kReport) {  // cluster report: the state this event left, the previous change of the node
                store_node(rp.snap + step, bn);
                rp.prev[step] = s_last[loc];
                s_last[loc] = step;
              }
              if (p.tag >= 0) {
                if (kTags) s_tm[loc] |= (uint16_t)(1u << p.tag);
                tag_add(rp.tags + (size_t)loc * kTagStride, p.tag, +1);  // HBM: an atomic, no read on the path
              }
            }
            out.node = loc;
            out.gpu_mask = mask;
          }
        }
      }
      if (lane == 0) rp.res[step] = out;
    }
  }
  __syncthreads();
  if (kReg) {
#pragma unroll
    for (int k = 0; k < kRegSlots; ++k)
      if (tid + kBlock * k < N) store_node(rp.nodes + tid + kBlock * k, rn[k]);
  } else {
    for (int i = tid; i < N; i += kBlock) store_node(rp.nodes + i, load_node(&s_nodes[i]));
  }
  if (a.done) {  // every wave's stores drained and released at agent scope, the barrier, then the queue entry
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (tid == 0) {
      const unsigned long long slot = __hip_atomic_fetch_add(a.done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.done + 2 + slot, (unsigned long long)a.epoch << 32 | blockIdx.x, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int kPol, bool kReport, bool kReg>
__global__ __launch_bounds__(kBlock) void k_scan1(Scan1Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ReplicaDev rp = a.reps[a.rep_list[blockIdx.x]];
  scan1_body<kPol, kReport, kReg>(a, rp, smem);
}

// Every cheap policy in one launch: workgroup b replays replica rep_list[b] under that replica's policy
// (a uniform branch per workgroup).  The host lists the replicas longest stream first, so the launch
// dispatches the long replays before the short ones fill in behind them.
// Six waves per SIMD (80 VGPRs, no spills; the default register budget gave 91 and five): six replicas per CU
// instead of five while the FGD group holds the rest of the CUs
template <bool kReport, bool kReg>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_scan1_mix(Scan1Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ReplicaDev rp = a.reps[a.rep_list[blockIdx.x]];
  switch (rp.policy) {
    case POL_BESTFIT: scan1_body<POL_BESTFIT, kReport, kReg, false, kPolMix>(a, rp, smem); break;
    case POL_DOTPROD: scan1_body<POL_DOTPROD, kReport, kReg, true, kPolMix>(a, rp, smem); break;
    case POL_PACKING: scan1_body<POL_PACKING, kReport, kReg, false, kPolMix>(a, rp, smem); break;
    case POL_CLUSTERING: scan1_body<POL_CLUSTERING, kReport, kReg, false, kPolMix>(a, rp, smem); break;
    default: scan1_body<POL_RANDOM, kReport, kReg, false, kPolMix>(a, rp, smem); break;
  }
}

}  // namespace ksim_scan1

// ksim_engine.hip -- MI355X (gfx950) scoring engine for the simulator's per-pod
// Filter+Score pass, behind the C ABI of include/ksim_engine.h.
//
// Device layout (HBM, struct-of-records, replica-major):
//   NodeRec  nodes[R][N]   32 B: cpu/mem left, 8 x u16 milli-GPU left, pods left,
//                          gpu count, model id, name rank
//   uint16   tags[R][N][16] GpuClustering affinity counts
//   PodDev   ev_r[E_r]      32 B per event, per replica
//   TypDev   tp[R][256]     typical-pod table (staged into LDS per workgroup)
//   ResultDev res_r[E_r]    24 B per event
//
// One pod step of every replica is ONE kernel launch (k_step):
//   workgroup (256 threads) = one replica x `nodes_per_block` nodes
//   phase 1  one thread per node: Filter; cheap policies score here
//   phase 2  FGD only: the (node, candidate placement) pairs of the workgroup
//            are compacted into an LDS work list and every thread evaluates
//            F = NodeGpuShareFragAmountScore of one candidate state against the
//            LDS-staged typical table (sequential fp64 bins, bit-exact)
//   phase 3  per node: score = int64(sigmoid((F0-Fk)/1000)*100), packed
//            argmax key (score | ~name_rank | gpu), workgroup max-reduce
//   commit   relaxed agent-scope atomics into the replica's Accum; the
//            workgroup that takes the last ticket reads the winner, runs
//            Reserve's GPU selector on it and scatters the Bind update.
// Steps are captured K at a time into a hipGraph (kernel i reads step = base+i;
// a one-thread kernel advances base) so a whole trace replays with no host
// round trip per pod.
#include <dlfcn.h>
#include <unistd.h>
#include <string>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <map>
#include <numeric>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <chrono>
#include <thread>

#include "ksim_device.hpp"
#include "ksim_engine.h"

using namespace ksim;

namespace {

constexpr int kBlock = 256;
constexpr int kNBMax = 64;
constexpr int kMaxCand = 9;
constexpr int kTagStride = 16;

struct StepArgs {
  ReplicaDev* reps;
  Accum* acc;
  int N;
  int NB;
  int bpr;        // workgroups per replica
  int rep_first;  // first replica of this launch
  const int* base;
  int step_off;
  const PodDev* pod_override;  // single-pod calls
  ResultDev* res_override;
  int mode;  // 0: commit (Reserve+Bind), 1: Filter+Score outputs only, 2: shard totals -> send
  unsigned long long* send;        // mode 2: this shard's {best key, nfeas, err, lo | hi << 32}
  const unsigned long long* recv;  // k_shard_commit: the `world` gathered shard records
  int world;
  uint8_t* out_feas;
  int32_t* out_score;
  int32_t* out_gpu;
};

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// allocateGpuId (open_gpu_share.go:252-283) on one node: the replica's gpuSelMethod.
// fgd_gpu: the FGD selector's device for share pods (first max-score index), -1 if none.
// Returns the GPU mask, 0 for pods without GPU milli, -1 where the reference panics / returns "".
// fgd_gpu: the FGD / PWR selectors' GPU index; for SEL_DOTPROD the best match group's GPU mask
// (dotprod_cfg_score, 0 = "": Reserve fails).
__device__ int select_gpus(const NodeV& n, const PodDev& p, int gpusel, int fgd_gpu, uint64_t seed, int step) {
  if (p.milli <= 0) return 0;                                         // open_gpu_share.go:185-187
  if (p.milli < kMilli && p.num > 1) return -1;                       // :266-268 panic
  if (gpusel == SEL_DOTPROD) return fgd_gpu <= 0 ? -1 : fgd_gpu;      // dot_product_score.go:102-107
  if (!is_share_pod(p)) return exclusive_gpu_mask(n, p);              // exclusive branch of every selector
  switch (gpusel) {
    case SEL_FGD:                                                     // fgd_score.go:153-156
    case SEL_PWR:                                                     // pwr_score.go:214-219
      return fgd_gpu < 0 ? -1 : (1 << fgd_gpu);
    case SEL_RANDOM: {                                                // :325-343 (Random contract)
      const uint64_t nk = rand_node_key(seed, step, n.name_rank);
      int pick = -1;
      uint64_t best = 0;
      for (int g = 0; g < kMaxGpu; ++g) {
        if (g < n.gpu_cnt() && n.gl(g) >= p.milli) {
          const uint64_t k = rand_gpu_key(nk, g);
          if (pick < 0 || k > best) { best = k; pick = g; }
        }
      }
      return pick < 0 ? -1 : (1 << pick);
    }
    case SEL_WORST: {                                                 // :305-323
      int c = -1, cv = 0;
#pragma unroll
      for (int g = 0; g < kMaxGpu; ++g) {
        const int v = n.gl(g);
        if (g < n.gpu_cnt() && v >= p.milli && (c < 0 || v > cv)) { c = g; cv = v; }
      }
      return c < 0 ? -1 : (1 << c);
    }
    default: {                                                        // best fit, :285-303
      int c = -1, cv = 0;
#pragma unroll
      for (int g = 0; g < kMaxGpu; ++g) {
        const int v = n.gl(g);
        if (g < n.gpu_cnt() && v >= p.milli && (c < 0 || v < cv)) { c = g; cv = v; }
      }
      return c < 0 ? -1 : (1 << c);
    }
  }
}

// Bind on a register image (see apply_bind).
__device__ __forceinline__ void bind_node(NodeV& n, const PodDev& p, int mask, int sign) {
  n.cpu_left -= sign * p.cpu_req;
  n.mem_left -= sign * p.mem;
  const int pods = n.pods_left() - sign;
  n.meta = (n.meta & 0xffff0000u) | ((uint32_t)pods & 0xffffu);
  const uint32_t d = (uint32_t)(sign * (int)p.milli) & 0xffffu;
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) {
    // u16 lanes never borrow across halves: 0 <= left - milli and left + milli <= 1000
    if ((mask >> g) & 1) n.g[g >> 1] = (g & 1) ? n.g[g >> 1] - (d << 16) : ((n.g[g >> 1] & 0xffff0000u) | ((n.g[g >> 1] - d) & 0xffffu));
  }
}

// Bind: scheduler cache assume (Requested += pod), open-gpu-share cache
// AddOrUpdatePod (devices += milli), NodeInfo.Pods += pod (affinity tags).
__device__ void apply_bind(NodeRec* nr, uint16_t* tags, const PodDev& p, int mask, int sign) {
  NodeV n = load_node(nr);
  n.cpu_left -= sign * p.cpu_req;
  n.mem_left -= sign * p.mem;
  const int pods = n.pods_left() - sign;
  n.meta = (n.meta & 0xffff0000u) | ((uint32_t)pods & 0xffffu);
  const uint32_t d = (uint32_t)(sign * (int)p.milli) & 0xffffu;
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) {
    // u16 lanes never borrow across halves: 0 <= left - milli and left + milli <= 1000
    if ((mask >> g) & 1) n.g[g >> 1] = (g & 1) ? n.g[g >> 1] - (d << 16) : ((n.g[g >> 1] & 0xffff0000u) | ((n.g[g >> 1] - d) & 0xffffu));
  }
  store_node(nr, n);
  if (p.tag >= 0) tags[p.tag] = (uint16_t)((int)tags[p.tag] + sign);
}

// Cluster report bookkeeping of k_step: the state event `step` left on `node` and the previous
// event that changed it (k_replay keeps the same per-node record in LDS).
__device__ __forceinline__ void note_change(const ReplicaDev& rp, int node, int step) {
  store_node(rp.snap + step, load_node(rp.nodes + node));
  rp.prev[step] = rp.last[node];
  rp.last[node] = step;
}

// Bit g set iff GPU g fits `milli` and no lower-index fitting GPU has the same milli left.
__device__ __forceinline__ unsigned first_of_class(const NodeV& n, int milli) {
  unsigned fm = 0u;
  const int cnt = n.gpu_cnt();
#pragma unroll
  for (int g = 0; g < kMaxGpu; ++g) {
    const int v = n.gl(g);
    bool first = g < cnt && v >= milli;
#pragma unroll
    for (int h = 0; h < g; ++h) first = first && !(n.gl(h) == v);
    fm |= first ? (1u << g) : 0u;
  }
  return fm;
}

// ---------------------------------------------------------------------------
// Per-node pieces shared by k_step (one launch per pod) and k_replay (persistent).
// ---------------------------------------------------------------------------

// The selector argument of select_gpus for a winner `n` (global node index `node`): the FGD / PWR
// GPU index from the key, or DotProduct's best-group mask recomputed on the node.
// kDp = false: a kernel specialised on a policy other than DotProduct (no DotProduct selector there).
template <bool kDp = true>
__device__ __forceinline__ int sel_arg(const ReplicaDev& rp, const NodeV& n, const PodDev& p, int node, int key_gpu) {
  if (!kDp || rp.gpusel != SEL_DOTPROD) return key_gpu;
  int gid = 0;
  (void)dotprod_cfg_score(n, p, dp_norm(rp.dpcfg) == NORM_NODE ? rp.cap[node] : 0, rp.dpcfg, &gid);
  return gid;
}

// Raw score of a feasible node under a non-FGD policy (compile-time policy, used by
// k_replay); *err on a Score error.  Same functions and semantics as node_phase1.
// `cap`: the node's MilliCpuCapacity (DotProduct's normMethod "node").
template <int kPol>
__device__ __forceinline__ int cheap_score(const NodeV& n, const PodDev& p, uint64_t seed, const uint16_t* tags,
                                           int step, bool* err, int dpcfg = 0, int cap = 0) {
  *err = false;
  if constexpr (kPol == POL_BESTFIT) {
    const int r = bestfit_score(n, p, n.total());
    if (r == -1) { *err = true; return kBfKeyBias; }
    return r + kBfKeyBias;  // biased (kBfKeyBias)
  } else if constexpr (kPol == POL_DOTPROD) {
    int gid = 0;
    // uniform per replica
    const int r = dpcfg == (DIM_MERGE | NORM_MAX << 4) ? dotprod_merge_max(n, p) : dotprod_cfg_score(n, p, cap, dpcfg, &gid);
    *err = r < 0 || r > 100;  // no NormalizeScore: the framework's range check (framework.go:686-704)
    return r;
  } else if constexpr (kPol == POL_PACKING) {
    bool perr = false;
    const int r = p.milli <= 0 ? 0 : packing_score(n, p, &perr);
    *err = perr;
    return r;
  } else if constexpr (kPol == POL_CLUSTERING) {
    if (p.tag == -2) { *err = true; return 0; }
    return clustering_score(tags, p.tag, n.total());
  } else {
    return (int)(rand_node_key(seed, step, n.name_rank) >> 40);
  }
}

// Filter, then the cheap scores; for FGD only the candidate count.  `tags` may
// point at global memory (k_step) or LDS (k_replay).
__device__ __forceinline__ bool node_phase1(const NodeV& n, const PodDev& p, const ReplicaDev& rp,
                                            const uint16_t* tags, int step, bool share, int* raw, int* nc,
                                            bool* err, int node = 0, int* pgpu = nullptr) {
  *raw = 0;
  *nc = 0;
  *err = false;
  if (!filter_node(n, p)) return false;
  const int total = n.total();
  switch (rp.policy) {
    case POL_FGD:
      // one candidate per DISTINCT milli-left value among the fitting GPUs: placing the pod on
      // any GPU of a value class yields the same multiset of GPU states, hence the same F
      // (frag.go depends on the multiset only) and the same score.
      *nc = share ? 1 + __builtin_popcount(first_of_class(n, p.milli)) : 2;
      break;
    case POL_BESTFIT:
      *raw = bestfit_score(n, p, total);
      *err = *raw == -1;
      *raw = (*err ? 0 : *raw) + kBfKeyBias;  // biased (kBfKeyBias)
      break;
    case POL_DOTPROD: {  // any dimExtMethod / normMethod; *pgpu: the best group's GPU mask
      int gid = 0;
      *raw = dotprod_cfg_score(n, p, rp.cap[node], rp.dpcfg, &gid);
      *err = *raw < 0 || *raw > 100;  // no NormalizeScore: the framework's range check
      if (pgpu) *pgpu = gid;
      break;
    }
    case POL_PACKING: {
      bool perr = false;
      *raw = p.milli <= 0 ? 0 : packing_score(n, p, &perr);
      *err = perr;
      break;
    }
    case POL_CLUSTERING:
      if (p.tag == -2) *err = true;
      else *raw = clustering_score(tags, p.tag, total);
      break;
    case POL_PWR:
    case POL_PWR_FGD: {  // pwr_score.go:48-91 (+ FGD's candidates for the weighted combination)
      int g = -1;
      bool perr = false;
      *raw = pwr_score(n, p, rp.cap[node], rp.cpum[node], *rp.pw, &g, &perr);
      *err = perr;
      if (pgpu) *pgpu = g;
      if (rp.policy == POL_PWR_FGD) *nc = share ? 1 + __builtin_popcount(first_of_class(n, p.milli)) : 2;
      break;
    }
    default:  // POL_RANDOM: RandomScorePlugin.PreScore pick, as a 24-bit hash key
      *raw = (int)(rand_node_key(rp.seed, step, n.name_rank) >> 40);
      break;
  }
  return true;
}

// FGD work list of one node: current state, then one candidate per GPU value class
// (share pod) or the NodeResource.Sub state.
__device__ __forceinline__ void emit_fgd_items(const NodeV& n, const PodDev& p, bool share, int local, int o,
                                               uint8_t* item_node, uint8_t* item_code) {
  item_node[o] = (uint8_t)local;
  item_code[o] = 0;  // current state
  ++o;
  if (share) {
    const unsigned fm = first_of_class(n, p.milli);
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      if ((fm >> g) & 1u) {
        item_node[o] = (uint8_t)local;
        item_code[o] = (uint8_t)(1 + g);  // fgd_score.go:111-118 candidate on GPU g
        ++o;
      }
    }
  } else {
    item_node[o] = (uint8_t)local;
    item_code[o] = 9;  // fgd_score.go:137-141 NodeResource.Sub
  }
}

// F of one candidate state.
__device__ __forceinline__ double eval_fgd_item(const NodeV& m, int code, const PodDev& p, const ReplicaDev& rp,
                                                const TypDev* __restrict__ tp) {
  int gl[kMaxGpu];
  unpack_gl(m, gl);
  int cpuL = m.cpu_left;
  if (code >= 1 && code <= 8) {
    cpuL -= p.cpu_nz;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) gl[g] -= (g == code - 1) ? (int)p.milli : 0;
  } else if (code == 9) {
    bool ok = false;
    const unsigned sm = sub_gpu_mask(gl, m.gpu_cnt(), cpuL, p, &ok);
    if (ok) {
      cpuL -= p.cpu_nz;
#pragma unroll
      for (int g = 0; g < kMaxGpu; ++g)
        if ((sm >> g) & 1u) gl[g] -= p.milli;
    }
  }
  return rp.typed ? frag_F<true>(cpuL, gl, 1u << m.gpu_type(), tp, rp.ncpu, rp.nt)
                  : frag_F<false>(cpuL, gl, 1u << m.gpu_type(), tp, rp.ncpu, rp.nt);
}

// Node score from its candidates' F values; *gpu = lowest GPU index reaching the max (share pods).
__device__ __forceinline__ void finalize_fgd(const double* F, const uint8_t* code, int o, int nc, bool share,
                                             int* raw, int* gpu) {
  const double F0 = F[o];
  *gpu = -1;
  if (share) {
    // candidates are in increasing first-index order: the first max is the lowest GPU index
    // reaching the max, as fgd_score.go:128 picks it
    int best = -1, bs = 0;
    for (int k = 1; k < nc; ++k) {
      const int fs = fgd_frag_score(F0, F[o + k]);
      if (best < 0 || fs > bs) { bs = fs; best = code[o + k] - 1; }
    }
    *raw = bs;
    *gpu = best;
  } else {
    *raw = fgd_frag_score(F0, F[o + 1]);
  }
}

// Winning total weighted score as the reference reports it (0 on the single-feasible shortcut).
__device__ __forceinline__ long long result_score(const ReplicaDev& rp, int nfeas, int wscore, int lo, int hi) {
  if (nfeas <= 1) return 0;
  if (rp.policy == POL_BESTFIT) return (hi > lo ? 100 : 0) * 1000LL;  // NormalizeScore (plugin_utils.go:48-74)
  if (rp.policy == POL_RANDOM) return 100 * 1000LL;
  if (rp.policy == POL_PWR_FGD) return (long long)wscore;  // already w_pwr * PWR + w_fgd * FGD
  // PWRScorePlugin.NormalizeScore maps the max raw score to 100 (and all-equal scores to 100), and
  // the winner holds the max raw score
  if (rp.policy == POL_PWR) return 100 * 1000LL;
  return (long long)wscore * 1000LL;
}


// The end of a scheduling cycle once the cluster-wide best key and counts are known: the result,
// Reserve's GPU selector and the Bind scatter (scheduler.go:509-554).  `node` is the local index
// of the winning node, or -1 when another shard owns it (sharded mode: the result then carries the
// winner's global rank and a provisional status; the owner's record is authoritative).
__device__ void finish_cycle(const StepArgs& a, const ReplicaDev& rp, const PodDev& p, int step, ResultDev* res_slot,
                             unsigned long long best, int nfeas, int anyerr, int glo, int ghi, int node) {
  ResultDev out{-1, 0, 0, nfeas, ST_UNSCHED};
  if (nfeas > 0) {
    out.status = (nfeas > 1 && anyerr) ? ST_ERROR : ST_OK;  // framework.go:650-656: a Score error aborts
    if (out.status == ST_OK) {
      out.score = result_score(rp, nfeas, key_score(best), glo, ghi);
      if (node < 0) {
        out.node = (int)key_rank(best);  // another shard binds
      } else {
        NodeRec* nr = rp.nodes + node;
        const NodeV wn = load_node(nr);
        const int mask = select_gpus(wn, p, rp.gpusel, sel_arg(rp, wn, p, node, key_gpu(best)), rp.seed, step);
        if (mask < 0) {
          out.status = ST_ERROR;  // Reserve failed: allocateGpuId returned "" / panicked
          out.score = 0;
        } else {
          apply_bind(nr, rp.tags + (size_t)node * kTagStride, p, mask, +1);
          if (rp.snap && !a.pod_override) note_change(rp, node, step);
          out.node = rp.node_off + node;
          out.gpu_mask = mask;
        }
      }
    }
  }
  *res_slot = out;
}

// PWR raw scores are energy deltas old - new <= 0 W (pwr_score.go:167,200); biased into the
// non-negative range of the Accum min / max.
constexpr int kPwrBias = 1 << 30;

__global__ __launch_bounds__(kBlock) void k_step(StepArgs a, const TypDev* __restrict__ tp_all) {
  const int r = a.rep_first + (int)blockIdx.x / a.bpr;
  const int b = (int)blockIdx.x % a.bpr;
  const int tid = (int)threadIdx.x;
  const ReplicaDev rp = a.reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  const int step = (a.base ? *a.base : 0) + a.step_off;
  if (!a.pod_override && step >= rp.n_events) return;
  const PodDev p = a.pod_override ? *a.pod_override : rp.ev[step];
  ResultDev* res_slot = a.res_override ? a.res_override : (rp.res + step);

  if (p.flags & kPodDelete) {
    // simulator.go:416-422 deletePod -> informer DeleteFunc -> GpuSharePlugin.removePod
    if ((a.mode == 0 || a.mode == 2) && b == 0 && tid == 0) {
      ResultDev out{-1, 0, 0, 0, ST_DELETED};
      if (p.ref >= 0 && p.ref < step) {
        const ResultDev c = rp.res[p.ref];
        const int local = c.node - rp.node_off;  // sharded: only the owner of the node undoes the bind
        if (c.node >= 0 && c.status == ST_OK && local >= 0 && local < a.N) {
          const PodDev cp = rp.ev[p.ref];
          apply_bind(rp.nodes + local, rp.tags + (size_t)local * kTagStride, cp, c.gpu_mask, -1);
          if (rp.snap && !a.pod_override) note_change(rp, local, step);
        }
        if (c.node >= 0 && c.status == ST_OK) {
          out.node = c.node;
          out.gpu_mask = c.gpu_mask;
        }
      }
      *res_slot = out;
    }
    return;
  }

  __shared__ NodeRec s_node[kNBMax];
  __shared__ int s_off[kNBMax + 1];
  __shared__ uint8_t s_item_node[kNBMax * kMaxCand];
  __shared__ uint8_t s_item_code[kNBMax * kMaxCand];
  __shared__ double s_F[kNBMax * kMaxCand];
  __shared__ unsigned long long s_rkey[kBlock / 64];
  __shared__ int s_rcnt[kBlock / 64], s_rerr[kBlock / 64], s_rlo[kBlock / 64], s_rhi[kBlock / 64];

  const int n0 = b * a.NB;
  const int nb = max(0, min(a.NB, a.N - n0));
  const bool fgd = rp.policy == POL_FGD || rp.policy == POL_PWR_FGD;
  const bool pwr = is_pwr_policy(rp.policy);
  const bool share = is_share_pod(p);

  // ---- phase 1: Filter (+ cheap scores; PWR's raw score) ----
  bool feas = false, err = false;
  int raw = 0, nc = 0, gpu = -1, pgpu = -1;
  NodeV n{};
  if (tid < nb) {
    n = load_node(rp.nodes + n0 + tid);
    store_node(&s_node[tid], n);
    feas = node_phase1(n, p, rp, rp.tags + (size_t)(n0 + tid) * kTagStride, step, share, &raw, &nc, &err, n0 + tid,
                       &pgpu);
  }
  const int praw = raw;  // PWR policies: the PWR score before NormalizeScore

  // ---- phase 2: FGD candidate evaluation over a compacted work list ----
  if (fgd) {
    if (tid < 64) {  // wave 0: exclusive scan of candidate counts
      int v = tid < nb ? nc : 0;
      int incl = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        int w = __shfl_up(incl, o, 64);
        if (tid >= o) incl += w;
      }
      s_off[tid] = incl - v;
      if (tid == 63) s_off[64] = incl;
    }
    __syncthreads();
    if (tid < nb && nc > 0) emit_fgd_items(n, p, share, tid, s_off[tid], s_item_node, s_item_code);
    __syncthreads();
    const int items = s_off[64];
    for (int j = tid; j < items; j += kBlock)
      s_F[j] = eval_fgd_item(load_node(&s_node[s_item_node[j]]), s_item_code[j], p, rp, tp);
    __syncthreads();
    if (tid < nb && feas) finalize_fgd(s_F, s_item_code, s_off[tid], nc, share, &raw, &gpu);
  }

  if (a.mode == 1) {
    if (tid < nb) {
      a.out_feas[n0 + tid] = feas ? 1 : 0;
      a.out_score[n0 + tid] = feas ? (pwr ? praw : raw) : 0;
      a.out_gpu[n0 + tid] =
          feas ? select_gpus(n, p, rp.gpusel, (rp.gpusel == SEL_PWR || rp.gpusel == SEL_DOTPROD) ? pgpu : gpu, rp.seed, step)
               : 0;
    }
    return;
  }
  if (pwr && tid < nb) {
    // phase A of a PWR cycle: PWRScorePlugin.NormalizeScore needs the min / max raw score over the
    // feasible nodes first, so the per-node scores wait in HBM for k_step_pwr (same step, next launch)
    const int fgpu = rp.policy == POL_PWR_FGD ? gpu : -1;
    rp.pws[n0 + tid] = make_int2(feas ? praw : INT_MIN,
                                 (rp.policy == POL_PWR_FGD ? (raw & 0xff) : 0) | ((pgpu + 1) & 0xf) << 8 |
                                     ((fgpu + 1) & 0xf) << 12);
  }
  if (pwr) raw = praw + kPwrBias;  // the min / max accumulators start at -1 (raw PWR scores are <= 0)

  // ---- phase 3: workgroup reduction of the packed argmax key ----
  unsigned long long key = (feas && !pwr) ? pack_key((unsigned)raw, n.name_rank, gpu) : 0ull;
  int cnt = feas ? 1 : 0;
  int lo = feas ? raw : 0x7fffffff, hi = feas ? raw : -1;
  key = wave_max_u64(key);
  cnt = wave_sum_i(cnt);
  const int e = wave_max_i(err ? 1 : 0);
  lo = wave_min_i(lo);
  hi = wave_max_i(hi);
  const int w = tid >> 6;
  if ((tid & 63) == 0) { s_rkey[w] = key; s_rcnt[w] = cnt; s_rerr[w] = e; s_rlo[w] = lo; s_rhi[w] = hi; }
  __syncthreads();
  if (tid != 0) return;
  for (int i = 1; i < kBlock / 64; ++i) {
    key = s_rkey[i] > key ? s_rkey[i] : key;
    cnt += s_rcnt[i];
    lo = min(lo, s_rlo[i]);
    hi = max(hi, s_rhi[i]);
  }
  int errb = s_rerr[0] | s_rerr[1] | s_rerr[2] | s_rerr[3];

  // ---- commit: last workgroup of the replica finishes the cycle ----
  Accum* ac = a.acc + r;
  if (cnt > 0) {
    __hip_atomic_fetch_max(&ac->best, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&ac->nfeas, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_min(&ac->lo, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(&ac->hi, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (errb) __hip_atomic_fetch_or(&ac->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (pwr) return;  // k_step_pwr finishes the cycle
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every contribution performed before the ticket
  const unsigned t = __hip_atomic_fetch_add(&ac->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t != (unsigned)(a.bpr - 1)) return;

  const unsigned long long best = __hip_atomic_exchange(&ac->best, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nfeas = __hip_atomic_exchange(&ac->nfeas, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int anyerr = __hip_atomic_exchange(&ac->err, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int glo = __hip_atomic_exchange(&ac->lo, 0x7fffffff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int ghi = __hip_atomic_exchange(&ac->hi, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&ac->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  if (a.mode == 2) {
    // node-sharded cluster: this shard's totals go to the exchange (k_shard_commit finishes)
    a.send[0] = best;
    a.send[1] = (unsigned long long)nfeas;
    a.send[2] = (unsigned long long)anyerr;
    a.send[3] = (unsigned long long)(unsigned)glo | ((unsigned long long)(unsigned)ghi << 32);
    return;
  }
  // the rank -> node index map lives right after the replica's tags (see host)
  const int* rank2idx = reinterpret_cast<const int*>(rp.tags + (size_t)a.N * kTagStride);
  finish_cycle(a, rp, p, step, res_slot, best, nfeas, anyerr, glo, ghi, best ? rank2idx[key_rank(best)] : -1);
}

// Phase B of a PWR / PWR+FGD cycle (after k_step's phase A of the same step): the normalized PWR
// score (pwr_score.go:104-141) with the replica's min / max raw score, the weighted sum with FGD
// (framework.go:686-704, generic_scheduler.go:511-519), the packed argmax key, and the last
// workgroup of the replica finishes the cycle as k_step does.
__global__ __launch_bounds__(kBlock) void k_step_pwr(StepArgs a) {
  const int r = a.rep_first + (int)blockIdx.x / a.bpr;
  const int b = (int)blockIdx.x % a.bpr;
  const int tid = (int)threadIdx.x;
  const ReplicaDev rp = a.reps[r];
  if (!is_pwr_policy(rp.policy)) return;
  const int step = (a.base ? *a.base : 0) + a.step_off;
  if (!a.pod_override && step >= rp.n_events) return;
  const PodDev p = a.pod_override ? *a.pod_override : rp.ev[step];
  if (p.flags & kPodDelete) return;
  ResultDev* res_slot = a.res_override ? a.res_override : (rp.res + step);
  Accum* ac = a.acc + r;
  const int lo = __hip_atomic_load(&ac->lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int hi = __hip_atomic_load(&ac->hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __shared__ unsigned long long s_rkey[kBlock / 64];
  const int n0 = b * a.NB;
  const int nb = max(0, min(a.NB, a.N - n0));
  unsigned long long key = 0ull;
  if (tid < nb) {
    const int2 v = rp.pws[n0 + tid];
    if (v.x != INT_MIN) {
      const int norm = pwr_normalize(v.x + kPwrBias, lo, hi);
      const int pg = ((v.y >> 8) & 0xf) - 1, fg = ((v.y >> 12) & 0xf) - 1;
      const int total = rp.policy == POL_PWR_FGD ? rp.w_pwr * norm + rp.w_fgd * (v.y & 0xff) : norm;
      key = pack_key((unsigned)total, rp.nodes[n0 + tid].name_rank, rp.gpusel == SEL_PWR ? pg : fg);
    }
  }
  key = wave_max_u64(key);
  const int w = tid >> 6;
  if ((tid & 63) == 0) s_rkey[w] = key;
  __syncthreads();
  if (tid != 0) return;
  for (int i = 1; i < kBlock / 64; ++i) key = s_rkey[i] > key ? s_rkey[i] : key;
  if (key) __hip_atomic_fetch_max(&ac->best, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the contribution performed before the ticket
  const unsigned t = __hip_atomic_fetch_add(&ac->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t != (unsigned)(a.bpr - 1)) return;
  const unsigned long long best = __hip_atomic_exchange(&ac->best, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nfeas = __hip_atomic_exchange(&ac->nfeas, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int anyerr = __hip_atomic_exchange(&ac->err, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int glo = __hip_atomic_exchange(&ac->lo, 0x7fffffff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int ghi = __hip_atomic_exchange(&ac->hi, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&ac->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int* rank2idx = reinterpret_cast<const int*>(rp.tags + (size_t)a.N * kTagStride);
  finish_cycle(a, rp, p, step, res_slot, best, nfeas, anyerr, glo, ghi, best ? rank2idx[key_rank(best)] : -1);
}

// Node-sharded cluster (ksim_engine_set_shard): one workgroup reduces the `world` shard records
// gathered by the exchange and finishes the cycle; only the shard owning the winning node binds.
// Node ranks are global and shard-contiguous (local node i has rank node_off + i).
__global__ __launch_bounds__(64) void k_shard_commit(StepArgs a) {
  const ReplicaDev rp = a.reps[0];
  const int step = (a.base ? *a.base : 0) + a.step_off;
  if (step >= rp.n_events || threadIdx.x != 0) return;
  const PodDev p = rp.ev[step];
  if (p.flags & kPodDelete) return;  // k_step applied it on the owner
  unsigned long long best = 0ull;
  int nfeas = 0, anyerr = 0, glo = 0x7fffffff, ghi = -1;
  for (int k = 0; k < a.world; ++k) {
    const unsigned long long* r4 = a.recv + 4 * k;
    best = r4[0] > best ? r4[0] : best;
    const int c = (int)r4[1];
    nfeas += c;
    anyerr |= (int)r4[2];
    if (c > 0) {
      glo = min(glo, (int)(unsigned)(r4[3] & 0xffffffffull));
      ghi = max(ghi, (int)(unsigned)(r4[3] >> 32));
    }
  }
  const int local = best ? (int)key_rank(best) - rp.node_off : -1;
  finish_cycle(a, rp, p, step, rp.res + step, best, nfeas, anyerr, glo, ghi, (local >= 0 && local < a.N) ? local : -1);
}

// In-process shard group: every shard's record to every shard's exchange buffer (one launch).
__global__ void k_shard_gather(unsigned long long* const* sends, unsigned long long* const* recvs, int world) {
  const int i = (int)threadIdx.x;  // world * world * 4 <= 1024
  if (i >= world * world * 4) return;
  const int dst = i / (world * 4), src = (i / 4) % world, f = i & 3;
  recvs[dst][4 * src + f] = sends[src][f];
}

#include "ksim_replay.hpp"
#include "ksim_report.hpp"
#include "ksim_memo.hpp"
#include "ksim_hmemo.hpp"

// ---------------------------------------------------------------------------
// k_replay: the whole event stream of every replica in one launch (see ksim_replay.hpp).
// Dynamic LDS: ReplayShared | NodeRec nodes[S+1] | u16 tags[S+1][16] | f64 F0[S+1] | f64 E0[S+1] |
// i32x2 pe[S+1] | i32 last[S+1] | i32 praw[S+1] | i32 pinf[S+1].
//
// PWR: NormalizeScore (pwr_score.go:104-141) sends exactly the nodes with the max raw score to 100,
// so the argmax of the normalized score is the argmax of the raw one: one key exchange per step, the
// raw score biased into the 24-bit key field.  PWR + FGD (the weighted sum, framework.go:686-704)
// needs the cluster's min / max raw PWR score before any node's total is known: an A round (min,
// max, feasible count, Score error) per step, then the normalized totals of the slice and the key
// round, which overlaps the next step's evaluation as for every other policy.
constexpr int kPfFeas = 1 << 30, kPfErr = 1 << 29;  // pinf flags (low 16 bits: FGD score, GPU choices)
constexpr int kPwrKeyBias = 1 << 23;                // raw PWR score -> 24-bit key field
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Polled granules of the pending exchange, per wave-0 lane: workgroups lane + 64 j, j < kSub.
template <int kSub>
struct GranV {
  unsigned long long g0[kSub], g1[kSub], g2[kSub];
};

// kSub = ceil(K / 64): 1 for K <= 64, 4 for K <= 256 (one wave-0 lane polls kSub workgroups); 0 for
// K = 1 (no exchange), where the cheap policies are built for two 1024-thread workgroups per CU (64
// VGPRs: 8 waves per SIMD), so the paper sweep's single-workgroup replicas pack two to a CU.
// kGeneral: the KSIM_PROFILE timers, the cluster-report stores and delete events (bind history);
// the lean instantiation (none of them: the bench, the paper sweeps, C5) compiles them out of the
// step loop, as k_memo's does.
#include "ksim_random_go.hpp"
#include "ksim_scan1.hpp"

template <int kPol, int kSub, bool kGeneral>
__global__ __launch_bounds__(ksim_replay::kRBlock, (kSub == 0 && kPol >= POL_BESTFIT && kPol <= POL_RANDOM &&
                                                     kPol != POL_DOTPROD) ? 8 : 1)
void k_replay(ksim_replay::ReplayArgs a,
                                                                 const TypDev* __restrict__ tp_all) {
  using namespace ksim_replay;
  constexpr int kS = kSub > 0 ? kSub : 1;  // granule columns per polling lane (K = 1 polls none)
  constexpr bool kPwr = kPol == POL_PWR;
  constexpr bool kPF = kPol == POL_PWR_FGD;
  constexpr bool kFgd = kPol == POL_FGD || kPF;  // the FGD candidate evaluation
  constexpr bool kMinMax = kPol == POL_BESTFIT;  // NormalizeScore needs the raw min / max
  constexpr bool kErr = kPol == POL_BESTFIT || kPol == POL_DOTPROD || kPol == POL_PACKING || kPol == POL_CLUSTERING || kPwr || kPF;
  // all LDS is dynamic (no static __shared__ in front of it), carved 16-byte aligned
  extern __shared__ __attribute__((aligned(16))) char smem[];
  ReplayShared& sh = *reinterpret_cast<ReplayShared*>(smem);
  const int r = a.rep_list[(int)blockIdx.x / a.K];
  const int w = (int)blockIdx.x % a.K;
  // the exchange: Kx columns (every workgroup of the replica; a node-sharded group, a.xK: every workgroup of
  // every shard), this workgroup's column wx
  const int Kx = a.xK > 0 ? a.xK : a.K;
  const int wx = (int)blockIdx.x % Kx;
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const ReplicaDev rp = a.reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  const int n_lo = w * a.S;
  const int ns = max(0, min(a.S, (a.group ? rp.n_local : a.N) - n_lo));
  constexpr bool kTags = kPol == POL_CLUSTERING;  // GpuClustering reads the tag counts per pod step
  const RLayout L = replay_layout(a.S, kPol, kGeneral, kPF ? a.pm_c : 0);
  ReplayFgd& fs = *reinterpret_cast<ReplayFgd*>(smem + L.fgd);  // FGD launches only
  NodeRec* s_nodes = reinterpret_cast<NodeRec*>(smem + L.nodes);
  uint16_t* s_tags = reinterpret_cast<uint16_t*>(smem + L.tags);  // kTags only
  // the other policies keep the slice's tag counts in HBM (changed by a Bind / delete, read by none)
  uint16_t* g_tags = rp.tags + (size_t)n_lo * kTagStride;
  double* s_F0 = reinterpret_cast<double*>(smem + L.F0);
  // PWR policies: the cached energy of each slot's current state (kEnergyStale: recompute) and the
  // node's static energy terms {rc, ncpus << 3 | CPU model} (energy_static)
  double* s_E0 = reinterpret_cast<double*>(smem + L.E0);
  int2* s_pe = reinterpret_cast<int2*>(smem + L.pe);
  // cluster report: the last event that changed each slot (-1: none yet)
  int* s_last = reinterpret_cast<int*>(smem + L.last);
  int* s_praw = reinterpret_cast<int*>(smem + L.praw);  // PWR+FGD per-slot scratch of the current step
  int* s_pinf = reinterpret_cast<int*>(smem + L.pinf);
  // PWR+FGD: each class's two most recent cluster-wide raw PWR ranges {lo0, hi0, lo1, hi1} (most recent first;
  // classes alias mod kPfGuess -- a guess only ever saves a round, the decision checks it)
  int4* s_gtab = reinterpret_cast<int4*>(smem + L.gtab);
  // PWR+FGD memo (a.pm_c > 0): every class's Filter + Score of every real slot, kept while the slot's
  // record is unchanged (s_pver), so a step evaluates only the slots changed since its class last came
  // and the virtual slot
  const bool pmon = kPF && a.pm_c > 0;
  unsigned* s_pver = reinterpret_cast<unsigned*>(smem + L.pver);
  uint2* s_pm = reinterpret_cast<uint2*>(smem + L.pm);
  auto pm_bump = [&](int i) {  // (one lane) slot i's record changed: its entries are stale
    unsigned v = s_pver[i] + 1u;
    if (v == kPmInvalid) {  // the version field wraps: forget the slot's entries first
      v = 0u;
      for (int c = 0; c < a.pm_c; ++c) s_pm[(size_t)c * a.S + i].y = kPmInvalid << 18;
    }
    s_pver[i] = v;
  };
  // hist[step]: (node, mask+1) bound here | (-1,0) no winner | (-2,0) winner elsewhere | (-3,0) Reserve failed here
  // (null when no replica of the launch has a delete event: nothing ever reads it)
  int2* hist = (kGeneral && a.hist) ? a.hist + (size_t)(r * a.K + w) * a.hist_stride : nullptr;
  NodeRec* const snap = kGeneral ? rp.snap : nullptr;
  unsigned long long* gr = a.gran + (size_t)(blockIdx.x / Kx) * 2 * Kx * kGranW;

  for (int i = tid; i < ns; i += kRBlock) store_node(&s_nodes[i], load_node(rp.nodes + n_lo + i));
  if (kTags)
    for (int i = tid; i < ns * kTagStride; i += kRBlock) s_tags[i] = rp.tags[(size_t)n_lo * kTagStride + i];
  if (kGeneral)
    for (int i = tid; i <= ns; i += kRBlock) s_last[i] = -1;
  if (kPwr || kPF) {
    for (int i = tid; i < (int)(sizeof(PowerDev) / 8); i += kRBlock)
      reinterpret_cast<unsigned long long*>(&sh.pw)[i] = reinterpret_cast<const unsigned long long*>(rp.pw)[i];
    for (int i = tid; i < ns; i += kRBlock) s_pe[i] = energy_static(rp.cap[n_lo + i], rp.cpum[n_lo + i], *rp.pw);
    for (int i = tid; i <= ns; i += kRBlock) s_E0[i] = kEnergyStale;
  }
  if (kPF)
    for (int i = tid; i < kPfGuess; i += kRBlock) s_gtab[i] = make_int4(1, 0, 1, 0);  // lo > hi: never a range
  if (pmon) {
    for (int i = tid; i <= ns; i += kRBlock) s_pver[i] = a.pm_ver0;
    for (int i = tid; i < a.pm_c * a.S; i += kRBlock) s_pm[i] = make_uint2(0u, kPmInvalid << 18);
  }
  if (kFgd) {
    for (int i = tid; i <= ns; i += kRBlock) s_F0[i] = -1.0;  // every cached F stale
    for (int i = tid; i < rp.nt * 2; i += kRBlock)
      reinterpret_cast<uint4*>(fs.tp)[i] = reinterpret_cast<const uint4*>(tp)[i];
  }
  auto reset_agg = [&]() {
    sh.agg_key = 0ull;
    sh.agg_key1 = 0ull;
    sh.agg_cnt = 0;
    sh.agg_err = 0;
    sh.agg_lo = 0x7fffffff;
    sh.agg_hi = kPF ? INT_MIN : -1;
  };
  if (tid == 0) { sh.stop = 0; sh.nitems = 0; sh.pend_valid = 0; sh.pend_b = -1; reset_agg(); }
  for (int i = tid; i < 32; i += kRBlock) sh.dead[i] = 0u;

  // wave 0's copy of the pending exchange (the previous pod step, published, not committed)
  int p_step = 0, p_seq = 0, p_b = -1, p_mask = -1, seq = 0, p_cls = 0;
  int p_tag = -1;  // the pending Bind's affinity tag (policies keeping the tag counts in HBM)
  unsigned long long p_key = 0ull;
  int p_st0 = 0, p_st1 = 0, p_st2 = 0, p_st3 = 0;  // K == 1: the step's own totals

  // phase timer (wall clock, 100 MHz): only with a profile buffer, thread 0 of each workgroup
  const bool prof = kGeneral && a.prof != nullptr;
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

  // Wave 0, lane k: the granules of workgroups k, k+64, .. (< K) of the pending exchange
  // (relaxed agent-scope loads).
  auto poll_once = [&](GranV<kS>& g) {
    const unsigned long long* slot = gr + (size_t)(p_seq & 1) * Kx * kGranW;
#pragma unroll
    for (int j = 0; j < kS; ++j) {
      const int k = lane + 64 * j;
      if (k < Kx) {
        g.g0[j] = gload(slot + (size_t)k * kGranW + 0);
        g.g1[j] = gload(slot + (size_t)k * kGranW + 1);
        g.g2[j] = gload(slot + (size_t)k * kGranW + 2);
      }
    }
  };
  // Wave 0, PWR+FGD: ONE round per pod step.  NormalizeScore needs the cluster-wide min / max raw PWR score
  // before any node's weighted total exists; instead of a round for it and then a key round, every slice
  // publishes its A totals (min, max, feasible count | Score error: words 4-6) together with its best key under
  // each of the two ranges last seen for the pod's class (words 0-1, 2-3).  When the true range is one of them
  // (or at most one node is feasible: no normalisation), that key column decides; else every slice re-keys
  // the step under the true range from its scratch (kept two steps) and a miss round (words 7-8) decides.
  // The round overlaps the next pod's evaluation like every policy's key round.
  // (x: an earlier poll when `have`, issued before the evaluation's last barrier so its latency overlaps the wait)
  auto pf_collect = [&](unsigned long long (&x)[kS][7], bool have, int* gc, int* ge, int* gl, int* gh,
                        unsigned long long* W0, unsigned long long* W1) -> bool {
    const unsigned long long* slot = gr + (size_t)(p_seq & 1) * Kx * kGranW;
    const unsigned long long tag = (unsigned long long)(unsigned)(p_seq + 1) << 32;
    auto load = [&]() {
#pragma unroll
      for (int j = 0; j < kS; ++j) {
        const int k = lane + 64 * j;
        if (k < Kx) {
#pragma unroll
          for (int q = 0; q < 7; ++q) x[j][q] = gload(slot + (size_t)k * kGranW + q);
        }
      }
    };
    auto ready = [&]() {
      bool r = true;
#pragma unroll
      for (int j = 0; j < kS; ++j) {
        bool t = true;
#pragma unroll
        for (int q = 0; q < 7; ++q) t = t && (x[j][q] & ~0xffffffffull) == tag;
        r = r && (lane + 64 * j >= Kx || t);
      }
      return r;
    };
    if (!have) load();
    unsigned spins = 0;
    bool ok = true;
    while (!__all(ready())) {
      if (++spins > kSpinLimit) { ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
      load();
    }
    if (prof && lane == 0) sh.prof[8] += spins;
    int cs = 0, lo = INT_MAX, hi = INT_MIN, e1 = 0;
    unsigned long long b0 = 0ull, b1 = 0ull;
#pragma unroll
    for (int j = 0; j < kS; ++j) {
      if (lane + 64 * j < Kx) {
        const unsigned long long k0 = ((x[j][1] & 0xffffffffull) << 32) | (x[j][0] & 0xffffffffull);
        const unsigned long long k1 = ((x[j][3] & 0xffffffffull) << 32) | (x[j][2] & 0xffffffffull);
        const unsigned st = (unsigned)x[j][6];
        const int c = (int)(st & 0x7fffffffu);
        cs += c;
        e1 |= (int)(st >> 31);
        if (c > 0) {
          lo = min(lo, (int)(unsigned)x[j][4]);
          hi = max(hi, (int)(unsigned)x[j][5]);
        }
        b0 = k0 > b0 ? k0 : b0;
        b1 = k1 > b1 ? k1 : b1;
      }
    }
    *gc = wave_sum_dpp(cs);
    *ge = __any(e1 != 0) ? 1 : 0;
    *gl = wave_min_dpp(lo);
    *gh = wave_max_dpp(hi);
    *W0 = wave_max_u64_dpp(b0);
    *W1 = wave_max_u64_dpp(b1);
    return ok;
  };
  auto pf_miss_round = [&](unsigned long long mine, unsigned long long* W) -> bool {
    unsigned long long* slot = gr + (size_t)(p_seq & 1) * Kx * kGranW;
    const unsigned long long tag = (unsigned long long)(unsigned)(p_seq + 1) << 32;
    if (lane == 0) {
      gstore(slot + (size_t)wx * kGranW + 7, tag | (mine & 0xffffffffull));
      gstore(slot + (size_t)wx * kGranW + 8, tag | (mine >> 32));
    }
    unsigned long long x0[kS], x1[kS];
    auto load = [&]() {
#pragma unroll
      for (int j = 0; j < kS; ++j) {
        const int k = lane + 64 * j;
        if (k < Kx) {
          x0[j] = gload(slot + (size_t)k * kGranW + 7);
          x1[j] = gload(slot + (size_t)k * kGranW + 8);
        }
      }
    };
    auto ready = [&]() {
      bool r = true;
#pragma unroll
      for (int j = 0; j < kS; ++j)
        r = r && (lane + 64 * j >= Kx || ((x0[j] & ~0xffffffffull) == tag && (x1[j] & ~0xffffffffull) == tag));
      return r;
    };
    load();
    unsigned spins = 0;
    bool ok = true;
    while (!__all(ready())) {
      if (++spins > kSpinLimit) { ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
      load();
    }
    unsigned long long b = 0ull;
#pragma unroll
    for (int j = 0; j < kS; ++j)
      if (lane + 64 * j < Kx) {
        const unsigned long long k = ((x1[j] & 0xffffffffull) << 32) | (x0[j] & 0xffffffffull);
        b = k > b ? k : b;
      }
    *W = wave_max_u64_dpp(b);
    return ok;
  };
  // Wave 0: the pending step's exchange result -- every workgroup's granules (K > 1) or
  // this workgroup's own totals (K == 1); g holds an earlier poll.  Returns the winning key.
  auto exchange = [&](GranV<kS>& g, int* gc, int* ge, int* gl, int* gh, bool* ok) -> unsigned long long {
    *ok = true;
    if (Kx == 1) {
      *gc = p_st0; *ge = p_st1; *gl = p_st2; *gh = p_st3;
      return p_key;
    }
    const unsigned long long tag = (unsigned long long)(unsigned)(p_seq + 1) << 32;
    auto ready = [&]() {
      bool r = true;
#pragma unroll
      for (int j = 0; j < kS; ++j)
        r = r && (lane + 64 * j >= Kx || ((g.g0[j] & ~0xffffffffull) == tag && (g.g1[j] & ~0xffffffffull) == tag &&
                                          (g.g2[j] & ~0xffffffffull) == tag));
      return r;
    };
    unsigned spins = 0;
    while (!__all(ready())) {
      if (++spins > kSpinLimit) { *ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
      poll_once(g);
    }
    if (prof && lane == 0) sh.prof[8] += spins;
    int c = 0, lo = 0x7fffffff, hi = -1;
    bool e1 = false;
    unsigned long long best = 0ull;
#pragma unroll
    for (int j = 0; j < kS; ++j) {
      const bool in = lane + 64 * j < Kx;
      const unsigned st = in ? (unsigned)(g.g2[j] & 0xffffffffull) : 0u;
      const int cj = (int)(st & 0x1ffff);
      c += cj;
      e1 = e1 || (st >> 31) != 0u;
      const unsigned long long kj = in ? ((g.g1[j] & 0xffffffffull) << 32) | (g.g0[j] & 0xffffffffull) : 0ull;
      if (kMinMax && cj > 0) {
        // BestFit: a slice's max raw score is its key's score field; its bit 17 says whether its scores differ.
        // NormalizeScore needs only whether any two feasible scores differ (result_score: hi > lo).
        const int sj = key_score(kj);
        lo = min(lo, sj - (int)((st >> 17) & 1u));
        hi = max(hi, sj);
      }
      best = kj > best ? kj : best;
    }
    *gc = wave_sum_dpp(c);
    *ge = __any(e1) ? 1 : 0;
    *gl = 0x7fffffff;
    *gh = -1;
    if (kMinMax) {
      *gl = wave_min_dpp(lo);
      *gh = wave_max_dpp(hi);
    }
    return wave_max_u64_dpp(best);
  };

  // Wave 0: commit the pending step -- the owner of the winning node turns the virtual slot
  // into that node (Reserve + Bind were applied to it when it was prepared).  Lanes 0-6 copy.
  auto commit = [&](unsigned long long W, int nfeas, int gerr, int glo, int ghi) {
    const bool owner = W != 0ull && W == p_key;
    // nothing feasible anywhere: the pending event's class stays infeasible (create-only streams)
    if (a.skip && nfeas == 0 && lane == 0) sh.dead[p_cls >> 5] |= 1u << (p_cls & 31);
    ResultDev out{-1, 0, 0, nfeas, ST_UNSCHED};
    int2 hrec = make_int2(-1, 0);
    bool writer = w == 0;
    if (nfeas > 0) {
      out.status = (nfeas > 1 && gerr) ? ST_ERROR : ST_OK;
      if (out.status == ST_OK) {
        out.score = result_score(rp, nfeas, key_score(W), glo, ghi);
        writer = owner;  // the owner of the winning node reports
        hrec.x = -2;
        if (owner) {
          if (p_mask < 0) {  // Reserve failed: allocateGpuId returned "" / panicked
            out.status = ST_ERROR;
            out.score = 0;
            hrec.x = -3;
          } else {
            if (lane < 2) reinterpret_cast<uint4*>(&s_nodes[p_b])[lane] = reinterpret_cast<const uint4*>(&s_nodes[ns])[lane];
            else if (lane < 6 && kTags)
              reinterpret_cast<uint2*>(&s_tags[(size_t)p_b * kTagStride])[lane - 2] =
                  reinterpret_cast<const uint2*>(&s_tags[(size_t)ns * kTagStride])[lane - 2];
            else if (lane == 2 && !kTags && p_tag >= 0) tag_add(g_tags + (size_t)p_b * kTagStride, p_tag, +1);
            else if (lane == 6 && kFgd) s_F0[p_b] = s_F0[ns];
            else if (lane == 8 && kPF) { s_praw[p_b] = s_praw[ns]; s_pinf[p_b] = s_pinf[ns]; }
            else if (lane == 10 && pmon) pm_bump(p_b);
            else if (lane == 9 && (kPwr || kPF)) s_E0[p_b] = s_E0[ns];
            else if (lane == 7 && snap) {  // cluster report: the post-Bind record (the virtual slot)
              store_node(snap + p_step, load_node(&s_nodes[ns]));
              rp.prev[p_step] = s_last[p_b];
              s_last[p_b] = p_step;
            }
            out.node = a.group ? (int)key_rank(W) : n_lo + p_b;
            out.gpu_mask = p_mask;
            hrec = make_int2(n_lo + p_b, p_mask + 1);
          }
        }
      }
    }
    if (lane == 0) {
      if (hist) hist[p_step] = hrec;
      if (writer) {
        rp.res[p_step] = out;
      } else if (a.group && w == 0) {  // a shard that does not own the winner names it (the owner's record rules)
        // (the owner's shard -- its ranks are [node_off, node_off + n_local) -- has its owning workgroup write)
        const uint32_t rk = key_rank(W);
        if (rk - (uint32_t)rp.node_off >= (uint32_t)rp.n_local) {
          out.node = (int)rk;
          rp.res[p_step] = out;
        }
      }
    }
  };

  // PWR+FGD: a feasible slot's packed key under the range [lo, hi]: w_pwr * NormalizeScore(PWR) + w_fgd * FGD
  // (framework.go:686-704; unsigned arithmetic: a guessed range that is not the step's may give any value, and
  // is then never used)
  auto pf_key = [&](int praw, int inf, int lo, int hi, int i) -> unsigned long long {
    // pwr_normalize in 32 bits: on the step's true range 0 <= praw - lo <= hi - lo < 2^24, so (praw - lo) * 100 < 2^31
    const unsigned norm = lo == hi ? 100u : (unsigned)(praw - lo) * 100u / (unsigned)(hi - lo);
    const unsigned total = (unsigned)rp.w_pwr * norm + (unsigned)rp.w_fgd * (unsigned)(inf & 0xff);
    const int kg = rp.gpusel == SEL_PWR ? ((inf >> 8) & 0xf) - 1 : ((inf >> 12) & 0xf) - 1;
    return pack_key(total, load_node(&s_nodes[i]).name_rank, kg, i);
  };
  // Wave 0: the pending step's best key of this slice under the true range, from its scratch
  auto pf_rekey = [&](int lo, int hi) -> unsigned long long {
    const int* q_praw = s_praw + (p_step & 1) * (a.S + 1);
    const int* q_pinf = s_pinf + (p_step & 1) * (a.S + 1);
    unsigned long long b = 0ull;
    for (int i = lane; i < ns; i += 64) {
      const int inf = q_pinf[i];
      if (inf & kPfFeas) {
        const unsigned long long k = pf_key(q_praw[i], inf, lo, hi, i);
        b = k > b ? k : b;
      }
    }
    return wave_max_u64_dpp(b);
  };
  // Wave 0: decide and commit the pending step.  The owner of the winner applies the virtual node when the winner
  // is the node it prepared (guess 0's local best), else Reserve + Bind on the winner's slot itself; `overlapped`:
  // this step's evaluation already ran, and *redo asks for it again (one of its slots changed under it).
  auto pf_resolve = [&](unsigned long long (&x)[kS][7], bool have, bool overlapped, bool* redo) -> bool {
    *redo = false;
    int gc = p_st0, ge = p_st1, gl = p_st2, gh = p_st3;
    const unsigned long long p_key1 = sh.pf_key1;
    const int4 p_g = sh.pf_g;
    unsigned long long W0 = p_key, W1 = p_key1;
    if (Kx > 1 && !pf_collect(x, have, &gc, &ge, &gl, &gh, &W0, &W1)) return false;
    const bool m0 = gc <= 1 || (gl == p_g.x && gh == p_g.y);  // at most one feasible node: no normalisation
    const bool m1 = !m0 && gl == p_g.z && gh == p_g.w;
    unsigned long long W = m0 ? W0 : W1, mine = m0 ? p_key : p_key1;
    if (!m0 && !m1 && !ge) {  // (a Score error aborts the cycle: no winner needed)
      if (prof && lane == 0) sh.prof[9] += 1ull;  // KSIM_PROFILE: misses (low half), re-evaluations (high)
      mine = pf_rekey(gl, gh);
      W = mine;
      if (Kx > 1 && !pf_miss_round(mine, &W)) return false;
    }
    if (gc > 1 && lane == 0 && a.pf_guess) {  // the class's most recent ranges (every workgroup updates alike)
      int4& t = s_gtab[p_cls & (kPfGuess - 1)];
      if (!(t.x == gl && t.y == gh)) t = make_int4(gl, gh, t.x, t.y);
    }
    // commit
    const bool owner = W != 0ull && W == mine;
    if (a.skip && gc == 0 && lane == 0) sh.dead[p_cls >> 5] |= 1u << (p_cls & 31);
    ResultDev out{-1, 0, 0, gc, ST_UNSCHED};
    int2 hrec = make_int2(-1, 0);
    bool writer = w == 0;
    if (gc > 0) {
      out.status = (gc > 1 && ge) ? ST_ERROR : ST_OK;  // framework.go:650-656: a Score error aborts
      if (out.status == ST_OK) {
        out.score = result_score(rp, gc, key_score(W), gl, gh);
        writer = owner;
        hrec.x = -2;
        if (owner) {
          const int x = key_loc(W);
          int mask = p_mask;
          const bool virt = x == p_b;
          NodeV bn{};
          const PodDev p_pod = sh.pf_pod;
          if (!virt) {  // Reserve + Bind on the winner's slot (the virtual node holds another)
            bn = load_node(&s_nodes[x]);
            mask = select_gpus(bn, p_pod, rp.gpusel, sel_arg<false>(rp, bn, p_pod, n_lo + x, key_gpu(W)), rp.seed, p_step);
            if (mask >= 0) bind_node(bn, p_pod, mask, +1);
          }
          if (mask < 0) {  // Reserve failed: allocateGpuId returned "" / panicked
            out.status = ST_ERROR;
            out.score = 0;
            hrec.x = -3;
          } else {
            const int tg = (int)p_pod.tag;
            if (virt) {
              if (lane < 2) reinterpret_cast<uint4*>(&s_nodes[x])[lane] = reinterpret_cast<const uint4*>(&s_nodes[ns])[lane];
              else if (lane == 6) s_F0[x] = s_F0[ns];
              else if (lane == 9) s_E0[x] = s_E0[ns];
              else if (lane == 8 && overlapped) {  // this step's scratch: the post-Bind node (the virtual slot's)
                int* c_pr = s_praw + ((p_step + 1) & 1) * (a.S + 1);
                int* c_pi = s_pinf + ((p_step + 1) & 1) * (a.S + 1);
                c_pr[x] = c_pr[ns];
                c_pi[x] = c_pi[ns];
              }
            } else {
              if (lane == 0) store_node(&s_nodes[x], bn);
              else if (lane == 6) s_F0[x] = -1.0;
              else if (lane == 9) s_E0[x] = kEnergyStale;
              *redo = overlapped;
              if (prof && lane == 0 && overlapped) sh.prof[9] += 1ull << 32;
            }
            if (lane == 2 && tg >= 0) tag_add(g_tags + (size_t)x * kTagStride, tg, +1);
            else if (lane == 10 && pmon) pm_bump(x);
            else if (lane == 7 && snap) {  // cluster report: the post-Bind record
              store_node(snap + p_step, virt ? load_node(&s_nodes[ns]) : bn);
              rp.prev[p_step] = s_last[x];
              s_last[x] = p_step;
            }
            out.node = n_lo + x;
            out.gpu_mask = mask;
            hrec = make_int2(n_lo + x, mask + 1);
          }
        }
      }
    }
    if (lane == 0) {
      if (hist) hist[p_step] = hrec;
      if (writer) rp.res[p_step] = out;
    }
    return true;
  };

  // Finish the pending step with nothing to overlap (before a delete / at the end).
  auto finish_pending = [&]() {
    if (wv == 0) {
      bool ok = true;
      if constexpr (kPF) {
        bool redo;
        unsigned long long x[kS][7];
        ok = pf_resolve(x, false, false, &redo);
      } else {
        GranV<kS> g{};
        if (Kx > 1) poll_once(g);
        int gc, ge, gl, gh;
        const unsigned long long W = exchange(g, &gc, &ge, &gl, &gh, &ok);
        if (ok) commit(W, gc, ge, gl, gh);
      }
      if (lane == 0) {
        if (!ok) { sh.stop = 1; atomicOr(a.fail, 1); }
        sh.pend_valid = 0;
        sh.pend_b = -1;
      }
    }
    __syncthreads();
  };

  __syncthreads();
  for (int step = 0; step < rp.n_events; ++step) {
    const int eb = step & (kEvBuf - 1);
    if (eb == 0) {
      // refill the LDS event window (every thread passed the previous step's final barrier)
      const int nl = min(kEvBuf, rp.n_events - step) * 2;
      const uint4* src = reinterpret_cast<const uint4*>(rp.ev + step);
      for (int i = tid; i < nl; i += kRBlock) reinterpret_cast<uint4*>(sh.ev)[i] = src[i];
      __syncthreads();
    }
    const PodDev p = uniform_pod(&sh.ev[eb]);
    const int2 pvb = *reinterpret_cast<const int2*>(&sh.pend_valid);
    const bool pend = __builtin_amdgcn_readfirstlane(pvb.x) != 0;
    // Dead-class skip (create-only streams): Filter is monotone in the resources a creation takes, so an
    // event whose class found no feasible node before finds none now -- unscheduled, 0 feasible, nothing
    // changes.  The pending step is finished first (its commit may add to the dead set); every workgroup
    // marks the same classes at the same commit, so all skip the same steps.
    if (a.skip && ((sh.dead[p.pad >> 5] >> (p.pad & 31)) & 1u)) {
      if (pend) finish_pending();
      if (sh.stop) break;
      if (tid == 0 && w == 0) rp.res[step] = ResultDev{-1, 0, 0, 0, ST_UNSCHED};
      __syncthreads();
      continue;
    }
    if (kGeneral && (p.flags & kPodDelete)) {  // lean: launched on create-only streams
      if (pend) finish_pending();
      if (sh.stop) break;
      // removePod on the owner of the creation (every workgroup recorded its view of it)
      if (tid == 0) {
        const int2 h = (p.ref >= 0 && p.ref < step) ? hist[p.ref] : make_int2(-1, 0);
        if (h.x >= 0) {
          PodDev cp = rp.ev[p.ref];
          const int loc = h.x - n_lo;
          if (!kTags && cp.tag >= 0) {  // the HBM counts: an atomic, not a read-modify-write
            tag_add(g_tags + (size_t)loc * kTagStride, cp.tag, -1);
            cp.tag = -1;
          }
          apply_bind(&s_nodes[loc], kTags ? &s_tags[(size_t)loc * kTagStride] : nullptr, cp, h.y - 1, -1);
          if (kFgd) s_F0[loc] = -1.0;
          if (kPwr || kPF) s_E0[loc] = kEnergyStale;
          if (pmon) pm_bump(loc);
          if (snap) {
            store_node(snap + step, load_node(&s_nodes[loc]));
            rp.prev[step] = s_last[loc];
            s_last[loc] = step;
          }
          rp.res[step] = ResultDev{h.x, h.y - 1, 0, 0, ST_DELETED};
        } else if ((h.x == -1 && w == 0) || h.x == -3) {
          rp.res[step] = ResultDev{-1, 0, 0, 0, ST_DELETED};
        }
        if (hist) hist[step] = make_int2(-1, 0);
      }
      __syncthreads();
      mark(0);
      continue;
    }
    mark(0);
    // ---- Filter + Score of the slice, the pending best node b excluded, plus the virtual node
    const bool share = is_share_pod(p);
    const int vb = pend ? __builtin_amdgcn_readfirstlane(pvb.y) : -1;
    const int nsv = ns + (vb >= 0 ? 1 : 0);
    // PWR+FGD: this step's per-slot scratch (by step parity: the pending step's stays intact for a miss round)
    int* const c_praw = s_praw + (step & 1) * (a.S + 1);
    int* const c_pinf = s_pinf + (step & 1) * (a.S + 1);
    unsigned long long px[kS][7];  // PWR+FGD: wave 0's early poll of the pending round
    // early poll of the pending exchange by wave 0 (consumed after the evaluation)
    GranV<kS> pg{};
    // one node's packed key into the workgroup aggregate (LDS atomics), or the excluded pair
    auto route = [&](bool leader, int i, bool feas, bool e1, int raw, unsigned long long k) {
      const bool excl = leader && (i == vb || i == ns);
      if (excl) {
        // the pending best node as it is / as it would be after the pending Bind
        if (i == ns) { sh.post_key = k; sh.post_feas = feas ? 1 : 0; sh.post_err = (feas && e1) ? 1 : 0; }
        else { sh.pre_key = k; sh.pre_feas = feas ? 1 : 0; sh.pre_err = (feas && e1) ? 1 : 0; }
      }
      const bool agg = leader && feas && !excl;
      const unsigned long long am = __ballot(agg);
      if (am) {
        if (agg) {
          atomicMax(&sh.agg_key, k);
          if (kMinMax) { atomicMin(&sh.agg_lo, raw); atomicMax(&sh.agg_hi, raw); }
        }
        if (lane == 0) atomicAdd(&sh.agg_cnt, (int)__popcll(am));
        if (kErr) {
          if (__any(agg && e1) && lane == 0) atomicOr(&sh.agg_err, 1);
        }
      }
    };
    if constexpr (kFgd) {
      for (int c0 = 0; c0 < nsv; c0 += kFChunk) {
        const int cn = min(kFChunk, nsv - c0);
        const int i = c0 + (tid >> 3), g = tid & 7;
        const bool valid = (tid >> 3) < cn;
        NodeV n{};
        bool feas = false;
        // PWR+FGD memo: a real slot unchanged since this class last came reuses its entry
        bool hit = false;
        uint2 me = make_uint2(0u, 0u);
        if (pmon && valid && i < ns) {
          me = s_pm[(size_t)p.pad * a.S + i];
          hit = pf_memo_hit(me, s_pver[i]);
        }
        if (valid && !hit) {
          n = load_node(&s_nodes[i]);
          feas = filter_node(n, p);
        }
        // lane g's candidate: share pod -> GPU g if it fits and no lower GPU has the same milli
        // left (equal values give the same GPU multiset, hence the same F); else the Sub state
        bool cand = false;
        if (feas) {
          if (share) {
            const int v = gl_dyn(n, g);
            cand = g < n.gpu_cnt() && v >= p.milli && (gl_equal_mask(n, v) & ((1u << g) - 1u)) == 0u;
          } else {
            cand = g == 0;
          }
        }
        const bool cur = feas && g == 0 && s_F0[i] < 0.0;  // cached F of the current state stale
        const unsigned long long cm = __ballot(cand), um = __ballot(cur);
        const int nw = __popcll(cm) + __popcll(um);
        int base = 0;
        if (nw > 0) {
          if (lane == 0) base = atomicAdd(&sh.nitems, nw);
          base = __builtin_amdgcn_readfirstlane(base);
        }
        int my_item = -1;
        if (cand) {
          my_item = base + lanes_below(cm);
          fs.item_node[my_item] = (uint16_t)i;
          fs.item_code[my_item] = (uint8_t)(share ? 1 + g : 9);
        }
        if (cur) {
          const int o = base + __popcll(cm) + lanes_below(um);
          fs.item_node[o] = (uint16_t)i;
          fs.item_code[o] = 0;
        }
        __syncthreads();
        mark(1);
        const int tot = sh.nitems;
        const int q = tid & 3;
        for (int j = tid >> 2; j < tot; j += kRBlock / 4) {  // one quad per item
          const int loc = fs.item_node[j], code = fs.item_code[j];
          const NodeV m = load_node(&s_nodes[loc]);
          int cpuL, total;
          uint32_t gs[4];
          fgd_candidate(m, code, p, &cpuL, gs, &total);
          const uint32_t tb = 1u << m.gpu_type();
          const double F = rp.typed ? frag_F_quad<true>(cpuL, gs, total, tb, tp, fs.tp, rp.ncpu, rp.nt, q)
                                    : frag_F_quad<false>(cpuL, gs, total, tb, tp, fs.tp, rp.ncpu, rp.nt, q);
          if (q == 0) {
            if (code == 0) s_F0[loc] = F;
            else fs.F[j] = F;
          }
        }
        __syncthreads();
        mark(2);
        if (!kPF && pend && Kx > 1 && wv == 0 && c0 == 0) poll_once(pg);
        if (tid == 0) sh.nitems = 0;  // every thread has read tot; the next writer is past a barrier
        // fgd_score.go:100-141: every candidate lane scores itself; the node keeps the max,
        // ties to the lowest GPU index (fgd_score.go:128 keeps the first max)
        int v = -1;
        if (cand) v = fgd_frag_score(s_F0[i], fs.F[my_item]) * 16 + (15 - g);
        v = group8_max(v);
        // PWR + FGD: the node's raw PWR score and GPU choice by the same 8 lanes
        int pv = -1;
        bool perr = false;
        if constexpr (kPF) {
          bool ovf = false;
          if (feas) {
            const int2 pe = s_pe[i == ns ? vb : i];
            double e0 = s_E0[i];
            if (e0 == kEnergyStale) {
              e0 = node_energy_now(n, pe, sh.pw);
              if (g == 0) s_E0[i] = e0;
            }
            pv = pwr_cand8(n, p, pe, e0, sh.pw, g, &perr, &ovf);
          }
          if (ovf) atomicOr(a.fail, 2);
          pv = group8_max(pv);
        }
        // a feasible node with no candidate (share pod with milli 0 on a GPU-less node) scores 0
        const int raw = v < 0 ? 0 : v >> 4;
        const int gpu = (share && v >= 0) ? 15 - (v & 15) : -1;
        if constexpr (kPF) {
          // the node's raw PWR score and GPU choice (pwr_score.go:48-91) beside its FGD score
          int pgpu = -1;
          int praw = pwr8_finish(pv, &pgpu);
          int pinf = feas ? (kPfFeas | (perr ? kPfErr : 0) | (raw & 0xff) | ((pgpu + 1) & 0xf) << 8 |
                             ((gpu + 1) & 0xf) << 12)
                          : 0;
          if (hit) {
            praw = (int)me.x;
            pinf = pf_memo_pinf(me);
            feas = (pinf & kPfFeas) != 0;
            perr = (pinf & kPfErr) != 0;
          }
          if (valid && g == 0) {
            c_praw[i] = praw;
            c_pinf[i] = pinf;
            if (pmon && !hit && i < ns) s_pm[(size_t)p.pad * a.S + i] = pf_memo_pack(praw, pinf, s_pver[i]);
          }
        } else {
          const unsigned long long k = feas ? pack_key((unsigned)raw, n.name_rank, gpu, i == ns ? vb : i) : 0ull;
          route(valid && g == 0, i, feas, false, raw, k);
        }
        if (c0 + kFChunk < nsv) __syncthreads();  // F / items are reused by the next chunk
        mark(3);
      }
    } else if constexpr (kPwr) {
      // PWR: eight lanes per node (lane g <-> GPU g), the raw score biased into the key field
      if (pend && Kx > 1 && wv == 0) poll_once(pg);
      for (int c0 = 0; c0 < nsv; c0 += kFChunk) {
        const int cn = min(kFChunk, nsv - c0);
        const int i = c0 + (tid >> 3), g = tid & 7;
        const bool valid = (tid >> 3) < cn;
        NodeV n{};
        bool feas = false, perr = false, ovf = false;
        int pv = -1;
        if (valid) {
          n = load_node(&s_nodes[i]);
          feas = filter_node(n, p);
          if (feas) {
            const int2 pe = s_pe[i == ns ? vb : i];
            double e0 = s_E0[i];
            if (e0 == kEnergyStale) {
              e0 = node_energy_now(n, pe, sh.pw);
              if (g == 0) s_E0[i] = e0;
            }
            pv = pwr_cand8(n, p, pe, e0, sh.pw, g, &perr, &ovf);
          }
        }
        if (ovf) atomicOr(a.fail, 2);
        pv = group8_max(pv);
        int pgpu = -1;
        const int pr = pwr8_finish(pv, &pgpu);
        const unsigned raw = (unsigned)(pr + kPwrKeyBias);  // |pr| < 2^23 (else the run fails)
        const unsigned long long k =
            feas ? pack_key(raw, n.name_rank, rp.gpusel == SEL_PWR ? pgpu : -1, i == ns ? vb : i) : 0ull;
        route(valid && g == 0, i, feas, perr, (int)raw, k);
      }
    } else {
      if (pend && Kx > 1 && wv == 0) poll_once(pg);
      for (int c0 = 0; c0 < nsv; c0 += kChunk) {
        const int cn = min(kChunk, nsv - c0);
        const int i = c0 + tid;
        bool feas = false, e1 = false;
        int raw = 0;
        NodeV n{};
        if (tid < cn) {
          n = load_node(&s_nodes[i]);
          feas = filter_node(n, p);
          if (feas) {
            const int cap = (kPol == POL_DOTPROD && dp_norm(rp.dpcfg) == NORM_NODE) ? rp.cap[n_lo + (i == ns ? vb : i)] : 0;
            raw = cheap_score<kPol>(n, p, rp.seed, kTags ? &s_tags[(size_t)i * kTagStride] : nullptr, step, &e1,
                                    rp.dpcfg, cap);
          }
        }
        const unsigned long long k = feas ? pack_key((unsigned)raw, n.name_rank, -1, i == ns ? vb : i) : 0ull;
        route(tid < cn, i, feas, e1, raw, k);
      }
    }
    if (kPF && pend && Kx > 1 && wv == 0) {  // the pending round's granules: loads in flight over the barrier
      const unsigned long long* slot = gr + (size_t)(p_seq & 1) * Kx * kGranW;
#pragma unroll
      for (int j = 0; j < kS; ++j)
        if (lane + 64 * j < Kx) {
#pragma unroll
          for (int q = 0; q < 7; ++q) px[j][q] = gload(slot + (size_t)(lane + 64 * j) * kGranW + q);
        }
    }
    __syncthreads();
    mark(4);
    if constexpr (kPF) {
      // 1. the pending step (its round overlapped the evaluation above): decide and commit.  The owner of a winner
      //    other than its virtual node re-evaluates this step: that slot changed under the evaluation.
      if (pend) {
        if (wv == 0) {
          bool redo = false;
          const bool ok = pf_resolve(px, Kx > 1, true, &redo);
          if (lane == 0) {
            sh.pf_redo = redo ? 1 : 0;
            sh.pend_valid = 0;
            sh.pend_b = -1;
            if (!ok) { sh.stop = 1; atomicOr(a.fail, 1); }
          }
        }
        __syncthreads();
        if (sh.stop) break;
        if (sh.pf_redo) {  // the same step again, nothing pending
          --step;
          continue;
        }
      }
      mark(5);
      // 2. the slice's A totals and its best key under each of the class's two guessed ranges
      const int4 gs = s_gtab[p.pad & (kPfGuess - 1)];
      if (wv * 64 < ns) {
        int c = 0, e = 0, lo = INT_MAX, hi = INT_MIN;
        unsigned long long k0 = 0ull, k1 = 0ull;
        for (int i = tid; i < ns; i += kRBlock) {
          const int inf = c_pinf[i];
          if (inf & kPfFeas) {
            const int pr = c_praw[i];
            ++c;
            e |= (inf & kPfErr) ? 1 : 0;
            lo = min(lo, pr);
            hi = max(hi, pr);
            const unsigned long long q0 = pf_key(pr, inf, gs.x, gs.y, i), q1 = pf_key(pr, inf, gs.z, gs.w, i);
            k0 = q0 > k0 ? q0 : k0;
            k1 = q1 > k1 ? q1 : k1;
          }
        }
        c = wave_sum_dpp(c);
        e = __any(e != 0) ? 1 : 0;
        lo = wave_min_dpp(lo);
        hi = wave_max_dpp(hi);
        k0 = wave_max_u64_dpp(k0);
        k1 = wave_max_u64_dpp(k1);
        if (lane == 0 && c > 0) {
          atomicAdd(&sh.agg_cnt, c);
          if (e) atomicOr(&sh.agg_err, 1);
          atomicMin(&sh.agg_lo, lo);
          atomicMax(&sh.agg_hi, hi);
          atomicMax(&sh.agg_key, k0);
          atomicMax(&sh.agg_key1, k1);
        }
      }
      __syncthreads();
      // 3. publish the round, then prepare the virtual node: guess 0's local best with this step's Reserve + Bind
      if (wv == 0) {
        const unsigned long long mk = sh.agg_key, mk1 = sh.agg_key1;
        const int c = sh.agg_cnt, e = sh.agg_err, l = sh.agg_lo, h = sh.agg_hi;
        if (lane == 0) {
          if (Kx > 1) {
            unsigned long long* slot = gr + (size_t)(seq & 1) * Kx * kGranW + (size_t)wx * kGranW;
            const unsigned long long tag = (unsigned long long)(unsigned)(seq + 1) << 32;
            gstore(slot + 0, tag | (mk & 0xffffffffull));
            gstore(slot + 1, tag | (mk >> 32));
            gstore(slot + 2, tag | (mk1 & 0xffffffffull));
            gstore(slot + 3, tag | (mk1 >> 32));
            gstore(slot + 4, tag | (unsigned)l);
            gstore(slot + 5, tag | (unsigned)h);
            gstore(slot + 6, tag | ((unsigned)e << 31) | ((unsigned)c & 0x7fffffffu));
          }
          reset_agg();
        }
        const int mloc = key_loc(mk);
        int mask = -1;
        if (mk != 0ull) {
          NodeV bn = load_node(&s_nodes[mloc]);
          mask = select_gpus(bn, p, rp.gpusel, sel_arg<kPol == POL_DOTPROD>(rp, bn, p, n_lo + mloc, key_gpu(mk)), rp.seed,
                             step);
          if (mask >= 0) bind_node(bn, p, mask, +1);
          if (lane == 0) store_node(&s_nodes[ns], bn);
          else if (kTags && lane >= 2 && lane < 6) {
            uint2 t = reinterpret_cast<const uint2*>(&s_tags[(size_t)mloc * kTagStride])[lane - 2];
            if (mask >= 0 && p.tag >= 0 && (p.tag >> 2) == lane - 2) {
              const uint32_t inc = 1u << (16 * (p.tag & 1));
              t.x += (p.tag & 2) ? 0u : inc;
              t.y += (p.tag & 2) ? inc : 0u;
            }
            reinterpret_cast<uint2*>(&s_tags[(size_t)ns * kTagStride])[lane - 2] = t;
          } else if (lane == 6) {
            s_F0[ns] = mask >= 0 ? -1.0 : s_F0[mloc];
          } else if (lane == 7) {
            s_E0[ns] = mask >= 0 ? kEnergyStale : s_E0[mloc];
          }
        }
        p_step = step;
        p_cls = p.pad;
        p_seq = seq;
        p_b = mk != 0ull ? mloc : -1;
        p_key = mk;
        if (lane == 0) {
          sh.pf_key1 = mk1;
          sh.pf_g = gs;
          sh.pf_pod = p;
        }
        p_st0 = c; p_st1 = e; p_st2 = l; p_st3 = h;
        p_mask = mask;
        p_tag = mask >= 0 ? (int)p.tag : -1;
        ++seq;
        if (lane == 0) { sh.pend_valid = 1; sh.pend_b = p_b; }
      }
    } else if (wv == 0) {
      // the slice's aggregate without b (LDS atomics above), then b's two versions
      unsigned long long mk = sh.agg_key;
      int c = sh.agg_cnt, e = sh.agg_err, l = sh.agg_lo, h = sh.agg_hi;
      const unsigned long long k_pre = sh.pre_key, k_post = sh.post_key;
      const int f_pre = sh.pre_feas, f_post = sh.post_feas, e_pre = sh.pre_err, e_post = sh.post_err;
      // finish the pending exchange (its latency overlapped the evaluation above)
      bool owner = false, ok = true;
      unsigned long long W = 0ull;
      int gc = 0, ge = 0, gl = 0, gh = 0;
      if (pend) {
        W = exchange(pg, &gc, &ge, &gl, &gh, &ok);
        // b's post-Bind version only if the pending step binds: a Score error (framework.go:650-656,
        // e.g. BestFit's -1 on a node with less CPU left than the non-zero request) aborts the cycle
        owner = W != 0ull && W == p_key && !(gc > 1 && ge);
      }
      mark(5);
      // add b back: post-Bind if this workgroup owned the pending winner, else as it was
      if (vb >= 0 && (owner ? f_post : f_pre)) {
        const unsigned long long vk = owner ? k_post : k_pre;
        mk = vk > mk ? vk : mk;
        ++c;
        e |= owner ? e_post : e_pre;
        if (kMinMax) { l = min(l, key_score(vk)); h = max(h, key_score(vk)); }
      }
      if (ok) {
        if (lane == 0) {
          // publish this step first: granules {tag, key lo32}, {tag, key hi32}, {tag, err|hi|lo|cnt}
          if (Kx > 1) {
            unsigned long long* slot = gr + (size_t)(seq & 1) * Kx * kGranW;
            const unsigned long long tag = (unsigned long long)(unsigned)(seq + 1) << 32;
            // bit 17 (BestFit): the slice's feasible raw scores are not all equal (its max is mk's score)
            const unsigned stat = ((unsigned)e << 31) | (l < h ? 1u << 17 : 0u) | ((unsigned)c & 0x1ffff);
            gstore(slot + (size_t)wx * kGranW + 0, tag | (mk & 0xffffffffull));
            gstore(slot + (size_t)wx * kGranW + 1, tag | (mk >> 32));
            gstore(slot + (size_t)wx * kGranW + 2, tag | stat);
          }
          reset_agg();
        }
        if (pend) commit(W, gc, ge, gl, gh);
        // prepare the virtual node: this step's best node with this step's Reserve + Bind applied
        const int mloc = key_loc(mk);
        int mask = -1;
        if (mk != 0ull) {
          NodeV bn = load_node(&s_nodes[mloc]);
          mask = select_gpus(bn, p, rp.gpusel, sel_arg<kPol == POL_DOTPROD>(rp, bn, p, n_lo + mloc, key_gpu(mk)), rp.seed,
                             step);
          if (mask >= 0) bind_node(bn, p, mask, +1);
          if (lane == 0) store_node(&s_nodes[ns], bn);
          else if (kTags && lane >= 2 && lane < 6) {
            uint2 t = reinterpret_cast<const uint2*>(&s_tags[(size_t)mloc * kTagStride])[lane - 2];
            if (mask >= 0 && p.tag >= 0 && (p.tag >> 2) == lane - 2) {
              // +1 on u16 tag p.tag (counts stay far below 2^16, no carry across halves)
              const uint32_t inc = 1u << (16 * (p.tag & 1));
              t.x += (p.tag & 2) ? 0u : inc;
              t.y += (p.tag & 2) ? inc : 0u;
            }
            reinterpret_cast<uint2*>(&s_tags[(size_t)ns * kTagStride])[lane - 2] = t;
          } else if (lane == 6 && kFgd) {
            s_F0[ns] = mask >= 0 ? -1.0 : s_F0[mloc];
          } else if (lane == 7 && kPwr) {
            s_E0[ns] = mask >= 0 ? kEnergyStale : s_E0[mloc];
          }
        }
        p_step = step;
        p_cls = p.pad;
        p_seq = seq;
        p_b = mk != 0ull ? mloc : -1;
        p_key = mk;
        p_mask = mask;
        p_tag = mask >= 0 ? (int)p.tag : -1;
        p_st0 = c; p_st1 = e; p_st2 = l; p_st3 = h;
        ++seq;
        if (lane == 0) { sh.pend_valid = 1; sh.pend_b = p_b; }
      } else if (lane == 0) {
        sh.stop = 1;
        atomicOr(a.fail, 1);
      }
    }
    mark(6);
    __syncthreads();
    mark(7);
    if (sh.stop) break;
  }
  if (!sh.stop && __builtin_amdgcn_readfirstlane(sh.pend_valid)) finish_pending();
  if (prof && tid == 0) {
    sh.prof[10] = __builtin_amdgcn_s_memtime() - c_start;
    sh.prof[11] = __builtin_amdgcn_s_memrealtime() - t_start;
  }
  __syncthreads();
  if (prof && tid < kProfPhases) a.prof[(size_t)blockIdx.x * kProfPhases + tid] = sh.prof[tid];
  // write the slice back (final cluster state)
  for (int i = tid; i < ns; i += kRBlock) store_node(rp.nodes + n_lo + i, load_node(&s_nodes[i]));
  if (kTags)
    for (int i = tid; i < ns * kTagStride; i += kRBlock) rp.tags[(size_t)n_lo * kTagStride + i] = s_tags[i];
}

__global__ void k_advance(int* base, int k) { *base += k; }

// Reserve on an explicit node (ksim_engine_reserve): candidate F values for the
// FGD selector are evaluated by one workgroup, then thread 0 binds.
__global__ __launch_bounds__(64) void k_reserve(ReplicaDev* reps, const TypDev* __restrict__ tp_all, int r, PodDev p,
                                                int node, int step, int* out_mask, int sign, int mask_in) {
  const ReplicaDev rp = reps[r];
  const TypDev* __restrict__ tp = tp_all + (size_t)r * kMaxTypical;
  __shared__ double s_F[kMaxCand];
  const int tid = (int)threadIdx.x;
  NodeRec* nr = rp.nodes + node;
  uint16_t* tg = rp.tags + (size_t)node * kTagStride;
  if (sign < 0) {
    // removePod (cache.go:100-111, deviceinfo.go:39-60): every released device gets its milli back
    // without exceeding the device (left + milli <= 1000, the invariant of the packed u16 lanes), and
    // the CPU and memory stay within the node's allocatable; else nothing changes (e.g. a second
    // Unreserve of the same pod on a node still hosting another one)
    if (tid == 0) {
      const NodeV n = load_node(nr);
      bool ok = n.pods_left() < 32767 && (long long)n.cpu_left + p.cpu_req <= (long long)rp.cap[node] &&
                (long long)n.mem_left + p.mem <= (long long)rp.mcap[node];
      for (int g = 0; g < kMaxGpu; ++g)
        if ((mask_in >> g) & 1) ok = ok && g < n.gpu_cnt() && n.gl(g) + (int)p.milli <= kMilli;
      if (ok) apply_bind(nr, tg, p, mask_in, -1);
      *out_mask = ok ? mask_in : -1;
    }
    return;
  }
  if (mask_in >= 0) {
    // a predefined gpu-index (open_gpu_share.go:260-271): every named device must hold the milli
    if (tid == 0) {
      const NodeV n = load_node(nr);
      bool ok = true;
      for (int g = 0; g < kMaxGpu; ++g)
        if ((mask_in >> g) & 1) ok = ok && g < n.gpu_cnt() && n.gl(g) >= (int)p.milli;
      if (ok) apply_bind(nr, tg, p, mask_in, +1);
      *out_mask = ok ? mask_in : -1;
    }
    return;
  }
  const NodeV n = load_node(nr);
  const bool need_fgd = rp.gpusel == SEL_FGD && is_share_pod(p) && p.milli > 0;
  if (need_fgd) {
    if (tid < kMaxCand) {
      int gl[kMaxGpu];
      unpack_gl(n, gl);
      int cpuL = n.cpu_left;
      bool valid = true;
      if (tid > 0) {
        cpuL -= p.cpu_nz;
#pragma unroll
        for (int g = 0; g < kMaxGpu; ++g) {
          if (g == tid - 1) {
            valid = g < n.gpu_cnt() && gl[g] >= p.milli;
            gl[g] -= valid ? (int)p.milli : 0;
          }
        }
      }
      double F = 0.0;
      if (valid)
        F = rp.typed ? frag_F<true>(cpuL, gl, 1u << n.gpu_type(), tp, rp.ncpu, rp.nt)
                     : frag_F<false>(cpuL, gl, 1u << n.gpu_type(), tp, rp.ncpu, rp.nt);
      s_F[tid] = F;
    }
    __syncthreads();
  }
  if (tid != 0) return;
  int fgd_gpu = -1;
  if (need_fgd) {
    int bs = 0;
#pragma unroll
    for (int g = 0; g < kMaxGpu; ++g) {
      if (g < n.gpu_cnt() && n.gl(g) >= p.milli) {
        const int fs = fgd_frag_score(s_F[0], s_F[1 + g]);
        if (fgd_gpu < 0 || fs > bs) { bs = fs; fgd_gpu = g; }
      }
    }
  }
  if (rp.gpusel == SEL_PWR && is_share_pod(p) && p.milli > 0) {  // allocateGpuIdBasedOnPWRScore
    bool perr = false;
    (void)pwr_score(n, p, rp.cap[node], rp.cpum[node], *rp.pw, &fgd_gpu, &perr);
    if (perr) fgd_gpu = -1;
  }
  const int mask = select_gpus(n, p, rp.gpusel, sel_arg(rp, n, p, node, fgd_gpu), rp.seed, step);
  *out_mask = mask;
  if (mask >= 0) apply_bind(nr, tg, p, mask, +1);
}

#define KSIM_HIP(x)                                \
  do {                                             \
    hipError_t _e = (x);                           \
    if (_e != hipSuccess) {                        \
      std::fprintf(stderr, "ksim: %s failed: %s\n", #x, hipGetErrorString(_e)); \
      return KSIM_EHIP;                            \
    }                                              \
  } while (0)

}  // namespace

// ---------------------------------------------------------------------------
// Host engine object
// ---------------------------------------------------------------------------
struct ksim_engine {
  int device = 0;
  int N = 0, R = 0, NB = 64, bpr = 0, K = 256;
  int run_mode = 0;        // 0: auto (k_memo for FGD when it fits, else k_replay), 1: k_step per pod (hipGraph),
                           // 2: k_replay only, 3: k_memo required for FGD
  int wgs_req = 0;         // requested workgroups per replica (0 = auto)
  int cus = 256;
  bool coop = true;  // K > 1 persistent grids through hipLaunchCooperativeKernel (KSIM_COOP=0: plain launch)
  unsigned long long* d_gran = nullptr;
  int2* d_hist = nullptr;
  size_t hist_cap = 0;
  int* d_fail = nullptr;
  int* d_replist = nullptr;              // replicas ordered by policy (k_replay groups)
  int last_groups = 0;
  unsigned long long* d_prof = nullptr;  // KSIM_PROFILE=1: k_replay phase timers
  size_t prof_cap = 0;
  int last_K = 0;
  hipStream_t stream = nullptr;
  NodeRec* d_nodes = nullptr;
  NodeRec* d_nodes_init = nullptr;  // cluster state given to set_nodes (run() restarts from it)
  uint16_t* d_tags = nullptr;  // per replica: N*16 u16 tags, then N int rank->index
  uint16_t* d_tags_init = nullptr;
  size_t tags_stride = 0;      // u16 elements per replica
  TypDev* d_tp = nullptr;
  Accum* d_acc = nullptr;
  ReplicaDev* d_reps = nullptr;
  int* d_base = nullptr;
  int* d_scratch = nullptr;     // single-pod calls: [0] mask
  PodDev* d_pod = nullptr;      // single-pod calls
  ResultDev* d_res1 = nullptr;  // single-pod calls
  uint8_t* d_feas = nullptr;
  int32_t* d_score = nullptr;
  int32_t* d_gpu = nullptr;
  std::vector<ReplicaDev> reps;
  std::vector<std::vector<ksim_node>> h_nodes;  // caller's static node fields per replica
  std::vector<PodDev*> d_ev;
  std::vector<ResultDev*> d_res;
  std::vector<int> n_events;
  std::vector<char> has_delete;  // the replica's stream has deletion events (k_replay keeps a bind history)
  // k_memo (memoised FGD replay): per replica the distinct pod requests of its creation events
  // (PodDev.pad = class id) and how many events each has
  std::vector<std::vector<PodDev>> h_cls;
  std::vector<std::vector<TypDev>> h_tp;  // each replica's typical table as uploaded (k_hmemo's per-model tables)
  std::vector<std::vector<int>> h_cls_n;
  std::vector<std::vector<int>> h_ev_cls;  // class of each event, -1 delete
  PodDev* d_m_pod = nullptr;
  int* d_m_owner = nullptr;
  int* d_m_wgcls = nullptr;
  int* d_m_wgref = nullptr;
  unsigned long long* d_m_wggrp = nullptr;
  unsigned* d_win = nullptr;
  int* d_m_evo = nullptr;
  int* d_m_evcls = nullptr;     // decider mode: class of each event
  unsigned* d_topg = nullptr;   // decider mode: top granules
  unsigned* d_m_hkeys = nullptr;  // k_memo with the keys in HBM (MemoPlan::hkeys)
  int* d_m_wgmap = nullptr;       // k_memo: each block's launch position << 8 | workgroup (MemoArgs::wg_map)
  unsigned long long* d_done = nullptr;  // [2 + R] the overlapped report's queue (ksim_scan1.hpp Scan1Args::done)
  __int128* d_ragg = nullptr;     // [R][kScanPartsMax][2][kFields] the multi-workgroup report scan's part sums
  size_t ragg_cap = 0;
  int done_cap = 0;
  unsigned done_epoch = 0;
  hipEvent_t ev_ovl = nullptr;    // the queue's tickets zeroed (the report's stream waits on it)
  size_t m_cap2[4] = {0, 0, 0, 0};
  double* d_th = nullptr;       // FGD score steps (build_score_thresholds), null if unusable
  size_t m_cap[7] = {0, 0, 0, 0, 0, 0, 0};
  struct MemoPlan* mplan = nullptr;  // the FGD replicas' k_memo plan, uploaded before the timed run
  bool mplan_dirty = true;           // events or policies changed since the plan was made
  bool mplan_ok = false;
  std::vector<int> mplan_all;   // the FGD replicas the plans were made for (cache key)
  std::vector<int> mplan_reps;  // the replicas of the k_memo plan
  std::vector<int> hplan_reps;  // the replicas of the k_hmemo plan
  std::vector<int> wgs_hint;    // per replica: workgroups asked by ksim_engine_set_replica_wgs (0: the engine's choice)
  bool split_fgd = false;       // the wide-hinted FGD replicas on k_memo beside the others on k_hmemo (one run)
  int mplan_max_ev = -1;
  int last_memo = 0;
  // k_hmemo (memoised FGD replay, keys in HBM): the plan and its device tables
  struct HPlan* hplan = nullptr;
  bool hplan_ok = false;
  int* d_h_cg = nullptr;
  PodDev* d_h_cls = nullptr;
  uint16_t* d_h_cgrp = nullptr;
  PodDev* d_h_gpod = nullptr;
  int* d_h_mtoff = nullptr;      // k_hmemo's per-model tables (typed replicas)
  uint8_t* d_h_mtab = nullptr;
  double* d_h_na = nullptr;      // their NA bins per (model, total), k_hinit_na
  int* d_h_evc = nullptr;
  NodeRec* d_h_st = nullptr;
  int* d_h_ns = nullptr;
  int* d_h_nstate = nullptr;
  unsigned* d_h_gsc = nullptr;
  unsigned* d_h_keys = nullptr;
  unsigned* d_h_l1 = nullptr;
  unsigned* d_h_l2 = nullptr;  // k_hmemo: initial second maxima (HPlan::l2)
  int* d_h_cnt = nullptr;
  unsigned long long* d_h_prof = nullptr;
  uint8_t* d_h_hist = nullptr;  // wide k_hmemo with deletes: per-workgroup bind history
  size_t h_cap[18] = {};
  int last_hmemo = 0;
  int last_rgo = 0;  // replicas the last run replayed on k_random_go
  int last_scan1 = 0;  // replicas the last run replayed on k_scan1
  int last_launches = 0, last_streams = 0;  // replay launches of the last run, side streams they ran on (0: none)
  std::vector<hipEvent_t> grp_rev;  // concurrent groups' report kernels: a timing event pair per group
  int grp_rev_used = 0;             // pairs recorded by the last run
  int scan1 = 2;       // single-workgroup cheap-policy groups on k_scan1, node records in VGPRs where they fit
                       // (KSIM_VARIANT scan1=1: records in LDS; 0: k_replay)
  std::vector<std::vector<NodeRec>> h_rec;  // the records set_nodes gave each replica (k_hmemo's initial states)
  bool last_step_path = false;  // the last run went through k_step (run_mode 1 or a PWR replica)
  std::vector<int> nt;
  hipGraphExec_t graph = nullptr;
  int graph_R = -1;
  bool graph_pwr = false;    // the graph carries k_step_pwr after every k_step
  PowerDev* d_pw = nullptr;  // [R] PWR energy model
  uint8_t* d_cpum = nullptr; // [R][N] CPU model id per node
  int2* d_pws = nullptr;     // [R][N] PWR phase-A scratch
  std::vector<char> pw_set;  // set_power_model called
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_mid = nullptr;
  // side streams for concurrent single-workgroup k_replay groups (created on first use)
  static constexpr int kSide = 6;
  hipStream_t side[kSide] = {};
  int* h_started = nullptr;   // residency gate: host-mapped flags, one per FGD workgroup (hipHostMalloc)
  int* d_started = nullptr;   // its device address
  int started_cap = 0, gate_epoch = 0;
  int last_ovl = 0;           // replicas the last run's overlapped report took (k_report_overlap)
  int last_gate = 0;          // the last run's residency gate: 0 none, 1 opened, -1 given up at its bound (stderr note)
  long long gate_timeouts = 0;  // gates given up at their bound, over the engine's life
  std::string last_kernels;    // the replay kernels the last run launched, '+'-joined in launch order
  hipEvent_t side_ev[kSide] = {};
  hipEvent_t ev_fork = nullptr;
  bool report_done = false;
  // KSIM_GROUP_TIMES=1: timing events at the fork and at each used side stream's end (the last run's
  // concurrent groups, printed on stderr after the run)
  hipEvent_t tev_fork = nullptr;
  hipEvent_t tev_side[kSide] = {};
  unsigned tev_used = 0u;
  int last_pf_memo = 0;      // PWR+FGD memo class stride of the last k_replay<PWR+FGD> launch (0: none)
  double last_ms = 0, last_report_ms = 0;
  // cluster report (ksim_engine_set_report)
  bool report = false;
  int32_t* d_cap = nullptr;   // [R][N] allocatable milli-CPU
  int32_t* d_mcap = nullptr;  // [R][N] allocatable memory, MiB (Unreserve's removePod guard)
  int32_t* d_last = nullptr;  // [R][N] k_step: last event that changed each node
  std::vector<NodeRec*> d_snap;
  std::vector<int32_t*> d_prev;
  std::vector<RepAcc*> d_rep;
  std::vector<int64_t> total_gpus;
  // node-sharded cluster (ksim_engine_set_shard)
  int shard_world = 0;        // 0: not sharded
  unsigned long long* d_ggran = nullptr;  // a node-sharded group's exchange granules (engine 0 of the group)
  void* d_hgargs = nullptr;               // its per-shard k_hmemo arguments
  unsigned long long* d_rgran = nullptr;  // a node-sharded k_replay group's exchange granules (engine 0)
  ReplicaDev* d_rgreps = nullptr;         // its shards' replicas, and their list
  int* d_rglist = nullptr;
  // one shard per process (ksim_shard_peer_handle / ksim_engine_set_shard_peers): this shard's exchange
  // buffer (uncached device memory, exported by IPC), the peers' buffers mapped here, the run epoch
  unsigned long long* d_pgran = nullptr;
  std::vector<uint8_t> pgran_handle;      // the handle ksim_shard_peer_handle returned (exports differ per call)
  std::vector<unsigned long long*> peers;
  std::vector<char> peer_opened;
  int peer_epoch = 0;
  int shard_rank = 0, node_off = 0, n_global = 0;
  ncclComm_t comm = nullptr;  // null: in-process shard group (ksim_shard_group_run) or world 1
  unsigned long long* d_send = nullptr;  // this shard's record {best, nfeas, err, lo|hi}
  unsigned long long* d_recv = nullptr;  // [world][4] gathered records
  unsigned long long** d_ptrs = nullptr; // group mode: send / recv pointer tables
  ksim_shard_exchange_fn xfn = nullptr;  // host exchange (ksim_engine_set_shard_exchange)
  void* xuser = nullptr;
  std::vector<uint64_t> h_send, h_recv;  // its staging records
  // the Random draw structure on Go's math/rand stream (ksim_engine_set_go_stream): per replica the
  // source state {vec[607], tap, feed}, empty = the hash contract
  std::vector<std::vector<unsigned long long>> go_state;
  unsigned long long* d_go = nullptr;
  size_t go_cap = 0;
  int64_t last_steps = 0;
};

// Environment knobs.  Besides the five plain ones (KSIM_PROFILE, KSIM_COOP, KSIM_CUS,
// KSIM_SIDE_STREAMS, KSIM_GROUP_TIMES), two comma-separated key=value lists: KSIM_VARIANT selects the measured
// alternative forms of the kernels and plans (A/B runs; the defaults are what the bench and the tests measure),
// KSIM_TEST the test-only settings (wrap points, stress delays, forced misses).
static long knob(const char* var, const char* key, long dflt) {
  const char* v = std::getenv(var);
  if (!v) return dflt;
  const size_t kl = std::strlen(key);
  for (const char* p = v; *p;) {
    const char* q = std::strchr(p, ',');
    const size_t len = q ? (size_t)(q - p) : std::strlen(p);
    if (len > kl && std::strncmp(p, key, kl) == 0 && p[kl] == '=') return std::strtol(p + kl + 1, nullptr, 0);
    if (!q) break;
    p = q + 1;
  }
  return dflt;
}
static long variant(const char* key, long dflt) { return knob("KSIM_VARIANT", key, dflt); }
static long test_knob(const char* key, long dflt) { return knob("KSIM_TEST", key, dflt); }

static int check_gfx950(int dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= dev) return KSIM_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return KSIM_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KSIM_ENODEV;
  return KSIM_OK;
}

static int alloc_report(ksim_engine* e, int r);
static void destroy_comm(ncclComm_t c);

static int upload_reps(ksim_engine* e) {
  KSIM_HIP(hipMemcpyAsync(e->d_reps, e->reps.data(), sizeof(ReplicaDev) * e->R, hipMemcpyHostToDevice, e->stream));
  return KSIM_OK;
}

// Workgroups of kernel `f` (1024 threads, `lds` B of dynamic LDS) that can be resident at once on the
// CUs the engine may use: the occupancy query times the CU count.  A persistent grid whose workgroups
// exchange granules (K > 1) must not exceed it.
static int resident_cap(const ksim_engine* e, const void* f, size_t lds);
static int run_hmemo_peer(ksim_engine* e, int max_ev);

// A persistent launch: K > 1 workgroups per replica poll each other's granules every step, so the
// whole grid must be resident -- a cooperative launch, which the runtime refuses up front
// (hipErrorCooperativeLaunchTooLarge) instead of letting a non-resident workgroup stall the pollers.
// K = 1 needs no co-residency: a plain launch (it may share the device with side-stream groups).
template <typename A>
static int launch_persistent(const void* f, int grid, int block, size_t lds, hipStream_t st, bool coop, A& args,
                             const TypDev*& tp) {
  KSIM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* params[] = {(void*)&args, (void*)&tp};
  const hipError_t r = coop ? hipLaunchCooperativeKernel(f, dim3(grid), dim3(block), params, (unsigned)lds, st)
                            : hipLaunchKernel(f, dim3(grid), dim3(block), params, lds, st);
  if (r == hipErrorCooperativeLaunchTooLarge) {
    std::fprintf(stderr, "ksim: %d co-resident workgroups of %zu B LDS do not fit the device\n", grid, lds);
    (void)hipGetLastError();
    return KSIM_ERANGE;
  }
  KSIM_HIP(r);
  return KSIM_OK;
}

// k_scan1 for the policies it serves, else null (reg: the node records in VGPRs)
template <bool R, bool G>
static const void* scan1_fn(int pol) {
  switch (pol) {
    case POL_BESTFIT: return (const void*)ksim_scan1::k_scan1<POL_BESTFIT, R, G>;
    case POL_DOTPROD: return (const void*)ksim_scan1::k_scan1<POL_DOTPROD, R, G>;
    case POL_PACKING: return (const void*)ksim_scan1::k_scan1<POL_PACKING, R, G>;
    case POL_CLUSTERING: return (const void*)ksim_scan1::k_scan1<POL_CLUSTERING, R, G>;
    case POL_RANDOM: return (const void*)ksim_scan1::k_scan1<POL_RANDOM, R, G>;
    default: return nullptr;
  }
}
static const void* scan1_fn(int pol, bool report, bool reg) {
  return report ? (reg ? scan1_fn<true, true>(pol) : scan1_fn<true, false>(pol))
                : (reg ? scan1_fn<false, true>(pol) : scan1_fn<false, false>(pol));
}

template <int P, bool G>
static const void* replay_fn(int K) {
  return K == 1 ? (const void*)k_replay<P, 0, G> : K <= 64 ? (const void*)k_replay<P, 1, G> : (const void*)k_replay<P, 4, G>;
}
template <int P>
static const void* replay_fn(int K, bool general) {
  return general ? replay_fn<P, true>(K) : replay_fn<P, false>(K);
}
static const void* replay_kernel(int pol, int K, bool general) {
  switch (pol) {
    case POL_FGD: return replay_fn<POL_FGD>(K, general);
    case POL_BESTFIT: return replay_fn<POL_BESTFIT>(K, general);
    case POL_DOTPROD: return replay_fn<POL_DOTPROD>(K, general);
    case POL_PACKING: return replay_fn<POL_PACKING>(K, general);
    case POL_CLUSTERING: return replay_fn<POL_CLUSTERING>(K, general);
    case POL_PWR: return replay_fn<POL_PWR>(K, general);
    case POL_PWR_FGD: return replay_fn<POL_PWR_FGD>(K, general);
    default: return replay_fn<POL_RANDOM>(K, general);
  }
}

// ---- k_memo planning (memoised FGD replay, ksim_memo.hpp) ----
struct MemoPlan {
  int K = 0, Cw = 0, nfw = 0, Cmax = 1;  // K: the most workgroups of a replica
  int nwg = 0;                            // workgroups of the launch (Σ Kr)
  std::vector<int> Kr, wgoff;             // [Rg] each replica's workgroups (r06: per replica), its first block
  bool decider = false;  // workgroup 0 decides, 1..K-1 own the classes
  bool hkeys = false;    // the keys in HBM (k_memo<..., kHKeys>): classes whose keys do not fit in LDS
  size_t lds = 0;
  std::vector<PodDev> pod;                  // [Rg][Cmax]
  std::vector<int> owner;                   // [Rg][Cmax]
  std::vector<int> wgcls, wgref;            // [nwg][Cw] (block wgoff[i] + w)
  std::vector<unsigned long long> wggrp;    // [nwg][Cw]
};

// Classes of one replica onto K workgroups, at most Cw slots each.  Classes with the same score
// request (cpu_nz, milli, num) stay in one workgroup (their candidate states are the same, so one
// refresh evaluates them once); groups go largest first to the workgroup with the fewest groups.
// split: a group that fits no workgroup whole is spread over the workgroups with the most free slots
// (each part's workgroup evaluates the group's candidate states for its own classes: the same keys,
// the states evaluated once per part) -- the typed gpuspec traces hold groups of up to 60 classes.
static bool memo_assign(const std::vector<PodDev>& cls, int K, int Cw, std::vector<int>& slot_cls, std::vector<int>& owner,
                        bool split = false) {
  std::vector<std::pair<std::vector<int32_t>, std::vector<int>>> groups;
  for (int c = 0; c < (int)cls.size(); ++c) {
    const std::vector<int32_t> k{cls[c].cpu_nz, cls[c].milli, cls[c].num};
    auto it = std::find_if(groups.begin(), groups.end(), [&](const auto& g) { return g.first == k; });
    if (it == groups.end()) groups.push_back({k, {c}});
    else it->second.push_back(c);
  }
  std::stable_sort(groups.begin(), groups.end(),
                   [](const auto& a, const auto& b) { return a.second.size() > b.second.size(); });
  std::vector<int> used(K, 0), ng(K, 0);
  slot_cls.assign((size_t)K * Cw, -1);
  owner.assign(cls.size(), -1);
  for (const auto& g : groups) {
    const int sz = (int)g.second.size();
    int best = -1;
    for (int w = 0; w < K; ++w)
      if (used[w] + sz <= Cw && (best < 0 || ng[w] < ng[best] || (ng[w] == ng[best] && used[w] < used[best]))) best = w;
    if (best < 0 && !split) return false;
    for (size_t k = 0; k < g.second.size();) {
      if (best < 0 || used[best] >= Cw) {  // split: the workgroup with the most free slots
        best = 0;
        for (int w = 1; w < K; ++w)
          if (used[w] < used[best]) best = w;
        if (used[best] >= Cw) return false;
        ++ng[best];
      } else if (k == 0) {
        ++ng[best];
      }
      const int c = g.second[k++];
      slot_cls[(size_t)best * Cw + used[best]] = c;
      owner[c] = (best << 8) | used[best];
      ++used[best];
    }
  }
  return true;
}

// forceK > 0: exactly that many workgroups per replica (a wide-hinted group, ksim_engine_set_replica_wgs);
// forceKr: that many for each replica (r06: the hints differ); hkeys_ok: when no K fits the keys in LDS, the keys
// may go to HBM (k_memo<..., kHKeys>, classes split over the workgroups as evenly as the slots allow).
static bool memo_plan(const ksim_engine* e, const std::vector<int>& reps, MemoPlan& pl, int forceK = 0,
                      bool hkeys_ok = false, const std::vector<int>* forceKr = nullptr) {
  using namespace ksim_memo;
  const int Rg = (int)reps.size();
  if (Rg == 0 || e->N > kMemoMaxRank + 1) return false;
  pl.Cmax = 1;
  for (int r : reps) pl.Cmax = std::max(pl.Cmax, (int)e->h_cls[r].size());
  const int K0 = forceK > 0 ? forceK : e->wgs_req > 0 ? e->wgs_req : std::min(64, e->cus / Rg);
  std::vector<int> Kr(Rg, K0);
  if (forceKr) Kr = *forceKr;
  if ((int)Kr.size() != Rg) return false;
  auto total = [&]() { int t = 0; for (int k : Kr) t += k; return t; };
  auto kmax = [&]() { return *std::max_element(Kr.begin(), Kr.end()); };
  if (*std::min_element(Kr.begin(), Kr.end()) < 1 || kmax() > 64 || total() > e->cus) return false;
  const bool forced = forceK > 0 || forceKr != nullptr;
  const int d0 = pl.decider ? 1 : 0;  // decider mode: classes on workgroups 1..K-1
  std::vector<std::vector<int>> sc(Rg), ow(Rg);
  // the smallest Cw >= Cw0 every replica's classes pack into (split: parts of a group on several workgroups)
  auto pack = [&](int Cw0, bool split) {
    for (int Cw = Cw0; Cw <= kMaxCw; ++Cw) {
      bool ok = true;
      for (int i = 0; ok && i < Rg; ++i) {
        const int K = Kr[i];
        std::vector<int> s1;
        ok = K > d0 && memo_assign(e->h_cls[reps[i]], K - d0, Cw, s1, ow[i], split);
        if (!ok) break;
        sc[i].assign((size_t)K * Cw, -1);
        std::copy(s1.begin(), s1.end(), sc[i].begin() + (size_t)d0 * Cw);
        for (int& o : ow[i]) o += d0 << 8;
      }
      if (ok) return Cw;
    }
    return 0;
  };
  auto cw0 = [&](int dd) {  // the fewest slots per workgroup that can hold every replica's classes
    int c = 1;
    for (int i = 0; i < Rg; ++i) c = std::max(c, ((int)e->h_cls[reps[i]].size() + Kr[i] - 1 - dd) / std::max(1, Kr[i] - dd));
    return c;
  };
  auto fold_waves = [&](int Cw, bool hk) {  // waves 1..9 need fold buffers on the critical path
    for (int f : {16, 12})
      if (memo_lds(e->N, Cw, f, hk) <= 160 * 1024) return f;
    return 0;
  };
  const void* fcap = (const void*)ksim_memo::k_memo<false, false>;
  int Cw = 0, nfw = 0;
  bool hk = false;
  for (;;) {
    Cw = pack(cw0(d0), false);
    nfw = Cw > 0 ? fold_waves(Cw, false) : 0;
    // every workgroup of the launch must be resident (they exchange granules every step)
    if (nfw > 0 && kmax() > 1 && total() > resident_cap(e, fcap, memo_lds(e->N, Cw, nfw)))
      return false;
    if (nfw > 0) break;
    if (hkeys_ok && !pl.decider) {  // the keys in HBM: LDS holds the cluster and the fold buffers only
      Cw = pack(cw0(0), true);
      nfw = Cw > 0 ? fold_waves(Cw, true) : 0;
      if (nfw > 0 && kmax() > 1 && total() > resident_cap(e, fcap, memo_lds(e->N, Cw, nfw, true))) return false;
      if (nfw > 0) {
        hk = true;
        break;
      }
    }
    const int K = Kr[0];
    if (forced || e->wgs_req > 0 || K >= 64 || Rg * (K + 1) > e->cus) return false;
    std::fill(Kr.begin(), Kr.end(), K + 1);
  }
  pl.K = kmax();
  pl.nwg = total();
  pl.Kr = Kr;
  pl.wgoff.assign(Rg, 0);
  for (int i = 1; i < Rg; ++i) pl.wgoff[i] = pl.wgoff[i - 1] + Kr[i - 1];
  pl.Cw = Cw;
  pl.nfw = nfw;
  pl.hkeys = hk;
  pl.lds = memo_lds(e->N, Cw, nfw, hk);
  pl.pod.assign((size_t)Rg * pl.Cmax, PodDev{});
  pl.owner.assign((size_t)Rg * pl.Cmax, -1);
  pl.wgcls.assign((size_t)pl.nwg * Cw, -1);
  pl.wgref.assign((size_t)pl.nwg * Cw, 0);
  pl.wggrp.assign((size_t)pl.nwg * Cw, 0ull);
  for (int i = 0; i < Rg; ++i) {
    const std::vector<PodDev>& cls = e->h_cls[reps[i]];
    for (size_t c = 0; c < cls.size(); ++c) {
      pl.pod[(size_t)i * pl.Cmax + c] = cls[c];
      pl.owner[(size_t)i * pl.Cmax + c] = ow[i][c];
    }
    for (int w = 0; w < Kr[i]; ++w) {
      const size_t o = ((size_t)pl.wgoff[i] + w) * Cw;
      for (int j = 0; j < Cw; ++j) {
        const int c = sc[i][(size_t)w * Cw + j];
        pl.wgcls[o + j] = c;
        pl.wgref[o + j] = j;
        if (c < 0) continue;
        for (int j2 = 0; j2 < j; ++j2) {  // first slot with the same score request
          const int c2 = sc[i][(size_t)w * Cw + j2];
          if (c2 >= 0 && cls[c2].cpu_nz == cls[c].cpu_nz && cls[c2].milli == cls[c].milli && cls[c2].num == cls[c].num) {
            pl.wgref[o + j] = j2;
            break;
          }
        }
        pl.wggrp[o + pl.wgref[o + j]] |= 1ull << j;
      }
    }
  }
  return true;
}

template <typename T>
static int ensure_buf(T*& p, size_t& cap, size_t n) {
  if (n <= cap && p) return KSIM_OK;
  if (p) KSIM_HIP(hipFree(p));
  p = nullptr;
  KSIM_HIP(hipMalloc(&p, sizeof(T) * std::max(n, (size_t)1)));
  cap = n;
  return KSIM_OK;
}

// The FGD score steps, built once per process on the host (nullptr if the check fails: k_memo
// then evaluates the sigmoid expression itself).
static const double* score_table() {
  static double th[102];
  static const bool ok = build_score_thresholds(th);
  return ok ? th : nullptr;
}

// ---- k_hmemo planning (memoised FGD replay with the keys in HBM, ksim_hmemo.hpp) ----
struct HPlan {
  int Cmax = 1, Gmax = 1, Smax = 1, Npad = 0, nb = 0;
  int K = 1, S = 0, nbw = 0;      // workgroups per replica, ranks per workgroup, L1 blocks per workgroup
  bool l2 = false;                // the second maxima beside L1 (the wide form, when they fit in LDS; KSIM_VARIANT hl2)
  size_t lds = 0;
  std::vector<int> cg;            // [Rg][2] classes, groups
  std::vector<PodDev> cls, gpod;  // [Rg][Cmax] (sorted by group), [Rg][Gmax]
  std::vector<uint16_t> cgrp;     // [Rg][Cmax]
  std::vector<int> evc;           // [Rg][stride] class slot of each event, -1 delete
  std::vector<NodeRec> st;        // [Rg][Smax] distinct initial node states
  std::vector<int> ns;            // [Rg]
  std::vector<int> nstate;        // [Rg][Npad] state of each rank, -1 padding
  // Typed replicas (a GPU typical pod names models): per GPU model of the cluster, the typical table cut to
  // the CPU-only pods and the GPU pods that accept the model (ksim_hmemo.hpp, "per-model tables")
  int Mtab = 0, Mslots = 0;       // longest replica's concatenated tables, most models of one replica
  std::vector<int> mtoff;         // [Rg][KSIM_MAX_TYPES] kMtPresent | slot << 21 | entries << 12 | offset
  std::vector<uint8_t> mtab;      // [Rg][Mtab] typical-table index of each entry
};

// Classes of each replica grouped by score request (cpu_nz, milli, num: the candidate states of
// fgd_score.go:99-149 depend on nothing else), and the distinct initial node states (the keys
// before the first event depend on the state, the class and the rank only).
static bool hmemo_plan(const ksim_engine* e, const std::vector<int>& reps, int stride, HPlan& pl, int forceK = 0,
                       int forceS = 0) {
  using namespace ksim_hmemo;
  const int Rg = (int)reps.size();
  if (Rg == 0 || e->N > kHRankMax || !score_table()) return false;
  pl.Npad = (e->N + kFan - 1) / kFan * kFan;
  pl.nb = pl.Npad / kFan;
  // one workgroup per replica while one L1 level covers the cluster; wider clusters are sliced over
  // K co-resident workgroups (at most 64: one granule column per polling lane), S a multiple of 64
  // (run_mode 5 with wgs_per_replica > 1 asks for the wide form on a small cluster too; when the
  // wide grid would not fit the usable CUs a small cluster keeps one workgroup per replica)
  const bool small = e->N <= kMaxNb * kFan;
  pl.K = 1;
  pl.S = e->N;
  pl.nbw = pl.nb;
  if (forceK > 0) {  // a node-sharded group: every shard's slices alike (the caller checked S, K)
    pl.S = forceS;
    pl.K = forceK;
    pl.nbw = forceS / kFan;
  } else if (!small || (e->run_mode == 5 && e->wgs_req > 1)) {
    const int want = e->wgs_req > 1 ? e->wgs_req : 64;
    const int S = std::max(kFan, (e->N + want - 1) / want + kFan - 1) / kFan * kFan;
    const int K = (e->N + S - 1) / S;
    if (S <= kMaxNb * kFan && (size_t)Rg * K <= (size_t)e->cus) {
      pl.S = S;
      pl.K = K;
      pl.nbw = S / kFan;
    } else if (!small) {
      return false;
    }
  }
  std::vector<std::vector<int>> ord(Rg), gof(Rg), slot(Rg), gfirst(Rg), sof(Rg);
  std::vector<std::vector<NodeRec>> sts(Rg);
  pl.Cmax = pl.Gmax = pl.Smax = 1;
  for (int i = 0; i < Rg; ++i) {
    const int r = reps[i];
    const std::vector<PodDev>& cls = e->h_cls[r];
    std::vector<std::array<int, 3>> gk;
    gof[i].resize(cls.size());
    for (size_t c = 0; c < cls.size(); ++c) {
      const std::array<int, 3> k{cls[c].cpu_nz, cls[c].milli, cls[c].num};
      const auto it = std::find(gk.begin(), gk.end(), k);
      gof[i][c] = (int)(it - gk.begin());
      if (it == gk.end()) { gk.push_back(k); gfirst[i].push_back((int)c); }
    }
    if ((int)cls.size() > kMaxClasses || (int)gk.size() > kMaxGroups) return false;
    ord[i].resize(cls.size());
    std::iota(ord[i].begin(), ord[i].end(), 0);
    std::stable_sort(ord[i].begin(), ord[i].end(), [&](int a, int b) { return gof[i][a] < gof[i][b]; });
    slot[i].assign(cls.size(), -1);
    for (size_t k = 0; k < ord[i].size(); ++k) slot[i][ord[i][k]] = (int)k;
    pl.Cmax = std::max(pl.Cmax, (int)cls.size());
    pl.Gmax = std::max(pl.Gmax, (int)gk.size());
    // distinct initial states (every field but the rank)
    if (e->h_rec[r].size() != (size_t)e->N) return false;
    std::map<std::array<uint32_t, 7>, int> sid;
    sof[i].assign(pl.Npad, -1);
    for (int j = 0; j < e->N; ++j) {
      const NodeRec& n = e->h_rec[r][j];
      std::array<uint32_t, 7> k;
      std::memcpy(k.data(), &n, sizeof k);
      auto it = sid.find(k);
      if (it == sid.end()) {
        it = sid.emplace(k, (int)sts[i].size()).first;
        sts[i].push_back(n);
      }
      sof[i][(int)(n.name_rank - (uint32_t)e->node_off)] = it->second;
    }
    pl.Smax = std::max(pl.Smax, (int)sts[i].size());
  }
  {
    // L2 spares the flagged blocks' key reloads.  They bound the wide form's class waves (C5: 100k nodes, the
    // keys far beyond L2, 55 flagged rows per refresh from HBM), while one workgroup over an openb cluster
    // keeps its keys in L2 and is bound by F: there L2 only adds update work (profiles/r04/hmemo/).
    // Off by default since r05: in the wide form its code alone cost C5 4.09 -> 4.22 s, and it is compiled only into
    // the one-workgroup instantiations; KSIM_VARIANT=hl2=1 turns it on there.
    const bool want = variant("hl2", 0) == 1 && pl.K == 1;
    pl.l2 = want && hmemo_layout(pl.S, pl.Cmax, pl.Gmax, pl.nbw, true, 0).total <= 160 * 1024;
  }
  {  // per-model tables of the typed replicas (KSIM_VARIANT=hmodel=0: the whole table for every model, as before r05)
    const bool on = variant("hmodel", 1) != 0;
    pl.Mtab = pl.Mslots = 0;
    pl.mtoff.assign((size_t)Rg * KSIM_MAX_TYPES, 0);
    std::vector<std::vector<uint8_t>> mt(Rg);
    for (int i = 0; on && pl.K == 1 && i < Rg; ++i) {  // (the wide form evaluates the whole table)
      const int r = reps[i];
      if (!e->reps[r].typed || e->h_tp[r].size() != (size_t)e->reps[r].nt) continue;
      const std::vector<TypDev>& tpv = e->h_tp[r];
      const int ncpu = e->reps[r].ncpu, nt = e->reps[r].nt;
      uint32_t models = 0u;
      for (const NodeRec& n : e->h_rec[r]) models |= 1u << n.gpu_type;
      int slot = 0;
      for (int m = 0; m < KSIM_MAX_TYPES; ++m) {
        if (!((models >> m) & 1u)) continue;
        const int off = (int)mt[i].size();
        for (int t = 0; t < nt; ++t)
          if (t < ncpu || (tpv[t].tmask >> m) & 1u) mt[i].push_back((uint8_t)t);
        const int len = (int)mt[i].size() - off;
        pl.mtoff[(size_t)i * KSIM_MAX_TYPES + m] = (int)(ksim_hmemo::kMtPresent | (uint32_t)slot << 21 | (uint32_t)len << 12 | (uint32_t)off);
        ++slot;
      }
      pl.Mtab = std::max(pl.Mtab, (int)mt[i].size());
      pl.Mslots = std::max(pl.Mslots, slot);
    }
    // tables that do not fit (a 12-bit offset, or the LDS beside the keys' L1 level): the whole-table form
    // (KSIM_VARIANT hmodel=0), which evaluates the same bits, rather than no k_hmemo at all
    if (pl.Mtab > 4095 || hmemo_layout(pl.S, pl.Cmax, pl.Gmax, pl.nbw, pl.l2, pl.Mtab).total > 160 * 1024) {
      pl.Mtab = pl.Mslots = 0;
      std::fill(pl.mtoff.begin(), pl.mtoff.end(), 0);
      for (auto& v : mt) v.clear();
    }
    pl.mtab.assign((size_t)Rg * std::max(pl.Mtab, 1), 0);
    for (int i = 0; i < Rg; ++i) std::copy(mt[i].begin(), mt[i].end(), pl.mtab.begin() + (size_t)i * std::max(pl.Mtab, 1));
  }
  pl.lds = hmemo_layout(pl.S, pl.Cmax, pl.Gmax, pl.nbw, pl.l2, pl.Mtab).total;
  if (pl.lds > 160 * 1024) return false;
  pl.cg.assign((size_t)Rg * 2, 0);
  pl.cls.assign((size_t)Rg * pl.Cmax, PodDev{});
  pl.cgrp.assign((size_t)Rg * pl.Cmax, 0);
  pl.gpod.assign((size_t)Rg * pl.Gmax, PodDev{});
  pl.evc.assign((size_t)Rg * stride, -1);
  pl.st.assign((size_t)Rg * pl.Smax, NodeRec{});
  pl.ns.assign(Rg, 0);
  pl.nstate.assign((size_t)Rg * pl.Npad, -1);
  for (int i = 0; i < Rg; ++i) {
    const int r = reps[i];
    const std::vector<PodDev>& cls = e->h_cls[r];
    pl.cg[2 * i] = (int)cls.size();
    pl.cg[2 * i + 1] = (int)gfirst[i].size();
    for (size_t k = 0; k < ord[i].size(); ++k) {
      pl.cls[(size_t)i * pl.Cmax + k] = cls[ord[i][k]];
      pl.cgrp[(size_t)i * pl.Cmax + k] = (uint16_t)gof[i][ord[i][k]];
    }
    // a group's request: its first class's (the score part, fgd_score.go:99-149, is the group's), with the
    // least demanding Filter part of every class of the group -- min CPU, min memory, every accepted GPU
    // model -- so that Filter of it on a node fails only when every class of the group fails (the group
    // pruning of k_hmemo's F list; nothing else reads these fields of a group's request)
    for (size_t g = 0; g < gfirst[i].size(); ++g) pl.gpod[(size_t)i * pl.Gmax + g] = cls[gfirst[i][g]];
    for (size_t c = 0; c < cls.size(); ++c) {
      PodDev& gp = pl.gpod[(size_t)i * pl.Gmax + gof[i][c]];
      gp.cpu_req = std::min(gp.cpu_req, cls[c].cpu_req);
      gp.mem = std::min(gp.mem, cls[c].mem);
      gp.tmask |= cls[c].tmask;
    }
    const std::vector<int>& ec = e->h_ev_cls[r];
    for (size_t k = 0; k < ec.size(); ++k) pl.evc[(size_t)i * stride + k] = ec[k] < 0 ? -1 : slot[i][ec[k]];
    std::copy(sts[i].begin(), sts[i].end(), pl.st.begin() + (size_t)i * pl.Smax);
    pl.ns[i] = (int)sts[i].size();
    std::copy(sof[i].begin(), sof[i].end(), pl.nstate.begin() + (size_t)i * pl.Npad);
  }
  return true;
}

template <typename T>
static int upload_vec(T*& p, size_t& cap, const std::vector<T>& v, hipStream_t st) {
  int rc = ensure_buf(p, cap, v.size());
  if (rc) return rc;
  KSIM_HIP(hipMemcpyAsync(p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, st));
  return KSIM_OK;
}

static int prepare_hmemo(ksim_engine* e, const std::vector<int>& reps, int max_ev, int forceK = 0, int forceS = 0) {
  e->hplan_ok = false;
  if (!e->hplan) e->hplan = new HPlan();
  HPlan& pl = *e->hplan;
  const int stride = std::max(max_ev, 1);
  if (!hmemo_plan(e, reps, stride, pl, forceK, forceS)) return KSIM_OK;
  const int Rg = (int)reps.size();
  e->hplan_reps = reps;
  hipStream_t st = e->stream;
  int rc;
  if ((rc = upload_vec(e->d_h_cg, e->h_cap[0], pl.cg, st))) return rc;
  if ((rc = upload_vec(e->d_h_cls, e->h_cap[1], pl.cls, st))) return rc;
  if ((rc = upload_vec(e->d_h_cgrp, e->h_cap[2], pl.cgrp, st))) return rc;
  if ((rc = upload_vec(e->d_h_gpod, e->h_cap[3], pl.gpod, st))) return rc;
  if ((rc = upload_vec(e->d_h_evc, e->h_cap[4], pl.evc, st))) return rc;
  if ((rc = upload_vec(e->d_h_st, e->h_cap[5], pl.st, st))) return rc;
  if ((rc = upload_vec(e->d_h_ns, e->h_cap[6], pl.ns, st))) return rc;
  if ((rc = upload_vec(e->d_h_nstate, e->h_cap[7], pl.nstate, st))) return rc;
  if ((rc = ensure_buf(e->d_h_gsc, e->h_cap[8], (size_t)Rg * pl.Gmax * pl.Smax))) return rc;
  if ((rc = ensure_buf(e->d_h_keys, e->h_cap[9], (size_t)Rg * pl.Cmax * pl.Npad))) return rc;
  if ((rc = ensure_buf(e->d_h_l1, e->h_cap[10], (size_t)Rg * pl.Cmax * pl.nb))) return rc;
  if (pl.l2 && (rc = ensure_buf(e->d_h_l2, e->h_cap[14], (size_t)Rg * pl.Cmax * pl.nb))) return rc;
  if ((rc = ensure_buf(e->d_h_cnt, e->h_cap[11], (size_t)Rg * pl.Cmax))) return rc;
  if (pl.Mtab > 0) {
    if ((rc = upload_vec(e->d_h_mtoff, e->h_cap[15], pl.mtoff, st))) return rc;
    if ((rc = upload_vec(e->d_h_mtab, e->h_cap[16], pl.mtab, st))) return rc;
    if ((rc = ensure_buf(e->d_h_na, e->h_cap[17], (size_t)Rg * pl.Mslots * ksim_hmemo::kNaStride))) return rc;
  }
  if (!e->d_th) {
    KSIM_HIP(hipMalloc(&e->d_th, sizeof(double) * 102));
    KSIM_HIP(hipMemcpyAsync(e->d_th, score_table(), sizeof(double) * 102, hipMemcpyHostToDevice, st));
  }
  KSIM_HIP(hipStreamSynchronize(st));  // the host vectors are pageable
  e->hplan_ok = true;
  return KSIM_OK;
}

// Plan and upload the k_memo launch of the FGD replicas (before the timed region of a run; cached
// until events or policies change).
static int upload_memo(ksim_engine* e, const std::vector<int>& reps, int max_ev);

static int prepare_memo(ksim_engine* e, int max_ev) {
  if (e->run_mode == 1 || e->run_mode == 2 || e->shard_world > 0) return KSIM_OK;
  std::vector<int> reps, wide, narrow;
  for (int r = 0; r < e->R; ++r)
    if (e->reps[r].policy == POL_FGD) {
      reps.push_back(r);
      (e->wgs_hint[r] > 1 ? wide : narrow).push_back(r);
    }
  if (!e->mplan_dirty && reps == e->mplan_all && max_ev == e->mplan_max_ev) return KSIM_OK;
  e->mplan_dirty = false;
  e->mplan_all = reps;
  e->mplan_max_ev = max_ev;
  e->mplan_ok = false;
  e->hplan_ok = false;
  e->split_fgd = false;
  e->mplan_reps.clear();
  e->hplan_reps.clear();
  if (reps.empty()) return KSIM_OK;
  if (e->run_mode == 5) return prepare_hmemo(e, reps, max_ev);  // k_hmemo required
  if (!e->mplan) e->mplan = new MemoPlan();
  MemoPlan& pl = *e->mplan;
  // run_mode 4 (or KSIM_VARIANT=memo_decider=1 with run_mode 0): the decider variant of k_memo
  pl.decider = e->run_mode == 4 || (e->run_mode == 0 && variant("memo_decider", 0) == 1);
  // run_mode 0 with some FGD replicas hinted wide (ksim_engine_set_replica_wgs, the paper sweep's longest chains):
  // those on k_memo, each at its hinted width (the keys in HBM when they do not fit in LDS), the others on k_hmemo at
  // one workgroup each, both groups in one concurrent run (run_persistent)
  if (e->run_mode == 0 && !wide.empty() && !narrow.empty() && !pl.decider) {
    std::vector<int> kr;  // each wide replica at its own hinted width
    for (int r : wide) kr.push_back(e->wgs_hint[r]);
    if (memo_plan(e, wide, pl, 0, true, &kr)) {
      int rc = upload_memo(e, wide, max_ev);
      if (rc) return rc;
      rc = prepare_hmemo(e, narrow, max_ev);
      if (rc) return rc;
      if (e->hplan_ok && e->hplan->K == 1) {
        e->split_fgd = true;
        return KSIM_OK;
      }
      e->mplan_ok = false;  // no one-workgroup plan for the others: one plan for every FGD replica, below
      e->mplan_reps.clear();
      e->hplan_ok = false;
    }
  }
  std::vector<int> kr;  // every FGD replica hinted: each at its width
  if (wide.size() == reps.size())
    for (int r : reps) kr.push_back(e->wgs_hint[r]);
  if (!memo_plan(e, reps, pl, 0, e->run_mode == 3 || !kr.empty(), kr.empty() ? nullptr : &kr))
    return e->run_mode == 0 ? prepare_hmemo(e, reps, max_ev) : KSIM_OK;
  return upload_memo(e, reps, max_ev);
}

// Upload the k_memo plan of `reps` (memo_plan made it): the per-class tables, the owner code of every event.
static int upload_memo(ksim_engine* e, const std::vector<int>& reps, int max_ev) {
  MemoPlan& pl = *e->mplan;
  const int Rg = (int)reps.size();
  int rc;
  if ((rc = ensure_buf(e->d_m_pod, e->m_cap[0], pl.pod.size()))) return rc;
  if ((rc = ensure_buf(e->d_m_owner, e->m_cap[1], pl.owner.size()))) return rc;
  if ((rc = ensure_buf(e->d_m_wgcls, e->m_cap[2], pl.wgcls.size()))) return rc;
  if ((rc = ensure_buf(e->d_m_wgref, e->m_cap[3], pl.wgref.size()))) return rc;
  if ((rc = ensure_buf(e->d_m_wggrp, e->m_cap[4], pl.wggrp.size()))) return rc;
  const int stride = std::max(max_ev, 1);
  if ((rc = ensure_buf(e->d_win, e->m_cap[5], (size_t)Rg * stride))) return rc;
  if ((rc = ensure_buf(e->d_m_evo, e->m_cap[6], (size_t)Rg * stride))) return rc;
  if ((rc = ensure_buf(e->d_m_evcls, e->m_cap2[0], (size_t)Rg * stride))) return rc;
  if ((rc = ensure_buf(e->d_topg, e->m_cap2[1], (size_t)Rg * stride * ksim_memo::kTopWords))) return rc;
  std::vector<int> evcls((size_t)Rg * stride, -1);
  for (int gi = 0; gi < Rg; ++gi) {
    const std::vector<int>& ec = e->h_ev_cls[reps[gi]];
    for (size_t i = 0; i < ec.size(); ++i) evcls[(size_t)gi * stride + i] = ec[i];
  }
  // owner code of every event: workgroup << 16 | first slot of its score group << 8 | slot; -1 delete
  std::vector<int> evo((size_t)Rg * stride, -1);
  for (int gi = 0; gi < Rg; ++gi) {
    const std::vector<int>& ec = e->h_ev_cls[reps[gi]];
    for (size_t i = 0; i < ec.size(); ++i) {
      if (ec[i] < 0) continue;
      const int o = pl.owner[(size_t)gi * pl.Cmax + ec[i]];
      const int w = o >> 8, slot = o & 0xff;
      const int ref = pl.wgref[((size_t)pl.wgoff[gi] + w) * pl.Cw + slot];
      evo[(size_t)gi * stride + i] = (w << 16) | (ref << 8) | slot;
    }
  }
  hipStream_t st = e->stream;
  KSIM_HIP(hipMemcpyAsync(e->d_m_evo, evo.data(), sizeof(int) * evo.size(), hipMemcpyHostToDevice, st));
  KSIM_HIP(hipMemcpyAsync(e->d_m_evcls, evcls.data(), sizeof(int) * evcls.size(), hipMemcpyHostToDevice, st));
  KSIM_HIP(hipMemcpyAsync(e->d_m_pod, pl.pod.data(), sizeof(PodDev) * pl.pod.size(), hipMemcpyHostToDevice, st));
  KSIM_HIP(hipMemcpyAsync(e->d_m_owner, pl.owner.data(), sizeof(int) * pl.owner.size(), hipMemcpyHostToDevice, st));
  KSIM_HIP(hipMemcpyAsync(e->d_m_wgcls, pl.wgcls.data(), sizeof(int) * pl.wgcls.size(), hipMemcpyHostToDevice, st));
  KSIM_HIP(hipMemcpyAsync(e->d_m_wgref, pl.wgref.data(), sizeof(int) * pl.wgref.size(), hipMemcpyHostToDevice, st));
  KSIM_HIP(hipMemcpyAsync(e->d_m_wggrp, pl.wggrp.data(), sizeof(unsigned long long) * pl.wggrp.size(),
                          hipMemcpyHostToDevice, st));
  if (!e->d_th && score_table()) {
    KSIM_HIP(hipMalloc(&e->d_th, sizeof(double) * 102));
    KSIM_HIP(hipMemcpyAsync(e->d_th, score_table(), sizeof(double) * 102, hipMemcpyHostToDevice, st));
  }
  std::vector<int> wgmap((size_t)pl.nwg);
  for (int gi = 0; gi < Rg; ++gi)
    for (int w = 0; w < pl.Kr[gi]; ++w) wgmap[(size_t)pl.wgoff[gi] + w] = (gi << 8) | w;
  if ((rc = ensure_buf(e->d_m_wgmap, e->m_cap2[3], wgmap.size()))) return rc;
  KSIM_HIP(hipMemcpyAsync(e->d_m_wgmap, wgmap.data(), sizeof(int) * wgmap.size(), hipMemcpyHostToDevice, st));
  KSIM_HIP(hipStreamSynchronize(st));  // the host vectors are pageable and short-lived
  if (pl.hkeys && (rc = ensure_buf(e->d_m_hkeys, e->m_cap2[2], (size_t)pl.nwg * pl.Cw * e->N))) return rc;
  e->mplan_reps = reps;
  e->mplan_ok = true;
  return KSIM_OK;
}

// KSIM_TEST=hdelay=<mask>: the memoised kernels' hand-over stress delays (ksim_memo.hpp hdelay; the bits are
// per kernel); a nonzero mask selects the general (non-lean) instantiation, which alone carries them.
static int hdelay_mask() { return (int)(test_knob("hdelay", 0) & 0xff); }

// st: the stream (a concurrent run's side stream, else the engine's); started / gate_epoch: the residency gate's
// flags (a concurrent run launches the next group once every workgroup of this one has started: a plain launch
// then, since the device is otherwise idle until the gate opens)
static int launch_memo(ksim_engine* e, const MemoPlan& pl, int Rg, int first, int max_ev, hipStream_t st,
                       int* started = nullptr, int gate_epoch = 0) {
  int rc;
  const int stride = std::max(max_ev, 1);
  KSIM_HIP(hipMemsetAsync(e->d_win, 0, sizeof(unsigned) * (size_t)Rg * stride, st));
  if (pl.decider)
    KSIM_HIP(hipMemsetAsync(e->d_topg, 0, sizeof(unsigned) * (size_t)Rg * stride * ksim_memo::kTopWords, st));
  ksim_memo::MemoArgs ma;
  ma.reps = e->d_reps;
  ma.rep_list = e->d_replist + first;
  ma.wg_map = e->d_m_wgmap;
  ma.N = e->N;
  ma.K = pl.K;
  ma.Cw = pl.Cw;
  ma.nfw = pl.nfw;
  ma.Cmax = pl.Cmax;
  ma.cls_pod = e->d_m_pod;
  ma.cls_owner = e->d_m_owner;
  ma.wg_cls = e->d_m_wgcls;
  ma.wg_ref = e->d_m_wgref;
  ma.wg_grp = e->d_m_wggrp;
  ma.ev_owner = e->d_m_evo;
  ma.th = e->d_th;
  ma.win = e->d_win;
  ma.win_stride = stride;
  ma.fail = e->d_fail;
  ma.prof = nullptr;
  ma.trace = nullptr;
  ma.trace_steps = 0;
  ma.decider = pl.decider ? 1 : 0;
  ma.ev_cls = e->d_m_evcls;
  ma.topg = e->d_topg;
  ma.hkeys = pl.hkeys ? e->d_m_hkeys : nullptr;
  ma.started = started;
  ma.gate_epoch = gate_epoch;
  ma.skip = variant("skip", 1) != 0;
  ma.delay = hdelay_mask();
  const char* pe = std::getenv("KSIM_PROFILE");
  const bool profile = pe && pe[0] == '1';
  const bool tracing = pe && pe[0] == '2';
  unsigned long long* d_trace = nullptr;
  const int TS = std::min(max_ev, 4000);
  constexpr int kT = ksim_memo::kTrace;
  if (tracing) {
    KSIM_HIP(hipMalloc(&d_trace, sizeof(unsigned long long) * kT * (size_t)pl.nwg * TS));
    KSIM_HIP(hipMemsetAsync(d_trace, 0, sizeof(unsigned long long) * kT * (size_t)pl.nwg * TS, st));
    ma.trace = d_trace;
    ma.trace_steps = TS;
  }
  if (profile) {
    if ((rc = ensure_buf(e->d_prof, e->prof_cap, (size_t)pl.nwg * ksim_memo::kProfPhases))) return rc;
    KSIM_HIP(hipMemsetAsync(e->d_prof, 0, sizeof(unsigned long long) * (size_t)pl.nwg * ksim_memo::kProfPhases, st));
    ma.prof = e->d_prof;
  }
  // the general instantiation for the profile / trace / deletes / no score table, else the lean one (with the
  // report's stores when the report is on)
  const bool general = profile || tracing || !e->d_th ||
                       std::any_of(e->mplan_reps.begin(), e->mplan_reps.end(), [&](int r) { return (bool)e->has_delete[r]; });
  // the hdelay test knob: the lean kernel with the stress delays compiled in (or the general one, which has them)
  using ksim_memo::k_memo;
  const void* f = pl.decider ? (const void*)k_memo<true, true>
                  : pl.hkeys ? (general ? (const void*)k_memo<false, true, false, false, true>
                                        : e->report ? (const void*)k_memo<false, false, false, true, true>
                                                    : (const void*)k_memo<false, false, false, false, true>)
                  : general ? (const void*)k_memo<false, true>
                  : ma.delay ? (const void*)k_memo<false, false, true>
                  : e->report ? (const void*)k_memo<false, false, false, true> : (const void*)k_memo<false, false>;
  const TypDev* tpp = e->d_tp;
  rc = launch_persistent(f, pl.nwg, ksim_memo::kMBlock, pl.lds, st, e->coop && pl.K > 1 && !started, ma, tpp);
  if (rc) return rc;
  hipLaunchKernelGGL(ksim_memo::k_memo_finish, dim3((unsigned)((stride + 255) / 256), (unsigned)Rg), dim3(256), 0, st,
                     e->d_reps, (const int*)(e->d_replist + first), e->N);
  KSIM_HIP(hipGetLastError());
  if (tracing) {
    // per step: owner's start -> publish, publish -> each other workgroup's receive, receive -> start
    // (s_memrealtime, 100 MHz); replica 0 only
    KSIM_HIP(hipStreamSynchronize(st));
    const int K = pl.Kr[0];
    std::vector<unsigned long long> h((size_t)kT * pl.nwg * TS);
    KSIM_HIP(hipMemcpy(h.data(), d_trace, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    KSIM_HIP(hipFree(d_trace));
    std::vector<int> evo((size_t)TS);
    KSIM_HIP(hipMemcpy(evo.data(), e->d_m_evo, sizeof(int) * TS, hipMemcpyDeviceToHost));
    auto at = [&](int w, int s, int k) { return (double)h[((size_t)w * TS + s) * kT + k]; };
    double crit = 0, hand = 0, hmax = 0, period = 0, lag = 0, f0 = 0, spin = 0;
    int nc = 0, nh = 0, nf = 0;
    for (int s = 1; s + 1 < TS; ++s) {
      if (evo[s] < 0 || evo[s + 1] < 0) continue;
      const int o = evo[s] >> 16, o2 = evo[s + 1] >> 16;
      crit += at(o, s, 1) - at(o, s, 0);
      if (at(o, s, 2) > 0 && at(o, s, 3) > 0) {
        f0 += at(o, s, 3) - at(o, s, 0);   // start -> all critical F done
        spin += at(o, s, 2) - at(o, s, 3); // -> fresh key known
        ++nf;
      }
      period += at(o2, s + 1, 1) - at(o, s, 1);
      if (o2 != o) lag += at(o2, s + 1, 0) - at(o2, s, 1);  // next owner: receive s -> start s+1
      ++nc;
      for (int w = 0; w < K; ++w) {
        if (w == o) continue;
        const double d = at(w, s, 1) - at(o, s, 1);
        hand += d;
        hmax = std::max(hmax, d);
        ++nh;
      }
    }
    if (nc && nh)
      std::fprintf(stderr, "ksim memo trace (replica 0, %d steps, us): owner start->publish %.3f; publish->receive mean %.3f max %.3f; "
                   "next owner receive->start %.3f; publish->publish %.3f; owner start->all F done %.3f, ->fresh key %.3f\n",
                   TS, crit / nc / 100, hand / nh / 100, hmax / 100, lag / nc / 100, period / nc / 100,
                   nf ? f0 / nf / 100 : 0.0, nf ? (f0 + spin) / nf / 100 : 0.0);
  }
  if (profile) {
    KSIM_HIP(hipStreamSynchronize(st));
    const int nb = pl.nwg, P = ksim_memo::kProfPhases;
    std::vector<unsigned long long> h((size_t)nb * P);
    KSIM_HIP(hipMemcpy(h.data(), e->d_prof, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    static const char* names[] = {"init", "A:crit-F+list", "syncA", "B:publish", "B:eval", "syncB", "C:keys", "top2",
                                  "poll+bind", "end-sync"};
    std::fprintf(stderr, "ksim memo profile: %d workgroups (K=%d Cw=%d nfw=%d), %d steps; us/step mean [max]:", nb, pl.K,
                 pl.Cw, pl.nfw, max_ev);
    double init = 0;
    for (int b = 0; b < nb; ++b) init += (double)h[(size_t)b * P] / 1e5;
    std::fprintf(stderr, " (init %.3f ms)", init / nb);
    for (int ph = 1; ph < 10; ++ph) {
      double sum = 0, mx = 0;
      for (int b = 0; b < nb; ++b) {
        const double us = (double)h[(size_t)b * P + ph] / 100.0 / std::max(max_ev, 1);
        sum += us;
        mx = std::max(mx, us);
      }
      std::fprintf(stderr, " %s %.3f [%.3f];", names[ph], sum / nb, mx);
    }
    double cyc = 0, tick = 0;
    for (int b = 0; b < nb; ++b) { cyc += (double)h[(size_t)b * P + 10]; tick += (double)h[(size_t)b * P + 11]; }
    for (int ph = 12; ph < 21; ++ph) {
      double sum = 0;
      for (int b = 0; b < nb; ++b) sum += (double)h[(size_t)b * P + ph] / 100.0 / std::max(max_ev, 1);
      static const char* extra[] = {"listwave-A", "listwave-C", "step-start loads", "owner A per step",
                                    "owner: prefetch done", "crit F all done", "keys", "result written",
                                    "granule stored"};
      // owner phases: summed over the K workgroups of a replica (one owner per step)
      std::fprintf(stderr, " %s %.3f;", extra[ph - 12], ph >= 15 ? sum / std::max(Rg, 1) : sum / nb);
    }
    if (pl.decider) {  // the deciders' own phases (workgroup 0 of each replica)
      static const char* dn[] = {"list + top wait", "F", "decide + bind", "end barrier"};
      std::fprintf(stderr, " | decider:");
      for (int ph = 20; ph < 24; ++ph) {
        double sum = 0;
        for (int b = 0; b < nb; b += pl.K) sum += (double)h[(size_t)b * P + ph] / 100.0 / std::max(max_ev, 1);
        std::fprintf(stderr, " %s %.3f;", dn[ph - 20], sum / std::max(nb / pl.K, 1));
      }
    }
    if (tick > 0) std::fprintf(stderr, " shader clock %.0f MHz, wall %.3f ms", cyc / tick * 100.0, tick / nb / 1e5);
    std::fprintf(stderr, "\n");
  }
  return KSIM_OK;
}

// The initial keys, L1 maxima and feasible counts of k_hmemo's plan (k_hinit_gk, k_hinit_keys); roff: a
// node-sharded engine's first global rank.
static int hmemo_init_keys(ksim_engine* e, int Rg, int first, hipStream_t st, int roff) {
  using namespace ksim_hmemo;
  const HPlan& pl = *e->hplan;
  HInitArgs ia;
  ia.roff = roff;
  ia.reps = e->d_reps;
  ia.rep_list = e->d_replist + first;
  ia.N = e->N;
  ia.Npad = pl.Npad;
  ia.nb = pl.nb;
  ia.Cmax = pl.Cmax;
  ia.Gmax = pl.Gmax;
  ia.Smax = pl.Smax;
  ia.cg = e->d_h_cg;
  ia.cls = e->d_h_cls;
  ia.cgrp = e->d_h_cgrp;
  ia.gpod = e->d_h_gpod;
  ia.st = e->d_h_st;
  ia.ns = e->d_h_ns;
  ia.nstate = e->d_h_nstate;
  ia.gsc = e->d_h_gsc;
  ia.keys = e->d_h_keys;
  ia.l1 = e->d_h_l1;
  ia.l2 = pl.l2 ? e->d_h_l2 : nullptr;
  ia.cnt = e->d_h_cnt;
  ia.th = e->d_th;
  ia.mtoff = pl.Mtab > 0 ? e->d_h_mtoff : nullptr;
  ia.na = pl.Mtab > 0 ? e->d_h_na : nullptr;
  ia.Mslots = pl.Mslots;
  if (pl.Mtab > 0) {
    hipLaunchKernelGGL(k_hinit_na, dim3((unsigned)((kNaStride + 255) / 256), (unsigned)pl.Mslots, (unsigned)Rg), dim3(256), 0,
                       st, ia, (const TypDev*)e->d_tp);
    KSIM_HIP(hipGetLastError());
  }
  KSIM_HIP(hipMemsetAsync(e->d_h_cnt, 0, sizeof(int) * (size_t)Rg * pl.Cmax, st));
  hipLaunchKernelGGL(k_hinit_gk, dim3((unsigned)((pl.Smax + 255) / 256), (unsigned)pl.Gmax, (unsigned)Rg), dim3(256), 0,
                     st, ia, (const TypDev*)e->d_tp);
  KSIM_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_hinit_keys, dim3((unsigned)((pl.Npad + 255) / 256), (unsigned)pl.Cmax, (unsigned)Rg), dim3(256), 0,
                     st, ia);
  KSIM_HIP(hipGetLastError());
  return KSIM_OK;
}

static bool dead_skip(const ksim_engine* e, const std::vector<int>& reps);

// k_hmemo's arguments for the planned launch (one group of Rg replicas from d_replist + first).
static ksim_hmemo::HMemoArgs hmemo_args(ksim_engine* e, int first, int stride) {
  using namespace ksim_hmemo;
  const HPlan& pl = *e->hplan;
  HMemoArgs ma;
  std::memset(&ma, 0, sizeof ma);  // every field a caller does not set (the gate, profile, exchange pointers) is null
  ma.reps = e->d_reps;
  ma.rep_list = e->d_replist + first;
  ma.Mtab = pl.Mtab;
  ma.Mslots = pl.Mslots;
  ma.mtoff = pl.Mtab > 0 ? e->d_h_mtoff : nullptr;
  ma.mtab = pl.Mtab > 0 ? e->d_h_mtab : nullptr;
  ma.na = pl.Mtab > 0 ? e->d_h_na : nullptr;
  ma.N = e->N;
  ma.Npad = pl.Npad;
  ma.nb = pl.nb;
  ma.Cmax = pl.Cmax;
  ma.Gmax = pl.Gmax;
  ma.cg = e->d_h_cg;
  ma.cls = e->d_h_cls;
  ma.cgrp = e->d_h_cgrp;
  ma.gpod = e->d_h_gpod;
  ma.evc = e->d_h_evc;
  ma.stride = stride;
  ma.keys = e->d_h_keys;
  ma.l1 = e->d_h_l1;
  ma.l2 = pl.l2 ? e->d_h_l2 : nullptr;
  ma.cnt0 = e->d_h_cnt;
  ma.th = e->d_th;
  ma.prof = nullptr;
  ma.K = pl.K;
  ma.S = pl.S;
  ma.nbw = pl.nbw;
  ma.gran = e->d_gran;
  ma.fail = e->d_fail;
  ma.hist = nullptr;
  ma.roff = 0;
  ma.wbase = 0;
  ma.Ktot = pl.K;
  ma.tp = e->d_tp;
  ma.npeer = 0;
  ma.epoch = 0;
  {
    std::vector<int> all(e->R);
    std::iota(all.begin(), all.end(), 0);
    ma.skip = dead_skip(e, all) ? 1 : 0;
  }
  {  // KSIM_VARIANT hpf (one workgroup per replica): 1 = wave 0 lists the next refresh (the default since r04: C4 190.7 ->
     // 178-185 ms, C2 run_mode 5 50.3 -> 47.7 ms, profiles/r04/memo/ab_runs.txt), 2 = touches its flagged rows, 0 = off
    ma.pf = (int)variant("hpf", 1) & 7;  // (4: the wide form lists on wave 0 too)
  }
  ma.delay = hdelay_mask();
  {  // KSIM_VARIANT hprune (A/B): the F list's group pruning for replicas with more than this many typical pods
    // (-1: every replica; default 64: the large typed tables, where the F rounds bound the step)
    ma.prune_t = (int)variant("hprune", 64);
  }
  for (int q = 0; q < kMaxPeers; ++q) ma.peer[q] = nullptr;
  return ma;
}

// started: the residency gate's flags (K = 1 only); *gated tells the caller whether the launch carries them --
// not when its Rg workgroups cannot all be resident at once (a gate that could never open)
static int launch_hmemo(ksim_engine* e, int Rg, int first, int max_ev, hipStream_t st, int* started = nullptr,
                        int gate_epoch = 0, bool* gated = nullptr) {
  using namespace ksim_hmemo;
  const HPlan& pl = *e->hplan;
  const int stride = std::max(max_ev, 1);
  int irc = hmemo_init_keys(e, Rg, first, st, 0);
  if (irc) return irc;
  HMemoArgs ma = hmemo_args(e, first, stride);
  ma.started = pl.K == 1 ? started : nullptr;
  ma.gate_epoch = gate_epoch;
  if (gated) *gated = false;
  bool any_delete = false;
  for (const int r : e->hplan_reps) any_delete = any_delete || e->has_delete[r];  // the FGD replicas
  if (pl.K > 1) {
    if (any_delete) {
      int rc = ensure_buf(e->d_h_hist, e->h_cap[13], (size_t)Rg * pl.K * stride);
      if (rc) return rc;
      ma.hist = e->d_h_hist;
    }
    KSIM_HIP(hipMemsetAsync(e->d_gran, 0, sizeof(unsigned long long) * (size_t)Rg * 2 * pl.K * 2, st));
  }
  const char* pe = std::getenv("KSIM_PROFILE");
  const bool profile = pe && pe[0] == '1';
  if (profile) {
    int rc = ensure_buf(e->d_h_prof, e->h_cap[12], (size_t)Rg * pl.K * kHProf);
    if (rc) return rc;
    KSIM_HIP(hipMemsetAsync(e->d_h_prof, 0, sizeof(unsigned long long) * (size_t)Rg * pl.K * kHProf, st));
    ma.prof = e->d_h_prof;
  }
  const bool gen = profile || ma.delay != 0;  // the general instantiation: timers, stress delays
  // the large-table instantiations (per-model tables of typed replicas, the F-list pruning) when a replica of
  // the launch has use for them
  bool model = pl.Mtab > 0;
  for (const int r : e->hplan_reps) model = model || e->reps[r].nt > ma.prune_t;  // the FGD replicas
  const void* f = pl.K == 1 ? (gen ? (model ? (const void*)k_hmemo<0, true, true> : (const void*)k_hmemo<0, true>)
                                   : (model ? (const void*)k_hmemo<0, false, true> : (const void*)k_hmemo<0, false>))
                  : pl.K <= 64 ? (gen ? (const void*)k_hmemo<1, true> : (const void*)k_hmemo<1, false>)
                               : (gen ? (const void*)k_hmemo<4, true> : (const void*)k_hmemo<4, false>);
  if (pl.K > 1 && Rg * pl.K > resident_cap(e, f, pl.lds)) {
    std::fprintf(stderr, "ksim: k_hmemo needs %d co-resident workgroups\n", Rg * pl.K);
    return KSIM_ERANGE;
  }
  if (ma.started && Rg > resident_cap(e, f, pl.lds)) ma.started = nullptr;
  if (gated) *gated = ma.started != nullptr;
  const TypDev* tpp = e->d_tp;
  const int lrc = launch_persistent(f, Rg * pl.K, kHBlock, pl.lds, st, e->coop && pl.K > 1, ma, tpp);
  if (lrc) return lrc;
  hipLaunchKernelGGL(ksim_memo::k_memo_finish, dim3((unsigned)((stride + 255) / 256), (unsigned)Rg), dim3(256), 0, st,
                     e->d_reps, (const int*)(e->d_replist + first), e->N);
  KSIM_HIP(hipGetLastError());
  if (profile) {
    // per workgroup phase sums; refresh phases 0-4 run on one workgroup per step (the owner of the
    // changed node), so they are summed over a replica's workgroups, phase 5 is averaged over them
    KSIM_HIP(hipStreamSynchronize(st));
    const int nwg = Rg * pl.K;
    std::vector<unsigned long long> h((size_t)nwg * kHProf);
    KSIM_HIP(hipMemcpy(h.data(), e->d_h_prof, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    // waves 1-15 (the bulk: every class but the event's own): 0 + 2 on the F waves, 4 on the class
    // waves beside them, then 3; wave 0: 1 (the own class's refresh, the critical path), 5 (the rest of
    // its step: decide + Bind, then the end-of-step barrier)
    static const char* names[] = {"bulk: list (wave 1)", "critical own-class refresh", "bulk: F (F waves)",
                                   "bulk: join + class update", "class waves: class pass + flagged blocks",
                                   "wave 0 decide+bind+wait"};
    std::fprintf(stderr, "ksim hmemo profile: %d replicas x K=%d (S %d), LDS %zu B, Cmax %d Gmax %d Smax %d; us/step mean [max]:",
                 Rg, pl.K, pl.S, pl.lds, pl.Cmax, pl.Gmax, pl.Smax);
    const double steps = std::max(max_ev, 1);
    for (int ph = 0; ph < 6; ++ph) {
      double sum = 0, mx = 0;
      for (int g = 0; g < Rg; ++g) {
        double us = 0;
        for (int k = 0; k < pl.K; ++k) us += (double)h[((size_t)g * pl.K + k) * kHProf + ph] / 100.0 / steps;
        if (ph == 5) us /= pl.K;
        sum += us;
        mx = std::max(mx, us);
      }
      std::fprintf(stderr, " %s %.3f [%.3f];", names[ph], sum / Rg, mx);
    }
    double it = 0, fl = 0, rs = 0, cyc = 0, tick = 0;
    for (int b = 0; b < nwg; ++b) {
      it += (double)h[(size_t)b * kHProf + 7];
      fl += (double)h[(size_t)b * kHProf + 8];
      rs += (double)h[(size_t)b * kHProf + 9];
      cyc += (double)h[(size_t)b * kHProf + 10];
      tick += (double)h[(size_t)b * kHProf + 11];
    }
    if (rs > 0) std::fprintf(stderr, " F items/refresh %.1f, flagged classes/refresh %.1f;", it / rs, fl / rs);
    if (tick > 0) std::fprintf(stderr, " shader clock %.0f MHz, wall %.3f ms", cyc / tick * 100.0, tick / nwg / 1e5);
    std::fprintf(stderr, "\n");
  }
  return KSIM_OK;
}

extern "C" {

const char* ksim_strerror(int code) {
  switch (code) {
    case KSIM_OK: return "ok";
    case KSIM_EINVAL: return "invalid argument";
    case KSIM_ENOMEM: return "out of memory";
    case KSIM_EHIP: return "HIP runtime error";
    case KSIM_ERANGE: return "value outside engine encoding";
    case KSIM_ESTATE: return "call out of order";
    case KSIM_ENOTSUP: return "not supported";
    case KSIM_ENODEV: return "no gfx950 device";
    case KSIM_EIO: return "trace I/O error";
    case KSIM_EPEER: return "peer shard's device not reachable from this one";
    default: return "unknown error";
  }
}

int ksim_abi_version(void) { return KSIM_ABI_VERSION; }

#ifndef KSIM_SOURCE_HASH
#define KSIM_SOURCE_HASH "unknown"
#endif
const char* ksim_build_id(void) { return KSIM_SOURCE_HASH; }

int ksim_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  int c = 0;
  for (int i = 0; i < n; ++i)
    if (check_gfx950(i) == KSIM_OK) ++c;
  return c;
}

int ksim_engine_create(const ksim_config* cfg, int n_nodes, int n_replicas, ksim_engine** out) {
  if (!out || n_nodes <= 0 || n_replicas <= 0) return KSIM_EINVAL;
  *out = nullptr;
  if (n_nodes > kMaxRank) return KSIM_ERANGE;  // name ranks are 24-bit fields of the argmax key
  if (cfg && (cfg->run_mode < 0 || cfg->run_mode > 5)) return KSIM_EINVAL;
  const int dev = cfg ? cfg->device : 0;
  int rc = check_gfx950(dev);
  if (rc) return rc;
  KSIM_HIP(hipSetDevice(dev));
  ksim_engine* e = new ksim_engine();
  e->device = dev;
  e->N = n_nodes;
  e->R = n_replicas;
  if (cfg && cfg->nodes_per_block > 0) e->NB = std::min(cfg->nodes_per_block, kNBMax);
  if (cfg && cfg->steps_per_graph > 0) e->K = cfg->steps_per_graph;
  if (cfg) {
    e->run_mode = cfg->run_mode;
    e->wgs_req = cfg->wgs_per_replica;
  }
  {
    hipDeviceProp_t prop;
    KSIM_HIP(hipGetDeviceProperties(&prop, dev));
    e->cus = prop.multiProcessorCount;
    // KSIM_CUS: use at most this many CUs for co-resident persistent grids (a device shared with
    // another process; also the tests' way to exercise the residency checks)
    if (const char* c = std::getenv("KSIM_CUS")) e->cus = std::max(1, std::min(e->cus, std::atoi(c)));
    // KSIM_COOP=0: launch K > 1 grids with hipLaunchKernel (the grid is still capped by resident_cap);
    // the profiler passes of scripts/profile_config.sh use it -- rocprofv3 7.2 faults at process exit
    // after a cooperative launch
    if (const char* c = std::getenv("KSIM_COOP")) e->coop = std::atoi(c) != 0;
    // KSIM_VARIANT scan1: single-workgroup cheap-policy groups on k_scan1 with the records in VGPRs (2, default),
    // in LDS (1), or on k_replay (0) -- A/B switches
    e->scan1 = (int)variant("scan1", 2);
  }
  e->bpr = (n_nodes + e->NB - 1) / e->NB;
  e->tags_stride = (size_t)n_nodes * kTagStride + (size_t)n_nodes * 2;  // + int rank2idx[N]
  KSIM_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  KSIM_HIP(hipMalloc(&e->d_nodes, sizeof(NodeRec) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMalloc(&e->d_tags, sizeof(uint16_t) * e->tags_stride * n_replicas));
  KSIM_HIP(hipMalloc(&e->d_nodes_init, sizeof(NodeRec) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMalloc(&e->d_tags_init, sizeof(uint16_t) * e->tags_stride * n_replicas));
  KSIM_HIP(hipMemset(e->d_nodes, 0, sizeof(NodeRec) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMemset(e->d_nodes_init, 0, sizeof(NodeRec) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMemset(e->d_tags_init, 0, sizeof(uint16_t) * e->tags_stride * n_replicas));
  KSIM_HIP(hipMalloc(&e->d_tp, sizeof(TypDev) * kMaxTypical * (size_t)n_replicas));
  KSIM_HIP(hipMalloc(&e->d_acc, sizeof(Accum) * (size_t)n_replicas));
  KSIM_HIP(hipMalloc(&e->d_reps, sizeof(ReplicaDev) * (size_t)n_replicas));
  KSIM_HIP(hipMalloc(&e->d_base, sizeof(int) * 4));
  KSIM_HIP(hipMalloc(&e->d_scratch, sizeof(int) * 4));
  KSIM_HIP(hipMalloc(&e->d_pod, sizeof(PodDev)));
  KSIM_HIP(hipMalloc(&e->d_res1, sizeof(ResultDev)));
  KSIM_HIP(hipMalloc(&e->d_feas, (size_t)n_nodes));
  KSIM_HIP(hipMalloc(&e->d_score, sizeof(int32_t) * n_nodes));
  KSIM_HIP(hipMalloc(&e->d_gpu, sizeof(int32_t) * n_nodes));
  KSIM_HIP(hipMalloc(&e->d_gran, sizeof(unsigned long long) * (size_t)n_replicas * 2 * ksim_replay::kMaxK *
                                     ksim_replay::kGranW));
  KSIM_HIP(hipMalloc(&e->d_fail, sizeof(int)));
  KSIM_HIP(hipMalloc(&e->d_replist, sizeof(int) * (size_t)n_replicas));
  KSIM_HIP(hipMalloc(&e->d_cap, sizeof(int32_t) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMalloc(&e->d_mcap, sizeof(int32_t) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMalloc(&e->d_pw, sizeof(PowerDev) * (size_t)n_replicas));
  KSIM_HIP(hipMalloc(&e->d_cpum, (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMalloc(&e->d_pws, sizeof(int2) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMemset(e->d_pw, 0, sizeof(PowerDev) * (size_t)n_replicas));
  KSIM_HIP(hipMemset(e->d_cpum, 0, (size_t)n_nodes * n_replicas));
  e->pw_set.assign(n_replicas, 0);
  KSIM_HIP(hipMalloc(&e->d_last, sizeof(int32_t) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMemset(e->d_cap, 0, sizeof(int32_t) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMemset(e->d_mcap, 0, sizeof(int32_t) * (size_t)n_nodes * n_replicas));
  KSIM_HIP(hipMemset(e->d_tags, 0, sizeof(uint16_t) * e->tags_stride * n_replicas));
  std::vector<Accum> acc(n_replicas);
  for (auto& a : acc) {
    std::memset(&a, 0, sizeof a);
    a.lo = 0x7fffffff;
    a.hi = -1;
  }
  KSIM_HIP(hipMemcpy(e->d_acc, acc.data(), sizeof(Accum) * n_replicas, hipMemcpyHostToDevice));
  e->reps.resize(n_replicas);
  e->h_nodes.resize(n_replicas);
  e->h_rec.resize(n_replicas);
  e->d_ev.assign(n_replicas, nullptr);
  e->d_res.assign(n_replicas, nullptr);
  e->n_events.assign(n_replicas, 0);
  e->has_delete.assign(n_replicas, 0);
  e->wgs_hint.assign(n_replicas, 0);
  e->go_state.assign(n_replicas, {});
  e->h_cls.resize(n_replicas);
  e->h_tp.resize(n_replicas);
  e->h_cls_n.resize(n_replicas);
  e->h_ev_cls.resize(n_replicas);
  e->nt.assign(n_replicas, 0);
  e->d_snap.assign(n_replicas, nullptr);
  e->d_prev.assign(n_replicas, nullptr);
  e->d_rep.assign(n_replicas, nullptr);
  e->total_gpus.assign(n_replicas, 0);
  for (int r = 0; r < n_replicas; ++r) {
    ReplicaDev& rp = e->reps[r];
    std::memset(&rp, 0, sizeof rp);
    rp.policy = POL_FGD;
    rp.gpusel = SEL_FGD;
    rp.tp = e->d_tp + (size_t)r * kMaxTypical;
    rp.nodes = e->d_nodes + (size_t)r * n_nodes;
    rp.n_local = n_nodes;
    rp.tags = e->d_tags + (size_t)r * e->tags_stride;
    rp.cap = e->d_cap + (size_t)r * n_nodes;
    rp.mcap = e->d_mcap + (size_t)r * n_nodes;
    rp.init = e->d_nodes_init + (size_t)r * n_nodes;
    rp.last = e->d_last + (size_t)r * n_nodes;
    rp.pw = e->d_pw + r;
    rp.cpum = e->d_cpum + (size_t)r * n_nodes;
    rp.pws = e->d_pws + (size_t)r * n_nodes;
    rp.w_pwr = 1000;
  }
  KSIM_HIP(hipEventCreate(&e->ev0));
  KSIM_HIP(hipEventCreate(&e->ev1));
  KSIM_HIP(hipEventCreate(&e->ev_mid));
  rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  *out = e;
  return KSIM_OK;
}

void ksim_engine_destroy(ksim_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  // drain every stream the engine launched on before anything they use is freed or destroyed: no
  // dispatch (or a profiler's completion callback on it) may outlive its buffers, streams or graph
  for (int i = 0; i < ksim_engine::kSide; ++i)
    if (e->side[i]) (void)hipStreamSynchronize(e->side[i]);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->graph) (void)hipGraphExecDestroy(e->graph);
  for (auto p : e->d_ev) (void)hipFree(p);
  for (auto p : e->d_res) (void)hipFree(p);
  for (auto p : e->d_snap) (void)hipFree(p);
  for (auto p : e->d_prev) (void)hipFree(p);
  for (auto p : e->d_rep) (void)hipFree(p);
  void* bufs[] = {e->d_nodes, e->d_tags, e->d_nodes_init, e->d_tags_init, e->d_tp, e->d_acc, e->d_reps, e->d_base, e->d_scratch,
                  e->d_pod, e->d_res1, e->d_feas, e->d_score, e->d_gpu, e->d_gran, e->d_hist, e->d_fail, e->d_prof, e->d_replist,
                  e->d_cap, e->d_mcap, e->d_last, e->d_send, e->d_recv, e->d_ptrs, e->d_m_pod, e->d_m_owner, e->d_m_wgcls,
                  e->d_m_wgref, e->d_m_wggrp, e->d_win, e->d_m_evo, e->d_th, e->d_pw, e->d_cpum, e->d_pws,
                  e->d_m_evcls, e->d_topg, e->d_m_hkeys, e->d_m_wgmap, e->d_h_cg, e->d_h_cls, e->d_h_cgrp, e->d_h_gpod, e->d_h_evc, e->d_h_st,
                  e->d_h_ns, e->d_h_nstate, e->d_h_gsc, e->d_h_mtoff, e->d_h_mtab, e->d_h_na, e->d_h_keys, e->d_h_l1, e->d_h_l2, e->d_h_cnt, e->d_h_prof,
                  e->d_h_hist, e->d_go, e->d_ggran, e->d_hgargs, e->d_rgran, e->d_rgreps, e->d_rglist, e->d_done, e->d_ragg};
  for (void* p : bufs) (void)hipFree(p);
  for (int i = 0; i < ksim_engine::kSide; ++i) {
    if (e->side[i]) (void)hipStreamDestroy(e->side[i]);
    if (e->side_ev[i]) (void)hipEventDestroy(e->side_ev[i]);
    if (e->tev_side[i]) (void)hipEventDestroy(e->tev_side[i]);
  }
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_ovl) (void)hipEventDestroy(e->ev_ovl);
  if (e->ev0) (void)hipEventDestroy(e->ev0);
  if (e->ev1) (void)hipEventDestroy(e->ev1);
  if (e->ev_mid) (void)hipEventDestroy(e->ev_mid);
  if (e->comm) destroy_comm(e->comm);
  for (size_t q = 0; q < e->peers.size(); ++q)
    if (e->peer_opened[q]) (void)hipIpcCloseMemHandle(e->peers[q]);
  if (e->d_pgran) (void)hipFree(e->d_pgran);
  if (e->tev_fork) (void)hipEventDestroy(e->tev_fork);
  for (hipEvent_t v : e->grp_rev) (void)hipEventDestroy(v);
  if (e->h_started) (void)hipHostFree(e->h_started);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e->mplan;
  delete e->hplan;
  delete e;
}

static int to_pod_dev(const ksim_pod& s, PodDev* d) {
  if (s.gpu_milli < 0 || s.gpu_milli > kMilli || s.gpu_count < 0 || s.gpu_count > kMaxGpu) return KSIM_ERANGE;
  if (s.cpu_milli < 0 || s.cpu_milli > 0x3fffffff || s.cpu_nz_milli < 0 || s.cpu_nz_milli > 0x3fffffff ||
      s.mem_mib < 0 || s.mem_mib > 0x3fffffff)
    return KSIM_ERANGE;
  std::memset(d, 0, sizeof *d);
  d->cpu_req = (int32_t)s.cpu_milli;
  d->cpu_nz = (int32_t)s.cpu_nz_milli;
  d->mem = (int32_t)s.mem_mib;
  d->milli = (int16_t)s.gpu_milli;
  d->num = (int8_t)s.gpu_count;
  // GetGpuAffinityFromPodAnnotation (open-gpu-share/utils/pod.go:111-123)
  if (s.gpu_count == 0) d->tag = -1;
  else if (s.gpu_count == 1 && s.gpu_milli < kMilli) d->tag = 0;
  else if (s.gpu_milli == kMilli) d->tag = (int8_t)s.gpu_count;
  else d->tag = -2;
  d->tmask = s.type_mask;
  d->ref = s.ref;
  d->flags = s.is_delete ? kPodDelete : 0u;
  return KSIM_OK;
}

int ksim_engine_set_nodes(ksim_engine* e, int replica, const ksim_node* nodes) {
  if (!e || !nodes || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  std::vector<NodeRec> h(e->N);
  std::vector<int32_t> cap(e->N), mcap(e->N);
  std::vector<uint8_t> cpum(e->N);
  int64_t gpus = 0;
  std::vector<uint16_t> tags(e->tags_stride, 0);
  int* rank2idx = reinterpret_cast<int*>(tags.data() + (size_t)e->N * kTagStride);
  std::vector<char> seen(e->N, 0);
  for (int i = 0; i < e->N; ++i) {
    const ksim_node& s = nodes[i];
    if (s.gpu_count < 0 || s.gpu_count > kMaxGpu || s.gpu_type < 0 || s.gpu_type >= KSIM_MAX_TYPES)
      return KSIM_ERANGE;
    // sharded cluster: ranks are global and shard-contiguous (local node i has rank node_off + i)
    if (e->shard_world > 0 && s.name_rank != (uint32_t)(e->node_off + i)) return KSIM_EINVAL;
    const uint32_t lr = s.name_rank - (uint32_t)e->node_off;
    if (lr >= (uint32_t)e->N || seen[lr]) return KSIM_EINVAL;
    if (s.cpu_alloc_milli < 0 || s.cpu_alloc_milli > 0x3fffffff) return KSIM_ERANGE;
    cap[i] = (int32_t)s.cpu_alloc_milli;
    if (s.mem_alloc_mib < 0 || s.mem_alloc_mib > 0x3fffffff) return KSIM_ERANGE;
    mcap[i] = (int32_t)s.mem_alloc_mib;
    if (s.cpu_model < 0 || s.cpu_model >= kMaxCpuModels) return KSIM_ERANGE;
    cpum[i] = (uint8_t)s.cpu_model;
    gpus += s.gpu_count;
    seen[lr] = 1;
    const int64_t cpu_left = s.cpu_alloc_milli - s.cpu_used_milli;
    const int64_t mem_left = s.mem_alloc_mib - s.mem_used_mib;
    const int64_t pods_left = (int64_t)s.pods_alloc - s.pods_used;
    if (cpu_left < -0x3fffffff || cpu_left > 0x3fffffff || mem_left < -0x3fffffff || mem_left > 0x3fffffff ||
        pods_left > 32767 || pods_left < -32768)
      return KSIM_ERANGE;
    NodeRec& n = h[i];
    std::memset(&n, 0, sizeof n);
    n.cpu_left = (int32_t)cpu_left;
    n.mem_left = (int32_t)mem_left;
    n.pods_left = (int16_t)pods_left;
    n.gpu_cnt = (uint8_t)s.gpu_count;
    n.gpu_type = (uint8_t)s.gpu_type;
    n.name_rank = s.name_rank;
    for (int g = 0; g < kMaxGpu; ++g) {
      const int left = g < s.gpu_count ? kMilli - s.gpu_used_milli[g] : 0;
      if (left < 0 || left > kMilli) return KSIM_ERANGE;
      n.gl[g] = (uint16_t)left;
    }
    for (int k = 0; k < kNumTags; ++k) tags[(size_t)i * kTagStride + k] = (uint16_t)s.tag_count[k];
    rank2idx[lr] = i;
  }
  e->h_nodes[replica].assign(nodes, nodes + e->N);
  e->h_rec[replica] = h;
  e->mplan_dirty = true;  // k_hmemo's plan holds the distinct initial node states
  e->total_gpus[replica] = gpus;
  KSIM_HIP(hipSetDevice(e->device));
  KSIM_HIP(hipMemcpyAsync(e->d_cap + (size_t)replica * e->N, cap.data(), sizeof(int32_t) * e->N, hipMemcpyHostToDevice,
                          e->stream));
  KSIM_HIP(hipMemcpyAsync(e->d_mcap + (size_t)replica * e->N, mcap.data(), sizeof(int32_t) * e->N, hipMemcpyHostToDevice,
                          e->stream));
  KSIM_HIP(hipMemcpyAsync(e->d_cpum + (size_t)replica * e->N, cpum.data(), e->N, hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipMemcpyAsync(e->reps[replica].nodes, h.data(), sizeof(NodeRec) * e->N, hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipMemcpyAsync(e->d_tags + (size_t)replica * e->tags_stride, tags.data(), sizeof(uint16_t) * e->tags_stride,
                          hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipMemcpyAsync(e->d_nodes_init + (size_t)replica * e->N, h.data(), sizeof(NodeRec) * e->N,
                          hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipMemcpyAsync(e->d_tags_init + (size_t)replica * e->tags_stride, tags.data(),
                          sizeof(uint16_t) * e->tags_stride, hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_set_typical(ksim_engine* e, int replica, const ksim_typical* tp, int n) {
  if (!e || replica < 0 || replica >= e->R || n < 0 || (n > 0 && !tp)) return KSIM_EINVAL;
  std::vector<TypDev> cpu, gpu;
  bool typed = false;
  for (int i = 0; i < n; ++i) {
    // frag.go:154-158: entries with freq outside [0,1] are skipped
    if (tp[i].freq < 0 || tp[i].freq > 1 || tp[i].freq != tp[i].freq) continue;
    if (tp[i].gpu_milli < 0 || tp[i].gpu_milli > 0x7fff || tp[i].cpu_milli > 0x3fffffff || tp[i].cpu_milli < -0x3fffffff)
      return KSIM_ERANGE;
    TypDev d;
    std::memset(&d, 0, sizeof d);
    d.cpu = (int32_t)tp[i].cpu_milli;
    d.milli = tp[i].gpu_milli;
    d.num_eff = std::max(tp[i].gpu_count, 1);
    d.tmask = tp[i].type_mask;
    d.freq = tp[i].freq;
    if (d.milli == 0) {
      cpu.push_back(d);  // XL/XR bins only (frag.go:463-469)
    } else {
      typed |= d.tmask != KSIM_TYPE_ANY;
      gpu.push_back(d);
    }
  }
  std::vector<TypDev> h(cpu);
  h.insert(h.end(), gpu.begin(), gpu.end());
  if ((int)h.size() > kMaxTypical) return KSIM_ERANGE;
  KSIM_HIP(hipSetDevice(e->device));
  if (!h.empty())
    KSIM_HIP(hipMemcpyAsync(e->d_tp + (size_t)replica * kMaxTypical, h.data(), sizeof(TypDev) * h.size(),
                            hipMemcpyHostToDevice, e->stream));
  e->reps[replica].nt = (int)h.size();
  e->reps[replica].ncpu = (int)cpu.size();
  e->reps[replica].typed = typed ? 1 : 0;
  e->h_tp[replica] = h;
  e->mplan_dirty = true;  // k_hmemo's plan holds per-model views of the table
  int rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_set_policy(ksim_engine* e, int replica, int policy, int gpusel, uint64_t seed) {
  if (e) e->mplan_dirty = true;
  if (!e || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  if (policy < POL_FGD || policy > POL_PWR_FGD || gpusel < SEL_BEST || gpusel > SEL_DOTPROD) return KSIM_ENOTSUP;
  // allocateGpuIdFunc only holds the selectors of the enabled plugins (fgd_score.go:37, pwr_score.go:40,
  // dot_product_score.go:37)
  if (gpusel == SEL_PWR && !is_pwr_policy(policy)) return KSIM_ENOTSUP;
  if (gpusel == SEL_DOTPROD && policy != POL_DOTPROD) return KSIM_ENOTSUP;
  if (policy == POL_PWR_FGD && e->reps[replica].policy != POL_PWR_FGD) {
    e->reps[replica].w_pwr = 500;  // "PWR 500 FGD 500" (generate_run_scripts.py:40) until set_weights
    e->reps[replica].w_fgd = 500;
  } else if (policy == POL_PWR) {
    e->reps[replica].w_pwr = 1000;
    e->reps[replica].w_fgd = 0;
  }
  e->reps[replica].policy = policy;
  e->reps[replica].gpusel = gpusel;
  e->reps[replica].seed = seed;
  KSIM_HIP(hipSetDevice(e->device));
  int rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_set_replica_wgs(ksim_engine* e, int replica, int wgs) {
  if (!e || replica < 0 || replica >= e->R || wgs < 0 || wgs > 64) return KSIM_EINVAL;
  e->wgs_hint[replica] = wgs;
  e->mplan_dirty = true;
  return KSIM_OK;
}

int ksim_engine_set_plugin_cfg(ksim_engine* e, int replica, int dim_ext, int norm) {
  if (!e || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  if (dim_ext < DIM_MERGE || dim_ext > DIM_EXTEND || norm < NORM_MAX || norm > NORM_POD) return KSIM_ENOTSUP;
  e->reps[replica].dpcfg = dim_ext | norm << 4;
  KSIM_HIP(hipSetDevice(e->device));
  int rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_set_go_stream(ksim_engine* e, int replica, const uint64_t* vec, int tap, int feed) {
  if (!e || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  if (!vec) {
    e->go_state[replica].clear();
    return KSIM_OK;
  }
  if (tap < 0 || tap >= ksim_random_go::kLen || feed < 0 || feed >= ksim_random_go::kLen) return KSIM_EINVAL;
  std::vector<unsigned long long>& s = e->go_state[replica];
  s.assign(vec, vec + ksim_random_go::kLen);
  s.push_back((unsigned long long)tap);
  s.push_back((unsigned long long)feed);
  return KSIM_OK;
}

// Replicas replaying the Random draw structure on Go's stream (k_random_go): policy Random with a
// source state set.
static bool go_random(const ksim_engine* e, int r) {
  return e->reps[r].policy == POL_RANDOM && !e->go_state[r].empty();
}

int ksim_engine_set_weights(ksim_engine* e, int replica, int32_t w_pwr, int32_t w_fgd) {
  if (!e || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  if (e->reps[replica].policy != POL_PWR_FGD) return KSIM_ESTATE;
  // framework weights are positive; the packed key holds w_pwr * 100 + w_fgd * 100 in 24 bits
  if (w_pwr <= 0 || w_fgd <= 0 || w_pwr > 50000 || w_fgd > 50000) return KSIM_ERANGE;
  e->reps[replica].w_pwr = w_pwr;
  e->reps[replica].w_fgd = w_fgd;
  KSIM_HIP(hipSetDevice(e->device));
  int rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_set_power_model(ksim_engine* e, int replica, const ksim_power_model* pm) {
  static_assert(sizeof(ksim_power_model) == sizeof(PowerDev), "ksim_power_model layout");
  if (!e || !pm || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  for (int c = 0; c < kMaxCpuModels; ++c)
    if (((pm->cpu_valid >> c) & 1u) && !(pm->cpu_cores[c] > 0)) return KSIM_ERANGE;
  KSIM_HIP(hipSetDevice(e->device));
  KSIM_HIP(hipMemcpyAsync(e->d_pw + replica, pm, sizeof(PowerDev), hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  e->pw_set[replica] = 1;
  e->reps[replica].has_pw = 1;
  int rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

static bool any_pwr(const ksim_engine* e) {
  for (int r = 0; r < e->R; ++r)
    if (is_pwr_policy(e->reps[r].policy)) return true;
  return false;
}

static StepArgs base_args(ksim_engine* e) {
  StepArgs a;
  std::memset(&a, 0, sizeof a);
  a.reps = e->d_reps;
  a.acc = e->d_acc;
  a.N = e->N;
  a.NB = e->NB;
  a.bpr = e->bpr;
  return a;
}

int ksim_engine_filter_score(ksim_engine* e, int replica, const ksim_pod* pod, int32_t step, uint8_t* feasible,
                             int32_t* score, int32_t* gpu_mask) {
  if (!e || !pod || replica < 0 || replica >= e->R || !feasible || !score || !gpu_mask) return KSIM_EINVAL;
  PodDev p;
  int rc = to_pod_dev(*pod, &p);
  if (rc) return rc;
  if (p.flags & kPodDelete) return KSIM_EINVAL;
  // one plugin's Score per call: a weighted combination has two (query PWR and FGD replicas)
  if (e->reps[replica].policy == POL_PWR_FGD) return KSIM_ENOTSUP;
  if (is_pwr_policy(e->reps[replica].policy) && !e->pw_set[replica]) return KSIM_ESTATE;
  KSIM_HIP(hipSetDevice(e->device));
  KSIM_HIP(hipMemcpyAsync(e->d_pod, &p, sizeof p, hipMemcpyHostToDevice, e->stream));
  StepArgs a = base_args(e);
  a.rep_first = replica;
  a.step_off = step;
  a.pod_override = e->d_pod;
  a.res_override = e->d_res1;
  a.mode = 1;
  a.out_feas = e->d_feas;
  a.out_score = e->d_score;
  a.out_gpu = e->d_gpu;
  hipLaunchKernelGGL(k_step, dim3(e->bpr), dim3(kBlock), 0, e->stream, a, (const TypDev*)e->d_tp);
  KSIM_HIP(hipGetLastError());
  KSIM_HIP(hipMemcpyAsync(feasible, e->d_feas, e->N, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipMemcpyAsync(score, e->d_score, sizeof(int32_t) * e->N, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipMemcpyAsync(gpu_mask, e->d_gpu, sizeof(int32_t) * e->N, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_schedule(ksim_engine* e, int replica, const ksim_pod* pod, int32_t step, ksim_result* out) {
  if (!e || !pod || !out || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  PodDev p;
  int rc = to_pod_dev(*pod, &p);
  if (rc) return rc;
  if (p.flags & kPodDelete) return KSIM_EINVAL;  // deletions go through ksim_engine_unreserve
  KSIM_HIP(hipSetDevice(e->device));
  KSIM_HIP(hipMemcpyAsync(e->d_pod, &p, sizeof p, hipMemcpyHostToDevice, e->stream));
  StepArgs a = base_args(e);
  a.rep_first = replica;
  a.step_off = step;
  a.pod_override = e->d_pod;
  a.res_override = e->d_res1;
  a.mode = 0;
  if (is_pwr_policy(e->reps[replica].policy) && !e->pw_set[replica]) return KSIM_ESTATE;
  hipLaunchKernelGGL(k_step, dim3(e->bpr), dim3(kBlock), 0, e->stream, a, (const TypDev*)e->d_tp);
  if (is_pwr_policy(e->reps[replica].policy))
    hipLaunchKernelGGL(k_step_pwr, dim3(e->bpr), dim3(kBlock), 0, e->stream, a);
  KSIM_HIP(hipGetLastError());
  ResultDev r;
  KSIM_HIP(hipMemcpyAsync(&r, e->d_res1, sizeof r, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  std::memcpy(out, &r, sizeof r);
  return KSIM_OK;
}

int ksim_engine_reserve(ksim_engine* e, int replica, const ksim_pod* pod, int node, int32_t step, int32_t* gpu_mask_out) {
  if (!e || !pod || !gpu_mask_out || replica < 0 || replica >= e->R || node < 0 || node >= e->N) return KSIM_EINVAL;
  PodDev p;
  int rc = to_pod_dev(*pod, &p);
  if (rc) return rc;
  KSIM_HIP(hipSetDevice(e->device));
  hipLaunchKernelGGL(k_reserve, dim3(1), dim3(64), 0, e->stream, e->d_reps, (const TypDev*)e->d_tp, replica, p, node, step, e->d_scratch, +1, -1);
  KSIM_HIP(hipGetLastError());
  int m = 0;
  KSIM_HIP(hipMemcpyAsync(&m, e->d_scratch, sizeof m, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  *gpu_mask_out = m;
  return m < 0 ? KSIM_ESTATE : KSIM_OK;
}

int ksim_engine_unreserve(ksim_engine* e, int replica, const ksim_pod* pod, int node, int32_t gpu_mask) {
  if (!e || !pod || replica < 0 || replica >= e->R || node < 0 || node >= e->N) return KSIM_EINVAL;
  PodDev p;
  int rc = to_pod_dev(*pod, &p);
  if (rc) return rc;
  if (p.flags & kPodDelete) return KSIM_EINVAL;
  // the devices a Reserve of this pod can have assigned on this node (open_gpu_share.go:242-283): none
  // for a pod without GPU milli, else `num` devices the node has
  if (e->h_nodes[replica].size() != (size_t)e->N) return KSIM_ESTATE;
  const int cnt = e->h_nodes[replica][node].gpu_count;
  if (gpu_mask < 0 || gpu_mask >= (1 << cnt)) return KSIM_EINVAL;
  if ((p.milli == 0) != (gpu_mask == 0)) return KSIM_EINVAL;
  if (p.milli > 0 && __builtin_popcount((unsigned)gpu_mask) != p.num) return KSIM_EINVAL;
  KSIM_HIP(hipSetDevice(e->device));
  hipLaunchKernelGGL(k_reserve, dim3(1), dim3(64), 0, e->stream, e->d_reps, (const TypDev*)e->d_tp, replica, p, node, 0, e->d_scratch, -1,
                     (int)gpu_mask);
  KSIM_HIP(hipGetLastError());
  int m = 0;
  KSIM_HIP(hipMemcpyAsync(&m, e->d_scratch, sizeof m, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return m < 0 ? KSIM_ESTATE : KSIM_OK;  // the node does not hold what the pod would release
}

int ksim_engine_bind(ksim_engine* e, int replica, const ksim_pod* pod, int node, int32_t gpu_mask) {
  if (!e || !pod || replica < 0 || replica >= e->R || node < 0 || node >= e->N) return KSIM_EINVAL;
  PodDev p;
  int rc = to_pod_dev(*pod, &p);
  if (rc) return rc;
  if (p.flags & kPodDelete) return KSIM_EINVAL;
  if (e->h_nodes[replica].size() != (size_t)e->N) return KSIM_ESTATE;
  const int cnt = e->h_nodes[replica][node].gpu_count;
  if (gpu_mask < 0 || gpu_mask >= (1 << cnt)) return KSIM_EINVAL;
  if ((p.milli == 0) != (gpu_mask == 0)) return KSIM_EINVAL;
  if (p.milli > 0 && __builtin_popcount((unsigned)gpu_mask) != p.num) return KSIM_EINVAL;
  KSIM_HIP(hipSetDevice(e->device));
  hipLaunchKernelGGL(k_reserve, dim3(1), dim3(64), 0, e->stream, e->d_reps, (const TypDev*)e->d_tp, replica, p, node, 0,
                     e->d_scratch, +1, (int)gpu_mask);
  KSIM_HIP(hipGetLastError());
  int m = 0;
  KSIM_HIP(hipMemcpyAsync(&m, e->d_scratch, sizeof m, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return m < 0 ? KSIM_ESTATE : KSIM_OK;  // a named device lacks the milli (the reference panics)
}

int ksim_engine_load_events(ksim_engine* e, int replica, const ksim_pod* events, int n) {
  if (e) e->mplan_dirty = true;
  if (!e || replica < 0 || replica >= e->R || n < 0 || (n > 0 && !events)) return KSIM_EINVAL;
  std::vector<PodDev> h(n);
  std::vector<char> gone(std::max(n, 1), 0);  // creations already deleted (the reference deletes a pod once)
  for (int i = 0; i < n; ++i) {
    int rc = to_pod_dev(events[i], &h[i]);
    if (rc) return rc;
    if (h[i].flags & kPodDelete) {
      const int ref = h[i].ref;
      if (ref < 0 || ref >= i || (h[ref].flags & kPodDelete) || gone[ref]) return KSIM_EINVAL;
      gone[ref] = 1;
    }
  }
  // pod classes for k_memo: the distinct Filter + Score requests of the creation events
  {
    std::vector<PodDev>& cls = e->h_cls[replica];
    std::vector<int>& cn = e->h_cls_n[replica];
    cls.clear();
    cn.clear();
    std::vector<std::pair<std::vector<int32_t>, int>> seen;  // small: linear probe by sorted insert
    auto key_of = [](const PodDev& q) {
      return std::vector<int32_t>{q.cpu_req, q.cpu_nz, q.mem, q.milli, q.num, (int32_t)q.tmask};
    };
    for (int i = 0; i < n; ++i) {
      if (h[i].flags & kPodDelete) { h[i].pad = -1; continue; }
      const std::vector<int32_t> k = key_of(h[i]);
      auto it = std::lower_bound(seen.begin(), seen.end(), k,
                                 [](const std::pair<std::vector<int32_t>, int>& a, const std::vector<int32_t>& b) {
                                   return a.first < b;
                                 });
      int id;
      if (it != seen.end() && it->first == k) {
        id = it->second;
      } else {
        id = (int)cls.size();
        seen.insert(it, {k, id});
        cls.push_back(h[i]);
        cls.back().pad = id;
        cn.push_back(0);
      }
      h[i].pad = id;
      ++cn[id];
    }
    e->h_ev_cls[replica].resize(n);
    for (int i = 0; i < n; ++i) e->h_ev_cls[replica][i] = h[i].pad;
  }
  KSIM_HIP(hipSetDevice(e->device));
  if (e->d_ev[replica]) { KSIM_HIP(hipFree(e->d_ev[replica])); e->d_ev[replica] = nullptr; }
  if (e->d_res[replica]) { KSIM_HIP(hipFree(e->d_res[replica])); e->d_res[replica] = nullptr; }
  const size_t ne = (size_t)std::max(n, 1);
  KSIM_HIP(hipMalloc(&e->d_ev[replica], sizeof(PodDev) * ne));
  KSIM_HIP(hipMalloc(&e->d_res[replica], sizeof(ResultDev) * ne));
  if (n > 0) KSIM_HIP(hipMemcpyAsync(e->d_ev[replica], h.data(), sizeof(PodDev) * n, hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipMemsetAsync(e->d_res[replica], 0xff, sizeof(ResultDev) * ne, e->stream));
  e->n_events[replica] = n;
  e->has_delete[replica] = false;
  for (int i = 0; i < n; ++i) e->has_delete[replica] = e->has_delete[replica] || events[i].is_delete;
  e->reps[replica].ev = e->d_ev[replica];
  e->reps[replica].res = e->d_res[replica];
  e->reps[replica].n_events = n;
  int rc = alloc_report(e, replica);
  if (rc) return rc;
  rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

// Every replica back to the cluster state given to set_nodes (device-to-device).
static int reset_state(ksim_engine* e) {
  KSIM_HIP(hipMemcpyAsync(e->d_nodes, e->d_nodes_init, sizeof(NodeRec) * (size_t)e->N * e->R, hipMemcpyDeviceToDevice,
                          e->stream));
  KSIM_HIP(hipMemcpyAsync(e->d_tags, e->d_tags_init, sizeof(uint16_t) * e->tags_stride * e->R, hipMemcpyDeviceToDevice,
                          e->stream));
  return KSIM_OK;
}

// Per-event report buffers of one replica (allocated while the report is enabled).
static int alloc_report(ksim_engine* e, int r) {
  ReplicaDev& rp = e->reps[r];
  if (e->d_snap[r]) { KSIM_HIP(hipFree(e->d_snap[r])); e->d_snap[r] = nullptr; }
  if (e->d_prev[r]) { KSIM_HIP(hipFree(e->d_prev[r])); e->d_prev[r] = nullptr; }
  if (e->d_rep[r]) { KSIM_HIP(hipFree(e->d_rep[r])); e->d_rep[r] = nullptr; }
  rp.snap = nullptr;
  rp.prev = nullptr;
  rp.rep = nullptr;
  if (!e->report || !e->d_ev[r]) return KSIM_OK;
  const size_t ne = (size_t)std::max(e->n_events[r], 1);
  KSIM_HIP(hipMalloc(&e->d_snap[r], sizeof(NodeRec) * ne));
  KSIM_HIP(hipMalloc(&e->d_prev[r], sizeof(int32_t) * ne));
  KSIM_HIP(hipMalloc(&e->d_rep[r], sizeof(RepAcc) * ne));
  rp.snap = e->d_snap[r];
  rp.prev = e->d_prev[r];
  rp.rep = e->d_rep[r];
  return KSIM_OK;
}

// The per-event cluster report of every replica from the run's snapshots (ksim_report.hpp).
// list (device, nullable): only these R replicas -- one concurrent group's, on its own stream behind its replay.
static int run_report(ksim_engine* e, int max_ev, hipStream_t st, const int* list, int R) {
  if (max_ev <= 0 || R <= 0) return KSIM_OK;
  const dim3 grid((unsigned)((max_ev + ksim_rep::kDeltaBlock - 1) / ksim_rep::kDeltaBlock), (unsigned)R);
  hipLaunchKernelGGL(ksim_rep::k_report_delta, grid, dim3(ksim_rep::kDeltaBlock), 0, st,
                     (const ReplicaDev*)e->d_reps, (const TypDev*)e->d_tp, list);
  KSIM_HIP(hipGetLastError());
  // the scan over B workgroups per replica when a few replicas would leave most CUs idle behind one workgroup's pass
  // (about a CU-full of workgroups, parts of >= 2048 events; KSIM_VARIANT report_parts=0: one workgroup each)
  const int B = variant("report_parts", 1) != 0
                    ? std::min({ksim_rep::kScanPartsMax, (e->cus + R - 1) / R, max_ev / 2048}) : 1;
  if (B > 1) {
    const size_t n = (size_t)e->R * ksim_rep::kScanPartsMax * 2 * ksim_rep::kFields;
    if (n > e->ragg_cap) {
      if (e->d_ragg) KSIM_HIP(hipFree(e->d_ragg));
      KSIM_HIP(hipMalloc(&e->d_ragg, sizeof(__int128) * n));
      e->ragg_cap = n;
    }
    hipLaunchKernelGGL(ksim_rep::k_report_part, dim3((unsigned)B, (unsigned)R), dim3(ksim_rep::kScanBlock), 0, st,
                       (const ReplicaDev*)e->d_reps, (const TypDev*)e->d_tp, e->N, list, e->d_ragg);
    KSIM_HIP(hipGetLastError());
    hipLaunchKernelGGL(ksim_rep::k_report_apply, dim3((unsigned)B, (unsigned)R), dim3(ksim_rep::kScanBlock), 0, st,
                       (const ReplicaDev*)e->d_reps, e->N, list, (const __int128*)e->d_ragg);
    KSIM_HIP(hipGetLastError());
    return KSIM_OK;
  }
  hipLaunchKernelGGL(ksim_rep::k_report_scan, dim3(R), dim3(ksim_rep::kScanBlock), 0, st,
                     (const ReplicaDev*)e->d_reps, (const TypDev*)e->d_tp, e->N, list);
  KSIM_HIP(hipGetLastError());
  return KSIM_OK;
}

// RCCL, loaded on first use (the node-sharded mode only): the library stays loadable without it.
struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*);
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*comm_destroy)(ncclComm_t);
  const char* (*error_string)(ncclResult_t);
};
static RcclApi* rccl() {
  static RcclApi api;
  static int state = 0;  // 0 untried, 1 ok, -1 unavailable
  if (state == 0) {
    // the RCCL beside the HIP runtime this process bound (torch's or /opt/rocm's, ksim.hip_runtime_path):
    // an RCCL from another install would NEED its own runtime and take this library's streams across
    // runtimes; the bare names last (a RUNPATH / SONAME match)
    void* h = nullptr;
    Dl_info di;
    if (dladdr((const void*)(hipError_t(*)(void**, size_t))&hipMalloc, &di) && di.dli_fname) {
      std::string dir(di.dli_fname);
      dir = dir.substr(0, dir.find_last_of('/') + 1);
      for (const char* nm : {"librccl.so.1", "librccl.so"})
        if (!h) h = dlopen((dir + nm).c_str(), RTLD_NOW | RTLD_GLOBAL);
    }
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    state = -1;
    if (h) {
      api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
      api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
      api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
      api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
      api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
      if (api.get_unique_id && api.comm_init_rank && api.all_gather && api.comm_destroy && api.error_string) state = 1;
    }
  }
  return state == 1 ? &api : nullptr;
}

static void destroy_comm(ncclComm_t c) {
  if (rccl()) (void)rccl()->comm_destroy(c);
}

// One pod step of a sharded cluster, enqueued on `st`: local Filter+Score (k_step mode 2), the
// exchange of the shard records, the cluster-wide finish on every shard (owner binds).
static int shard_local(ksim_engine* e, hipStream_t st, const int* base, int step_off) {
  StepArgs a = base_args(e);
  a.base = base;
  a.step_off = step_off;
  a.mode = 2;
  a.send = e->d_send;
  hipLaunchKernelGGL(k_step, dim3(e->bpr), dim3(kBlock), 0, st, a, (const TypDev*)e->d_tp);
  KSIM_HIP(hipGetLastError());
  return KSIM_OK;
}
static int shard_commit(ksim_engine* e, hipStream_t st, const int* base, int step_off) {
  StepArgs a = base_args(e);
  a.base = base;
  a.step_off = step_off;
  a.recv = e->d_recv;
  a.world = e->shard_world;
  hipLaunchKernelGGL(k_shard_commit, dim3(1), dim3(64), 0, st, a);
  KSIM_HIP(hipGetLastError());
  return KSIM_OK;
}
static int shard_exchange(ksim_engine* e, hipStream_t st) {
  if (e->comm) {
    const ncclResult_t r = rccl()->all_gather(e->d_send, e->d_recv, 4, ncclUint64, e->comm, st);
    if (r != ncclSuccess) {
      std::fprintf(stderr, "ksim: ncclAllGather failed: %s\n", rccl()->error_string(r));
      return KSIM_EHIP;
    }
    return KSIM_OK;
  }
  KSIM_HIP(hipMemcpyAsync(e->d_recv, e->d_send, 4 * sizeof(unsigned long long), hipMemcpyDeviceToDevice, st));
  return KSIM_OK;
}

// Sharded run over RCCL (or a world of one): steps captured K at a time into a hipGraph when the
// stream capture accepts the collective, else enqueued eagerly.
static int run_sharded(ksim_engine* e, int max_ev) {
  int rc;
  if (e->xfn) {  // host exchange: the record goes through the caller's transport, one step at a time
    const size_t rec = 4 * sizeof(unsigned long long);
    for (int s = 0; s < max_ev; ++s) {
      if ((rc = shard_local(e, e->stream, nullptr, s))) return rc;
      KSIM_HIP(hipMemcpyAsync(e->h_send.data(), e->d_send, rec, hipMemcpyDeviceToHost, e->stream));
      KSIM_HIP(hipStreamSynchronize(e->stream));
      if (e->xfn(e->h_send.data(), e->h_recv.data(), e->xuser) != 0) return KSIM_ESTATE;
      // the caller's gather must hold this shard's own record at its rank
      if (std::memcmp(e->h_recv.data() + 4 * (size_t)e->shard_rank, e->h_send.data(), rec) != 0) return KSIM_ESTATE;
      KSIM_HIP(hipMemcpyAsync(e->d_recv, e->h_recv.data(), rec * (size_t)e->shard_world, hipMemcpyHostToDevice,
                              e->stream));
      if ((rc = shard_commit(e, e->stream, nullptr, s))) return rc;
    }
    return KSIM_OK;
  }
  if (e->shard_world > 1 && !e->comm) return KSIM_ESTATE;  // in-process group: ksim_shard_group_run
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  const int K = std::min(e->K, std::max(max_ev, 1));
  if (hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal) == hipSuccess) {
    bool ok = true;
    for (int i = 0; i < K && ok; ++i)
      ok = shard_local(e, e->stream, e->d_base, i) == KSIM_OK && shard_exchange(e, e->stream) == KSIM_OK &&
           shard_commit(e, e->stream, e->d_base, i) == KSIM_OK;
    if (ok) hipLaunchKernelGGL(k_advance, dim3(1), dim3(1), 0, e->stream, e->d_base, K);
    const hipError_t ce = hipStreamEndCapture(e->stream, &g);
    if (ok && ce == hipSuccess && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) ge = nullptr;
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
  }
  if (ge) {
    KSIM_HIP(hipMemsetAsync(e->d_base, 0, sizeof(int), e->stream));
    for (int s0 = 0; s0 < max_ev; s0 += K) {
      if (hipGraphLaunch(ge, e->stream) != hipSuccess) { (void)hipGraphExecDestroy(ge); return KSIM_EHIP; }
    }
    (void)hipGraphExecDestroy(ge);
    return KSIM_OK;
  }
  for (int s = 0; s < max_ev; ++s) {
    if ((rc = shard_local(e, e->stream, nullptr, s))) return rc;
    if ((rc = shard_exchange(e, e->stream))) return rc;
    if ((rc = shard_commit(e, e->stream, nullptr, s))) return rc;
  }
  return KSIM_OK;
}

static int build_graph(ksim_engine* e) {
  const bool pwr = any_pwr(e);
  if (e->graph && e->graph_R == e->R && e->graph_pwr == pwr) return KSIM_OK;
  if (e->graph) { (void)hipGraphExecDestroy(e->graph); e->graph = nullptr; }
  hipGraph_t g;
  KSIM_HIP(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
  StepArgs a = base_args(e);
  a.rep_first = 0;
  a.base = e->d_base;
  for (int i = 0; i < e->K; ++i) {
    a.step_off = i;
    hipLaunchKernelGGL(k_step, dim3(e->bpr * e->R), dim3(kBlock), 0, e->stream, a, (const TypDev*)e->d_tp);
    if (pwr) hipLaunchKernelGGL(k_step_pwr, dim3(e->bpr * e->R), dim3(kBlock), 0, e->stream, a);
  }
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(1), 0, e->stream, e->d_base, e->K);
  KSIM_HIP(hipStreamEndCapture(e->stream, &g));
  KSIM_HIP(hipGraphInstantiate(&e->graph, g, nullptr, nullptr, 0));
  KSIM_HIP(hipGraphDestroy(g));
  e->graph_R = e->R;
  e->graph_pwr = pwr;
  return KSIM_OK;
}

// KSIM_PROFILE=1: per-phase k_replay time (us per step, mean and max over workgroups) on stderr.
static void print_replay_profile(ksim_engine* e, int R, int K, int steps) {
  const int nb = R * K, P = ksim_replay::kProfPhases;
  std::vector<unsigned long long> h((size_t)nb * P);
  if (hipMemcpy(h.data(), e->d_prof, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
  static const char* names[] = {"pod", "filter(+emit)", "fgd-eval", "fgd-final", "agg-sync", "poll", "commit+publish", "end-sync"};
  std::fprintf(stderr, "ksim profile: %d workgroups (K=%d), %d steps, us/step mean [max]:", nb, K, steps);
  for (int ph = 0; ph < 8; ++ph) {
    double sum = 0, mx = 0;
    for (int b = 0; b < nb; ++b) {
      const double us = (double)h[(size_t)b * P + ph] / 100.0 / steps;  // 100 MHz ticks
      sum += us;
      mx = std::max(mx, us);
    }
    std::fprintf(stderr, " %s %.3f [%.3f];", names[ph], sum / nb, mx);
  }
  double spins = 0;
  for (int b = 0; b < nb; ++b) spins += (double)h[(size_t)b * P + 8];
  std::fprintf(stderr, " poll spins/step %.2f", spins / nb / steps);
  double miss = 0, redo = 0;  // PWR+FGD: guessed-range misses (every workgroup alike), re-evaluations
  for (int b = 0; b < nb; ++b) {
    miss += (double)(h[(size_t)b * P + 9] & 0xffffffffull);
    redo += (double)(h[(size_t)b * P + 9] >> 32);
  }
  if (miss + redo > 0) std::fprintf(stderr, " pf misses/step %.4f re-evaluations/step %.4f", miss / nb / steps, redo / nb / steps * K);
  double cyc = 0, tick = 0;
  for (int b = 0; b < nb; ++b) { cyc += (double)h[(size_t)b * P + 10]; tick += (double)h[(size_t)b * P + 11]; }
  if (tick > 0) std::fprintf(stderr, " shader clock %.0f MHz", cyc / tick * 100.0);
  std::fprintf(stderr, "\n");
}

// Workgroups per replica for k_replay: every workgroup of a launch must be
// co-resident (they exchange granules every step), so R*K never exceeds one
// workgroup per CU; K = 1 needs no co-residency at all.
static int choose_wgs(const ksim_engine* e, int R) {
  // auto: one workgroup per CU up to 64 per replica; large clusters (C5: 100k nodes) go wider
  // so that a slice stays near 384 nodes (one to two FGD evaluation rounds per step)
  int K = e->wgs_req;
  if (K <= 0) {
    K = std::min(e->cus / R, 64);
    K = std::max(K, std::min(e->cus / R, (e->N + 383) / 384));
  }
  K = std::max(1, std::min(K, ksim_replay::kMaxK));
  K = std::min(K, e->N);
  if (R * K > e->cus) K = 1;
  return K;
}

static int resident_cap(const ksim_engine* e, const void* f, size_t lds) {
  (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 1024, lds) != hipSuccess) {
    (void)hipGetLastError();
    nb = 0;
  }
  return nb * e->cus;
}

static size_t replay_lds(int S, int pol, bool general) {  // S real slots + the virtual node
  return ksim_replay::replay_layout(S, pol, general).total;
}


// The dead-class skip (k_memo, k_hmemo, k_scan1): on create-only streams a class that once found no
// feasible node never finds one again (Filter is monotone in the resources a creation takes), so its
// later events are decided without a scan.  Needs every replica create-only with class ids < 1024;
// KSIM_VARIANT=skip=0 turns it off (A/B runs).
static bool dead_skip(const ksim_engine* e, const std::vector<int>& reps) {
  if (variant("skip", 1) == 0) return false;
  for (int r : reps)
    if (e->has_delete[r] || e->h_cls[r].size() > 1024) return false;
  return true;
}

// One k_replay launch per policy present (the kernel is specialised on the policy);
// launches of different policies run back to back on the engine stream.
constexpr int kPolRandomGo = 64;  // run_persistent's group id of the k_random_go replicas
constexpr int kPolFgdH = 66;      // ... of the one-workgroup FGD replicas on k_hmemo beside wide ones on k_memo (split_fgd)

// The residency gate's host-mapped start flags: n of them, and a fresh epoch the next launch stores into them.
static int gate_flags(ksim_engine* e, int n, int** d_flags, int* epoch) {
  if (n > e->started_cap) {
    if (e->h_started) KSIM_HIP(hipHostFree(e->h_started));
    e->h_started = nullptr;
    KSIM_HIP(hipHostMalloc((void**)&e->h_started, sizeof(int) * (size_t)n, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(e->h_started, 0, sizeof(int) * (size_t)n);
    KSIM_HIP(hipHostGetDevicePointer((void**)&e->d_started, e->h_started, 0));
    e->started_cap = n;
  }
  *d_flags = e->d_started;
  *epoch = e->gate_epoch = (e->gate_epoch % 0x3fffffff) + 1;
  return KSIM_OK;
}

// Wait until the n workgroups of the launch just made have stored `epoch` (bounded: past 2 s the gate gives up,
// counts it and says so on stderr -- it orders work, it decides nothing).
static void gate_wait(ksim_engine* e, int n, int epoch, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  volatile int* fl = e->h_started;
  if (e->last_gate == 0) e->last_gate = 1;
  for (int w = 0; w < n;) {
    if (fl[w] == epoch) { ++w; continue; }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      e->last_gate = -1;
      ++e->gate_timeouts;
      std::fprintf(stderr, "ksim: residency gate given up after 2 s (%d of %d %s workgroups started); the next "
                   "groups launch unordered\n", w, n, what);
      break;
    }
    std::this_thread::yield();
  }
}

static void note_kernel(ksim_engine* e, const char* name) {
  for (size_t p = 0; p < e->last_kernels.size();) {  // each name once
    size_t q = e->last_kernels.find('+', p);
    if (q == std::string::npos) q = e->last_kernels.size();
    if (e->last_kernels.compare(p, q - p, name) == 0) return;
    p = q + 1;
  }
  if (!e->last_kernels.empty()) e->last_kernels += '+';
  e->last_kernels += name;
}

static int run_persistent(ksim_engine* e, int max_ev) {
  std::vector<int> order;
  std::vector<std::pair<int, int>> groups;  // (policy, count) in `order`
  if (e->split_fgd) {  // the wide FGD replicas (k_memo) first, then the one-workgroup ones (k_hmemo): the plans' orders
    order = e->mplan_reps;
    order.insert(order.end(), e->hplan_reps.begin(), e->hplan_reps.end());
    groups.push_back({POL_FGD, (int)e->mplan_reps.size()});
    groups.push_back({kPolFgdH, (int)e->hplan_reps.size()});
  }
  for (int pol = e->split_fgd ? POL_BESTFIT : POL_FGD; pol <= POL_PWR_FGD; ++pol) {
    int c = 0;
    for (int r = 0; r < e->R; ++r)
      if (e->reps[r].policy == pol && !go_random(e, r)) { order.push_back(r); ++c; }
    if (c) groups.push_back({pol, c});
  }
  {  // Random on Go's stream: one k_random_go workgroup per replica, last
    int c = 0;
    for (int r = 0; r < e->R; ++r)
      if (go_random(e, r)) { order.push_back(r); ++c; }
    if (c) {
      groups.push_back({kPolRandomGo, c});
      const size_t words = (size_t)e->R * ksim_random_go::kStateWords;
      if (words > e->go_cap) {
        if (e->d_go) KSIM_HIP(hipFree(e->d_go));
        KSIM_HIP(hipMalloc(&e->d_go, sizeof(unsigned long long) * words));
        e->go_cap = words;
      }
      std::vector<unsigned long long> h(words, 0ull);
      for (int r = 0; r < e->R; ++r)
        if (go_random(e, r))
          std::copy(e->go_state[r].begin(), e->go_state[r].end(), h.begin() + (size_t)r * ksim_random_go::kStateWords);
      KSIM_HIP(hipMemcpyAsync(e->d_go, h.data(), sizeof(unsigned long long) * words, hipMemcpyHostToDevice, e->stream));
      KSIM_HIP(hipStreamSynchronize(e->stream));  // h is a local
    }
  }
  bool any_delete = false;
  for (int r = 0; r < e->R; ++r) any_delete = any_delete || e->has_delete[r];
  const char* pe = std::getenv("KSIM_PROFILE");
  const bool profile = pe && pe[0] == '1';
  int first = 0;
  e->last_memo = 0;
  e->last_hmemo = 0;
  e->last_rgo = 0;
  e->last_scan1 = 0;
  e->last_launches = (int)groups.size();
  e->last_streams = 0;
  // Groups whose replicas each fit ONE workgroup (K = 1: no cross-workgroup exchange, so no
  // co-residency needed) run concurrently on side streams: a paper-sweep group fills 170 of 256 CUs,
  // the next group's workgroups take the rest.  Any group needing K > 1 (or a k_memo launch, or the
  // profile timers) keeps the launches back to back on the engine stream.
  bool concurrent = !profile && groups.size() >= 2;
  const bool gen_any = profile || e->report || any_delete;
  for (const auto& gp : groups) {
    if (!concurrent) break;
    if (gp.first == kPolRandomGo || gp.first == kPolFgdH) continue;  // one workgroup per replica
    if (gp.first == POL_FGD && e->split_fgd) continue;  // the wide k_memo group, launched first behind its gate
    if (gp.first == POL_FGD && e->run_mode != 2 && e->mplan_ok) { concurrent = false; break; }
    if (gp.first == POL_FGD && e->run_mode != 2 && e->hplan_ok) {
      if (e->hplan->K > 1) { concurrent = false; break; }  // a co-resident wide launch
      continue;  // one workgroup per replica
    }
    int K = choose_wgs(e, gp.second);
    int S = (e->N + K - 1) / K;
    while (replay_lds(S, gp.first, gen_any) > 160 * 1024 && K < ksim_replay::kMaxK && gp.second * (K + 1) <= e->cus) {
      ++K;
      S = (e->N + K - 1) / K;
    }
    concurrent = K == 1;
  }
  // The cheap-policy groups a concurrent run would give one k_scan1 launch each become ONE k_scan1_mix
  // launch (policy per workgroup), its replicas longest stream first: the run then needs one side stream
  // beside the FGD group's, whatever the hardware-queue mapping of the process.
  const bool reg1 = e->scan1 == 2 && e->N <= ksim_scan1::kBlock * ksim_scan1::kRegSlots;
  if (concurrent && !any_delete && e->scan1 && e->N <= kMaxSlice && variant("scan1_mix", 1) != 0 &&
      ksim_scan1::scan1_lds(e->N, ksim_scan1::kPolMix, e->report, reg1) <= 160 * 1024) {
    std::vector<int> mix, norder;
    std::vector<std::pair<int, int>> ngroups;
    int f = 0, at = -1, nmix = 0;
    for (const auto& gp : groups) {
      bool m = gp.first >= POL_BESTFIT && gp.first <= POL_RANDOM;
      for (int j = f; m && j < f + gp.second; ++j)
        m = gp.first != POL_DOTPROD || e->reps[order[j]].dpcfg == (DIM_MERGE | NORM_MAX << 4);
      if (m) {
        mix.insert(mix.end(), order.begin() + f, order.begin() + f + gp.second);
        if (at < 0) at = (int)ngroups.size();
        ++nmix;
      } else {
        ngroups.push_back(gp);
        norder.insert(norder.end(), order.begin() + f, order.begin() + f + gp.second);
      }
      f += gp.second;
    }
    if (nmix >= 2) {
      std::stable_sort(mix.begin(), mix.end(), [&](int x, int y) { return e->n_events[x] > e->n_events[y]; });
      int off = 0;
      for (int g = 0; g < at; ++g) off += ngroups[g].second;
      norder.insert(norder.begin() + off, mix.begin(), mix.end());
      ngroups.insert(ngroups.begin() + at, {ksim_scan1::kPolMix, (int)mix.size()});
      order.swap(norder);
      groups.swap(ngroups);
      e->last_launches = (int)groups.size();
    }
  }
  KSIM_HIP(hipMemcpyAsync(e->d_replist, order.data(), sizeof(int) * order.size(), hipMemcpyHostToDevice, e->stream));
  KSIM_HIP(hipMemsetAsync(e->d_fail, 0, sizeof(int), e->stream));
  int gidx = 0;
  // The side streams share the process's hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4), and two
  // streams on one queue run their kernels one after the other.  So no more side streams than queues:
  // the first group (FGD on k_hmemo, the longest in a paper sweep) gets one to itself, the others take
  // the rest round robin (the engine stream, which only waits meanwhile, shares a queue with one of them).
  int nq = 4;
  if (const char* q = std::getenv("GPU_MAX_HW_QUEUES")) nq = std::atoi(q) > 0 ? std::atoi(q) : nq;
  if (const char* q = std::getenv("KSIM_SIDE_STREAMS")) nq = std::atoi(q) > 0 ? std::atoi(q) : nq;
  nq = std::max(1, std::min(nq, (int)ksim_engine::kSide));
  unsigned used = 0u;
  // Stream of concurrent group g: a side stream each (the first one alone on its own, the rest round robin), except
  // that a split FGD run's wide k_memo group runs on the engine stream itself -- which otherwise only waits -- so the
  // run needs one stream fewer: three groups on the engine stream and two side streams, within the hardware queues a
  // process gets (with three side streams two groups shared a queue and ran one after the other: 64 -> 133 ms for a
  // C4 share, profiles/r06/c4_wide/)
  const int g_off = concurrent && e->split_fgd ? 1 : 0;
  auto side_of = [&](int g) {
    const int j = g - g_off;
    return j < 0 ? -1 : (j == 0 || nq == 1) ? 0 : 1 + (j - 1) % (nq - 1);
  };
  if (concurrent) {
    if (!e->ev_fork) KSIM_HIP(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
    KSIM_HIP(hipEventRecord(e->ev_fork, e->stream));
    const char* gt0 = std::getenv("KSIM_GROUP_TIMES");
    if (gt0 && gt0[0] == '1') {
      if (!e->tev_fork) KSIM_HIP(hipEventCreate(&e->tev_fork));
      KSIM_HIP(hipEventRecord(e->tev_fork, e->stream));
    }
  }
  // The overlapped report (KSIM_VARIANT report_overlap=0 off): a cheap group with more replicas than the CUs the FGD
  // groups leave can hold at once runs in waves of workgroups, so its last replicas end well after its first ones; its
  // replicas then report one by one as each ends (k_report_overlap, behind the first group on that group's stream)
  // instead of all after the last one.  ovl[g]: the group gets the queue and that report.
  std::vector<char> ovl(groups.size(), 0);
  int fgd_cus = 0;  // CUs the FGD groups hold (a k_memo / k_hmemo workgroup fills a CU's registers)
  for (const auto& gp : groups) {
    if (gp.first == kPolFgdH) fgd_cus += gp.second;
    else if (gp.first == POL_FGD && e->run_mode != 2)
      fgd_cus += e->mplan_ok ? e->mplan->nwg : gp.second * (e->hplan_ok ? e->hplan->K : 1);
  }
  unsigned ovl_epoch = 0;
  for (const auto& gp : groups) {
    const int Rg = gp.second;
    hipStream_t gs = e->stream;
    if (concurrent && side_of(gidx) >= 0) {
      const int i = side_of(gidx);
      if (!e->side[i]) {
        KSIM_HIP(hipStreamCreateWithFlags(&e->side[i], hipStreamNonBlocking));
        KSIM_HIP(hipEventCreateWithFlags(&e->side_ev[i], hipEventDisableTiming));
      }
      gs = e->side[i];
      if (!(used & (1u << i))) KSIM_HIP(hipStreamWaitEvent(gs, e->ev_fork, 0));
      used |= 1u << i;
    }
    ++gidx;
    if (gp.first == kPolRandomGo) {
      ksim_random_go::RandGoArgs ga{e->d_reps, e->d_replist + first, e->d_go, e->N};
      const bool in_lds = ksim_random_go::lds_bytes(e->N, true) <= 160 * 1024;
      const size_t lds = ksim_random_go::lds_bytes(e->N, in_lds);
      if (in_lds) {
        KSIM_HIP(hipFuncSetAttribute((const void*)ksim_random_go::k_random_go<true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(ksim_random_go::k_random_go<true>, dim3(Rg), dim3(ksim_random_go::kBlock), lds, gs, ga);
      } else {
        hipLaunchKernelGGL(ksim_random_go::k_random_go<false>, dim3(Rg), dim3(ksim_random_go::kBlock), lds, gs, ga);
      }
      KSIM_HIP(hipGetLastError());
      note_kernel(e, "k_random_go");
      e->last_groups = (int)groups.size();
      e->last_rgo += Rg;
      first += Rg;
      continue;
    }
    if (gp.first == ksim_scan1::kPolMix) {
      using namespace ksim_scan1;
      const void* f = e->report ? (reg1 ? (const void*)k_scan1_mix<true, true> : (const void*)k_scan1_mix<true, false>)
                                : (reg1 ? (const void*)k_scan1_mix<false, true> : (const void*)k_scan1_mix<false, false>);
      const size_t lds = ksim_scan1::scan1_lds(e->N, ksim_scan1::kPolMix, e->report, reg1);
      ksim_scan1::Scan1Args sa{e->d_reps, e->d_replist + first, e->N,
                               dead_skip(e, std::vector<int>(order.begin() + first, order.begin() + first + Rg)) ? 1 : 0,
                               nullptr, 0};
      KSIM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      if (concurrent && e->report && gidx > 1 && variant("report_overlap", 1) != 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, ksim_scan1::kBlock, lds) != hipSuccess) {
          (void)hipGetLastError();
          nb = 0;
        }
        // (KSIM_TEST report_overlap=1: whatever the size, for the parity tests)
        if (nb > 0 && (Rg > std::max(0, e->cus - fgd_cus) * nb || test_knob("report_overlap", 0) != 0)) {
          if (Rg > e->done_cap) {
            if (e->d_done) KSIM_HIP(hipFree(e->d_done));
            KSIM_HIP(hipMalloc(&e->d_done, sizeof(unsigned long long) * (2 + (size_t)Rg)));
            KSIM_HIP(hipMemset(e->d_done, 0, sizeof(unsigned long long) * (2 + (size_t)Rg)));
            e->done_cap = Rg;
          }
          if (!e->ev_ovl) KSIM_HIP(hipEventCreateWithFlags(&e->ev_ovl, hipEventDisableTiming));
          KSIM_HIP(hipMemsetAsync(e->d_done, 0, 2 * sizeof(unsigned long long), gs));  // tickets; entries keep epochs
          KSIM_HIP(hipEventRecord(e->ev_ovl, gs));
          ovl[gidx - 1] = 1;
          e->last_ovl += Rg;
          ovl_epoch = e->done_epoch = e->done_epoch % 0x7fffffffu + 1;
          sa.done = e->d_done;
          sa.epoch = ovl_epoch;
        }
      }
      void* params[] = {(void*)&sa};
      KSIM_HIP(hipLaunchKernel(f, dim3(Rg), dim3(ksim_scan1::kBlock), params, lds, gs));
      note_kernel(e, "k_scan1_mix");
      e->last_K = 1;
      e->last_groups = (int)groups.size();
      e->last_scan1 += Rg;
      first += Rg;
      continue;
    }
    // FGD: the memoised replay when the cluster and the classes fit (run_mode 0 / 3)
    if (gp.first == POL_FGD && e->run_mode != 2) {
      if (e->mplan_ok) {  // prepared by prepare_memo (the FGD replicas are the first group of `order`)
        const MemoPlan& pl = *e->mplan;
        // a concurrent run (split_fgd): on its side stream, the next group launched once all Rg x K workgroups
        // have started (the gate; without it the later groups' workgroups could hold the CUs a wide replica's
        // exchange waits on)
        const bool gate = concurrent && gidx < (int)groups.size();
        int* flags = nullptr;
        int epoch = 0;
        if (gate) {
          const int rc = gate_flags(e, pl.nwg, &flags, &epoch);
          if (rc) return rc;
        }
        const int rc = launch_memo(e, pl, Rg, first, max_ev, gs, flags, epoch);
        if (rc) return rc;
        if (gate) gate_wait(e, pl.nwg, epoch, "FGD k_memo");
        note_kernel(e, pl.hkeys ? "k_memo_hkeys" : "k_memo");
        e->last_K = pl.K;
        e->last_groups = (int)groups.size();
        e->last_memo += Rg;
        first += Rg;
        if (profile) std::fprintf(stderr, "ksim memo%s: %d replicas, K=%d, Cw=%d, F waves %d, LDS %zu B\n",
                                  pl.decider ? " (decider)" : "", Rg, pl.K, pl.Cw, pl.nfw, pl.lds);
        continue;
      }
    }
    if ((gp.first == POL_FGD && e->run_mode != 2) || gp.first == kPolFgdH) {
      if (e->hplan_ok) {  // k_hmemo: one workgroup per replica, keys in HBM
        // The residency gate (concurrent groups behind a K = 1 FGD group; KSIM_VARIANT gate=0 off): the long FGD
        // replays take their CUs before any short group's workgroup is dispatched, so none of them waits
        // for a CU that short replays hold.  The host waits for every workgroup's start flag (bounded: a
        // gate that does not open in 2 s lets the launches go on, it orders work, it decides nothing).
        const bool gate = concurrent && gidx < (int)groups.size() && e->hplan->K == 1 && variant("gate", 1) != 0;
        int* flags = nullptr;
        int epoch = 0;
        if (gate) {
          const int rc = gate_flags(e, Rg, &flags, &epoch);
          if (rc) return rc;
        }
        bool gated = false;
        const int rc = launch_hmemo(e, Rg, first, max_ev, gs, flags, epoch, &gated);
        if (rc) return rc;
        if (gated) gate_wait(e, Rg, epoch, "FGD k_hmemo");
        note_kernel(e, e->hplan->K == 1 ? "k_hmemo" : "k_hmemo_wide");
        e->last_K = e->hplan->K;
        e->last_groups = (int)groups.size();
        e->last_hmemo += Rg;
        first += Rg;
        continue;
      }
      if (e->run_mode >= 3 && e->run_mode <= 5) return KSIM_ENOTSUP;
    }
    int K = choose_wgs(e, Rg);
    int S = (e->N + K - 1) / K;
    const bool general = profile || e->report || any_delete;
    // one workgroup per replica, create-only, a cheap policy: the 256-thread k_scan1 (ksim_scan1.hpp)
    const bool reg = reg1;
    if (K == 1 && !profile && !any_delete && e->scan1 && e->N <= kMaxSlice && scan1_fn(gp.first, e->report, reg) &&
        ksim_scan1::scan1_lds(e->N, gp.first, e->report, reg) <= 160 * 1024) {
      const void* f = scan1_fn(gp.first, e->report, reg);
      const size_t lds = ksim_scan1::scan1_lds(e->N, gp.first, e->report, reg);
      ksim_scan1::Scan1Args sa{e->d_reps, e->d_replist + first, e->N,
                               dead_skip(e, std::vector<int>(order.begin() + first, order.begin() + first + Rg)) ? 1 : 0,
                               nullptr, 0};
      KSIM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      void* params[] = {(void*)&sa};
      KSIM_HIP(hipLaunchKernel(f, dim3(Rg), dim3(ksim_scan1::kBlock), params, lds, gs));
      note_kernel(e, "k_scan1");
      e->last_K = 1;
      e->last_groups = (int)groups.size();
      e->last_scan1 += Rg;
      first += Rg;
      continue;
    }
    while (replay_lds(S, gp.first, general) > 160 * 1024 && K < ksim_replay::kMaxK && Rg * (K + 1) <= e->cus) {
      ++K;
      S = (e->N + K - 1) / K;
    }
    if (replay_lds(S, gp.first, general) > 160 * 1024) return KSIM_ERANGE;
    if (K > 1) {
      // the occupancy query bounds the co-resident grid: fewer, larger slices when it is short
      const int cap = resident_cap(e, replay_kernel(gp.first, K, general), replay_lds(S, gp.first, general));
      if (Rg * K > cap) {
        if (e->wgs_req > 0 && cap < Rg) return KSIM_ERANGE;
        K = std::max(1, std::min(K, cap / Rg));
        S = (e->N + K - 1) / K;
        if (replay_lds(S, gp.first, general) > 160 * 1024) {
          std::fprintf(stderr, "ksim: k_replay needs %d co-resident workgroups; the device holds %d\n", Rg * K, cap);
          return KSIM_ERANGE;
        }
      }
    }
    const size_t need = any_delete ? (size_t)e->R * K * std::max(max_ev, 1) : 0;
    if (need > e->hist_cap) {
      if (e->d_hist) KSIM_HIP(hipFree(e->d_hist));
      KSIM_HIP(hipMalloc(&e->d_hist, sizeof(int2) * need));
      e->hist_cap = need;
    }
    size_t lds = replay_lds(S, gp.first, general);
    // PWR+FGD: the per-(class, slot) memo when every class of the group fits beside the slice
    // (KSIM_VARIANT pf_memo=0: evaluate every slot every step, as before r04)
    int pm_c = 0;
    if (gp.first == POL_PWR_FGD) {
      if (variant("pf_memo", 1) != 0) {
        for (int j = first; j < first + Rg; ++j) pm_c = std::max(pm_c, (int)e->h_cls[order[j]].size());
        const size_t lm = ksim_replay::replay_layout(S, gp.first, general, pm_c).total;
        if (pm_c > 0 && lm <= 160 * 1024 &&
            (K == 1 || resident_cap(e, replay_kernel(gp.first, K, general), lm) >= Rg * K))
          lds = lm;
        else
          pm_c = 0;
      }
    }
    e->last_pf_memo = pm_c;
    ksim_replay::ReplayArgs ra;
    ra.xK = 0;
    ra.group = 0;
    ra.pm_c = pm_c;
    {
      const long v = test_knob("pf_memo_ver0", 0);
      ra.pm_ver0 = v > 0 && v < (long)ksim_replay::kPmInvalid ? (unsigned)v : 0u;
      ra.pf_guess = test_knob("pf_guess", 1) != 0 ? 1 : 0;
    }
    ra.reps = e->d_reps;
    ra.rep_list = e->d_replist + first;
    ra.N = e->N;
    ra.K = K;
    ra.S = S;
    ra.gran = e->d_gran;
    ra.hist = any_delete ? e->d_hist : nullptr;
    ra.hist_stride = std::max(max_ev, 1);
    ra.fail = e->d_fail;
    ra.prof = nullptr;
    ra.skip = dead_skip(e, std::vector<int>(order.begin() + first, order.begin() + first + Rg)) ? 1 : 0;
    if (profile) {
      const size_t words = (size_t)Rg * K * ksim_replay::kProfPhases;
      if (words > e->prof_cap) {
        if (e->d_prof) KSIM_HIP(hipFree(e->d_prof));
        KSIM_HIP(hipMalloc(&e->d_prof, sizeof(unsigned long long) * words));
        e->prof_cap = words;
      }
      KSIM_HIP(hipMemsetAsync(e->d_prof, 0, sizeof(unsigned long long) * words, e->stream));
      ra.prof = e->d_prof;
    }
    // re-initialise every polled word before the launch (granule tags restart at step 1; K = 1 polls none)
    if (K > 1)
      KSIM_HIP(hipMemsetAsync(e->d_gran, 0,
                              sizeof(unsigned long long) * (size_t)e->R * 2 * ksim_replay::kMaxK * ksim_replay::kGranW,
                              e->stream));
    const int grid = Rg * K;
    const TypDev* tp = e->d_tp;
    const int lrc = launch_persistent(replay_kernel(gp.first, K, general), grid, ksim_replay::kRBlock, lds, gs, e->coop && K > 1, ra, tp);
    if (lrc) return lrc;
    note_kernel(e, "k_replay");
    e->last_K = K;
    e->last_groups = (int)groups.size();
    first += Rg;
    if (profile) {
      // phase timers of this group (the stream is in order; read back before the next group reuses them)
      KSIM_HIP(hipStreamSynchronize(e->stream));
      print_replay_profile(e, Rg, K, max_ev);
    }
  }
  if (concurrent && e->report) {
    // each group's report on its own stream, behind its replay: the groups that finish early report while
    // the longest still runs; a timing event pair around each (last_report_ms sums them)
    int f = 0;
    if (e->grp_rev.size() < 2 * groups.size()) {
      const size_t had = e->grp_rev.size();
      e->grp_rev.resize(2 * groups.size(), nullptr);
      for (size_t q = had; q < e->grp_rev.size(); ++q) KSIM_HIP(hipEventCreate(&e->grp_rev[q]));
    }
    for (size_t g = 0; g < groups.size(); ++g) {
      const int Rg = groups[g].second;
      const int i = side_of((int)g);
      hipStream_t rs = i < 0 ? e->stream : e->side[i];
      int mev = 0;
      for (int j = f; j < f + Rg; ++j) mev = std::max(mev, e->n_events[order[j]]);
      if (ovl[g]) {  // behind the first group on its stream, each replica's report as soon as its replay ends
        const int i0 = side_of(0);
        rs = i0 < 0 ? e->stream : e->side[i0];
        KSIM_HIP(hipStreamWaitEvent(rs, e->ev_ovl, 0));
      }
      KSIM_HIP(hipEventRecord(e->grp_rev[2 * g], rs));
      if (ovl[g]) {
        hipLaunchKernelGGL(ksim_rep::k_report_overlap, dim3(std::min(Rg, std::max(1, e->cus - e->cus / 16))), dim3(ksim_rep::kScanBlock),
                           0, rs, (const ReplicaDev*)e->d_reps, (const TypDev*)e->d_tp, e->N,
                           (const int*)(e->d_replist + f), Rg, e->d_done, ovl_epoch, e->d_fail);
        KSIM_HIP(hipGetLastError());
      } else {
        const int rc = run_report(e, mev, rs, e->d_replist + f, Rg);
        if (rc) return rc;
      }
      KSIM_HIP(hipEventRecord(e->grp_rev[2 * g + 1], rs));
      f += Rg;
    }
    e->grp_rev_used = (int)groups.size();
    e->report_done = true;
  }
  e->tev_used = 0u;
  const char* gt = std::getenv("KSIM_GROUP_TIMES");
  if (concurrent && gt && gt[0] == '1') {
    if (!e->tev_fork) KSIM_HIP(hipEventCreate(&e->tev_fork));
    for (int i = 0; i < (int)ksim_engine::kSide; ++i) {
      if (!(used & (1u << i))) continue;
      if (!e->tev_side[i]) KSIM_HIP(hipEventCreate(&e->tev_side[i]));
      KSIM_HIP(hipEventRecord(e->tev_side[i], e->side[i]));
    }
    e->tev_used = used;
  }
  e->last_streams = __builtin_popcount(used);
  if (concurrent)  // join: the engine stream waits for every side stream used
    for (int i = 0; i < (int)ksim_engine::kSide; ++i) {
      if (!(used & (1u << i))) continue;
      KSIM_HIP(hipEventRecord(e->side_ev[i], e->side[i]));
      KSIM_HIP(hipStreamWaitEvent(e->stream, e->side_ev[i], 0));
    }
  return KSIM_OK;
}

static int run_graph(ksim_engine* e, int max_ev) {
  int rc = build_graph(e);
  if (rc) return rc;
  KSIM_HIP(hipMemsetAsync(e->d_base, 0, sizeof(int), e->stream));
  const int reps = (max_ev + e->K - 1) / e->K;
  for (int i = 0; i < reps; ++i) KSIM_HIP(hipGraphLaunch(e->graph, e->stream));
  return KSIM_OK;
}

int ksim_engine_run(ksim_engine* e) {
  if (!e) return KSIM_EINVAL;
  int max_ev = 0;
  for (int r = 0; r < e->R; ++r) {
    if (!e->d_ev[r]) return KSIM_ESTATE;
    max_ev = std::max(max_ev, e->n_events[r]);
  }
  KSIM_HIP(hipSetDevice(e->device));
  e->report_done = false;
  e->grp_rev_used = 0;
  e->tev_used = 0u;  // KSIM_GROUP_TIMES: only run_persistent's concurrent groups record side-stream ends
  e->last_launches = 0;
  e->last_streams = 0;
  e->last_gate = 0;
  e->last_ovl = 0;
  e->last_kernels.clear();
  int rc = prepare_memo(e, max_ev);
  if (rc) return rc;
  KSIM_HIP(hipEventRecord(e->ev0, e->stream));
  rc = reset_state(e);
  if (rc) return rc;
  if (e->report) KSIM_HIP(hipMemsetAsync(e->d_last, 0xff, sizeof(int32_t) * (size_t)e->N * e->R, e->stream));
  // run_mode 1: the per-pod path (k_step, + k_step_pwr for the PWR policies, hipGraph)
  const bool step_path = e->run_mode == 1;
  for (int r = 0; r < e->R; ++r)
    if (is_pwr_policy(e->reps[r].policy) && !e->pw_set[r]) return KSIM_ESTATE;
  for (int r = 0; r < e->R; ++r)  // Go-stream Random: the persistent path, best / worst / random selectors
    if (go_random(e, r) && (step_path || e->shard_world > 0 ||
                            (e->reps[r].gpusel != SEL_BEST && e->reps[r].gpusel != SEL_WORST && e->reps[r].gpusel != SEL_RANDOM)))
      return KSIM_ENOTSUP;
  if (e->shard_world > 0 && !e->peers.empty()) rc = run_hmemo_peer(e, max_ev);
  else if (e->shard_world > 0) rc = any_pwr(e) ? KSIM_ENOTSUP : run_sharded(e, max_ev);
  else rc = step_path ? run_graph(e, max_ev) : run_persistent(e, max_ev);
  if (!rc && e->shard_world > 0) note_kernel(e, !e->peers.empty() ? "k_hmemo_wide" : "k_step");
  if (!rc && step_path) note_kernel(e, any_pwr(e) ? "k_step+k_step_pwr" : "k_step");
  if (rc) return rc;
  KSIM_HIP(hipEventRecord(e->ev_mid, e->stream));
  if (e->report && !e->report_done) {
    rc = run_report(e, max_ev, e->stream, nullptr, e->R);
    if (rc) return rc;
  }
  KSIM_HIP(hipEventRecord(e->ev1, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  float ms = 0, rms = 0;
  KSIM_HIP(hipEventElapsedTime(&ms, e->ev0, e->ev1));
  KSIM_HIP(hipEventElapsedTime(&rms, e->ev_mid, e->ev1));
  e->last_ms = ms;
  e->last_report_ms = e->report ? rms : 0.0;
  for (int g = 0; g < e->grp_rev_used; ++g) {  // concurrent groups: each group's report on its side stream
    float gms = 0.f;
    KSIM_HIP(hipEventElapsedTime(&gms, e->grp_rev[2 * g], e->grp_rev[2 * g + 1]));
    e->last_report_ms += gms;
  }
  if (e->tev_used) {  // KSIM_GROUP_TIMES=1
    std::fprintf(stderr, "ksim group times (ms from the fork to each side stream's end):");
    for (int i = 0; i < (int)ksim_engine::kSide; ++i) {
      float gms = 0.f;
      if ((e->tev_used >> i) & 1u && hipEventElapsedTime(&gms, e->tev_fork, e->tev_side[i]) == hipSuccess)
        std::fprintf(stderr, " side%d %.3f;", i, gms);
    }
    for (int g = 0; g < e->grp_rev_used; ++g) {  // each group's replay end (= its report's start) and report end
      float a = 0.f, b = 0.f;
      if (hipEventElapsedTime(&a, e->tev_fork, e->grp_rev[2 * g]) == hipSuccess &&
          hipEventElapsedTime(&b, e->tev_fork, e->grp_rev[2 * g + 1]) == hipSuccess)
        std::fprintf(stderr, " g%d replay %.3f report %.3f;", g, a, b);
    }
    std::fprintf(stderr, " run %.3f\n", ms);
  }
  e->last_steps = max_ev;
  e->last_step_path = step_path;
  if (!step_path && e->shard_world == 0) {
    int fail = 0;
    KSIM_HIP(hipMemcpy(&fail, e->d_fail, sizeof(int), hipMemcpyDeviceToHost));
    if (fail & 2) return KSIM_ERANGE;  // a raw PWR score outside the 24-bit key field
    if (fail & 60) std::fprintf(stderr, "ksim: a memoised kernel's LDS wait timed out (fail bits 0x%x)\n", fail);
    if (fail & 64) std::fprintf(stderr, "ksim: the overlapped report waited too long for a replay (fail bits 0x%x)\n", fail);
    if (fail) return KSIM_ESTATE;  // a granule poll or an LDS wait timed out
  }
  return KSIM_OK;
}

int ksim_shard_comm_id(uint8_t* out) {
  if (!out) return KSIM_EINVAL;
  RcclApi* r = rccl();
  if (!r) return KSIM_ENOTSUP;
  ncclUniqueId id;
  if (r->get_unique_id(&id) != ncclSuccess) return KSIM_EHIP;
  std::memcpy(out, id.internal, KSIM_SHARD_ID_BYTES);
  return KSIM_OK;
}

int ksim_engine_set_shard(ksim_engine* e, int rank, int world, int node_offset, int n_global, const uint8_t* comm_id) {
  if (!e || world < 1 || world > 16 || rank < 0 || rank >= world || node_offset < 0 || n_global < e->N ||
      node_offset + e->N > n_global || n_global > kMaxRank || e->R != 1)
    return KSIM_EINVAL;
  if (e->shard_world > 0) return KSIM_ESTATE;  // once per engine, before set_nodes
  KSIM_HIP(hipSetDevice(e->device));
  if (comm_id) {
    RcclApi* r = rccl();
    if (!r) return KSIM_ENOTSUP;
    ncclUniqueId id;
    std::memcpy(id.internal, comm_id, KSIM_SHARD_ID_BYTES);
    const ncclResult_t nr = r->comm_init_rank(&e->comm, world, id, rank);
    if (nr != ncclSuccess) {
      std::fprintf(stderr, "ksim: ncclCommInitRank failed: %s\n", r->error_string(nr));
      e->comm = nullptr;
      return KSIM_EHIP;
    }
  }
  KSIM_HIP(hipMalloc(&e->d_send, 4 * sizeof(unsigned long long)));
  KSIM_HIP(hipMalloc(&e->d_recv, 4 * sizeof(unsigned long long) * (size_t)world));
  KSIM_HIP(hipMemset(e->d_send, 0, 4 * sizeof(unsigned long long)));
  e->shard_world = world;
  e->shard_rank = rank;
  e->node_off = node_offset;
  e->n_global = n_global;
  e->reps[0].node_off = node_offset;
  int rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_set_shard_exchange(ksim_engine* e, ksim_shard_exchange_fn fn, void* user) {
  if (!e) return KSIM_EINVAL;
  if (e->shard_world < 1 || e->comm) return KSIM_ESTATE;  // after set_shard, and not beside RCCL
  e->xfn = fn;
  e->xuser = user;
  e->h_send.assign(4, 0);
  e->h_recv.assign(4 * (size_t)e->shard_world, 0);
  return KSIM_OK;
}

// ---- one shard per process: device-initiated exchange through IPC-mapped granule buffers ----
constexpr size_t kPeerGranBytes = sizeof(unsigned long long) * 2 * 256 * 2;  // 2 slots x 256 columns x 2
constexpr uint32_t kPeerMagic = 0x4850534bu;  // "KSPH" after the IPC handle (include/ksim_engine.h)

// The device ordinal in this process of the GPU a peer handle names (PCI domain / bus / device), -1 if it
// is not visible here; -2 for a malformed handle.
static int peer_device(const uint8_t* hd) {
  uint32_t tail[5];
  std::memcpy(tail, hd + sizeof(hipIpcMemHandle_t), sizeof tail);
  if (tail[0] != kPeerMagic) return -2;
  char bus[32];
  std::snprintf(bus, sizeof bus, "%04x:%02x:%02x.0", tail[1], tail[2], tail[3]);
  int dev = -1;
  if (hipDeviceGetByPCIBusId(&dev, bus) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return dev;
}

int ksim_shard_peer_handle(ksim_engine* e, uint8_t* out) {
  if (!e || !out) return KSIM_EINVAL;
  if (e->shard_world < 1 || e->comm || e->xfn) return KSIM_ESTATE;
  KSIM_HIP(hipSetDevice(e->device));
  if (!e->d_pgran) {
    // uncached device memory: the peers' stores land in it over xGMI and the local polls read it there
    KSIM_HIP(hipExtMallocWithFlags((void**)&e->d_pgran, kPeerGranBytes, hipDeviceMallocUncached));
    KSIM_HIP(hipMemset(e->d_pgran, 0, kPeerGranBytes));
  }
  if (e->pgran_handle.empty()) {
    hipIpcMemHandle_t h;
    KSIM_HIP(hipIpcGetMemHandle(&h, e->d_pgran));
    static_assert(sizeof(hipIpcMemHandle_t) + 20 <= KSIM_SHARD_HANDLE_BYTES, "IPC handle size");
    hipDeviceProp_t prop;
    KSIM_HIP(hipGetDeviceProperties(&prop, e->device));
    const uint32_t tail[5] = {kPeerMagic, (uint32_t)prop.pciDomainID, (uint32_t)prop.pciBusID,
                              (uint32_t)prop.pciDeviceID, (uint32_t)getpid()};
    e->pgran_handle.assign(KSIM_SHARD_HANDLE_BYTES, 0);
    std::memcpy(e->pgran_handle.data(), &h, sizeof h);
    std::memcpy(e->pgran_handle.data() + sizeof h, tail, sizeof tail);
  }
  std::memcpy(out, e->pgran_handle.data(), KSIM_SHARD_HANDLE_BYTES);
  return KSIM_OK;
}

int ksim_engine_set_shard_peers(ksim_engine* e, const uint8_t* handles) {
  if (!e || !handles) return KSIM_EINVAL;
  if (e->shard_world < 1 || !e->d_pgran || e->pgran_handle.empty() || !e->peers.empty()) return KSIM_ESTATE;
  KSIM_HIP(hipSetDevice(e->device));
  const int world = e->shard_world;
  if (const long ep = test_knob("peer_epoch0", 0))  // tests: start the run epoch near its wrap
    e->peer_epoch = (int)(ep & 0xffffff);
  e->peers.assign(world, nullptr);
  e->peer_opened.assign(world, 0);
  if (e->pgran_handle.empty() ||
      std::memcmp(handles + (size_t)e->shard_rank * KSIM_SHARD_HANDLE_BYTES, e->pgran_handle.data(),
                  KSIM_SHARD_HANDLE_BYTES) != 0) {
    e->peers.clear();
    return KSIM_EINVAL;  // this shard's own handle must sit at its rank
  }
  // every peer's device first: visible here and reachable (xGMI / P2P), or nothing is mapped
  for (int q = 0; q < world; ++q) {
    if (q == e->shard_rank) continue;
    const int pd = peer_device(handles + (size_t)q * KSIM_SHARD_HANDLE_BYTES);
    int can = pd == e->device ? 1 : 0;
    if (pd >= 0 && pd != e->device) {
      if (hipDeviceCanAccessPeer(&can, e->device, pd) != hipSuccess) {
        (void)hipGetLastError();
        can = 0;
      }
    }
    if (pd < 0 || !can) {
      std::fprintf(stderr, "ksim: shard %d's exchange buffer is %s\n", q,
                   pd == -2 ? "a malformed handle" : pd == -1 ? "on a GPU not visible in this process"
                                                               : "on a GPU without a peer path from this one");
      e->peers.clear();
      e->peer_opened.clear();
      return pd == -2 ? KSIM_EINVAL : KSIM_EPEER;
    }
  }
  for (int q = 0; q < world; ++q) {
    if (q == e->shard_rank) {
      e->peers[q] = e->d_pgran;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles + (size_t)q * KSIM_SHARD_HANDLE_BYTES, sizeof h);
    void* p = nullptr;
    const hipError_t r = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (r != hipSuccess) {
      std::fprintf(stderr, "ksim: hipIpcOpenMemHandle (shard %d): %s\n", q, hipGetErrorString(r));
      (void)hipGetLastError();
      for (int k = 0; k < q; ++k)
        if (e->peer_opened[k]) (void)hipIpcCloseMemHandle(e->peers[k]);
      e->peers.clear();
      e->peer_opened.clear();
      return KSIM_EHIP;
    }
    e->peers[q] = reinterpret_cast<unsigned long long*>(p);
    e->peer_opened[q] = 1;
  }
  return KSIM_OK;
}

// ksim_engine_run of a shard with peers: k_hmemo over this shard's slices, the exchange spanning every
// shard's workgroups (K per shard, the same K and S on every rank: from n_global and world only).
static int run_hmemo_peer(ksim_engine* e, int max_ev) {
  using namespace ksim_hmemo;
  if (e->R != 1 || e->reps[0].policy != POL_FGD || e->report || go_random(e, 0) || !score_table())
    return KSIM_ENOTSUP;
  const int world = e->shard_world;
  const int nmax = (e->n_global + world - 1) / world;
  int K = std::max(1, 64 / world);
  int S = std::max(kFan, (nmax + K - 1) / K + kFan - 1) / kFan * kFan;
  if (S > kMaxNb * kFan) {
    S = kMaxNb * kFan;
    K = (nmax + S - 1) / S;
  }
  const int Kt = world * K;
  if (Kt > 256 || e->N > K * S) return KSIM_ENOTSUP;
  const int stride = std::max(max_ev, 1);
  hipStream_t st = e->stream;
  const int zero = 0;
  KSIM_HIP(hipMemcpyAsync(e->d_replist, &zero, sizeof(int), hipMemcpyHostToDevice, st));
  int rc = prepare_hmemo(e, std::vector<int>{0}, max_ev, K, S);
  if (rc) return rc;
  if (!e->hplan_ok) return KSIM_ENOTSUP;
  e->mplan_dirty = true;
  KSIM_HIP(hipMemcpyAsync(e->d_nodes, e->d_nodes_init, sizeof(NodeRec) * (size_t)e->N, hipMemcpyDeviceToDevice, st));
  KSIM_HIP(hipMemcpyAsync(e->d_tags, e->d_tags_init, sizeof(uint16_t) * e->tags_stride, hipMemcpyDeviceToDevice, st));
  KSIM_HIP(hipMemsetAsync(e->d_res[0], 0xff, sizeof(ResultDev) * (size_t)stride, st));
  if ((rc = hmemo_init_keys(e, 1, 0, st, e->node_off))) return rc;
  HMemoArgs a = hmemo_args(e, 0, stride);
  a.roff = e->node_off;
  a.wbase = e->shard_rank * K;
  a.Ktot = Kt;
  a.gran = e->d_pgran;
  a.npeer = world;
  e->peer_epoch = (e->peer_epoch + 1) & 0xffffff;  // every rank runs the same runs: the same epoch (24 bits)
  if (e->peer_epoch == 0) e->peer_epoch = 1;
  a.epoch = e->peer_epoch;
  for (int q = 0; q < world; ++q) a.peer[q] = e->peers[q];
  if (e->has_delete[0]) {
    if ((rc = ensure_buf(e->d_h_hist, e->h_cap[13], (size_t)K * stride))) return rc;
    a.hist = e->d_h_hist;
  }
  KSIM_HIP(hipMemsetAsync(e->d_fail, 0, sizeof(int), st));
  const bool gen = a.delay != 0;
  const void* f = Kt <= 64 ? (gen ? (const void*)k_hmemo<1, true> : (const void*)k_hmemo<1, false>)
                           : (gen ? (const void*)k_hmemo<4, true> : (const void*)k_hmemo<4, false>);
  if (K > resident_cap(e, f, e->hplan->lds)) return KSIM_ERANGE;
  KSIM_HIP(hipEventRecord(e->ev0, st));
  const TypDev* tpp = e->d_tp;
  // a plain launch: K <= 64 one-per-CU workgroups are resident (checked above), and a cooperative launch
  // takes the device's one global-wave-sync resource, which a second shard process on the same device
  // would wait for behind the first's persistent kernel
  if ((rc = launch_persistent(f, K, kHBlock, e->hplan->lds, st, false, a, tpp))) return rc;
  KSIM_HIP(hipEventRecord(e->ev1, st));
  KSIM_HIP(hipStreamSynchronize(st));
  int fail = 0;
  KSIM_HIP(hipMemcpy(&fail, e->d_fail, sizeof(int), hipMemcpyDeviceToHost));
  if (fail) return KSIM_ESTATE;
  float ms = 0;
  KSIM_HIP(hipEventElapsedTime(&ms, e->ev0, e->ev1));
  e->last_ms = ms;
  e->last_steps = max_ev;
  e->last_K = K;
  e->last_hmemo = 1;
  return KSIM_OK;
}

// ---- a node-sharded FGD cluster on k_hmemo (one launch for the whole in-process group) ----
// Every shard engine keeps its own plan, keys, L1 and node records; the launch's workgroups are the
// shards' slices (K per shard, S ranks each), and each pod step's slice maxima go through ONE exchange of
// world x K granule columns: selectHost over the union (generic_scheduler.go:187-212), the owner of the
// winner binds.  Results carry global ranks as the k_step shards' do (ksim/shard.py merge_results).
static bool hmemo_group_eligible(ksim_engine* const* engines, int world) {
  if (variant("shard_hmemo", 1) == 0) return false;
  if (!score_table()) return false;
  for (int k = 0; k < world; ++k) {
    const ksim_engine* e = engines[k];
    if (e->R != 1 || e->reps[0].policy != POL_FGD || e->report || e->run_mode == 1 || e->run_mode == 2 ||
        go_random(e, 0))
      return false;
  }
  return true;
}

// The cheap policies' node-sharded group on k_replay slices (r06, round-5 verdict item 7): every shard's K slices in
// ONE launch, one exchange of Kt = world x K columns per pod step (the keys carry global name ranks, so the max is
// selectHost over the union, generic_scheduler.go:187-212; BestFit's NormalizeScore range rides in the same granules
// as in the unsharded k_replay, plugin_utils.go:48-74).  Lean runs only: one replica per shard,
// a create-only stream, no report, no profile.
static bool replay_group_eligible(ksim_engine* const* engines, int world) {
  const int pol = engines[0]->reps[0].policy;
  if (pol < POL_BESTFIT || pol > POL_RANDOM || variant("shard_replay", 1) == 0) return false;
  for (int k = 0; k < world; ++k) {
    const ksim_engine* e = engines[k];
    if (e->R != 1 || e->reps[0].policy != pol || e->report || e->run_mode == 1 || e->has_delete[0] || go_random(e, 0))
      return false;
  }
  const char* pe = std::getenv("KSIM_PROFILE");
  return !(pe && pe[0] != '0');
}

// KSIM_OK with *done = false: the group does not fit (the caller keeps the per-pod k_step path).
static int run_replay_group(ksim_engine* const* engines, int world, int max_ev, bool* done) {
  using namespace ksim_replay;
  *done = false;
  ksim_engine* e0 = engines[0];
  int N = 1;  // slices cover the largest shard
  for (int k = 0; k < world; ++k) N = std::max(N, engines[k]->N);
  const int pol = e0->reps[0].policy;
  // slices of about 384 nodes (choose_wgs), at most 256 columns in all
  int K = std::max(1, std::min(256 / world, (N + 383) / 384));
  K = std::min(K, std::max(1, e0->cus / world));
  int S = (N + K - 1) / K;
  while (replay_lds(S, pol, false) > 160 * 1024 && (K + 1) * world <= std::min(256, e0->cus)) {
    ++K;
    S = (N + K - 1) / K;
  }
  const int Kt = world * K;
  if (Kt < 2 || replay_lds(S, pol, false) > 160 * 1024) return KSIM_OK;
  const void* f = replay_kernel(pol, Kt, false);
  const size_t lds = replay_lds(S, pol, false);
  if (Kt > resident_cap(e0, f, lds)) return KSIM_OK;
  hipStream_t st = e0->stream;
  KSIM_HIP(hipSetDevice(e0->device));
  int rc;
  if (!e0->d_rgran) KSIM_HIP(hipMalloc(&e0->d_rgran, sizeof(unsigned long long) * 2 * 256 * kGranW));
  if (!e0->d_rgreps) KSIM_HIP(hipMalloc(&e0->d_rgreps, sizeof(ReplicaDev) * 16));
  if (!e0->d_rglist) {
    KSIM_HIP(hipMalloc(&e0->d_rglist, sizeof(int) * 16));
    std::vector<int> id(16);
    std::iota(id.begin(), id.end(), 0);
    KSIM_HIP(hipMemcpy(e0->d_rglist, id.data(), sizeof(int) * 16, hipMemcpyHostToDevice));
  }
  bool skip = true;
  for (int k = 0; k < world; ++k) {
    ksim_engine* e = engines[k];
    KSIM_HIP(hipStreamSynchronize(e->stream));
    KSIM_HIP(hipMemcpyAsync(e->d_nodes, e->d_nodes_init, sizeof(NodeRec) * (size_t)e->N, hipMemcpyDeviceToDevice, st));
    KSIM_HIP(hipMemcpyAsync(e->d_tags, e->d_tags_init, sizeof(uint16_t) * e->tags_stride, hipMemcpyDeviceToDevice, st));
    KSIM_HIP(hipMemsetAsync(e->d_res[0], 0xff, sizeof(ResultDev) * (size_t)std::max(e->n_events[0], 1), st));
    KSIM_HIP(hipMemcpyAsync(e0->d_rgreps + k, e->d_reps, sizeof(ReplicaDev), hipMemcpyDeviceToDevice, st));
    skip = skip && dead_skip(e, std::vector<int>{0});
  }
  ReplayArgs ra;
  std::memset(&ra, 0, sizeof ra);
  ra.reps = e0->d_rgreps;
  ra.rep_list = e0->d_rglist;
  ra.N = N;
  ra.K = K;
  ra.S = S;
  ra.gran = e0->d_rgran;
  ra.hist = nullptr;
  ra.hist_stride = std::max(max_ev, 1);
  ra.fail = e0->d_fail;
  ra.prof = nullptr;
  ra.skip = skip ? 1 : 0;
  ra.pf_guess = 1;
  ra.xK = Kt;
  ra.group = 1;
  KSIM_HIP(hipMemsetAsync(e0->d_rgran, 0, sizeof(unsigned long long) * 2 * (size_t)Kt * kGranW, st));
  KSIM_HIP(hipMemsetAsync(e0->d_fail, 0, sizeof(int), st));
  KSIM_HIP(hipEventRecord(e0->ev0, st));
  const TypDev* tp = e0->d_tp;  // (the cheap policies read no typical table)
  if ((rc = launch_persistent(f, Kt, kRBlock, lds, st, e0->coop, ra, tp))) return rc;
  KSIM_HIP(hipEventRecord(e0->ev1, st));
  KSIM_HIP(hipStreamSynchronize(st));
  int fail = 0;
  KSIM_HIP(hipMemcpy(&fail, e0->d_fail, sizeof(int), hipMemcpyDeviceToHost));
  if (fail) return KSIM_ESTATE;
  float ms = 0;
  KSIM_HIP(hipEventElapsedTime(&ms, e0->ev0, e0->ev1));
  for (int k = 0; k < world; ++k) {
    engines[k]->last_ms = ms;
    engines[k]->last_steps = max_ev;
    engines[k]->last_K = K;
    engines[k]->last_kernels = "k_replay_group";
  }
  *done = true;
  return KSIM_OK;
}

// KSIM_OK with *done = false: the group does not fit k_hmemo (the caller keeps the per-pod k_step path).
static int run_hmemo_group(ksim_engine* const* engines, int world, int max_ev, bool* done) {
  using namespace ksim_hmemo;
  *done = false;
  ksim_engine* e0 = engines[0];
  const int stride = std::max(max_ev, 1);
  int nmax = 1;
  for (int k = 0; k < world; ++k) nmax = std::max(nmax, engines[k]->N);
  const int want = std::max(1, std::min(64, e0->cus / world));
  int S = std::max(kFan, (nmax + want - 1) / want + kFan - 1) / kFan * kFan;
  S = std::min(S, kMaxNb * kFan);
  const int K = (nmax + S - 1) / S;
  const int Kt = world * K;
  if (K < 1 || Kt > 256 || K * S < nmax) return KSIM_OK;
  std::vector<HMemoArgs> args(world);
  size_t lds = 0;
  for (int k = 0; k < world; ++k) {
    ksim_engine* e = engines[k];
    const int zero = 0;
    KSIM_HIP(hipMemcpyAsync(e->d_replist, &zero, sizeof(int), hipMemcpyHostToDevice, e->stream));
    int rc = prepare_hmemo(e, std::vector<int>{0}, max_ev, K, S);
    if (rc) return rc;
    if (!e->hplan_ok) return KSIM_OK;
    e->mplan_dirty = true;  // the unsharded plan is not this one
    lds = std::max(lds, e->hplan->lds);
  }
  const bool gen = hdelay_mask() != 0;  // the hdelay test knob: the general instantiation
  const void* f = Kt <= 64 ? (gen ? (const void*)k_hmemo_group<1, true> : (const void*)k_hmemo_group<1, false>)
                           : (gen ? (const void*)k_hmemo_group<4, true> : (const void*)k_hmemo_group<4, false>);
  if (Kt > resident_cap(e0, f, lds)) return KSIM_OK;
  hipStream_t st = e0->stream;
  KSIM_HIP(hipSetDevice(e0->device));
  if (!e0->d_ggran) KSIM_HIP(hipMalloc(&e0->d_ggran, sizeof(unsigned long long) * 2 * 256 * 2));
  if (!e0->d_hgargs) KSIM_HIP(hipMalloc(&e0->d_hgargs, sizeof(HMemoArgs) * 16));
  for (int k = 0; k < world; ++k) {
    ksim_engine* e = engines[k];
    KSIM_HIP(hipStreamSynchronize(e->stream));
    KSIM_HIP(hipMemcpyAsync(e->d_nodes, e->d_nodes_init, sizeof(NodeRec) * (size_t)e->N, hipMemcpyDeviceToDevice, st));
    KSIM_HIP(hipMemcpyAsync(e->d_tags, e->d_tags_init, sizeof(uint16_t) * e->tags_stride, hipMemcpyDeviceToDevice, st));
    KSIM_HIP(hipMemsetAsync(e->d_res[0], 0xff, sizeof(ResultDev) * (size_t)std::max(e->n_events[0], 1), st));
    int rc = hmemo_init_keys(e, 1, 0, st, e->node_off);
    if (rc) return rc;
    HMemoArgs a = hmemo_args(e, 0, stride);
    a.roff = e->node_off;
    a.wbase = k * K;
    a.Ktot = Kt;
    a.gran = e0->d_ggran;
    a.fail = e0->d_fail;
    if (e->has_delete[0]) {
      rc = ensure_buf(e->d_h_hist, e->h_cap[13], (size_t)K * stride);
      if (rc) return rc;
      a.hist = e->d_h_hist;
    }
    args[k] = a;
  }
  KSIM_HIP(hipMemcpyAsync(e0->d_hgargs, args.data(), sizeof(HMemoArgs) * world, hipMemcpyHostToDevice, st));
  KSIM_HIP(hipMemsetAsync(e0->d_ggran, 0, sizeof(unsigned long long) * 2 * (size_t)Kt * 2, st));
  KSIM_HIP(hipMemsetAsync(e0->d_fail, 0, sizeof(int), st));
  KSIM_HIP(hipStreamSynchronize(st));  // `args` is pageable
  KSIM_HIP(hipEventRecord(e0->ev0, st));
  KSIM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const HMemoArgs* ap = reinterpret_cast<const HMemoArgs*>(e0->d_hgargs);
  int Kk = K;
  void* params[] = {(void*)&ap, (void*)&Kk};
  const hipError_t lr = e0->coop ? hipLaunchCooperativeKernel(f, dim3(Kt), dim3(kHBlock), params, (unsigned)lds, st)
                                 : hipLaunchKernel(f, dim3(Kt), dim3(kHBlock), params, lds, st);
  if (lr == hipErrorCooperativeLaunchTooLarge) {
    (void)hipGetLastError();
    return KSIM_OK;
  }
  KSIM_HIP(lr);
  KSIM_HIP(hipEventRecord(e0->ev1, st));
  KSIM_HIP(hipStreamSynchronize(st));
  int fail = 0;
  KSIM_HIP(hipMemcpy(&fail, e0->d_fail, sizeof(int), hipMemcpyDeviceToHost));
  if (fail) return KSIM_ESTATE;
  float ms = 0;
  KSIM_HIP(hipEventElapsedTime(&ms, e0->ev0, e0->ev1));
  for (int k = 0; k < world; ++k) {
    engines[k]->last_ms = ms;
    engines[k]->last_steps = max_ev;
    engines[k]->last_K = K;
    engines[k]->last_hmemo = 1;
  }
  *done = true;
  return KSIM_OK;
}

int ksim_shard_group_run(ksim_engine* const* engines, int world) {
  if (!engines || world < 1 || world > 16) return KSIM_EINVAL;
  ksim_engine* e0 = engines[0];
  int max_ev = 0;
  for (int k = 0; k < world; ++k) {
    ksim_engine* e = engines[k];
    if (!e || e->shard_world != world || e->shard_rank != k || e->comm || e->xfn || e->device != e0->device ||
        !e->d_ev[0])
      return KSIM_EINVAL;
    if (e->n_events[0] != e0->n_events[0]) return KSIM_EINVAL;  // every shard sees the same events
    max_ev = std::max(max_ev, e->n_events[0]);
  }
  KSIM_HIP(hipSetDevice(e0->device));
  if (hmemo_group_eligible(engines, world)) {
    bool done = false;
    const int rc = run_hmemo_group(engines, world, max_ev, &done);
    if (!rc && done)
      for (int k = 0; k < world; ++k) engines[k]->last_kernels = "k_hmemo_group";
    if (rc || done) return rc;
  }
  if (replay_group_eligible(engines, world)) {
    bool done = false;
    const int rc = run_replay_group(engines, world, max_ev, &done);
    if (rc || done) return rc;
  }
  for (int k = 0; k < world; ++k) engines[k]->last_kernels = "k_step";
  if (!e0->d_ptrs) KSIM_HIP(hipMalloc(&e0->d_ptrs, sizeof(unsigned long long*) * 32));
  std::vector<unsigned long long*> ptrs(32, nullptr);
  for (int k = 0; k < world; ++k) {
    ptrs[k] = engines[k]->d_send;
    ptrs[16 + k] = engines[k]->d_recv;
  }
  hipStream_t st = e0->stream;
  KSIM_HIP(hipMemcpyAsync(e0->d_ptrs, ptrs.data(), sizeof(unsigned long long*) * 32, hipMemcpyHostToDevice, st));
  for (int k = 0; k < world; ++k) {
    ksim_engine* e = engines[k];
    KSIM_HIP(hipStreamSynchronize(e->stream));
    KSIM_HIP(hipMemcpyAsync(e->d_nodes, e->d_nodes_init, sizeof(NodeRec) * (size_t)e->N, hipMemcpyDeviceToDevice, st));
    KSIM_HIP(hipMemcpyAsync(e->d_tags, e->d_tags_init, sizeof(uint16_t) * e->tags_stride, hipMemcpyDeviceToDevice, st));
    if (e->report) KSIM_HIP(hipMemsetAsync(e->d_last, 0xff, sizeof(int32_t) * (size_t)e->N, st));
  }
  KSIM_HIP(hipEventRecord(e0->ev0, st));
  int rc;
  for (int s = 0; s < max_ev; ++s) {
    for (int k = 0; k < world; ++k)
      if ((rc = shard_local(engines[k], st, nullptr, s))) return rc;
    hipLaunchKernelGGL(k_shard_gather, dim3(1), dim3(1024), 0, st, (unsigned long long* const*)e0->d_ptrs,
                       (unsigned long long* const*)(e0->d_ptrs + 16), world);
    KSIM_HIP(hipGetLastError());
    for (int k = 0; k < world; ++k)
      if ((rc = shard_commit(engines[k], st, nullptr, s))) return rc;
  }
  for (int k = 0; k < world; ++k)
    if (engines[k]->report && (rc = run_report(engines[k], max_ev, engines[k]->stream, nullptr, engines[k]->R))) return rc;
  KSIM_HIP(hipEventRecord(e0->ev1, st));
  KSIM_HIP(hipStreamSynchronize(st));
  float ms = 0;
  KSIM_HIP(hipEventElapsedTime(&ms, e0->ev0, e0->ev1));
  for (int k = 0; k < world; ++k) {
    engines[k]->last_ms = ms;
    engines[k]->last_steps = max_ev;
  }
  return KSIM_OK;
}

int ksim_engine_set_report(ksim_engine* e, int enable) {
  if (!e) return KSIM_EINVAL;
  e->report = enable != 0;
  KSIM_HIP(hipSetDevice(e->device));
  for (int r = 0; r < e->R; ++r) {
    int rc = alloc_report(e, r);
    if (rc) return rc;
  }
  int rc = upload_reps(e);
  if (rc) return rc;
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_get_reports(ksim_engine* e, int replica, ksim_report* out, int n) {
  if (!e || !out || replica < 0 || replica >= e->R || n < 0 || n > e->n_events[replica]) return KSIM_EINVAL;
  if (!e->report || !e->d_rep[replica]) return KSIM_ESTATE;
  if (n == 0) return KSIM_OK;
  std::vector<RepAcc> h((size_t)n);
  KSIM_HIP(hipSetDevice(e->device));
  KSIM_HIP(hipMemcpyAsync(h.data(), e->d_rep[replica], sizeof(RepAcc) * n, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  for (int i = 0; i < n; ++i) {
    ksim_report& o = out[i];
    // exact fixed-point sum -> nearest double (the int128 -> double conversion rounds to nearest
    // even; the 2^-80 scaling is exact)
    for (int k = 0; k < 7; ++k) o.frag_bins[k] = std::ldexp((double)h[i].fx[k], -80);
    o.used_nodes = h[i].cnt[0];
    o.used_gpus = h[i].cnt[1];
    o.used_gpu_milli = h[i].cnt[2];
    o.total_gpus = e->total_gpus[replica];
    o.arrived_gpu_milli = h[i].cnt[4];
    o.used_cpu_milli = h[i].cnt[3];
    o.arrived_cpu_milli = h[i].cnt[5];
  }
  return KSIM_OK;
}

int ksim_engine_get_power_reports(ksim_engine* e, int replica, ksim_power_report* out, int n) {
  if (!e || !out || replica < 0 || replica >= e->R || n < 0 || n > e->n_events[replica]) return KSIM_EINVAL;
  if (!e->report || !e->d_rep[replica] || !e->pw_set[replica]) return KSIM_ESTATE;
  if (n == 0) return KSIM_OK;
  std::vector<RepAcc> h((size_t)n);
  KSIM_HIP(hipSetDevice(e->device));
  KSIM_HIP(hipMemcpyAsync(h.data(), e->d_rep[replica], sizeof(RepAcc) * n, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  for (int i = 0; i < n; ++i) {
    ksim_power_report& o = out[i];
    o.cpu_w = std::ldexp((double)h[i].fx[7], -80);
    o.gpu_w = std::ldexp((double)h[i].fx[8], -80);
    o.cluster_w = o.cpu_w + o.gpu_w;  // analysis.go:54 powerCPUCluster + powerGPUCluster
    o.invalid_nodes = h[i].cnt[6];
  }
  return KSIM_OK;
}

int ksim_engine_last_report_ms(ksim_engine* e, double* ms) {
  if (!e || !ms) return KSIM_EINVAL;
  *ms = e->last_report_ms;
  return KSIM_OK;
}

int ksim_engine_last_run_launches(ksim_engine* e, int* launches, int* side_streams) {
  if (!e || !launches || !side_streams) return KSIM_EINVAL;
  *launches = e->last_launches;
  *side_streams = e->last_streams;
  return KSIM_OK;
}

int ksim_engine_last_run_kernels(ksim_engine* e, char* out, int cap) {
  if (!e || !out || cap <= 0) return KSIM_EINVAL;
  if ((int)e->last_kernels.size() >= cap) return KSIM_ERANGE;
  std::memcpy(out, e->last_kernels.c_str(), e->last_kernels.size() + 1);
  return KSIM_OK;
}

int ksim_engine_last_run_gate(ksim_engine* e, int* gate, long long* timeouts) {
  if (!e || !gate || !timeouts) return KSIM_EINVAL;
  *gate = e->last_gate;
  *timeouts = e->gate_timeouts;
  return KSIM_OK;
}

int ksim_engine_last_run_report_overlap(ksim_engine* e, int* replicas) {
  if (!e || !replicas) return KSIM_EINVAL;
  *replicas = e->last_ovl;
  return KSIM_OK;
}

int ksim_engine_last_run_wgs(ksim_engine* e, int* wgs_per_replica) {
  if (!e || !wgs_per_replica) return KSIM_EINVAL;
  *wgs_per_replica = e->run_mode == 1 ? e->bpr : e->last_K;
  return KSIM_OK;
}

int ksim_engine_last_run_path(ksim_engine* e, int* path) {
  if (!e || !path) return KSIM_EINVAL;
  if (e->shard_world > 0) *path = KSIM_PATH_SHARDED;
  else if (e->run_mode == 1 || e->last_step_path) *path = KSIM_PATH_STEP;
  else if (e->last_rgo == e->R) *path = KSIM_PATH_RANDOM_GO;
  else if (e->last_scan1 == e->R) *path = KSIM_PATH_SCAN1;
  else if (e->last_memo == 0 && e->last_hmemo == 0) *path = KSIM_PATH_REPLAY;
  else if (e->last_memo == e->R) *path = KSIM_PATH_MEMO;
  else if (e->last_hmemo == e->R) *path = KSIM_PATH_HMEMO;
  else *path = KSIM_PATH_MIXED;
  return KSIM_OK;
}

int ksim_engine_time_steps(ksim_engine* e, int n_steps, double* mean_kernel_us) {
  if (!e || !mean_kernel_us || n_steps <= 0) return KSIM_EINVAL;
  KSIM_HIP(hipSetDevice(e->device));
  std::vector<hipEvent_t> evs(2 * n_steps);
  for (auto& x : evs) KSIM_HIP(hipEventCreate(&x));
  int rc = reset_state(e);
  if (rc) return rc;
  StepArgs a = base_args(e);
  a.rep_first = 0;
  a.base = nullptr;
  for (int i = 0; i < n_steps; ++i) {
    a.step_off = i;
    KSIM_HIP(hipEventRecord(evs[2 * i], e->stream));
    hipLaunchKernelGGL(k_step, dim3(e->bpr * e->R), dim3(kBlock), 0, e->stream, a, (const TypDev*)e->d_tp);
    if (any_pwr(e)) hipLaunchKernelGGL(k_step_pwr, dim3(e->bpr * e->R), dim3(kBlock), 0, e->stream, a);
    KSIM_HIP(hipEventRecord(evs[2 * i + 1], e->stream));
  }
  KSIM_HIP(hipStreamSynchronize(e->stream));
  double tot = 0;
  for (int i = 0; i < n_steps; ++i) {
    float ms = 0;
    KSIM_HIP(hipEventElapsedTime(&ms, evs[2 * i], evs[2 * i + 1]));
    tot += ms;
  }
  for (auto& x : evs) (void)hipEventDestroy(x);
  *mean_kernel_us = tot * 1000.0 / n_steps;
  return KSIM_OK;
}

int ksim_engine_last_run_ms(ksim_engine* e, double* ms) {
  if (!e || !ms) return KSIM_EINVAL;
  *ms = e->last_ms;
  return KSIM_OK;
}

int ksim_engine_last_run_steps(ksim_engine* e, int64_t* steps) {
  if (!e || !steps) return KSIM_EINVAL;
  *steps = e->last_steps;
  return KSIM_OK;
}

int ksim_engine_get_results(ksim_engine* e, int replica, ksim_result* out, int n) {
  if (!e || !out || replica < 0 || replica >= e->R || n < 0 || n > e->n_events[replica]) return KSIM_EINVAL;
  if (n == 0) return KSIM_OK;
  KSIM_HIP(hipSetDevice(e->device));
  KSIM_HIP(hipMemcpyAsync(out, e->d_res[replica], sizeof(ResultDev) * n, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  return KSIM_OK;
}

int ksim_engine_get_nodes(ksim_engine* e, int replica, ksim_node* out) {
  if (!e || !out || replica < 0 || replica >= e->R) return KSIM_EINVAL;
  KSIM_HIP(hipSetDevice(e->device));
  std::vector<NodeRec> h(e->N);
  std::vector<uint16_t> tags(e->tags_stride);
  KSIM_HIP(hipMemcpyAsync(h.data(), e->reps[replica].nodes, sizeof(NodeRec) * e->N, hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipMemcpyAsync(tags.data(), e->d_tags + (size_t)replica * e->tags_stride, sizeof(uint16_t) * e->tags_stride,
                          hipMemcpyDeviceToHost, e->stream));
  KSIM_HIP(hipStreamSynchronize(e->stream));
  if (e->h_nodes[replica].size() != (size_t)e->N) return KSIM_ESTATE;
  for (int i = 0; i < e->N; ++i) {
    ksim_node& o = out[i];
    const NodeRec& n = h[i];
    o = e->h_nodes[replica][i];  // static fields as given to set_nodes
    o.cpu_used_milli = o.cpu_alloc_milli - n.cpu_left;
    o.mem_used_mib = o.mem_alloc_mib - n.mem_left;
    o.pods_used = o.pods_alloc - n.pods_left;
    for (int g = 0; g < kMaxGpu; ++g) o.gpu_used_milli[g] = g < n.gpu_cnt ? kMilli - (int)n.gl[g] : 0;
    for (int k = 0; k < kNumTags; ++k) o.tag_count[k] = tags[(size_t)i * kTagStride + k];
  }
  return KSIM_OK;
}

}  // extern "C"

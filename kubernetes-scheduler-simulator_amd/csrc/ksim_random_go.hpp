// ksim_random_go.hpp -- the Random policy's draw structure on Go's math/rand stream (k_random_go).
//
// The reference's Random policy is RandomScorePlugin: PreScore draws rand.Intn(len(feasible)) from
// Go's global source and Score gives that node MaxNodeScore (random_score.go:42-68).  The same
// global source is drawn, per scheduling cycle, by scheduleOne (scheduler.go:464, Intn(100)), by
// DefaultPreemption when no node is feasible (default_preemption.go:183, Int31n(#nodes): every node
// is Unschedulable, none ...AndUnresolvable), and by the random GPU selector at Reserve
// (open_gpu_share.go:325-343, Intn(k) at the k-th fitting GPU).  PreScore runs for every policy
// (utils.go:241-248) but only when two or more nodes are feasible (generic_scheduler.go:158-164).
// This kernel replays exactly that sequence from a given source state (the stream as the replay
// driver leaves it, ksim_trace_replay_go_state), with the feasible list in node order -- what
// parallelize.Until gives with one worker; the reference's 16 workers make its order, and so its
// pick, timing-dependent, so no run of the reference is reproducible and this is the contract the
// oracle checks (fgd_oracle.c, orc_policy.go_stream).
//
// One 1024-thread workgroup per replica: thread t owns the contiguous node range [t*c, t*c+c) so a
// block-wide exclusive scan of the per-thread feasible counts (ballots per count bit, then the 16
// waves' totals) orders the feasible list by node index; lane 0 of wave 0 owns the generator
// (vec[607] in LDS, tap / feed in registers) and makes every draw; the owner of the pick finds it in
// its range; lane 0 reserves and binds.  The node records sit in LDS when they fit (kLds), else in
// HBM (a workgroup reads its own stores after a barrier); the events come through a 128-event LDS
// window, and the GpuClustering tag counts (HBM) take fire-and-forget atomics, so neither a load
// of the next event nor a tag read-modify-write sits on the step's chain.  (r04: 256 threads were
// slower, 41.7 against 38.5-38.9 ms at C2: five nodes per thread in the Filter and the pick's search.)
#pragma once

namespace ksim_random_go {

constexpr int kBlock = 1024;
constexpr int kEvWin = 128;  // events per LDS window
constexpr int kLen = 607, kTap = 273;  // rng.go rngLen, rngTap
constexpr int kStateWords = kLen + 2;  // vec, tap, feed (the host's upload layout)

struct RandGoArgs {
  ReplicaDev* reps;
  const int* rep_list;
  const unsigned long long* state;  // [R][kStateWords]
  int N;
};

struct GoShared {
  unsigned long long vec[kLen];
  PodDev ev[kEvWin];
  int wsum[kBlock / 64];
  int pick;  // index in the feasible list (-1: none)
  int node;  // the picked node
};


inline size_t lds_bytes(int N, bool lds_nodes) {
  return ((sizeof(GoShared) + 15) & ~(size_t)15) + (lds_nodes ? sizeof(NodeRec) * (size_t)N : 0);
}

// rng.go rngSource.Uint64 / rand.go Int31n, on lane 0's (tap, feed) and the LDS vector
struct GoGen {
  int tap, feed;
  __device__ __forceinline__ unsigned long long u64(unsigned long long* vec) {
    if (--tap < 0) tap += kLen;
    if (--feed < 0) feed += kLen;
    const unsigned long long x = vec[feed] + vec[tap];
    vec[feed] = x;
    return x;
  }
  __device__ __forceinline__ int int31(unsigned long long* vec) {
    return (int)((u64(vec) & 0x7fffffffffffffffull) >> 32);
  }
  __device__ int int31n(unsigned long long* vec, int n) {
    if ((n & (n - 1)) == 0) return int31(vec) & (n - 1);
    const int max = (int)((1u << 31) - 1u - (1u << 31) % (unsigned)n);
    int v = int31(vec);
    while (v > max) v = int31(vec);
    return v % n;
  }
};

template <bool kLds>
__global__ __launch_bounds__(kBlock) void k_random_go(RandGoArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GoShared& sh = *reinterpret_cast<GoShared*>(smem);
  const int r = a.rep_list[blockIdx.x];
  const ReplicaDev rp = a.reps[r];
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = a.N;
  NodeRec* nodes = kLds ? reinterpret_cast<NodeRec*>(smem + ((sizeof(GoShared) + 15) & ~(size_t)15)) : rp.nodes;
  const unsigned long long* st = a.state + (size_t)r * kStateWords;
  for (int i = tid; i < kLen; i += kBlock) sh.vec[i] = st[i];
  if (kLds)
    for (int i = tid; i < N; i += kBlock) store_node(&nodes[i], load_node(rp.nodes + i));
  GoGen gen{(int)st[kLen], (int)st[kLen + 1]};  // used by thread 0 only
  const int c = (N + kBlock - 1) / kBlock;
  const int lo = min(N, tid * c), hi = min(N, lo + c);
  __syncthreads();

  for (int step = 0; step < rp.n_events; ++step) {
    const int eb = step & (kEvWin - 1);
    if (eb == 0) {  // the next window of events (every thread passed the previous step's last barrier)
      const int nl = min(kEvWin, rp.n_events - step) * 2;
      const uint4* src = reinterpret_cast<const uint4*>(rp.ev + step);
      for (int i = tid; i < nl; i += kBlock) reinterpret_cast<uint4*>(sh.ev)[i] = src[i];
      __syncthreads();
    }
    const PodDev p = ksim_replay::uniform_pod(&sh.ev[eb]);
    if (p.flags & kPodDelete) {  // simulator.go:416-422 deletePod -> removePod: no draw
      if (tid == 0) {
        ResultDev out{-1, 0, 0, 0, ST_DELETED};
        if (p.ref >= 0 && p.ref < step) {
          const ResultDev cr = rp.res[p.ref];
          if (cr.node >= 0 && cr.status == ST_OK) {
            PodDev cp = rp.ev[p.ref];
            const int tg = cp.tag;
            cp.tag = -1;
            apply_bind(&nodes[cr.node], nullptr, cp, cr.gpu_mask, -1);
            if (tg >= 0) tag_add(rp.tags + (size_t)cr.node * kTagStride, tg, -1);
            if (rp.snap) {
              store_node(rp.snap + step, load_node(&nodes[cr.node]));
              rp.prev[step] = rp.last[cr.node];
              rp.last[cr.node] = step;
            }
            out.node = cr.node;
            out.gpu_mask = cr.gpu_mask;
          }
        }
        rp.res[step] = out;
      }
      __syncthreads();
      continue;
    }
    // Filter over this thread's range, then the block-wide exclusive scan of the counts
    int cnt = 0;
    for (int i = lo; i < hi; ++i) cnt += filter_node(load_node(&nodes[i]), p) ? 1 : 0;
    // this lane's exclusive prefix within the wave and the wave's total, one ballot per bit of the count
    int wexcl = 0, wtot = 0;
    for (int k = 0; (1 << k) <= c; ++k) {
      const unsigned long long m = __ballot((cnt >> k) & 1);
      wexcl += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << k;
      wtot += __popcll(m) << k;
    }
    if (lane == 0) sh.wsum[wv] = wtot;
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      const int s = sh.wsum[w];
      base += w < wv ? s : 0;
      total += s;
    }
    const int excl = base + wexcl;
    if (tid == 0) {
      (void)gen.int31n(sh.vec, 100);  // scheduler.go:464
      int pick = -1;
      if (total == 0) (void)gen.int31n(sh.vec, N);  // default_preemption.go:183 (N >= 1: a launch has nodes)
      else if (total == 1) pick = 0;                // the single-feasible shortcut: no PreScore
      else pick = gen.int31n(sh.vec, total);        // random_score.go:44
      sh.pick = pick;
      sh.node = -1;
    }
    __syncthreads();
    const int pick = sh.pick;
    if (pick >= excl && pick < excl + cnt) {
      int k = pick - excl;
      for (int i = lo; i < hi; ++i)
        if (filter_node(load_node(&nodes[i]), p) && k-- == 0) { sh.node = i; break; }
    }
    __syncthreads();
    if (tid == 0) {
      ResultDev out{-1, 0, 0, total, ST_UNSCHED};
      const int node = sh.node;
      if (node >= 0) {
        NodeRec* nr = &nodes[node];
        const NodeV n = load_node(nr);
        int mask;  // allocateGpuId (open_gpu_share.go:252-283)
        if (p.milli <= 0) mask = 0;                                   // Reserve skips the pod (:185-187)
        else if (p.milli < kMilli && p.num > 1) mask = -1;            // :274-276 panic
        else if (!is_share_pod(p)) mask = exclusive_gpu_mask(n, p);  // exclusive branch of every selector
        else if (rp.gpusel == SEL_RANDOM) {                          // :325-343 one draw per fitting GPU
          int k = 0;
          mask = -1;
          for (int g = 0; g < n.gpu_cnt(); ++g)
            if (n.gl(g) >= p.milli && gen.int31n(sh.vec, ++k) == 0) mask = 1 << g;
        } else {
          mask = select_gpus(n, p, rp.gpusel, -1, rp.seed, step);  // best / worst fit (host-checked)
        }
        if (mask < 0) {
          out.status = ST_ERROR;  // Reserve failed: allocateGpuId returned "" / panicked
        } else {
          out.status = ST_OK;
          out.score = result_score(rp, total, 0, 0, 0);
          PodDev q = p;
          q.tag = -1;
          apply_bind(nr, nullptr, q, mask, +1);
          if (p.tag >= 0) tag_add(rp.tags + (size_t)node * kTagStride, p.tag, +1);
          if (rp.snap) {
            store_node(rp.snap + step, load_node(nr));
            rp.prev[step] = rp.last[node];
            rp.last[node] = step;
          }
          out.node = node;
          out.gpu_mask = mask;
        }
      }
      rp.res[step] = out;
    }
    __syncthreads();
  }
  if (kLds)
    for (int i = tid; i < N; i += kBlock) store_node(rp.nodes + i, load_node(&nodes[i]));
}

}  // namespace ksim_random_go

// ksim_replay.hpp -- persistent whole-trace replay kernel (k_replay).
//
// One launch replays every replica to completion.  Replica r is owned by K
// co-resident workgroups; workgroup w keeps the node records of its slice
// [w*S, min(N,(w+1)*S)) in LDS for the whole run, so the per-pod loop touches
// no node record in HBM.  Per pod step:
//   1. Filter + Score of the slice (the k_step phases, on LDS records);
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

constexpr int kRBlock = 256;
constexpr int kChunk = 128;        // nodes per evaluation chunk
constexpr int kRMaxCand = 9;
constexpr int kMaxK = 64;          // workgroups per replica
constexpr int kGran = 3;           // granules per workgroup per step
constexpr unsigned kSpinLimit = 1u << 22;  // ~seconds: only a non-resident workgroup can stall a poll

struct ReplayArgs {
  ReplicaDev* reps;
  int N;
  int K;            // workgroups per replica
  int S;            // slice size (nodes per workgroup)
  unsigned long long* gran;  // [R][2][K][4]
  int2* hist;       // [R][K][hist_stride]: (node, mask+1) of pods this workgroup bound
  int hist_stride;
  int* fail;
};

// Small per-workgroup state at the start of the dynamic LDS region (16-B aligned);
// NodeRec nodes[S] and u16 tags[S][16] follow it.
struct __align__(16) ReplayShared {
  unsigned long long rkey[kRBlock / 64];
  unsigned long long win;
  int rcnt[kRBlock / 64], rerr[kRBlock / 64], rlo[kRBlock / 64], rhi[kRBlock / 64];
  int wstat[4];
  int tmp[kRBlock / 64];
  int stop;
  int pad0[3];
  int off[kChunk + 4];
  double F[kChunk * kRMaxCand];
  uint8_t item_node[kChunk * kRMaxCand];
  uint8_t item_code[kChunk * kRMaxCand];
};
static_assert(sizeof(ReplayShared) % 16 == 0, "keep the node records 16-B aligned");

__device__ __forceinline__ unsigned long long gload(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup-wide exclusive scan of one int per thread (256 threads), total in *tot.
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
  for (int i = 0; i < kRBlock / 64; ++i) {
    base += i < w ? s_tmp[i] : 0;
    t += s_tmp[i];
  }
  *tot = t;
  __syncthreads();
  return base + incl - v;
}

}  // namespace ksim_replay

// Micro-benchmark of the k_memo building blocks on one wave (cycles from s_memtime).
// Build (scripts/ubench/build.sh): hipcc -O3 --offload-arch=gfx950 -ffp-contract=off ... ubench_memo.hip
// Run on a GPU box: ./scripts/ubench/ubench_memo
#include "ksim_engine.hip"

using namespace ksim;

__global__ void k_ub(const TypDev* tp_g, int nt, int ncpu, const NodeRec* nodes, const PodDev* pods,
                     unsigned long long* out, double* sink, const double* th_g) {
  __shared__ TypDev tp[kMaxTypical];
  __shared__ double fold[ksim_memo::kFoldBuf];
  __shared__ double th[104];
  const int lane = threadIdx.x;
  for (int i = lane; i < nt * 2; i += 64) reinterpret_cast<uint4*>(tp)[i] = reinterpret_cast<const uint4*>(tp_g)[i];
  for (int i = lane; i < 102; i += 64) th[i] = th_g[i];
  __syncthreads();
  const NodeV n = ksim_replay::uniform_node(nodes);
  const PodDev p = ksim_replay::uniform_pod(pods);
  double acc = 0;
  // 1. wave_F, chained through cpuL
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 64; ++it) {
    int cpuL, total;
    uint32_t gs[4];
    ksim_replay::fgd_candidate(n, 1 + (it & 1), p, &cpuL, gs, &total);
    const double F = ksim_memo::wave_F(cpuL + (acc > 1e300 ? 1 : 0), gs, total, 1u << n.gpu_type(), true, tp, ncpu,
                                       nt, lane, fold);
    acc += F;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  // 2. the score: direct expression, chained
  double x = acc;
  int sc = 0;
  for (int it = 0; it < 64; ++it) {
    sc += fgd_score_of_delta(x - 500.0 - sc);
    x += 1.0;
  }
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  // 3. the score through the step table, chained
  for (int it = 0; it < 64; ++it) {
    sc += fgd_score_lookup(x - 500.0 - sc, th);
    x += 1.0;
  }
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  // 4. filter + candidate mask per lane (lane = class), chained
  int cnt = 0;
  for (int it = 0; it < 64; ++it) {
    PodDev q = pods[lane & 15];
    q.cpu_req += cnt & 1;
    const bool f = filter_node(n, q);
    const unsigned fm = first_of_class(n, 0) & ksim_memo::ge_mask(n, q.milli);
    cnt += (f ? 1 : 0) + __popc(fm);
  }
  unsigned long long t4 = __builtin_amdgcn_s_memtime();
  // 5. scalar frag_F (eval_fgd_item) per thread
  ReplicaDev rp{};
  rp.typed = 1;
  rp.nt = nt;
  rp.ncpu = ncpu;
  double y = 0;
  for (int it = 0; it < 16; ++it) y += eval_fgd_item(n, 1 + ((it + lane) & 3), p, rp, tp_g);
  unsigned long long t5 = __builtin_amdgcn_s_memtime();
  // 6. dependent LDS round trip
  int v = lane;
  for (int it = 0; it < 64; ++it) v = reinterpret_cast<volatile int*>(fold)[(v + it) & 63] & 63;
  unsigned long long t6 = __builtin_amdgcn_s_memtime();
  asm volatile("" ::"v"(v));
  // 7. dependent v_add_f64 chain (the fold's critical path)
  double z = acc * 1e-300;
  const double inc = tp_g[lane & 7].freq;
  asm volatile("" ::"v"(inc));
  const unsigned long long t6b = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int it = 0; it < 64; ++it) z += inc;
  asm volatile("" ::"v"(z));
  unsigned long long t7 = __builtin_amdgcn_s_memtime();
  t6 = t6b;
  if (lane == 0) {
    out[6] = (t7 - t6) / 64;
    out[0] = (t1 - t0) / 64;
    out[1] = (t2 - t1) / 64;
    out[2] = (t3 - t2) / 64;
    out[3] = (t4 - t3) / 64;
    out[4] = (t5 - t4) / 16;
    out[5] = (t6 - t5) / 64;
  }
  sink[lane] = acc + y + sc + cnt + v + z;
}

int main() {
  const int nt = 35, ncpu = 4;
  std::vector<TypDev> tp(kMaxTypical);
  for (int t = 0; t < nt; ++t) {
    tp[t] = TypDev{};
    tp[t].cpu = 1000 * (t % 17);
    tp[t].milli = t < ncpu ? 0 : (t % 3 == 0 ? 1000 : 100 * (t % 9 + 1));
    tp[t].num_eff = t % 7 == 0 ? 2 : 1;
    tp[t].tmask = 0xffffffffu;
    tp[t].freq = 1.0 / (t + 3);
  }
  NodeRec nd{};
  nd.cpu_left = 64000;
  nd.mem_left = 100000;
  for (int g = 0; g < 8; ++g) nd.gl[g] = (uint16_t)(g < 3 ? 1000 : 400 + 50 * g);
  nd.pods_left = 100;
  nd.gpu_cnt = 8;
  nd.gpu_type = 1;
  nd.name_rank = 7;
  std::vector<PodDev> pods(16);
  for (int i = 0; i < 16; ++i) {
    pods[i] = PodDev{};
    pods[i].cpu_req = pods[i].cpu_nz = 1000 * (i + 1);
    pods[i].mem = 100;
    pods[i].milli = (int16_t)(i % 4 == 0 ? 1000 : 200 + 50 * i);
    pods[i].num = (int8_t)(i % 4 == 0 ? 1 + i / 4 : 1);
    pods[i].tmask = 0xffffffffu;
  }
  TypDev* d_tp;
  NodeRec* d_n;
  PodDev* d_p;
  unsigned long long* d_o;
  double* d_s;
  double* d_th;
  double th[102];
  if (!build_score_thresholds(th)) return 2;
  (void)hipMalloc(&d_th, sizeof th);
  (void)hipMemcpy(d_th, th, sizeof th, hipMemcpyHostToDevice);
  (void)hipMalloc(&d_tp, sizeof(TypDev) * kMaxTypical);
  (void)hipMalloc(&d_n, sizeof(NodeRec));
  (void)hipMalloc(&d_p, sizeof(PodDev) * 16);
  (void)hipMalloc(&d_o, 64);
  (void)hipMalloc(&d_s, 64 * 8);
  (void)hipMemcpy(d_tp, tp.data(), sizeof(TypDev) * kMaxTypical, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_n, &nd, sizeof nd, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_p, pods.data(), sizeof(PodDev) * 16, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_ub, dim3(1), dim3(64), 0, 0, d_tp, nt, ncpu, d_n, d_p, d_o, d_s, d_th);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
  }
  unsigned long long o[7];
  (void)hipMemcpy(o, d_o, sizeof o, hipMemcpyDeviceToHost);
  std::printf("s_memtime ticks per op: wave_F %llu, score direct %llu, score table %llu, filter+cand-mask %llu, "
              "scalar eval_fgd_item %llu, LDS round trip %llu, dependent f64 add %llu\n",
              o[0], o[1], o[2], o[3], o[4], o[5], o[6]);
  return 0;
}

// Host-side harness for the engine's __host__ __device__ math (ksim_device.hpp):
// the exact functions the gfx950 kernels inline, run on the CPU so the CPU test
// suite can compare them with the oracle without a GPU.  Test infrastructure only.
#include <cstring>

#include "ksim_device.hpp"

using namespace ksim;

extern "C" {

double dm_go_exp(double x) { return go_exp(x); }
double dm_go_tanh(double x) { return go_tanh(x); }

// FGD score from delta = cur - new: direct, and through the threshold table k_memo uses
int dm_score_of_delta(double delta) { return fgd_score_of_delta(delta); }
int dm_score_thresholds(double* th102) { return build_score_thresholds(th102) ? 1 : 0; }
int dm_score_lookup(double delta, const double* th102) { return fgd_score_lookup(delta, th102); }

// host copy of the engine's split table: CPU-only entries first, then GPU entries (order kept)
static int split_table(int T, const int* tpi4, const double* tpf, TypDev* out, int* ncpu, bool* typed) {
  int k = 0;
  *typed = false;
  for (int pass = 0; pass < 2; ++pass)
    for (int t = 0; t < T; ++t) {
      const bool cpu = tpi4[4 * t + 1] == 0;
      if ((pass == 0) != cpu) continue;
      TypDev d;
      std::memset(&d, 0, sizeof d);
      d.cpu = tpi4[4 * t];
      d.milli = tpi4[4 * t + 1];
      d.num_eff = tpi4[4 * t + 2];
      d.tmask = (uint32_t)tpi4[4 * t + 3];
      d.freq = tpf[t];
      if (!cpu && d.tmask != 0xFFFFFFFFu) *typed = true;
      out[k++] = d;
      if (pass == 0) *ncpu = k;
    }
  if (*ncpu > k) *ncpu = 0;
  return k;
}

static double F_of(int cpuL, const int (&gl)[kMaxGpu], uint32_t typebit, const TypDev* tp, int ncpu, int nt,
                   bool typed) {
  return typed ? frag_F<true>(cpuL, gl, typebit, tp, ncpu, nt) : frag_F<false>(cpuL, gl, typebit, tp, ncpu, nt);
}

// F(state) for a node state given as (cpu_left, gl[8], type id) and a typical table {cpu,milli,num_eff,mask},freq
double dm_frag_F(int cpu_left, const int* gl8, int type_id, int T, const int* tpi4, const double* tpf) {
  static TypDev tp[kMaxTypical];
  int ncpu = 0;
  bool typed = false;
  const int nt = split_table(T, tpi4, tpf, tp, &ncpu, &typed);
  int gl[kMaxGpu];
  for (int g = 0; g < kMaxGpu; ++g) gl[g] = gl8[g];
  return F_of(cpu_left, gl, 1u << type_id, tp, ncpu, nt, typed);
}

// all 7 NodeGpuShareFragAmount bins (the report's per-node term)
void dm_frag_bins7(int cpu_left, const int* gl8, int type_id, int T, const int* tpi4, const double* tpf, double* out7) {
  static TypDev tp[kMaxTypical];
  int ncpu = 0;
  bool typed = false;
  const int nt = split_table(T, tpi4, tpf, tp, &ncpu, &typed);
  int gl[kMaxGpu];
  for (int g = 0; g < kMaxGpu; ++g) gl[g] = gl8[g];
  double b[7];
  frag_bins7(cpu_left, gl, 1u << type_id, tp, ncpu, nt, b);
  for (int k = 0; k < 7; ++k) out7[k] = b[k];
}

// fix80 as two 64-bit halves (lo, hi)
void dm_fix80(double x, unsigned long long* lo, long long* hi) {
  const __int128 v = fix80(x);
  *lo = (unsigned long long)v;
  *hi = (long long)(v >> 64);
}

static NodeV mk(int cpu_left, int mem_left, const int* gl8, int gpu_cnt, int type_id, int pods_left) {
  NodeV n;
  std::memset(&n, 0, sizeof n);
  n.cpu_left = cpu_left;
  n.mem_left = mem_left;
  for (int g = 0; g < 4; ++g) n.g[g] = (uint32_t)gl8[2 * g] | ((uint32_t)gl8[2 * g + 1] << 16);
  n.meta = ((uint32_t)pods_left & 0xffffu) | ((uint32_t)gpu_cnt << 16) | ((uint32_t)type_id << 24);
  return n;
}

static PodDev pod(int cpu, int milli, int num, unsigned mask) {
  PodDev p;
  std::memset(&p, 0, sizeof p);
  p.cpu_req = p.cpu_nz = cpu;
  p.milli = (int16_t)milli;
  p.num = (int8_t)num;
  p.tmask = mask;
  p.tag = num == 0 ? -1 : (num == 1 && milli < kMilli ? 0 : (milli == kMilli ? num : -2));
  return p;
}

// FGD score of one node for one pod, as k_step computes it (current state + one candidate per
// distinct fitting milli-left value, or the Sub state)
int dm_fgd_score(int cpu_left, const int* gl8, int gpu_cnt, int type_id, int cpu, int milli, int num, int T,
                 const int* tpi4, const double* tpf, int* gpu_out) {
  static TypDev tp[kMaxTypical];
  int ncpu = 0;
  bool typed = false;
  const int nt = split_table(T, tpi4, tpf, tp, &ncpu, &typed);
  const NodeV n = mk(cpu_left, 0, gl8, gpu_cnt, type_id, 100);
  const PodDev p = pod(cpu, milli, num, 0xffffffffu);
  int gl[kMaxGpu];
  unpack_gl(n, gl);
  const double F0 = F_of(n.cpu_left, gl, 1u << type_id, tp, ncpu, nt, typed);
  *gpu_out = -1;
  if (is_share_pod(p)) {
    int best = -1, bs = 0;
    for (int g = 0; g < kMaxGpu; ++g) {
      bool first = g < gpu_cnt && gl[g] >= milli;
      for (int h = 0; h < g; ++h) first = first && !(gl[h] == gl[g]);
      if (!first) continue;
      int c[kMaxGpu];
      for (int k = 0; k < kMaxGpu; ++k) c[k] = gl[k] - (k == g ? milli : 0);
      const int fs = fgd_frag_score(F0, F_of(n.cpu_left - cpu, c, 1u << type_id, tp, ncpu, nt, typed));
      if (best < 0 || fs > bs) { bs = fs; best = g; }
    }
    *gpu_out = best;
    return bs;
  }
  bool ok = false;
  const unsigned sm = sub_gpu_mask(gl, gpu_cnt, n.cpu_left, p, &ok);
  int c[kMaxGpu];
  int cl = n.cpu_left;
  for (int k = 0; k < kMaxGpu; ++k) c[k] = gl[k];
  if (ok) {
    cl -= cpu;
    for (int k = 0; k < kMaxGpu; ++k) c[k] -= ((sm >> k) & 1u) ? milli : 0;
  }
  return fgd_frag_score(F0, F_of(cl, c, 1u << type_id, tp, ncpu, nt, typed));
}

int dm_filter(int cpu_left, int mem_left, const int* gl8, int gpu_cnt, int type_id, int pods_left, int cpu, int mem,
              int milli, int num, unsigned mask) {
  PodDev p = pod(cpu, milli, num, mask);
  p.mem = mem;
  return filter_node(mk(cpu_left, mem_left, gl8, gpu_cnt, type_id, pods_left), p) ? 1 : 0;
}
// k_scan1's branch-free form of the same Filter
int dm_filter_scan(int cpu_left, int mem_left, const int* gl8, int gpu_cnt, int type_id, int pods_left, int cpu, int mem,
                   int milli, int num, unsigned mask) {
  PodDev p = pod(cpu, milli, num, mask);
  p.mem = mem;
  return filter_scan(mk(cpu_left, mem_left, gl8, gpu_cnt, type_id, pods_left), p) ? 1 : 0;
}

int dm_bestfit(int cpu_left, const int* gl8, int gpu_cnt, int cpu, int milli, int num) {
  const NodeV n = mk(cpu_left, 0, gl8, gpu_cnt, 0, 1);
  return bestfit_score(n, pod(cpu, milli, num, ~0u), n.total());
}
int dm_dotprod_mm(int cpu_left, const int* gl8, int gpu_cnt, int cpu, int milli, int num) {
  return dotprod_merge_max(mk(cpu_left, 0, gl8, gpu_cnt, 0, 1), pod(cpu, milli, num, ~0u));
}
int dm_dotprod(int cpu_left, const int* gl8, int gpu_cnt, int cpu, int milli, int num, int cap, int cfg, int* gid) {
  const NodeV n = mk(cpu_left, 0, gl8, gpu_cnt, 0, 1);
  return dotprod_cfg_score(n, pod(cpu, milli, num, ~0u), cap, cfg, gid);
}
int dm_packing(const int* gl8, int gpu_cnt, int cpu, int milli, int num, int* err) {
  bool e = false;
  const int s = packing_score(mk(64000, 0, gl8, gpu_cnt, 0, 1), pod(cpu, milli, num, ~0u), &e);
  *err = e ? 1 : 0;
  return s;
}
int dm_clustering(const int* tags9, const int* gl8, int gpu_cnt, int milli, int num) {
  uint16_t t[16] = {0};
  for (int k = 0; k < 9; ++k) t[k] = (uint16_t)tags9[k];
  const NodeV n = mk(64000, 0, gl8, gpu_cnt, 0, 1);
  const PodDev p = pod(1000, milli, num, ~0u);
  return clustering_score(t, p.tag, n.total());
}
// k_scan1's form: the presence bits of the same counts (clustering_score_mask)
int dm_clustering_mask(const int* tags9, const int* gl8, int gpu_cnt, int milli, int num) {
  unsigned m = 0u;
  for (int k = 0; k < 9; ++k) m |= tags9[k] > 0 ? 1u << k : 0u;
  const NodeV n = mk(64000, 0, gl8, gpu_cnt, 0, 1);
  const PodDev p = pod(1000, milli, num, ~0u);
  return clustering_score_mask(m, p.tag, n.total());
}
int dm_exclusive(const int* gl8, int gpu_cnt, int milli, int num) {
  return exclusive_gpu_mask(mk(0, 0, gl8, gpu_cnt, 0, 1), pod(0, milli, num, ~0u));
}

// PWR (pwr_score.go:143-212) with a power model given as the ksim_power_model layout
int dm_pwr_score(int cpu_left, int cap, int cpu_model, const int* gl8, int gpu_cnt, int type_id, int cpu, int milli,
                 int num, const void* pm, int* gpu_out, int* err_out) {
  const NodeV n = mk(cpu_left, 0, gl8, gpu_cnt, type_id, 1);
  bool err = false;
  const int s = pwr_score(n, pod(cpu, milli, num, ~0u), cap, cpu_model, *static_cast<const PowerDev*>(pm), gpu_out, &err);
  *err_out = err ? 1 : 0;
  return s;
}
int dm_pwr_normalize(int s, int lo, int hi) { return pwr_normalize(s, lo, hi); }

}  // extern "C"

// ksim_trace.cpp -- host-side replay driver (include/ksim_trace.h): trace
// loading, target-workload table, event order, workload tuning and node
// naming.  Pure host C++; every step cites the reference code it restates
// (Fr4nz83/kubernetes-scheduler-simulator @ 2024_08_07).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "go_rand.hpp"
#include "ksim_trace.h"

namespace {

struct Node {
  std::string name;
  int64_t cpu = 0, mem = 0;
  int gpu = 0;
  std::string model;
};

struct Pod {
  std::string name;
  int64_t cpu = 0, mem = 0;
  int gpu_milli = 0;  // annotation value (pod_csv_to_yaml.py:106-118)
  int gpu_count = 0;
  std::string spec;   // normalised pipe list
};

// xoshiro256** seeded through splitmix64: draws of the synthetic-cluster generator
// (ksim_trace_synthetic; not part of the reference).  Replays use Go's math/rand (go_rand.hpp).
struct Rng {
  uint64_t s[4];
  static uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  explicit Rng(uint64_t seed) {
    uint64_t x = seed;
    for (auto& v : s) v = splitmix(x);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  int64_t int63() { return (int64_t)(next() >> 1); }
  // Int63n-style unbiased draw in [0, n)
  int64_t intn(int64_t n) {
    if (n <= 1) return 0;
    const int64_t max = (int64_t)((1ULL << 63) - 1 - (1ULL << 63) % (uint64_t)n);
    int64_t v = int63();
    while (v > max) v = int63();
    return v % n;
  }
};

std::vector<std::string> split_csv_line(const std::string& line) {
  std::vector<std::string> out;
  std::string cur;
  bool q = false;
  for (char c : line) {
    if (c == '"') q = !q;
    else if (c == ',' && !q) { out.push_back(cur); cur.clear(); }
    else if (c != '\r') cur.push_back(c);
  }
  out.push_back(cur);
  return out;
}

bool parse_i64(const std::string& s, int64_t* v) {
  if (s.empty()) return false;
  char* end = nullptr;
  double d = std::strtod(s.c_str(), &end);
  if (end == s.c_str()) return false;
  *v = (int64_t)d;  // pod_csv_to_yaml.py formats with %d (truncation)
  return true;
}

std::string normalise_spec(const std::string& spec) {
  // pod_csv_to_yaml.py:120-123: drop empty elements, re-join with '|'
  std::string out, cur;
  auto flush = [&]() {
    if (!cur.empty()) { if (!out.empty()) out.push_back('|'); out += cur; }
    cur.clear();
  };
  for (char c : spec) {
    if (c == '|') flush();
    else cur.push_back(c);
  }
  flush();
  return out;
}

}  // namespace

struct ksim_trace {
  std::vector<Node> nodes;             // sorted by name (simulator.go:577-579)
  std::vector<Pod> pods;               // name order (SetWorkloadPods, simulator.go:963-966)
  std::vector<std::string> vocab;      // GPU model vocabulary (ids)
  std::vector<int> node_type;          // vocab id per node
  std::vector<uint32_t> pod_mask;      // accepted-model mask per pod
};

namespace {

int vocab_id(ksim_trace* t, const std::string& m) {
  for (size_t i = 0; i < t->vocab.size(); ++i)
    if (t->vocab[i] == m) return (int)i;
  t->vocab.push_back(m);
  return (int)t->vocab.size() - 1;
}

uint32_t spec_mask(ksim_trace* t, const std::string& spec, bool* overflow) {
  if (spec.empty()) return KSIM_TYPE_ANY;  // IsNodeAccessibleToPodByType: empty list = any
  uint32_t m = 0;
  std::stringstream ss(spec);
  std::string item;
  while (std::getline(ss, item, '|')) {
    if (item.empty()) continue;
    const int id = vocab_id(t, item);
    if (id >= KSIM_MAX_TYPES) { *overflow = true; continue; }
    m |= 1u << id;
  }
  return m;
}

int finalize(ksim_trace* t) {
  std::stable_sort(t->nodes.begin(), t->nodes.end(), [](const Node& a, const Node& b) { return a.name < b.name; });
  std::stable_sort(t->pods.begin(), t->pods.end(), [](const Pod& a, const Pod& b) { return a.name < b.name; });
  // vocabulary: node models in sorted order first, then models only pods ask for
  t->vocab.clear();
  std::vector<std::string> models;
  for (auto& n : t->nodes) models.push_back(n.model);
  std::sort(models.begin(), models.end());
  models.erase(std::unique(models.begin(), models.end()), models.end());
  for (auto& m : models) vocab_id(t, m);
  t->node_type.clear();
  for (auto& n : t->nodes) t->node_type.push_back(vocab_id(t, n.model));
  bool overflow = false;
  t->pod_mask.clear();
  for (auto& p : t->pods) t->pod_mask.push_back(spec_mask(t, p.spec, &overflow));
  if (overflow || t->vocab.size() > KSIM_MAX_TYPES) return KSIM_ERANGE;
  return KSIM_OK;
}

ksim_pod to_engine_pod(const Pod& p, uint32_t mask) {
  ksim_pod e;
  std::memset(&e, 0, sizeof e);
  e.cpu_milli = p.cpu;
  e.cpu_nz_milli = p.cpu;  // trace pods always carry a cpu request (GetNonzeroRequests keeps it)
  e.mem_mib = p.mem;
  e.gpu_milli = p.gpu_milli;
  e.gpu_count = p.gpu_count;
  e.type_mask = p.gpu_count > 0 ? mask : KSIM_TYPE_ANY;
  e.ref = -1;
  return e;
}

}  // namespace

extern "C" {

int ksim_trace_load_openb(const char* node_csv, const char* pod_csv, ksim_trace** out) {
  if (!node_csv || !pod_csv || !out) return KSIM_EINVAL;
  *out = nullptr;
  auto t = new ksim_trace();
  {
    std::ifstream f(node_csv);
    if (!f) { delete t; return KSIM_EIO; }
    std::string line;
    std::getline(f, line);
    auto hdr = split_csv_line(line);
    auto col = [&](const char* n) { return (int)(std::find(hdr.begin(), hdr.end(), n) - hdr.begin()); };
    const int c_sn = col("sn"), c_cpu = col("cpu_milli"), c_mem = col("memory_mib"), c_gpu = col("gpu"),
              c_model = col("model");
    if (c_sn >= (int)hdr.size() || c_cpu >= (int)hdr.size() || c_gpu >= (int)hdr.size()) { delete t; return KSIM_EIO; }
    while (std::getline(f, line)) {
      if (line.empty() || line == "\r") continue;
      auto v = split_csv_line(line);
      if (c_sn >= (int)v.size() || c_cpu >= (int)v.size() || c_gpu >= (int)v.size()) { delete t; return KSIM_EIO; }
      Node n;
      n.name = v[c_sn];
      int64_t x = 0;
      if (!parse_i64(v[c_cpu], &x)) { delete t; return KSIM_EIO; }
      n.cpu = x;
      n.mem = (c_mem < (int)v.size() && parse_i64(v[c_mem], &x)) ? x : 0;
      n.gpu = parse_i64(v[c_gpu], &x) ? (int)x : 0;
      n.model = (c_model < (int)v.size() && n.gpu > 0) ? v[c_model] : std::string();
      if (n.model == "nan") n.model.clear();
      t->nodes.push_back(n);
    }
  }
  {
    std::ifstream f(pod_csv);
    if (!f) { delete t; return KSIM_EIO; }
    std::string line;
    std::getline(f, line);
    auto hdr = split_csv_line(line);
    auto col = [&](const char* n) { return (int)(std::find(hdr.begin(), hdr.end(), n) - hdr.begin()); };
    const int c_name = col("name"), c_cpu = col("cpu_milli"), c_mem = col("memory_mib"), c_num = col("num_gpu"),
              c_milli = col("gpu_milli"), c_spec = col("gpu_spec");
    if (c_name >= (int)hdr.size() || c_cpu >= (int)hdr.size() || c_num >= (int)hdr.size()) { delete t; return KSIM_EIO; }
    while (std::getline(f, line)) {
      if (line.empty() || line == "\r") continue;
      auto v = split_csv_line(line);
      if (c_name >= (int)v.size() || c_cpu >= (int)v.size() || c_num >= (int)v.size()) { delete t; return KSIM_EIO; }
      Pod p;
      p.name = v[c_name];
      int64_t x = 0;
      if (!parse_i64(v[c_cpu], &x)) { delete t; return KSIM_EIO; }
      p.cpu = x;
      p.mem = (c_mem < (int)v.size() && parse_i64(v[c_mem], &x)) ? x : 0;
      const int num = parse_i64(v[c_num], &x) ? (int)x : 0;
      if (num != 0) {  // pod_csv_to_yaml.py:106-123 annotations only for GPU pods
        int64_t milli = 1000;
        if (c_milli < (int)v.size() && parse_i64(v[c_milli], &x)) milli = x;
        p.gpu_milli = (0 < milli && milli <= 1000) ? (int)milli : (milli > 1000 ? 1000 : 0);
        p.gpu_count = num;
        if (c_spec < (int)v.size()) {
          std::string s = v[c_spec];
          if (s == "nan") s.clear();
          p.spec = normalise_spec(s);
        }
      }
      t->pods.push_back(p);
    }
  }
  int rc = finalize(t);
  if (rc) { delete t; return rc; }
  *out = t;
  return KSIM_OK;
}

int ksim_trace_synthetic(const ksim_trace* base, int n_nodes, int n_pods, uint64_t seed, ksim_trace** out) {
  if (!base || !out || n_nodes <= 0 || n_pods < 0 || base->nodes.empty() || base->pods.empty()) return KSIM_EINVAL;
  auto t = new ksim_trace();
  Rng rn(seed), rp(seed + 1);
  char buf[64];
  for (int i = 0; i < n_nodes; ++i) {
    Node n = base->nodes[(size_t)rn.intn((int64_t)base->nodes.size())];
    std::snprintf(buf, sizeof buf, "synth-node-%06d", i);
    n.name = buf;
    t->nodes.push_back(n);
  }
  for (int i = 0; i < n_pods; ++i) {
    Pod p = base->pods[(size_t)rp.intn((int64_t)base->pods.size())];
    std::snprintf(buf, sizeof buf, "synth-pod-%07d", i);
    p.name = buf;
    t->pods.push_back(p);
  }
  int rc = finalize(t);
  if (rc) { delete t; return rc; }
  *out = t;
  return KSIM_OK;
}

void ksim_trace_free(ksim_trace* t) { delete t; }

int ksim_trace_num_nodes(const ksim_trace* t) { return t ? (int)t->nodes.size() : KSIM_EINVAL; }
int ksim_trace_num_pods(const ksim_trace* t) { return t ? (int)t->pods.size() : KSIM_EINVAL; }
int ksim_trace_num_types(const ksim_trace* t) { return t ? (int)t->vocab.size() : KSIM_EINVAL; }

int ksim_trace_type_name(const ksim_trace* t, int id, char* buf, int cap) {
  if (!t || !buf || cap <= 0 || id < 0 || id >= (int)t->vocab.size()) return KSIM_EINVAL;
  std::snprintf(buf, (size_t)cap, "%s", t->vocab[id].c_str());
  return KSIM_OK;
}

int ksim_trace_node_at(const ksim_trace* t, int i, ksim_trace_node* out) {
  if (!t || !out || i < 0 || i >= (int)t->nodes.size()) return KSIM_EINVAL;
  std::memset(out, 0, sizeof *out);
  std::snprintf(out->name, sizeof out->name, "%s", t->nodes[i].name.c_str());
  out->cpu_milli = t->nodes[i].cpu;
  out->mem_mib = t->nodes[i].mem;
  out->gpu_count = t->nodes[i].gpu;
  out->gpu_type = t->node_type[i];
  return KSIM_OK;
}

int ksim_trace_pod_at(const ksim_trace* t, int i, ksim_trace_pod* out) {
  if (!t || !out || i < 0 || i >= (int)t->pods.size()) return KSIM_EINVAL;
  std::memset(out, 0, sizeof *out);
  const Pod& p = t->pods[i];
  std::snprintf(out->name, sizeof out->name, "%s", p.name.c_str());
  out->cpu_milli = p.cpu;
  out->mem_mib = p.mem;
  out->gpu_milli = p.gpu_milli;
  out->gpu_count = p.gpu_count;
  out->type_mask = p.gpu_count > 0 ? t->pod_mask[i] : KSIM_TYPE_ANY;
  std::snprintf(out->gpu_spec, sizeof out->gpu_spec, "%s", p.spec.c_str());
  return KSIM_OK;
}

// GetTypicalPods (frag.go:285-380) + SortTargetPodInDecreasingCount (:436-445)
// + TargetPodList.Less (resource.go:24-42).
int ksim_trace_typical(const ksim_trace* t, const ksim_typical_cfg* cfg, ksim_typical* out, int cap, int* n_out) {
  if (!t || !cfg || !n_out || (cap > 0 && !out)) return KSIM_EINVAL;
  struct Key {
    int64_t cpu;
    int milli, num;
    std::string type;
    bool operator<(const Key& o) const {
      return std::tie(cpu, milli, num, type) < std::tie(o.cpu, o.milli, o.num, o.type);
    }
  };
  std::map<Key, double> cnt;
  std::map<Key, uint32_t> mask;
  double total = 0;
  for (size_t i = 0; i < t->pods.size(); ++i) {
    const Pod& p = t->pods[i];
    Key k{p.cpu, p.gpu_milli, p.gpu_count, p.gpu_count > 0 ? p.spec : std::string()};
    if (!cfg->is_involved_cpu_pods && k.num == 0) continue;
    double w = 1;
    if (cfg->gpu_res_weight > 0 && k.milli == 1000) w = 1 + (double)k.num * cfg->gpu_res_weight;
    cnt[k] = cnt[k] + w;
    mask[k] = p.gpu_count > 0 ? t->pod_mask[i] : KSIM_TYPE_ANY;
    total += w;
  }
  struct TP { Key k; double pct; };
  std::vector<TP> l;
  for (auto& kv : cnt) l.push_back({kv.first, kv.second});
  // sort.Reverse(TargetPodList): descending Percentage, then descending PodResource.Less
  std::sort(l.begin(), l.end(), [](const TP& a, const TP& b) {
    if (a.pct != b.pct) return a.pct > b.pct;
    return b.k < a.k;
  });
  const double expected = (double)(cfg->pod_popularity_threshold > 0 ? cfg->pod_popularity_threshold : 60) * total / 100.0;
  const int step = cfg->pod_increase_step > 0 ? cfg->pod_increase_step : 10;
  size_t i = 0;
  int podResNum = 0;
  double cum = 0;
  while (cum < expected) {
    podResNum += step;
    while ((int)i < podResNum && i < l.size()) {
      cum += l[i].pct;
      l[i].pct = l[i].pct / total;
      ++i;
    }
    if (i >= l.size() && cum < expected) break;  // the Go loop would not terminate
  }
  size_t nout = i;
  if (i < l.size()) {
    for (size_t j = 0; j < i; ++j) l[j].pct /= cum / total;
  } else {
    nout = l.size();
  }
  *n_out = (int)nout;
  if ((int)nout > cap) return KSIM_ERANGE;
  for (size_t j = 0; j < nout; ++j) {
    ksim_typical& o = out[j];
    std::memset(&o, 0, sizeof o);
    o.cpu_milli = l[j].k.cpu;
    o.gpu_milli = l[j].k.milli;
    o.gpu_count = l[j].k.num;
    o.type_mask = mask[l[j].k];
    o.freq = l[j].pct;
  }
  return KSIM_OK;
}

static int replay_impl(const ksim_trace* t, const ksim_replay_cfg* cfg, ksim_pod* events, int cap, int* n_events,
                       int32_t* pod_index, ksim_node* nodes, int32_t* name_prefix, ksim_go::Rand* rng_out) {
  // Go's global math/rand, seeded as core.go:115 does; the draws below are every draw the
  // reference makes from it between rand.Seed and the first scheduling cycle.
  ksim_go::Rand rng((int64_t)cfg->seed);
  (void)rng.Int();  // core.go:116: rand.Int() evaluated as a Debugf argument
  const int np = (int)t->pods.size();
  std::vector<int> order(np);
  for (int i = 0; i < np; ++i) order[i] = i;  // name order
  if (cfg->shuffle) {
    // SortClusterPods (simulator.go:975-984): sort.Slice by name, then rand.Shuffle
    rng.Shuffle(np, [&](int64_t i, int64_t j) { std::swap(order[i], order[j]); });
  }
  // TunePodsByNodeTotalResource (simulator.go:1201-1248)
  int64_t pod_total = 0, node_total = 0, pod_cpu = 0, node_cpu = 0;
  for (int i = 0; i < np; ++i) {
    pod_total += (int64_t)t->pods[i].gpu_milli * t->pods[i].gpu_count;
    pod_cpu += t->pods[i].cpu;
  }
  for (auto& n : t->nodes) {
    node_total += (int64_t)n.gpu * 1000;
    node_cpu += n.cpu;
  }
  std::vector<int> ev = order;
  const double ratio = cfg->tune_ratio;
  // simulator.go:1203-1211: the reference panics when the workload or the cluster has no CPU or no GPU
  // to tune against (tuneUpPods would never stop, Intn(0) would panic)
  if (ratio > 0 && (np == 0 || pod_cpu <= 0 || pod_total <= 0 || node_cpu <= 0 || node_total <= 0)) return KSIM_EINVAL;
  if (ratio > 0) {
    const double target = ratio * (double)node_total;
    if ((double)pod_total > target) {
      // tuneDownPods (simulator.go:1249-1262): rand.Intn(len(pods)), remove that index
      while ((double)pod_total > ratio * (double)node_total && !ev.empty()) {
        const int idx = (int)rng.Intn((int64_t)ev.size());
        const Pod& p = t->pods[ev[idx]];
        ev.erase(ev.begin() + idx);
        pod_total -= (int64_t)p.gpu_milli * p.gpu_count;
      }
    } else if ((double)pod_total < target) {
      // tuneUpPods (simulator.go:1263-1282): rand.Intn(len(workloadPods)) over the name-sorted
      // workload (simulator.go:966-968); note the MilliGpu vs TotalMilliGpu asymmetry
      for (;;) {
        const int idx = (int)rng.Intn(np);
        const Pod& p = t->pods[idx];
        if ((double)(pod_total + p.gpu_milli) > ratio * (double)node_total) break;
        pod_total += (int64_t)p.gpu_milli * p.gpu_count;
        ev.push_back(idx);
      }
    }
  }
  *n_events = (int)ev.size();
  // RunCluster -> runScheduler (simulator.go:286-289) starts the informers and waits for their
  // caches; each reflector's watch loop draws rand.Float64() once (reflector.go:400)
  const int draws = cfg->informer_draws < 0 ? KSIM_REPLAY_INFORMER_DRAWS : cfg->informer_draws;
  for (int i = 0; i < draws; ++i) (void)rng.Float64();
  // node naming: sort by name, rand.Perm prefix (simulator.go:577-588)
  const int nn = (int)t->nodes.size();
  const std::vector<int> perm = rng.Perm(nn);
  std::vector<std::string> full(nn);
  char buf[32];
  for (int i = 0; i < nn; ++i) {
    std::snprintf(buf, sizeof buf, "%04d-", perm[i]);
    full[i] = std::string(buf) + t->nodes[i].name;
  }
  std::vector<int> byname(nn);
  for (int i = 0; i < nn; ++i) byname[i] = i;
  std::sort(byname.begin(), byname.end(), [&](int a, int b) { return full[a] < full[b]; });
  for (int r = 0; r < nn; ++r) {
    const int i = byname[r];
    ksim_node& o = nodes[i];
    std::memset(&o, 0, sizeof o);
    o.cpu_alloc_milli = t->nodes[i].cpu;
    o.mem_alloc_mib = t->nodes[i].mem;
    o.pods_alloc = 1001;  // data/node_yaml/openb_node_list_gpu_node.yaml: allocatable pods
    o.gpu_count = t->nodes[i].gpu;
    o.gpu_type = t->node_type[i];
    o.name_rank = (uint32_t)r;
  }
  if (name_prefix)
    for (int i = 0; i < nn; ++i) name_prefix[i] = perm[i];
  if (rng_out) *rng_out = rng;  // the stream as the first scheduling cycle finds it
  if ((int)ev.size() > cap || !events) return KSIM_ERANGE;
  for (size_t k = 0; k < ev.size(); ++k) {
    events[k] = to_engine_pod(t->pods[ev[k]], t->pod_mask[ev[k]]);
    if (pod_index) pod_index[k] = ev[k];
  }
  return KSIM_OK;
}

int ksim_trace_replay(const ksim_trace* t, const ksim_replay_cfg* cfg, ksim_pod* events, int cap, int* n_events,
                      int32_t* pod_index, ksim_node* nodes, int32_t* name_prefix) {
  if (!t || !cfg || !n_events || !nodes) return KSIM_EINVAL;
  return replay_impl(t, cfg, events, cap, n_events, pod_index, nodes, name_prefix, nullptr);
}

int ksim_trace_replay_go_state(const ksim_trace* t, const ksim_replay_cfg* cfg, uint64_t* vec, int32_t* tap_feed,
                               int64_t* draws) {
  if (!t || !cfg || !vec || !tap_feed) return KSIM_EINVAL;
  int n = 0;
  std::vector<ksim_node> nodes(t->nodes.size() + 1);
  ksim_go::Rand rng(0);
  const int rc = replay_impl(t, cfg, nullptr, 0, &n, nullptr, nodes.data(), nullptr, &rng);
  if (rc != KSIM_OK && rc != KSIM_ERANGE) return rc;  // (ERANGE: no event buffer was asked for)
  int tap = 0, feed = 0;
  rng.State(vec, &tap, &feed);
  tap_feed[0] = tap;
  tap_feed[1] = feed;
  if (draws) *draws = (int64_t)rng.Draws();
  return KSIM_OK;
}

int ksim_trace_power_model(const ksim_trace* t, ksim_power_model* out) {
  if (!t || !out) return KSIM_EINVAL;
  std::memset(out, 0, sizeof *out);
  // const.go:62-69 MapGpuTypeEnergyConsumption via const.go:115-124 MapGpuTypeModelEnergy
  static const struct { const char* name; double idle, full; } kGpu[] = {
      {"T4", 10, 70}, {"A10", 30, 150}, {"P100", 25, 250}, {"V100M16", 30, 300},
      {"V100M32", 30, 300}, {"A100", 50, 400}, {"G2", 30, 150}, {"G3", 50, 400}};
  // const.go:48-55 MapCpuTypeEnergyConsumption
  static const struct { double idle, full, cores; } kCpu[] = {
      {15, 120, 16}, {20, 205, 26}, {20, 165, 24}, {15, 120, 16}, {20, 185, 16}, {20, 270, 32}};
  for (size_t v = 0; v < t->vocab.size() && v < (size_t)KSIM_MAX_TYPES; ++v) {
    if (t->vocab[v].empty()) { out->gpu_unlabelled |= 1u << v; continue; }
    for (const auto& g : kGpu)
      if (t->vocab[v] == g.name) {
        out->gpu_idle_w[v] = g.idle;
        out->gpu_full_w[v] = g.full;
        out->gpu_valid |= 1u << v;
      }
  }
  for (int c = 0; c < (int)(sizeof kCpu / sizeof kCpu[0]); ++c) {
    out->cpu_idle_w[c] = kCpu[c].idle;
    out->cpu_full_w[c] = kCpu[c].full;
    out->cpu_cores[c] = kCpu[c].cores;
    out->cpu_valid |= 1u << c;
  }
  return KSIM_OK;
}

int ksim_go_rand(int64_t seed, int op, int64_t arg, int n, int64_t* out) {
  if (n < 0 || (n > 0 && !out)) return KSIM_EINVAL;
  if ((op == KSIM_GO_INTN || op == KSIM_GO_PERM) && arg <= 0) return KSIM_EINVAL;
  ksim_go::Rand r(seed);
  switch (op) {
    case KSIM_GO_INT63:
      for (int i = 0; i < n; ++i) out[i] = r.Int63();
      return KSIM_OK;
    case KSIM_GO_INTN:
      for (int i = 0; i < n; ++i) out[i] = r.Intn(arg);
      return KSIM_OK;
    case KSIM_GO_FLOAT64:
      for (int i = 0; i < n; ++i) {
        const double f = r.Float64();
        std::memcpy(&out[i], &f, sizeof f);
      }
      return KSIM_OK;
    case KSIM_GO_PERM: {
      if (n < arg) return KSIM_ERANGE;
      const std::vector<int> m = r.Perm((int)arg);
      for (int64_t i = 0; i < arg; ++i) out[i] = m[i];
      return KSIM_OK;
    }
    case KSIM_GO_SHUFFLE: {
      for (int i = 0; i < n; ++i) out[i] = i;
      r.Shuffle(n, [&](int64_t i, int64_t j) { std::swap(out[i], out[j]); });
      return KSIM_OK;
    }
    default:
      return KSIM_EINVAL;
  }
}

}  // extern "C"

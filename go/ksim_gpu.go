// ksim_gpu.go -- the MI355X scoring engine as a kube-scheduler framework plugin of the simulator.
//
// Drop-in for Fr4nz83/kubernetes-scheduler-simulator @ 2024_08_07: copy this file to
// pkg/simulator/plugin/ and register it (see INTEGRATION.md §2).  It binds the C ABI of
// include/ksim_engine.h (libksim_hip.so) through cgo.  No Go toolchain exists in the build image,
// so this file is source only: written against the vendored framework
// (vendor/k8s.io/kubernetes/pkg/scheduler/framework/interface.go:257-407, cycle_state.go) and the
// reference's own accessors; tests/test_abi.py checks that every C.ksim_* it calls is declared.
//
// One plugin, KsimGpu, stands in for the Open-Gpu-Share Filter, one score plugin (FGDScore,
// BestFitScore, DotProductScore, GpuPackingScore, GpuClusteringScore, RandomScore or PWRScore)
// and the Reserve GPU selector:
//   PreFilter   one device call scores every node for the pod (ksim_engine_filter_score) and
//               stores the batch in CycleState (the framework calls Filter / Score 16-wide per
//               node, generic_scheduler.go:274-346, framework.go:635-710: they become lookups)
//   Filter      fitsRequest ∧ GpuSharePlugin.Filter (noderesources/fit.go:230-290,
//               open_gpu_share.go:81-118)
//   Score       the policy's Score; NormalizeScore as the reference's plugin does it
//               (plugin_utils.go:48-74 BestFit, pwr_score.go:104-141 PWR)
//   Reserve     allocateGpuId + Bind on the device (open_gpu_share.go:178-283), the gpu-index
//               annotation written as updatePodGpuAnno does (open_gpu_share.go:242-250)
//   Unreserve   removePod (open_gpu_share.go:208-218), and pod deletions through the informer's
//               DeleteFunc (open_gpu_share.go:58-70)
// The engine keeps the cluster state (CPU, memory, pods, per-GPU milli, affinity tags) on the
// device; it is built from the scheduler's snapshot at the first cycle, because the simulator
// creates its nodes after the plugins (simulator.go:185-193 vs :571-593).
package plugin

/*
#cgo CFLAGS: -I${SRCDIR}/../../../third_party/ksim/include
#cgo LDFLAGS: -L${SRCDIR}/../../../third_party/ksim/lib -lksim_hip -Wl,-rpath,${SRCDIR}/../../../third_party/ksim/lib
#include <stdlib.h>
#include "ksim_engine.h"
*/
import "C"

import (
	"context"
	"fmt"
	"sort"
	"strings"
	"sync"

	log "github.com/sirupsen/logrus"
	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/apimachinery/pkg/types"
	"k8s.io/client-go/tools/cache"
	resourcehelper "k8s.io/kubectl/pkg/util/resource"
	"k8s.io/kubernetes/pkg/scheduler/framework"
	frameworkruntime "k8s.io/kubernetes/pkg/scheduler/framework/runtime"
	schedulerutil "k8s.io/kubernetes/pkg/scheduler/util"

	simontype "github.com/hkust-adsl/kubernetes-scheduler-simulator/pkg/type"
	gpushareutils "github.com/hkust-adsl/kubernetes-scheduler-simulator/pkg/type/open-gpu-share/utils"
	"github.com/hkust-adsl/kubernetes-scheduler-simulator/pkg/utils"
)

const (
	KsimGpuPluginName                    = "KsimGpu"
	KsimGpuCompanionName                 = "KsimGpuCompanion"
	ksimStateKey      framework.StateKey = "PreFilter-" + KsimGpuPluginName
	mib                                  = int64(1) << 20
)

// The primary plugin of each scheduler framework, for its companion score plugin (same profile, same
// handle; the framework builds the two independently and in any order).
var ksimPrimaries sync.Map // framework.Handle -> *KsimGpuPlugin

// KsimGpuPluginCfg is the plugin's args in the scheduler configuration (pluginConfig), next to the
// reference's OpenGpuSharePluginCfg (pkg/type/config.go:50-61).
type KsimGpuPluginCfg struct {
	// Policy: the score plugin the engine computes, by its reference name (pkg/type/const.go:7-13).
	Policy string `json:"policy,omitempty"`
	// GpuSelMethod: Open-Gpu-Share's gpuSelMethod ("best", "worst", "random", "FGDScore", "PWRScore",
	// "DotProductScore").
	GpuSelMethod string `json:"gpuSelMethod,omitempty"`
	// DimExtMethod / NormMethod: DotProductScore's GpuPluginCfg (pkg/type/config.go:3-55); the
	// reference's harness gives the score plugin and Open-Gpu-Share the same values.
	simontype.GpuPluginCfg
	// Seed of the Random contract (RandomScore and the random GPU selector; DESIGN.md §4).
	Seed int64 `json:"seed,omitempty"`
	// WriteGpuIndex: patch the alibabacloud.com/gpu-index annotation in Reserve (set when
	// Open-Gpu-Share's Reserve is disabled; with it enabled it writes the same id itself).
	WriteGpuIndex bool `json:"writeGpuIndex,omitempty"`
	// Device: the HIP device ordinal.
	Device int `json:"device,omitempty"`
	// Companion: a second score plugin computed on the same device state, by its reference name (e.g.
	// "PWRScore" beside "FGDScore" for the fork's weighted "PWR 500 FGD 500" runs,
	// experiments/run_scripts/generate_run_scripts.py:31-42).  Its scores reach the framework through
	// the KsimGpuCompanion score plugin, which the scheduler configuration enables with the companion's
	// weight next to KsimGpu's; the framework then sums weight x normalized score per plugin as it does
	// for the reference's two plugins (framework.go:686-704).
	Companion string `json:"companion,omitempty"`
}

var ksimPolicies = map[string]C.int{
	simontype.FGDScorePluginName:           C.KSIM_POLICY_FGD,
	simontype.BestFitScorePluginName:       C.KSIM_POLICY_BESTFIT,
	simontype.DotProductScorePluginName:    C.KSIM_POLICY_DOTPROD,
	simontype.GpuPackingScorePluginName:    C.KSIM_POLICY_GPUPACKING,
	simontype.GpuClusteringScorePluginName: C.KSIM_POLICY_GPUCLUSTERING,
	simontype.RandomScorePluginName:        C.KSIM_POLICY_RANDOM,
	simontype.PWRScorePluginName:           C.KSIM_POLICY_PWR,
}

var ksimGpuSels = map[string]C.int{
	string(simontype.SelBestFitGpu):  C.KSIM_GPUSEL_BEST,
	string(simontype.SelWorstFitGpu): C.KSIM_GPUSEL_WORST,
	string(simontype.SelRandomGpu):   C.KSIM_GPUSEL_RANDOM,
	simontype.FGDScorePluginName:     C.KSIM_GPUSEL_FGD,
	simontype.PWRScorePluginName:     C.KSIM_GPUSEL_PWR,
	simontype.DotProductScorePluginName: C.KSIM_GPUSEL_DOTPROD,
}

var ksimDimExt = map[simontype.GpuDimExtMethod]C.int{
	simontype.MergeGpuDim:                     C.KSIM_DIMEXT_MERGE,
	simontype.SeparateGpuDimAndShareOtherDim:  C.KSIM_DIMEXT_SHARE,
	simontype.SeparateGpuDimAndDivideOtherDim: C.KSIM_DIMEXT_DIVIDE,
	simontype.ExtGpuDim:                       C.KSIM_DIMEXT_EXTEND,
}

var ksimNorm = map[simontype.NormMethod]C.int{
	simontype.NormByMax:  C.KSIM_NORM_MAX,
	simontype.NormByNode: C.KSIM_NORM_NODE,
	simontype.NormByPod:  C.KSIM_NORM_POD,
}

// The engine's CPU model ids: the order of the CPU table ksim_trace_power_model fills
// (pkg/type/open-gpu-share/utils/const.go:48-55 MapCpuTypeEnergyConsumption).
var ksimCpuModels = []string{"", "Intel-Xeon-8269CY", "Intel-Xeon-8163", "Intel-Xeon-ES-2682-V4", "Intel-Xeon-6326",
	"Intel-Xeon-8369B"}

// One cycle's device batch (the framework's CycleState carries it from PreFilter to Score).
type ksimCycle struct {
	feasible []C.uint8_t
	score    []C.int32_t
	gpuMask  []C.int32_t
	score2   []C.int32_t // the companion policy's scores (replica 1), when configured
	step     int32
}

func (s *ksimCycle) Clone() framework.StateData { return s }

// A pod bound through the engine: where, on which devices (Unreserve and deletions undo it).
type ksimBinding struct {
	node int
	mask int32
	pod  C.ksim_pod
}

type KsimGpuPlugin struct {
	sync.Mutex
	cfg         KsimGpuPluginCfg
	handle      framework.Handle
	typicalPods *simontype.TargetPodList
	policy      C.int
	gpuSel      C.int
	companion   C.int // the companion policy (replica 1 of the engine), -1 none

	eng   *C.ksim_engine
	names []string       // engine node index -> node name
	index map[string]int // node name -> engine node index
	vocab map[string]int // GPU model -> type id (bit of a type mask)
	bound map[types.UID]ksimBinding
	step  int32 // scheduling cycles so far (the Random contract's step)
}

var _ framework.PreFilterPlugin = &KsimGpuPlugin{}
var _ framework.FilterPlugin = &KsimGpuPlugin{}
var _ framework.ScorePlugin = &KsimGpuPlugin{}
var _ framework.ScoreExtensions = &KsimGpuPlugin{}
var _ framework.ReservePlugin = &KsimGpuPlugin{}

func ksimError(what string, rc C.int) error {
	return fmt.Errorf("ksim: %s: %s (%d)", what, C.GoString(C.ksim_strerror(rc)), int(rc))
}

// NewKsimGpuPlugin is the registry factory (simulator.go:153-181):
//
//	KsimGpuPluginName: func(cfg runtime.Object, h framework.Handle) (framework.Plugin, error) {
//		return simonplugin.NewKsimGpuPlugin(cfg, h, &sim.typicalPods)
//	},
func NewKsimGpuPlugin(configuration runtime.Object, handle framework.Handle,
	typicalPods *simontype.TargetPodList) (framework.Plugin, error) {
	cfg := KsimGpuPluginCfg{Policy: simontype.FGDScorePluginName, GpuSelMethod: simontype.FGDScorePluginName}
	if configuration != nil {
		if err := frameworkruntime.DecodeInto(configuration, &cfg); err != nil {
			return nil, err
		}
	}
	policy, ok := ksimPolicies[cfg.Policy]
	if !ok {
		return nil, fmt.Errorf("ksim: unknown policy %q", cfg.Policy)
	}
	gpuSel, ok := ksimGpuSels[cfg.GpuSelMethod]
	if !ok {
		return nil, fmt.Errorf("ksim: unknown gpuSelMethod %q", cfg.GpuSelMethod)
	}
	if C.ksim_abi_version() != C.KSIM_ABI_VERSION {
		return nil, fmt.Errorf("ksim: library ABI %d, built against %d", int(C.ksim_abi_version()), C.KSIM_ABI_VERSION)
	}
	if C.ksim_device_count() <= C.int(cfg.Device) { // no CPU fallback: fail at construction
		return nil, ksimError("device", C.KSIM_ENODEV)
	}
	companion := C.int(-1)
	if cfg.Companion != "" {
		c, ok := ksimPolicies[cfg.Companion]
		if !ok {
			return nil, fmt.Errorf("ksim: unknown companion policy %q", cfg.Companion)
		}
		companion = c
	}
	p := &KsimGpuPlugin{cfg: cfg, handle: handle, typicalPods: typicalPods, policy: policy, gpuSel: gpuSel,
		companion: companion, index: map[string]int{}, vocab: map[string]int{}, bound: map[types.UID]ksimBinding{}}
	ksimPrimaries.Store(handle, p)
	// a deleted pod leaves its node (informer DeleteFunc, open_gpu_share.go:58-70; the scheduler cache
	// releases its cpu / memory, simulator.go:416-422): the device state follows
	handle.SharedInformerFactory().Core().V1().Pods().Informer().AddEventHandler(cache.ResourceEventHandlerFuncs{
		DeleteFunc: func(obj interface{}) {
			if pod, ok := obj.(*v1.Pod); ok {
				p.Lock()
				defer p.Unlock()
				if err := p.release(pod); err != nil {
					log.Errorf("ksim: removePod (%s/%s): %s", pod.Namespace, pod.Name, err)
				}
			}
		}})
	return p, nil
}

func (p *KsimGpuPlugin) Name() string { return KsimGpuPluginName }

// typeID: the engine's id of a GPU model (KSIM_MAX_TYPES ids; a pod may name models no node has).
func (p *KsimGpuPlugin) typeID(model string) (int, error) {
	if id, ok := p.vocab[model]; ok {
		return id, nil
	}
	if len(p.vocab) >= C.KSIM_MAX_TYPES {
		return 0, fmt.Errorf("ksim: more than %d GPU models", C.KSIM_MAX_TYPES)
	}
	p.vocab[model] = len(p.vocab)
	return p.vocab[model], nil
}

// typeMask: the models a pod accepts, from its gpu-card-model pipe list; empty = any
// (IsNodeAccessibleToPodByType, pkg/utils/utils.go:957-1006).
func (p *KsimGpuPlugin) typeMask(spec string) (C.uint32_t, error) {
	if spec == "" {
		return C.KSIM_TYPE_ANY, nil
	}
	var m uint32
	for _, model := range strings.Split(spec, "|") {
		id, err := p.typeID(model)
		if err != nil {
			return 0, err
		}
		m |= 1 << uint(id)
	}
	return C.uint32_t(m), nil
}

func cpuModelID(model string) int {
	for i, m := range ksimCpuModels {
		if m == model {
			return i
		}
	}
	return len(ksimCpuModels) // outside the power model's cpu_valid: the PWR Score fails, as the reference's nil map
}

// toKsimPod: the Filter request (fit.go computePodResourceRequest via PodRequestsAndLimits) and
// the Score request (GetPodResource, pkg/utils/utils.go:1008-1029: non-zero CPU default).
func (p *KsimGpuPlugin) toKsimPod(pod *v1.Pod) (C.ksim_pod, error) {
	reqs, _ := resourcehelper.PodRequestsAndLimits(pod)
	res := utils.GetPodResource(pod)
	mem := reqs.Memory().Value()
	if mem%mib != 0 { // the engine counts memory in MiB; the traces' requests are whole MiB
		return C.ksim_pod{}, fmt.Errorf("ksim: pod %s/%s memory request %d B is not a whole MiB", pod.Namespace, pod.Name, mem)
	}
	mask, err := p.typeMask(res.GpuType)
	if err != nil {
		return C.ksim_pod{}, err
	}
	return C.ksim_pod{cpu_milli: C.int64_t(reqs.Cpu().MilliValue()), cpu_nz_milli: C.int64_t(res.MilliCpu),
		mem_mib: C.int64_t(mem / mib), gpu_milli: C.int32_t(res.MilliGpu), gpu_count: C.int32_t(res.GpuNumber),
		type_mask: mask, ref: -1}, nil
}

// gpuIndexString: "i" or "i-j-k" (DevIdSep, open-gpu-share/utils/const.go:13), ascending device ids.
func gpuIndexString(mask int32) string {
	var ids []string
	for g := 0; g < C.KSIM_MAX_GPU; g++ {
		if mask&(1<<uint(g)) != 0 {
			ids = append(ids, fmt.Sprint(g))
		}
	}
	return strings.Join(ids, gpushareutils.DevIdSep)
}

// maskFromGpuIndexAnnotation: the devices a pod's gpu-index annotation names (GpuIdStrToIntList,
// open-gpu-share/utils/pod.go:148-162); ok = false when it has none.
func maskFromGpuIndexAnnotation(pod *v1.Pod) (mask int32, ok bool, err error) {
	idl, err := gpushareutils.GetGpuIdListFromAnnotation(pod)
	if err != nil || len(idl) == 0 {
		return 0, false, err
	}
	for _, id := range idl {
		if id < 0 || id >= C.KSIM_MAX_GPU {
			return 0, false, fmt.Errorf("ksim: gpu-index %d out of range", id)
		}
		mask |= 1 << uint(id)
	}
	return mask, true, nil
}

// affinityTag: the GpuClustering tag of a pod (GetGpuAffinityFromPodAnnotation, pod.go:111-123) as
// the engine's tag index: 0 share-gpu, k k-gpu, -1 no-gpu.
func affinityTag(pod *v1.Pod) int {
	switch tag := gpushareutils.GetGpuAffinityFromPodAnnotation(pod); tag {
	case gpushareutils.NoGpuTag:
		return -1
	case gpushareutils.ShareGpuTag:
		return 0
	default:
		var k int
		fmt.Sscanf(tag, "%d-gpu", &k)
		return k
	}
}

// ensureEngine builds the engine from the scheduler's snapshot at the first cycle: every node, its
// allocatable and what its pods already hold (GetNodeResourceViaNodeInfo, utils.go:1053-1148), the
// name ranks of selectHost's byte-wise tie-break (generic_scheduler.go:187-212), the typical pods.
func (p *KsimGpuPlugin) ensureEngine() error {
	infos, err := p.handle.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return err
	}
	if p.eng != nil {
		if len(infos) != len(p.names) {
			return fmt.Errorf("ksim: the node set changed (%d -> %d nodes)", len(p.names), len(infos))
		}
		return nil
	}
	if len(infos) == 0 {
		return fmt.Errorf("ksim: no nodes")
	}
	names := make([]string, len(infos))
	for i, ni := range infos {
		names[i] = ni.Node().Name
	}
	byName := append([]string(nil), names...)
	sort.Strings(byName) // Go compares strings byte-wise, as selectHost does
	rank := map[string]int{}
	for r, n := range byName {
		rank[n] = r
	}
	cn := make([]C.ksim_node, len(infos))
	for i, ni := range infos {
		node := ni.Node()
		gpus := gpushareutils.GetGpuCountOfNode(node)
		if gpus > C.KSIM_MAX_GPU {
			return fmt.Errorf("ksim: node %s has %d GPUs", node.Name, gpus)
		}
		tid := 0
		if gpus > 0 {
			if tid, err = p.typeID(gpushareutils.GetGpuModelOfNode(node)); err != nil {
				return err
			}
		}
		n := C.ksim_node{cpu_alloc_milli: C.int64_t(ni.Allocatable.MilliCPU),
			mem_alloc_mib: C.int64_t(ni.Allocatable.Memory / mib), pods_alloc: C.int32_t(ni.Allocatable.AllowedPodNumber),
			gpu_count: C.int32_t(gpus), gpu_type: C.int32_t(tid), name_rank: C.uint32_t(rank[node.Name]),
			cpu_used_milli: C.int64_t(ni.Requested.MilliCPU), mem_used_mib: C.int64_t(ni.Requested.Memory / mib),
			pods_used: C.int32_t(len(ni.Pods)), cpu_model: C.int32_t(cpuModelID(gpushareutils.GetCpuModelOfNode(node)))}
		for _, pi := range ni.Pods { // the devices and affinity tags of the pods already there
			milli := gpushareutils.GetGpuMilliFromPodAnnotation(pi.Pod)
			if mask, ok, _ := maskFromGpuIndexAnnotation(pi.Pod); ok && milli > 0 {
				for g := 0; g < C.KSIM_MAX_GPU; g++ {
					if mask&(1<<uint(g)) != 0 {
						n.gpu_used_milli[g] += C.int32_t(milli)
					}
				}
			}
			if tag := affinityTag(pi.Pod); tag >= 0 {
				n.tag_count[tag]++
			}
		}
		cn[i] = n
	}
	var eng *C.ksim_engine
	cfg := C.ksim_config{device: C.int32_t(p.cfg.Device)}
	replicas := 1
	if p.companion >= 0 {
		replicas = 2
	}
	if rc := C.ksim_engine_create(&cfg, C.int(len(infos)), C.int(replicas), &eng); rc != 0 {
		return ksimError("create", rc)
	}
	fail := func(what string, rc C.int) error {
		C.ksim_engine_destroy(eng)
		return ksimError(what, rc)
	}
	if rc := C.ksim_engine_set_nodes(eng, 0, &cn[0]); rc != 0 {
		return fail("set_nodes", rc)
	}
	// the target workload (GetTypicalPods, frag.go:285-380; core.go:110 SetTypicalPods)
	var ct []C.ksim_typical
	if p.typicalPods != nil && len(*p.typicalPods) > 0 {
		ct = make([]C.ksim_typical, len(*p.typicalPods))
		for i, t := range *p.typicalPods {
			mask, err := p.typeMask(t.TargetPodResource.GpuType)
			if err != nil {
				C.ksim_engine_destroy(eng)
				return err
			}
			ct[i] = C.ksim_typical{cpu_milli: C.int64_t(t.TargetPodResource.MilliCpu),
				gpu_milli: C.int32_t(t.TargetPodResource.MilliGpu), gpu_count: C.int32_t(t.TargetPodResource.GpuNumber),
				type_mask: mask, freq: C.double(t.Percentage)}
		}
		if rc := C.ksim_engine_set_typical(eng, 0, &ct[0], C.int(len(ct))); rc != 0 {
			return fail("set_typical", rc)
		}
	}
	if rc := C.ksim_engine_set_policy(eng, 0, p.policy, p.gpuSel, C.uint64_t(p.cfg.Seed)); rc != 0 {
		return fail("set_policy", rc)
	}
	if err := p.setupPolicy(eng, 0, p.policy); err != nil {
		C.ksim_engine_destroy(eng)
		return err
	}
	if p.companion >= 0 { // replica 1: the same cluster under the companion's score
		if rc := C.ksim_engine_set_nodes(eng, 1, &cn[0]); rc != 0 {
			return fail("set_nodes", rc)
		}
		if len(ct) > 0 {
			if rc := C.ksim_engine_set_typical(eng, 1, &ct[0], C.int(len(ct))); rc != 0 {
				return fail("set_typical", rc)
			}
		}
		if rc := C.ksim_engine_set_policy(eng, 1, p.companion, C.KSIM_GPUSEL_BEST, C.uint64_t(p.cfg.Seed)); rc != 0 {
			return fail("set_policy", rc)
		}
		if err := p.setupPolicy(eng, 1, p.companion); err != nil {
			C.ksim_engine_destroy(eng)
			return err
		}
	}
	p.eng, p.names = eng, names
	for i, n := range names {
		p.index[n] = i
	}
	return nil
}

// setupPolicy: the per-policy configuration of one engine replica -- DotProduct's GpuPluginCfg
// (GenerateSchedulingMatchGroups' cfg, utils.go:1274-1342; an empty or unknown method is an error, as
// the reference panics on it, resource.go:290,377) and PWR's energy model.
func (p *KsimGpuPlugin) setupPolicy(eng *C.ksim_engine, r C.int, policy C.int) error {
	if policy == C.KSIM_POLICY_DOTPROD {
		dim, ok := ksimDimExt[p.cfg.DimExtMethod]
		if !ok {
			return fmt.Errorf("ksim: undefined gpu dimension extension method: %q", p.cfg.DimExtMethod)
		}
		norm, ok := ksimNorm[p.cfg.NormMethod]
		if !ok {
			return fmt.Errorf("ksim: undefined normalization for dot product: %q", p.cfg.NormMethod)
		}
		if rc := C.ksim_engine_set_plugin_cfg(eng, r, dim, norm); rc != 0 {
			return ksimError("set_plugin_cfg", rc)
		}
	}
	if policy == C.KSIM_POLICY_PWR {
		pm := p.powerModel()
		if rc := C.ksim_engine_set_power_model(eng, r, &pm); rc != 0 {
			return ksimError("set_power_model", rc)
		}
	}
	return nil
}

// powerModel: GetEnergyConsumptionNode's tables (resource.go:536-563) for the engine's model ids:
// each GPU model's idle / full watts are its MapGpuTypeModelEnergy function at one idle / one busy GPU
// (const.go:70-124), the CPU models' from MapCpuTypeEnergyConsumption (const.go:48-55).
func (p *KsimGpuPlugin) powerModel() C.ksim_power_model {
	var pm C.ksim_power_model
	for model, id := range p.vocab {
		if model == "" {
			pm.gpu_unlabelled |= 1 << uint(id)
			continue
		}
		if f, ok := gpushareutils.MapGpuTypeModelEnergy[model]; ok {
			pm.gpu_idle_w[id] = C.double(f(1, 0))
			pm.gpu_full_w[id] = C.double(f(0, 1))
			pm.gpu_valid |= 1 << uint(id)
		}
	}
	for id, model := range ksimCpuModels {
		e := gpushareutils.MapCpuTypeEnergyConsumption[model]
		pm.cpu_idle_w[id], pm.cpu_full_w[id], pm.cpu_cores[id] = C.double(e["idle"]), C.double(e["full"]), C.double(e["ncores"])
		pm.cpu_valid |= 1 << uint(id)
	}
	return pm
}

// PreFilter: the cycle's device batch -- Filter and Score of every node for this pod.
func (p *KsimGpuPlugin) PreFilter(ctx context.Context, state *framework.CycleState, pod *v1.Pod) *framework.Status {
	p.Lock()
	defer p.Unlock()
	if err := p.ensureEngine(); err != nil {
		return framework.AsStatus(err)
	}
	cp, err := p.toKsimPod(pod)
	if err != nil {
		return framework.AsStatus(err)
	}
	n := len(p.names)
	s := &ksimCycle{feasible: make([]C.uint8_t, n), score: make([]C.int32_t, n), gpuMask: make([]C.int32_t, n), step: p.step}
	p.step++
	if rc := C.ksim_engine_filter_score(p.eng, 0, &cp, C.int32_t(s.step), &s.feasible[0], &s.score[0], &s.gpuMask[0]); rc != 0 {
		return framework.AsStatus(ksimError("filter_score", rc))
	}
	if p.companion >= 0 {
		s.score2 = make([]C.int32_t, n)
		feas2, gpu2 := make([]C.uint8_t, n), make([]C.int32_t, n)
		if rc := C.ksim_engine_filter_score(p.eng, 1, &cp, C.int32_t(s.step), &feas2[0], &s.score2[0], &gpu2[0]); rc != 0 {
			return framework.AsStatus(ksimError("filter_score", rc))
		}
	}
	state.Write(ksimStateKey, s)
	return framework.NewStatus(framework.Success)
}

func (p *KsimGpuPlugin) PreFilterExtensions() framework.PreFilterExtensions { return nil }

func cycleOf(state *framework.CycleState) (*ksimCycle, *framework.Status) {
	c, err := state.Read(ksimStateKey)
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	s, ok := c.(*ksimCycle)
	if !ok {
		return nil, framework.NewStatus(framework.Error, "ksim: bad cycle state")
	}
	return s, nil
}

// Filter: fitsRequest ∧ the GPU-share fit, as computed for this node in PreFilter.
func (p *KsimGpuPlugin) Filter(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeInfo *framework.NodeInfo) *framework.Status {
	s, st := cycleOf(state)
	if st != nil {
		return st
	}
	i, ok := p.index[nodeInfo.Node().Name]
	if !ok {
		return framework.NewStatus(framework.Error, "ksim: unknown node "+nodeInfo.Node().Name)
	}
	if s.feasible[i] == 0 {
		return framework.NewStatus(framework.Unschedulable, "Node:"+nodeInfo.Node().Name)
	}
	return framework.NewStatus(framework.Success)
}

// Score: the policy's score of this node (before NormalizeScore).
func (p *KsimGpuPlugin) Score(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeName string) (int64, *framework.Status) {
	s, st := cycleOf(state)
	if st != nil {
		return 0, st
	}
	i, ok := p.index[nodeName]
	if !ok {
		return 0, framework.NewStatus(framework.Error, "ksim: unknown node "+nodeName)
	}
	if p.policy == C.KSIM_POLICY_RANDOM {
		// the reference's draw: RandomScorePlugin.PreScore, which the simulator enables in every profile
		// (pkg/simulator/utils.go:241-248), picked rand.Intn(len(nodes)) over the framework's feasible list
		// on Go's global math/rand (random_score.go:42-51); Score gives that node 100
		// (random_score.go:53-68) -- the same stream, the same draw, nothing drawn twice
		c, err := state.Read(preScoreStateKey)
		if err != nil {
			return 0, framework.AsStatus(fmt.Errorf("reading %q from cycleState: %w", preScoreStateKey, err))
		}
		ps, ok := c.(*preScoreState)
		if !ok {
			return 0, framework.NewStatus(framework.Error, "ksim: bad RandomScore pre-score state")
		}
		if nodeName == ps.nodeName {
			return framework.MaxNodeScore, framework.NewStatus(framework.Success)
		}
		return framework.MinNodeScore, framework.NewStatus(framework.Success)
	}
	return int64(s.score[i]), framework.NewStatus(framework.Success)
}

// ScoreExtensions: the policies whose reference plugin normalizes (BestFit: best_fit_score.go:55-61
// -> NormalizeScore; PWR: pwr_score.go:100-141) get the same normalization.
func (p *KsimGpuPlugin) ScoreExtensions() framework.ScoreExtensions {
	if p.policy == C.KSIM_POLICY_BESTFIT || p.policy == C.KSIM_POLICY_PWR {
		return p
	}
	return nil
}

func (p *KsimGpuPlugin) NormalizeScore(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	scores framework.NodeScoreList) *framework.Status {
	if p.policy == C.KSIM_POLICY_PWR {
		return (&PWRScorePlugin{}).NormalizeScore(ctx, state, pod, scores)
	}
	return NormalizeScore(scores)
}

// Reserve: allocateGpuId on the chosen node (the replica's gpuSelMethod, or the devices a predefined
// gpu-index names) and the Bind on the device; the gpu-index annotation as updatePodGpuAnno writes it.
func (p *KsimGpuPlugin) Reserve(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeName string) *framework.Status {
	p.Lock()
	defer p.Unlock()
	i, ok := p.index[nodeName]
	if !ok {
		return framework.NewStatus(framework.Error, "ksim: unknown node "+nodeName)
	}
	cp, err := p.toKsimPod(pod)
	if err != nil {
		return framework.AsStatus(err)
	}
	step := p.step - 1
	if s, st := cycleOf(state); st == nil {
		step = s.step
	}
	var mask C.int32_t
	if pre, ok, err := maskFromGpuIndexAnnotation(pod); err != nil {
		return framework.AsStatus(err)
	} else if ok && cp.gpu_milli > 0 { // open_gpu_share.go:260-271: a predefined id is kept
		mask = C.int32_t(pre)
		if rc := C.ksim_engine_bind(p.eng, 0, &cp, C.int(i), mask); rc != 0 {
			return framework.AsStatus(ksimError("bind", rc))
		}
	} else if p.gpuSel == C.KSIM_GPUSEL_RANDOM && cp.gpu_milli > 0 {
		// allocateGpuIdBasedOnRandomFit itself (open_gpu_share.go:325-343): its rand.Intn per fitting GPU
		// on Go's global math/rand, over the node's devices as the engine holds them.  With this selector
		// Open-Gpu-Share's reserve must be disabled (writeGpuIndex: true) or the stream is drawn twice.
		m, err := p.randomFitMask(i, pod)
		if err != nil {
			return framework.AsStatus(err)
		}
		mask = C.int32_t(m)
		if rc := C.ksim_engine_bind(p.eng, 0, &cp, C.int(i), mask); rc != 0 {
			return framework.AsStatus(ksimError("bind", rc))
		}
	} else if rc := C.ksim_engine_reserve(p.eng, 0, &cp, C.int(i), C.int32_t(step), &mask); rc != 0 {
		// allocateGpuId returned "": updatePodGpuAnno's error (open_gpu_share.go:242-247)
		return framework.NewStatus(framework.Error, fmt.Sprintf("failed to allocate gpu to pod(%s) to node(%s)",
			utils.GeneratePodKey(pod), nodeName))
	}
	if p.companion >= 0 { // the companion's replica follows the same Bind
		if rc := C.ksim_engine_bind(p.eng, 1, &cp, C.int(i), mask); rc != 0 {
			_ = C.ksim_engine_unreserve(p.eng, 0, &cp, C.int(i), mask)
			return framework.AsStatus(ksimError("bind", rc))
		}
	}
	p.bound[pod.UID] = ksimBinding{node: i, mask: int32(mask), pod: cp}
	if p.cfg.WriteGpuIndex && cp.gpu_milli > 0 {
		podCopy := gpushareutils.UpdatePodDeviceAnnoSpec(pod, gpuIndexString(int32(mask)))
		if err := schedulerutil.PatchPod(p.handle.ClientSet(), pod, podCopy); err != nil {
			_ = p.release(pod)
			return framework.AsStatus(err)
		}
	}
	return framework.NewStatus(framework.Success)
}

// Unreserve: undo Reserve (removePod, open_gpu_share.go:208-218).
func (p *KsimGpuPlugin) Unreserve(ctx context.Context, state *framework.CycleState, pod *v1.Pod, nodeName string) {
	p.Lock()
	defer p.Unlock()
	if err := p.release(pod); err != nil {
		log.Errorf("ksim: unreserve (%s) on %s: %s", utils.GeneratePodKey(pod), nodeName, err)
	}
}

// release: the pod leaves the node it was bound to through this plugin (caller holds the lock).
func (p *KsimGpuPlugin) release(pod *v1.Pod) error {
	b, ok := p.bound[pod.UID]
	if !ok {
		return nil
	}
	delete(p.bound, pod.UID)
	if rc := C.ksim_engine_unreserve(p.eng, 0, &b.pod, C.int(b.node), C.int32_t(b.mask)); rc != 0 {
		return ksimError("unreserve", rc)
	}
	if p.companion >= 0 {
		if rc := C.ksim_engine_unreserve(p.eng, 1, &b.pod, C.int(b.node), C.int32_t(b.mask)); rc != 0 {
			return ksimError("unreserve", rc)
		}
	}
	return nil
}

// randomFitMask: the random GPU selector on node i (caller holds the lock): the reference's own
// allocateGpuIdBasedOnRandomFit over the node's per-device milli left read back from the engine.
func (p *KsimGpuPlugin) randomFitMask(i int, pod *v1.Pod) (int32, error) {
	nodes := make([]C.ksim_node, len(p.names))
	if rc := C.ksim_engine_get_nodes(p.eng, 0, &nodes[0]); rc != 0 {
		return 0, ksimError("get_nodes", rc)
	}
	n := nodes[i]
	left := make([]int64, int(n.gpu_count))
	for g := range left {
		left[g] = int64(gpushareutils.MILLI) - int64(n.gpu_used_milli[g])
	}
	nodeRes := simontype.NodeResource{NodeName: p.names[i], MilliCpuLeft: int64(n.cpu_alloc_milli - n.cpu_used_milli),
		MilliCpuCapacity: int64(n.cpu_alloc_milli), MilliGpuLeftList: left, GpuNumber: int(n.gpu_count)}
	id := allocateGpuIdBasedOnRandomFit(nodeRes, utils.GetPodResource(pod), p.cfg.GpuPluginCfg, p.typicalPods)
	if id == "" {
		return 0, fmt.Errorf("failed to allocate gpu to pod(%s) to node(%s)", utils.GeneratePodKey(pod), p.names[i])
	}
	idl, err := gpushareutils.GpuIdStrToIntList(id)
	if err != nil {
		return 0, err
	}
	var mask int32
	for _, g := range idl {
		mask |= 1 << uint(g)
	}
	return mask, nil
}

// KsimGpuCompanion: the companion score plugin -- the second score of a weighted pair (KsimGpuPluginCfg.
// Companion), computed by the primary KsimGpu plugin in the same PreFilter batch on the same device
// state.  Registry entry (simulator.go:153-181):
//
//	KsimGpuCompanionName: func(cfg runtime.Object, h framework.Handle) (framework.Plugin, error) {
//		return simonplugin.NewKsimGpuCompanion(cfg, h)
//	},
type KsimGpuCompanion struct {
	handle framework.Handle
}

var _ framework.ScorePlugin = &KsimGpuCompanion{}
var _ framework.ScoreExtensions = &KsimGpuCompanion{}

func NewKsimGpuCompanion(_ runtime.Object, handle framework.Handle) (framework.Plugin, error) {
	return &KsimGpuCompanion{handle: handle}, nil
}

func (c *KsimGpuCompanion) Name() string { return KsimGpuCompanionName }

func (c *KsimGpuCompanion) primary() (*KsimGpuPlugin, *framework.Status) {
	v, ok := ksimPrimaries.Load(c.handle)
	if !ok {
		return nil, framework.NewStatus(framework.Error, "ksim: KsimGpuCompanion without a KsimGpu plugin in the profile")
	}
	p := v.(*KsimGpuPlugin)
	if p.companion < 0 {
		return nil, framework.NewStatus(framework.Error, "ksim: KsimGpu has no companion policy configured")
	}
	return p, nil
}

// Score: the companion policy's score of this node (before its NormalizeScore).
func (c *KsimGpuCompanion) Score(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	nodeName string) (int64, *framework.Status) {
	p, st := c.primary()
	if st != nil {
		return 0, st
	}
	s, st := cycleOf(state)
	if st != nil {
		return 0, st
	}
	i, ok := p.index[nodeName]
	if !ok || s.score2 == nil {
		return 0, framework.NewStatus(framework.Error, "ksim: no companion score for node "+nodeName)
	}
	return int64(s.score2[i]), framework.NewStatus(framework.Success)
}

func (c *KsimGpuCompanion) ScoreExtensions() framework.ScoreExtensions { return c }

// NormalizeScore: the companion policy's own (PWR: pwr_score.go:100-141; BestFit: plugin_utils.go:48-74;
// the others keep their raw scores).
func (c *KsimGpuCompanion) NormalizeScore(ctx context.Context, state *framework.CycleState, pod *v1.Pod,
	scores framework.NodeScoreList) *framework.Status {
	p, st := c.primary()
	if st != nil {
		return st
	}
	switch p.companion {
	case C.KSIM_POLICY_PWR:
		return (&PWRScorePlugin{}).NormalizeScore(ctx, state, pod, scores)
	case C.KSIM_POLICY_BESTFIT:
		return NormalizeScore(scores)
	}
	return framework.NewStatus(framework.Success)
}

#!/bin/bash
# Builds the k_memo micro-benchmark (one wave, cycle counts) next to this script.
set -e
cd "$(dirname "$0")/../.."
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -munsafe-fp-atomics \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -I include -I kubernetes-scheduler-simulator_amd/csrc \
  scripts/ubench/ubench_memo.hip -o scripts/ubench/ubench_memo

#!/bin/bash
# Counter passes for the bench configurations named on the command line (profile_key() in bench.py):
#   bash scripts/profile_all.sh c2 c2-rm5 c2-BestFit c4 c5
# each -> gpurun_out/prof/<name>/{pmc.json,kernel_stats.csv,*.log}; copy them to profiles/r03/prof/.
set -u
cd "$(dirname "$0")/.."
for name in "$@"; do
  case $name in
    c2) a="";;
    c2-rm5) a="--run-mode 5";;
    c2-rm2) a="--run-mode 2";;
    c2-BestFit) a="--policy BestFit";;
    c2-PWR) a="--policy PWR";;
    c2-PWR_500_FGD_500) a="--policy PWR_500_FGD_500";;
    c2-DotProd) a="--policy DotProd";;
    c2-report) a="--report";;
    c2-Random-go) a="--policy Random --random-stream go";;
    c4) a="--config c4";;
    c5) a="--config c5";;
    *) echo "unknown configuration $name"; exit 2;;
  esac
  bash scripts/profile_config.sh $name $a || exit 1
done

#!/bin/bash
# r04: the key-store timing experiment (scripts/r04_check12.sh), then the final counter passes
# (scripts/r04_prof2.sh).
set -u
cd "$(dirname "$0")/.."
bash scripts/r04_check12.sh || exit $?
bash scripts/r04_prof2.sh

#!/bin/bash
# Build a committed revision's package (default HEAD) into ab_alt/, an A/B baseline the GPU box can
# run next to the working tree's build in the same gpurun call (boxes differ by up to ~10%):
#   ab_alt/bench.py              the revision's headline bench (imports ab_alt/mpi_cuda_process_amd)
#   ab_alt/bench/kernel_ab.py    its kernel A/B harness
# usage: scripts/make_ab_alt.sh [REV]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
rm -rf /tmp/ab_alt_wt ab_alt
git worktree add -q /tmp/ab_alt_wt "$REV"
(cd /tmp/ab_alt_wt && make -j8 lib pymod >/dev/null)
mkdir -p ab_alt/bench
cp -r /tmp/ab_alt_wt/mpi_cuda_process_amd ab_alt/
cp /tmp/ab_alt_wt/bench/kernel_ab.py ab_alt/bench/
cp /tmp/ab_alt_wt/bench.py ab_alt/
git worktree remove --force /tmp/ab_alt_wt
echo "ab_alt/ = $(git rev-parse --short "$REV")"

#!/bin/bash
# Build the committed HEAD's package into ab_alt/ (an A/B baseline the GPU box can run next to the
# working tree's build): ab_alt/bench/kernel_ab.py imports ab_alt/mpi_cuda_process_amd.
set -e
cd "$(dirname "$0")/.."
rm -rf /tmp/ab_alt_wt ab_alt
git worktree add -q /tmp/ab_alt_wt HEAD
(cd /tmp/ab_alt_wt && make -j8 lib pymod >/dev/null)
mkdir -p ab_alt/bench
cp -r /tmp/ab_alt_wt/mpi_cuda_process_amd ab_alt/
cp /tmp/ab_alt_wt/bench/kernel_ab.py ab_alt/bench/
git worktree remove --force /tmp/ab_alt_wt
echo "ab_alt/ = $(git rev-parse --short HEAD)"

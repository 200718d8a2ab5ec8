#!/bin/bash
# Full CMake build + native tests (CPU), as an alternative to the Makefile.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=${1:-$R/build-cmake}
cmake -S "$R" -B "$B" -G Ninja -DCMAKE_HIP_ARCHITECTURES=gfx950
cmake --build "$B" -j"${MAX_JOBS:-8}"
HIP_VISIBLE_DEVICES= ctest --test-dir "$B" --output-on-failure

#!/bin/bash
# After swapping __syncthreads for the LDS-only barrier: the configs whose kernels changed.
B="python bench.py"
LIMIT=200 bash "$(dirname "$0")/gpu_session.sh" \
 "nb_b27=$B --stencil box27 --n 512 --steps 100 --warmup 10" \
 "nb_b27d=$B --stencil box27 --n 512 --dtype f64 --steps 50 --warmup 5" \
 "nb_f64=$B --n 2048 --dtype f64 --steps 20 --warmup 2 --residual-every 10" \
 "nb_t1=$B --temporal 1" "nb_b27_t1=$B --stencil box27 --n 512 --temporal 1 --steps 100 --warmup 10" \
 "nb_cube=$B"

#!/bin/bash
# Round 5, session Y: the BASELINE configs that K = 5 changes (1024^3 default form, 512^3, 3072^3,
# the N = 2 / 4 / 8 rank proxies), then the 8-process shared-GPU rehearsal of the N = 8 bench.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05y
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  echo "$tag $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; v=c.get('verified'); print(r['value'], r['ms_per_step'], c.get('temporal_block'), r.get('measured_copy_TBps'), v.get('max_abs_diff') if isinstance(v, dict) else v)" $O/$tag.json)"; }
run default
run driver --gpus 1 --steps 20 --warmup 5
run heat512 --n 512 --steps 100 --warmup 10
run heat3072 --n 3072 --steps 20 --warmup 5
run p2 --rank-proxy 2 --steps 50 --warmup 10
run p4 --rank-proxy 4 --steps 50 --warmup 10
run p8 --rank-proxy 8 --steps 50 --warmup 10
timeout -k 10 600 python bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $O/rehearsal8.json 2> $O/rehearsal8.err || { tail -20 $O/rehearsal8.err; exit 1; }
grep -o '"value": [0-9.]*\|"transport": "[a-z_]*"\|"verified": {[^}]*}\|"repeats_ms_per_step": \[[^]]*\]\|"temporal_block": [0-9]*' $O/rehearsal8.json | head -6

#!/bin/bash
# torchrun launch of the bench (the driver's N > 1 form) with 2 and 4 ranks sharing the one GPU of a
# gpurun box: rccl fails its gate there (two ranks on one device), ipc passes and is timed.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) \
    bench.py --gpus $n --share-gpu --steps 20 --warmup 5 --timeout 60 > gpurun_out/torchrun_$n.log 2>&1 || { tail -30 gpurun_out/torchrun_$n.log; exit 1; }
  grep '^{' gpurun_out/torchrun_$n.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print($n, r['value'], r['config']['transport'], r['config']['overlap'], r['config']['graph'], [(g['transport'], g['graph'], g['passed']) for g in r['config']['gate']['runs']])"
done

#!/bin/bash
# RCCL world-1 line under queue / plan-CU variants (name:ENV=V ...)
set -o pipefail
O=gpurun_out/r4pgq2; mkdir -p $O
for v in "$@"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --force-pg --backend nccl --no-cpu-baseline --consumer-msgs 0 --e2e-steps 0 --no-phase-pass \
    > $O/$n.jsonl 2> $O/$n.log || { tail -20 $O/$n.log; exit 5; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d['hot_book']['ns_per_order'], (d.get('publisher') or {}).get('digest_check'))" $O/$n.jsonl $n
done

#!/bin/bash
# RCCL line (nccl at world 1) and the plain line at 8 / 16 hardware queues.
set -o pipefail
O=gpurun_out/${1:-r4pq}
mkdir -p $O
for q in 8 16; do
  GOME_HW_QUEUES=$q timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --force-pg --backend nccl --no-cpu-baseline --consumer-msgs 0 --e2e-steps 0 \
    > $O/rccl_q$q.jsonl 2> $O/rccl_q$q.log || { tail -20 $O/rccl_q$q.log; exit 5; }
  GOME_HW_QUEUES=$q timeout -k 10 400 python3 bench.py --no-cpu-baseline --consumer-msgs 0 --e2e-steps 0 > $O/plain_q$q.jsonl 2> $O/plain_q$q.log \
    || { tail -20 $O/plain_q$q.log; exit 6; }
  for f in rccl plain; do
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['early_plans'])" $O/${f}_q$q.jsonl
  done
done

#!/bin/bash
# Multi-rank schedule A/B on a one-GPU box (run from the repo root):
#   bash tools/rccl_streams_ab.sh <tag>
# bench.py --dist-at-world1 initialises torch.distributed (RCCL) for one rank, so the
# sub-batch streams run beside an RCCL process group exactly as on every rank of an N-GPU run:
# communicator created lazily (at the accumulator all-reduce after the timed region) or eagerly
# (device_id at init_process_group), 1 or 3 streams.  Plain single-process runs bracket them.
set -e
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29512
B="python3 $R/bench.py --steps 6 --warmup 1 --no-cpu-baseline --kernel-reps 1"
timeout -k 10 120 $B --streams 3 > "$O/plain_s3.log" 2>&1
for INIT in lazy eager; do
  for S in 3 1; do
    RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 120 $B --dist-at-world1 --rccl-init $INIT \
        --streams $S > "$O/dist_${INIT}_s$S.log" 2>&1
  done
done
timeout -k 10 120 $B --streams 1 > "$O/plain_s1.log" 2>&1
for f in "$O"/*.log; do
  python3 -c "import json,sys; l=[json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')][-1]; print(sys.argv[1].split('/')[-1], round(l['value']), l['config'].get('rccl_init'), l['config']['streams_per_gpu'])" "$f"
done

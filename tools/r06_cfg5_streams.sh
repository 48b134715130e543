#!/bin/bash
# cfg5 grid: stream count x hardware queues (the grid is a latency chain per call: more calls in flight?)
O=gpurun_out/r06_c5s; mkdir -p $O
for arm in "3 4" "4 8" "6 8" "8 12" "12 16"; do
  set -- $arm
  timeout -k 10 240 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline --streams $1 --hw-queues $2 \
      > $O/s$1_q$2.log 2>&1 || exit $?
done

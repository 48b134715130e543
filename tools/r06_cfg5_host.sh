#!/bin/bash
# cfg5 on one box: streams x hardware queues x host enqueue threads (graphs on)
O=gpurun_out/r06_c5h2; mkdir -p $O
B="timeout -k 10 240 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline"
$B > $O/s3.log 2>&1 || exit $?
$B --enqueue threads > $O/s3t.log 2>&1 || exit $?
$B --streams 4 --hw-queues 8 > $O/s4q8.log 2>&1 || exit $?
$B --streams 4 --hw-queues 8 --enqueue threads > $O/s4q8t.log 2>&1 || exit $?
$B --streams 8 --hw-queues 12 > $O/s8q12.log 2>&1 || exit $?
$B --streams 3 > $O/s3b.log 2>&1

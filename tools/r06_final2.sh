#!/bin/bash
# closing bench lines after the cfg5 stream default (4 streams, 8 hardware queues): cfg1 default, cfg5
O=gpurun_out/r06_final2; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_cfg1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config cfg5 > $O/bench_cfg5.log 2>&1

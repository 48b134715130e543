#!/bin/bash
# the small M-step shapes added for the panel solve (n_rx 3 / 4, ragged last panel)
O=gpurun_out/r06_r10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_em.py -m gpu -x -v --timeout 120 --timeout-method thread -k "small_mstep or captured" > $O/tests.log 2>&1

#!/bin/bash
timeout -k 10 120 python tools/ab_small.py 120 20 > gpurun_out/r06_ab_small3.log 2>&1 &&
timeout -k 10 120 python tools/ab_small.py 15 20 >> gpurun_out/r06_ab_small3.log 2>&1

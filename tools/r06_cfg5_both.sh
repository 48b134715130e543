#!/bin/bash
# cfg5: raw kernel trace of one grid step, then the stream-count x hardware-queue sweep
bash tools/r06_cfg5_trace.sh || exit $?
bash tools/r06_cfg5_streams.sh

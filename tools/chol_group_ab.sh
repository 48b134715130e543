#!/bin/bash
# (historical: SBCE_CHOL_GROUP was removed after this A/B, see profiles/r06/chol; git history)
# A/B of the trial-grouped Cholesky at cfg1 (bench.py default line, 3 stream sub-batches of ~333
# trials): SBCE_CHOL_GROUP unset / 167 / 111 / 84, each in its own process
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_cgrp}
mkdir -p $O
for G in 0 167 111 84 0; do
    if [ $G = 0 ]; then unset SBCE_CHOL_GROUP; else export SBCE_CHOL_GROUP=$G; fi
    timeout -k 10 200 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/g$G.log 2>&1 || exit 1
    python3 -c "import json,sys;L=[l for l in open('$O/g$G.log') if l.startswith('{')];d=json.loads(L[-1]);print('G=$G', round(d['value']), d['ms_per_step'], d['chol_roofline']['ms'])" >> $O/summary.txt
done
unset SBCE_CHOL_GROUP

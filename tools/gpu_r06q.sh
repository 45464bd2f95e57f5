#!/bin/bash
# r06q: the register-weight policy kernel's grid (USV_POLICY_GRID cap) against the field chain it shares CUs with
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06q
mkdir -p $O
cd $R
for rep in 1 2; do
  for g in 0 448 384 320; do
    USV_POLICY_GRID=$g timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
      --c2-steps 0 --milestone-seconds 0 > $O/bench_g$g.$rep.json 2> $O/bench_g$g.$rep.err || exit $?
  done
done

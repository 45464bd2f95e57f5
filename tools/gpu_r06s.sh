#!/bin/bash
# r06s: the overlapped step's scheduling switches re-measured with the round-6 kernels (register-weight policy,
# no k_field_exact): default / USV_LATE_ON_JOIN=0 / USV_STATS_FIRST=1 / USV_RESET_ON_SIDE=1, interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06s
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in base USV_LATE_ON_JOIN=0 USV_STATS_FIRST=1 USV_RESET_ON_SIDE=1; do
    if [ $v = base ]; then e=USV_DUMMY=0; else e=$v; fi
    env $e timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_${v%%=*}.$rep.json 2> $O/bench_${v%%=*}.$rep.err || exit $?
  done
done

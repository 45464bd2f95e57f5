#!/bin/bash
# GPU box: rocprofv3 kernel stats of a short bench under several environment settings (one run each).
#   CASES="a:VAR=1 b:VAR=0" bash tools/gpu_kstats_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/kstats_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in $CASES; do
  name=${c%%:*}; vars=${c#*:}
  for kv in ${vars//,/ }; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o t -- python3 $R/bench.py \
    --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/$name.log 2>&1 || exit $?
  for kv in ${vars//,/ }; do unset "${kv%%=*}"; done
  echo "== $name"
  python3 $R/tools/kstats.py $O/$name/t_kernel_stats.csv 2>/dev/null | head -${TOP:-14} || head -14 $O/$name/t_kernel_stats.csv | cut -c1-150
done

#!/bin/bash
# GPU box: rocprofv3 kernel stats of a short bench for each library variant in VARIANTS
# (lib/<name>.so, "base" = lib/libusv_hip.so); prints the top kernels of each.
#   VARIANTS="base v1" bash tools/gpu_kvariants.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/kvariants
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in $VARIANTS; do
  lib=""; [ "$v" != "base" ] && lib="$v.so"
  USV_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o trace -- \
    python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --c2-steps 0 > $O/$v.log 2>&1 || exit $?
  echo "== $v"
  python3 $R/tools/kstats.py $(find $O/$v -name "*kernel_stats.csv" | head -1) ${TOP:-4}
  find $O/$v -name "*kernel_trace.csv" -delete   # the per-dispatch trace: tens of MB, not copied back
done

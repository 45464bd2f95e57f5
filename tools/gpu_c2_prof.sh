#!/bin/bash
# GPU box: kernel stats + bench line of the 4096-env workload (BASELINE configs[1]) alone, for the small-batch
# field path (k_field_wave, one env per CU).   LIB=<variant>.so optional (USV_HIP_LIB).  Output in gpurun_out/c2prof/
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c2prof${TAG:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--envs ${ENVS:-4096} --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --c2-steps 0"
USV_HIP_LIB=${LIB:-} timeout -k 10 300 python3 $R/bench.py $A > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));e=d['extra'];print('value %.4gM ms/epoch %.3f rollout %.3f update %.3f host_gap %.3f' % (d['value']/1e6, d['ms_per_step'], e['rollout_ms'], e['update_ms'], e['host_gap_ms']))"
USV_HIP_LIB=${LIB:-} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- \
  python3 $R/bench.py $A > $O/prof.log 2>&1 || exit $?
python3 $R/tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) ${TOP:-14}
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/trace.csv \; -delete

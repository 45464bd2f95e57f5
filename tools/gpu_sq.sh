set -euo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
cd /tmp && export TMPDIR=/tmp

timeout -k 10 300 python3 $R/tools/env_step_probe.py 4096 32 > $R/gpurun_out/sq/probe.log 2>&1
timeout -k 10 300 python3 $R/tools/env_step_probe.py 131072 32 >> $R/gpurun_out/sq/probe.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex k_env_step --output-format csv -d $R/gpurun_out/sq -o sq131072 -- python3 $R/tools/env_step_probe.py 131072 8 > $R/gpurun_out/sq/pmc.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex k_env_step --output-format csv -d $R/gpurun_out/sq -o sq4096 -- python3 $R/tools/env_step_probe.py 4096 8 >> $R/gpurun_out/sq/pmc.log 2>&1
cat $R/gpurun_out/sq/probe.log

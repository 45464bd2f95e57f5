#!/bin/bash
# GPU box: the round's committed evidence in one call -- rocprofv3 kernel stats + separate
# FETCH_SIZE / WRITE_SIZE passes on the env-step kernel at the bench size (4096 envs) and the C5
# per-GPU size (131072), condensed into profiles/, then the default bench line (with the CPU
# baseline) reading the fresh traffic numbers.   bash tools/gpu_profile_round.sh <tag>
set -uo pipefail
TAG=${1:-r01d}
R=$GRAFT_REPO_ROOT
cd $R
bash profiles/run_profiles.sh $TAG 4096 || exit $?
python3 profiles/pmc_traffic.py $TAG 4096 profiles/env_step_traffic.json || exit $?
bash profiles/run_profiles.sh ${TAG}_131072 131072 || exit $?
python3 profiles/pmc_traffic.py ${TAG}_131072 131072 || exit $?
mkdir -p gpurun_out/$TAG
cp profiles/${TAG}_* profiles/env_step_traffic*.json gpurun_out/$TAG/ || exit $?
rm -rf gpurun_out/prof_${TAG} gpurun_out/prof_${TAG}_131072   # raw traces: condensed above (the merge-back cap is 64 MiB)
timeout -k 10 600 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cat gpurun_out/$TAG/bench.json

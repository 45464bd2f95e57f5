#!/bin/bash
# GPU box, round 4 evidence in one call: the XCD-group fold A/B (USV_PPO_FOLD=1 vs 0, headline bench A B A B), the
# peer exchange's memory-ordering A/B (two-rank one-device rehearsal), then the profile round (kernel trace,
# sequential-step trace, PMC FETCH / WRITE passes at 4096 and 131072 envs, the default bench line).
# A step that ends in a time limit, an abort or a fault ends the call (no further GPU step).
#   TAG=r04b bash tools/gpu_round4.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r04b}
mkdir -p gpurun_out/$TAG
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
if [ "${SKIP_FOLD:-0}" != "1" ]; then CASES="fold1:USV_PPO_FOLD=1 fold0:USV_PPO_FOLD=0" REPS=2 STEPS=10 bash tools/gpu_envvar_ab.sh; rc=$?; fatal $rc fold_ab; fi
cp -r gpurun_out/envvar_ab gpurun_out/$TAG/fold_ab 2>/dev/null
[ "${SKIP_DP:-0}" = "1" ] || { TAG=$TAG bash tools/gpu_dp2_order_ab.sh; rc=$?; fatal $rc dp_order_ab; }
bash tools/gpu_profile_round.sh $TAG; rc=$?; fatal $rc profile_round
exit $rc

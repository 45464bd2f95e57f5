set -o pipefail
timeout -k 10 1100 bash tools/gpu_profile_round.sh r05fin > gpurun_out/r05fin_round.log 2>&1; rc=$?; tail -3 gpurun_out/r05fin_round.log; exit $rc

set -o pipefail
timeout -k 10 1100 bash tools/gpu_profile_round.sh r05v > gpurun_out/r05v_round.log 2>&1; rc=$?; tail -5 gpurun_out/r05v_round.log; exit $rc

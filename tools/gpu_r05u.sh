set -o pipefail
mkdir -p gpurun_out/r05u
timeout -k 10 300 python3 tools/phase_probe.py 131072 > gpurun_out/r05u/probe.log 2>&1; rc=$?; grep -A12 "k_policy_step" gpurun_out/r05u/probe.log; exit $rc

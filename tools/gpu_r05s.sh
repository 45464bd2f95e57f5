set -o pipefail
mkdir -p gpurun_out/r05s
timeout -k 10 300 python3 -u tools/env_parts_probe.py 131072 24 > gpurun_out/r05s/parts.log 2>&1 && \
VARIANTS="base notop5 notexel" TAG=r05s timeout -k 10 700 bash tools/gpu_env_ab.sh > gpurun_out/r05s/ab.log 2>&1

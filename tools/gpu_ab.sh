#!/bin/bash
# GPU box: [GPU tests], then bench A and bench B alternately (A B A B) on the same box.
#   LIB_A / LIB_B: lib/<name>.so builds of the same ABI (USV_HIP_LIB), empty = lib/libusv_hip.so
#   BENCH_A_ARGS / BENCH_B_ARGS: extra bench.py arguments
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  USV_HIP_LIB=${LIB_A:-} timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_A_ARGS:-} > $O/a$rep.json 2> $O/a$rep.err || exit $?
  USV_HIP_LIB=${LIB_B:-} timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_B_ARGS:-} > $O/b$rep.json 2> $O/b$rep.err || exit $?
done
python3 - <<'PY'
import json, os
for k in ("a1", "b1", "a2", "b2"):
    d = json.load(open(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/ab", k + ".json")))
    e = d["extra"]
    print(k, "value %.4gM ms/step %.3f rollout %.3f update %.3f env_kernel %.1f us envonly131k %.1fM/s kernel %.1f us" % (
        d["value"] / 1e6, d["ms_per_step"], e.get("rollout_ms", 0), e.get("update_ms", 0),
        d["roofline"]["launch_ms"] * 1e3, e.get("env_only_fps", 0) / 1e6, e.get("env_step_kernel_ms", 0) * 1e3))
PY

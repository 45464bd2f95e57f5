#!/bin/bash
# GPU box: SQ / TCC counters of the field pipeline's kernels (sequential step, 131072 envs), one pass per counter
# group:  bash tools/gpu_field_pmc.sh <tag>
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04f}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export USV_STEP_OVERLAP=0
B="$R/bench.py --steps 3 --warmup 1 --envs 131072 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0"
RX='k_field_stats|k_field_wave_pack|k_field_place|k_policy_step'
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex "$RX" --output-format csv -d $O -o sq -- python3 $B > $O/sq.log 2>&1 || exit $?
echo "sq done"
timeout -k 10 400 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d $O -o sq2 -- python3 $B > $O/sq2.log 2>&1 || exit $?
echo "sq2 done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O -o fetch -- python3 $B > $O/fetch.log 2>&1 || exit $?
echo "fetch done"
python3 - $O <<'PY'
import csv, sys, glob, collections, re
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        nm = re.sub(r"^void ", "", r["Kernel_Name"]).replace("(anonymous namespace)::", "")
        nm = re.split(r"[<(]", nm)[0]
        acc[nm][r["Counter_Name"]].append(float(r["Counter_Value"]))
for nm, d in sorted(acc.items()):
    print(nm)
    for k, v in sorted(d.items()):
        print("   %-22s mean per dispatch %.4g  (dispatches %d)" % (k, sum(v) / len(v), len(v)))
PY

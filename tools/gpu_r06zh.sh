#!/bin/bash
# r06zh: the losses' divisions by sigma as div_rn (libusv_hip_divrn.so, -DUSV_LOSS_DIVRN=1) vs the IEEE divisions:
# bits of a 3-epoch run at 4096 envs under each library, then k_mb_grad's per-dispatch median, twice, interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zh
mkdir -p $O
cd $R
timeout -k 10 200 python3 tools/lib_bits.py $O/base.npz > $O/bits.log 2>&1 || exit $?
USV_HIP_LIB=libusv_hip_divrn.so timeout -k 10 200 python3 tools/lib_bits.py $O/divrn.npz >> $O/bits.log 2>&1 || exit $?
python3 tools/lib_bits.py --compare $O/base.npz $O/divrn.npz | tee -a $O/bits.log
for rep in 1 2; do
  CASES="divrn:USV_HIP_LIB=libusv_hip_divrn.so base:USV_DUMMY=0" KERNELS="k_mb_grad k_reduce_partials" STEPS=3 \
    bash tools/gpu_kmed_ab.sh > $O/kmed.$rep.txt 2>&1 || exit $?
  cat $O/kmed.$rep.txt
done

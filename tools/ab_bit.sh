#!/bin/bash
# A knob: bit-identity of 6 headline-shape steps with / without it, the NB parity subset under it, then headline benches
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=${1:-ab}; KNOB=${2:?knob}
timeout -k 10 120 python tools/bitcheck.py gpurun_out/$TAG.base.npz > gpurun_out/$TAG.bit.log 2>&1 || { tail -5 gpurun_out/$TAG.bit.log; exit 1; }
env $KNOB timeout -k 10 120 python tools/bitcheck.py gpurun_out/$TAG.knob.npz bf16x3 gpurun_out/$TAG.base.npz >> gpurun_out/$TAG.bit.log 2>&1; rc=$?
tail -1 gpurun_out/$TAG.bit.log; [ $rc -eq 0 ] || exit 7
bash tools/ab_env.sh $TAG "$KNOB" bf16x3

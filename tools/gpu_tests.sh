#!/bin/bash
# GPU test subset: bash tools/gpu_tests.sh TAG "pytest selection args..."
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1
rc=$?; tail -15 gpurun_out/$TAG.test.log; exit $rc

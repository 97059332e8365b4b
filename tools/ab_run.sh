#!/bin/bash
# parity subset on the in-tree build, then ab_lib against a variant build
# Usage: bash tools/ab_run.sh TAG NAME "models" "dtypes" "test files"
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=$1; NAME=$2; MODELS=${3:-nb}; DTS=${4:-bf16x3}; TESTS=${5:-"tests/test_gpu_nb.py tests/test_gpu_tiling.py tests/test_gpu_graph.py"}
timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG.test.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh $TAG $NAME "$MODELS" "$DTS"

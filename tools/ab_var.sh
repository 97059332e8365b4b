#!/bin/bash
# A variant build (tools/build_variant.sh NAME): NB parity subset on it, then headline benches base / variant
# Usage: bash tools/ab_var.sh TAG NAME [dtypes] [models]
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=$1; NAME=$2; DTS=${3:-bf16x3}; MODELS=${4:-nb}
MMVAE_LIB=mm-vae_amd/lib_$NAME/libmmvae.so timeout -k 10 400 python -u -m pytest tests/test_gpu_nb.py tests/test_gpu_tiling.py tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG.test.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh $TAG $NAME "$MODELS" "$DTS"

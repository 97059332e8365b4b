#!/bin/bash
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
export MMVAE_LIB=mm-vae_amd/lib_diag/libmmvae.so
UPDATE=1 DTYPE=bf16x3 timeout -k 10 120 python tools/stamps_dec.py > gpurun_out/r5_st_base.txt 2>&1 || exit 1
cp gpurun_out/stamps_dec.npy gpurun_out/stamps_base.npy
MMVAE_DEC_FS=1 UPDATE=1 DTYPE=bf16x3 timeout -k 10 120 python tools/stamps_dec.py > gpurun_out/r5_st_fs.txt 2>&1 || exit 2
cp gpurun_out/stamps_dec.npy gpurun_out/stamps_fs.npy
cat gpurun_out/r5_st_base.txt gpurun_out/r5_st_fs.txt

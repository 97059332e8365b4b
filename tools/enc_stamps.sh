#!/bin/bash
# phase stamps of k_enc_fwd (x3 and bf16) and the latent kernels (diagnostic build)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
export MMVAE_LIB=$R/mm-vae_amd/lib_diag/libmmvae.so
DTYPE=bf16x3 timeout -k 10 120 python tools/stamps.py > gpurun_out/enc_stamps_x3.txt 2>&1 && \
KER=fwd timeout -k 10 150 python tools/stamps_lat.py > gpurun_out/lat_fwd.txt 2>&1 && \
KER=bwd timeout -k 10 150 python tools/stamps_lat.py > gpurun_out/lat_bwd.txt 2>&1

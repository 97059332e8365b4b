#!/bin/bash
# phase stamps of pass B (x3, training) and the latent kernels on the diagnostic build
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
export MMVAE_LIB=mm-vae_amd/lib_diag/libmmvae.so
UPDATE=1 DTYPE=bf16x3 timeout -k 10 120 python tools/stamps_dec.py || exit 3
KER=fwd timeout -k 10 120 python tools/stamps_lat.py || exit 1
KER=bwd timeout -k 10 120 python tools/stamps_lat.py || exit 2

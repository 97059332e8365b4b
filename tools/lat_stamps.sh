#!/bin/bash
# phase stamps of k_latent_fwd / k_latent_bwd (diagnostic build: tools/build_variant.sh diag -DMMVAE_DIAG)
# EXTRA: more MMVAE_DBG bits for the forward run (4096: no Philox noise)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
export MMVAE_LIB=$R/mm-vae_amd/lib_diag/libmmvae.so
KER=fwd timeout -k 10 150 python tools/stamps_lat.py > gpurun_out/lat_fwd.txt 2>&1 && \
KER=fwd EXTRA=4096 timeout -k 10 150 python tools/stamps_lat.py > gpurun_out/lat_fwd_nophilox.txt 2>&1 && \
KER=bwd timeout -k 10 150 python tools/stamps_lat.py > gpurun_out/lat_bwd.txt 2>&1

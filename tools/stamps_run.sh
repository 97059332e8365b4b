#!/bin/bash
# phase stamps of the latent kernels and decoder pass B (diagnostic builds of the same kernels)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
# the stamp bits live only in the diagnostic build (bash tools/build_variant.sh diag -DMMVAE_DIAG, on the CPU first)
export MMVAE_LIB=mm-vae_amd/lib_diag/libmmvae.so
#KER=fwd timeout -k 10 120 python tools/stamps_lat.py || exit 1
#KER=bwd timeout -k 10 120 python tools/stamps_lat.py || exit 2
UPDATE=1 DTYPE=bf16x3 timeout -k 10 120 python tools/stamps_dec.py || exit 3
UPDATE=1 DTYPE=bf16 timeout -k 10 120 python tools/stamps_dec.py || exit 4

#!/bin/bash
# Gene-split occupancy scan (diagnostic): bench per MMVAE_NSPLIT_{E,D,A} setting.
mkdir -p gpurun_out; out=gpurun_out/split_scan.txt; : > $out
run() {
  env "$@" timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/ss.json 2> gpurun_out/ss.err || { tail -3 gpurun_out/ss.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/ss.json')); k=j['kernel_ms']; print(sys.argv[1:], 'step', j['ms_per_step'], {n: k.get(n) for n in ['k_enc_fwd','k_enc_bwd','k_dec_nb','k_dec_lse','k_dec_tail','k_latent_fwd','k_latent_bwd','k_grad_genes']})" "$@" >> $out
}
run X=0
run MMVAE_NSPLIT_E=16
run MMVAE_NSPLIT_E=32
run MMVAE_NSPLIT_D=16
run MMVAE_NSPLIT_D=4
run MMVAE_NSPLIT_A=16
run MMVAE_NSPLIT_A=64
cat $out

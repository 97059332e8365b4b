R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for dt in bf16x3 bf16; do for a in 16 24 32 48; do
  MMVAE_NSPLIT_A=$a timeout -k 10 200 python bench.py --no-extras --no-cpu --dtype $dt --steps 150 > gpurun_out/sa.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sa.json'));k=d['kernel_ms'];print('$dt A=$a', round(d['value']), d['ms_per_step'], k['k_dec_lse'], k['k_dec_tail'])"
done; done

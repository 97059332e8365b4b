# long-warmup bench + PMC passes (clock, stall, bytes)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python bench.py --no-cpu --warmup 300 --steps 200 --kernel-steps 50 > gpurun_out/p2.bench.json 2>gpurun_out/p2.bench.err || exit 1
cat gpurun_out/p2.bench.json
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM -d $R/gpurun_out/pmc2a -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 100 --kernel-steps 2 --no-cpu > /dev/null 2>$R/gpurun_out/pmc2a.err || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc2b -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 100 --kernel-steps 2 --no-cpu > /dev/null 2>$R/gpurun_out/pmc2b.err || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc2c -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 100 --kernel-steps 2 --no-cpu > /dev/null 2>$R/gpurun_out/pmc2c.err || exit 4
echo done

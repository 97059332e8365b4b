R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; export TMPDIR=/tmp; cd /tmp
rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $R/gpurun_out/prof1_bench.json 2>$R/gpurun_out/prof1.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU --kernel-include-regex k_dec -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>$R/gpurun_out/pmc1.err
find $R/gpurun_out -name "*.csv" | head; tail -3 $R/gpurun_out/pmc1.err

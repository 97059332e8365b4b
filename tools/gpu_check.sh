# GPU iteration script: parity tests then a short bench.  Usage: bash tools/gpu_check.sh TAG [bench args]
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG.test.log 2>&1; rc=$?
tail -15 gpurun_out/$TAG.test.log
if [ $rc -ne 0 ]; then echo "tests failed rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
brc=$?; cat gpurun_out/$TAG.bench.json; tail -3 gpurun_out/$TAG.bench.err; exit $brc

#!/bin/bash
# short-window vs long-window timing of the headline (the driver times 20 steps after 5 warm-up)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for a in "20 5" "20 5" "20 5" "1000 50"; do
  set -- $a
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu --no-extras > gpurun_out/probe_$1_$2.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/probe_$1_$2.json')); print('steps',$1,'warm',$2, d['value'], d['ms_per_step'], d.get('median_ms_per_step_synced'), d['device_ms_per_step'])"
done

#!/bin/bash
# development: bench lines of $WL (no CPU baseline), one JSON summary each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b
for w in ${WL:-pages4k zipf chunks}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --cpu-seconds ${CPUS:-0} > gpurun_out/b/$w.json 2> gpurun_out/b/$w.err || { tail -3 gpurun_out/b/$w.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b/$w.json')); r=d['roofline']; print('$w', round(d['value'],1), d['unit'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'parity', d.get('parity_ok'))"
done

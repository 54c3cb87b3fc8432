#!/bin/bash
# development: same-box A/B of bench lines ($WL) across engine builds ($LIBS), interleaved, NPASS passes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in $(seq ${NPASS:-2}); do
for w in ${WL:-zipf}; do
for L in ${LIBS:-new}; do
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 300 python bench.py --workload $w --steps 20 --cpu-seconds 0 > gpurun_out/ab/${w}_$L.json 2> gpurun_out/ab/${w}_$L.err || { tail -3 gpurun_out/ab/${w}_$L.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/${w}_$L.json')); r=d['roofline']; print('$w $L', round(d['value'],1), 'ms', d['ms_per_step'], 'frac', r['frac'], 'parity', d.get('parity_ok'))"
done; done; done

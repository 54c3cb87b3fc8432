#!/bin/bash
# development: GPU tests ($TESTS, -k $KEXPR), then optional XXH3 probes ($XPROBE) per library ($LIBS)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
timeout -k 10 ${TLIM:-500} python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread ${TESTS:-tests} ${KEXPR:+-k "$KEXPR"} > gpurun_out/t/tests.log 2>&1
rc=$?; tail -6 gpurun_out/t/tests.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$XPROBE" ]; then ARGS="$XPROBE" bash tools/gpu_xprobe.sh; fi

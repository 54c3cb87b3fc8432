#!/bin/bash
# development: A/B of engine builds on one box (LIBS, PROBES, FDBCRC_ROUTE from the caller)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/prof_libs.sh
